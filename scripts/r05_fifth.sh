#!/bin/bash
# Round-5 fifth GPU call: pytest -m gpu (worklist counters zeroed and published by a kernel, sampled
# timing events), A/B of the timing events' sampling, and the sparse deferral reasons at the 1M-peer
# flood's peak (TGSIM_DEFER_STATS build, TGSIM_TRACE_LIST=1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05/fifth; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|error" $O/pytest_gpu.log | head -20; exit 1; }
TGSIM_LIB=$PWD/testground_amd/libtgsim_defer.so TGSIM_TRACE_LIST=1 timeout -k 10 300 python bench.py --workload gossip --peers 1000000 --no-cpu > $O/defer.json 2> $O/defer.err || { tail $O/defer.err; exit 1; }
grep -c "deferred" $O/defer.err
AB=fifth_open ARGS="--no-cpu --no-1m --no-variants --shapes open" VARIANTS="cur TGSIM_DV_TIMING=4 TGSIM_SIM_TIMING=4 TGSIM_DV_TIMING=0" bash scripts/r05_gossip_ab.sh || exit 1
AB=fifth_epochs ARGS="--no-cpu --workload epochs" VARIANTS="cur TGSIM_SIM_TIMING=4" bash scripts/r05_gossip_ab.sh || exit 1
AB=fifth_gossip VARIANTS="cur TGSIM_SIM_TIMING=4" bash scripts/r05_gossip_ab.sh || exit 1
