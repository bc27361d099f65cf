#!/bin/bash
# Round-5 twelfth GPU call: parity of this tree; LDS promotion of private arrays on/off on the
# sub-capacity storm and the gossip; a kernel trace of the bucketed 1M-peer window; the fused test
# that fails only in the TGSIM_CHECK build, with and without the small slot limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05/twelfth; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|error" $O/pytest_gpu.log | head -20; exit 1; }
REPS=3 AB=twelfth_open ARGS="--no-cpu --no-1m --no-variants --shapes open" VARIANTS="cur nopromote" bash scripts/r05_gossip_ab.sh || exit 1
AB=twelfth_gossip VARIANTS="cur nopromote" bash scripts/r05_gossip_ab.sh || exit 1
TAG=gossip_trace_bkt bash scripts/r05_gossip_trace.sh || exit 1
for v in check check_full; do
  TGSIM_LIB=$PWD/testground_amd/libtgsim_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py -m gpu -v -s \
    --timeout 200 --timeout-method thread > $O/fused_$v.log 2>&1; echo "$v rc=$?"; tail -3 $O/fused_$v.log
  grep "EXEC CHECK" $O/fused_$v.log | sort | uniq -c | head
done
