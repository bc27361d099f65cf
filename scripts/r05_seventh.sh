#!/bin/bash
# Round-5 seventh GPU call: the timing-event pool (prefilled, harvested when it runs dry) and the
# one-rank epochs overlap, A/B against round 4's HEAD; k_sim_list grid hint vs a fixed grid, and
# alloca promotion, on the 1M-peer gossip.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05/seventh; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gossip.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|error" $O/pytest_gpu.log | head -20; exit 1; }
AB=seventh_gossip VARIANTS="cur TGSIM_LIST_GRID=16384 alloca occ8 nosort nodv tree:bisect/f8367ce" bash scripts/r05_gossip_ab.sh || exit 1
AB=seventh_open ARGS="--no-cpu --no-1m --no-variants --shapes open" VARIANTS="cur TGSIM_DV_TIMING=0 TGSIM_DV_TIMING=8" bash scripts/r05_gossip_ab.sh || exit 1
REPS=3 AB=seventh_epochs ARGS="--no-cpu --workload epochs --steps 30" VARIANTS="cur tree:bisect/f8367ce" bash scripts/r05_gossip_ab.sh || exit 1
