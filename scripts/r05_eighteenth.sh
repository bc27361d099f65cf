#!/bin/bash
# Round-5 eighteenth GPU call: the histogram scan of a bucketed window on the simulate stream (per-set
# scan buffers; the overflow list was reverted), parity first, then A/B against
# the scan on the delivery stream (TGSIM_SCAN_ON_SIM=0) and the previous commit's tree.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05/eighteenth; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|error" $O/pytest_gpu.log | head -20; exit 1; }
REPS=3 AB=eighteenth_gossip VARIANTS="cur TGSIM_SCAN_ON_SIM=0 tree:bisect/e8dcbdb" bash scripts/r05_gossip_ab.sh || exit 1
AB=eighteenth_open ARGS="--no-cpu --no-1m --no-variants --shapes open" VARIANTS="cur TGSIM_SCAN_ON_SIM=0" bash scripts/r05_gossip_ab.sh || exit 1
