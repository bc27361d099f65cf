#!/bin/bash
# Round-5 eighth GPU call: records placed by their destination slot (the histogram increment's
# return value) instead of scatter cursor atomics; parity first, then A/B against the cursors
# (TGSIM_DST_SLOT=0) on the 1M-peer gossip and the sub-capacity storm.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05/eighth; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|error" $O/pytest_gpu.log | head -20; exit 1; }
AB=eighth_gossip VARIANTS="cur TGSIM_DST_SLOT=0" bash scripts/r05_gossip_ab.sh || exit 1
AB=eighth_open ARGS="--no-cpu --no-1m --no-variants --shapes open" VARIANTS="cur TGSIM_DST_SLOT=0" bash scripts/r05_gossip_ab.sh || exit 1
