#!/bin/bash
# Round-5 twenty-first GPU call: the bucketed sort on a grid of resident workgroups (grid-stride over
# destination groups) and the slot scatter skipping the 256-source blocks that wrote no emit record;
# parity, then A/B against one workgroup per group (TGSIM_SORT_GRID=-1) and the previous tree.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05/twentyfirst; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|error" $O/pytest_gpu.log | head -20; exit 1; }
REPS=3 AB=twentyfirst_gossip VARIANTS="cur TGSIM_SORT_GRID=-1 tree:bisect/b2bbabd" bash scripts/r05_gossip_ab.sh || exit 1
AB=twentyfirst_open ARGS="--no-cpu --no-1m --no-variants --shapes open" VARIANTS="cur tree:bisect/b2bbabd" bash scripts/r05_gossip_ab.sh || exit 1
