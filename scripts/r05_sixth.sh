#!/bin/bash
# Round-5 sixth GPU call: pytest -m gpu, then A/B of this tree (k_sim_list grid from the last
# deferral count, no alloca-to-LDS promotion, lazy timing harvest) against round 4's HEAD on the
# 1M-peer gossip, the sub-capacity storm, C5 epochs and C3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05/sixth; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|error" $O/pytest_gpu.log | head -20; exit 1; }
AB=sixth_gossip VARIANTS="cur xcd tree:bisect/f8367ce" bash scripts/r05_gossip_ab.sh || exit 1
AB=sixth_open ARGS="--no-cpu --no-1m --no-variants --shapes open" VARIANTS="cur TGSIM_DV_TIMING=0 TGSIM_SIM_TIMING=0" bash scripts/r05_gossip_ab.sh || exit 1
AB=sixth_epochs ARGS="--no-cpu --workload epochs" VARIANTS="cur tree:bisect/f8367ce" bash scripts/r05_gossip_ab.sh || exit 1
AB=sixth_storm ARGS="--no-cpu --no-1m --no-variants" VARIANTS="cur" bash scripts/r05_gossip_ab.sh || exit 1
