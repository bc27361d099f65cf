#!/bin/bash
# Round-5 twenty-third GPU call: the bucket sort's resident grid size on the 1M-peer gossip.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPS=2 AB=twentythird_gossip VARIANTS="cur TGSIM_SORT_GRID=1024 TGSIM_SORT_GRID=2048 TGSIM_SORT_GRID=8192" bash scripts/r05_gossip_ab.sh || exit 1
