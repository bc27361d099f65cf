#!/bin/bash
# Round-5 twenty-fourth GPU call: the bucket sort's resident grid below 1,024 workgroups.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPS=2 AB=twentyfourth_gossip VARIANTS="TGSIM_SORT_GRID=1024 TGSIM_SORT_GRID=256 TGSIM_SORT_GRID=512 TGSIM_SORT_GRID=768 TGSIM_SORT_GRID=1536" bash scripts/r05_gossip_ab.sh || exit 1
AB=twentyfourth_open ARGS="--no-cpu --no-1m --no-variants --shapes open" VARIANTS="cur TGSIM_SORT_GRID=1024 TGSIM_SORT_GRID=512" bash scripts/r05_gossip_ab.sh || exit 1
