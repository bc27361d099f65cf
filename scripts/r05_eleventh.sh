#!/bin/bash
# Round-5 eleventh GPU call: A/B of the bucketed sparse windows against the slot scatter
# (TGSIM_DST_BKT=0) and the cursors (TGSIM_DST_SLOT=0), then the TGSIM_CHECK build over every GPU
# test (guard violations attributed to source lines).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
AB=eleventh_gossip VARIANTS="cur TGSIM_DST_BKT=0 TGSIM_DST_SLOT=0" bash scripts/r05_gossip_ab.sh || exit 1
AB=eleventh_open ARGS="--no-cpu --no-1m --no-variants --shapes open" VARIANTS="cur TGSIM_DST_BKT=0 TGSIM_DST_SLOT=0" bash scripts/r05_gossip_ab.sh || exit 1
bash scripts/r05_check_build.sh
