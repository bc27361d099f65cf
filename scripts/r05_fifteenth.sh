#!/bin/bash
# Round-5 fifteenth GPU call: the delivery stream at high priority (TGSIM_DST_PRIO=0) on the bucketed
# 1M-peer gossip, and the bench's sampled timing on the sub-capacity storm.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
AB=fifteenth_gossip VARIANTS="cur TGSIM_DST_PRIO=0" bash scripts/r05_gossip_ab.sh || exit 1
REPS=3 AB=fifteenth_open ARGS="--no-cpu --no-1m --no-variants --shapes open" VARIANTS="cur TGSIM_DST_PRIO=0" bash scripts/r05_gossip_ab.sh || exit 1
