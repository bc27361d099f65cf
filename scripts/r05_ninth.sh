#!/bin/bash
# Round-5 ninth GPU call: the sub-capacity storm fell with the destination-slot scatter and the LDS
# promotion in the eighth call (noisy pair); three interleaved runs of each combination.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPS=3 AB=ninth_open ARGS="--no-cpu --no-1m --no-variants --shapes open" VARIANTS="cur TGSIM_DST_SLOT=0 nopromote" bash scripts/r05_gossip_ab.sh || exit 1
AB=ninth_gossip VARIANTS="cur nopromote" bash scripts/r05_gossip_ab.sh || exit 1
