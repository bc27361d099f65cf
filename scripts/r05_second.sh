#!/bin/bash
# Round-5 second GPU call: the gossip A/B of the sparse-kernel variants (after the VGPR-spill fix),
# round 4's HEAD beside them, then the sub-capacity bisect.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
AB=second_ab VARIANTS="cur tree:bisect/f8367ce xcd w2x w4x nofwd hint xfh" bash scripts/r05_gossip_ab.sh || exit 1
COMMITS="f6d001e 0362bf1 ae9aa0a 7ff58ac 769e16c d6e535a f8367ce HEAD" bash scripts/r05_bisect_open.sh
