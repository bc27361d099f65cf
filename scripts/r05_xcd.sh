#!/bin/bash
# Round-5: XCD-contiguous source order in k_sim_sparse (blocks b and b + 8 share an XCD's L2; with
# it they take neighbouring sources) with the bucketed delivery; A/B and the simulate kernels' PMC.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPS=3 AB=xcd_gossip VARIANTS="cur xcd xcd2" bash scripts/r05_gossip_ab.sh || exit 1
WL=gossip VARIANTS="xcd" bash scripts/r05_pmc.sh || exit 1
