#!/bin/bash
# Round-5 final evidence, part 1: PMC passes (FETCH_SIZE, WRITE_SIZE, wave counters; one rocprofv3 run
# each) of the four workloads of the default line at the frozen kernel source, summarized for the
# simulate and the delivery kernels (profiles/pmc_*.json after the copy).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for wl in storm gossip open epochs; do
  WL=$wl VARIANTS=cur bash scripts/r05_pmc.sh || { echo "pmc $wl failed"; exit 1; }
done
