#!/bin/bash
# Round-5 twentieth GPU call: the C3 heavy-source chain measured (sub-windows per
# batch, us per sub-window and the admission-ended share for the 512 slowest sources, profile build;
# the fused launch's chains), then the routed N > 1 step at one rank (item 5).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05/twentieth; mkdir -p $O
timeout -k 10 300 python -u scripts/stamps.py --steps 65 > $O/stamps_storm_prof.txt 2> $O/stamps_storm_prof.err || { tail $O/stamps_storm_prof.err; exit 1; }
grep -E "512 slowest|per batch|kernel span" $O/stamps_storm_prof.txt
timeout -k 10 300 python -u scripts/stamps_chains.py > $O/stamps_chains.txt 2> $O/stamps_chains.err || { tail $O/stamps_chains.err; exit 1; }
head -20 $O/stamps_chains.txt
TAG=routed bash scripts/r05_routed.sh || exit 1
