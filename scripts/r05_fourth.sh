#!/bin/bash
# Round-5 fourth GPU call: kernel trace of the 1M-peer gossip window, PMC bytes of its simulate and
# delivery kernels for three builds, and A/B of the delivery timing events and the scatter choice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05/fourth; mkdir -p $O
B="--workload gossip --peers 1000000 --no-cpu"
rm -rf $O/trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py $B > $O/trace.log 2>&1 || { tail $O/trace.log; exit 1; }
echo "trace ok"
AB=fourth_open ARGS="--no-cpu --no-1m --no-variants --shapes open" VARIANTS="cur TGSIM_DV_TIMING=0 TGSIM_LOCAL_SCATTER=1" bash scripts/r05_gossip_ab.sh || exit 1
AB=fourth_gossip VARIANTS="cur TGSIM_DV_TIMING=0" bash scripts/r05_gossip_ab.sh || exit 1
WL=gossip PMC_GROUPS="FETCH_SIZE|WRITE_SIZE" VARIANTS="cur xcd nofwd" bash scripts/r05_pmc.sh || exit 1
