#!/bin/bash
# Kernel trace of the routed storm at one rank (TGSIM_COMM_ROUTE1=1, persistent grid): per-kernel
# totals of the timed run.
O=gpurun_out/r04/${TAG:-prof_routed}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
env ${ENVS:-TGSIM_COMM_ROUTE1=1 TGSIM_FUSED_PERSIST=1} timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rp -o run -- python bench.py --no-cpu --no-1m ${ARGS:---sharded} > $O/bench.json 2> $O/bench.err || { echo "failed rc=$?"; tail $O/bench.err; exit 1; }
f=$(find $O/rp -name '*kernel_stats.csv' | head -1)
cut -d, -f1-4 "$f" | head -25 > $O/stats_head.txt; cat $O/stats_head.txt
