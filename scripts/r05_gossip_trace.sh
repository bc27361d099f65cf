#!/bin/bash
# Kernel trace of the 1M-peer gossip window (70 timed windows) and its per-window breakdown.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05/${TAG:-gossip_trace}; rm -rf $O; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o run -- python3 bench.py --workload gossip --peers 1000000 --no-cpu --steps 70 > $O/tr.log 2>&1 || { tail $O/tr.log; exit 1; }
cp $(find $O/tr -name "*kernel_trace.csv" | head -1) $O/kernel_trace.csv && cp $(find $O/tr -name "*kernel_stats.csv" | head -1) $O/kernel_stats.csv && rm -rf $O/tr
python scripts/gossip_window_breakdown.py $O/kernel_trace.csv > $O/breakdown.txt 2>&1
gzip -f $O/kernel_trace.csv
head -30 $O/breakdown.txt
