#!/bin/bash
# Kernel trace of the sharded gossip loop at one rank (bench --sharded, 125k peers) with the per-window
# breakdown on the simulate stream.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp; O=gpurun_out/r03s; rm -rf $O; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python3 bench.py --workload gossip --peers 125000 --no-cpu --sharded > $O/tr.log 2>&1 || { tail $O/tr.log; exit 1; }
cp $(find $O/tr -name "*kernel_trace.csv" | head -1) $O/kernel_trace.csv && rm -rf $O/tr
python scripts/gossip_window_breakdown.py $O/kernel_trace.csv > $O/breakdown.txt 2>&1
gzip -f $O/kernel_trace.csv
head -30 $O/breakdown.txt
