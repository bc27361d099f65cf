#!/bin/bash
# Round-5: kernel trace of the routed gossip step at one rank (TGSIM_COMM_ROUTE1=1, 125k peers).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05/routed_trace; rm -rf $O; mkdir -p $O
TGSIM_COMM_ROUTE1=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o run -- python3 bench.py --workload gossip --peers 125000 --sharded --no-cpu > $O/tr.json 2> $O/tr.err || { tail $O/tr.err; exit 1; }
cp $(find $O/tr -name "*kernel_trace.csv" | head -1) $O/kernel_trace.csv && cp $(find $O/tr -name "*kernel_stats.csv" | head -1) $O/kernel_stats.csv && rm -rf $O/tr
head -25 $O/kernel_stats.csv | cut -c1-160
gzip -f $O/kernel_trace.csv
