#!/bin/bash
# Kernel trace of the 1M-peer gossip windows (bench --workload gossip) for a per-window timeline.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp; O=gpurun_out/gtr; rm -rf $O; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/tr -o run -- python3 bench.py --workload gossip --peers 1000000 --no-cpu --steps 70 > $O/tr.log 2>&1 || { tail $O/tr.log; exit 1; }
cp $(find $O/tr -name "*kernel_trace.csv" | head -1) $O/kernel_trace.csv
cp $(find $O/tr -name "*memory_copy_trace.csv" | head -1) $O/memory_copy_trace.csv 2>/dev/null
tail -c 300 $O/tr.log
