#!/bin/bash
# Kernel trace of the 1M-peer gossip bench (timeline per window: scripts/window_timeline.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04/trace2; mkdir -p $O
export TMPDIR=/tmp
rm -rf $O/t
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $O/t -o run -- python3 bench.py --workload gossip --peers 1000000 --no-cpu --no-1m > $O/t.log 2>&1 || { tail $O/t.log; exit 1; }
python scripts/window_timeline.py "$(find $O/t -name '*kernel_trace.csv' | head -1)" > $O/timeline.txt && tail -40 $O/timeline.txt
