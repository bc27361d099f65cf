#!/bin/bash
# Kernel trace of the sub-capacity storm (bench --shapes open) for a per-window timeline.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp; O=gpurun_out/otr; rm -rf $O; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python3 bench.py --shapes open --no-cpu --no-1m --no-variants --steps 30 ${EXTRA} > $O/tr.log 2>&1 || { tail $O/tr.log; exit 1; }
cp $(find $O/tr -name "*kernel_trace.csv" | head -1) $O/kernel_trace.csv
tail -c 300 $O/tr.log
