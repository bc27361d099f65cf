#!/bin/bash
# Kernel trace of the sharded storm (one rank, RCCL path, fused slotted groups) for a timeline.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp; O=gpurun_out/shtr; rm -rf $O; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/tr -o run -- python3 bench.py --sharded --no-1m --no-cpu --steps 24 --warmup 8 > $O/tr.log 2>&1 || { tail $O/tr.log; exit 1; }
cp $(find $O/tr -name "*kernel_trace.csv" | head -1) $O/kernel_trace.csv
cp $(find $O/tr -name "*memory_copy_trace.csv" | head -1) $O/memory_copy_trace.csv 2>/dev/null; echo ok
