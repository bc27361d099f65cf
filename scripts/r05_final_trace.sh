#!/bin/bash
# Round-5 final evidence, part 2: rocprofv3 --kernel-trace --stats of the default bench command, and
# the TGSIM_CHECK build over every GPU test at the frozen kernel source.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05/final; rm -rf $O/tr; mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o run -- python3 bench.py > $O/bench_prof.json 2> $O/bench_prof.err || { tail $O/bench_prof.err; exit 1; }
cp $(find $O/tr -name "*kernel_stats.csv" | head -1) $O/kernel_stats.csv && rm -rf $O/tr
head -15 $O/kernel_stats.csv
bash scripts/r05_check_build.sh
