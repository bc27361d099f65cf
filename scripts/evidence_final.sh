#!/bin/bash
# Final evidence at the frozen kernel source: rocprofv3 --kernel-trace --stats of the default bench
# command (its summary for profiles/), then the TGSIM_CHECK build over every GPU test.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06/final; rm -rf $O/tr; mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o run -- python3 bench.py > $O/bench_prof.json 2> $O/bench_prof.err || { tail $O/bench_prof.err; exit 1; }
cp "$(find $O/tr -name "*kernel_stats.csv" | head -1)" $O/kernel_stats.csv
python scripts/trace_summary.py "$(find $O/tr -name "*kernel_trace.csv" | head -1)" 20 > $O/k_sim_timed.json
rm -rf $O/tr
head -15 $O/kernel_stats.csv
[ "${CHECK:-1}" = 1 ] && bash scripts/check_build.sh
