#!/bin/bash
# Round-5 final evidence at the frozen kernel source: parity (product build), the TGSIM_CHECK build
# over every GPU test, PMC passes of the four workloads of the default line, rocprofv3 kernel-trace
# stats of the default bench command (its line is the one printed under the profiler).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05/final2; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|error" $O/pytest_gpu.log | head -20; exit 1; }
bash scripts/r05_check_build.sh || exit 1
for wl in storm gossip open epochs; do
  WL=$wl VARIANTS=cur bash scripts/r05_pmc.sh || { echo "pmc $wl failed"; exit 1; }
done
rm -rf $O/tr
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o run -- python3 bench.py > $O/bench_prof.json 2> $O/bench_prof.err || { tail $O/bench_prof.err; exit 1; }
cp $(find $O/tr -name "*kernel_stats.csv" | head -1) $O/kernel_stats.csv && rm -rf $O/tr
python scripts/line_summary.py $O/bench_prof.json
