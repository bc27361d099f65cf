#!/bin/bash
# Round-5: the default bench line twice at the final tree (no profiler).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05/lines; mkdir -p $O
for r in 1 2; do
  timeout -k 10 600 python -u bench.py > $O/bench_$r.json 2> $O/bench_$r.err || { echo "bench $r failed"; tail -5 $O/bench_$r.err; exit 1; }
  python scripts/line_summary.py $O/bench_$r.json
done
