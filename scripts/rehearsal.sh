#!/bin/bash
# The driver's round-end sequence on this tree (built beforehand, here, by __graft_entry__.build()):
# pytest -m gpu, smoke(), then the default bench line twice.  -> gpurun_out/r06/rehearsal/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06/rehearsal; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
for i in 1 2; do
  timeout -k 10 600 python bench.py > $O/bench_$i.json 2> $O/bench_$i.err || { tail $O/bench_$i.err; exit 1; }
  python scripts/line_summary.py $O/bench_$i.json 2>/dev/null || tail -c 300 $O/bench_$i.json
done
