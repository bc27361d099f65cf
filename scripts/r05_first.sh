#!/bin/bash
# Round-5 first GPU call: pytest -m gpu at HEAD (new: stopped-rank timeouts, late gossip windows
# queued ahead), the default bench line, then the 1M-peer gossip A/B of the sparse-kernel variants.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05/first; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|error" $O/pytest_gpu.log | head -20; exit 1; }
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail $O/bench.err; exit 1; }
python scripts/line_summary.py $O/bench.json
AB=first_ab VARIANTS="cur xcd w2x w4x nofwd hint xfh" bash scripts/r05_gossip_ab.sh
