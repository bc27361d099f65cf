#!/bin/bash
# Round-5 first GPU call: pytest -m gpu at HEAD (new: stopped-rank timeouts, late gossip windows
# queued ahead), the sub-capacity bisect, and the default bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05/first; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|error" $O/pytest_gpu.log | head -20; exit 1; }
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail $O/bench.err; exit 1; }
python - $O/bench.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
m = d.get("at_1M_peers") or {}
print("C3", round(d["value"] / 1e9, 3), "ms", round(d["ms_per_step"], 4), "frac", round(d["roofline"]["frac"], 4),
      "| 1M:", round(m["value"] / 1e9, 3), "ms", round(m["ms_per_step"], 4), "frac", round(m["roofline"]["frac"], 4))
PY
bash scripts/r05_bisect_open.sh
