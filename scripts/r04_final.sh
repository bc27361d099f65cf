#!/bin/bash
# Round-4 final check at HEAD: pytest -m gpu, smoke, and the default bench line exactly as the
# driver runs it (no flags).  Every GPU step has its own time limit; the first failure stops it.
O=gpurun_out/r04/final; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed rc=$?"; tail $O/bench.err; exit 1; }
python - $O/bench.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
m = d.get("at_1M_peers") or {}
print(d["metric"], round(d["value"] / 1e9, 3), "G", d["unit"], "ms/step", round(d["ms_per_step"], 4), "frac", d["roofline"]["frac"],
      "traffic", d["roofline"].get("traffic"), "cpu", d["cpu_baseline"]["value"] if d.get("cpu_baseline") else None,
      "| 1M:", m and round(m["value"] / 1e9, 3), m and m["roofline"].get("traffic"))
PY
