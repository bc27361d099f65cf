#!/bin/bash
# Round-4 GPU check: parity tests (TESTS, default all of tests/), then bench lines (BENCHES: a
# ';'-separated list of bench.py argument sets, each run REPS times).  Every GPU step has its own
# time limit and the script stops at the first failure.
O=gpurun_out/r04/${TAG:-check}
mkdir -p $O
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 ${TEST_LIMIT:-900} python -u -m pytest -x -v -m gpu --timeout 900 --timeout-method thread \
    ${TESTS:-tests/} > $O/pytest_gpu.log 2>&1 || { rc=$?; echo "pytest failed rc=$rc"; tail -40 $O/pytest_gpu.log; exit 1; }
  tail -2 $O/pytest_gpu.log
fi
IFS=';' read -ra SETS <<< "${BENCHES:---no-cpu}"
i=0
for args in "${SETS[@]}"; do
  for rep in $(seq 1 ${REPS:-1}); do
    f=$O/bench_${i}_$rep
    timeout -k 10 ${BENCH_LIMIT:-400} python bench.py $args > $f.json 2> $f.err || { rc=$?; echo "bench '$args' failed rc=$rc"; tail $f.err; exit 1; }
    python - "$f.json" "$args" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d.get("roofline") or {}
m = d.get("at_1M_peers") or {}
print(sys.argv[2], "|", round(d["value"] / 1e9, 3), "G", round(d["ms_per_step"], 4), "ms/step frac",
      r.get("frac"), "kernel_ms", r.get("kernel_ms_avg"), "| 1M:", m and round(m["value"] / 1e9, 3))
EOF
  done
  i=$((i+1))
done
