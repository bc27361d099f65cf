#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprof kernel trace.  Each GPU step has its own time
# limit; a crash/abort/timeout stops the script (no further GPU work in the same call).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { # rc 0 = pass, 1 = test failures (keep going), anything else = stop
  local rc=$1; local what=$2
  echo "$what rc=$rc"
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "stopping after $what"; exit "$rc"; fi
}
STEPS="${STEPS:-all}"
if [[ "$STEPS" == *test* || "$STEPS" == all ]]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
  ok $? pytest; tail -30 gpurun_out/pytest_gpu.log
fi
if [[ "$STEPS" == *smoke* || "$STEPS" == all ]]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
  ok $? smoke; tail -5 gpurun_out/smoke.log
fi
if [[ "$STEPS" == *bench* || "$STEPS" == all ]]; then
  timeout -k 10 600 python bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
  ok $? bench; tail -5 gpurun_out/bench.log
fi
if [[ "$STEPS" == *prof* || "$STEPS" == all ]]; then
  rm -rf gpurun_out/prof
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --no-cpu --steps 5 --warmup 2 ${PROF_ARGS} > gpurun_out/prof.log 2>&1
  ok $? rocprof; tail -3 gpurun_out/prof.log
  find gpurun_out/prof -name "*stats*" | head
fi
