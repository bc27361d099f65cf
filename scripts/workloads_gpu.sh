#!/bin/bash
# C4 / C5 workloads on one GPU: parity tests, then one bench line per workload.  Each GPU step has
# its own time limit; a crash/abort/timeout stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() {
  local rc=$1; local what=$2
  echo "$what rc=$rc"
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "stopping after $what"; exit "$rc"; fi
}
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -x -q ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
  ok $? pytest; tail -15 gpurun_out/pytest_gpu.log
fi
# BENCHES: ';'-separated bench.py argument lists
IFS=';' read -r -a runs <<< "${BENCHES:---workload gossip --no-cpu;--workload epochs --no-cpu;--workload gossip --peers 1000000}"
for args in "${runs[@]}"; do
  tag=$(echo "$args" | tr -c 'a-zA-Z0-9' '_')
  timeout -k 10 900 python bench.py $args > "gpurun_out/bench_${tag}.log" 2>&1
  ok $? "bench $args"; tail -3 "gpurun_out/bench_${tag}.log"
done
