#!/bin/bash
# Round evidence for one storm variant (SHAPES=storm|open): optional GPU parity tests and smoke
# (TESTS=1), the bench line with its CPU baseline, a rocprofv3 kernel trace of the bench, and the
# PMC passes of k_sim's HBM traffic and wave counters.  Output under gpurun_out/ev_$SHAPES/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
SHAPES=${SHAPES:-storm}
O=gpurun_out/ev_$SHAPES
mkdir -p $O
export TMPDIR=/tmp
set -o pipefail
if [ "${TESTS:-0}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log
  [ $rc -le 1 ] || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
  tail -1 $O/smoke.log
fi
B="--shapes $SHAPES --no-1m"
timeout -k 10 600 python bench.py $B ${BENCH_ARGS} > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
tail -c 400 $O/bench.json; echo
rm -rf $O/trace
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py $B --no-cpu > $O/trace.log 2>&1 || { tail $O/trace.log; exit 1; }
python scripts/trace_summary.py "$(find $O/trace -name "*kernel_trace.csv" | head -1)" 30 > $O/k_sim_timed.json && cat $O/k_sim_timed.json
rm -rf $O/pmc && mkdir -p $O/pmc
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY"; do
  i=$((i+1))
  timeout -k 10 600 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $O/pmc/p$i -o run -- python3 bench.py $B --no-cpu --steps 8 --warmup 8 > $O/pmc/p$i.log 2>&1 || { tail $O/pmc/p$i.log; exit 1; }
  echo "pmc pass $i ok"
done
LAM=$(python -c "import json; print(json.load(open('$O/bench.json'))['config']['lambda_per_tick'])")
python scripts/pmc_summary.py $O/pmc 8 10000 $LAM 2000 $SHAPES > $O/pmc_k_sim.json && cat $O/pmc_k_sim.json
