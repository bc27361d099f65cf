#!/bin/bash
# Round evidence: GPU parity tests, smoke, bench line (with CPU baseline), rocprofv3 kernel trace of
# the bench, PMC passes for k_sim HBM traffic.  Output under gpurun_out/ev/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ev
export TMPDIR=/tmp
set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/ev/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/ev/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/ev/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/ev/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/ev/bench.json 2> gpurun_out/ev/bench.err || { tail gpurun_out/ev/bench.err; exit 1; }
tail -c 600 gpurun_out/ev/bench.json
rm -rf gpurun_out/ev/trace
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ev/trace -o run -- python3 bench.py --no-cpu > gpurun_out/ev/trace.log 2>&1 || { tail gpurun_out/ev/trace.log; exit 1; }
echo trace ok
python scripts/trace_summary.py gpurun_out/ev/trace/run_kernel_trace.csv k_sim 30 > gpurun_out/ev/k_sim_timed.json && cat gpurun_out/ev/k_sim_timed.json
rm -rf gpurun_out/ev/pmc && mkdir -p gpurun_out/ev/pmc
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY"; do
  i=$((i+1))
  timeout -k 10 600 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d gpurun_out/ev/pmc/p$i -o run -- python3 bench.py --no-cpu --steps 5 --warmup 1 > gpurun_out/ev/pmc/p$i.log 2>&1 || { tail gpurun_out/ev/pmc/p$i.log; exit 1; }
  echo "pmc pass $i ok"
done
python scripts/pmc_summary.py gpurun_out/ev/pmc 5 10000 0.5 2000 > gpurun_out/ev/pmc_k_sim.json && cat gpurun_out/ev/pmc_k_sim.json
