#!/bin/bash
# Round-5 thirteenth GPU call: parity of this tree (product build), the TGSIM_CHECK build over every
# GPU test, then the default bench line (headline, at_1M_peers, at_subcapacity, at_epochs, CPU legs).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05/thirteenth; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|error" $O/pytest_gpu.log | head -20; exit 1; }
bash scripts/r05_check_build.sh; echo "check rc=$?"
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
python scripts/line_summary.py $O/bench.json
