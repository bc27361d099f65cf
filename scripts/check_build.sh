#!/bin/bash
# pytest -m gpu once on the TGSIM_CHECK build of the engine (queue invariants and
# the cross-lane exec-mask guards of every readlane / DPP scan / wave shuffle: a read of an inactive
# lane prints "EXEC CHECK ..." and is counted).  The multi-rank tests load the test transport's
# library (product objects), so they run unchecked.  Log: gpurun_out/r06/check/pytest_gpu_check.log.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06/check; mkdir -p $O
TGSIM_LIB=$PWD/testground_amd/libtgsim_check.so timeout -k 10 900 python -u -m pytest tests -m gpu -v -s \
  --timeout 600 --timeout-method thread > $O/pytest_gpu_check.log 2>&1; rc=$?
tail -4 $O/pytest_gpu_check.log
echo "EXEC CHECK lines (one per source line): $(grep -c "EXEC CHECK" $O/pytest_gpu_check.log)"; grep "EXEC CHECK" $O/pytest_gpu_check.log | sort | uniq | head -40
echo "queue CHECK lines: $(grep -c '^CHECK tag' $O/pytest_gpu_check.log)"
grep -m1 "TGSIM_CHECK exec-mask guard violations" $O/pytest_gpu_check.log
exit $rc
