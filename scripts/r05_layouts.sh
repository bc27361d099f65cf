#!/bin/bash
# Round-5: the parity test over the delivery-layout switches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05/layouts; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "layouts or gossip" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -12 $O/pytest.log
exit $rc
