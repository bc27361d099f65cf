#!/bin/bash
# Round-4 evidence at the final kernel: parity tests + smoke, the storm headline's bench line with its
# CPU baseline, kernel trace and PMC passes (scripts/round_evidence.sh), then the 1M-peer gossip's
# (scripts/round_evidence_gossip.sh).  Every GPU step has its own time limit; the first failure stops it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04/evidence; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
SHAPES=storm bash scripts/round_evidence.sh || exit 1
bash scripts/round_evidence_gossip.sh || exit 1
