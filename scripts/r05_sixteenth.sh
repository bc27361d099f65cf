#!/bin/bash
# Round-5 sixteenth GPU call: the bucketed sort with 16 lanes per destination (several bucket entries
# per lane) and the total check folded into the scatter and the sort (no k_deliver_guard dispatch),
# against the previous commit's tree; parity first.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05/sixteenth; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|error" $O/pytest_gpu.log | head -20; exit 1; }
REPS=3 AB=sixteenth_gossip VARIANTS="cur tree:bisect/c7b3020" bash scripts/r05_gossip_ab.sh || exit 1
TAG=gossip_trace_l16 bash scripts/r05_gossip_trace.sh || exit 1
