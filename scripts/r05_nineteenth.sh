#!/bin/bash
# Round-5 nineteenth GPU call: three emit/bucket sets in rotation (a window's delivery may lag until
# window k + 3 starts); parity, then A/B against two sets (TGSIM_EMIT_SETS=2) on the 1M-peer gossip,
# the sub-capacity storm and C5 epochs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05/nineteenth; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|error" $O/pytest_gpu.log | head -20; exit 1; }
REPS=3 AB=nineteenth_gossip VARIANTS="cur TGSIM_EMIT_SETS=2" bash scripts/r05_gossip_ab.sh || exit 1
AB=nineteenth_open ARGS="--no-cpu --no-1m --no-variants --shapes open" VARIANTS="cur TGSIM_EMIT_SETS=2" bash scripts/r05_gossip_ab.sh || exit 1
AB=nineteenth_epochs ARGS="--no-cpu --workload epochs --steps 30" VARIANTS="cur TGSIM_EMIT_SETS=2" bash scripts/r05_gossip_ab.sh || exit 1
TAG=gossip_trace_3sets bash scripts/r05_gossip_trace.sh || exit 1
