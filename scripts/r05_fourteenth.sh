#!/bin/bash
# Round-5 fourteenth GPU call: buckets of 8-64 records chosen per window; parity, A/B against the
# slot scatter (TGSIM_DST_BKT=0), kernel trace of the 1M-peer window.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05/fourteenth; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|error" $O/pytest_gpu.log | head -20; exit 1; }
AB=fourteenth_gossip VARIANTS="cur TGSIM_DST_BKT=0" bash scripts/r05_gossip_ab.sh || exit 1
AB=fourteenth_open ARGS="--no-cpu --no-1m --no-variants --shapes open" VARIANTS="cur TGSIM_DST_BKT=0" bash scripts/r05_gossip_ab.sh || exit 1
TAG=gossip_trace_bkt_adaptive bash scripts/r05_gossip_trace.sh || exit 1
