#!/bin/bash
# Round-5 tenth GPU call: sparse windows written straight into destination buckets by the simulate
# kernels (no scatter pass for the records that fit; k_dst_sort_bkt orders them).  Parity (product
# build), then the TGSIM_CHECK build once (slot fallback from rank kBktC + 3, exec-mask guards), then
# A/B against the slot scatter (TGSIM_DST_BKT=0) and the cursors (TGSIM_DST_SLOT=0).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05/tenth; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|error" $O/pytest_gpu.log | head -20; exit 1; }
bash scripts/r05_check_build.sh || exit 1
AB=tenth_gossip VARIANTS="cur TGSIM_DST_BKT=0 TGSIM_DST_SLOT=0" bash scripts/r05_gossip_ab.sh || exit 1
AB=tenth_open ARGS="--no-cpu --no-1m --no-variants --shapes open" VARIANTS="cur TGSIM_DST_BKT=0 TGSIM_DST_SLOT=0" bash scripts/r05_gossip_ab.sh || exit 1
