#!/bin/bash
# Round-5 third GPU call: pytest -m gpu with the compact emit layout, the default bench line, then
# A/B: 1M-peer gossip (this tree, compact off, round 4's HEAD), the sub-capacity storm's delivery
# kernels (flattened vs per-destination sort, lane- vs wave-per-source scatter; round 2's tree), C3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05/third; mkdir -p $O
if [ "${TESTS:-1}" = 1 ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|error" $O/pytest_gpu.log | head -20; exit 1; }
fi
timeout -k 10 600 python -u -m pytest tests/test_gpu_multirank_fullsize.py -k c4 -v -s --timeout 900 --timeout-method thread > $O/pytest_c4_mem.log 2>&1 || { tail -20 $O/pytest_c4_mem.log; exit 1; }
grep -E "device memory|passed|failed" $O/pytest_c4_mem.log
timeout -k 10 600 python bench.py > $O/bench.json 2> >(tee $O/bench.err >&2) || { echo "bench failed"; tail $O/bench.err; exit 1; }
python scripts/line_summary.py $O/bench.json
AB=third_gossip VARIANTS="cur TGSIM_EMIT_COMPACT=0 tree:bisect/f8367ce" bash scripts/r05_gossip_ab.sh || exit 1
AB=third_open ARGS="--no-cpu --no-1m --shapes open" VARIANTS="cur TGSIM_SPARSE_SORT=1 TGSIM_LOCAL_SCATTER=2 tree:bisect/f6d001e" bash scripts/r05_gossip_ab.sh || exit 1
AB=third_storm ARGS="--no-cpu --no-1m --no-variants" VARIANTS="cur tree:bisect/f8367ce" bash scripts/r05_gossip_ab.sh || exit 1
