#!/bin/bash
# Round-5 twenty-second GPU call: parity of the tree to be frozen, A/B of the resident-grid sort on the
# gossip, sub-capacity and epochs runs, then the default bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05/twentysecond; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|error" $O/pytest_gpu.log | head -20; exit 1; }
REPS=3 AB=twentysecond_gossip VARIANTS="cur TGSIM_SORT_GRID=-1" bash scripts/r05_gossip_ab.sh || exit 1
AB=twentysecond_open ARGS="--no-cpu --no-1m --no-variants --shapes open" VARIANTS="cur TGSIM_SORT_GRID=-1" bash scripts/r05_gossip_ab.sh || exit 1
AB=twentysecond_epochs ARGS="--no-cpu --workload epochs --steps 30" VARIANTS="cur TGSIM_SORT_GRID=-1" bash scripts/r05_gossip_ab.sh || exit 1
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
python scripts/line_summary.py $O/bench.json
