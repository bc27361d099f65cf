#!/bin/bash
# bisect the sub-capacity storm (--shapes open) regression, r02 1.29-1.38 ->
# r04 HEAD 1.15 G pkt/s.  Each commit's own tree (git worktrees under bisect/, built here with its
# own build.py) runs its own bench.py; two interleaved rounds.  Output: gpurun_out/r05/bisect/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=$PWD/gpurun_out/r05/bisect; mkdir -p $O
COMMITS=${COMMITS:-"f6d001e 0362bf1 c211684 ae9aa0a 7c96a29 7ff58ac 769e16c 77bbd37 d6e535a f8367ce HEAD"}
for round in 1 2; do
  for c in $COMMITS; do
    d=bisect/$c; [ "$c" = HEAD ] && d=.
    ( cd $d && timeout -k 10 240 python bench.py --shapes open --no-1m --no-cpu > $O/${c}_$round.json 2> $O/${c}_$round.err ) || { echo "FAIL $c rc=$?"; tail -5 $O/${c}_$round.err; exit 1; }
    python -c "import json,sys; d=json.loads(open('$O/${c}_$round.json').read().strip().splitlines()[-1]); print('$c', $round, round(d['value']/1e9,3), 'G', 'ms/step', round(d['ms_per_step'],4), 'k_sim', round(d['roofline']['kernel_ms_avg'],4))"
  done
done
