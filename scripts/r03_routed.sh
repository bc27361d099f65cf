#!/bin/bash
# The routed N > 1 step timed at one rank (TGSIM_COMM_ROUTE1=1): gossip at one GPU's share of 1M at
# 8 GPUs (125k peers), storm and epochs through the engine's exchange.  Lines under gpurun_out/routed/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/routed; mkdir -p $O
export TGSIM_COMM_ROUTE1=1
for wl in "gossip --peers 125000" "storm --no-1m" "epochs --no-1m --peers 100000"; do
  n=${wl%% *}
  timeout -k 10 300 python bench.py --workload $wl --no-cpu --sharded > $O/$n.json 2> $O/$n.err || { tail $O/$n.err; exit 1; }
  python -c "import json; d=json.load(open('$O/$n.json')); print('$n', round(d['value']/1e9,3), 'G pkt/s', round(d['ms_per_step'],4), 'ms/step', d['config']['parallelism'], d['config'].get('exchange'))"
done
