#!/bin/bash
# A/B of engine environment settings on the 1M-peer gossip bench (VARIANTS as ab_env_bench.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/abeg; mkdir -p $O
for rep in 1 2; do
  for v in $VARIANTS; do
    timeout -k 10 300 env ${v//,/ } python bench.py --workload gossip --peers 1000000 --no-cpu > $O/b.json 2> $O/b.err || { tail $O/b.err; exit 1; }
    python -c "import json; d=json.load(open('$O/b.json')); r=d['roofline']; print('$v', round(d['value']/1e9,3), 'G pkt/s', round(d['ms_per_step'],4), 'ms/step k_sim', round(r['kernel_ms_avg'],4))"
  done
done
