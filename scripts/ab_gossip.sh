#!/bin/bash
# A/B of library variants on the 1M-peer gossip bench (VARIANTS: cur or <name> of libtgsim_<name>.so).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/abg; mkdir -p $O
libof() { if [ "$1" = cur ]; then echo testground_amd/libtgsim.so; else echo testground_amd/libtgsim_$1.so; fi; }
for rep in 1 2; do
  for v in $VARIANTS; do
    TGSIM_LIB=$PWD/$(libof $v) timeout -k 10 300 python bench.py --workload gossip --peers 1000000 --no-cpu > $O/b.json 2> $O/b.err || { tail $O/b.err; exit 1; }
    python -c "import json; d=json.load(open('$O/b.json')); r=d['roofline']; print('$v', round(d['value']/1e9,3), 'G pkt/s', round(d['ms_per_step'],4), 'ms/step k_sim', round(r['kernel_ms_avg'],4), 'frac', round(r['frac'],4))"
  done
done
