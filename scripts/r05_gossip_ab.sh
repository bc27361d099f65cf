#!/bin/bash
# (round 5: output under gpurun_out/r05/$AB)
# A/B of the 1M-peer gossip window: libraries (testground_amd/libtgsim_<v>.so, "cur" = libtgsim.so) and
# engine environment settings (NAME=VALUE), interleaved, two runs each.
O=gpurun_out/r05/${AB:-gossip_ab}; mkdir -p $O
for rep in 1 2; do
  for v in ${VARIANTS:-cur}; do
    lib=testground_amd/libtgsim.so; env=TGSIM_X=0
    case $v in cur) ;; *=*) env=$v;; *) lib=testground_amd/libtgsim_$v.so;; esac
    tag=$(echo $v | tr '=' '_')
    env $env TGSIM_LIB=$PWD/$lib timeout -k 10 300 python bench.py --no-cpu --no-1m --workload gossip --peers ${PEERS:-1000000} > $O/${tag}_$rep.json 2> $O/${tag}_$rep.err || { echo "$v failed"; tail $O/${tag}_$rep.err; exit 1; }
    python -c "import json;d=json.loads(open('$O/${tag}_$rep.json').read().strip().splitlines()[-1]);print('$v', round(d['value']/1e9,3), 'G pkt/s', round(d['ms_per_step'],4), 'ms/step sim', round(d['roofline']['kernel_ms_avg'],4))"
  done
done
