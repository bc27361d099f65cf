#!/bin/bash
# Occupancy A/B: k_sim_fused with a smaller LDS queue (libtgsim_capN.so, -DTGSIM_FUSED_CAP=N) against
# the default build, both at a netem limit that fits N.
O=gpurun_out/r03/cap_ab
mkdir -p $O
for rep in 1 2; do
  for v in "base 500" "cap512 500" "base 250" "cap256 250"; do
    set -- $v
    lib=testground_amd/libtgsim.so; [ $1 != base ] && lib=testground_amd/libtgsim_$1.so
    TGSIM_LIB=$PWD/$lib timeout -k 10 300 python bench.py --no-cpu --no-1m --queue-limit $2 > $O/b_$1_$2_$rep.json 2> $O/b_$1_$2_$rep.err || { echo "bench $v failed"; tail $O/b_$1_$2_$rep.err; exit 1; }
    python -c "import json;d=json.load(open('$O/b_$1_$2_$rep.json'));print('$1 ql $2', round(d['value']/1e9,3),'G pkt/s', round(d['ms_per_step'],4),'ms/step kernel',round(d['roofline']['kernel_ms_avg'],4))"
  done
done
