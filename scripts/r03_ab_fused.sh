#!/bin/bash
# A/B: source-major k_sim_fused (current; LPT order by measured chains, or by the last window's HTB
# records) against the r02 window-major one (libtgsim_r02.so): bench storm lines (interleaved,
# twice) and in-kernel stamps.
O=gpurun_out/r03/ab_fused${TAG}
mkdir -p $O
for rep in 1 2; do
  for v in ${VARIANTS:-r02 cur rec}; do
    lib=testground_amd/libtgsim.so; env=""
    [ $v = r02 ] && lib=testground_amd/libtgsim_r02.so
    [ $v = rec ] && env="TGSIM_FUSED_ORDER=records"
    env $env TGSIM_LIB=$PWD/$lib timeout -k 10 300 python bench.py --no-cpu --no-1m --steps 30 > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err || { echo "bench $v failed"; tail $O/bench_${v}_$rep.err; exit 1; }
    python -c "import json;d=json.load(open('$O/bench_${v}_$rep.json'));print('$v', round(d['value']/1e9,2),'G pkt/s', round(d['ms_per_step'],4),'ms/step k_sim',round(d['roofline']['kernel_ms_avg'],4))"
  done
done
timeout -k 10 300 python scripts/stamps_chains.py > $O/stamps_cur.log 2>&1 || { echo "stamps cur failed"; tail $O/stamps_cur.log; exit 1; }
cat $O/stamps_cur.log
