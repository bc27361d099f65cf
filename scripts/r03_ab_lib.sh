#!/bin/bash
# A/B of two engine libraries on one workload, interleaved: LIBS="base cur" WL="epochs" scripts/r03_ab_lib.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/ablib; mkdir -p $O
for rep in 1 2; do
  for l in ${LIBS:-base cur}; do
    lib=$PWD/testground_amd/libtgsim.so; [ "$l" != cur ] && lib=$PWD/testground_amd/libtgsim_$l.so
    for wl in ${WL:-epochs}; do
      TGSIM_LIB=$lib timeout -k 10 300 python bench.py --workload $wl --no-cpu --no-1m ${BENCH_ARGS} > $O/b.json 2> $O/b.err || { tail $O/b.err; exit 1; }
      python -c "import json; d=json.load(open('$O/b.json')); r=d['roofline']; print('$l $wl', round(d['value']/1e9,3), 'G pkt/s', round(d['ms_per_step'],4), 'ms/step sim', round(r['kernel_ms_avg'],4))"
    done
  done
done
