#!/bin/bash
# A/B of engine environment settings on the current library: ENVS is a ';'-separated list of
# environment assignments ("-" for none); each runs the bench (BENCH_ARGS) twice, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/abe
IFS=';' read -r -a envs <<< "${ENVS:--}"
for rep in 1 2; do
  i=0
  for e in "${envs[@]}"; do
    i=$((i+1))
    [ "$e" = "-" ] && e=""
    env $e timeout -k 10 300 python bench.py --no-cpu --steps 30 ${BENCH_ARGS} > gpurun_out/abe/b_${i}_$rep.json 2> gpurun_out/abe/b_${i}_$rep.err || { echo "bench $e failed"; tail -5 gpurun_out/abe/b_${i}_$rep.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/abe/b_${i}_$rep.json'));print('[$e]', round(d['value']/1e9,2),'G pkt/s', round(d['ms_per_step'],3),'ms/step sim',round(d['roofline']['kernel_ms_avg'],3),'frac',round(d['roofline']['frac'],4))"
  done
done
