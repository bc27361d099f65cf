#!/bin/bash
# A/B of library variants (testground_amd/libtgsim_<v>.so, "cur" = libtgsim.so) on bench argument
# lists: BENCHES=';'-separated, VARIANTS=space-separated.  One bench line summary per run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/abw
IFS=';' read -r -a runs <<< "$BENCHES"
for args in "${runs[@]}"; do
  for v in $VARIANTS; do
    lib=testground_amd/libtgsim_$v.so; [ "$v" = cur ] && lib=testground_amd/libtgsim.so
    TGSIM_LIB=$PWD/$lib timeout -k 10 300 python bench.py --no-cpu $args > gpurun_out/abw/out.json 2> gpurun_out/abw/err.log || { tail -5 gpurun_out/abw/err.log; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/abw/out.json')); print('$v', '$args', round(d['value']/1e9,3), round(d['ms_per_step'],4), round(d['roofline']['kernel_ms_avg'],4), d['steps'])"
  done
done
