#!/bin/bash
# A/B of the 1M-peer gossip window (round 5): libraries (testground_amd/libtgsim_<v>.so, "cur" =
# libtgsim.so), engine environment settings (NAME=VALUE) or another tree's own bench and library
# (tree:DIR, e.g. tree:bisect/f8367ce = round 4's HEAD), interleaved, two runs each.
# Output under gpurun_out/r05/$AB.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=$PWD/gpurun_out/r05/${AB:-gossip_ab}; mkdir -p $O
ARGS=${ARGS:-"--no-cpu --no-1m --workload gossip --peers ${PEERS:-1000000}"}
for rep in $(seq 1 ${REPS:-2}); do
  for v in ${VARIANTS:-cur}; do
    lib=$PWD/testground_amd/libtgsim.so; env=TGSIM_X=0; dir=.
    case $v in cur) ;; tree:*) dir=${v#tree:}; lib=$PWD/$dir/testground_amd/libtgsim.so;; *=*) env=$v;; *) lib=$PWD/testground_amd/libtgsim_$v.so;; esac
    tag=$(echo $v | tr '=:/' '___')
    targs=$ARGS; case $v in tree:*) targs=${ARGS//--no-variants/};; esac  # older trees lack the flag
    ( cd $dir && env $env TGSIM_LIB=$lib timeout -k 10 300 python bench.py $targs > $O/${tag}_$rep.json 2> $O/${tag}_$rep.err ) || { echo "$v failed"; tail $O/${tag}_$rep.err; exit 1; }
    python -c "import json;d=json.loads(open('$O/${tag}_$rep.json').read().strip().splitlines()[-1]);print('$v', round(d['value']/1e9,3), 'G pkt/s', round(d['ms_per_step'],4), 'ms/step sim', round(d['roofline']['kernel_ms_avg'],4))"
  done
done
