#!/bin/bash
# Round-5: the routed step at one rank (TGSIM_COMM_ROUTE1=1), this tree against the previous
# commit's library (libtgsim_prev.so): gossip at 125k peers, C5 epochs, storm; parity of the
# multi-rank and stepper tests first.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05/routed_ab; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_stepper.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|error" $O/pytest.log | head -20; exit 1; }
for rep in 1 2; do
  for v in cur prev; do
    lib=$PWD/testground_amd/libtgsim.so; [ $v = prev ] && lib=$PWD/testground_amd/libtgsim_prev.so
    for wl in "gossip125k --workload gossip --peers 125000" "epochs --workload epochs --steps 30" "storm --no-1m --no-variants"; do
      set -- $wl; tag=$1; shift
      TGSIM_LIB=$lib TGSIM_COMM_ROUTE1=1 timeout -k 10 240 python bench.py --no-cpu --sharded "$@" > $O/${tag}_${v}_$rep.json 2> $O/${tag}_${v}_$rep.err || { echo "$tag $v failed"; tail -5 $O/${tag}_${v}_$rep.err; exit 1; }
      python -c "import json;d=json.loads(open('$O/${tag}_${v}_$rep.json').read().strip().splitlines()[-1]);print('$tag $v', round(d['value']/1e9,3), 'G pkt/s', round(d['ms_per_step'],4))"
    done
  done
done
