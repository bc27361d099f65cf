#!/bin/bash
# Round-5: the destination-slot atomic issued before the HTB scan (sparse and multi sources), against the previous library: the routed
# gossip at 125k peers (one rank) and the 1M-peer single engine; full parity first.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05/early_atomic_ab; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|error" $O/pytest.log | head -20; exit 1; }
for rep in 1 2 3; do
  for v in cur prev; do
    lib=$PWD/testground_amd/libtgsim.so; [ $v = prev ] && lib=$PWD/testground_amd/libtgsim_prev.so
    TGSIM_LIB=$lib TGSIM_COMM_ROUTE1=1 timeout -k 10 240 python bench.py --no-cpu --sharded --workload gossip --peers 125000 > $O/r125_${v}_$rep.json 2> $O/r125_${v}_$rep.err || { echo "r125 $v failed"; tail -5 $O/r125_${v}_$rep.err; exit 1; }
    python -c "import json;d=json.loads(open('$O/r125_${v}_$rep.json').read().strip().splitlines()[-1]);print('routed125k $v', round(d['value']/1e9,3), 'G pkt/s', round(d['ms_per_step'],4))"
    TGSIM_LIB=$lib timeout -k 10 240 python bench.py --no-cpu --no-1m --workload gossip --peers 1000000 > $O/g1m_${v}_$rep.json 2> $O/g1m_${v}_$rep.err || { echo "g1m $v failed"; tail -5 $O/g1m_${v}_$rep.err; exit 1; }
    python -c "import json;d=json.loads(open('$O/g1m_${v}_$rep.json').read().strip().splitlines()[-1]);print('gossip1M $v', round(d['value']/1e9,3), 'G pkt/s', round(d['ms_per_step'],4))"
  done
done
