#!/bin/bash
# Gossip window work (round 3): gossip parity tests, A/B of engine settings on the 1M-peer bench,
# then a kernel trace with the per-window breakdown.  usage: VARIANTS="A=1 A=0" scripts/r03_gossip_ab.sh [notest]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03g; rm -rf $O; mkdir -p $O
if [ "$1" != notest ]; then
  timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ \
    > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
  tail -3 $O/pytest.log
fi
for rep in 1 2; do
  for v in ${VARIANTS:-BASE=1}; do
    timeout -k 10 300 env ${v//,/ } python bench.py --workload gossip --peers 1000000 --no-cpu > $O/b.json 2> $O/b.err || { tail $O/b.err; exit 1; }
    python -c "import json; d=json.load(open('$O/b.json')); r=d['roofline']; print('$v', round(d['value']/1e9,3), 'G pkt/s', round(d['ms_per_step'],4), 'ms/step sim', round(r['kernel_ms_avg'],4))"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python3 bench.py --workload gossip --peers 1000000 --no-cpu --steps 70 > $O/tr.log 2>&1 || { tail $O/tr.log; exit 1; }
cp $(find $O/tr -name "*kernel_trace.csv" | head -1) $O/kernel_trace.csv && rm -rf $O/tr
python scripts/gossip_window_breakdown.py $O/kernel_trace.csv > $O/breakdown.txt 2>&1
gzip -f $O/kernel_trace.csv
head -24 $O/breakdown.txt
# one GPU's share of C4 (125k peers): single engine vs the engine's own exchange at one rank
for sh in "" --sharded; do
  timeout -k 10 300 python bench.py --workload gossip --peers 125000 --no-cpu $sh > $O/b125.json 2> $O/b125.err || { tail $O/b125.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b125.json')); r=d['roofline']; print('125k $sh', round(d['value']/1e9,3), 'G pkt/s', round(d['ms_per_step'],4), 'ms/step sim', round(r['kernel_ms_avg'],4))"
done
# the C3 headline beside it (no regression of the dense path)
if [ -n "$STORM" ]; then
  timeout -k 10 300 python bench.py --no-cpu --no-1m > $O/storm.json 2> $O/storm.err || { tail $O/storm.err; exit 1; }
  python -c "import json; d=json.load(open('$O/storm.json')); r=d['roofline']; print('storm', round(d['value']/1e9,3), 'G pkt/s', round(d['ms_per_step'],4), 'ms/step k_sim', round(r['kernel_ms_avg'],4))"
fi
