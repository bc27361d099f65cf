#!/bin/bash
# Round-3 GPU call: TUN probe, the whole -m gpu suite (incl. full-size oracle digests and the engine's
# own RCCL exchange), smoke, bench lines.
O=gpurun_out/r03/first
mkdir -p $O
(python scripts/probe_tun.py > $O/tun.json 2>&1 || echo "plain rc=$?" >> $O/tun.json)
(unshare -Urn python scripts/probe_tun.py >> $O/tun.json 2>&1 || echo "unshare rc=$?" >> $O/tun.json)
(ls -la /dev/net/ >> $O/tun.json 2>&1 || true)
timeout -k 10 900 python -u -m pytest -x -v -m gpu --timeout 900 --timeout-method thread tests/ > $O/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 $O/pytest_gpu.log; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail $O/smoke.log; exit 1; }
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed rc=$?"; tail -20 $O/bench.err; exit 1; }
timeout -k 10 300 python bench.py --sharded --no-1m --no-cpu > $O/bench_sharded.json 2> $O/bench_sharded.err || { echo "sharded bench failed rc=$?"; tail -20 $O/bench_sharded.err; exit 1; }
timeout -k 10 300 python bench.py --sharded --workload gossip --no-cpu > $O/bench_sharded_gossip.json 2> $O/bench_sharded_gossip.err || { echo "sharded gossip failed rc=$?"; tail -20 $O/bench_sharded_gossip.err; exit 1; }
timeout -k 10 300 python bench.py --workload gossip --no-cpu > $O/bench_gossip.json 2> $O/bench_gossip.err || { echo "gossip failed rc=$?"; tail -20 $O/bench_gossip.err; exit 1; }
echo done
