#!/bin/bash
# Round-3 first GPU call: TUN probe, full-size oracle digest tests, default bench line.
O=gpurun_out/r03/first
mkdir -p $O
(python scripts/probe_tun.py > $O/tun.json 2>&1 || echo "plain rc=$?" >> $O/tun.json)
(unshare -Urn python scripts/probe_tun.py >> $O/tun.json 2>&1 || echo "unshare rc=$?" >> $O/tun.json)
(ls -la /dev/net/ >> $O/tun.json 2>&1 || true)
timeout -k 10 900 python -u -m pytest -x -v --timeout 900 --timeout-method thread tests/test_gpu_fullsize_digests.py tests/test_bridge.py > $O/pytest.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 $O/pytest.log; exit 1; }
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed rc=$?"; tail -20 $O/bench.err; exit 1; }
echo done
