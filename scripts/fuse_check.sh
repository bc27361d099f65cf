#!/bin/bash
# Fused windows: parity tests, then the storm bench with 1 (no fusion), 2 and 4 windows per launch.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/fuse
O=gpurun_out/fuse
timeout -k 10 400 python -u -m pytest tests/test_gpu_fused.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -8 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for f in ${FUSES:-1 4 2}; do
  TGSIM_FUSE=$f timeout -k 10 300 python bench.py --no-1m --no-cpu > $O/bench_f$f.json 2> $O/bench_f$f.err || { tail $O/bench_f$f.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_f$f.json')); r=d['roofline']; print('fuse $f', round(d['value']/1e9,2), 'G pkt/s', round(d['ms_per_step'],4), 'ms/step k_sim', round(r['kernel_ms_avg'],4), 'frac', round(r['frac'],4))"
done
