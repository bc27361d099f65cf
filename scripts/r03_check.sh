#!/bin/bash
# GPU parity tests of the current library, then bench A/B variants (VARIANTS: r02 = libtgsim_r02.so,
# cur, sm = TGSIM_FUSED_MAJOR=source, or NAME=ENV pairs), interleaved twice.
O=gpurun_out/r03/check${TAG}
mkdir -p $O
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 900 --timeout-method thread ${TESTS:-tests/} > $O/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 $O/pytest_gpu.log; exit 1; }
  tail -2 $O/pytest_gpu.log
fi
for rep in 1 2; do
  for v in ${VARIANTS:-r02 cur sm}; do
    lib=testground_amd/libtgsim.so; env=""
    case $v in r02) lib=testground_amd/libtgsim_r02.so;; sm) env="TGSIM_FUSED_MAJOR=source";; cur) ;; *=*) env="$v";; esac
    tag=$(echo $v | tr '=' '_')
    env $env TGSIM_LIB=$PWD/$lib timeout -k 10 300 python bench.py --no-cpu ${BENCH_ARGS:---no-1m} > $O/bench_${tag}_$rep.json 2> $O/bench_${tag}_$rep.err || { echo "bench $v failed"; tail $O/bench_${tag}_$rep.err; exit 1; }
    python -c "import json;d=json.load(open('$O/bench_${tag}_$rep.json'));print('$v', round(d['value']/1e9,3),'G pkt/s', round(d['ms_per_step'],4),'ms/step kernel',round(d['roofline']['kernel_ms_avg'],4))"
  done
done
