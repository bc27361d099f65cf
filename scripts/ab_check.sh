#!/bin/bash
# A/B session: GPU parity tests of the current library, then, for each library variant
# (testground_amd/libtgsim_<v>.so for v in $VARIANTS, "cur" = libtgsim.so), bench (no CPU leg,
# run twice, interleaved) and in-kernel stamps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
stop() { echo "stopping after $1 (rc=$2)"; exit "$2"; }
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/ab/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/ab/pytest_gpu.log
  [ $rc -eq 0 ] || stop pytest $rc
fi
libof() { if [ "$1" = cur ]; then echo testground_amd/libtgsim.so; else echo testground_amd/libtgsim_$1.so; fi; }
for rep in 1 2; do
  for v in ${VARIANTS:-base cur}; do
    lib=$(libof $v)
    TGSIM_LIB=$PWD/$lib timeout -k 10 300 python bench.py --no-cpu --steps 20 ${BENCH_ARGS} > gpurun_out/ab/bench_${v}_$rep.json 2> gpurun_out/ab/bench_${v}_$rep.err || stop bench_$v $?
    python -c "import json;d=json.load(open('gpurun_out/ab/bench_${v}_$rep.json'));print('$v', round(d['value']/1e9,2),'G pkt/s', round(d['ms_per_step'],3),'ms/step k_sim',round(d['roofline']['kernel_ms_avg'],3),'frac',round(d['roofline']['frac'],4))"
  done
done
for v in ${VARIANTS:-base cur}; do
  TGSIM_LIB=$PWD/$(libof $v) timeout -k 10 300 python scripts/stamps.py --top 3 > gpurun_out/ab/stamps_$v.log 2>&1 || stop stamps_$v $?
  echo "== $v"; sed -n '2,9p' gpurun_out/ab/stamps_$v.log
done
if [ "${PROF:-0}" = 1 ]; then
  TGSIM_LIB=$PWD/testground_amd/libtgsim_prof.so timeout -k 10 300 python scripts/stamps.py > gpurun_out/ab/stamps_prof.log 2>&1 || stop stamps $?
  head -16 gpurun_out/ab/stamps_prof.log
fi
