cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/sh
timeout -k 10 400 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_stepper.py -x -v --timeout 300 --timeout-method thread > gpurun_out/sh/pytest.log 2>&1
rc=$?; tail -15 gpurun_out/sh/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in 1 8; do
  TGSIM_SHARD_FUSE=$v timeout -k 10 300 python bench.py --sharded --no-1m --no-cpu > gpurun_out/sh/b$v.json 2> gpurun_out/sh/b$v.err || { tail gpurun_out/sh/b$v.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/sh/b$v.json')); r=d['roofline']; print('sharded fuse $v', round(d['value']/1e9,2), 'G pkt/s', round(d['ms_per_step'],4), 'ms/step k_sim', round(r['kernel_ms_avg'],4), 'frac', round(r['frac'],4))"
done
