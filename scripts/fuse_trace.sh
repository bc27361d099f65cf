cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/fuse2; mkdir -p $O
for v in "TGSIM_FUSE=8" "TGSIM_FUSE=4"; do
  env $v timeout -k 10 300 python bench.py --no-1m --no-cpu > $O/b.json 2> $O/b.err || { tail $O/b.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b.json')); r=d['roofline']; print('$v', round(d['value']/1e9,2), 'G pkt/s', round(d['ms_per_step'],4), 'ms/step k_sim', round(r['kernel_ms_avg'],4), 'frac', round(r['frac'],4))"
done
rm -rf $O/tr; timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python3 bench.py --no-1m --no-cpu --steps 12 --warmup 0 > $O/tr.log 2>&1 || { tail $O/tr.log; exit 1; }
f=$(find $O/tr -name "*kernel_trace.csv" | head -1); cp $f $O/kernel_trace.csv; ls -la $O
