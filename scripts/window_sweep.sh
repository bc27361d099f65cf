cd $GRAFT_REPO_ROOT
for w in 2000 4000 8000 2000 4000 8000; do
  timeout -k 10 300 python bench.py --no-cpu --window $w > gpurun_out/win_$w.json 2>gpurun_out/win_$w.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/win_$w.json'));print($w, round(d['value']/1e9,2),'G pkt/s', round(d['ms_per_step'],3),'ms/step k_sim',round(d['roofline']['kernel_ms_avg'],3),'frac',round(d['roofline']['frac'],4))"
done
