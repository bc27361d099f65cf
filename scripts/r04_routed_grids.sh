O=gpurun_out/r04/grids; mkdir -p $O
for rep in 1 2; do for g in 0 80 90 1; do
  TGSIM_COMM_ROUTE1=1 TGSIM_FUSED_PERSIST=$g timeout -k 10 240 python bench.py --no-cpu --sharded --no-1m > $O/g${g}_$rep.json 2> $O/g${g}_$rep.err || { echo fail; tail $O/g${g}_$rep.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/g${g}_$rep.json').read().strip().splitlines()[-1]);print('grid $g', round(d['value']/1e9,3), round(d['ms_per_step'],4), round(d['roofline']['kernel_ms_avg'],4))"
done; done
