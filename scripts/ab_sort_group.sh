cd $GRAFT_REPO_ROOT; O=gpurun_out/abg2; mkdir -p $O
for rep in 1 2; do for v in 8 16 64; do
TGSIM_SORT_GROUP_MAX=$v timeout -k 10 300 python bench.py --workload gossip --peers 1000000 --no-cpu > $O/b.json 2> $O/b.err || { tail $O/b.err; exit 1; }
python -c "import json; d=json.load(open('$O/b.json')); r=d['roofline']; print('group_max $v', round(d['value']/1e9,3), 'G pkt/s', round(d['ms_per_step'],4), 'ms/step k_sim', round(r['kernel_ms_avg'],4))"
done; done
