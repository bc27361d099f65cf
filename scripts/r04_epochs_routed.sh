#!/bin/bash
# C5 epochs through the routed path at one rank (TGSIM_COMM_ROUTE1=1) beside the single engine,
# REPS runs each (routed >= 11.5 G pkt/s).
O=gpurun_out/r04/${TAG:-epochs_routed}; mkdir -p $O
for rep in $(seq 1 ${REPS:-2}); do
  for mode in routed single; do
    if [ $mode = routed ]; then E=TGSIM_COMM_ROUTE1=1; X=--sharded; else E=TGSIM_X=0; X=; fi
    env $E timeout -k 10 240 python bench.py --no-cpu --workload epochs $X > $O/${mode}_$rep.json 2> $O/${mode}_$rep.err || { echo "$mode failed rc=$?"; tail -5 $O/${mode}_$rep.err; exit 1; }
    python -c "import json;d=json.loads(open('$O/${mode}_$rep.json').read().strip().splitlines()[-1]);print('$mode', round(d['value']/1e9,3), 'G pkt/s', round(d['ms_per_step'],4), 'ms/step')"
  done
done
