#!/bin/bash
# The routed N > 1 step timed at one rank (TGSIM_COMM_ROUTE1=1), VERDICT r03 items 3-4: gossip at
# one GPU's share of 1M peers, C5 epochs, and the C3 storm's slotted fused groups with the grid the
# N > 1 path uses (TGSIM_FUSED_PERSIST: 0 turnover, 1 persistent, NN = NN % of the resident grid).
# Each line: label, then the bench's JSON summary.  Every GPU step has its own time limit.
O=gpurun_out/r04/${TAG:-routed}
mkdir -p $O
run() {  # label env... -- bench args
  local label=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done
  shift
  env "${envs[@]}" timeout -k 10 240 python bench.py --no-cpu "$@" > $O/$label.json 2> $O/$label.err || { echo "$label failed rc=$?"; tail -5 $O/$label.err; exit 1; }
  python - "$O/$label.json" "$label" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d.get("roofline") or {}
print(sys.argv[2], round(d["value"] / 1e9, 3), "G pkt/s", round(d["ms_per_step"], 4), "ms/step kernel", r.get("kernel_ms_avg"))
PY
}
for rep in ${REPS_LIST:-1 2}; do
  run gossip125k_single_$rep TGSIM_X=0 -- --workload gossip --peers 125000
  run gossip125k_routed_$rep TGSIM_COMM_ROUTE1=1 -- --workload gossip --peers 125000 --sharded
  run epochs_single_$rep TGSIM_X=0 -- --workload epochs
  run epochs_routed_$rep TGSIM_COMM_ROUTE1=1 -- --workload epochs --sharded
  for g in ${GRIDS:-0 1 80}; do
    run storm_routed_grid${g}_$rep TGSIM_COMM_ROUTE1=1 TGSIM_FUSED_PERSIST=$g -- --sharded --no-1m
  done
done
