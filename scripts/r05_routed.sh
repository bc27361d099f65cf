#!/bin/bash
# The routed N > 1 step timed at one rank (TGSIM_COMM_ROUTE1=1) beside the single engine, three
# runs each (C5 routed >= 12 G pkt/s within 10 %, gossip at 125k >= 2.9, storm
# >= 36).  Every GPU step has its own time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05/${TAG:-routed}; mkdir -p $O
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
for rep in ${REPS_LIST:-1 2 3}; do
  run gossip125k_single_$rep TGSIM_X=0 -- --workload gossip --peers 125000
  run gossip125k_routed_$rep TGSIM_COMM_ROUTE1=1 -- --workload gossip --peers 125000 --sharded
  run epochs_single_$rep TGSIM_X=0 -- --workload epochs --steps 30
  run epochs_routed_$rep TGSIM_COMM_ROUTE1=1 -- --workload epochs --sharded --steps 30
  run storm_routed_$rep TGSIM_COMM_ROUTE1=1 -- --sharded --no-1m --no-variants
done
