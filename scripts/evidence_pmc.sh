#!/bin/bash
# PMC passes (FETCH_SIZE, WRITE_SIZE; then the wave counters) of one workload of the default bench
# line, each pass its own rocprofv3 run with the kernel trace only (MI355X_MICROARCH.md §HBM),
# summarized for the simulate kernels (pmc_summary.py) and the delivery kernels (pmc_delivery.py);
# the summaries carry the kernel source's sha16, which bench.py checks before it quotes them.
#   WL=storm|open|epochs|gossip scripts/evidence_pmc.sh      -> gpurun_out/r06/pmc_$WL/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
WL=${WL:-storm}
case $WL in
  gossip) B="--workload gossip --peers 1000000 --no-cpu"; STEPS=70; PEERS=1000000; LAM=0.5; WIN=5000; SH=gossip;;
  storm) B="--no-1m --no-variants --no-cpu --steps 8 --warmup 8"; STEPS=8; PEERS=10000; LAM=0.5; WIN=2000; SH=storm;;
  open) B="--no-1m --no-variants --no-cpu --shapes open --steps 8 --warmup 8"; STEPS=8; PEERS=10000; LAM=0.008; WIN=2000; SH=open;;
  epochs) B="--workload epochs --no-cpu --steps 8 --warmup 3"; STEPS=8; PEERS=100000; LAM=0.2; WIN=1000; SH=epochs;;
esac
O=gpurun_out/r06/pmc_$WL; rm -rf $O; mkdir -p $O
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $O/p$i -o run -- python3 bench.py $B > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
done
python scripts/pmc_summary.py $O $STEPS $PEERS $LAM $WIN $SH > $O/pmc_k_sim.json
python scripts/pmc_delivery.py $O $STEPS $PEERS $LAM $WIN $SH $([ $WL = storm ] && echo 8) > $O/pmc_delivery.json
python - $O <<'PY'
import json, sys
o = sys.argv[1]
a = json.load(open(f"{o}/pmc_k_sim.json")); d = json.load(open(f"{o}/pmc_delivery.json"))
c = a["counters_avg_per_launch"]
w = (c.get("SQ_WAIT_ANY", 0) / c["SQ_WAVE_CYCLES"]) if c.get("SQ_WAVE_CYCLES") else None
print(o, "sim MB/window", round((a["hbm_bytes_per_launch"] or 0) / 1e6, 1), "delivery MB/window",
      round((d["hbm_bytes_per_launch"] or 0) / 1e6, 1), "wait ratio", w and round(w, 3))
PY
rm -rf $O/p*/  # the raw traces stay on the box; the summaries and logs come back
