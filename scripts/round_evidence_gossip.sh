#!/bin/bash
# Evidence of the 1M-peer gossip half of the metric (the at_1M_peers object of the default bench
# line): the bench line, a rocprofv3 kernel trace and the PMC passes of the simulate kernels
# (k_sim_sparse + k_sim_list per window).  Output under gpurun_out/ev_gossip/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/ev_gossip; mkdir -p $O
export TMPDIR=/tmp
set -o pipefail
B="--workload gossip --peers 1000000 --no-cpu"
timeout -k 10 600 python bench.py $B > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
tail -c 300 $O/bench.json; echo
rm -rf $O/trace
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py $B > $O/trace.log 2>&1 || { tail $O/trace.log; exit 1; }
python scripts/trace_summary.py "$(find $O/trace -name "*kernel_trace.csv" | head -1)" 70 > $O/k_sim_timed.json && cat $O/k_sim_timed.json
rm -rf $O/pmc && mkdir -p $O/pmc
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY"; do
  i=$((i+1))
  timeout -k 10 600 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $O/pmc/p$i -o run -- python3 bench.py $B > $O/pmc/p$i.log 2>&1 || { tail $O/pmc/p$i.log; exit 1; }
  echo "pmc pass $i ok"
done
python scripts/pmc_summary.py $O/pmc 70 1000000 0.5 5000 gossip > $O/pmc_k_sim_gossip.json && cat $O/pmc_k_sim_gossip.json
