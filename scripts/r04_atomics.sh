#!/bin/bash
# Memory-side atomic requests per kernel of the 1M-peer gossip window (TCC_EA0_ATOMIC: every
# device-scope atomic executes at the memory side, MI355X_MICROARCH.md §Global float atomics), one
# PMC pass of its own; summed per kernel name over the bench's run (scripts/pmc_kernels.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04/atomics; mkdir -p $O
export TMPDIR=/tmp
B="--workload gossip --peers ${PEERS:-1000000} --no-cpu --no-1m"
rm -rf $O/p1
timeout -k 10 600 rocprofv3 --kernel-trace --pmc ${COUNTERS:-TCC_EA0_ATOMIC_sum TCC_EA0_WRREQ_sum} --output-format csv -d $O/p1 -o run -- python3 bench.py $B > $O/p1.log 2>&1 || { tail $O/p1.log; exit 1; }
python scripts/pmc_kernels.py "$(find $O/p1 -name '*counter_collection.csv' | head -1)" | tee $O/summary.txt
