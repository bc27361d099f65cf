#!/bin/bash
# 1M-peer gossip: the deferred-source count of every sparse window (TGSIM_TRACE_LIST), then an A/B of
# the sparse/dense switch threshold (TGSIM_DENSE_DIV: dense when a sparse window deferred > S / div).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/dense; mkdir -p $O
TGSIM_TRACE_LIST=1 timeout -k 10 300 python bench.py --workload gossip --peers 1000000 --no-cpu > $O/trace.json 2> $O/trace.err || { tail $O/trace.err; exit 1; }
grep "deferred" $O/trace.err | awk '{print $5}' | tr '\n' ' '; echo
VARIANTS="TGSIM_DENSE_DIV=4 TGSIM_DENSE_DIV=8 TGSIM_DENSE_DIV=16 TGSIM_DENSE_DIV=1000000" bash scripts/ab_env_gossip.sh
