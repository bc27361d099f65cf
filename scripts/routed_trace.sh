#!/bin/bash
# Kernel trace of the routed step at one rank (TGSIM_COMM_ROUTE1=1, bench --sharded) for a workload:
#   WL=gossip125k|storm scripts/routed_trace.sh -> gpurun_out/rtr/kernel_trace.csv
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp; O=gpurun_out/rtr; rm -rf $O; mkdir -p $O
case ${WL:-gossip125k} in
  gossip125k) B="--workload gossip";;
  storm) B="--no-1m --no-variants";;
esac
TGSIM_COMM_ROUTE1=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python3 bench.py --sharded --no-cpu $B > $O/tr.log 2>&1 || { tail $O/tr.log; exit 1; }
cp $(find $O/tr -name "*kernel_trace.csv" | head -1) $O/kernel_trace.csv
tail -c 300 $O/tr.log
