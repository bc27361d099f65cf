#!/bin/bash
# Kernel-trace summary (per kernel: calls, mean, total) of one bench workload, for each library given:
# LIBS="base cur" WL=epochs scripts/r03_trace_wl.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp; O=gpurun_out/trwl; rm -rf $O; mkdir -p $O
for l in ${LIBS:-cur}; do
  lib=$PWD/testground_amd/libtgsim.so; [ "$l" != cur ] && lib=$PWD/testground_amd/libtgsim_$l.so
  TGSIM_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$l -o run -- python3 bench.py --workload ${WL:-epochs} --no-cpu --no-1m > $O/$l.log 2>&1 || { tail $O/$l.log; exit 1; }
  f=$(find $O/$l -name "*kernel_stats.csv" | head -1)
  echo "== $l"; python3 -c "
import pandas as pd; d=pd.read_csv('$f'); d['Name']=d['Name'].str.replace(r'^(void )?tgsim::','',regex=True).str.slice(0,40)
print(d[['Name','Calls','AverageNs','TotalDurationNs']].head(14).to_string(index=False))"
done
