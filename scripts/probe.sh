#!/bin/bash
# k_sim bottleneck probes: one bench line per variant (kernel time in roofline.kernel_ms_avg).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for args in "" "--queue-limit 64" "--shapes fixed" "--lam 0.05" "--window 500" "--peers 60000 --window 500"; do
  timeout -k 10 300 python bench.py --no-cpu --steps 5 --warmup 2 $args > gpurun_out/probe.log 2>&1
  rc=$?
  echo "== $args rc=$rc"
  python -c "
import json,sys
l=[x for x in open('gpurun_out/probe.log') if x.startswith('{')]
if l:
  r=json.loads(l[-1]); print('value %.3g pkt/s  step %.2f ms  k_sim %.2f ms  pkts/step %.3g  sched %s' % (r['value'], r['ms_per_step'], r['roofline']['kernel_ms_avg'], r['config']['packets_per_step'], r['roofline']['algorithmic_bytes_per_launch']))
else: print(open('gpurun_out/probe.log').read()[-2000:])
"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
