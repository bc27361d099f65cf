#!/bin/bash
# FETCH_SIZE / WRITE-free probe of scattered 16-B reads (scripts/fetch_probe.hip): one plain run,
# then a FETCH_SIZE pass; per-kernel counter totals into gpurun_out/r04/fetch_probe/.
O=gpurun_out/r04/fetch_probe
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 60 ./scripts/fetch_probe > $O/run.txt 2>&1 || exit 1
cat $O/run.txt
timeout -s KILL 60 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/pmc -o run -- ./scripts/fetch_probe > $O/pmc.log 2>&1 || { tail $O/pmc.log; exit 1; }
python3 - "$O" <<'PY'
import csv, glob, sys
from collections import defaultdict
tot = defaultdict(float)
for f in glob.glob(sys.argv[1] + "/pmc/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        tot[r["Kernel_Name"].split("(")[0]] += float(r["Counter_Value"])
for k, v in tot.items():
    print(f"{k}: FETCH_SIZE {v:.0f} KB -> x2 {2 * v * 1024 / 1e6:.1f} MB")
PY
