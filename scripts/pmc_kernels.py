"""Sums each PMC counter of a rocprofv3 counter_collection.csv per kernel name (all dispatches) and
prints, per kernel, dispatches and the counter's total and mean per dispatch."""
import csv
import sys
from collections import defaultdict

tot = defaultdict(lambda: defaultdict(float))
disp = defaultdict(set)
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"].split("(")[0]
    tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
    disp[k].add(r["Dispatch_Id"])
for k in sorted(tot, key=lambda k: -max(tot[k].values())):
    n = len(disp[k])
    print(f"{k[:48]:48s} {n:5d} " + "  ".join(f"{c} {v:.4g} ({v / n:.4g}/disp)" for c, v in sorted(tot[k].items())))
