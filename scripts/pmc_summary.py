"""Turns the rocprofv3 PMC passes of scripts/pmc.sh into profiles/pmc_k_sim.json.

HBM bytes per step of the simulate kernels = 2 * FETCH_SIZE + WRITE_SIZE (KiB counters -> bytes); the factor 2 is
the gfx950 correction of MI355X_MICROARCH.md §HBM (FETCH_SIZE reports half of a wide coalesced
read).  Only the last `steps` k_sim dispatches (the bench's timed steps) are averaged."""
import csv
import glob
import json
import hashlib
import subprocess
import sys
from collections import defaultdict
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]

root, steps = sys.argv[1], int(sys.argv[2])
vals = defaultdict(dict)
FIRST = ("k_sim(", "k_sim_sparse(")  # one of these opens every step; k_sim_list joins the sparse step
for f in glob.glob(f"{root}/p*/**/*counter_collection.csv", recursive=True):
    per = defaultdict(lambda: defaultdict(float))
    name = {}
    for r in csv.DictReader(open(f)):
        if any(k in r["Kernel_Name"] for k in FIRST + ("k_sim_list(",)):
            per[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
            name[int(r["Dispatch_Id"])] = r["Kernel_Name"]
    step = []  # counters summed per step, in dispatch order
    for i in sorted(per):
        if any(k in name[i] for k in FIRST) or not step:
            step.append(defaultdict(float))
        for k, v in per[i].items():
            step[-1][k] += v
    for sv in step[-steps:]:
        for k, v in sv.items():
            vals[k].setdefault("v", []).append(v)
avg = {k: sum(d["v"]) / len(d["v"]) for k, d in vals.items()}
out = {"kernel": "tgsim::k_sim (dense steps) | k_sim_sparse + k_sim_list (sparse steps), per step", "counters_avg_per_launch": avg,
       "hbm_bytes_per_launch": (2 * avg.get("FETCH_SIZE", 0) + avg.get("WRITE_SIZE", 0)) * 1024
       if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg else None,
       "fetch_correction": "x2 (gfx950 FETCH_SIZE counts 64 B per 128 B request)",
       "peers": int(sys.argv[3]), "lam": float(sys.argv[4]), "window": int(sys.argv[5]),
       "shapes": sys.argv[6] if len(sys.argv) > 6 else "storm",
       # provenance: bench.py reports this traffic only for the same k_sim source and configuration
       "kernel_sha16": hashlib.sha256((REPO / "testground_amd/csrc/tgsim_kernels.hip").read_bytes()).hexdigest()[:16],
       "commit": subprocess.run(["git", "-C", str(REPO), "rev-parse", "--short=12", "HEAD"], capture_output=True,
                                text=True).stdout.strip() or None}
print(json.dumps(out, indent=1))
