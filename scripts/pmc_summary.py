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
FUSE = 8  # bench.py's storm windows run through tgsim_step_n: groups of at most 8 per k_sim_fused dispatch
vals = defaultdict(dict)
FIRST = ("k_sim(", "k_sim_sparse(", "k_sim_fused(")  # one opens every dispatch group; k_sim_list joins the sparse one
for f in glob.glob(f"{root}/p*/**/*counter_collection.csv", recursive=True):
    per = defaultdict(lambda: defaultdict(float))
    name = {}
    for r in csv.DictReader(open(f)):
        if any(k in r["Kernel_Name"] for k in FIRST + ("k_sim_list(", "k_sim_multi(")):
            per[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
            name[int(r["Dispatch_Id"])] = r["Kernel_Name"]
    step = []  # counters summed per dispatch group, in dispatch order, with its window count
    for i in sorted(per):
        if any(k in name[i] for k in FIRST) or not step:
            step.append([defaultdict(float), "k_sim_fused(" in name[i]])
        for k, v in per[i].items():
            step[-1][0][k] += v
    # the timed windows: groups of FUSE, then the remainder (tgsim_step_n); a group of w windows
    # counts w times, with 1/w of its counters each
    fused = any(f for _, f in step)  # per-window dispatches otherwise (sparse steps, gossip)
    groups = [FUSE] * (steps // FUSE) + ([steps % FUSE] if steps % FUSE else []) if fused else [1] * steps
    for (sv, _), w in zip(reversed(step), reversed(groups)):
        for k, v in sv.items():
            vals[k].setdefault("v", []).extend([v / w] * w)
avg = {k: sum(d["v"]) / len(d["v"]) for k, d in vals.items()}
out = {"kernel": "tgsim::k_sim | k_sim_fused (dense windows) | k_sim_sparse + k_sim_multi + k_sim_list (sparse windows), per window", "counters_avg_per_launch": avg,
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
