"""Turns rocprofv3 PMC passes into profiles/pmc_delivery_<tag>.json: HBM bytes per window of the
delivery (K5) kernels -- the local scatter (k_local_scatter_ls / k_local_scatter) or the inbound
histogram + scatter (k_dst_hist/k_dst_scatter/k_dst_slot), the per-destination sort (k_dst_sort_flat /
k_dst_sort_wide), the guard, and the destination-count scan.  The scan kernels (k_scan_local,
k_scan_sums, k_scan_add) carry the same names for the gossip generation's scan over the sources, so
every scan dispatch counts one half (two scans of equal size per window: generation and delivery).
2 * FETCH_SIZE + WRITE_SIZE (KiB -> bytes; x2: MI355X_MICROARCH.md §HBM gfx950 FETCH correction).
Only the last `steps` windows are averaged.  usage: pmc_delivery.py ROOT STEPS PEERS LAM WINDOW SHAPES [GROUP]"""
import csv
import glob
import hashlib
import json
import subprocess
import sys
from collections import defaultdict
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
root, steps = sys.argv[1], int(sys.argv[2])
# one marker per window (k_local_scatter_group: one per fused group of GROUP windows, argv[7])
MARK = ("k_local_scatter_ls", "k_local_scatter(", "k_local_scatter<", "k_dst_scatter(", "k_dst_slot<true>",
        "k_local_scatter_group")
BODY = MARK + ("k_dst_sort_flat", "k_dst_sort_wide", "k_dst_sort_bkt", "k_deliver_guard", "k_dst_hist", "k_dst_slot<false>",
               "k_scan_w1", "k_scan_w2")
SCAN = ("k_scan_local", "k_scan_sums", "k_scan_add")
GROUP = int(sys.argv[7]) if len(sys.argv) > 7 else 1
avg = {}
for f in glob.glob(f"{root}/p*/**/*counter_collection.csv", recursive=True):
    per = defaultdict(lambda: defaultdict(float))
    name = {}
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if any(m in k for m in BODY + SCAN):
            per[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
            name[int(r["Dispatch_Id"])] = k
    windows = []  # per window: the counters of its marker and of everything up to the next marker
    wins = []     # windows each entry stands for (a fused group's: GROUP)
    scans = defaultdict(float)
    n_scan = 0
    for i in sorted(per):
        if any(s in name[i] for s in SCAN):
            for c, v in per[i].items():
                scans[c] += v
            n_scan += 1
            continue
        if any(m in name[i] for m in MARK) or not windows:
            windows.append(defaultdict(float))
            wins.append(GROUP if "k_local_scatter_group" in name[i] else 1)
        for c, v in per[i].items():
            windows[-1][c] += v
    # the last `steps` windows (whole entries)
    k, got = len(windows), 0
    while k > 0 and got < steps:
        k -= 1
        got += wins[k]
    last, n_last = windows[k:], max(1, sum(wins[k:]))
    n_win = max(1, sum(wins))
    for c in set().union(*[w.keys() for w in last]):
        # a window's scan: every scan dispatch halved, spread evenly over the windows
        avg[c] = sum(w[c] for w in last) / n_last + 0.5 * scans.get(c, 0.0) / n_win
out = {"kernel": "delivery (K5) per window: scatter + per-destination sort + guard + half of the scan dispatches",
       "counters_avg_per_launch": avg,
       "hbm_bytes_per_launch": (2 * avg["FETCH_SIZE"] + avg["WRITE_SIZE"]) * 1024 if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg else None,
       "fetch_correction": "x2 (gfx950 FETCH_SIZE counts 64 B per 128 B request)",
       "peers": int(sys.argv[3]), "lam": float(sys.argv[4]), "window": int(sys.argv[5]), "shapes": sys.argv[6],
       "kernel_sha16": hashlib.sha256((REPO / "testground_amd/csrc/tgsim_kernels.hip").read_bytes()).hexdigest()[:16],
       "commit": subprocess.run(["git", "-C", str(REPO), "rev-parse", "--short=12", "HEAD"], capture_output=True,
                                text=True).stdout.strip() or None}
print(json.dumps(out, indent=1))
