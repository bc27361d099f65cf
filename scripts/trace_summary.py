"""Average per-window duration of the simulate kernels in a rocprofv3 kernel trace, over the last N
windows (the bench's timed windows follow its untimed settle/warm-up windows, which the --stats
table averages in).  A window runs the dense k_sim, the sparse pair k_sim_sparse + k_sim_list, or
is one of the windows of a fused k_sim_fused dispatch (tgsim_step_n: groups of at most FUSE windows,
a group of one runs k_sim); the bench's HIP events bracket the same dispatches."""
import csv
import json
import sys

trace, n = sys.argv[1], int(sys.argv[2])
fuse = int(sys.argv[3]) if len(sys.argv) > 3 else 8
FIRST = ("k_sim(", "k_sim_sparse(", "k_sim_fused(")  # one of these opens every dispatch group
rows = [r for r in csv.DictReader(open(trace)) if any(k in r["Kernel_Name"] for k in FIRST + ("k_sim_list(", "k_sim_multi("))]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
disp = []
for r in rows:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    name = next(k for k in FIRST + ("k_sim_list(", "k_sim_multi(") if k in r["Kernel_Name"])
    if name in FIRST or not disp:
        disp.append({"ms": 0.0, "kernels": []})
    disp[-1]["ms"] += d
    disp[-1]["kernels"].append(name.rstrip("("))


# the timed windows: tgsim_step_n(n) runs groups of fuse windows, then the remainder (a lone
# window unfused); matched to the last dispatch groups
fused = any("k_sim_fused" in d["kernels"] for d in disp)  # per-window dispatches otherwise
groups = [fuse] * (n // fuse) + ([n % fuse] if n % fuse else []) if fused else [1] * n
timed = [(d, w) for d, w in zip(reversed(disp), reversed(groups))]
ms = sum(d["ms"] for d, _ in timed)
wins = sum(w for _, w in timed)
mix = {}
for d, w in timed:
    k = "+".join(d["kernels"]) + (f" x{w} windows" if w > 1 else "")
    mix[k] = mix.get(k, 0) + 1
print(json.dumps({"kernels": "k_sim | k_sim_sparse + k_sim_multi + k_sim_list | k_sim_fused (per window)", "dispatch_groups": len(disp),
                  "timed_windows": wins, "timed_dispatch_groups": len(timed),
                  "timed_avg_ms_per_window": ms / max(1, wins),
                  "timed_min_ms_per_window": min(d["ms"] / w for d, w in timed),
                  "timed_max_ms_per_window": max(d["ms"] / w for d, w in timed),
                  "timed_dispatch_kinds": mix}, indent=1))
