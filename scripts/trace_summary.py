"""Average per-step duration of the simulate kernels in a rocprofv3 kernel trace, over the last N
steps (the bench's timed steps follow its untimed settle/warm-up steps, which the --stats table
averages in).  A step runs either the dense k_sim or the sparse pair k_sim_sparse + k_sim_list;
the step's time is the sum of its simulate dispatches, what the bench's HIP events bracket."""
import csv
import json
import sys

trace, n = sys.argv[1], int(sys.argv[2])
FIRST = ("k_sim(", "k_sim_sparse(")  # one of these opens every step
rows = [r for r in csv.DictReader(open(trace)) if any(k in r["Kernel_Name"] for k in FIRST + ("k_sim_list(",))]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
steps = []
for r in rows:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    name = next(k for k in FIRST + ("k_sim_list(",) if k in r["Kernel_Name"])
    if name in FIRST or not steps:
        steps.append({"ms": 0.0, "kernels": []})
    steps[-1]["ms"] += d
    steps[-1]["kernels"].append(name.rstrip("("))
last = steps[-n:]
mix = {}
for s in last:
    k = "+".join(s["kernels"])
    mix[k] = mix.get(k, 0) + 1
ms = [s["ms"] for s in last]
print(json.dumps({"kernels": "k_sim | k_sim_sparse + k_sim_list", "steps": len(steps), "timed_steps": len(last),
                  "timed_avg_ms": sum(ms) / len(ms), "timed_min_ms": min(ms), "timed_max_ms": max(ms),
                  "all_avg_ms": sum(s["ms"] for s in steps) / len(steps), "timed_step_kinds": mix}, indent=1))
