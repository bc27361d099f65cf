"""Prints the tail of a rocprofv3 kernel/memory-copy trace as a per-queue timeline (us from the
4th-last k_sim): start, duration, hardware queue, kernel."""
import sys

import pandas as pd

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/sp"
k = pd.read_csv(f"{d}/run_kernel_trace.csv")
k["name"] = k["Kernel_Name"].str.slice(0, 40)
k["q"] = k["Queue_Id"]
ev = [k[["name", "Start_Timestamp", "End_Timestamp", "q"]]]
try:
    m = pd.read_csv(f"{d}/run_memory_copy_trace.csv")
    ev.append(m.assign(name="copy " + m["Direction"].astype(str), q=-1)[["name", "Start_Timestamp", "End_Timestamp", "q"]])
except FileNotFoundError:
    pass
ev = pd.concat(ev).sort_values("Start_Timestamp")
ks = ev[ev.name.str.contains("k_sim")]
t0 = ks.Start_Timestamp.iloc[-int(sys.argv[2]) if len(sys.argv) > 2 else -4]
for _, r in ev[ev.Start_Timestamp >= t0].head(int(sys.argv[3]) if len(sys.argv) > 3 else 60).iterrows():
    print(f"{(r.Start_Timestamp - t0) / 1e3:9.1f} {(r.End_Timestamp - r.Start_Timestamp) / 1e3:8.1f} q{r.q} {r['name']}")
