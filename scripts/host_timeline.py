"""Merged host/device timeline from a rocprofv3 run with --kernel-trace --hip-runtime-trace: kernel
executions (GPU, per hardware queue) and the main thread's HIP calls that launch, wait or take
longer than 3 us, in us from the n-th last k_sim.  Usage: host_timeline.py DIR [n] [rows]."""
import sys

import pandas as pd

d = sys.argv[1]
nth = int(sys.argv[2]) if len(sys.argv) > 2 else 5
rows = int(sys.argv[3]) if len(sys.argv) > 3 else 100
k = pd.read_csv(f"{d}/run_kernel_trace.csv")
h = pd.read_csv(f"{d}/run_hip_api_trace.csv")
t0 = k[k.Kernel_Name.str.contains("k_sim")].Start_Timestamp.iloc[-nth]
ev = []
for _, r in k[k.Start_Timestamp >= t0 - 50000].iterrows():
    ev.append((r.Start_Timestamp, "GPU ", r.End_Timestamp - r.Start_Timestamp,
               f"q{r.Queue_Id} {r.Kernel_Name[:30]} c{r.Correlation_Id}"))
main = h.Thread_Id.mode()[0]
for _, r in h[(h.Start_Timestamp >= t0 - 50000)].iterrows():
    du = r.End_Timestamp - r.Start_Timestamp
    if du > 3000 or any(w in r.Function for w in ("Launch", "Synchron", "Wait")):
        who = "HOST" if r.Thread_Id == main else f"T{r.Thread_Id % 1000}"
        ev.append((r.Start_Timestamp, who, du, f"{r.Function} c{r.Correlation_Id}"))
ev.sort()
for t, w, du, n in ev[:rows]:
    print(f"{(t - t0) / 1e3:8.1f} {du / 1e3:7.1f} {w} {n}")
