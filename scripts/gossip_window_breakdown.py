"""Per-window breakdown of the gossip closed loop from a rocprofv3 kernel trace: window = from one
k_sim_sparse start to the next; per kernel, its summed duration inside the window and the time the
simulate stream (k_sim_sparse's queue) spent in it; idle = gaps on that queue."""
import sys
import pandas as pd

k = pd.read_csv(sys.argv[1])
k["name"] = k["Kernel_Name"].str.replace(r"^(void )?tgsim::", "", regex=True).str.split("(").str[0]
k = k.sort_values("Start_Timestamp")
sims = k[k.name == "k_sim_sparse"]
q_sim = sims.Queue_Id.iloc[-1]
starts = sims.Start_Timestamp.values
rows = []
for i in range(len(starts) - 1):
    a, b = starts[i], starts[i + 1]
    w = k[(k.Start_Timestamp >= a) & (k.Start_Timestamp < b)]
    on = w[w.Queue_Id == q_sim]
    busy = (on.End_Timestamp - on.Start_Timestamp).sum()
    r = {"win": i, "ms": (b - a) / 1e6, "simq_busy": busy / 1e6}
    for n, g in w.groupby("name"):
        r[n] = (g.End_Timestamp - g.Start_Timestamp).sum() / 1e6
    rows.append(r)
df = pd.DataFrame(rows).fillna(0)
pd.set_option("display.width", 250, "display.max_columns", 40)
cols = ["ms", "simq_busy"] + [c for c in df.columns if c not in ("win", "ms", "simq_busy")]
print("simulate queue", q_sim, "; kernels on it:", sorted(k[k.Queue_Id == q_sim].name.unique()))
print(df[cols].describe().T[["mean", "min", "50%", "max"]].round(3))
peak = df.ms.idxmax()
print("slowest window", peak, df.loc[peak, cols].round(3).to_dict())
w = k[(k.Start_Timestamp >= starts[peak]) & (k.Start_Timestamp < starts[peak + 1])]
t0 = starts[peak]
for _, r in w.iterrows():
    print(f"{(r.Start_Timestamp - t0) / 1e3:9.1f} {(r.End_Timestamp - r.Start_Timestamp) / 1e3:8.1f} q{r.Queue_Id} {r['name']}")
