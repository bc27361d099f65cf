"""Per-window timeline of a gossip bench kernel trace: for the last 70 windows (one k_sim_sparse
each), the window's period and, per hardware queue, the kernels in it (start/end relative to the
window's k_sim_sparse start, in us); every 5th window in full."""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "k_sim_sparse" in r["Kernel_Name"]][-70:]
for w in range(len(idx) - 1):
    a = int(rows[idx[w]]["Start_Timestamp"])
    b = int(rows[idx[w + 1]]["Start_Timestamp"])
    seg = [r for r in rows if a <= int(r["Start_Timestamp"]) < b]
    busy = {}
    for r in seg:
        busy[r["Queue_Id"]] = busy.get(r["Queue_Id"], 0) + int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    print(f"w{w:2d} period {(b - a) / 1e3:7.0f} us  " + "  ".join(f"q{q} busy {v / 1e3:6.0f}" for q, v in sorted(busy.items())))
    if w % 5 == 0:
        for r in seg:
            print(f"     q{r['Queue_Id']} {r['Kernel_Name'].split('(')[0][:34]:34s} {(int(r['Start_Timestamp']) - a) / 1e3:8.1f} "
                  f"{(int(r['End_Timestamp']) - a) / 1e3:8.1f}")
