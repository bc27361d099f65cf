"""Per-dispatch durations (us) of a kernel in a rocprofv3 kernel trace, plus the gap to the
previous kernel on the same queue: where a step's time goes besides the kernel itself."""
import csv
import sys

trace, kernel, n = sys.argv[1], sys.argv[2], int(sys.argv[3])
rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
out = []
prev_end = None
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if kernel in r["Kernel_Name"]:
        out.append(((e - s) / 1e3, (s - prev_end) / 1e3 if prev_end else 0.0))
    prev_end = e
last = out[-n:]
print("duration us:", [round(d, 1) for d, _ in last])
print("gap before us:", [round(g, 1) for _, g in last])
print(f"mean {sum(d for d, _ in last) / len(last):.1f} us, min {min(d for d, _ in last):.1f}, max {max(d for d, _ in last):.1f}")
