"""Average duration of the last N dispatches of a kernel in a rocprofv3 kernel trace (the bench's
timed steps follow its untimed settle/warm-up steps, which the --stats table averages in)."""
import csv
import json
import sys

trace, kernel, n = sys.argv[1], sys.argv[2], int(sys.argv[3])
rows = [r for r in csv.DictReader(open(trace)) if kernel in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
last = d[-n:]
print(json.dumps({"kernel": kernel, "dispatches": len(d), "timed_dispatches": len(last),
                  "timed_avg_ms": sum(last) / len(last), "all_avg_ms": sum(d) / len(d),
                  "timed_min_ms": min(last), "timed_max_ms": max(last)}, indent=1))
