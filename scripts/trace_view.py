"""Print a rocprofv3 kernel trace as a per-sweep timeline (queue, start offset, duration, gap)."""
import csv
import re
import sys

path = sys.argv[1]
start_at = sys.argv[2] if len(sys.argv) > 2 else "gamma2_partial"
nsweeps = int(sys.argv[3]) if len(sys.argv) > 3 else 2
skip = int(sys.argv[4]) if len(sys.argv) > 4 else 30
rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
short = lambda n: re.sub(r"\(.*", "", re.sub(r"^void ", "", n)).replace("hmsc::", "")  # noqa: E731
idx = [k for k, r in enumerate(rows) if start_at in r["Kernel_Name"]]
k0 = idx[skip]
k1 = idx[skip + nsweeps] if skip + nsweeps < len(idx) else len(rows)
t0 = int(rows[k0]["Start_Timestamp"])
last_end = {}
for r in rows[k0:k1]:
    q = r["Queue_Id"]
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - last_end[q]) / 1e3 if q in last_end else 0.0
    last_end[q] = e
    print(f"q{q:>2} {(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  gap {gap:7.1f}  {short(r['Kernel_Name'])}")
span = [int(rows[k]["Start_Timestamp"]) for k in idx]
d = [(span[k + 1] - span[k]) / 1e3 for k in range(len(span) - 1)]
print("sweep period us: first-half mean %.1f  last-half mean %.1f" % (sum(d[5:55]) / 50, sum(d[-50:]) / 50))
