"""Per-sweep timeline of a rocprofv3 kernel trace (run_kernel_trace.csv): for the steady
sweeps, each kernel's start / end relative to the sweep's gamma2_bl start, with queues, and
the median over sweeps.  usage: trace_timeline.py TRACE.csv [first_sweep] [n_sweeps]"""
import csv
import sys
from collections import defaultdict

import numpy as np

rows = list(csv.DictReader(open(sys.argv[1])))
rows = [r for r in rows if r["Kind"] == "KERNEL_DISPATCH"]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
first = int(sys.argv[2]) if len(sys.argv) > 2 else 200
nsw = int(sys.argv[3]) if len(sys.argv) > 3 else 200
short = lambda n: n.split("(")[0].replace("void ", "").replace("hmsc::", "")[:28]
starts = [i for i, r in enumerate(rows) if "gamma2_bl_kernel" in r["Kernel_Name"]]
rel = defaultdict(list)
period = []
for s_i in range(first, min(first + nsw, len(starts) - 1)):
    a, b = starts[s_i], starts[s_i + 1]
    t0 = int(rows[a]["Start_Timestamp"])
    period.append(int(rows[b]["Start_Timestamp"]) - t0)
    seen = defaultdict(int)
    for r in rows[a:b]:
        k = short(r["Kernel_Name"])
        seen[k] += 1
        key = f"{k}#{seen[k]}" if seen[k] > 1 else k
        rel[key].append((int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0, r["Queue_Id"]))
print(f"sweep period median {np.median(period)/1e3:.2f} us  (n={len(period)})")
for k, v in sorted(rel.items(), key=lambda kv: np.median([x[0] for x in kv[1]])):
    s = np.median([x[0] for x in v]) / 1e3
    e = np.median([x[1] for x in v]) / 1e3
    q = max(set(x[2] for x in v), key=[x[2] for x in v].count)
    print(f"{k:32s} q{q:>3s} start {s:8.2f} end {e:8.2f} dur {e - s:7.2f}  (n={len(v)})")
