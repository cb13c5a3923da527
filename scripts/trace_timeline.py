"""Per-sweep timeline from a rocprofv3 kernel-trace CSV: each kernel's start, duration and
the idle gap before it on its queue, for the last sweep, plus the mean sweep period.

    python scripts/trace_timeline.py gpurun_out/<tag>/run_kernel_trace.csv [anchor-kernel]

The anchor kernel (default gamma2_partial) starts every sweep.
"""
import csv
import sys


def short(name):
    return name.split("(")[0].replace("void ", "").replace("hmsc::", "")[:44]


def main():
    path = sys.argv[1]
    anchor = sys.argv[2] if len(sys.argv) > 2 else "gamma2_partial"
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), int(r["Queue_Id"])))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if anchor in r[2]]
    sweeps = list(zip(starts[:-1], starts[1:]))[-30:]
    per = [(rows[b][0] - rows[a][0]) / 1e3 for a, b in sweeps]
    print(f"sweep period: mean {sum(per) / len(per):.1f} us, min {min(per):.1f} over {len(per)} sweeps")
    a, b = sweeps[-1]
    t0 = rows[a][0]
    last_end = {}
    busy = 0.0
    print(f"{'kernel':46s} {'q':>2s} {'start':>8s} {'dur':>7s} {'gap':>6s}")
    for s, e, n, q in rows[a:b]:
        g = (s - last_end[q]) / 1e3 if q in last_end else 0.0
        last_end[q] = max(e, last_end.get(q, 0))
        print(f"{n:46s} {q:2d} {(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f} {g:6.1f}")


if __name__ == "__main__":
    main()
