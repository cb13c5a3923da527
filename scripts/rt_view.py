"""The driver-shaped 20-step run on one shared clock, from a rocprofv3 --runtime-trace of
bench.py --steps 20 --warmup 5: the timed run is the one whose run_start_kernel is followed by
20 z launches and then another 20 (the bench's eager profile run).  Prints the HIP API calls of
the launcher thread and the kernel dispatches of that run, relative to its run_start_kernel's
enqueue, and a summary: host time to the first Gamma2 launch, the replay boundaries, the tail
after the last z."""
import csv
import glob
import os
import sys


def rows(pattern):
    f = sorted(glob.glob(pattern, recursive=True))
    if not f:
        sys.exit(f"no file {pattern}")
    with open(f[0]) as fh:
        return list(csv.DictReader(fh))


def main(d):
    kt = rows(os.path.join(d, "**", "*kernel_trace.csv"))
    api = rows(os.path.join(d, "**", "*hip_api_trace.csv"))
    kn = lambda r: r.get("Kernel_Name") or r.get("Name", "")  # noqa: E731
    ts = lambda r, k: int(r[k])  # noqa: E731
    kt.sort(key=lambda r: ts(r, "Start_Timestamp"))
    starts = [i for i, r in enumerate(kt) if "run_start_kernel" in kn(r)]
    zc = []
    for a, b in zip(starts, starts[1:] + [len(kt)]):
        zc.append(sum(1 for r in kt[a:b] if "z_wave_kernel" in kn(r)))
    pick = None
    for q in range(len(starts) - 1):
        if zc[q] == 20 and zc[q + 1] == 20:
            pick = q
    if pick is None:
        sys.exit(f"no 20-sweep run pair found: z counts {zc}")
    a, b = starts[pick], starts[pick + 1]
    run = kt[a:b]
    t0 = ts(run[0], "Start_Timestamp")
    # the API call that enqueued run_start_kernel: the last hipLaunchKernel before its start
    fn = lambda r: r.get("Function") or r.get("Name", "")  # noqa: E731
    api.sort(key=lambda r: ts(r, "Start_Timestamp"))
    tend = ts(run[-1], "End_Timestamp")
    calls = [r for r in api if t0 - 2_000_000 <= ts(r, "Start_Timestamp") <= tend + 1_000_000]
    print("t (us) rel. to run_start_kernel start; API calls (thread, dur) and kernels (queue, dur)")
    ev = [(ts(r, "Start_Timestamp"), "api", fn(r), r.get("Thread_Id", ""), ts(r, "End_Timestamp") - ts(r, "Start_Timestamp"))
          for r in calls if fn(r) not in ("hipGetLastError", "hipPeekAtLastError")]
    ev += [(ts(r, "Start_Timestamp"), "krn", kn(r)[:60], r.get("Queue_Id", r.get("Stream_Id", "")),
            ts(r, "End_Timestamp") - ts(r, "Start_Timestamp")) for r in run]
    ev.sort()
    for t, kind, name, who, dur in ev:
        print(f"{(t - t0) / 1e3:10.1f}  {kind}  {name:60s}  {who:>8}  {dur / 1e3:8.1f}")
    g2 = [r for r in run if "gamma2_bl" in kn(r)]
    z = [r for r in run if "z_wave" in kn(r)]
    if g2 and z:
        print(f"first Gamma2 start at {(ts(g2[0], 'Start_Timestamp') - t0) / 1e3:.1f} us; last z end at "
              f"{(ts(z[-1], 'End_Timestamp') - t0) / 1e3:.1f} us; last kernel end {(tend - t0) / 1e3:.1f} us")
        gaps = [(ts(g2[i + 1], "Start_Timestamp") - ts(z[i], "End_Timestamp")) / 1e3 for i in range(len(z) - 1) if i + 1 < len(g2)]
        print("z end -> next Gamma2 (us):", " ".join(f"{g:.1f}" for g in gaps))


if __name__ == "__main__":
    main(sys.argv[1])
