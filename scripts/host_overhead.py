"""Diagnostic: wall time per sweep at the bench workload with recording / profiling on or off.

Run on the GPU box:  python scripts/host_overhead.py
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import hmsc_amd as H  # noqa: E402
from hmsc_amd.workloads import synthetic_probit  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    hM = synthetic_probit(ny=10000, ns=1000, nc=20, nf=10)
    ch = H.Chain(hM, 1234567, device=0, updater={"GammaEta": False})
    ch.init([10])
    ch.run(transient=50, samples=0, adaptNf=[0], record=False)
    it0 = 50
    for prof in (False, True):
        ch.profile(prof)
        for record in (False, True):
            ch.sync()
            t0 = time.perf_counter()
            if record:
                ch.run(transient=0, samples=steps, thin=1, adaptNf=[0], iter0=it0, record=True)
            else:
                ch.run(transient=steps, samples=0, adaptNf=[0], iter0=it0, record=False)
            ch.sync()
            dt = time.perf_counter() - t0
            it0 += steps
            line = f"profile={prof} record={record}: {1e6 * dt / steps:8.1f} us/sweep"
            if prof:
                tot, n = ch.profile_get("sweep")
                line += f"   device sweep span {1e3 * tot / max(1, n):8.1f} us"
            print(line, flush=True)
    ch.close()


if __name__ == "__main__":
    main()
