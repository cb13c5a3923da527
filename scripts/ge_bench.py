"""Eager GammaEta updates at the config-3 shape (vignette_3, ns = 300) for rocprofv3
kernel-trace passes over the blocked updateGammaEta path:  python scripts/ge_bench.py [reps]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import hmsc_amd as H  # noqa: E402
from hmsc_amd.workloads import vignette3_phylo  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
hM = vignette3_phylo()
ch = H.Chain(hM, 20261015, device=0, updater={})
ch.init([2])
for it in range(1, 4):
    ch.sweep(it)
ch.sync()
for name in ("GammaEta", "BetaLambda"):
    t = time.perf_counter()
    for r in range(reps):
        ch.update(name, 10 + r)
    ch.sync()
    print(f"{name}: {1e3 * (time.perf_counter() - t) / reps:.3f} ms per update (eager, host-timed)", flush=True)
ch.close()
