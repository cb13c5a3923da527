"""Fixed cost of one hmsc_run call at the synthetic config 4 (GPU box): wall time of
run(samples=S) for S = 1, 8, 20, 100, 1000, recorded and unrecorded, after warm-up; with
HMSC_DIAG_TIMING=1 the library prints enqueue / completion / unpack / slot-wait times."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import hmsc_amd as H  # noqa: E402
from hmsc_amd.workloads import synthetic_probit  # noqa: E402

hM = synthetic_probit()
ch = H.Chain(hM, 1234567, device=0, updater={"GammaEta": False})
ch.init([10])
ch.run(transient=0, samples=1, thin=1, adaptNf=[0], record=True)
ch.prepare_graphs(2)
it = 1
ch.run(transient=0, samples=400, thin=1, adaptNf=[0], iter0=it, record=True)
it += 400
ch.sync()
for rec in (True, False):
    for S in (1, 8, 20, 20, 100, 1000):
        t0 = time.perf_counter()
        if rec:
            ch.run(transient=0, samples=S, thin=1, adaptNf=[0], iter0=it, record=True)
            t1 = time.perf_counter()
        else:
            ch.run(transient=S, samples=0, thin=1, adaptNf=[0], iter0=it, record=False)
        ch.sync()
        dt = time.perf_counter() - t0
        it += S
        extra = f" (run() returned at {1e3 * (t1 - t0):.3f} ms)" if rec else ""
        print(f"record={rec} S={S}: {1e3 * dt:.3f} ms, {1e3 * dt / S:.4f} ms/sweep{extra}", flush=True)
t0 = time.perf_counter()
a = np.zeros((20, 10, 10000))
a[:] = 1.0
print(f"alloc+touch 16 MB: {1e3 * (time.perf_counter() - t0):.3f} ms")
ch.close()
