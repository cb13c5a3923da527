"""Where a short recorded run's time goes (the driver's 20-step line): the bench's chain
prepared the same way (graphs prebuilt, clock warm-up), then repeated 20-sweep recorded
runs timed piecewise on the host; HMSC_DIAG_TIMING adds the library's own breakdown."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import hmsc_amd as H  # noqa: E402
from hmsc_amd.workloads import synthetic_probit  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
hM = synthetic_probit()
ch = H.Chain(hM, 1234567, device=0, updater={"GammaEta": False})
ch.init([10])
ch.kernel_timing(True)
ch.run(transient=0, samples=1, thin=1, adaptNf=[0], record=True)
ch.prepare_graphs(2)
it = 1
t_w = time.perf_counter()
while time.perf_counter() - t_w < 0.5:
    ch.run(transient=0, samples=50, thin=1, adaptNf=[0], iter0=it, record=True)
    it += 50
ch.sync()
rows = []
for rep in range(8):
    t0 = time.perf_counter()
    rec = ch.run(transient=0, samples=n, thin=1, adaptNf=[0], iter0=it, record=True)
    t1 = time.perf_counter()
    ch.sync()
    t2 = time.perf_counter()
    it += n
    rows.append((t1 - t0, t2 - t1))
r = np.array(rows) * 1e3
print(f"{n}-sweep recorded run: run() {np.median(r[:, 0]):.3f} ms, sync() {np.median(r[:, 1]):.3f} ms, "
      f"per sweep {np.median(r.sum(1)) / n * 1e3:.1f} us")
t0 = time.perf_counter()
ch.run(transient=0, samples=1000, thin=1, adaptNf=[0], iter0=it, record=True)
ch.sync()
print(f"1000-sweep recorded run: {(time.perf_counter() - t0) / 1000 * 1e6:.1f} us per sweep")
