"""The driver's 20-step line, sweep by sweep: the bench's preparation (graphs prebuilt, clock
warm-up), one 20-sweep recorded run timed on the host, then the live launch timers of its
sweeps (wall clock, 100 MHz) -- where the run's time beyond 20 steady sweeps goes."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import hmsc_amd as H  # noqa: E402
from hmsc_amd.workloads import synthetic_probit  # noqa: E402

KT_SLOTS, KT_N = 8192, 7
n = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 20
hM = synthetic_probit()
ch = H.Chain(hM, 1234567, device=0, updater={"GammaEta": False})
ch.init([10])
ch.kernel_timing(True)
ch.run(transient=0, samples=1, thin=1, adaptNf=[0], record=True)
ch.prepare_graphs(2)
ch.run(transient=0, samples=4, thin=1, adaptNf=[0], iter0=1, record=True)
ch.sync()
it = 5
t_w = time.perf_counter()
while time.perf_counter() - t_w < 0.5:
    ch.run(transient=0, samples=50, thin=1, adaptNf=[0], iter0=it, record=True)
    ch.sync()
    it += 50
for rep in range(3):
    ch.kernel_timing(True)
    t0 = time.perf_counter()
    ch.run(transient=0, samples=n, thin=1, adaptNf=[0], iter0=it, record=True)
    ch.sync()
    t_host = (time.perf_counter() - t0) * 1e6
    kt = ch.debug_get("kt", KT_N * 2 * KT_SLOTS).reshape(KT_N, 2, KT_SLOTS).astype(np.float64)
    its = (np.arange(it + 1, it + n + 1)) % KT_SLOTS
    it += n
    names = ("z", "eta", "bl", "tail", "g2", "side")
    st = {k: kt[i, 0, its] for i, k in enumerate(names)}
    en = {k: kt[i, 1, its] for i, k in enumerate(names)}
    base = st["g2"][0]
    us = lambda v: (v - base) * 0.01  # noqa: E731
    print(f"run {rep}: host {t_host:.1f} us for {n} sweeps; device first Gamma2 start -> last z end "
          f"{us(en['z'][-1]):.1f} us")
    gaps = us(st["g2"][1:]) - us(en["z"][:-1])
    print(f"  z end -> next Gamma2: median {np.median(gaps):.1f} us, max {gaps.max():.1f} us before sweep {int(gaps.argmax()) + 1}")
    its_k = kt[6, 0, its]  # replay starts (set_iters_kernel): the replay's first sweep's slot
    for k in range(1, n):
        if its_k[k] < 2 ** 63:
            print(f"  replay at sweep {k}: prev z end {us(en['z'][k - 1]):.1f}, set_iters {us(its_k[k]):.1f}, "
                  f"Gamma2 start {us(st['g2'][k]):.1f}, side start {us(st['side'][k]):.1f} us")
    if "--brief" in sys.argv:
        continue
    for k in range(n):
        print(f"  sweep {k:2d}: g2 {us(st['g2'][k]):8.1f}  bl_end {us(en['bl'][k]):8.1f}  tail_end {us(en['tail'][k]):8.1f}"
              f"  eta {us(st['eta'][k]):8.1f}-{us(en['eta'][k]):8.1f}  z {us(st['z'][k]):8.1f}-{us(en['z'][k]):8.1f}"
              f"  side {us(st['side'][k]):8.1f}-{us(en['side'][k]):8.1f}")
