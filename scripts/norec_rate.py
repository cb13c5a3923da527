"""No-record sweeps/s of the synthetic chain (diagnostic for launch-structure experiments)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import hmsc_amd as H
from hmsc_amd.workloads import synthetic_probit
hM = synthetic_probit()
ch = H.Chain(hM, 1234567, device=0, updater={"GammaEta": False})
ch.init([10])
ch.run(transient=40, samples=0, adaptNf=[0], record=False)
ch.sync()
it0 = 40
N = 1000
for rep in range(3):
    t = time.perf_counter(); ch.run(transient=N, samples=0, adaptNf=[0], iter0=it0, record=False); ch.sync()
    dt = time.perf_counter() - t; it0 += N
    print(f"{os.environ.get('TAG', '')} no record: {N / dt:.1f} sweeps/s ({1e6 * dt / N:.1f} us/sweep)", flush=True)
