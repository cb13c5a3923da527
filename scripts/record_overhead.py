"""Sweeps/s of the synthetic chain with and without per-sweep recording (diagnostic),
for several unpack worker counts (HMSC_UNPACK_THREADS is read by every hmsc_run call)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import hmsc_amd as H
from hmsc_amd.workloads import synthetic_probit
hM = synthetic_probit()
ch = H.Chain(hM, 1234567, device=0, updater={"GammaEta": False})
ch.init([10])
ch.run(transient=30, samples=0, adaptNf=[0], record=False)
ch.sync()
it0 = 30
N = 400
for rep in range(2):
    t = time.perf_counter(); ch.run(transient=N, samples=0, adaptNf=[0], iter0=it0, record=False); ch.sync()
    dt = time.perf_counter() - t; it0 += N
    print(f"no record: {N / dt:.1f} sweeps/s ({1e6 * dt / N:.1f} us/sweep)", flush=True)
    for w in sys.argv[1:] or ["1", "2", "4"]:
        os.environ["HMSC_UNPACK_THREADS"] = w
        t = time.perf_counter(); ch.run(transient=0, samples=N, thin=1, adaptNf=[0], iter0=it0, record=True); ch.sync()
        dt = time.perf_counter() - t; it0 += N
        print(f"record every sweep, {w} unpack threads: {N / dt:.1f} sweeps/s ({1e6 * dt / N:.1f} us/sweep)", flush=True)
