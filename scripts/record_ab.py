"""Recorded vs unrecorded sweeps/s in one process (diagnostic): python scripts/record_ab.py"""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import hmsc_amd as H
from hmsc_amd.workloads import synthetic_probit
H._lib.lib()
hM = synthetic_probit()
ch = H.Chain(hM, 1234567, device=0, updater={"GammaEta": False})
ch.init([10])
ch.run(transient=40, samples=0, adaptNf=[0], record=False)
ch.sync()
it0 = 40
N = 1000
keep = []
for rep in range(2):
    t = time.perf_counter(); ch.run(transient=N, samples=0, adaptNf=[0], iter0=it0, record=False); ch.sync()
    dt = time.perf_counter() - t; it0 += N
    print(f"no record: {1e6 * dt / N:.1f} us/sweep", flush=True)
    t = time.perf_counter(); keep.append(ch.run(transient=0, samples=N, thin=1, adaptNf=[0], iter0=it0, record=True)); ch.sync()
    dt = time.perf_counter() - t; it0 += N
    print(f"record: {1e6 * dt / N:.1f} us/sweep", flush=True)
    keep.clear()
