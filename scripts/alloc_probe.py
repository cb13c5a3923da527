"""Timing probe: the Python-side record array allocation of Chain.run on this host."""
import time
import numpy as np
S, ns, nc, nf, ny = 400, 1000, 20, 10, 10000
for rep in range(3):
    t = time.perf_counter()
    arrays = dict(Beta=np.zeros((S, ns, nc)), Gamma=np.zeros((S, 1, nc)), iV=np.zeros((S, nc, nc)), iSigma=np.zeros((S, ns)),
                  Eta0=np.zeros((S, nf, ny)), Lambda0=np.zeros((S, ns, nf)), Psi0=np.zeros((S, ns, nf)))
    t1 = time.perf_counter()
    for a in arrays.values():
        a.reshape(-1)[::512] = 1.0   # touch every page
    t2 = time.perf_counter()
    del arrays
    t3 = time.perf_counter()
    print(f"alloc {1e3 * (t1 - t):.2f} ms, first touch {1e3 * (t2 - t1):.2f} ms, free {1e3 * (t3 - t2):.2f} ms")
