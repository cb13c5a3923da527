"""Standalone run of the blocked fp64 Cholesky (hmsc_dense_chol_solve, dense.hip) at the
config-5 size, for rocprofv3 kernel-trace / PMC passes:  python scripts/chol_bench.py [n] [reps]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hmsc_amd import _lib as L  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 5000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
rng = np.random.default_rng(0)
X = rng.standard_normal((n, n + 5))
A0 = np.asfortranarray(X @ X.T / n + np.eye(n))
b0 = rng.standard_normal(n)
info = np.zeros(1, dtype=np.int32)
for r in range(reps):
    A = A0.copy(order="F")
    b = b0.copy()
    t = time.perf_counter()
    L.check(L.lib().hmsc_dense_chol_solve(0, L.fptr(A), n, L.fptr(b), L.iptr(info)))
    print(f"rep {r}: n={n} info={int(info[0])} wall {1e3 * (time.perf_counter() - t):.1f} ms "
          f"(incl. host copies)", flush=True)
res = np.linalg.norm(A0 @ b - b0) / np.linalg.norm(b0)
print(f"relative residual {res:.2e}")
