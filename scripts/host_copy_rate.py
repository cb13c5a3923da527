"""Host memory: first-touch vs warm copy rate of 1.13 MB samples into a fresh record array."""
import time
import numpy as np
from concurrent.futures import ThreadPoolExecutor
src = np.random.rand(141000)
N = 1000
for trial in range(2):
    a = np.zeros((N, 141000))
    t = time.perf_counter()
    for k in range(N):
        a[k] = src
    dt = time.perf_counter() - t
    print(f"fresh 1 thread: {1e6 * dt / N:.1f} us/sample")
    t = time.perf_counter()
    for k in range(N):
        a[k] = src
    print(f"warm 1 thread: {1e6 * (time.perf_counter() - t) / N:.1f} us/sample")
    for W in (2, 4, 8):
        a = np.zeros((N, 141000))
        def work(w):
            for k in range(w, N, W):
                a[k] = src
        t = time.perf_counter()
        with ThreadPoolExecutor(W) as ex:
            list(ex.map(work, range(W)))
        print(f"fresh {W} threads: {1e6 * (time.perf_counter() - t) / N:.1f} us/sample")
