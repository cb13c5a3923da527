"""In-kernel launch timer (hmsc_kernel_timing), the source of bench.py's roofline figure.

The timer must count exactly one launch per sweep for each timed kernel, on the eager path
and on the captured-graph replays alike, and must not change the chain (it only reads the
wall clock and does two atomics per workgroup into its own buffer)."""
import numpy as np
import pytest

from helpers import H, synthetic_model

pytestmark = pytest.mark.gpu


def _run(hM, timing, n=12):
    ch = H.Chain(hM, 4242, device=0, updater={"GammaEta": False})
    ch.init()
    if timing:
        ch.kernel_timing(True)
    rec = ch.run(transient=0, samples=n, thin=1, adaptNf=[0], record=True)
    out = {}
    if timing:
        for k in ("z", "eta", "betalambda"):
            out[k] = ch.kernel_timing_get(k)
    ch.close()
    return rec, out


def test_timer_counts_every_launch_and_leaves_chain_unchanged():
    hM = synthetic_model(ny=400, ns=48, nc=20, nf=10, seed=12)
    n = 12
    rec_t, t = _run(hM, True, n)
    rec_0, _ = _run(hM, False, n)
    for k, (tot_us, cnt) in t.items():
        assert cnt == n, (k, cnt)
        assert 0.0 < tot_us / cnt < 1e5, (k, tot_us)
    np.testing.assert_array_equal(rec_t["Beta"], rec_0["Beta"])
    np.testing.assert_array_equal(rec_t["Eta0"], rec_0["Eta0"])
