"""A recorded run's samples are the same bits whichever way they reach the host: host-issued
copies after each replay (HMSC_KERNEL_COPY=0) or the per-sample copy kernels of the run's last
replays (the default, capi.cpp / kernels.hip rec_copy_kernel), for run lengths that end on
replays of every size and with thinning and a transient."""
import numpy as np
import pytest

from helpers import H, synthetic_model

pytestmark = pytest.mark.gpu


def _record(monkeypatch, kcopy, runs):
    if kcopy:
        monkeypatch.delenv("HMSC_KERNEL_COPY", raising=False)
    else:
        monkeypatch.setenv("HMSC_KERNEL_COPY", "0")
    hM = synthetic_model(ny=300, ns=40, nc=4, nf=3, seed=81)
    ch = H.Chain(hM, 4242, device=0, updater={"GammaEta": False})
    ch.init()
    ch.run(transient=0, samples=1, thin=1, adaptNf=[0], record=True)
    ch.prepare_graphs(2)
    out, it = [], 2
    for transient, samples, thin in runs:
        out.append(ch.run(transient=transient, samples=samples, thin=thin, adaptNf=[0], iter0=it, record=True))
        it += transient + samples * thin
    ch.close()
    return out


def test_kernel_copies_match_host_copies(monkeypatch):
    runs = [(0, 20, 1), (0, 7, 1), (3, 13, 2), (0, 45, 1), (0, 1, 1)]
    a = _record(monkeypatch, True, runs)
    b = _record(monkeypatch, False, runs)
    for ra, rb in zip(a, b):
        assert set(ra) == set(rb)
        for k in ra:
            np.testing.assert_array_equal(np.asarray(ra[k]), np.asarray(rb[k]), err_msg=k)
