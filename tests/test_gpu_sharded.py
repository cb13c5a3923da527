"""The species-sharded single chain, executed: two ranks on one GPU, each a
hmsc_create_sharded_host state owning an even-sized species block, every cross-shard sum
(Eta precision / numerator, GammaV, Gamma2, MGP row sums, updateNf counts) all-reduced through
a host transport (two threads, a barrier-based sum) in place of RCCL.  Eta, delta, iV and
Gamma are drawn redundantly on both ranks from the same Philox counters, so the sharded chain
must follow the unsharded chain of the same seed up to reduction-order rounding: the same
kernels, the same all-reduce call sites, only the transport differs from an RCCL run."""
import threading

import numpy as np
import pytest

from helpers import H, rel_err, synthetic_model
from hmsc_amd.sampler import shard_range

pytestmark = pytest.mark.gpu


class HostAllReduce:
    """In-process sum over `n` ranks (threads): deposit, barrier, sum, barrier."""

    def __init__(self, n, timeout=60.0):
        self.n = n
        # a rank that fails before an all-reduce would leave its peers waiting: the barrier
        # times out (BrokenBarrierError -> the callback returns -1 -> the library raises)
        self.bar = threading.Barrier(n, timeout=timeout)
        self.parts = [None] * n

    def abort(self):
        self.bar.abort()

    def for_rank(self, r):
        def f(x):
            self.parts[r] = x.copy()
            self.bar.wait()
            total = np.sum(self.parts, axis=0)     # identical order on every rank
            self.bar.wait()
            x[:] = total
        return f


def _run_ranks(fns, red=None):
    err = []

    def wrap(f):
        try:
            f()
        except Exception as e:
            err.append(e)
            if red is not None:
                red.abort()        # release the peers blocked in the all-reduce
    th = [threading.Thread(target=wrap, args=(f,)) for f in fns]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in th), "a rank is still inside a sweep"
    if err:
        raise err[0]


@pytest.mark.parametrize("kw", [dict(ny=300, ns=41, nc=4, nf=3, seed=61),
                                dict(ny=240, ns=30, nc=3, nf=2, nt=2, n_normal=4, seed=62)])
def test_sharded_chain_follows_unsharded(kw):
    hM = synthetic_model(**kw)
    up = {"GammaEta": False}
    seed, nr = 97531, 2
    full = H.Chain(hM, seed, device=0, updater=up)
    full.init()
    red = HostAllReduce(nr)
    ranks = [H.Chain(hM, seed, device=0, updater=up, rank=r, nranks=nr, host_allreduce=red.for_rank(r))
             for r in range(nr)]
    _run_ranks([ch.init for ch in ranks], red)
    for it in range(1, 6):
        full.sweep(it)
        _run_ranks([lambda ch=ch, it=it: ch.sweep(it) for ch in ranks], red)
    g = full.get_state()
    parts = [ch.get_state() for ch in ranks]
    blocks = [shard_range(hM.ns, r, nr) for r in range(nr)]
    assert blocks[0][0] == 0 and blocks[-1][0] + blocks[-1][1] == hM.ns
    for r, (a, n) in enumerate(blocks):
        p = parts[r]
        assert rel_err(p["Beta"], g["Beta"][:, a:a + n]) < 1e-8, (r, "Beta")
        assert rel_err(p["Lambda"][0], g["Lambda"][0][:, a:a + n]) < 1e-8, (r, "Lambda")
        assert rel_err(p["Z"], g["Z"][:, a:a + n]) < 1e-8, (r, "Z")
        assert rel_err(p["iSigma"], g["iSigma"][a:a + n]) < 1e-8, (r, "iSigma")
        for k in ("Gamma", "iV"):                  # drawn redundantly on every rank
            assert rel_err(p[k], g[k]) < 1e-8, (r, k)
        assert rel_err(p["Eta"][0], g["Eta"][0]) < 1e-8, (r, "Eta")
        np.testing.assert_array_equal(p["Gamma"], parts[0]["Gamma"])
        np.testing.assert_array_equal(p["Eta"][0], parts[0]["Eta"][0])
    for ch in ranks + [full]:
        ch.close()


def test_shard_range_blocks():
    for ns in (2, 7, 41, 1000, 1003):
        for n in (1, 2, 4, 8):
            if n > (ns + 1) // 2:
                continue
            bl = [shard_range(ns, r, n) for r in range(n)]
            assert bl[0][0] == 0 and sum(b for _, b in bl) == ns
            assert all(a % 2 == 0 for a, _ in bl)
            assert all(bl[i][0] + bl[i][1] == bl[i + 1][0] for i in range(n - 1))
