"""The species-sharded single chain (state.h "species-sharded chain",
kernels.hip "species-sharded sweep"): each rank owns an even-aligned block of species, every
cross-species sum of a sweep goes through exactly two all-reduces (A after updateZ: Gamma2's
sums; B after updateBetaLambda: Eta's ZL / CR / NA rows, GammaV's and LambdaPriors' sums), and
Gamma, iV, Delta and Eta are drawn redundantly on every rank from the same Philox counters.

* one rank with a transport (RCCL or a host callback) runs the sharded kernels and collectives
  and must reproduce the unsharded chain bit for bit -- at the config-4 size;
* 2 and 4 ranks over a host transport (threads, a barrier-based sum standing in for RCCL)
  follow the unsharded chain of the same seed to reduction-order rounding (1e-8), eager and
  through the sweep graphs, also at the config-4 size;
* sharded graph replay is bit-equal to sharded eager sweeps, with two all-reduces per sweep;
* the general path (NA rows, grouped units, normal species, two levels) follows too.
The two-process (gloo) form is tests/test_gpu_sharded_procs.py."""
import threading

import numpy as np
import pytest

from helpers import H, rel_err, synthetic_model
from hmsc_amd.sampler import comm_unique_id, shard_range
from hmsc_amd.workloads import synthetic_probit

pytestmark = pytest.mark.gpu

UP = {"GammaEta": False}


class HostAllReduce:
    """In-process sum over `n` ranks (threads): deposit, barrier, sum, barrier."""

    def __init__(self, n, timeout=120.0):
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
    out = [None] * len(fns)

    def wrap(k, f):
        try:
            out[k] = f()
        except Exception as e:
            err.append(e)
            if red is not None:
                red.abort()        # release the peers blocked in the all-reduce
    th = [threading.Thread(target=wrap, args=(k, f)) for k, f in enumerate(fns)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=240)
    assert not any(t.is_alive() for t in th), "a rank is still inside a sweep"
    if err:
        raise err[0]
    return out


def _ranks(hM, seed, nr, up=UP):
    red = HostAllReduce(nr)
    return red, [H.Chain(hM, seed, device=0, updater=up, rank=r, nranks=nr, host_allreduce=red.for_rank(r))
                 for r in range(nr)]


def _check_follows(hM, g, parts, nr, tol=1e-8, rec_full=None, recs=None):
    blocks = [shard_range(hM.ns, r, nr) for r in range(nr)]
    assert blocks[0][0] == 0 and blocks[-1][0] + blocks[-1][1] == hM.ns
    for r, (a, n) in enumerate(blocks):
        p = parts[r]
        assert rel_err(p["Beta"], g["Beta"][:, a:a + n]) < tol, (r, "Beta")
        for lv in range(hM.nr):
            assert rel_err(p["Lambda"][lv], g["Lambda"][lv][:, a:a + n]) < tol, (r, "Lambda", lv)
            assert rel_err(p["Eta"][lv], g["Eta"][lv]) < tol, (r, "Eta", lv)
            np.testing.assert_array_equal(p["Eta"][lv], parts[0]["Eta"][lv])   # redundant draws agree
            np.testing.assert_array_equal(p["Delta"][lv], parts[0]["Delta"][lv])
        assert rel_err(p["Z"], g["Z"][:, a:a + n]) < tol, (r, "Z")
        assert rel_err(p["iSigma"], g["iSigma"][a:a + n]) < tol, (r, "iSigma")
        for k in ("Gamma", "iV"):
            assert rel_err(p[k], g[k]) < tol, (r, k)
            np.testing.assert_array_equal(p[k], parts[0][k])
        if recs is not None:
            assert rel_err(recs[r]["Beta"], rec_full["Beta"][:, :, a:a + n]) < tol, (r, "recorded Beta")
            assert rel_err(recs[r]["Gamma"], rec_full["Gamma"]) < tol, (r, "recorded Gamma")


@pytest.fixture(scope="module")
def config4():
    return synthetic_probit()   # BASELINE config 4: ny = 10 000, ns = 1 000, nc = 20, nf = 10


@pytest.mark.parametrize("transport", ["host", "rccl"])
def test_one_rank_sharded_is_unsharded_bitwise(config4, transport):
    """The sharded sweep's kernels (fused Gamma2 + BetaLambda with Gamma2's sums from
    all-reduce A, the Eta stream / solve split at all-reduce B, the side chain on the reduced
    sums) at one rank: the unsharded chain bit for bit, eager and through the sweep graphs."""
    hM, seed = config4, 97531
    full = H.Chain(hM, seed, device=0, updater=UP)
    full.init([10])
    if transport == "host":
        sh = H.Chain(hM, seed, device=0, updater=UP, rank=0, nranks=1, host_allreduce=lambda x: None)
    else:
        sh = H.Chain(hM, seed, device=0, updater=UP, rank=0, nranks=1, comm_id=comm_unique_id())
    sh.init([10])
    for ch in (full, sh):
        ch.sweep(1)
        ch.sweep(2)
    rf = full.run(transient=0, samples=20, thin=1, adaptNf=[0], iter0=2, record=True)
    rs = sh.run(transient=0, samples=20, thin=1, adaptNf=[0], iter0=2, record=True)
    g, p = full.get_state(), sh.get_state()
    for k in ("Beta", "Gamma", "iV", "iSigma", "Z"):
        np.testing.assert_array_equal(p[k], g[k], err_msg=k)
    for k in ("Eta", "Lambda", "Psi", "Delta"):
        np.testing.assert_array_equal(p[k][0], g[k][0], err_msg=k)
    for k in ("Beta", "Gamma", "iV", "Eta0", "Lambda0", "Psi0", "Delta0"):
        np.testing.assert_array_equal(rs[k], rf[k], err_msg="recorded " + k)
    ar = sh.debug_get("ar_calls", 4)
    assert ar[3] == 1 and ar[2] == 2, ar          # sharded; two all-reduces per captured sweep
    assert full.debug_get("ar_calls", 4)[3] == 0
    for ch in (full, sh):
        ch.close()


@pytest.mark.parametrize("nr", [2, 4])
def test_fullsize_ranks_follow_unsharded(config4, nr):
    """Config 4 at its own size, species-sharded over 2 and 4 host-transport ranks: 3 eager
    sweeps, then a recorded run through the sweep graphs (segments split at the all-reduces)."""
    hM, seed = config4, 4242
    full = H.Chain(hM, seed, device=0, updater=UP)
    full.init([10])
    red, ranks = _ranks(hM, seed, nr)
    _run_ranks([lambda ch=ch: ch.init([10]) for ch in ranks], red)
    for it in range(1, 4):
        full.sweep(it)
        _run_ranks([lambda ch=ch, it=it: ch.sweep(it) for ch in ranks], red)
    rec_full = full.run(transient=0, samples=6, thin=1, adaptNf=[0], iter0=3, record=True)
    recs = _run_ranks([lambda ch=ch: ch.run(transient=0, samples=6, thin=1, adaptNf=[0], iter0=3, record=True)
                       for ch in ranks], red)
    g = full.get_state()
    parts = [ch.get_state() for ch in ranks]
    _check_follows(hM, g, parts, nr, rec_full=rec_full, recs=recs)
    for ch in ranks:
        a = ch.debug_get("ar_calls", 4)
        assert a[2] == 2, a                       # two all-reduces per captured sweep
    for ch in ranks + [full]:
        ch.close()


def test_graph_replay_equals_eager_two_allreduces():
    """Two host-transport ranks: the sweep graphs (RCCL-free: segments with the host sum between
    them) give bit for bit the eager sweeps' chain; a steady sweep issues exactly two
    all-reduces (the debug counter), eager and replayed."""
    hM = synthetic_model(ny=1500, ns=120, nc=5, nf=4, seed=71)
    seed, nr, n = 2468, 2, 12
    red_e, eager = _ranks(hM, seed, nr)
    red_g, graph = _ranks(hM, seed, nr)
    _run_ranks([lambda ch=ch: ch.init() for ch in eager], red_e)
    _run_ranks([lambda ch=ch: ch.init() for ch in graph], red_g)
    for ch in eager + graph:
        assert ch.debug_get("ar_calls", 4)[3] == 1
    _run_ranks([lambda ch=ch: ch.sweep(1) for ch in eager], red_e)
    c1 = [ch.debug_get("ar_calls", 4)[0] for ch in eager]
    for it in range(2, n + 1):
        _run_ranks([lambda ch=ch, it=it: ch.sweep(it) for ch in eager], red_e)
    for ch, c in zip(eager, c1):
        assert ch.debug_get("ar_calls", 4)[0] - c == 2 * (n - 1)   # <= 2 all-reduces per sweep
    _run_ranks([lambda ch=ch: ch.run(transient=n, samples=0, thin=1, adaptNf=[0], iter0=0, record=False)
                for ch in graph], red_g)
    for ch in graph:
        gd = ch.debug_get("graph", 4)
        assert gd[0] == 1, "the sweep graphs were not built"
        assert ch.debug_get("ar_calls", 4)[2] == 2
    for a, b in zip(eager, graph):
        sa, sb = a.get_state(), b.get_state()
        for k in ("Beta", "Gamma", "iV", "iSigma", "Z"):
            np.testing.assert_array_equal(sa[k], sb[k], err_msg=k)
        for k in ("Eta", "Lambda", "Psi", "Delta"):
            np.testing.assert_array_equal(sa[k][0], sb[k][0], err_msg=k)
    for ch in eager + graph:
        ch.close()


@pytest.mark.parametrize("kw", [dict(ny=300, ns=41, nc=4, nf=3, seed=61),
                                dict(ny=240, ns=30, nc=3, nf=2, nt=2, n_normal=4, seed=62),
                                dict(ny=300, ns=36, nc=4, nf=3, na_frac=0.05, seed=63),
                                dict(ny=240, ns=30, nc=3, nf=2, na_frac=0.08, units=[60, 240], nr=2, seed=64),
                                dict(ny=400, ns=50, nc=3, nf=2, n_normal=6, na_frac=0.03, units=[100], seed=65)])
def test_general_path_follows_unsharded(kw):
    """Models off the fused path -- NA rows (the row-masked CR all-reduced once), grouped
    units, normal species, traits, two levels: 2 and 3 ranks follow the unsharded chain."""
    hM = synthetic_model(**kw)
    seed = 97531
    full = H.Chain(hM, seed, device=0, updater=UP)
    full.init()
    for nr in (2, 3):
        if (hM.ns + 1) // 2 < nr:
            continue
        red, ranks = _ranks(hM, seed, nr)
        _run_ranks([ch.init for ch in ranks], red)
        for it in range(1, 6):
            _run_ranks([lambda ch=ch, it=it: ch.sweep(it) for ch in ranks], red)
        parts = [ch.get_state() for ch in ranks]
        if nr == 2:
            for it in range(1, 6):
                full.sweep(it)
            g = full.get_state()
        _check_follows(hM, g, parts, nr)
        for ch in ranks:
            ch.close()
    full.close()


def test_single_updaters_on_shards():
    """hmsc_update(which) on a sharded chain runs each updater with its own all-reduce: in the
    reference order they reproduce a sweep of the unsharded chain."""
    hM = synthetic_model(ny=300, ns=40, nc=4, nf=3, seed=66, na_frac=0.04)
    seed, nr = 1357, 2
    full = H.Chain(hM, seed, device=0, updater=UP)
    full.init()
    red, ranks = _ranks(hM, seed, nr)
    _run_ranks([ch.init for ch in ranks], red)
    order = ["Gamma2", "BetaLambda", "GammaV", "LambdaPriors", "Eta", "InvSigma", "Z"]
    for name in order:
        full.update(name, 1)
        _run_ranks([lambda ch=ch, name=name: ch.update(name, 1) for ch in ranks], red)
    _check_follows(hM, full.get_state(), [ch.get_state() for ch in ranks], nr)
    for ch in ranks + [full]:
        ch.close()


def test_shard_range_blocks():
    for ns in (2, 7, 41, 1000, 1003):
        for n in (1, 2, 4, 8):
            if n > (ns + 3) // 4:
                continue
            bl = [shard_range(ns, r, n) for r in range(n)]
            assert bl[0][0] == 0 and sum(b for _, b in bl) == ns
            assert all(a % 4 == 0 for a, _ in bl)
            assert all(bl[i][0] + bl[i][1] == bl[i + 1][0] for i in range(n - 1))
