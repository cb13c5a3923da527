"""The species-sharded chain against the oracle directly (the sharded
tests compared it with the unsharded HIP chain only).  1, 2 and 3 ranks over the in-process
host transport (tests/test_gpu_sharded.py HostAllReduce), species blocks of whole quads
(uneven at ns = 41): every rank's initial state and its state after three sweeps, eager and
through the sweep graphs, equal the oracle's (oracle/hmsc_oracle.py, the same Philox
counters) restricted to its species -- init and single draws to 1e-9, three sweeps to 1e-7,
the tolerances of tests/test_gpu_parity.py."""
import pytest

from helpers import O, oracle_model, rel_err, synthetic_model
from hmsc_amd.sampler import shard_range
from oracle.rng import Rng
from test_gpu_sharded import _ranks, _run_ranks

pytestmark = pytest.mark.gpu
UP = {"GammaEta": False}


def _compare(hM, o, parts, nr, tol):
    for r, (a, n) in enumerate(shard_range(hM.ns, q, nr) for q in range(nr)):
        p = parts[r]
        assert rel_err(p["Beta"], o["Beta"][:, a:a + n]) < tol, (nr, r, "Beta", rel_err(p["Beta"], o["Beta"][:, a:a + n]))
        assert rel_err(p["Z"], o["Z"][:, a:a + n]) < tol, (nr, r, "Z")
        for k in ("Gamma", "iV"):
            assert rel_err(p[k], o[k]) < tol, (nr, r, k, rel_err(p[k], o[k]))
        for lv in range(hM.nr):
            assert rel_err(p["Lambda"][lv], o["Lambda"][lv][:, a:a + n]) < tol, (nr, r, "Lambda", lv)
            assert rel_err(p["Psi"][lv], o["Psi"][lv][:, a:a + n]) < tol, (nr, r, "Psi", lv)
            assert rel_err(p["Delta"][lv], o["Delta"][lv]) < tol, (nr, r, "Delta", lv)
            assert rel_err(p["Eta"][lv], o["Eta"][lv]) < tol, (nr, r, "Eta", lv)


@pytest.mark.parametrize("nr", [1, 2, 3])
@pytest.mark.parametrize("graph", [False, True])
def test_sharded_ranks_follow_oracle(nr, graph):
    hM = synthetic_model(ny=300, ns=41, nc=4, nf=3, seed=91)
    m = oracle_model(hM)
    seed = 13579
    rng = Rng(seed)
    o = O.compute_initial_parameters(m, rng)
    red, ranks = _ranks(hM, seed, nr)
    try:
        _run_ranks([lambda ch=ch: ch.init() for ch in ranks], red)
        _compare(hM, o, [ch.get_state() for ch in ranks], nr, 1e-9)
        for it in (1, 2, 3):
            o = O.sweep(o, m, rng, it, updater=UP)
        if graph:   # one eager sweep (the steady state the graphs are captured from), then replays
            _run_ranks([lambda ch=ch: ch.sweep(1) for ch in ranks], red)
            _run_ranks([lambda ch=ch: ch.run(transient=2, samples=0, thin=1, adaptNf=[0], iter0=1, record=False)
                        for ch in ranks], red)
        else:
            for it in (1, 2, 3):
                _run_ranks([lambda ch=ch, it=it: ch.sweep(it) for ch in ranks], red)
        _compare(hM, o, [ch.get_state() for ch in ranks], nr, 1e-7)
    finally:
        for ch in ranks:
            ch.close()
