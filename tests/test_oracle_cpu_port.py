"""The C++ CPU restatement (oracle/cpu/hmsc_cpu.cpp, bench.py's cpu_baseline) against the numpy
oracle: same Philox key, init + full sweeps in the reference block order, states equal to
fp64 rounding -- so the baseline bench.py times is the same algorithm the GPU is checked
against.  CPU only."""
import numpy as np
import pytest

from helpers import O, oracle_model, rel_err, synthetic_model
from oracle import cpu_port
from oracle.rng import Rng


@pytest.mark.parametrize("kw", [dict(ny=150, ns=14, nc=3, nf=2, seed=71),
                                dict(ny=120, ns=9, nc=4, nf=3, nt=2, n_normal=3, seed=72),
                                dict(ny=200, ns=10, nc=3, nf=2, units=[40], seed=73)])
def test_cpu_port_matches_numpy_oracle(kw):
    hM = synthetic_model(**kw)
    m = oracle_model(hM)
    seed, n = 4321, 3
    up = {"GammaEta": False}
    rng = Rng(seed)
    o = O.compute_initial_parameters(m, rng)
    for it in range(1, n + 1):
        o = O.sweep(o, m, rng, it, updater=up)
    c, _ = cpu_port.run(m, seed, n_sweeps=n)
    for k in ("Beta", "Gamma", "iV", "Z", "iSigma"):
        assert rel_err(c[k], o[k]) < 1e-9, (k, rel_err(c[k], o[k]))
    for k in ("Lambda", "Eta", "Psi", "Delta"):
        assert rel_err(c[k], o[k][0]) < 1e-9, (k, rel_err(c[k], o[k][0]))


def test_cpu_port_chains_are_independent_threads():
    hM = synthetic_model(ny=100, ns=8, nc=3, nf=2, seed=74)
    m = oracle_model(hM)
    a, _ = cpu_port.run(m, 99, n_sweeps=2, nchains=1)
    b, sec = cpu_port.run(m, 99, n_sweeps=2, nchains=3)
    np.testing.assert_array_equal(a["Beta"], b["Beta"])       # chain 0 does not depend on the others
    assert sec > 0
