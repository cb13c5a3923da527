"""Poisson updateZ restatement (R/updateZ.R:65-90): the Polya-Gamma moments the oracle and
rng.h use, checked against the PG(b, c) series definition (Polson, Scott & Windle 2013,
eq. 1: PG(b, c) = 1/(2 pi^2) sum_k g_k / ((k - 1/2)^2 + c^2 / (4 pi^2)), g_k ~ Gamma(b, 1)),
whose mean and variance are the convergent sums below; and the Z conditional of the
negative-binomial limit with r = 1000 against its closed form."""
import numpy as np
import pytest

from helpers import O, oracle_model, synthetic_model
from oracle.rng import Rng


def _pg_series(b, c, n=2_000_000):
    k = np.arange(1, n + 1, dtype=np.float64)
    d = (k - 0.5) ** 2 + c * c / (4 * np.pi ** 2)
    mean = b / (2 * np.pi ** 2) * (np.sum(1.0 / d[::-1]))
    var = b / (4 * np.pi ** 4) * (np.sum(1.0 / (d * d)[::-1]))
    # tail of the mean sum beyond n: integral of 1/(k-1/2)^2 ~ 1/n
    mean += b / (2 * np.pi ** 2) / n
    return mean, var


@pytest.mark.parametrize("c", [0.0, 1e-6, 0.3, 0.9999, 1.0001, 2.5, 7.0, 35.0, -4.0])
def test_pg_moments_match_series(c):
    b = 1003.0
    m, v = O.pg_moments(b, np.array([c]))
    ms, vs = _pg_series(b, c)
    assert abs(m[0] / ms - 1) < 1e-6
    assert abs(v[0] / vs - 1) < 1e-9


def test_poisson_z_conditional_closed_form():
    # zero noise: omega = E[PG], Z = its conditional mean (R/updateZ.R:80-83)
    y, e, sd, zp = np.array([3.0]), np.array([0.4]), np.array([0.1]), np.array([0.7])
    z = O.poisson_z_draw(y, e, sd, zp, np.array([0.5]), np.array([0.5]), zero_noise=True)
    lr = np.log(1000.0)
    x = abs(zp[0] - lr)
    w = (y[0] + 1000.0) * np.tanh(x / 2) / (2 * x)
    prec = sd[0] ** -2
    sz = 1 / (prec + w)
    assert abs(z[0] - (sz * ((y[0] - 1000.0) / 2 + prec * (e[0] - lr)) + lr)) < 1e-14


def test_poisson_chain_tracks_counts():
    """A Poisson-only chain of the oracle: Z stays finite across sweeps (the reference prints
    'Fail in Poisson Z update' otherwise) and the chain's mean intensity exp(Z) per species
    stays within a factor e^2 of the observed mean count (a sanity bound: the lognormal
    mean inflation and the shrinkage of 120 sites make the ratio ~1.3-2.9 here)."""
    hM = synthetic_model(ny=120, ns=6, nc=2, nf=1, n_poisson=6, seed=3)
    m = oracle_model(hM)
    rng = Rng(11)
    st = O.compute_initial_parameters(m, rng)
    acc = []
    for it in range(1, 80):
        st = O.sweep(st, m, rng, it, updater={"GammaEta": False})
        assert np.all(np.isfinite(st["Z"]))
        if it > 30:
            acc.append(np.exp(st["Z"]).mean(axis=0))
    ratio = np.log(np.mean(acc, axis=0) / m["Y"].mean(axis=0))
    assert np.all(np.abs(ratio) < 2.0), ratio


def test_waic_poisson_matches_quadrature():
    """computeWAIC's Poisson term (R/computeWAIC.R:108-118) against adaptive quadrature of
    log int Pois(y | e^z) N(z; E, sd) dz, on an all-Poisson model (where R's recycling of Y
    is the per-cell likelihood)."""
    from scipy import integrate, stats
    from hmsc_amd.post import computeWAIC
    hM = synthetic_model(ny=12, ns=3, nc=2, nf=1, n_poisson=3, seed=5)
    rng = np.random.default_rng(0)
    post = []
    for _ in range(4):
        post.append(dict(Beta=rng.normal(0, 0.3, (2, 3)), Eta=[rng.normal(0, 1, (12, 1))],
                         Lambda=[rng.normal(0, 0.3, (1, 3))], sigma=np.full(3, 0.5)))
    hM.postList = [post]
    w = computeWAIC(hM, ghN=120)
    vals = []
    for s in post:
        E = hM.X @ s["Beta"] + s["Eta"][0][hM.Pi[:, 0] - 1] @ s["Lambda"][0]
        sd = 0.5 ** -0.5
        L = np.zeros(12)
        for i in range(12):
            for j in range(3):
                f = lambda z: stats.poisson.pmf(hM.Y[i, j], np.exp(z)) * stats.norm.pdf(z, E[i, j], sd)
                L[i] += np.log(integrate.quad(f, E[i, j] - 12 * sd, E[i, j] + 12 * sd, epsabs=1e-13)[0])
        vals.append(L)
    val = np.stack(vals)
    ref = float(np.mean(-np.log(np.mean(np.exp(val), axis=0)) + val.var(axis=0, ddof=1)))
    assert abs(w - ref) < 1e-8 * max(1.0, abs(ref))
