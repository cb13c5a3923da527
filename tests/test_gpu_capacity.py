"""Latent-dimension capacity K = nc + sum(nf) <= 128 (hmsc_amd/csrc/common.h HMSC_KCAP).

R's default nfMax = Inf becomes ns (R/Hmsc.R:554) and a model may have many covariates, so
the device chain must hold K past 64: updateZ's 128-row instantiation (z_kernel.h NKB = 8),
BetaLambda's K x K factor in LDS, Eta / LambdaPriors with sum(nf) > 64 (two ZL passes),
predict and the post-sampling kernels (VP with nc > 64, Omega with nf > 64).  Each case runs
against the oracle restatement on the same state and Philox key, to the tolerances of
test_gpu_parity.py.
"""
import warnings

import numpy as np
import pytest

from helpers import H, O, oracle_model, rel_err, synthetic_model
from oracle import post_oracle as P
from oracle.rng import Rng

pytestmark = pytest.mark.gpu

TOL_DRAW = 1e-9
# Gamma / iV at nc = 70: a 70-dimensional solve whose summation order differs between the
# device and numpy; the condition number (~1e6 here) scales the fp64 rounding past 1e-9
TOL_WIDE_GAMMA = 1e-8


def _oracle_state(m, seed, n_sweeps=2):
    rng = Rng(seed)
    st = O.compute_initial_parameters(m, rng)
    for it in range(1, n_sweeps + 1):
        st = O.sweep(st, m, rng, it, updater={"GammaEta": False})
    return st


def _chain(hM, seed, st=None, **kw):
    ch = H.Chain(hM, seed, device=0, updater={"GammaEta": False}, **kw)
    ch.init()
    if st is not None:
        ch.set_state(st)
    return ch


def _track(hM, m, seed, st, its=range(10, 13), keys=("Beta", "Gamma", "iV", "Z")):
    ch = _chain(hM, seed, st)
    rng = Rng(seed)
    o = st
    for it in its:
        ch.sweep(it)
        o = O.sweep(o, m, rng, it, updater={"GammaEta": False})
    g = ch.get_state()
    for k in keys:
        assert rel_err(g[k], o[k]) < 1e-7, (k, rel_err(g[k], o[k]))
    for r in range(hM.nr):
        assert rel_err(g["Lambda"][r], o["Lambda"][r]) < 1e-7, r
    ch.close()


def test_default_nfmax_is_held():
    """nc = 20, ns = 100 with the reference's default priors (nfMax = ns = 100): K up to 120
    fits, no capacity warning, and three sweeps follow the oracle."""
    hM = synthetic_model(ny=300, ns=100, nc=20, nf=2, seed=21, nf_default=True)
    assert hM.rL[0].nfMax == 100
    m = oracle_model(hM)
    seed = 1357
    with warnings.catch_warnings():
        warnings.simplefilter("error")
        ch = H.Chain(hM, seed, device=0, updater={"GammaEta": False})
    assert ch.nf_cap == [100]
    dims = ch.debug_get("dims", 8)
    assert int(dims[2]) == 120  # Kmax
    ch.close()
    _track(hM, m, seed, _oracle_state(m, seed))


def test_capacity_error_mode():
    """nf_capacity='error' refuses a model whose nfMax the device cannot hold."""
    hM = synthetic_model(ny=200, ns=200, nc=40, nf=2, seed=22, nf_default=True)
    with pytest.raises(ValueError, match="128"):
        H.Chain(hM, 1, device=0, updater={"GammaEta": False}, nf_capacity="error")
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        ch = H.Chain(hM, 1, device=0, updater={"GammaEta": False})
    assert any("held as 88" in str(x.message) for x in w)
    ch.close()


WIDE = {
    # K = 72: updateZ's 128-row instantiation, BetaLambda's workgroup path with a 72 x 72 factor,
    # GammaV / Gamma2 with nc = 70 (global scratch)
    "nc70": dict(ny=200, ns=40, nc=70, nf=2, seed=23),
    # sum(nf) = 70 > 64: two ZL passes, LambdaPriors / Eta at nf = 70 (eta_unit_kernel, nf^2 LDS)
    "nf70": dict(ny=240, ns=30, nc=4, nf=70, seed=24),
    # two levels, K = 100, NA cells (masked XZ rows of the 128-row kernel)
    "k100_na": dict(ny=220, ns=36, nc=60, nf=20, nr=2, units=[220, 40], na_frac=0.03, seed=25),
    # N = nc nt = 300 > 256: Gamma2's final stage in its sized LDS layout, the prep's and GammaV's
    # 300 x 300 systems in global scratch
    "n300": dict(ny=200, ns=80, nc=6, nf=2, nt=50, seed=27),
}


@pytest.fixture(scope="module", params=list(WIDE))
def wide(request):
    hM = synthetic_model(**WIDE[request.param])
    m = oracle_model(hM)
    seed = 24680
    return request.param, hM, m, seed, _oracle_state(m, seed)


def test_wide_init_parity(wide):
    name, hM, m, seed, _ = wide
    ch = _chain(hM, seed)
    g = ch.get_state()
    o = O.compute_initial_parameters(m, Rng(seed))
    for k in ("Gamma", "iV", "Beta", "iSigma", "Z"):
        assert rel_err(g[k], o[k]) < TOL_DRAW, (name, k, rel_err(g[k], o[k]))
    ch.close()


@pytest.mark.parametrize("upd", ["BetaLambda", "GammaV", "Gamma2", "LambdaPriors", "Eta", "Z"])
def test_wide_updater_parity(wide, upd):
    name, hM, m, seed, st = wide
    it = 7
    ch = _chain(hM, seed, st)
    ch.update(upd, it)
    g = ch.get_state()
    rng = Rng(seed)
    if upd == "BetaLambda":
        B, Lam = O.update_beta_lambda(st, m, rng, it)
        assert rel_err(g["Beta"], B) < TOL_DRAW, name
        for r in range(hM.nr):
            assert rel_err(g["Lambda"][r], Lam[r]) < TOL_DRAW, (name, r)
    elif upd == "GammaV":
        Gm, iV = O.update_gamma_v(st, m, rng, it)
        assert rel_err(g["iV"], iV) < TOL_WIDE_GAMMA, name
        assert rel_err(g["Gamma"], Gm) < TOL_WIDE_GAMMA, name
    elif upd == "Gamma2":
        assert rel_err(g["Gamma"], O.update_gamma2(st, m, rng, it)) < TOL_WIDE_GAMMA, name
    elif upd == "LambdaPriors":
        Psi, Delta = O.update_lambda_priors(st, m, rng, it)
        for r in range(hM.nr):
            assert rel_err(g["Psi"][r], Psi[r]) < TOL_DRAW, (name, r)
            assert rel_err(g["Delta"][r], Delta[r]) < TOL_DRAW, (name, r)
    elif upd == "Eta":
        Eta = O.update_eta(st, m, rng, it)
        for r in range(hM.nr):
            assert rel_err(g["Eta"][r], Eta[r]) < TOL_DRAW, (name, r, rel_err(g["Eta"][r], Eta[r]))
    elif upd == "Z":
        assert rel_err(g["Z"], O.update_z(st, m, rng, it)) < TOL_DRAW, name
    ch.close()


def test_wide_contractions(wide):
    """XZ and G of the 128-row z kernel equal their definitions on the stored Z."""
    name, hM, m, seed, st = wide
    ch = _chain(hM, seed, st)
    ch.update("Z", 5)
    Z = ch.get_state()["Z"]
    XEta, _ = O._xeta_and_prior(dict(st, Z=Z), m)
    K = XEta.shape[1]
    Kmax = int(ch.debug_get("dims", 8)[2])
    Yx = ~np.isnan(m["Y"])
    XZ = ch.debug_get("XZ", K * hM.ns).reshape(hM.ns, K).T
    assert rel_err(XZ, XEta.T @ np.where(Yx, Z, 0.0)) < 1e-12, name
    G = ch.debug_get("G", Kmax * Kmax).reshape(Kmax, Kmax).T[:K, :K]
    assert rel_err(G, XEta.T @ XEta) < 1e-12, name
    ch.close()


def test_wide_sweeps_track_oracle(wide):
    name, hM, m, seed, st = wide
    _track(hM, m, seed, st)


def test_wide_sample_predict_post():
    """sampleMcmc, predict (K = 72), variance partitioning (nc = 70) and associations
    (nf = 70) past the old 64 limits, against the oracle restatements."""
    hM = synthetic_model(ny=150, ns=24, nc=70, nf=2, seed=26)
    hM = H.sampleMcmc(hM, samples=6, transient=4, nChains=1, updater={"GammaEta": False}, seed=7, verbose=0)
    post = H.poolMcmcChains(hM.postList)
    Pi = hM.Pi.astype(np.int32)
    fam = hM.distr[:, 0].astype(int)
    ysp = np.asarray(hM.YScalePar)
    g = H.predict(hM, post=post, expected=True, seed=11)
    o = O.predict_samples(np.asarray(hM.X, dtype=np.float64), post, Pi, fam, ysp, True, Rng(11))
    for gs, os_ in zip(g, o):
        assert np.max(np.abs(gs - os_)) < 1e-9 * max(1.0, np.max(np.abs(os_)))
    d = H.computeVariancePartitioning(hM)
    v = P.computeVariancePartitioning(hM)
    assert rel_err(d["vals"], v["vals"]) < 1e-9
    # associations with nf = 70 factors per sample (a stored posterior, as test_gpu_post.py)
    rng = np.random.default_rng(5)
    hA = synthetic_model(ny=50, ns=20, nc=2, nf=2, seed=4)
    samples = [dict(Beta=rng.standard_normal((2, 20)), Gamma=rng.standard_normal((2, 1)),
                    Lambda=[rng.standard_normal((70 if k % 2 else 66, 20))]) for k in range(8)]
    hA.postList = [samples[:4], samples[4:]]
    hA.samples = 4
    d = H.computeAssociations(hA)
    o = P.computeAssociations(hA)
    assert rel_err(d[0]["mean"], o[0]["mean"]) < 1e-12
    np.testing.assert_array_equal(d[0]["support"], o[0]["support"])


@pytest.mark.parametrize("force_global", [False, True])
def test_gamma2_large_n(monkeypatch, force_global):
    """updateGamma2 past the old nc nt <= 256 (R/updateGamma2.R has no limit): N = 6 x 50 = 300
    and N = 12 x 30 = 360 against the oracle, with the final stage's arrays in LDS and, forced,
    in global memory (the layout a workgroup's LDS cannot hold, N >~ 1800)."""
    if force_global:
        monkeypatch.setenv("HMSC_G2F_GLOBAL", "1")
    for kw in (dict(ny=200, ns=80, nc=6, nf=2, nt=50, seed=28), dict(ny=180, ns=64, nc=12, nf=3, nt=30, seed=29)):
        hM = synthetic_model(**kw)
        m = oracle_model(hM)
        seed = 4242
        st = _oracle_state(m, seed)
        ch = _chain(hM, seed, st)
        ch.update("Gamma2", 9)
        g = ch.get_state()
        assert rel_err(g["Gamma"], O.update_gamma2(st, m, Rng(seed), 9)) < TOL_WIDE_GAMMA, kw
        ch.close()
