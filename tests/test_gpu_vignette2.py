"""BASELINE.json config 2 on the device: vignettes/vignette_2_multivariate_low.Rmd.

Both of the vignette's non-latent models have no random level (nr = 0): the 5-species
normal model (:55) and the normal / probit / Poisson / lognormal-Poisson model (:299).
With nr = 0 the sweep is Gamma2 (acts only when every iSigma == 1), BetaLambda over the
nc covariates alone, GammaV, InvSigma and Z (R/sampleMcmc.R:221-294; GammaEta switches
itself off, :150-152).  Checked against the oracle:
  * init, one updater at a time (draws 1e-9) and BetaLambda's conditional moments (1e-10),
  * three full sweeps (1e-7) and graph-replayed recorded runs equal to eager ones,
  * sampleMcmc end to end (72 hM fields, 13 per sample, empty Eta / Lambda lists),
  * the posterior of 8 GPU chains against 4 oracle chains (tests/golden/vignette2_posterior.npz)
    for the two nr = 0 models and the vignette's sample-level model (:143, GammaEta on):
    means within Monte Carlo error, Gelman-Rubin over both sides, KS on thinned draws.
The posterior fixture is produced by this repository's CPU oracle
(tests/golden/make_vignette2_fixture.py), not by the reference: R is absent and
/root/reference holds no vignette_2 posterior draws (its PDF shows only ESS / summary tables),
so the posterior checks are oracle-relative -- the device chains against the oracle's chains.
The oracle itself is pinned to the reference by the TD fixtures.
"""
import os

import numpy as np
import pytest
from scipy import stats

import hmsc_amd as H
from helpers import O, oracle_model, rel_err
from oracle.rng import Rng
from vignette2_common import (MODELS, SAMPLES, THIN, TRANSIENT, UPDATER, model, summarise, unpack_state)

pytestmark = pytest.mark.gpu

FIX = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "vignette2_posterior.npz"))
NR0 = ("linear", "mixed")
UP = {"GammaEta": False}


@pytest.fixture(scope="module", params=NR0)
def nr0(request):
    hM = model(request.param)
    assert hM.nr == 0
    m = oracle_model(hM)
    seed = 24680
    rng = Rng(seed)
    st = O.compute_initial_parameters(m, rng)
    for it in range(1, 4):
        st = O.sweep(st, m, rng, it, updater=UP)
    return request.param, hM, m, seed, st


def _chain(hM, seed, st=None):
    ch = H.Chain(hM, seed, device=0, updater=UP)
    ch.init()
    if st is not None:
        ch.set_state(st)
    return ch


def test_nr0_init(nr0):
    name, hM, m, seed, _ = nr0
    ch = _chain(hM, seed)
    g = ch.get_state()
    ch.close()
    o = O.compute_initial_parameters(m, Rng(seed))
    for k in ("Gamma", "iV", "Beta", "iSigma", "Z"):
        assert rel_err(g[k], o[k]) < 1e-9, (name, k)
    assert g["Eta"] == [] and g["Lambda"] == []


@pytest.mark.parametrize("upd", ["BetaLambda", "GammaV", "Gamma2", "InvSigma", "Z"])
def test_nr0_updater_draws(nr0, upd):
    name, hM, m, seed, st = nr0
    it = 9
    ch = _chain(hM, seed, st)
    ch.update(upd, it)
    g = ch.get_state()
    ch.close()
    rng = Rng(seed)
    if upd == "BetaLambda":
        B, _ = O.update_beta_lambda(st, m, rng, it)
        assert rel_err(g["Beta"], B) < 1e-9
    elif upd == "GammaV":
        Gm, iV = O.update_gamma_v(st, m, rng, it)
        assert rel_err(g["iV"], iV) < 1e-9 and rel_err(g["Gamma"], Gm) < 1e-9
    elif upd == "Gamma2":
        assert rel_err(g["Gamma"], O.update_gamma2(st, m, rng, it)) < 1e-9
    elif upd == "InvSigma":
        assert rel_err(g["iSigma"], O.update_inv_sigma(st, m, rng, it)) < 1e-9
    else:
        assert rel_err(g["Z"], O.update_z(st, m, rng, it)) < 1e-9


def test_nr0_beta_moments(nr0):
    name, hM, m, seed, st = nr0
    ch = _chain(hM, seed, st)
    ch.set_noise_mode(1 | 2)
    ch.update("BetaLambda", 3)
    g = ch.get_state()
    K = hM.nc
    dp = ch.debug_get("BL_prec", hM.ns * K * K).reshape(hM.ns, K, K).transpose(0, 2, 1)
    ch.close()
    precs, means = O.beta_lambda_moments(st, m)
    assert means.shape[0] == K
    assert rel_err(g["Beta"], means) < 1e-10
    assert rel_err(dp, precs) < 1e-10


def test_nr0_full_sweeps(nr0):
    name, hM, m, seed, st = nr0
    ch = _chain(hM, seed, st)
    rng = Rng(seed)
    o = st
    for it in range(20, 23):
        ch.sweep(it)
        o = O.sweep(o, m, rng, it, updater=UP)
    g = ch.get_state()
    ch.close()
    for k in ("Beta", "Gamma", "iV", "iSigma", "Z"):
        assert rel_err(g[k], o[k]) < 1e-7, (name, k, rel_err(g[k], o[k]))


def test_nr0_graph_replay_matches_eager(monkeypatch, nr0):
    name, hM, _, seed, _ = nr0
    out = []
    for no_graph in ("1", "0"):
        monkeypatch.setenv("HMSC_NO_GRAPH", no_graph)
        monkeypatch.setenv("HMSC_GRAPH_SWEEPS", "4")
        ch = _chain(hM, seed)
        out.append(ch.run(transient=3, samples=21, thin=2, adaptNf=[]))
        ch.close()
    for k in ("Beta", "Gamma", "iV", "iSigma"):
        np.testing.assert_array_equal(out[0][k], out[1][k], err_msg=k)


def test_nr0_sample_mcmc_end_to_end():
    hM = model("mixed")
    out = H.sampleMcmc(hM, samples=30, transient=10, nChains=2, seed=5, verbose=0)   # default updaters
    assert len(out) == 72 and len(out.postList) == 2 and len(out.postList[0]) == 30
    s = out.postList[1][7]
    assert len(s) == 13 and s["Beta"].shape == (3, 4) and s["Eta"] == [] and s["Lambda"] == []
    assert np.all(np.isfinite(s["Beta"])) and s["sigma"].shape == (4,)
    mp, cols = H.convertToCodaObject(out)
    assert mp["Beta"][0].shape == (30, 12) and cols["Beta"][0].startswith("B[(Intercept) (C1)")


# ---------------------------------------------------------------------------------------
# posterior against the oracle's chains
# ---------------------------------------------------------------------------------------
N_GPU = 8


@pytest.fixture(scope="module", params=MODELS)
def both(request):
    name = request.param
    hM = model(name)
    start = unpack_state(FIX, f"{name}/start", hM.nr)
    chains = []
    for c in range(N_GPU):
        ch = H.Chain(hM, 1 + c, device=0, updater=UPDATER[name])
        ch.init()
        ch.set_state(start)
        rec = ch.run(transient=TRANSIENT, samples=SAMPLES, thin=THIN[name], adaptNf=[0] * hM.nr)
        ch.close()
        d = dict(Beta=rec["Beta"], Gamma=rec["Gamma"], iV=rec["iV"], iSigma=rec["iSigma"])
        if hM.nr:
            d["Lambda0"] = rec["Lambda0"][:, :int(rec["nf"][0][0]), :]
        chains.append(d)
    g = summarise(hM, chains)
    c = {k: FIX[f"{name}/{k}"] for k in ("draws", "mean", "sd", "ess")}
    return name, g, c


def _pooled(s):
    mean = s["mean"].mean(axis=0)
    var = np.sum(s["sd"] ** 2 / np.maximum(s["ess"], 1.0), axis=0) / s["mean"].shape[0] ** 2
    return mean, var


def test_posterior_means(both):
    name, g, c = both
    mg, vg = _pooled(g)
    mc, vc = _pooled(c)
    live = (vg + vc) > 0
    z = np.abs(mg - mc)[live] / np.sqrt(vg + vc)[live]
    assert np.mean(z > 3.5) <= 0.03 and z.max() < 6.0, (name, np.sort(z)[-5:])


def test_posterior_gelman_rubin(both):
    name, g, c = both
    chains = [x.astype(np.float64) for x in list(g["draws"]) + list(c["draws"])]
    live = (np.std(np.concatenate(chains), axis=0) > 0) & (np.minimum(g["ess"].min(0), c["ess"].min(0)) >= 10)
    point, _ = H.gelman_diag([x[:, live] for x in chains])
    assert np.all(point < 1.2) and np.mean(point > 1.1) <= 0.05, (name, np.sort(point)[-5:])


def test_posterior_ks(both):
    name, g, c = both
    dg = g["draws"].reshape(-1, g["draws"].shape[-1])
    dc = c["draws"].reshape(-1, c["draws"].shape[-1])
    ess = np.minimum(g["ess"].sum(axis=0), c["ess"].sum(axis=0))
    pvals = []
    for p in range(dg.shape[1]):
        if np.std(dc[:, p]) == 0:
            continue
        step = max(1, int(round(dg.shape[0] / max(ess[p], 1.0))))
        pvals.append(stats.ks_2samp(dg[::step, p], dc[::step, p]).pvalue)
    pvals = np.array(pvals)
    assert np.mean(pvals < 1e-3) <= 0.03, (name, np.sort(pvals)[:5])
