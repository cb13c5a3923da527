"""BASELINE config 3 as the vignette specifies it, under -m gpu: vignette_3's model
(vignettes/vignette_3_multivariate_high.Rmd:42-133) at 300 species -- NORMAL-family Y, so the
residual precisions iSigma != 1 enter the phylogeny BetaLambda system
(R/updateBetaLambda.R:124-147, kron(XEtaTXEta, diag(iSigma))) and updateGammaEta's id weights
(R/updateGammaEta.R:26-60) -- with the phylogeny (Rho on), traits (nt = 3), nc = 4 and the
default updaters.  nc ns = 1200 and (nc + nf) ns >= 1800 put both dense systems on the blocked
multi-workgroup factorizations (dense.hip).  Every check is against the oracle on the same
Philox stream: one-update conditional moments (noise mode) to 1e-10, draws to 1e-9,
default-updater sweeps, and an updateNf adaptive phase (nfMin = 2, nfMax = 15) followed
sweep by sweep with both the phylogeny and GammaEta on (R/updateNf.R:3-70)."""
import numpy as np
import pytest

from helpers import H, O, oracle_model, rel_err
from oracle.rng import Rng
from hmsc_amd import workloads as W

pytestmark = pytest.mark.gpu

TOL_MOMENT = 1e-10
TOL_DRAW = 1e-9
TOL_SWEEP = 1e-7
SEED = 30303


@pytest.fixture(scope="module")
def cfg3():
    hM = W.vignette3_phylo(ns=300, ny=200)
    m = oracle_model(hM)
    dp = O.compute_data_parameters(m)
    rng = Rng(SEED)
    st = O.compute_initial_parameters(m, rng)
    for it in range(1, 3):
        st = O.sweep(st, m, rng, it, data_par=dp)
    st["rho"] = 37   # an interior grid point of rhopw
    return hM, m, dp, st


def _chain(hM, st):
    ch = H.Chain(hM, SEED, device=0, updater={})
    ch.init()
    ch.set_state(st)
    return ch


def test_config3_is_the_vignette_model(cfg3):
    hM, m, dp, st = cfg3
    assert hM.ns == 300 and hM.nc == 4 and hM.nt == 3 and hM.C is not None
    assert np.all(np.asarray(hM.distr)[:, 0] == 1)          # normal family
    assert np.ptp(st["iSigma"]) > 0.1                        # iSigma != 1 in the state fed below
    assert hM.nc * hM.ns > 512                               # GammaEta on the blocked path
    K = hM.nc + st["Lambda"][0].shape[0]
    assert K * hM.ns > 1024                                  # phylogeny BetaLambda blocked too


def test_config3_phylo_beta_lambda_moments(cfg3):
    hM, m, dp, st = cfg3
    ch = _chain(hM, st)
    ch.set_noise_mode(1)
    ch.update("BetaLambda", 4)
    g = ch.get_state()
    BL = O._beta_lambda_phylo(st, m, Rng(SEED), 4, dp, zero_noise=True)
    nc = hM.nc
    assert rel_err(g["Beta"], BL[:nc]) < TOL_MOMENT, rel_err(g["Beta"], BL[:nc])
    assert rel_err(g["Lambda"][0], BL[nc:]) < TOL_MOMENT, rel_err(g["Lambda"][0], BL[nc:])
    ch.close()


def test_config3_phylo_beta_lambda_draw(cfg3):
    hM, m, dp, st = cfg3
    ch = _chain(hM, st)
    ch.update("BetaLambda", 5)
    g = ch.get_state()
    B, Lam = O.update_beta_lambda(st, m, Rng(SEED), 5, dp)
    assert rel_err(g["Beta"], B) < TOL_DRAW, rel_err(g["Beta"], B)
    assert rel_err(g["Lambda"][0], Lam[0]) < TOL_DRAW
    ch.close()


def test_config3_gamma_eta_moments(cfg3):
    hM, m, dp, st = cfg3
    ch = _chain(hM, st)
    ch.set_noise_mode(1)
    ch.update("GammaEta", 6)
    g = ch.get_state()
    Gm, Eta = O.update_gamma_eta(st, m, Rng(SEED), 6, data_par=dp, zero_noise=True)
    assert rel_err(g["Gamma"], Gm) < TOL_MOMENT, rel_err(g["Gamma"], Gm)
    assert rel_err(g["Eta"][0], Eta[0]) < TOL_MOMENT, rel_err(g["Eta"][0], Eta[0])
    ch.close()


def test_config3_gamma_eta_draws(cfg3):
    hM, m, dp, st = cfg3
    ch = _chain(hM, st)
    ch.update("GammaEta", 7)
    g = ch.get_state()
    Gm, Eta = O.update_gamma_eta(st, m, Rng(SEED), 7, data_par=dp)
    assert rel_err(g["Gamma"], Gm) < TOL_DRAW, rel_err(g["Gamma"], Gm)
    assert rel_err(g["Eta"][0], Eta[0]) < TOL_DRAW
    ch.close()


def test_config3_default_updater_sweeps(cfg3):
    hM, m, dp, st = cfg3
    ch = _chain(hM, st)
    rng = Rng(SEED)
    o = dict(st)
    for it in range(3, 7):
        ch.sweep(it)
        o = O.sweep(o, m, rng, it, data_par=dp)
    g = ch.get_state()
    assert g["rho"] == o["rho"]
    for k in ("Beta", "Gamma", "iV", "iSigma", "Z"):
        assert rel_err(g[k], o[k]) < TOL_SWEEP, (k, rel_err(g[k], o[k]))
    assert rel_err(g["Eta"][0], o["Eta"][0]) < TOL_SWEEP
    assert rel_err(g["Lambda"][0], o["Lambda"][0]) < TOL_SWEEP
    ch.close()


def test_config3_update_nf_with_phylogeny_and_gamma_eta(cfg3):
    """The adaptive phase of the config-3 bench: from nfMin = 2 the level gains factors
    (R/updateNf.R:24-45) while the phylogeny BetaLambda (its (nc + nf) ns system growing with
    nf) and the blocked GammaEta (its workspace growing with nf) run every sweep."""
    hM, m, dp, _ = cfg3
    ch = H.Chain(hM, SEED, device=0, updater={})
    ch.init([2])
    rng = Rng(SEED)
    o = O.compute_initial_parameters(m, rng, nf=[2])
    n_adapt = 40
    nf_dev, nf_orc = [], []
    for it in range(1, n_adapt + 1):
        ch.sweep(it, adapt=True)
        o = O.sweep(o, m, rng, it, data_par=dp, adapt_nf=[n_adapt])
        nf_dev.append(int(ch.nf()[0]))
        nf_orc.append(o["Lambda"][0].shape[0])
    assert nf_dev == nf_orc
    assert max(nf_dev) > 2, "nf never grew: the test did not exercise updateNf"
    g = ch.get_state()
    assert g["rho"] == o["rho"]
    for k in ("Beta", "Gamma", "iV", "iSigma"):
        assert rel_err(g[k], o[k]) < 1e-6, (k, rel_err(g[k], o[k]))
    assert rel_err(g["Lambda"][0], o["Lambda"][0]) < 1e-6
    assert rel_err(g["Eta"][0], o["Eta"][0]) < 1e-6
    assert rel_err(g["Delta"][0], o["Delta"][0]) < 1e-6
    # then the steady state at the adapted nf (captured graphs of the dense sweep)
    rec = ch.run(transient=0, samples=4, thin=1, adaptNf=[0], iter0=n_adapt)
    assert np.all(rec["nf"] == nf_dev[-1]) and np.all(np.isfinite(rec["Beta"]))
    ch.close()
