"""The reference's DEFAULT usage on the device, against the oracle.

* vignette_3's ``ma500`` (vignettes/vignette_3_multivariate_high.Rmd:445-453): a fresh
  HmscRandomLevel with default nfMin = 2 / nfMax = Inf (= ns = 50, R/Hmsc.R:554) and default
  updaters -- updateGammaEta on because nr >= 1 (R/sampleMcmc.R:124-152), with the phylogeny.
  The device bounds GammaEta's work by the nf in use (its workspace grows with updateNf), so
  nfMax = 50 is accepted.
* the same model with 5 % of Y missing: R's phylogeny branch factors the full
  kron(XEtaTXEta, diag(iSigma)) + P over the imputed Z (R/updateBetaLambda.R:124-146), and so
  does the device (no per-species masking in the phylogeny system).
* a model whose default nfMax exceeds this build's K = nc + sum(nf) <= 64: the level's buffers
  hold the capacity hmsc_get_nf_cap reports, the wrapper warns, and the chain runs.
* updateGammaEta with more than 16 factors in use, on the one-workgroup and the blocked path.
Every run follows the oracle on the same Philox stream."""
import warnings

import numpy as np
import pytest

from helpers import H, O, oracle_model, rel_err, synthetic_model
from oracle.rng import Rng
from hmsc_amd import workloads as W

pytestmark = pytest.mark.gpu

TOL_SWEEP = 1e-7
SEED = 50505


def _track(hM, n_sweeps=3, st=None, adapt=0, it0=1):
    """Device vs oracle over n_sweeps default-updater sweeps (the first `adapt` of them
    adaptive) from the oracle's initial state (or `st`)."""
    m = oracle_model(hM)
    dp = O.compute_data_parameters(m)
    rng = Rng(SEED)
    ch = H.Chain(hM, SEED, device=0, updater={})
    if st is None:
        ch.init()
        o = O.compute_initial_parameters(m, rng)
    else:
        ch.init()
        ch.set_state(st)
        o = dict(st)
    nf_dev, nf_orc = [], []
    for it in range(it0, it0 + n_sweeps):
        ad = it - it0 < adapt
        ch.sweep(it, adapt=ad)
        o = O.sweep(o, m, rng, it, data_par=dp, adapt_nf=[it0 + adapt - 1] * hM.nr if ad else None)
        nf_dev.append(tuple(int(v) for v in ch.nf()))
        nf_orc.append(tuple(l.shape[0] for l in o["Lambda"]))
    g = ch.get_state()
    return ch, g, o, nf_dev, nf_orc


def _assert_close(g, o, hM, tol=TOL_SWEEP):
    for k in ("Beta", "Gamma", "iV", "iSigma", "Z"):
        assert rel_err(g[k], o[k]) < tol, (k, rel_err(g[k], o[k]))
    for r in range(hM.nr):
        assert rel_err(g["Eta"][r], o["Eta"][r]) < tol, ("Eta", r, rel_err(g["Eta"][r], o["Eta"][r]))
        assert rel_err(g["Lambda"][r], o["Lambda"][r]) < tol, ("Lambda", r)


def test_ma500_default_spec_three_sweeps():
    hM = W.vignette3_ma500()
    assert hM.rL[0].nfMax == hM.ns == 50 and hM.rL[0].nfMin == 2
    with warnings.catch_warnings():
        warnings.simplefilter("error")          # nfMax = 50 fits: no capacity warning
        ch, g, o, _, _ = _track(hM, n_sweeps=3)
    assert ch.nf_cap == [50]
    assert g["rho"] == o["rho"]
    _assert_close(g, o, hM)
    ch.close()


def test_ma500_adaptive_phase_tracks_oracle():
    """updateNf during the transient (adaptNf = transient by default) with GammaEta and the
    phylogeny on: nf follows the oracle sweep by sweep."""
    hM = W.vignette3_ma500()
    ch, g, o, nf_dev, nf_orc = _track(hM, n_sweeps=30, adapt=30)
    assert nf_dev == nf_orc
    assert g["rho"] == o["rho"]
    _assert_close(g, o, hM, tol=1e-6)
    ch.close()


@pytest.mark.parametrize("ns", [50, 300])
def test_phylogeny_with_na_tracks_oracle(ns):
    """5 % NA in Y with the phylogeny (ns = 300: the blocked (nc + nf) ns system)."""
    hM = W.vignette3_ma500(ns=ns, na_frac=0.05)
    assert np.isnan(hM.Y).any()
    m = oracle_model(hM)
    dp = O.compute_data_parameters(m)
    rng = Rng(SEED)
    st = O.compute_initial_parameters(m, rng)
    st = O.sweep(st, m, rng, 1, data_par=dp)
    st["rho"] = 41
    # one-update conditional moments of the phylogeny BetaLambda over the imputed Z
    ch = H.Chain(hM, SEED, device=0, updater={})
    ch.init()
    ch.set_state(st)
    ch.set_noise_mode(1)
    ch.update("BetaLambda", 2)
    gm = ch.get_state(with_z=False)
    BL = O._beta_lambda_phylo(st, m, Rng(SEED), 2, dp, zero_noise=True)
    assert rel_err(gm["Beta"], BL[:hM.nc]) < 1e-10, rel_err(gm["Beta"], BL[:hM.nc])
    ch.close()
    ch, g, o, _, _ = _track(hM, n_sweeps=3, st=st, it0=2)
    assert g["rho"] == o["rho"]
    _assert_close(g, o, hM)
    ch.close()


def test_default_nfmax_above_the_latent_cap_runs():
    """nc = 20 and 200 species: R's default nfMax = 200 > 128 - 20.  The level holds 108
    factors (hmsc_get_nf_cap), the wrapper says so, and default-updater sweeps still follow the
    oracle."""
    hM = synthetic_model(ny=120, ns=200, nc=20, nf=2, seed=61)
    H.setPriors(hM.rL[0], nfMin=2, nfMax=200)
    with pytest.warns(UserWarning, match="held as 108"):
        ch = H.Chain(hM, SEED, device=0, updater={"GammaEta": False})
    assert ch.nf_cap == [108]
    ch.close()
    ch, g, o, _, _ = _track(hM, n_sweeps=3)
    _assert_close(g, o, hM)
    ch.close()


@pytest.mark.parametrize("kw", [dict(ny=60, ns=30, nc=2, nf=20, seed=62),      # one workgroup (nc ns = 60)
                                dict(ny=80, ns=300, nc=2, nf=18, seed=63)])    # blocked (nc ns = 600)
def test_gamma_eta_above_16_factors(kw):
    hM = synthetic_model(**kw)
    m = oracle_model(hM)
    dp = O.compute_data_parameters(m)
    rng = Rng(SEED)
    st = O.compute_initial_parameters(m, rng)
    st = O.sweep(st, m, rng, 1, data_par=dp)
    ch = H.Chain(hM, SEED, device=0, updater={})
    ch.init()
    ch.set_state(st)
    ch.set_noise_mode(1)
    ch.update("GammaEta", 2)
    g = ch.get_state(with_z=False)
    Gm, Eta = O.update_gamma_eta(st, m, Rng(SEED), 2, data_par=dp, zero_noise=True)
    assert rel_err(g["Gamma"], Gm) < 1e-10, rel_err(g["Gamma"], Gm)
    assert rel_err(g["Eta"][0], Eta[0]) < 1e-10, rel_err(g["Eta"][0], Eta[0])
    ch.set_noise_mode(0)
    ch.set_state(st)
    ch.update("GammaEta", 3)
    g = ch.get_state(with_z=False)
    Gm, Eta = O.update_gamma_eta(st, m, Rng(SEED), 3, data_par=dp)
    assert rel_err(g["Eta"][0], Eta[0]) < 1e-9
    ch.close()
