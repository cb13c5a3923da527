"""GPU parity of updateGammaEta (R/updateGammaEta.R:7-206, non-spatial levels) against the
oracle restatement, which tests/test_oracle_gamma_eta.py pins to brute-force Gaussian
conditioning.  The device kernel (hmsc_amd/csrc/gamma_eta.hip) shares the Philox counters
with the oracle: the conditional means (noise mode 1) agree to 1e-10 and the draws to fp64
rounding; full default-updater sweeps (GammaEta on, as in TD$m and vignette_3) agree too."""
import numpy as np
import pytest

from helpers import H, O, oracle_model, phylo_corr, rel_err, synthetic_model
from oracle.rng import Rng

pytestmark = pytest.mark.gpu

TOL_MOMENT = 1e-10
TOL_DRAW = 1e-9
TOL_SWEEP = 1e-7

MODELS = {
    # TD's dimensions: ns = 4, nc = 3, nt = 3, 50 sites, observation-level units
    "td_dims": dict(ny=50, ns=4, nc=3, nf=2, nt=3, seed=41),
    "grouped_units": dict(ny=60, ns=6, nc=2, nf=2, units=[12], seed=42),
    "two_levels": dict(ny=48, ns=5, nc=3, nf=2, nr=2, units=[48, 8], seed=43),
    "phylo_td_dims": dict(ny=50, ns=4, nc=3, nf=2, nt=3, seed=44, phylo=True),
    # vignette_3 class: 50 species, nc = 3 -> a 150 x 150 dense system
    "vignette3_class": dict(ny=100, ns=50, nc=3, nf=3, seed=45, phylo=True),
    # nc ns > 512: the blocked path (one launch per segment, dense.hip factorizations)
    "blocked_obs": dict(ny=120, ns=200, nc=3, nf=3, seed=46, phylo=True),
    "blocked_grouped": dict(ny=90, ns=180, nc=3, nf=2, units=[15], seed=47),
    # config 3 (vignette_3: nc = 4, two traits + intercept, phylogeny) at 300 species
    "blocked_cfg3": dict(ny=200, ns=300, nc=4, nt=3, nf=5, seed=48, phylo=True),
    # nf > 64: the 128-factor instantiations, one workgroup and blocked
    "wide_nf80": dict(ny=60, ns=10, nc=3, nf=80, seed=49),
    "wide_nf72_blocked": dict(ny=80, ns=200, nc=3, nf=72, units=[20], seed=50),
}


@pytest.fixture(scope="module", params=list(MODELS))
def setup(request):
    kw = dict(MODELS[request.param])
    phylo = kw.pop("phylo", False)
    if phylo:
        kw["C"] = phylo_corr(kw["ns"], seed=kw["seed"])
    hM = synthetic_model(**kw)
    m = oracle_model(hM)
    dp = O.compute_data_parameters(m)
    seed = 31337
    rng = Rng(seed)
    st = O.compute_initial_parameters(m, rng)
    for it in range(1, 3):
        st = O.sweep(st, m, rng, it, data_par=dp)
    if phylo:
        st["rho"] = 37
    return request.param, hM, m, dp, seed, st


def _chain(hM, seed, st):
    ch = H.Chain(hM, seed, device=0, updater={})
    ch.init()
    ch.set_state(st)
    return ch


def test_gamma_eta_moments(setup):
    name, hM, m, dp, seed, st = setup
    ch = _chain(hM, seed, st)
    ch.set_noise_mode(1)
    ch.update("GammaEta", 5)
    g = ch.get_state()
    Gm, Eta = O.update_gamma_eta(st, m, Rng(seed), 5, data_par=dp, zero_noise=True)
    assert rel_err(g["Gamma"], Gm) < TOL_MOMENT, (name, rel_err(g["Gamma"], Gm))
    for r in range(hM.nr):
        assert rel_err(g["Eta"][r], Eta[r]) < TOL_MOMENT, (name, r, rel_err(g["Eta"][r], Eta[r]))
    ch.close()


def test_gamma_eta_draws(setup):
    name, hM, m, dp, seed, st = setup
    ch = _chain(hM, seed, st)
    ch.update("GammaEta", 6)
    g = ch.get_state()
    Gm, Eta = O.update_gamma_eta(st, m, Rng(seed), 6, data_par=dp)
    assert rel_err(g["Gamma"], Gm) < TOL_DRAW, (name, rel_err(g["Gamma"], Gm))
    for r in range(hM.nr):
        assert rel_err(g["Eta"][r], Eta[r]) < TOL_DRAW, (name, r)
    ch.close()


def test_default_updater_sweeps(setup):
    """Three sweeps of the reference's default updater set (GammaEta on) on both sides."""
    name, hM, m, dp, seed, st = setup
    ch = _chain(hM, seed, st)
    rng = Rng(seed)
    o = dict(st)
    for it in range(3, 6):
        ch.sweep(it)
        o = O.sweep(o, m, rng, it, data_par=dp)
    g = ch.get_state()
    for k in ("Beta", "Gamma", "iV", "Z"):
        assert rel_err(g[k], o[k]) < TOL_SWEEP, (name, k, rel_err(g[k], o[k]))
    for r in range(hM.nr):
        assert rel_err(g["Eta"][r], o["Eta"][r]) < TOL_SWEEP, (name, r)
    ch.close()


def test_recorded_run_with_gamma_eta():
    """sampleMcmc-style recorded run (graph replays) with GammaEta on: finite, right shapes."""
    hM = synthetic_model(**{k: v for k, v in MODELS["two_levels"].items()})
    ch = H.Chain(hM, 7, device=0, updater={})
    ch.init()
    rec = ch.run(transient=20, samples=30, thin=2)
    assert rec["Beta"].shape == (30, hM.nc, hM.ns)
    assert np.all(np.isfinite(rec["Beta"])) and np.all(np.isfinite(rec["Gamma"]))
    ch.close()
