"""GPU parity of spatial latent factors ('Full', 'NNGP', 'GPP') against the oracle:
updateEta's spatial branch (R/updateEta.R:111-140: one dense (np nf)^2 system over the
alphapw grid matrices iWg[,,alpha_h]) and updateAlpha (R/updateAlpha.R:20-79: grid
posterior from |RiWg eta_h|^2 and detWg).  The grids are computeDataParameters' (host,
R/computeDataParameters.R:53-81; the oracle recomputes them itself from the distances).
Both sides share the Philox counters: moments to 1e-10, draws to fp64 rounding, the drawn
grid indices exactly, and full sweeps; updateGammaEta's spatial branch further down."""
import numpy as np
import pytest

from helpers import H, O, oracle_model, phylo_corr, rel_err, synthetic_model
from oracle.rng import Rng

pytestmark = pytest.mark.gpu

TOL_MOMENT = 1e-10
TOL_DRAW = 1e-9
TOL_SWEEP = 1e-7
UPD = {"GammaEta": False}

MODELS = {
    # TD's plot level: 10 spatial units over 50 sampling units, plus the sample level
    "td_like": dict(ny=50, ns=4, nc=3, nf=2, nr=2, units=[50, 10], spatial=[1], seed=51, alpha_n=30),
    # observation-level spatial factors (np = ny), the default 101-point grid
    "obs_level": dict(ny=40, ns=6, nc=2, nf=2, nr=1, spatial=[0], seed=52),
    # NNGP (R/computeDataParameters.R:82-136) reaches the device as the unit coordinates: the
    # library builds the sparse Vecchia factor and factors the banded precision in reverse
    # Cuthill-McKee order (spatial.hip); GPP (:138-194) as R's low-rank arrays, sampled in R's form on both sides
    # (R/updateEta.R:148-196: oracle gpp_eta_literal, spatial.hip gpp_*); the oracle's GPP
    # updateAlpha is R's literal knot formula (R/updateAlpha.R:35-75)
    "nngp": dict(ny=40, ns=6, nc=2, nf=2, nr=1, spatial=[0], seed=53, spatial_method="NNGP", n_neighbours=6),
    "gpp": dict(ny=40, ns=6, nc=2, nf=2, nr=1, spatial=[0], seed=54, spatial_method="GPP", n_knots=4),
    # TD's shape with a phylogeny: updateGammaEta's spatial branch with iQ != I
    "td_like_phylo": dict(ny=50, ns=4, nc=3, nf=2, nr=2, units=[50, 10], spatial=[1], seed=56, alpha_n=30,
                          C=phylo_corr(4, seed=3)),
    "nngp_two_levels": dict(ny=40, ns=5, nc=2, nf=2, nr=2, units=[40, 8], spatial=[0], seed=55,
                            spatial_method="NNGP", alpha_n=20),
    # np nf > 1024: updateEta's system on the multi-workgroup blocked path (dense.hip)
    "large_full": dict(ny=700, ns=6, nc=2, nf=2, nr=1, spatial=[0], seed=57, alpha_n=20),
    "large_nngp": dict(ny=600, ns=5, nc=2, nf=2, nr=1, spatial=[0], seed=58, alpha_n=20,
                       spatial_method="NNGP", n_neighbours=8),
    # GPP in R's low-rank form at a size the dense path would not take cheaply: 25 knots, 3 factors
    "large_gpp": dict(ny=800, ns=5, nc=2, nf=3, nr=1, spatial=[0], seed=59, alpha_n=20,
                      spatial_method="GPP", n_knots=5),
}


@pytest.fixture(scope="module", params=list(MODELS))
def setup(request):
    hM = synthetic_model(**MODELS[request.param])
    m = oracle_model(hM)
    dp = O.compute_data_parameters(m)
    seed = 777
    rng = Rng(seed)
    st = O.compute_initial_parameters(m, rng)
    for it in range(1, 3):
        st = O.sweep(st, m, rng, it, updater=UPD, data_par=dp)
    r = [k for k, rl in enumerate(m["rL"]) if rl["sDim"]][0]
    # a smooth spatial field in Eta_r and an interior alpha: exercises both the grid
    # likelihood of updateAlpha and iWg[,,alpha] != I in updateEta
    xy = np.asarray(hM.rL[r].s)
    st["Eta"] = list(st["Eta"])
    st["Eta"][r] = np.column_stack([np.sin(3 * xy[:, 0]) + xy[:, 1], np.cos(2 * xy[:, 1]),
                                    xy[:, 0] * xy[:, 1] - 0.25])[:, :st["Eta"][r].shape[1]]
    st["Alpha"] = list(st["Alpha"])
    st["Alpha"][r] = np.array([7, 12, 4])[:st["Eta"][r].shape[1]]
    return request.param, hM, m, dp, seed, st, r


def _chain(hM, seed, st):
    ch = H.Chain(hM, seed, device=0, updater=UPD)
    ch.init()
    ch.set_state(st)
    return ch


def test_state_roundtrip_alpha(setup):
    name, hM, m, dp, seed, st, r = setup
    ch = _chain(hM, seed, st)
    g = ch.get_state()
    assert np.array_equal(g["Alpha"][r], st["Alpha"][r])
    ch.close()


def test_spatial_eta_moments(setup):
    name, hM, m, dp, seed, st, r = setup
    ch = _chain(hM, seed, st)
    ch.set_noise_mode(1)
    ch.update("Eta", 4)
    g = ch.get_state()
    Eta = O.update_eta(st, m, Rng(seed), 4, zero_noise=True, data_par=dp)
    for q in range(hM.nr):
        assert rel_err(g["Eta"][q], Eta[q]) < TOL_MOMENT, (name, q, rel_err(g["Eta"][q], Eta[q]))
    ch.close()


def test_spatial_eta_draws(setup):
    name, hM, m, dp, seed, st, r = setup
    ch = _chain(hM, seed, st)
    ch.update("Eta", 5)
    g = ch.get_state()
    Eta = O.update_eta(st, m, Rng(seed), 5, data_par=dp)
    for q in range(hM.nr):
        assert rel_err(g["Eta"][q], Eta[q]) < TOL_DRAW, (name, q)
    ch.close()


def test_alpha_draws(setup):
    name, hM, m, dp, seed, st, r = setup
    ch = _chain(hM, seed, st)
    picks = []
    for it in (6, 7, 8, 9):
        ch.update("Alpha", it)
        g = ch.get_state()
        a = O.update_alpha(st, m, Rng(seed), it, dp)
        assert np.array_equal(g["Alpha"][r], a[r]), (name, it, g["Alpha"][r], a[r])
        picks.append(a[r])
    assert np.any(np.concatenate(picks) > 1), picks   # the smooth field moves alpha off 0
    ch.close()


def test_spatial_sweeps(setup):
    name, hM, m, dp, seed, st, r = setup
    ch = _chain(hM, seed, st)
    rng = Rng(seed)
    o = dict(st)
    for it in range(3, 6):
        ch.sweep(it)
        o = O.sweep(o, m, rng, it, updater=UPD, data_par=dp)
    g = ch.get_state()
    for k in ("Beta", "Gamma", "iV", "Z"):
        assert rel_err(g[k], o[k]) < TOL_SWEEP, (name, k, rel_err(g[k], o[k]))
    for q in range(hM.nr):
        assert rel_err(g["Eta"][q], o["Eta"][q]) < TOL_SWEEP, (name, q)
        assert np.array_equal(g["Alpha"][q], o["Alpha"][q])
    ch.close()


def test_spatial_recorded_run(setup):
    name, hM, m, dp, seed, st, r = setup
    ch = _chain(hM, seed, st)
    rec = ch.run(transient=10, samples=20, thin=1, iter0=5)
    a = rec[f"Alpha{r}"]
    assert a.shape[0] == 20 and np.all(a >= 1) and np.all(a <= hM.rL[r].alphapw.shape[0])
    assert np.all(np.isfinite(rec["Beta"]))
    ch.close()


# updateGammaEta's spatial 'Full' branch (R/updateGammaEta.R:139-198): the joint (Gamma, Eta_r)
# draw with Beta integrated out, default updater set (GammaEta on, as TD$m runs it)
GE_MODELS = [k for k in MODELS if "nngp" not in k and "gpp" not in k]


@pytest.fixture(scope="module", params=GE_MODELS)
def ge_setup(request):
    hM = synthetic_model(**MODELS[request.param])
    m = oracle_model(hM)
    dp = O.compute_data_parameters(m)
    seed = 778
    rng = Rng(seed)
    st = O.compute_initial_parameters(m, rng)
    for it in range(1, 3):
        st = O.sweep(st, m, rng, it, data_par=dp)
    r = [k for k, rl in enumerate(m["rL"]) if rl["sDim"]][0]
    st["Alpha"] = list(st["Alpha"])
    st["Alpha"][r] = np.array([7, 12])[:st["Eta"][r].shape[1]]
    return request.param, hM, m, dp, seed, st


def _ge_chain(hM, seed, st):
    ch = H.Chain(hM, seed, device=0, updater={})
    ch.init()
    ch.set_state(st)
    return ch


# "auto": one workgroup up to nc nt + np nf = 1024 (large_full is above it: the blocked grid
# path); "blocked": every model forced onto the blocked path (grid stages, dense.hip Cholesky)
GE_PATHS = ["auto", "blocked"]


@pytest.mark.parametrize("path", GE_PATHS)
def test_spatial_gamma_eta_moments(ge_setup, path, monkeypatch):
    name, hM, m, dp, seed, st = ge_setup
    if path == "blocked":
        monkeypatch.setenv("HMSC_GES_BLOCKED", "1")
    ch = _ge_chain(hM, seed, st)
    ch.set_noise_mode(1)
    ch.update("GammaEta", 5)
    g = ch.get_state()
    Gm, Eta = O.update_gamma_eta(st, m, Rng(seed), 5, data_par=dp, zero_noise=True)
    assert rel_err(g["Gamma"], Gm) < TOL_MOMENT, (name, rel_err(g["Gamma"], Gm))
    for q in range(hM.nr):
        assert rel_err(g["Eta"][q], Eta[q]) < TOL_MOMENT, (name, q, rel_err(g["Eta"][q], Eta[q]))
    ch.close()


@pytest.mark.parametrize("path", GE_PATHS)
def test_spatial_gamma_eta_draws(ge_setup, path, monkeypatch):
    name, hM, m, dp, seed, st = ge_setup
    if path == "blocked":
        monkeypatch.setenv("HMSC_GES_BLOCKED", "1")
    ch = _ge_chain(hM, seed, st)
    ch.update("GammaEta", 6)
    g = ch.get_state()
    Gm, Eta = O.update_gamma_eta(st, m, Rng(seed), 6, data_par=dp)
    assert rel_err(g["Gamma"], Gm) < TOL_DRAW, (name, rel_err(g["Gamma"], Gm))
    for q in range(hM.nr):
        assert rel_err(g["Eta"][q], Eta[q]) < TOL_DRAW, (name, q)
    ch.close()


def test_spatial_default_updater_sweeps(ge_setup):
    name, hM, m, dp, seed, st = ge_setup
    ch = _ge_chain(hM, seed, st)
    rng = Rng(seed)
    o = dict(st)
    for it in range(3, 6):
        ch.sweep(it)
        o = O.sweep(o, m, rng, it, data_par=dp)
    g = ch.get_state()
    for k in ("Beta", "Gamma", "iV", "Z"):
        assert rel_err(g[k], o[k]) < TOL_SWEEP, (name, k, rel_err(g[k], o[k]))
    for q in range(hM.nr):
        assert rel_err(g["Eta"][q], o["Eta"][q]) < TOL_SWEEP, (name, q)
        assert np.array_equal(g["Alpha"][q], o["Alpha"][q])
    ch.close()


def test_spatial_recorded_run_default_updaters(ge_setup):
    name, hM, m, dp, seed, st = ge_setup
    ch = _ge_chain(hM, seed, st)
    rec = ch.run(transient=10, samples=20, thin=1, iter0=5)
    assert np.all(np.isfinite(rec["Beta"])) and np.all(np.isfinite(rec["Gamma"]))
    ch.close()
