"""GPU parity of the phylogeny branch (hM$C != NULL) against the oracle.

The oracle follows the reference literally: the dense iQg / RQg / detQg grid of
R/computeDataParameters.R:19-39, iQg[,,rho] in updateGammaV (R/updateGammaV.R:14-32), 101
backsolves in updateRho (R/updateRho.R:14-17) and the dense (ns K)^2 Cholesky of
updateBetaLambda (R/updateBetaLambda.R:124-147).  The device uses the spectral form of the
same grid (hmsc_amd/csrc/phylo.hip); both share the Philox counters, so draws agree to fp64
rounding and the grid index drawn by updateRho agrees exactly.
"""
import numpy as np
import pytest

from helpers import H, O, oracle_model, phylo_corr, rel_err, synthetic_model
from oracle.rng import Rng

pytestmark = pytest.mark.gpu

TOL_MOMENT = 1e-10
TOL_DRAW = 1e-9
UPD = {"GammaEta": False}

MODELS = {
    # TD's dimensions (R/data-raw/simulateTestData.R: ns = 4, nc = 3, nt = 3, 50 sites)
    "phylo_td_dims": dict(ny=50, ns=4, nc=3, nf=2, nt=3, seed=21),
    "phylo_mid": dict(ny=120, ns=24, nc=3, nf=2, nt=2, seed=22),
    "phylo_two_levels": dict(ny=90, ns=10, nc=2, nf=2, nr=2, units=[90, 15], seed=23),
    # (nc + nf) ns above 1024: the multi-workgroup blocked Cholesky path (dense.hip)
    "phylo_blocked": dict(ny=150, ns=300, nc=3, nf=2, nt=2, seed=25),
    # config-3 class (vignette_3 scaled to hundreds of species): ns = 300, nf = 15, N = 5400
    "phylo_cfg3": dict(ny=200, ns=300, nc=3, nf=15, nt=2, seed=26),
}


@pytest.fixture(scope="module", params=list(MODELS))
def setup(request):
    kw = MODELS[request.param]
    hM = synthetic_model(C=phylo_corr(kw["ns"], seed=kw["seed"]), **kw)
    m = oracle_model(hM)
    dp = O.compute_data_parameters(m)
    seed = 55501
    rng = Rng(seed)
    st = O.compute_initial_parameters(m, rng)
    for it in range(1, 4):
        st = O.sweep(st, m, rng, it, updater=UPD, data_par=dp)
    st["rho"] = 37   # an interior grid point: exercises w = 1/q_rho away from rho = 0
    return request.param, hM, m, dp, seed, st


def _chain(hM, seed, st):
    ch = H.Chain(hM, seed, device=0, updater=UPD)
    ch.init()
    ch.set_state(st)
    return ch


def test_phylo_init_has_rho_one(setup):
    name, hM, m, dp, seed, _ = setup
    ch = H.Chain(hM, seed, device=0, updater=UPD)
    ch.init()
    assert ch.get_state()["rho"] == 1   # R/computeInitialParameters.R:226
    ch.close()


def test_phylo_beta_lambda_moments(setup):
    name, hM, m, dp, seed, st = setup
    ch = _chain(hM, seed, st)
    ch.set_noise_mode(1)
    ch.update("BetaLambda", 3)
    g = ch.get_state()
    BL = O._beta_lambda_phylo(st, m, Rng(seed), 3, dp, zero_noise=True)
    assert rel_err(g["Beta"], BL[:hM.nc]) < TOL_MOMENT, rel_err(g["Beta"], BL[:hM.nc])
    ch.close()


def test_phylo_beta_lambda_draw(setup):
    name, hM, m, dp, seed, st = setup
    ch = _chain(hM, seed, st)
    ch.update("BetaLambda", 9)
    g = ch.get_state()
    B, Lam = O.update_beta_lambda(st, m, Rng(seed), 9, dp)
    assert rel_err(g["Beta"], B) < TOL_DRAW
    for r in range(hM.nr):
        assert rel_err(g["Lambda"][r], Lam[r]) < TOL_DRAW
    ch.close()


def test_phylo_gamma_v_draw(setup):
    name, hM, m, dp, seed, st = setup
    ch = _chain(hM, seed, st)
    ch.update("GammaV", 6)
    g = ch.get_state()
    Gm, iV = O.update_gamma_v(st, m, Rng(seed), 6, dp)
    assert rel_err(g["iV"], iV) < TOL_DRAW
    assert rel_err(g["Gamma"], Gm) < TOL_DRAW
    ch.close()


def test_phylo_rho_draws(setup):
    """updateRho's categorical draw over the rhopw grid: the same index for many sweeps."""
    name, hM, m, dp, seed, st = setup
    ch = _chain(hM, seed, st)
    got, want = [], []
    for it in range(100, 140):
        ch.set_state({"rho": st["rho"]})
        ch.update("Rho", it)
        got.append(ch.get_state(with_z=False)["rho"])
        want.append(O.update_rho(st, m, Rng(seed), it, dp))
    assert got == want
    assert len(set(want)) > 3   # the posterior over the grid is not degenerate here
    ch.close()


def test_phylo_full_sweeps_track_oracle(setup):
    name, hM, m, dp, seed, st = setup
    ch = _chain(hM, seed, st)
    rng = Rng(seed)
    o = st
    for it in range(10, 14):
        ch.sweep(it)
        o = O.sweep(o, m, rng, it, updater=UPD, data_par=dp)
    g = ch.get_state()
    assert g["rho"] == o["rho"]
    for k in ("Beta", "Gamma", "iV", "Z"):
        assert rel_err(g[k], o[k]) < 1e-7, (name, k, rel_err(g[k], o[k]))
    ch.close()


def test_phylo_sample_mcmc_records_rho():
    hM = synthetic_model(ny=60, ns=6, nc=2, nf=2, seed=24, C=phylo_corr(6, seed=24))
    out = H.sampleMcmc(hM, samples=30, transient=10, nChains=1, updater=UPD, seed=4, verbose=0)
    rho = np.array([s["rho"] for s in out.postList[0]])
    assert np.all((rho >= 0) & (rho <= 1)) and np.unique(rho).size > 1
