"""Spatial levels past the sizes of tests/test_gpu_spatial.py (BASELINE config 5):

  * NNGP in the sparse Vecchia form (spatial.hip): the device's reverse Cuthill-McKee order of
    the units equals the oracle's (oracle/hmsc_oracle.py nngp_rcm), and at np = 1000 with two
    factors updateEta's conditional mean (noise off) matches the oracle to 1e-9, its draw to
    1e-8, updateAlpha's grid indices exactly, two full sweeps to 1e-7;
  * 'Full' at np = 2048 (the blocked multi-workgroup Eta system, the device-built alphapw grid
    on a reduced 11-point grid so that the oracle's dense grid fits): Eta moments, draws and
    Alpha draws against the oracle.
"""
import numpy as np
import pytest

from helpers import H, O, oracle_model, rel_err, synthetic_model
from oracle.rng import Rng

pytestmark = pytest.mark.gpu

UPD = {"GammaEta": False}


def _setup(kw, seed=777, sweeps=1):
    hM = synthetic_model(**kw)
    m = oracle_model(hM)
    dp = O.compute_data_parameters(m)
    rng = Rng(seed)
    st = O.compute_initial_parameters(m, rng)
    for it in range(1, sweeps + 1):
        st = O.sweep(st, m, rng, it, updater=UPD, data_par=dp)
    r = 0
    xy = np.asarray(hM.rL[r].s)
    nf = st["Eta"][r].shape[1]
    st["Eta"] = list(st["Eta"])
    st["Eta"][r] = np.column_stack([np.sin(3 * xy[:, 0]) + xy[:, 1], np.cos(2 * xy[:, 1])])[:, :nf]
    st["Alpha"] = [np.array([4, 7])[:nf]]
    return hM, m, dp, seed, st


def _chain(hM, seed, st):
    ch = H.Chain(hM, seed, device=0, updater=UPD)
    ch.init()
    ch.set_state(st)
    return ch


NNGP_SMALL = dict(ny=300, ns=5, nc=2, nf=2, nr=1, spatial=[0], seed=71, alpha_n=10, spatial_method="NNGP",
                  n_neighbours=10)
NNGP_LARGE = dict(ny=1000, ns=5, nc=2, nf=2, nr=1, spatial=[0], seed=72, alpha_n=20, spatial_method="NNGP",
                  n_neighbours=10)
FULL_LARGE = dict(ny=2048, ns=5, nc=2, nf=1, nr=1, spatial=[0], seed=73, alpha_n=10)


def test_nngp_order_matches_oracle():
    hM, m, dp, seed, st = _setup(NNGP_SMALL)
    ch = _chain(hM, seed, st)
    perm = ch.debug_get("nngp_perm0", hM.np[0]).astype(np.int64)
    bw = int(ch.debug_get("nngp_bw0", 1)[0])
    ch.close()
    par = dp["rLPar"][0]
    np.testing.assert_array_equal(perm, par["perm"])
    assert bw == par["bw_units"] and bw < hM.np[0] // 2


@pytest.fixture(scope="module")
def nngp_large():
    return _setup(NNGP_LARGE)


def test_nngp_large_eta_moments_and_draws(nngp_large):
    hM, m, dp, seed, st = nngp_large
    ch = _chain(hM, seed, st)
    ch.set_noise_mode(1)
    ch.update("Eta", 4)
    g = ch.get_state()
    mean = O.update_eta(st, m, Rng(seed), 4, zero_noise=True, data_par=dp)
    assert rel_err(g["Eta"][0], mean[0]) < 1e-9
    ch.set_noise_mode(0)
    ch.set_state(st)
    ch.update("Eta", 5)
    g = ch.get_state()
    draw = O.update_eta(st, m, Rng(seed), 5, data_par=dp)
    ch.close()
    assert rel_err(g["Eta"][0], draw[0]) < 1e-8


def test_nngp_large_alpha_draws(nngp_large):
    hM, m, dp, seed, st = nngp_large
    ch = _chain(hM, seed, st)
    for it in (6, 7, 8):
        ch.update("Alpha", it)
        a = O.update_alpha(st, m, Rng(seed), it, dp)
        assert np.array_equal(ch.get_state()["Alpha"][0], a[0]), it
    ch.close()


def test_nngp_large_sweeps(nngp_large):
    hM, m, dp, seed, st = nngp_large
    ch = _chain(hM, seed, st)
    rng = Rng(seed)
    o = dict(st)
    for it in range(3, 5):
        ch.sweep(it)
        o = O.sweep(o, m, rng, it, updater=UPD, data_par=dp)
    g = ch.get_state()
    ch.close()
    for k in ("Beta", "Gamma", "iV", "Z"):
        assert rel_err(g[k], o[k]) < 1e-7, (k, rel_err(g[k], o[k]))
    assert rel_err(g["Eta"][0], o["Eta"][0]) < 1e-7
    assert np.array_equal(g["Alpha"][0], o["Alpha"][0])


@pytest.fixture(scope="module")
def full_large():
    return _setup(FULL_LARGE)


def test_full_large_eta_and_alpha(full_large):
    hM, m, dp, seed, st = full_large
    ch = _chain(hM, seed, st)
    ch.set_noise_mode(1)
    ch.update("Eta", 4)
    mean = O.update_eta(st, m, Rng(seed), 4, zero_noise=True, data_par=dp)
    assert rel_err(ch.get_state()["Eta"][0], mean[0]) < 1e-9
    ch.set_noise_mode(0)
    ch.set_state(st)
    ch.update("Eta", 5)
    draw = O.update_eta(st, m, Rng(seed), 5, data_par=dp)
    assert rel_err(ch.get_state()["Eta"][0], draw[0]) < 1e-8
    ch.set_state(st)
    for it in (6, 7):
        ch.update("Alpha", it)
        a = O.update_alpha(st, m, Rng(seed), it, dp)
        assert np.array_equal(ch.get_state()["Alpha"][0], a[0]), it
    ch.close()


def test_nngp_band_storage_is_linear():
    """np = 12000, nf = 2: the NNGP level's band matrix is held in the tile-band layout
    (dense.hip aix), O(N bw) doubles -- a dense (np nf)^2 array would be 4.6 GB -- and
    default-updater sweeps run on it with finite states (R factors the same matrix as a sparse
    one, R/updateEta.R:137-147)."""
    hM = synthetic_model(ny=12000, ns=3, nc=2, nf=2, nr=1, spatial=[0], seed=74, alpha_n=10,
                         spatial_method="NNGP", n_neighbours=10)
    ch = H.Chain(hM, 5, device=0, updater=UPD)
    ch.init()
    units = int(ch.debug_get("nngp_bw0", 1)[0])
    N, bw = 12000 * 2, (units + 1) * 2 - 1
    work = float(ch.debug_get("spwork_doubles0", 1)[0])
    assert work < N * (bw + 200) + 64 * N + 4e6, (work, N, bw)
    assert work < 0.05 * N * N
    for it in range(1, 4):
        ch.sweep(it)
    g = ch.get_state()
    assert np.isfinite(g["Eta"][0]).all() and np.isfinite(g["Beta"]).all()
    ch.close()
