"""GPU parity: every device updater against the CPU oracle on the same state and key.

Fed a fixed state, each HIP updater (through the C ABI) must reproduce the oracle
restatement of the reference R updater: conditional means and precisions to
1e-10 relative (noise mode 1 zeroes every Gaussian innovation), and the draws
themselves to fp64 rounding because both sides share the Philox counter contract.
"""
import numpy as np
import pytest

from helpers import H, O, oracle_model, rel_err, synthetic_model
from oracle.rng import Rng

pytestmark = pytest.mark.gpu

TOL_MOMENT = 1e-10   # north_star: conditional mean/precision within 1e-10 relative (fp64)
TOL_DRAW = 1e-9      # draws: same Philox stream; differences are libm ulps through erfcinv/log/cos


def _state_from_oracle(m, seed, n_sweeps=2):
    rng = Rng(seed)
    st = O.compute_initial_parameters(m, rng)
    for it in range(1, n_sweeps + 1):
        st = O.sweep(st, m, rng, it, updater={"GammaEta": False})
    return st, rng


def _chain(hM, seed, st=None):
    ch = H.Chain(hM, seed, device=0, updater={"GammaEta": False})
    ch.init()
    if st is not None:
        ch.set_state(st)
    return ch


MODELS = {
    "probit": dict(ny=300, ns=40, nc=4, nf=3),
    "probit_na": dict(ny=200, ns=30, nc=3, nf=2, na_frac=0.05, seed=3),
    "mixed_normal": dict(ny=150, ns=20, nc=3, nf=2, n_normal=5, seed=4),
    "two_levels_units": dict(ny=240, ns=25, nc=3, nf=2, nr=2, units=[240, 37], seed=5),
    "grouped_units": dict(ny=240, ns=20, nc=3, nf=3, nr=1, units=[40], seed=8),
    "traits": dict(ny=120, ns=35, nc=3, nf=2, nt=3, seed=6),
    # nc*nt = 36 > 32: GammaV / Gamma2 take the LDS workgroup path instead of the wave path
    "wide_traits": dict(ny=150, ns=40, nc=12, nf=2, nt=3, seed=9),
    # nc = 20 (wave bucket 24), K = 30: the bench's dimension class at small ny / ns
    "bench_dims": dict(ny=300, ns=50, nc=20, nf=10, seed=10),
    # vignette_2's mixed families: normal, Poisson and lognormal Poisson (Polya-Gamma Z), with NA
    "mixed_poisson": dict(ny=160, ns=24, nc=3, nf=2, n_normal=3, n_poisson=6, n_lognormal=4,
                          na_frac=0.03, seed=11),
    "poisson_only": dict(ny=200, ns=20, nc=3, nf=2, n_poisson=20, seed=12),
}


@pytest.fixture(scope="module", params=list(MODELS))
def setup(request):
    hM = synthetic_model(**MODELS[request.param])
    m = oracle_model(hM)
    seed = 987654321
    st, rng = _state_from_oracle(m, seed)
    return request.param, hM, m, seed, st, rng


def test_init_parity(setup):
    name, hM, m, seed, _, _ = setup
    ch = _chain(hM, seed)
    g = ch.get_state()
    o = O.compute_initial_parameters(m, Rng(seed))
    for k in ("Gamma", "iV", "Beta", "iSigma", "Z"):
        assert rel_err(g[k], o[k]) < TOL_DRAW, (name, k, rel_err(g[k], o[k]))
    for r in range(hM.nr):
        for k in ("Eta", "Lambda", "Psi", "Delta"):
            assert rel_err(g[k][r], o[k][r]) < TOL_DRAW, (name, k, r)
    ch.close()


@pytest.mark.parametrize("upd", ["BetaLambda", "GammaV", "Gamma2", "LambdaPriors", "Eta", "InvSigma", "Z"])
def test_updater_draw_parity(setup, upd):
    name, hM, m, seed, st, _ = setup
    it = 7
    ch = _chain(hM, seed, st)
    ch.update(upd, it)
    g = ch.get_state()
    rng = Rng(seed)
    if upd == "BetaLambda":
        B, Lam = O.update_beta_lambda(st, m, rng, it)
        assert rel_err(g["Beta"], B) < TOL_DRAW
        for r in range(hM.nr):
            assert rel_err(g["Lambda"][r], Lam[r]) < TOL_DRAW
    elif upd == "GammaV":
        Gm, iV = O.update_gamma_v(st, m, rng, it)
        assert rel_err(g["iV"], iV) < TOL_DRAW
        assert rel_err(g["Gamma"], Gm) < TOL_DRAW
    elif upd == "Gamma2":
        Gm = O.update_gamma2(st, m, rng, it)
        assert rel_err(g["Gamma"], Gm) < TOL_DRAW
    elif upd == "LambdaPriors":
        Psi, Delta = O.update_lambda_priors(st, m, rng, it)
        for r in range(hM.nr):
            assert rel_err(g["Psi"][r], Psi[r]) < TOL_DRAW
            assert rel_err(g["Delta"][r], Delta[r]) < TOL_DRAW
    elif upd == "Eta":
        Eta = O.update_eta(st, m, rng, it)
        for r in range(hM.nr):
            assert rel_err(g["Eta"][r], Eta[r]) < TOL_DRAW, (name, r, rel_err(g["Eta"][r], Eta[r]))
    elif upd == "InvSigma":
        iS = O.update_inv_sigma(st, m, rng, it)
        assert rel_err(g["iSigma"], iS) < TOL_DRAW
    elif upd == "Z":
        Z = O.update_z(st, m, rng, it)
        assert rel_err(g["Z"], Z) < TOL_DRAW
    ch.close()


def test_beta_lambda_moments(setup):
    """Conditional mean (noise mode 1) and precision of updateBetaLambda to 1e-10."""
    name, hM, m, seed, st, _ = setup
    ch = _chain(hM, seed, st)
    ch.set_noise_mode(1 | 2)
    ch.update("BetaLambda", 3)
    g = ch.get_state()
    precs, means = O.beta_lambda_moments(st, m)
    K = means.shape[0]
    assert rel_err(g["Beta"], means[:hM.nc]) < TOL_MOMENT
    dp = ch.debug_get("BL_prec", hM.ns * K * K).reshape(hM.ns, K, K).transpose(0, 2, 1)
    assert rel_err(dp, precs) < TOL_MOMENT
    ch.close()


def test_eta_moments(setup):
    name, hM, m, seed, st, _ = setup
    ch = _chain(hM, seed, st)
    ch.set_noise_mode(1)
    ch.update("Eta", 3)
    g = ch.get_state()
    Eta = O.update_eta(st, m, Rng(seed), 3, zero_noise=True)
    for r in range(hM.nr):
        assert rel_err(g["Eta"][r], Eta[r]) < TOL_MOMENT, (name, r)
    ch.close()


def test_gamma_moments(setup):
    name, hM, m, seed, st, _ = setup
    ch = _chain(hM, seed, st)
    ch.set_noise_mode(1)
    ch.update("Gamma2", 3)
    g = ch.get_state()
    if np.all(st["iSigma"] == 1):
        muG, _ = O.gamma2_moments(st, m)
        assert rel_err(g["Gamma"].reshape(-1, order="F"), muG) < TOL_MOMENT
    else:
        assert rel_err(g["Gamma"], st["Gamma"]) == 0.0   # Gamma2 acts only if all(iSigma == 1)
    ch.close()


def test_linear_predictor_and_contractions(setup):
    """The fused updateZ contractions equal their definitions on the stored Z."""
    name, hM, m, seed, st, _ = setup
    ch = _chain(hM, seed, st)
    ch.update("Z", 5)
    g = ch.get_state()
    Z = g["Z"]
    stz = dict(st, Z=Z)
    XEta, _ = O._xeta_and_prior(stz, m)
    K = XEta.shape[1]
    dims = ch.debug_get("dims", 8)
    Kmax = int(dims[2])
    Yx = ~np.isnan(m["Y"])
    XZ = ch.debug_get("XZ", K * hM.ns).reshape(hM.ns, K).T
    assert rel_err(XZ, XEta.T @ np.where(Yx, Z, 0.0)) < 1e-12
    G = ch.debug_get("G", Kmax * Kmax).reshape(Kmax, Kmax).T[:K, :K]
    assert rel_err(G, XEta.T @ XEta) < 1e-12
    if np.isnan(m["Y"]).any():  # Z Tr is formed only where it is consumed (NA models)
        ZTr = ch.debug_get("ZTr", hM.ny * hM.nt).reshape(hM.nt, hM.ny).T
        assert rel_err(ZTr, Z @ m["Tr"]) < 1e-12
    ch.close()


def test_full_sweeps_track_oracle(setup):
    """Three complete sweeps in the reference block order stay on the oracle's path."""
    name, hM, m, seed, st, _ = setup
    ch = _chain(hM, seed, st)
    rng = Rng(seed)
    o = st
    for it in range(10, 13):
        ch.sweep(it)
        o = O.sweep(o, m, rng, it, updater={"GammaEta": False})
    g = ch.get_state()
    for k in ("Beta", "Gamma", "iV", "Z"):
        assert rel_err(g[k], o[k]) < 1e-7, (name, k, rel_err(g[k], o[k]))
    ch.close()


def test_sample_mcmc_layout():
    """sampleMcmc end to end: 13 fields per sample, 72 hM fields, aligned chains."""
    hM = synthetic_model(ny=100, ns=12, nc=3, nf=2, seed=11)
    out = H.sampleMcmc(hM, samples=20, transient=10, nChains=2, updater={"GammaEta": False}, seed=3, verbose=0)
    assert len(out) == 72
    assert len(out.postList) == 2 and len(out.postList[0]) == 20
    assert len(out.postList[0][0]) == 13
    s = out.postList[1][5]
    assert s["Beta"].shape == (3, 12) and s["Lambda"][0].shape == (2, 12) and s["Eta"][0].shape == (100, 2)
    mp, cols = H.convertToCodaObject(out)
    assert mp["Beta"][0].shape == (20, 36) and cols["Beta"][0].startswith("B[(Intercept) (C1), sp01 (S1)]")


@pytest.mark.parametrize("thin", [1, 2])
def test_graph_replay_matches_eager(monkeypatch, thin):
    """hmsc_run replays captured graphs of several sweeps (the record pack inside, its ring
    slot chosen on the device); the recorded chain must equal the eager launch sequence bit
    for bit (same kernels, same order, same Philox counters), also when the run length is
    not a multiple of the sweeps per replay (remainders replay the graphs of the smaller
    powers of two: 46 = 32 + 8 + 4 + 2 at the default 32 sweeps per replay).  Inside a
    replay the side chain is joined on the device (flags, no cross-queue graph edges) unless
    HMSC_SIDE_EDGES=1; both equal the eager sequence."""
    hM = synthetic_model(ny=200, ns=30, nc=4, nf=3, nt=2, seed=12)
    # HMSC_SIDE_PARTIALS=1: GammaV's / psi's species partials from post_bl_kernel, forked on the
    # device inside a replay (its own summation order: compared among themselves)
    cases = (("1", "4", "0", "0"), ("0", "4", "0", "0"), ("0", "3", "0", "0"), ("0", "1", "0", "0"),
             ("0", "32", "0", "0"), ("0", "32", "1", "0"), ("1", "4", "0", "1"), ("0", "4", "0", "1"),
             ("0", "32", "0", "1"), ("0", "32", "1", "1"))
    out = {}
    for no_graph, per, edges, sidep in cases:
        monkeypatch.setenv("HMSC_NO_GRAPH", no_graph)
        monkeypatch.setenv("HMSC_GRAPH_SWEEPS", per)
        monkeypatch.setenv("HMSC_SIDE_EDGES", edges)
        monkeypatch.setenv("HMSC_SIDE_PARTIALS", sidep)
        ch = H.Chain(hM, 77, device=0, updater={"GammaEta": False})
        ch.init()
        rec = ch.run(transient=5, samples=41, thin=thin, adaptNf=[0])
        rec2 = ch.run(transient=2, samples=7, thin=thin, adaptNf=[0], iter0=5 + 41 * thin)
        out.setdefault(sidep, []).append((rec, rec2))
        ch.close()
    for runs in out.values():
        for o in runs[1:]:
            for i in range(2):
                for k in ("Beta", "Gamma", "iV", "iSigma", "Lambda0", "Eta0", "Delta0", "Psi0"):
                    np.testing.assert_array_equal(runs[0][i][k], o[i][k], err_msg=k)
    for i in range(2):  # the two partial paths differ by summation order only
        for k in ("Beta", "Gamma", "iV", "Lambda0", "Eta0", "Psi0"):
            np.testing.assert_allclose(out["1"][0][i][k], out["0"][0][i][k], rtol=1e-6, atol=1e-9, err_msg=k)


def test_init_par_fixed_effects_chain_start():
    """initPar = "fixed effects": the chain starts from the GLM Beta / Gamma / V (host,
    hmsc_amd/initpar.py) and its Z is then drawn by the initial updateZ from that state
    (R/computeInitialParameters.R:229-254, hmsc_init_z), equal to the oracle's draw."""
    from hmsc_amd.initpar import fixed_effects_init
    hM = synthetic_model(ny=150, ns=12, nc=3, nf=2, n_normal=2, n_poisson=2, seed=21)
    m = oracle_model(hM)
    seed = 2468
    fe = fixed_effects_init(hM)
    ch = H.Chain(hM, seed, device=0, updater={"GammaEta": False})
    ch.init()
    ch.set_state(fe)
    ch.init_z()
    g = ch.get_state()
    ch.close()
    assert rel_err(g["Beta"], fe["Beta"]) < 1e-14 and rel_err(g["Gamma"], fe["Gamma"]) < 1e-14
    assert rel_err(np.linalg.inv(g["iV"]), fe["V"]) < 1e-12
    st = {k: v for k, v in g.items() if k != "Z"}   # init: Poisson ZPrev = LFix + LRan (:250-254)
    Z = O.update_z(st, m, Rng(seed), 0, Y=m["Yraw"])
    assert rel_err(g["Z"], Z) < TOL_DRAW
    out = H.sampleMcmc(hM, samples=5, transient=3, initPar="fixed effects", updater={"GammaEta": False},
                       seed=5, verbose=0)
    assert len(out.postList[0]) == 5 and np.all(np.isfinite(out.postList[0][-1]["Beta"]))
