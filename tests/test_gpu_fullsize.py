"""Config 4 at its full size (BASELINE.json: ny=10 000, ns=1 000, nc=20, nf=10, probit), the
exact shape the bench times: one-update parity of updateZ, updateBetaLambda and updateEta
against the CPU oracle on the same state and Philox key, conditional moments of
BetaLambda / Eta (noise mode) to 1e-10 normwise and elementwise, then two full sweeps.
This exercises the production geometry of the z kernel (32 species blocks x site chunks,
slab-sum partials), the batched BetaLambda solve over 1 000 species and the fused Eta pass,
which the small parity models do not reach."""
import numpy as np
import pytest

from helpers import O, oracle_model, rel_err, rel_err_elem
from hmsc_amd.sampler import Chain
from hmsc_amd.workloads import synthetic_probit
from oracle.rng import Rng

pytestmark = pytest.mark.gpu
UP = {"GammaEta": False}


@pytest.fixture(scope="module")
def cfg4():
    hM = synthetic_probit()
    m = oracle_model(hM)
    seed = 20261016
    rng = Rng(seed)
    st = O.compute_initial_parameters(m, rng)
    st = O.sweep(st, m, rng, 1, updater=UP)       # a state one sweep into the chain
    return hM, m, seed, st


def _chain(hM, seed, st):
    ch = Chain(hM, seed, device=0, updater=UP)
    ch.init()
    ch.set_state(st)
    return ch


@pytest.mark.parametrize("upd", ["Z", "BetaLambda", "Eta", "GammaV", "Gamma2", "LambdaPriors"])
def test_full_size_update_parity(cfg4, upd):
    hM, m, seed, st = cfg4
    ch = _chain(hM, seed, st)
    it = 9
    ch.update(upd, it)
    g = ch.get_state()
    rng = Rng(seed)
    if upd == "Z":
        ref = {"Z": O.update_z(st, m, rng, it)}
    elif upd == "BetaLambda":
        B, Lam = O.update_beta_lambda(st, m, rng, it)
        ref = {"Beta": B, "Lambda": Lam[0]}
        g["Lambda"] = g["Lambda"][0]
    elif upd == "Eta":
        ref = {"Eta": O.update_eta(st, m, rng, it)[0]}
        g["Eta"] = g["Eta"][0]
    elif upd == "GammaV":
        Gm, iV = O.update_gamma_v(st, m, rng, it)
        ref = {"Gamma": Gm, "iV": iV}
    elif upd == "Gamma2":
        ref = {"Gamma": O.update_gamma2(st, m, rng, it)}
        # R/updateGamma2.R:44-52 forms SigmaG = V0 - V0 X'X V0 + V0 X'X iP X'X V0 + ..., which
        # cancels: the oracle's own answer moves by this much when iV moves by 1e-15
        pert = dict(st, iV=st["iV"] * (1.0 + 1e-15))
        sens = rel_err(O.update_gamma2(pert, m, Rng(seed), it), ref["Gamma"])
        tol = max(1e-9, 1e3 * sens)
    else:
        Psi, Delta = O.update_lambda_priors(st, m, rng, it)
        ref = {"Psi": Psi[0], "Delta": Delta[0]}
        g["Psi"], g["Delta"] = g["Psi"][0], g["Delta"][0]
    ch.close()
    tol = locals().get("tol", 1e-9)
    for k, v in ref.items():
        assert rel_err(g[k], v) < tol, (k, rel_err(g[k], v), tol)


def test_full_size_moments(cfg4):
    """Noise mode: BetaLambda's conditional means and Eta's conditional means, 1e-10."""
    hM, m, seed, st = cfg4
    ch = _chain(hM, seed, st)
    ch.set_noise_mode(1)
    ch.update("BetaLambda", 3)
    g = ch.get_state()
    _, means = O.beta_lambda_moments(st, m)
    assert rel_err(g["Beta"], means[:hM.nc]) < 1e-10
    assert rel_err_elem(g["Beta"], means[:hM.nc]) < 1e-8
    assert rel_err(g["Lambda"][0], means[hM.nc:]) < 1e-10
    ch.set_state(st)
    ch.update("Eta", 3)
    e = ch.get_state()["Eta"][0]
    ref = O.update_eta(st, m, Rng(seed), 3, zero_noise=True)[0]
    assert rel_err(e, ref) < 1e-10
    assert rel_err_elem(e, ref) < 1e-8
    ch.close()


def test_full_size_two_sweeps(cfg4):
    """Two whole sweeps from the same state: every update above agrees to ~1e-12, and what
    remains is fp64 rounding (factorization order, the reversed-Cholesky route to chol(Vn))
    carried through 2 x 10M truncated-normal draws into the next sweep's sufficient
    statistics; 1e-6 bounds that drift while any real disagreement shows up as O(1)."""
    hM, m, seed, st = cfg4
    ch = _chain(hM, seed, st)
    rng = Rng(seed)
    o = st
    for it in (2, 3):
        ch.sweep(it)
        o = O.sweep(o, m, rng, it, updater=UP)
    g = ch.get_state()
    ch.close()
    for k in ("Beta", "Gamma", "iV", "Z"):
        assert rel_err(g[k], o[k]) < 1e-6, (k, rel_err(g[k], o[k]))
    assert rel_err(g["Lambda"][0], o["Lambda"][0]) < 1e-6
    assert rel_err(g["Eta"][0], o["Eta"][0]) < 1e-6
