"""updateGammaEta restatement (R/updateGammaEta.R:7-206) against brute-force Gaussian
conditioning.  With mGamma = 0, Gamma ~ N(0, U), B_.j ~ N(Gamma Tr_j, V) (rows coupled by
Q) and Eta rows ~ N(0, I), the reference draws vec(Beta) from its conditional with Gamma
AND Eta integrated out: prior N(0, A), A = (Tr x I) U (Tr x I)' + Q x V (:32), and
vec(S) = (I x X) vec(Beta) + vec(P Eta Lambda) + eps with Cov(vec S) =
Lambda'Lambda x P P' + D^-1 x I.  At zero noise the function's Gamma is then
E[Gamma | Beta = that mean] and its Eta E[Eta | Beta, S]; both are checked here against
dense numpy conditioning at small sizes, for observation-level (np = ny) and grouped
(np < ny) units, with and without a phylogeny Q."""
import numpy as np
import pytest

from helpers import O, oracle_model, phylo_corr, synthetic_model
from oracle.rng import Rng


def _brute(st, m, r_level=0, dp=None):
    X, Tr, Z = m["X"], m["Tr"], st["Z"]
    ny, ns = Z.shape
    nc, nt = X.shape[1], Tr.shape[1]
    dp = dp or O.compute_data_parameters(m)
    g = st.get("rho", 1) - 1 if m.get("C") is not None else 0
    Q, iQ = dp["Qg"][g], dp["iQg"][g]
    V = np.linalg.inv(st["iV"])
    U = m["UGamma"]
    lam = st["Lambda"][r_level]
    nf = lam.shape[0]
    npr = int(m["np"][r_level])
    P = np.zeros((ny, npr))
    P[np.arange(ny), m["Pi"][:, r_level] - 1] = 1.0
    idv = st["iSigma"]
    KT = np.kron(Tr, np.eye(nc))
    A = KT @ U @ KT.T + np.kron(Q, V)
    Sig = np.kron(lam.T @ lam, P @ P.T) + np.kron(np.diag(1 / idv), np.eye(ny))
    H = np.kron(np.eye(ns), X)
    iSig = np.linalg.inv(Sig)
    prec = np.linalg.inv(A) + H.T @ iSig @ H
    mb = np.linalg.solve(prec, H.T @ iSig @ Z.ravel(order="F"))
    Beta = mb.reshape((nc, ns), order="F")
    iU = np.linalg.inv(U)
    Pg = iU + np.kron(Tr.T @ iQ @ Tr, st["iV"])
    Gamma = np.linalg.solve(Pg, ((st["iV"] @ Beta) @ (iQ @ Tr)).ravel(order="F")).reshape((nc, nt), order="F")
    # Eta | Beta, S: prior N(0, I) per unit row, S1 = P Eta Lambda + eps
    S1 = Z - X @ Beta
    D = np.diag(idv)
    Eta = np.empty((npr, nf))
    for q in range(npr):
        rows = P[:, q] == 1
        Wq = np.eye(nf) + rows.sum() * lam @ D @ lam.T
        Eta[q] = np.linalg.solve(Wq, lam @ D @ S1[rows].sum(axis=0))
    return Gamma, Eta


CASES = {
    "obs_units": dict(ny=14, ns=4, nc=2, nf=2, seed=31),
    "grouped": dict(ny=15, ns=3, nc=2, nf=2, units=[5], seed=32),
    "traits": dict(ny=12, ns=5, nc=2, nf=1, nt=2, seed=33),
}


@pytest.mark.parametrize("name", list(CASES))
@pytest.mark.parametrize("phylo", [False, True])
def test_gamma_eta_zero_noise_matches_conditioning(name, phylo):
    kw = dict(CASES[name])
    if phylo:
        kw["C"] = phylo_corr(kw["ns"], seed=4)
    hM = synthetic_model(**kw)
    m = oracle_model(hM)
    rng = Rng(77)
    st = O.compute_initial_parameters(m, rng)
    dp = O.compute_data_parameters(m)
    st = O.sweep(st, m, rng, 1, updater={"GammaEta": False}, data_par=dp)
    st["iSigma"] = np.linspace(0.7, 1.6, hM.ns)     # exercise a non-unit diagonal
    if phylo:
        st["rho"] = 37
    Gm, Eta = O.update_gamma_eta(st, m, rng, 2, data_par=dp, zero_noise=True)
    Gb, Eb = _brute(st, m, dp=dp)
    assert np.max(np.abs(Gm - Gb)) < 1e-9 * max(1.0, np.max(np.abs(Gb)))
    assert np.max(np.abs(Eta[0] - Eb)) < 1e-9 * max(1.0, np.max(np.abs(Eb)))


def test_gamma_eta_in_sweep_two_levels():
    """Default updater set (GammaEta on) over two levels: runs, finite, Eta shapes kept."""
    hM = synthetic_model(ny=30, ns=4, nc=2, nf=2, nr=2, units=[30, 6], seed=34)
    m = oracle_model(hM)
    rng = Rng(5)
    st = O.compute_initial_parameters(m, rng)
    for it in range(1, 6):
        st = O.sweep(st, m, rng, it)
    assert st["Eta"][0].shape == (30, 2) and st["Eta"][1].shape == (6, 2)
    assert np.all(np.isfinite(st["Gamma"])) and all(np.all(np.isfinite(e)) for e in st["Eta"])


def _brute_spatial(st, m, r, dp):
    """(vec Gamma, vec Eta_r) | S with Beta integrated out, by dense conditioning on
    vec(S) = (Tr x X) gamma + (Lambda' x P) eta + (I x X) e + eps, e ~ N(0, Q x V),
    eps ~ N(0, D^-1 x I), gamma ~ N(0, U), eta ~ N(0, bdiag(W_alpha_h)) -- the model
    R/updateGammaEta.R:139-198 draws from ('Full' spatial level, other levels' LRan
    subtracted from Z as at :37-42; levels before r enter with their new Eta, which the
    caller puts in st).  Returns (mean, precision)."""
    X, Tr, Z = m["X"], m["Tr"], st["Z"]
    ny, ns = Z.shape
    g = st.get("rho", 1) - 1 if m.get("C") is not None else 0
    Q = dp["Qg"][g]
    V = np.linalg.inv(st["iV"])
    lam = st["Lambda"][r]
    npr = int(m["np"][r])
    P = np.zeros((ny, npr))
    P[np.arange(ny), m["Pi"][:, r] - 1] = 1.0
    S = Z - sum(O.l_ran(st, m, q) for q in range(len(m["rL"])) if q != r)
    iWg = dp["rLPar"][r]["iWg"]
    alpha = np.asarray(st["Alpha"][r], dtype=np.int64) - 1
    K = np.zeros((npr * lam.shape[0],) * 2)
    for h, a in enumerate(alpha):
        K[h * npr:(h + 1) * npr, h * npr:(h + 1) * npr] = np.linalg.inv(iWg[a])
    J = np.hstack([np.kron(Tr, X), np.kron(lam.T, P)])
    HX = np.kron(np.eye(ns), X)
    Sig = HX @ np.kron(Q, V) @ HX.T + np.kron(np.diag(1 / st["iSigma"]), np.eye(ny))
    iSig = np.linalg.inv(Sig)
    nG = m["UGamma"].shape[0]
    prior = np.zeros((J.shape[1],) * 2)
    prior[:nG, :nG] = np.linalg.inv(m["UGamma"])
    prior[nG:, nG:] = np.linalg.inv(K)
    prec = prior + J.T @ iSig @ J
    return np.linalg.solve(prec, J.T @ iSig @ S.ravel(order="F")), prec


SPATIAL_CASES = {
    "one_level": dict(ny=16, ns=4, nc=2, nf=2, nr=1, spatial=[0], seed=61),
    "two_levels_traits": dict(ny=18, ns=4, nc=2, nf=2, nr=2, units=[18, 6], spatial=[1],
                              nt=2, alpha_n=20, seed=62),
}


@pytest.mark.parametrize("name", list(SPATIAL_CASES))
@pytest.mark.parametrize("phylo", [False, True])
def test_spatial_gamma_eta_matches_conditioning(name, phylo):
    """The spatial 'Full' branch (R/updateGammaEta.R:139-198, oracle.gamma_eta_spatial_literal,
    the device's natural form pinned equal to it in test_oracle_spatial.py) against dense
    conditioning: zero-noise Gamma and Eta_r are the posterior mean, and R's joint precision
    iG = iG1 + iG2 - iG3 is the posterior precision -- an independent derivation, not a
    second restatement of R's chain."""
    kw = dict(SPATIAL_CASES[name])
    if phylo:
        kw["C"] = phylo_corr(kw["ns"], seed=5)
    hM = synthetic_model(**kw)
    m = oracle_model(hM)
    rng = Rng(78)
    dp = O.compute_data_parameters(m)
    st = O.compute_initial_parameters(m, rng)
    st = O.sweep(st, m, rng, 1, updater={"GammaEta": False}, data_par=dp)
    st["iSigma"] = np.linspace(0.6, 1.5, hM.ns)
    r = [k for k, rl in enumerate(m["rL"]) if rl["sDim"]][0]
    st["Alpha"] = list(st["Alpha"])
    st["Alpha"][r] = np.arange(len(st["Alpha"][r])) * 5 + 3        # distinct spatial scales
    if phylo:
        st["rho"] = 41
    Gm, Eta = O.update_gamma_eta(st, m, rng, 2, data_par=dp, zero_noise=True)
    st = dict(st, Eta=[Eta[q] if q < r else st["Eta"][q] for q in range(len(Eta))])
    mb, pb = _brute_spatial(st, m, r, dp)
    mo = np.r_[Gm.ravel(order="F"), Eta[r].ravel(order="F")]
    assert np.max(np.abs(mo - mb)) < 1e-8 * max(1.0, np.max(np.abs(mb)))
    g = st.get("rho", 1) - 1 if m.get("C") is not None else 0
    iQ, Q = dp["iQg"][g], dp["Qg"][g]
    iV = st["iV"]
    V = np.linalg.inv(iV)
    U = m["UGamma"]
    KT = np.kron(m["Tr"], np.eye(m["X"].shape[1]))
    iA = np.linalg.inv(KT @ U @ KT.T + np.kron(Q, V))
    S = st["Z"] - sum(O.l_ran(st, m, q) for q in range(len(m["rL"])) if q != r)
    _, iG = O.gamma_eta_spatial_literal(st, m, r, S, dp, iQ, iV, U, np.linalg.inv(U), iA)
    assert np.max(np.abs(iG - pb)) < 1e-8 * np.max(np.abs(pb))
