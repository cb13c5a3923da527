"""The oracle's covariate-dependent levels (HmscRandomLevel(xData=...), rL$xDim > 0) against
independent restatements (CPU only).  R runs these levels through the xDim branches of
R/updateZ.R:24-29, R/updateBetaLambda.R:22-53,150-154, R/updateLambdaPriors.R:34-48,
R/updateEta.R:93-108, R/computeInitialParameters.R:172-198 and R/updateNf.R:41-66; the
reference's tests hold no fixture for them (tests/testthat/test-setRL.R only checks xDim), so
the oracle is pinned here by brute-force Gaussian conditioning of the same model and by R's
array layouts -- "parity unpinned" against R's own draws."""
import numpy as np

from helpers import O, oracle_model, synthetic_model
from oracle.rng import Rng


def _model(na_frac=0.0, units=(30,)):
    hM = synthetic_model(ny=90, ns=9, nc=3, nf=2, seed=21, x_dim=2, units=list(units), na_frac=na_frac)
    m = oracle_model(hM)
    st = O.compute_initial_parameters(m, Rng(8))
    st["Z"] = np.random.default_rng(3).standard_normal(st["Z"].shape) + O.linear_predictor(st, m)
    return hM, m, st


def test_layouts_follow_r():
    hM, m, st = _model()
    nf, ns = 2, hM.ns
    assert st["Lambda"][0].shape == (nf, ns, 2) and st["Psi"][0].shape == (nf, ns, 2)
    assert st["Delta"][0].shape == (nf, 2) and st["Eta"][0].shape == (30, nf)
    # LRan = sum_k (Eta[Pi,] * x[dfPi, k]) %*% Lambda[,,k]   (R/updateZ.R:24-29)
    x = m["rL"][0]["x"]
    pi = m["Pi"][:, 0] - 1
    lran = sum((st["Eta"][0][pi] * x[pi, k:k + 1]) @ st["Lambda"][0][:, :, k] for k in range(2))
    np.testing.assert_allclose(O.l_ran(st, m, 0), lran, rtol=1e-13, atol=1e-13)
    # priorLambda rows f + nf k = Psi[f, j, k] * cumprod(Delta[, k])[f]   (R/updateBetaLambda.R:42-53)
    _, prior = O._xeta_and_prior(st, m)
    tau = np.cumprod(st["Delta"][0], axis=0)
    for k in range(2):
        np.testing.assert_allclose(prior[k * nf:(k + 1) * nf], st["Psi"][0][:, :, k] * tau[:, k:k + 1], rtol=1e-14)


def _brute_eta(st, m, r):
    """Conditional of vec(Eta_r) given everything else: Z = LFix + sum_k (Eta[Pi] * x_k) Lambda_k
    + (other levels) + e, e ~ N(0, 1/iSigma) over the observed cells, Eta ~ N(0, I)."""
    Y, Z = m["Y"], st["Z"]
    ny, ns = Z.shape
    iS = st["iSigma"]
    pi = m["Pi"][:, r] - 1
    npr, nf = st["Eta"][r].shape
    x = m["rL"][r]["x"]
    S = Z - m["X"] @ st["Beta"]
    for r2 in range(m["Pi"].shape[1]):
        if r2 != r:
            S = S - O.l_ran(st, m, r2)
    lam = st["Lambda"][r]
    obs = ~np.isnan(Y)
    P = np.eye(npr * nf)
    b = np.zeros(npr * nf)
    for i in range(ny):
        q = pi[i]
        lL = np.tensordot(lam, x[q], axes=([2], [0]))              # nf x ns
        for j in range(ns):
            if not obs[i, j]:
                continue
            ix = q + npr * np.arange(nf)                           # vec(Eta) column-major
            P[np.ix_(ix, ix)] += iS[j] * np.outer(lL[:, j], lL[:, j])
            b[ix] += iS[j] * S[i, j] * lL[:, j]
    return P, np.linalg.solve(P, b)


def test_eta_conditional_equals_brute_force():
    for na in (0.0, 0.15):
        hM, m, st = _model(na_frac=na)
        S = st["Z"] - m["X"] @ st["Beta"]
        precs, means = O.eta_unit_moments_x(st, m, 0, S)
        P, mean = _brute_eta(st, m, 0)
        npr, nf = means.shape
        np.testing.assert_allclose(means.ravel(order="F"), mean, rtol=1e-10, atol=1e-12)
        for q in range(npr):
            ix = q + npr * np.arange(nf)
            np.testing.assert_allclose(precs[q], P[np.ix_(ix, ix)], rtol=1e-12, atol=1e-12)
        # the draw is mean + chol(Q)^-1 xi: zero noise gives the mean
        eta0 = O.update_eta(st, m, Rng(1), 4, zero_noise=True)[0]
        np.testing.assert_allclose(eta0, means, rtol=1e-12, atol=1e-13)


def test_beta_lambda_regression_on_scaled_columns():
    """BetaLambda of species j is a Bayesian regression on [X, Eta[Pi,] x_1, Eta[Pi,] x_2]; the
    drawn Lambda comes back as R's nf x ns x ncr array (aperm(array(rows, c(nf, ncr, ns)), c(1,3,2)))."""
    hM, m, st = _model()
    precs, means = O.beta_lambda_moments(st, m)
    XEta, prior = O._xeta_and_prior(st, m)
    j = 4
    P = np.diag(np.r_[np.zeros(hM.nc), prior[:, j]])
    P[:hM.nc, :hM.nc] = st["iV"]
    np.testing.assert_allclose(precs[j], P + XEta.T @ XEta * st["iSigma"][j], rtol=1e-12)
    B, Lam = O.update_beta_lambda(st, m, Rng(2), 3, zero_noise=True)
    assert Lam[0].shape == (2, hM.ns, 2)
    np.testing.assert_allclose(Lam[0][:, :, 1], means[hM.nc + 2:hM.nc + 4], rtol=1e-12)


def test_lambda_priors_are_per_column_chains():
    """Column k of Psi / Delta is the matrix branch on Lambda[,,k] (device level v0 + k)."""
    hM, m, st = _model()
    psi, delta = O.update_lambda_priors(st, m, Rng(6), 7)
    assert psi[0].shape == (2, hM.ns, 2) and delta[0].shape == (2, 2)
    assert np.all(psi[0] > 0) and np.all(delta[0] > 0)
    # column 1 equals the matrix branch of a one-column level on device stream level 1
    m1 = dict(m, rL=[dict(m["rL"][0], xDim=0, nu=3.0, a1=50.0, b1=1.0, a2=50.0, b2=1.0)])
    st1 = dict(st, Lambda=[st["Lambda"][0][:, :, 1]], Delta=[st["Delta"][0][:, 1]])
    import oracle.rng as R
    old = R.LEVEL_STRIDE
    p1, d1 = O.update_lambda_priors(st1, dict(m1, rL=[dict(m1["rL"][0])]), _ShiftedRng(Rng(6), old), 7)
    np.testing.assert_allclose(p1[0], psi[0][:, :, 1], rtol=1e-13)
    np.testing.assert_allclose(d1[0], delta[0][:, 1], rtol=1e-13)


class _ShiftedRng:
    """Rng whose level streams are moved up by one level (stream + LEVEL_STRIDE)."""

    def __init__(self, rng, stride):
        self.r, self.s = rng, stride

    def gamma(self, idx, stream, it, a, b):
        return self.r.gamma(idx, stream + self.s, it, a, b)


def test_update_nf_adapts_every_column_together():
    hM, m, st = _model()
    nf = st["Lambda"][0].shape[0]
    m["rL"][0]["nfMax"] = 5
    grown = None
    for it in range(21, 400):
        e, lam, a, p, d = O.update_nf(st, m, 0, Rng(11), it)
        if lam.shape[0] != nf:
            grown = (e, lam, a, p, d)
            break
    assert grown is not None
    e, lam, a, p, d = grown
    assert lam.shape == (nf + 1, hM.ns, 2) and p.shape == (nf + 1, hM.ns, 2) and d.shape == (nf + 1, 2)
    assert e.shape[1] == nf + 1 and np.all(lam[nf] == 0) and np.all(p[nf] > 0) and np.all(d[nf] > 0)
    # a factor whose loadings are ~0 in every column is redundant: factor 1 goes (R's quirk, :56)
    st2 = dict(st, Lambda=[np.concatenate([st["Lambda"][0], np.zeros((1, hM.ns, 2))])],
               Psi=[np.concatenate([st["Psi"][0], np.ones((1, hM.ns, 2))])],
               Delta=[np.concatenate([st["Delta"][0], np.ones((1, 2))])],
               Eta=[np.hstack([st["Eta"][0], np.zeros((30, 1))])], Alpha=[np.ones(nf + 1, dtype=np.int64)])
    for it in range(1, 400):
        e, lam, a, p, d = O.update_nf(st2, m, 0, Rng(11), it)
        if lam.shape[0] != nf + 1:
            assert lam.shape[0] == nf and np.allclose(lam, st2["Lambda"][0][1:])
            np.testing.assert_allclose(e, st2["Eta"][0][:, 1:])
            break
    else:
        raise AssertionError("no adaptation in 400 sweeps")
