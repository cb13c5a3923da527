"""initPar = "fixed effects" (R/computeInitialParameters.R:52-79), CPU only.

Known answer from the reference's own tests: computeInitialParameters(TD$m, initPar =
'fixed effects') has round(Gamma) = t(matrix(c(-4,2,4,1,0,0,0,-2,-1), 3, 3))
(tests/testthat/test-initialParameters.R:128-132).  The GLM restatement of stats::glm.fit
(IRLS) is checked against an independent maximum-likelihood fit (scipy BFGS on the exact
log-likelihood), and Gamma / V against their definitions (:72-77)."""
import numpy as np
from scipy.optimize import minimize
from scipy.special import log_ndtr

from hmsc_amd.initpar import fixed_effects_init, glm_fit_poisson, glm_fit_probit
from test_golden_td import td_model


def test_td_fixed_effects_gamma_known_answer():
    fe = fixed_effects_init(td_model())
    expect = np.array([[-4, 2, 4], [1, 0, 0], [0, -2, -1]], dtype=float)   # test-initialParameters.R:131
    np.testing.assert_array_equal(np.round(fe["Gamma"]) + 0.0, expect)


def _mle(nll, p):
    return minimize(nll, np.zeros(p), method="BFGS", options=dict(gtol=1e-10, maxiter=10000)).x


def test_glm_matches_independent_mle():
    rng = np.random.default_rng(7)
    n = 400
    X = np.column_stack([np.ones(n), rng.standard_normal((n, 2))])
    b = np.array([0.3, -0.8, 0.5])
    yb = (X @ b + rng.standard_normal(n) > 0).astype(float)
    yp = rng.poisson(np.exp(0.2 + 0.4 * X[:, 1])).astype(float)
    cb = glm_fit_probit(X, yb)
    cp = glm_fit_poisson(X, yp)
    nll_b = lambda c: -np.sum(yb * log_ndtr(X @ c) + (1 - yb) * log_ndtr(-(X @ c)))  # noqa: E731
    nll_p = lambda c: -np.sum(yp * (X @ c) - np.exp(X @ c))                            # noqa: E731
    np.testing.assert_allclose(cb, _mle(nll_b, 3), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(cp, _mle(nll_p, 3), rtol=1e-5, atol=1e-6)


def test_gamma_and_v_definitions():
    hM = td_model()
    fe = fixed_effects_init(hM)
    Tr = np.asarray(hM.Tr)
    for k in range(hM.nc):                                   # Gamma[k,] = lm.fit(hM$Tr, Beta[k,])
        coef, *_ = np.linalg.lstsq(Tr, fe["Beta"][k], rcond=None)
        np.testing.assert_allclose(fe["Gamma"][k], coef, rtol=1e-12, atol=1e-12)
    E = fe["Beta"] - fe["Gamma"] @ Tr.T
    np.testing.assert_allclose(fe["V"], np.cov(E) + np.eye(hM.nc), rtol=1e-12)
