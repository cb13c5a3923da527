"""``initPar = "fixed effects"`` of computeInitialParameters (R/computeInitialParameters.R:52-79).

Every species gets the single-species GLM estimate of its Beta on hM$XScaled -- lm.fit for
normal species, glm.fit(family = binomial(link = "probit")) for probit and
glm.fit(family = poisson()) for Poisson and lognormal Poisson species (:64-70) -- then
Gamma[k, ] = lm.fit(hM$Tr, Beta[k, ]) (:72-76; the reference regresses on the unscaled Tr)
and V = cov(t(Beta - Gamma Tr')) + I (:77, NA entries dropped from the sum).  The remaining
parameters are drawn from the priors as for initPar = NULL (:79 sets initPar to NULL).

glm.fit is restated as R's IRLS (stats::glm.fit): starting values mustart = (y + 0.5) / 2
(binomial, weights 1) and y + 0.1 (Poisson), eta = linkfun(mustart), then weighted least
squares steps until |dev - devold| / (|dev| + 0.1) < 1e-8 (glm.control: epsilon 1e-8,
maxit 25).  Host code: it runs once per chain start, like the reference.
"""
import numpy as np
from scipy.special import ndtr, ndtri

_EPS, _MAXIT = 1e-8, 25


def _wls(X, z, w):
    sw = np.sqrt(w)
    coef, *_ = np.linalg.lstsq(X * sw[:, None], z * sw, rcond=None)
    return coef


def _probit_dev(y, mu):
    mu = np.clip(mu, 1e-300, 1 - 1e-16)
    return 2.0 * np.sum(np.where(y > 0, -y * np.log(mu), 0.0) + np.where(y < 1, -(1 - y) * np.log1p(-mu), 0.0))


def _poisson_dev(y, mu):
    r = np.where(y > 0, y * np.log(np.where(y > 0, y, 1.0) / mu), 0.0)
    return 2.0 * np.sum(r - (y - mu))


def glm_fit_probit(X, y):
    """stats::glm.fit(X, y, family = binomial(link = "probit")) coefficients."""
    mu = (y + 0.5) / 2.0
    eta = ndtri(mu)
    dev_old = _probit_dev(y, mu)
    coef = None
    for _ in range(_MAXIT):
        dmu = np.exp(-0.5 * eta * eta) / np.sqrt(2.0 * np.pi)         # mu.eta = dnorm(eta)
        dmu = np.maximum(dmu, np.finfo(float).eps)                     # binomial()$mu.eta clamp
        var = mu * (1.0 - mu)
        z = eta + (y - mu) / dmu
        w = dmu * dmu / var
        coef = _wls(X, z, w)
        eta = X @ coef
        mu = np.clip(ndtr(eta), np.finfo(float).eps, 1 - np.finfo(float).eps)
        dev = _probit_dev(y, mu)
        if abs(dev - dev_old) / (abs(dev) + 0.1) < _EPS:
            break
        dev_old = dev
    return coef


def glm_fit_poisson(X, y):
    """stats::glm.fit(X, y, family = poisson()) coefficients."""
    mu = y + 0.1
    eta = np.log(mu)
    dev_old = _poisson_dev(y, mu)
    coef = None
    for _ in range(_MAXIT):
        z = eta + (y - mu) / mu
        w = mu
        coef = _wls(X, z, w)
        eta = X @ coef
        mu = np.exp(eta)
        dev = _poisson_dev(y, mu)
        if abs(dev - dev_old) / (abs(dev) + 0.1) < _EPS:
            break
        dev_old = dev
    return coef


def lm_fit(X, y):
    coef, *_ = np.linalg.lstsq(X, y, rcond=None)
    return coef


def fixed_effects_init(hM):
    """(Beta, Gamma, V) of R/computeInitialParameters.R:52-77 in the sampler's parameterisation
    (XScaled columns)."""
    X = np.asarray(hM.XScaled, dtype=np.float64)
    Y = np.asarray(hM.Y, dtype=np.float64)
    nc, ns = X.shape[1], Y.shape[1]
    Beta = np.full((nc, ns), np.nan)
    for j in range(ns):
        obs = ~np.isnan(Y[:, j])                                       # glm.fit's default na handling via lm / glm
        Xj, yj = X[obs], Y[obs, j]
        fam = int(hM.distr[j, 0])
        if fam == 1:
            Beta[:, j] = lm_fit(Xj, yj)
        elif fam == 2:
            Beta[:, j] = glm_fit_probit(Xj, yj)
        elif fam == 3:
            Beta[:, j] = glm_fit_poisson(Xj, yj)
        else:
            raise ValueError(f"unknown distr family {fam}")
    Tr = np.asarray(hM.Tr, dtype=np.float64)                           # :74 hM$Tr (unscaled)
    Gamma = np.stack([lm_fit(Tr, Beta[k]) for k in range(nc)])         # (nc, nt)
    E = Beta - Gamma @ Tr.T
    C = np.cov(E) if ns > 1 else np.full((nc, nc), np.nan)
    V = np.nan_to_num(np.atleast_2d(C), nan=0.0) + np.eye(nc)          # rowSums(abind(.., diag), na.rm=TRUE)
    return dict(Beta=Beta, Gamma=Gamma, V=V)
