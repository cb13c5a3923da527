"""Synthetic workloads named by BASELINE.json / BASELINE.md §2.

``synthetic_probit`` builds the headline configuration (config 4): seed 20261015,
ny=10 000 sites, ns=1 000 species, nc=20 (intercept named "(Intercept)" + 19 N(0,1)
covariates), nt=1, one unstructured sample-level random level with
nfMin=nfMax=10, probit.  True Gamma ~ N(0, 0.5^2); B_.j ~ N(Gamma, 0.3^2 I);
Eta ~ N(0,1); Lambda_hj ~ N(0, 1/h^2); Y = 1[XB + Eta Lambda + N(0,1) > 0]; no NA.
"""
import numpy as np

from .model import Hmsc, HmscRandomLevel, setPriors

SYNTHETIC_SEED = 20261015


def synthetic_probit(ny=10000, ns=1000, nc=20, nf=10, seed=SYNTHETIC_SEED, return_truth=False):
    rng = np.random.default_rng(seed)
    X = np.column_stack([np.ones(ny), rng.standard_normal((ny, nc - 1))])
    Gamma = rng.normal(0.0, 0.5, (nc, 1))
    B = Gamma + rng.normal(0.0, 0.3, (nc, ns))
    Eta = rng.standard_normal((ny, nf))
    Lam = rng.standard_normal((nf, ns)) / np.arange(1, nf + 1)[:, None]
    L = X @ B + Eta @ Lam + rng.standard_normal((ny, ns))
    Y = (L > 0).astype(np.float64)
    units = np.arange(1, ny + 1)
    rl = HmscRandomLevel(units=units)
    setPriors(rl, nfMin=nf, nfMax=nf)
    covNames = ["(Intercept)"] + [f"x{k}" for k in range(1, nc)]
    study = {"sample": units}
    try:
        import pandas as pd
        study = pd.DataFrame(study)
    except Exception:  # pragma: no cover
        pass
    hM = Hmsc(Y=Y, X=X, covNames=covNames, XScale=True, distr="probit", studyDesign=study,
              ranLevels={"sample": rl})
    if return_truth:
        return hM, dict(Gamma=Gamma, Beta=B, Eta=Eta, Lambda=Lam)
    return hM


def spatial_vignette4(ny=5000, method="Full", seed=SYNTHETIC_SEED, nNeighbours=10, knotDist=0.2,
                      minKnotDist=0.4):
    """BASELINE.json config 5: vignettes/vignette_4_spatial.Rmd:54-118 scaled to ny sampling
    units -- ns=5 probit species, intercept + one N(0,1) covariate (beta1 = -2..2), uniform
    coordinates in the unit square, a spatial latent factor with exponential covariance
    (sigma 2, alpha 0.35) and loadings (1, 2, -2, -1, 0), one sample-level spatial random
    level with nfMin = nfMax = 1 ('Full', 'NNGP' with nNeighbours, or 'GPP' on the
    constructKnots(knotDist, minKnotDist) grid)."""
    from .dataparams import constructKnots
    rng = np.random.default_rng(seed)
    ns = 5
    beta = np.column_stack([np.zeros(ns), [-2.0, -1.0, 0.0, 1.0, 2.0]])
    x = np.column_stack([np.ones(ny), rng.standard_normal(ny)])
    Lf = x @ beta.T
    xy = rng.random((ny, 2))
    d = np.sqrt(((xy[:, None, :] - xy[None, :, :]) ** 2).sum(-1))
    Sigma = 4.0 * np.exp(-d / 0.35)
    del d
    eta1 = np.linalg.cholesky(Sigma + 1e-10 * np.eye(ny)) @ rng.standard_normal(ny)
    del Sigma
    lam = np.array([1.0, 2.0, -2.0, -1.0, 0.0])
    L = Lf + np.outer(eta1, lam)
    Y = ((L + rng.standard_normal((ny, ns))) > 0).astype(np.float64)
    units = np.arange(1, ny + 1)
    kw = {}
    if method == "NNGP":
        kw["nNeighbours"] = nNeighbours
    elif method == "GPP":
        kw["sKnot"] = constructKnots(xy, knotDist=knotDist, minKnotDist=minKnotDist)
    try:
        import pandas as pd
        sData = pd.DataFrame(xy, index=[str(u) for u in units], columns=["x-coordinate", "y-coordinate"])
        study = pd.DataFrame({"sample": units.astype(str)})
    except Exception:  # pragma: no cover
        sData, study = xy, {"sample": units}
    rl = HmscRandomLevel(sData=sData, sMethod=method, **kw)
    setPriors(rl, nfMin=1, nfMax=1)
    return Hmsc(Y=Y, X=x, covNames=["(Intercept)", "x1"], XScale=True, distr="probit", studyDesign=study,
                ranLevels={"sample": rl})
