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
