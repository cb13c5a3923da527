"""Shared test helpers: synthetic Hmsc models and the hM -> oracle-model mapping."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import hmsc_amd as H  # noqa: E402
from oracle import hmsc_oracle as O  # noqa: E402


def synthetic_model(ny=200, ns=30, nc=4, nf=3, seed=1, na_frac=0.0, n_normal=0, units=None, nr=1,
                    nf_fit=None, nt=1, yscale=False, C=None, n_poisson=0, n_lognormal=0, spatial=None,
                    alpha_n=None, spatial_method="Full", n_neighbours=None, n_knots=None, nf_default=False,
                    x_dim=0):
    """Probit JSDM generated like BASELINE.md's synthetic config; optionally the first
    n_normal species normal, the next n_poisson Poisson and n_lognormal lognormal Poisson
    (counts ~ Poisson(exp(L / 2)), vignette_2's mixed-distribution model).  x_dim > 0: level 0
    is covariate-dependent (HmscRandomLevel(xData=...) with an intercept column and x_dim - 1
    normal covariates per unit, R's LRan = sum_k (Eta[Pi,] * x[, k]) Lambda[,,k])."""
    rng = np.random.default_rng(seed)
    X = np.column_stack([np.ones(ny), rng.standard_normal((ny, nc - 1))])
    Tr = np.column_stack([np.ones(ns)] + [rng.standard_normal(ns) for _ in range(nt - 1)]) if nt > 1 else None
    G = rng.normal(0, 0.5, (nc, 1))
    B = G + rng.normal(0, 0.3, (nc, ns))
    L = X @ B
    sd = {}
    levels = {}
    ranLevels = {}
    for r in range(nr):
        npr = ny if units is None else units[r]
        pi = np.arange(ny) % npr if npr < ny else np.arange(ny)
        rng.shuffle(pi) if npr < ny else None
        eta = rng.standard_normal((npr, nf))
        lam = rng.standard_normal((nf, ns)) / (np.arange(1, nf + 1)[:, None])
        xr = None
        if x_dim and r == 0:
            xr = np.column_stack([np.ones(npr)] + [rng.standard_normal(npr) for _ in range(x_dim - 1)])
            for k in range(x_dim):
                L = L + (eta[pi] * xr[pi, k:k + 1]) @ (lam / (k + 1))
        else:
            L = L + eta[pi] @ lam
        name = f"lev{r}"
        if spatial is not None and r in spatial:
            # spatial 'Full' level: unit coordinates on the unit square, zero-padded unit
            # names so levels(dfPi) order is the coordinate row order
            sd[name] = np.array([f"s{k:05d}" for k in pi])
            xy = rng.random((npr, 2))
            sKnot = None
            if spatial_method == "GPP":
                from hmsc_amd.dataparams import constructKnots
                sKnot = constructKnots(xy, nKnots=n_knots or 4)
            rl = H.HmscRandomLevel(sData=xy, sMethod=spatial_method, nNeighbours=n_neighbours, sKnot=sKnot)
            if alpha_n is not None:
                diag = np.sqrt(2.0)
                H.setPriors(rl, alphapw=np.column_stack([diag * np.arange(alpha_n + 1) / alpha_n,
                                                          np.r_[0.5, np.full(alpha_n, 0.5 / alpha_n)]]))
        elif xr is not None:
            import pandas as pd
            sd[name] = np.array([f"u{k:05d}" for k in pi])
            xdf = pd.DataFrame(xr, columns=[f"x{k}" for k in range(x_dim)], index=[f"u{k:05d}" for k in range(npr)])
            rl = H.HmscRandomLevel(xData=xdf)
        else:
            sd[name] = np.array([f"u{k}" for k in pi])
            rl = H.HmscRandomLevel(units=sd[name])
        nff = nf if nf_fit is None else nf_fit
        if not nf_default:  # (nf_default: the reference's priors, nfMin 2 and nfMax Inf = ns)
            H.setPriors(rl, nfMin=nff, nfMax=nff)
        ranLevels[name] = rl
        levels[name] = pi
    Ylat = L + rng.standard_normal((ny, ns))
    Y = (Ylat > 0).astype(float)
    distr = ["probit"] * ns
    for j in range(n_normal):
        Y[:, j] = Ylat[:, j] * 2.0 + 1.0
        distr[j] = "normal"
    for k in range(n_poisson + n_lognormal):
        j = n_normal + k
        Y[:, j] = rng.poisson(np.exp(np.clip(0.5 * Ylat[:, j], -20, 3))).astype(float)
        distr[j] = "poisson" if k < n_poisson else "lognormal poisson"
    if na_frac > 0:
        mask = rng.random((ny, ns)) < na_frac
        Y[mask] = np.nan
    import pandas as pd
    studyDesign = pd.DataFrame(sd) if nr > 0 else None
    covn = ["(Intercept)"] + [f"x{k}" for k in range(1, nc)]
    hM = H.Hmsc(Y=Y, X=X, covNames=covn, XScale=True, YScale=yscale, Tr=Tr, distr=distr, C=C,
                studyDesign=studyDesign, ranLevels=ranLevels if nr > 0 else None)
    return hM


def phylo_corr(ns, seed=0, scale=0.6):
    """Positive-definite phylogenetic correlation matrix: exp(-distance / scale) between random
    points on a line (an exponential / Ornstein-Uhlenbeck kernel), unit diagonal like vcv(tree, corr=TRUE)."""
    rng = np.random.default_rng(seed)
    x = np.sort(rng.random(ns))
    return np.exp(-np.abs(x[:, None] - x[None, :]) / scale)


def oracle_model(hM):
    m = dict(X=hM.XScaled, Y=hM.YScaled, Yraw=hM.Y, Tr=hM.TrScaled, Pi=hM.Pi, np=hM.np, distr=hM.distr,
             V0=hM.V0, f0=hM.f0, mGamma=hM.mGamma, UGamma=hM.UGamma, aSigma=hM.aSigma, bSigma=hM.bSigma,
             rhopw=hM.rhopw, C=hM.C,
             rL=[dict(nu=rl.nu, a1=rl.a1, b1=rl.b1, a2=rl.a2, b2=rl.b2, nfMin=rl.nfMin, nfMax=rl.nfMax,
                      sDim=rl.sDim, xDim=rl.xDim) for rl in (hM.rL or [])])
    for r, (d, rl) in enumerate(zip(m["rL"], hM.rL or [])):
        if rl.xDim:   # covariate-dependent level: rL$x in the unit order of Eta
            from hmsc_amd.sampler import x_unit_order
            d["x"] = x_unit_order(hM, r, rl)
        if rl.sDim:   # spatial 'Full': the distance matrix of the unit coordinates, alphapw grid
            # rows of rl$s in levels(dfPi[,r]) order, the unit order of Eta (R indexes s by
            # the unit names, R/computeDataParameters.R:56,92,142)
            from hmsc_amd.dataparams import _level_order
            xy = np.asarray(rl.s, dtype=np.float64)[_level_order(hM, r, rl)]
            d.update(spatialMethod=rl.spatialMethod, alphapw=np.asarray(rl.alphapw, dtype=np.float64),
                     dist=np.sqrt(((xy[:, None, :] - xy[None, :, :]) ** 2).sum(-1)),
                     s=xy, nNeighbours=rl.nNeighbours,
                     sKnot=rl["sKnot"] if "sKnot" in rl.names() else None)
    return m


def rel_err(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.max(np.abs(a - b)) / max(1e-300, np.max(np.abs(b))))


def rel_err_elem(a, b, floor=1e-3):
    """Elementwise relative error max_i |a_i - b_i| / max(|b_i|, floor * max|b|): unlike the
    normwise rel_err, a small entry cannot hide a large relative error (entries below
    floor * max|b| are measured against that floor)."""
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    scale = np.maximum(np.abs(b), floor * max(1e-300, float(np.max(np.abs(b)))))
    return float(np.max(np.abs(a - b) / scale))
