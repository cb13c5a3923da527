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


def coalescent_corr(ns, rng):
    """vcv(ape::rcoal(ns), corr=TRUE): correlation matrix of a random Kingman coalescent tree
    (ultrametric; C_ij = 1 - t_ij / T, t_ij the coalescence time of tips i and j, T the root's)."""
    groups = [[i] for i in range(ns)]
    t = 0.0
    tij = np.zeros((ns, ns))
    while len(groups) > 1:
        k = len(groups)
        t += rng.exponential(1.0 / (k * (k - 1) / 2.0))
        a, b = rng.choice(k, size=2, replace=False)
        ga, gb = groups[a], groups[b]
        tij[np.ix_(ga, gb)] = t
        tij[np.ix_(gb, ga)] = t
        groups = [g for q, g in enumerate(groups) if q not in (a, b)] + [ga + gb]
    return 1.0 - tij / t


def vignette3_phylo(ns=300, ny=200, seed=SYNTHETIC_SEED):
    """BASELINE.json config 3: vignettes/vignette_3_multivariate_high.Rmd:42-128 with ns species
    ("hundreds of species"): a coalescent phylogeny C, two traits (habitat use, thermal optimum)
    drawn N(0, C), habitat (forest/open) and climate covariates, X = [1, forest, climate,
    climate^2] (nc = 4), TrFormula ~habitat.use + thermal.optimum (nt = 3), species niches
    mu + 0.25 N(0, 1), normal Y = X beta + N(0, 1), one sample-level random level with
    nfMax = 15 (nfMin default 2), default updaters (GammaEta, Rho on)."""
    rng = np.random.default_rng(seed)
    C = coalescent_corr(ns, rng)
    Lc = np.linalg.cholesky(C + 1e-12 * np.eye(ns))
    traits = np.column_stack([Lc @ rng.standard_normal(ns) for _ in range(2)])
    habitat = rng.random(ny) < 0.5
    climate = rng.standard_normal(ny)
    nc = 4
    mu = np.zeros((nc, ns))
    mu[0] = -traits[:, 1] ** 2 / 4 - traits[:, 0]
    mu[1] = 2 * traits[:, 0]
    mu[2] = traits[:, 1] / 2
    mu[3] = -0.25
    beta = mu + 0.25 * rng.standard_normal((nc, ns))
    X = np.column_stack([np.ones(ny), habitat.astype(float), climate, climate ** 2])
    Y = X @ beta + rng.standard_normal((ny, ns))
    Tr = np.column_stack([np.ones(ns), traits])
    units = np.array([f"sample_{i:03d}" for i in range(1, ny + 1)])
    rl = HmscRandomLevel(units=units)
    setPriors(rl, nfMax=15)
    try:
        import pandas as pd
        study = pd.DataFrame({"sample": units})
    except Exception:  # pragma: no cover
        study = {"sample": units}
    return Hmsc(Y=Y, X=X, covNames=["(Intercept)", "habitatforest", "climate", "climate2"], XScale=True,
                Tr=Tr, C=C, distr="normal", studyDesign=study, ranLevels={"sample": rl})


def vignette3_ma500(ns=50, ny=200, seed=SYNTHETIC_SEED, na_frac=0.0):
    """vignette_3's ``ma500`` (vignettes/vignette_3_multivariate_high.Rmd:445-453): the data of
    vignette3_phylo, XFormula.1 = ~poly(climate, degree = 2, raw = TRUE) (nc = 3), the same
    traits and phylogeny, and a FRESH HmscRandomLevel with setPriors(a1 = 500, a2 = 500) only --
    R's default nfMin = 2 and nfMax = Inf (= ns, R/Hmsc.R:554) and default updaters (GammaEta
    and Rho on).  na_frac > 0 blanks that share of Y cells (NA), the phylogeny-with-NA case."""
    base = vignette3_phylo(ns=ns, ny=ny, seed=seed)
    rng = np.random.default_rng(seed + 1)
    X = base.X[:, [0, 2, 3]]   # intercept, climate, climate^2 (no habitat)
    Y = np.array(base.Y, dtype=np.float64)
    if na_frac > 0:
        Y[rng.random(Y.shape) < na_frac] = np.nan
    units = np.array([f"sample_{i:03d}" for i in range(1, ny + 1)])
    rl = HmscRandomLevel(units=units)
    setPriors(rl, a1=500, a2=500)
    try:
        import pandas as pd
        study = pd.DataFrame({"sample": units})
    except Exception:  # pragma: no cover
        study = {"sample": units}
    return Hmsc(Y=Y, X=X, covNames=["(Intercept)", "climate", "climate2"], XScale=True, Tr=base.Tr,
                C=base.C, distr="normal", studyDesign=study, ranLevels={"sample": rl})


def vignette2(model="linear", n=100, seed=SYNTHETIC_SEED):
    """BASELINE.json config 2: the models of vignettes/vignette_2_multivariate_low.Rmd with its
    generators (numpy's stream in place of R's set.seed):
      "linear"     :55   Hmsc(Y, XData, XFormula=~x1+x2), 5 normal species, NO random level (nr = 0)
      "latent"     :143  the same with a sample-level random level (units = 1..n)
      "reduced"    :189  XFormula = ~x1 with the sample level (x2 left to the latent factors)
      "ordination" :253  XFormula = ~1, sample level with nfMin = nfMax = 2
      "mixed"      :299  4 species normal / probit / Poisson / lognormal Poisson, ~x1+x2, nr = 0
    """
    rng = np.random.default_rng(seed)
    x1, x2 = rng.standard_normal(n), rng.standard_normal(n)
    if model == "mixed":
        b1, b2 = np.array([1.0, 1, -1, -1]), np.array([1.0, -1, 1, -1])       # :277-279
        L = np.outer(x1, b1) + np.outer(x2, b2)
        Y = np.empty((n, 4))
        Y[:, 0] = L[:, 0] + rng.standard_normal(n)                             # :287-290
        Y[:, 1] = ((L[:, 1] + rng.standard_normal(n)) > 0).astype(np.float64)
        Y[:, 2] = rng.poisson(np.exp(L[:, 2]))
        Y[:, 3] = rng.poisson(np.exp(L[:, 3] + rng.standard_normal(n)))
        X = np.column_stack([np.ones(n), x1, x2])
        return Hmsc(Y=Y, X=X, covNames=["(Intercept)", "x1", "x2"], XScale=True,
                    distr=["normal", "probit", "poisson", "lognormal poisson"])
    b1, b2 = np.array([1.0, 1, -1, -1, 0]), np.array([1.0, -1, 1, -1, 0])      # :36-38
    Y = np.outer(x1, b1) + np.outer(x2, b2) + rng.standard_normal((n, 5))      # :41-44
    cols = {"linear": [x1, x2], "latent": [x1, x2], "reduced": [x1], "ordination": []}[model]
    X = np.column_stack([np.ones(n)] + cols)
    covNames = ["(Intercept)"] + ["x1", "x2"][:len(cols)]
    if model == "linear":
        return Hmsc(Y=Y, X=X, covNames=covNames, XScale=True, distr="normal")
    units = np.arange(1, n + 1)
    rl = HmscRandomLevel(units=units)                                          # :142-143
    if model == "ordination":
        setPriors(rl, nfMin=2, nfMax=2)                                        # :250-251
    try:
        import pandas as pd
        study = pd.DataFrame({"sample": units})
    except Exception:  # pragma: no cover
        study = {"sample": units}
    return Hmsc(Y=Y, X=X, covNames=covNames, XScale=True, distr="normal", studyDesign=study,
                ranLevels={"sample": rl})
