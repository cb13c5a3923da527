"""Model specification — the host-side mirror of the reference's R API for the
sampler's inputs: ``Hmsc()`` (R/Hmsc.R:109-635), ``HmscRandomLevel()``
(R/HmscRandomLevel.R:38-94) and ``setPriors()`` (R/setPriors.Hmsc.R:20-105,
R/setPriors.HmscRandomLevel.R:18-110).

Same argument names, meanings, defaults and error messages as the R functions,
so that a user of ``Hmsc(...)`` / ``sampleMcmc(...)`` finds the same surface.
The object keeps R's 72 field names (the layout the reference's
tests/testthat/test-sampling.R:167 asserts).  Matrices are numpy arrays in R's
orientation (rows = sampling units, columns = species / covariates).
"""
import math
import re

import numpy as np

try:  # pandas is the natural stand-in for R data.frames; optional
    import pandas as pd
except Exception:  # pragma: no cover
    pd = None

HM_FIELDS = [
    "Y", "XData", "XFormula", "X", "XScaled", "XRRRData", "XRRRFormula", "XRRRScaled", "YScaled",
    "XInterceptInd", "studyDesign", "ranLevels", "ranLevelsUsed", "dfPi", "rL", "Pi", "TrData", "TrFormula",
    "Tr", "TrScaled", "TrInterceptInd", "C", "phyloTree", "distr", "ny", "ns", "nc", "ncNRRR", "ncRRR",
    "ncORRR", "ncsel", "nr", "nt", "nf", "ncr", "ncs", "np", "spNames", "covNames", "trNames", "rLNames",
    "XScalePar", "XRRRScalePar", "YScalePar", "TrScalePar", "V0", "f0", "mGamma", "UGamma", "aSigma",
    "bSigma", "nu", "a1", "b1", "a2", "b2", "rhopw", "nuRRR", "a1RRR", "b1RRR", "a2RRR", "b2RRR", "samples",
    "transient", "thin", "verbose", "adaptNf", "initPar", "repN", "randSeed", "postList", "repList"]


class _RList:
    """An R named list: ordered fields with attribute access; ``len`` = field count."""

    _field_names = ()

    def __init__(self):
        object.__setattr__(self, "_f", {k: None for k in self._field_names})

    def __getattr__(self, k):
        f = object.__getattribute__(self, "_f")
        if k in f:
            return f[k]
        raise AttributeError(k)

    def __setattr__(self, k, v):
        self._f[k] = v

    def __getitem__(self, k):
        return self._f[k]

    def __setitem__(self, k, v):
        self._f[k] = v

    def __len__(self):
        return len(self._f)

    def names(self):
        return list(self._f)

    def copy(self):
        new = type(self).__new__(type(self))
        object.__setattr__(new, "_f", dict(self._f))
        return new


class HmscRandomLevel(_RList):
    _field_names = ("pi", "s", "sDim", "spatialMethod", "x", "xDim", "N", "distMat", "nfMax", "nfMin",
                    "nNeighbours", "nu", "a1", "b1", "a2", "b2", "alphapw")

    def __init__(self, sData=None, sMethod="Full", distMat=None, xData=None, units=None, N=None,
                 nNeighbours=None, sKnot=None):
        """R/HmscRandomLevel.R:38-94."""
        super().__init__()
        if all(a is None for a in (sData, distMat, xData, units, N)):
            raise ValueError("HmscRandomLevel: At least one argument must be specified")
        if distMat is not None and sData is not None:
            raise ValueError("HmscRandomLevel: sData and distMat cannot both be specified")
        self.sDim = 0
        if sData is not None:
            s = np.asarray(sData, dtype=np.float64)
            self.s = s
            # rownames(sData): R indexes rL$s by unit name (computeDataParameters, predictLatentFactor)
            self["sNames"] = [str(i) for i in sData.index] if hasattr(sData, "index") else None
            self.N = s.shape[0]
            self.sDim = s.shape[1]
            self.spatialMethod = sMethod
            self.nNeighbours = nNeighbours
            self["sKnot"] = sKnot
        if distMat is not None:
            self.distMat = np.asarray(distMat, dtype=np.float64)
            # rownames(distMat): R indexes rL$distMat by unit name (predictLatentFactor)
            self["distNames"] = [str(i) for i in distMat.index] if hasattr(distMat, "index") else None
            self.N = self.distMat.shape[0]
            self.spatialMethod = sMethod
            self.sDim = math.inf
        self.xDim = 0
        if xData is not None:
            self.x = xData
            self.xDim = np.asarray(xData).shape[1]
            self.N = np.asarray(xData).shape[0]
        if units is not None:
            if self.pi is not None:
                raise ValueError("HmscRandomLevel: duplicated specification of unit names")
            self.pi = _factor_levels(units)
            self.N = len(units)
            self.sDim = 0
        if N is not None:
            if self.pi is not None:
                raise ValueError("HmscRandomLevel: duplicated specification of the number of units")
            self.N = N
            self.pi = [str(i) for i in range(1, N + 1)]
            self.sDim = 0
        setPriors(self, setDefault=True)


def _factor_levels(x):
    """Levels of R's as.factor(x): category order for categoricals, else sorted unique values."""
    if pd is not None and isinstance(getattr(x, "dtype", None), pd.CategoricalDtype):
        return [str(c) for c in x.cat.categories]
    vals = list(x)
    uniq = sorted(set(vals), key=lambda v: (0, float(v)) if _isnum(v) else (1, str(v)))
    return [str(v) for v in uniq]


def _isnum(v):
    try:
        float(v)
        return not isinstance(v, str)
    except (TypeError, ValueError):
        return False


def _as_factor_codes(x):
    """as.numeric(as.factor(x)) -> 1-based codes (R/Hmsc.R:547-549)."""
    if pd is not None and isinstance(getattr(x, "dtype", None), pd.CategoricalDtype):
        codes = np.asarray(x.cat.codes) + 1
        used = np.unique(codes)
        remap = {c: k + 1 for k, c in enumerate(used)}
        return np.array([remap[c] for c in codes], dtype=np.int64)
    levels = _factor_levels(x)
    pos = {lv: k + 1 for k, lv in enumerate(levels)}
    return np.array([pos[str(v)] for v in x], dtype=np.int64)


def _parse_formula(formula, columns):
    f = formula.replace(" ", "")
    if not f.startswith("~"):
        raise ValueError("formula must start with '~'")
    rhs = f[1:]
    intercept = True
    terms = []
    for tok in re.findall(r"[+-]?[^+-]+", rhs):
        sign = -1 if tok.startswith("-") else 1
        name = tok.lstrip("+-")
        if name in ("1", "0"):
            if (name == "1" and sign < 0) or name == "0":
                intercept = False
            continue
        if name == ".":
            for c in columns:
                if c not in terms:
                    terms.append(c)
            continue
        if any(ch in name for ch in ":*^("):
            raise NotImplementedError(f"formula term '{name}': only main effects are supported")
        if sign < 0:
            terms = [t for t in terms if t != name]
        else:
            terms.append(name)
    return intercept, terms


def model_matrix(formula, data):
    """R's model.matrix(formula, data) for main effects with treatment contrasts."""
    if pd is None:
        raise RuntimeError("XData / TrData need pandas")
    df = pd.DataFrame(data)
    intercept, terms = _parse_formula(formula, list(df.columns))
    cols, names = [], []
    if intercept:
        cols.append(np.ones(len(df)))
        names.append("(Intercept)")
    for t in terms:
        v = df[t]
        if pd.api.types.is_numeric_dtype(v) and not pd.api.types.is_bool_dtype(v):
            cols.append(np.asarray(v, dtype=np.float64))
            names.append(t)
        else:
            levels = _factor_levels(v)
            sv = np.array([str(x) for x in v])
            use = levels[1:] if intercept or len(names) > 0 else levels
            for lv in use:
                cols.append((sv == lv).astype(np.float64))
                names.append(f"{t}{lv}")
    return np.column_stack(cols) if cols else np.zeros((len(df), 0)), names


def _r_scale(A, center=True):
    """R's scale(): centre by column means, divide by column sd (n-1)."""
    A = np.asarray(A, dtype=np.float64)
    n = A.shape[0]
    with np.errstate(divide="ignore", invalid="ignore"):
        mu = A.mean(axis=0) if center else np.zeros(A.shape[1])
        C = A - mu
        sd = np.sqrt((C ** 2).sum(axis=0) / (n - 1))
        return C / sd, mu, sd


def _is01(col):
    return np.all(np.isin(col, [0.0, 1.0]))


class Hmsc(_RList):
    """R/Hmsc.R:109 — Hierarchical Modelling of Species Communities model object."""

    _field_names = tuple(HM_FIELDS)

    def __init__(self, Y, XFormula="~.", XData=None, X=None, XScale=True, XSelect=None, XRRRData=None,
                 XRRRFormula="~.-1", XRRR=None, ncRRR=2, XRRRScale=True, YScale=False, studyDesign=None,
                 ranLevels=None, ranLevelsUsed=None, TrFormula=None, TrData=None, Tr=None, TrScale=True,
                 phyloTree=None, C=None, distr="normal", truncateNumberOfFactors=True, spNames=None,
                 covNames=None):
        super().__init__()
        Y = np.asarray(Y, dtype=np.float64)
        if Y.ndim != 2:
            raise ValueError("Hmsc.setData: Y argument must be a matrix of sampling units times species")
        self.Y = Y
        self.ny, self.ns = Y.shape
        ny, ns = Y.shape
        w = math.ceil(math.log10(ns)) if ns > 1 else 1
        self.spNames = list(spNames) if spNames is not None else [f"sp{k:0{w}d}" for k in range(1, ns + 1)]
        if XSelect is not None or XRRRData is not None or XRRR is not None:
            raise NotImplementedError("XSelect / reduced-rank regression are out of scope (SURVEY.md §2 row 5)")
        # ---- covariates (R/Hmsc.R:185-330)
        if XData is not None and X is not None:
            raise ValueError("Hmsc.setData: only single of XData and X arguments must be specified")
        if XData is not None:
            if isinstance(XData, list):
                raise NotImplementedError("species-specific X lists are out of scope (used only with XSelect)")
            Xm, names = model_matrix(XFormula, XData)
            if Xm.shape[0] != ny:
                raise ValueError("Hmsc.setData: the number of rows in XData must be equal to the number of sampling units")
            self.XData = XData
            self.XFormula = XFormula
            self.X = Xm
            self.covNames = names
        elif X is not None:
            Xm = np.asarray(X, dtype=np.float64)
            if Xm.ndim == 1:
                Xm = Xm[:, None]
            if Xm.shape[0] != ny:
                raise ValueError("Hmsc.setData: the number of rows in X must be equal to the number of sampling units")
            if np.isnan(Xm).any():
                raise ValueError("Hmsc.setData: X must contain no NA values")
            self.X = Xm
            nc = Xm.shape[1]
            wc = math.ceil(math.log10(nc)) if nc > 1 else 1
            self.covNames = list(covNames) if covNames is not None else [f"cov{k:0{wc}d}" for k in range(1, nc + 1)]
        else:
            self.X = np.zeros((ny, 0))
            self.covNames = []
        self.nc = self.X.shape[1]
        if XScale is False:
            self.XScalePar = np.vstack([np.zeros(self.nc), np.ones(self.nc)])
            self.XScaled = self.X.copy()
            self.XInterceptInd = None
        else:
            ii = [k for k, n in enumerate(self.covNames) if n in ("Intercept", "(Intercept)")]
            if len(ii) > 1:
                raise ValueError("Hmsc.setData: only one column of X matrix could be named Intercept or (Intercept)")
            if ii and not np.all(self.X[:, ii[0]] == 1):
                raise ValueError("Hmsc.setData: intercept column in X matrix must be a column of ones")
            self.XInterceptInd = ii[0] + 1 if ii else None
            if XScale is True:
                scaleInd = np.array([not _is01(self.X[:, k]) for k in range(self.nc)], dtype=bool)
            else:
                scaleInd = np.asarray(XScale, dtype=bool)
            if ii:
                scaleInd[ii[0]] = False
            par = np.vstack([np.zeros(self.nc), np.ones(self.nc)])
            XS = self.X.copy()
            sc, mu, sd = _r_scale(self.X, center=bool(ii))
            par[0, scaleInd] = mu[scaleInd] if ii else 0.0
            par[1, scaleInd] = sd[scaleInd]
            XS[:, scaleInd] = sc[:, scaleInd]
            self.XScalePar = par
            self.XScaled = XS
        self.ncsel = 0
        self.ncNRRR = self.nc
        self.ncRRR = 0
        self.ncORRR = 0
        # ---- traits (R/Hmsc.R:423-498)
        if TrData is not None and Tr is not None:
            raise ValueError("Hmsc.setData: at maximum one of TrData and Tr arguments can be specified")
        if TrData is not None:
            if TrFormula is None:
                raise ValueError("Hmsc.setData: TrFormula argument must be specified if TrData is provided")
            Trm, trn = model_matrix(TrFormula, TrData)
            if Trm.shape[0] != ns:
                raise ValueError("Hmsc.setData: the number of rows in TrData should be equal to number of columns in Y")
            self.TrData, self.TrFormula, self.Tr, self.trNames = TrData, TrFormula, Trm, trn
        elif Tr is not None:
            Trm = np.asarray(Tr, dtype=np.float64)
            if Trm.shape[0] != ns:
                raise ValueError("Hmsc.setData: the number of rows in Tr should be equal to number of columns in Y")
            self.Tr = Trm
            nt = Trm.shape[1]
            wt = math.ceil(math.log10(nt)) if nt > 1 else 1
            self.trNames = [f"tr{k:0{wt}d}" for k in range(1, nt + 1)]
        else:
            self.Tr = np.ones((ns, 1))
            self.trNames = ["tr1"]
        self.nt = self.Tr.shape[1]
        if TrScale is False:
            self.TrScalePar = np.vstack([np.zeros(self.nt), np.ones(self.nt)])
            self.TrScaled = self.Tr.copy()
            self.TrInterceptInd = None
        else:
            ii = [k for k, n in enumerate(self.trNames) if n in ("Intercept", "(Intercept)")]
            if len(ii) > 1:
                raise ValueError("Hmsc.setData: only one column of Tr matrix could be named Intercept or (Intercept)")
            self.TrInterceptInd = ii[0] + 1 if ii else None
            scaleInd = np.array([not _is01(self.Tr[:, k]) for k in range(self.nt)], dtype=bool) \
                if TrScale is True else np.asarray(TrScale, dtype=bool)
            if ii:
                scaleInd[ii[0]] = False
            par = np.vstack([np.zeros(self.nt), np.ones(self.nt)])
            TS = self.Tr.copy()
            sc, mu, sd = _r_scale(self.Tr, center=bool(ii))
            par[0, scaleInd] = mu[scaleInd] if ii else 0.0
            par[1, scaleInd] = sd[scaleInd]
            TS[:, scaleInd] = sc[:, scaleInd]
            self.TrScalePar = par
            self.TrScaled = TS
        # ---- phylogeny (R/Hmsc.R:501-515)
        if C is not None and phyloTree is not None:
            raise ValueError("Hmsc.setData: at maximum one of phyloTree and C arguments can be specified")
        if phyloTree is not None:
            # corM = vcv.phylo(phyloTree, model="Brownian", corr=TRUE)[spNames, spNames] (:504-508)
            from .phylo import read_tree, vcv_phylo
            tree = read_tree(phyloTree) if isinstance(phyloTree, str) else phyloTree
            corM, tips = vcv_phylo(tree, corr=True)
            where = {t: k for k, t in enumerate(tips)}
            missing = [s for s in self.spNames if s not in where]
            if missing:
                raise ValueError(f"Hmsc.setData: species {missing[:5]} are not tips of phyloTree")
            ix = np.array([where[s] for s in self.spNames])
            self.phyloTree = tree
            C = corM[np.ix_(ix, ix)]
        if C is not None:
            C = np.asarray(C, dtype=np.float64)
            if C.shape != (ns, ns):
                raise ValueError("Hmsc.setData: the size of square matrix C must be equal to number of species")
            self.C = C
        # ---- random levels (R/Hmsc.R:518-558)
        if studyDesign is None:
            self.Pi = np.zeros((ny, 0), dtype=np.int64)
            self.np = np.zeros(0, dtype=np.int64)
            self.nr = 0
            self.rLNames = []
            self.rL = []
            if ranLevels:
                raise ValueError("Hmsc.setData: studyDesign is empty, but ranLevels is not")
        else:
            if ranLevelsUsed is None:
                ranLevelsUsed = list(ranLevels.keys()) if ranLevels else []
            sd_cols = list(studyDesign.columns) if hasattr(studyDesign, "columns") else list(studyDesign)
            n_sd = len(studyDesign) if hasattr(studyDesign, "columns") else len(next(iter(studyDesign.values())))
            if n_sd != ny:
                raise ValueError("Hmsc.setData: the number of rows in studyDesign must be equal to number of rows in Y")
            if not all(r in (ranLevels or {}) for r in ranLevelsUsed):
                raise ValueError("Hmsc.setData: ranLevels must contain named elements corresponding to all levels listed in ranLevelsUsed")
            if not all(r in sd_cols for r in ranLevelsUsed):
                raise ValueError("Hmsc.setData: studyDesign must contain named columns corresponding to all levels listed in ranLevelsUsed")
            self.studyDesign = studyDesign
            self.ranLevels = ranLevels
            self.ranLevelsUsed = list(ranLevelsUsed)
            self.dfPi = {r: studyDesign[r] for r in ranLevelsUsed}
            self.rL = [ranLevels[r].copy() for r in ranLevelsUsed]
            self.rLNames = list(ranLevelsUsed)
            self.Pi = np.column_stack([_as_factor_codes(self.dfPi[r]) for r in ranLevelsUsed]).astype(np.int64) \
                if ranLevelsUsed else np.zeros((ny, 0), dtype=np.int64)
            self.np = np.array([len(np.unique(self.Pi[:, r])) for r in range(self.Pi.shape[1])], dtype=np.int64)
            self.nr = self.Pi.shape[1]
            if truncateNumberOfFactors:
                for rl in self.rL:
                    rl.nfMax = min(rl.nfMax, ns)
                    rl.nfMin = min(rl.nfMin, rl.nfMax)
        # ---- observation models (R/Hmsc.R:560-612)
        self.distr = _distr_matrix(distr, ns)
        # ---- response scaling (R/Hmsc.R:614-629)
        if YScale is False:
            self.YScalePar = np.vstack([np.zeros(ns), np.ones(ns)])
            self.YScaled = self.Y.copy()
        else:
            ind = np.nonzero(self.distr[:, 0] == 1)[0]
            par = np.vstack([np.zeros(ns), np.ones(ns)])
            YS = self.Y.copy()
            if len(ind):
                mu = np.nanmean(self.Y, axis=0)
                cnt = np.sum(~np.isnan(self.Y), axis=0)
                sd = np.sqrt(np.nansum((self.Y - mu) ** 2, axis=0) / (cnt - 1))
                par[0, ind] = mu[ind]
                par[1, ind] = sd[ind]
                YS[:, ind] = (self.Y[:, ind] - mu[ind]) / sd[ind]
            self.YScalePar = par
            self.YScaled = YS
        setPriors(self, setDefault=True)


def _distr_matrix(distr, ns):
    codes = {"normal": (1, 1), "probit": (2, 0), "poisson": (3, 0), "lognormal poisson": (3, 1)}
    if isinstance(distr, np.ndarray) and distr.ndim == 2:
        d = distr.astype(np.float64)
    else:
        if isinstance(distr, str):
            distr = [distr] * ns
        d = np.zeros((ns, 4))
        for i, name in enumerate(distr):
            fam, var = codes.get(name, (0, 0))
            d[i, 0], d[i, 1] = fam, var
    if np.any(d[:, 0] == 0):
        raise ValueError("Hmsc.setData: some of the distributions ill defined")
    return d


def setPriors(obj, setDefault=False, **kw):
    """Dispatch like R's S3 setPriors (R/setPriors.R)."""
    if isinstance(obj, Hmsc):
        return _set_priors_hmsc(obj, setDefault=setDefault, **kw)
    if isinstance(obj, HmscRandomLevel):
        return _set_priors_rl(obj, setDefault=setDefault, **kw)
    raise TypeError("setPriors: unsupported object")


def _set_priors_hmsc(hM, V0=None, f0=None, mGamma=None, UGamma=None, aSigma=None, bSigma=None, rhopw=None,
                     setDefault=False, **_):
    """R/setPriors.Hmsc.R:20-105."""
    nc, nt, ns = hM.nc, hM.nt, hM.ns
    if V0 is not None:
        V0 = np.asarray(V0, dtype=np.float64)
        if V0.shape != (nc, nc) or not np.allclose(V0, V0.T):
            raise ValueError("HMSC.setPriors: V0 must be a positive definite matrix of size equal to number of covariates nc")
        hM.V0 = V0
    elif setDefault:
        hM.V0 = np.eye(nc)
    if f0 is not None:
        if f0 < nc:
            raise ValueError("HMSC.setPriors: f0 must be greater than number of covariates in the model nc")
        hM.f0 = float(f0)
    elif setDefault:
        hM.f0 = float(nc + 1)
    if mGamma is not None:
        mGamma = np.asarray(mGamma, dtype=np.float64).ravel()
        if mGamma.size != nc * nt:
            raise ValueError("HMSC.setPriors: mGamma must be a vector of length equal to number of covariates times traits: nc x nt")
        hM.mGamma = mGamma
    elif setDefault:
        hM.mGamma = np.zeros(nc * nt)
    if UGamma is not None:
        UGamma = np.asarray(UGamma, dtype=np.float64)
        if UGamma.shape != (nc * nt, nc * nt):
            raise ValueError("HMSC.setPriors: UGamma must be a positive definite matrix of size equal to nc x nt")
        hM.UGamma = UGamma
    elif setDefault:
        hM.UGamma = np.eye(nc * nt)
    if aSigma is not None:
        hM.aSigma = np.broadcast_to(np.asarray(aSigma, dtype=np.float64), (ns,)).copy()
    elif setDefault:
        hM.aSigma = np.ones(ns)
    if bSigma is not None:
        hM.bSigma = np.broadcast_to(np.asarray(bSigma, dtype=np.float64), (ns,)).copy()
    elif setDefault:
        hM.bSigma = np.full(ns, 5.0)
    if rhopw is not None:
        if hM.C is None:
            raise ValueError("HMSC.setPriors: prior for phylogeny given, but no phylogenic relationship matrix was specified")
        hM.rhopw = np.asarray(rhopw, dtype=np.float64)
    elif setDefault:
        rhoN = 100
        hM.rhopw = np.column_stack([np.arange(rhoN + 1) / rhoN, np.r_[0.5, np.full(rhoN, 0.5 / rhoN)]])
    if setDefault:
        hM.nuRRR, hM.a1RRR, hM.b1RRR, hM.a2RRR, hM.b2RRR = 3, 1, 1, 50, 1
    return hM


def _set_priors_rl(rL, nu=None, a1=None, b1=None, a2=None, b2=None, alphapw=None, nfMax=None, nfMin=None,
                   setDefault=False, **_):
    """R/setPriors.HmscRandomLevel.R:18-110.  The shrinkage priors are one value per column of
    rL$x for a covariate-dependent level (xDim = max(rL$xDim, 1), :21-80: a scalar is repeated,
    a vector must have length xDim), a scalar otherwise."""
    xDim = max(int(rL.xDim or 0), 1)
    for name, val, dflt in (("nu", nu, 3.0), ("a1", a1, 50.0), ("b1", b1, 1.0), ("a2", a2, 50.0), ("b2", b2, 1.0)):
        if val is not None:
            v = np.atleast_1d(np.asarray(val, dtype=np.float64))
            if v.size == 1:
                rL[name] = float(v[0]) if not rL.xDim else np.full(xDim, float(v[0]))
            elif v.size == xDim:
                rL[name] = v.copy()
            else:
                raise ValueError(f"HmscRandomLevel.setPriors: length of {name} argument must be either 1 or rL$xDim")
        elif setDefault:
            rL[name] = dflt if not rL.xDim else np.full(xDim, dflt)
    if alphapw is not None:
        if not rL.sDim:
            raise ValueError("HmscRandomLevel.setPriors: prior for spatial scale was given, but not spatial coordinates were specified")
        rL.alphapw = np.asarray(alphapw, dtype=np.float64)
    elif setDefault and rL.sDim:
        alphaN = 100
        if rL.distMat is None:
            diag = math.sqrt(float(np.sum((rL.s.max(axis=0) - rL.s.min(axis=0)) ** 2)))
        else:
            diag = float(np.max(rL.distMat))
        rL.alphapw = np.column_stack([diag * np.arange(alphaN + 1) / alphaN, np.r_[0.5, np.full(alphaN, 0.5 / alphaN)]])
    if nfMax is not None:
        rL.nfMax = nfMax
    elif setDefault:
        rL.nfMax = math.inf
    if nfMin is not None:
        if nfMin > rL.nfMax:
            raise ValueError("HmscRandomLevel.setPriors: nfMin must be not greater than nfMax")
        rL.nfMin = nfMin
    elif setDefault:
        rL.nfMin = 2
    return rL
