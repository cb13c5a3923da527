"""Post-sampling callers of the hot path, host side of the R wrapper.

predict (R/predict.R:1-231) keeps R's host logic -- argument checks, predictLatentFactor for
the prediction units (R/predictLatentFactor.R), the Pi of the new study design -- and hands
the per-sample loop (linear predictor, expected values or draws, Y back-scaling) to the HIP
kernel behind ``hmsc_predict`` (hmsc_amd/csrc/predict.hip).  computePredictedValues
(R/computePredictedValues.R:66-142) and evaluateModelFit (R/evaluateModelFit.R) sit on top.
There is no CPU fallback: without the HIP library predict raises HmscNativeError.
"""
import ctypes as C

import numpy as np
from scipy import stats

from . import _lib as L
from .model import _factor_levels
from .post import poolMcmcChains


def _levels(values):
    """levels(as.factor(x)) by the same rule hM$Pi was built with (model._as_factor_codes)."""
    return [str(v) for v in _factor_levels(values)]


def _coords(rL, names, units):
    """Rows of rL$s for the given unit names (R indexes rL$s by rownames)."""
    sn = rL["sNames"] if "sNames" in rL.names() else None
    s = np.asarray(rL.s, dtype=np.float64)
    if sn is None:            # unnamed coordinates: row k is the k-th level of the fitted units
        pos = {u: k for k, u in enumerate(units)}
        if any(n not in pos for n in names) or s.shape[0] != len(units):
            raise ValueError("predictLatentFactor: coordinates of new spatial units are needed: give sData "
                             "as a DataFrame whose index names every unit (rownames of rL$s)")
    else:
        pos = {str(u): k for k, u in enumerate(sn)}
    return s[[pos[str(n)] for n in names]]


def _dist_rows(rL, names, units):
    """Row / column indices of rL$distMat for the given unit names (R indexes it by
    rownames, R/predictLatentFactor.R:69-70,100)."""
    dn = rL["distNames"] if "distNames" in rL.names() else None
    if dn is None:            # unnamed: row k is the k-th level of the fitted units
        pos = {u: k for k, u in enumerate(units)}
        if any(n not in pos for n in names) or rL.distMat.shape[0] != len(units):
            raise ValueError("predictLatentFactor: distances to new spatial units are needed: give distMat "
                             "as a DataFrame whose index names every unit (rownames of rL$distMat)")
    else:
        pos = {str(u): k for k, u in enumerate(dn)}
        missing = [n for n in names if str(n) not in pos]
        if missing:
            raise ValueError(f"predictLatentFactor: units {missing[:5]} are not rows of rL$distMat")
    return np.array([pos[str(n)] for n in names], dtype=np.int64)


def _pdist(a, b):
    return np.sqrt(((a[:, None, :] - b[None, :, :]) ** 2).sum(-1))


def predictLatentFactor(unitsPred, units, postEta, rL, predictMean=False, rng=None, postAlpha=None,
                        predictMeanField=False):
    """R/predictLatentFactor.R:35-210 (host side of predict, as in R): known units keep their
    posterior Eta rows; new units of a non-spatial level get N(0, 1) draws (0 with
    predictMean); new units of a spatial level are kriged from the sample's Eta with its
    alphapw grid scale alpha_h (:59-204): predictMean / predictMeanField (:62-92), or the
    method's joint conditional -- Full (:95-117), NNGP over the nNeighbours nearest fitted
    units (:118-160), GPP through the knots (:161-203; R uses alpha[nf] for every factor
    there, and so does this restatement)."""
    if predictMean and predictMeanField:
        raise ValueError("Hmsc.predictLatentFactor: predictMean and predictMeanField arguments cannot be simultaneously TRUE")
    units = [str(u) for u in units]
    unitsPred = [str(u) for u in unitsPred]
    pos = {u: k for k, u in enumerate(units)}
    old = np.array([u in pos for u in unitsPred], dtype=bool)
    new = ~old
    nn = int(new.sum())
    rng = rng or np.random.default_rng()
    spatial = bool(rL.sDim) and nn > 0
    if spatial:
        if postAlpha is None:
            raise ValueError("predictLatentFactor: postAlpha is needed for new units of a spatial level")
        newu = [u for u, o in zip(unitsPred, old) if not o]
        if rL.distMat is not None:
            # a level given by distances (R/predictLatentFactor.R:69-70,100): D from rL$distMat;
            # 'NNGP' and 'GPP' need coordinates in R too (rL$s, :120,163)
            if not (predictMean or predictMeanField) and rL.spatialMethod != "Full":
                raise ValueError(f"predictLatentFactor: spatialMethod '{rL.spatialMethod}' needs coordinates "
                                 f"(sData); a distMat level predicts with 'Full'")
            s1 = _dist_rows(rL, units, units)
            s2 = _dist_rows(rL, newu, units)
        else:
            s1 = _coords(rL, units, units)
            s2 = _coords(rL, newu, units)
        alphapw = np.asarray(rL.alphapw, dtype=np.float64)
    out = []
    for k, eta in enumerate(postEta):
        nf = eta.shape[1]
        e = np.empty((len(unitsPred), nf))
        if old.any():
            e[old] = eta[[pos[u] for u, o in zip(unitsPred, old) if o]]
        if nn and not spatial:
            e[new] = 0.0 if predictMean else rng.standard_normal((nn, nf))
        elif nn:
            e[new] = _krige(rL, eta, np.asarray(postAlpha[k]), alphapw, s1, s2, predictMean, predictMeanField, rng)
        out.append(e)
    return out


def _krige(rL, eta, alpha, alphapw, s1, s2, predictMean, predictMeanField, rng):
    npo, nf, nn = s1.shape[0], eta.shape[1], s2.shape[0]
    res = np.empty((nn, nf))
    dm = rL.distMat
    if predictMean or predictMeanField:                                       # :62-92
        # (with distMat R's :69-70 index rL$distMat by s1 / s2, which that branch never sets --
        # an error in R; the fitted and new units' rows are what it evidently means)
        if dm is not None:
            D11, D12 = dm[np.ix_(s1, s1)], dm[np.ix_(s1, s2)]
        else:
            D11, D12 = _pdist(s1, s1), _pdist(s1, s2)
        for h in range(nf):
            a = alphapw[alpha[h] - 1, 0]
            if a > 0:
                K11, K12 = np.exp(-D11 / a), np.exp(-D12 / a)
                m = K12.T @ np.linalg.solve(K11, eta[:, h])
                if predictMean:
                    res[:, h] = m
                else:
                    iLK = np.linalg.solve(np.linalg.cholesky(K11), K12)
                    res[:, h] = m + rng.standard_normal(nn) * np.sqrt(1 - (iLK ** 2).sum(axis=0))
            else:
                res[:, h] = 0.0 if predictMean else rng.standard_normal(nn)
        return res
    method = rL.spatialMethod
    if method == "Full":                                                      # :95-117
        if dm is not None:
            ua = np.concatenate([s1, s2])
            D = dm[np.ix_(ua, ua)]
        else:
            D = _pdist(np.vstack([s1, s2]), np.vstack([s1, s2]))
        for h in range(nf):
            a = alphapw[alpha[h] - 1, 0]
            if a > 0:
                K = np.exp(-D / a)
                K11, K12, K22 = K[:npo, :npo], K[:npo, npo:], K[npo:, npo:]
                m = K12.T @ np.linalg.solve(K11, eta[:, h])
                W = K22 - K12.T @ np.linalg.solve(K11, K12)
                res[:, h] = m + np.linalg.cholesky(W) @ rng.standard_normal(nn)
            else:
                res[:, h] = rng.standard_normal(nn)
    elif method == "NNGP":                                                    # :118-160
        k = int(rL.nNeighbours) if rL.nNeighbours is not None else 10
        d = _pdist(s2, s1)
        ind = np.argsort(d, axis=1, kind="stable")[:, :k]                     # FNN::knnx.index
        for h in range(nf):
            a = alphapw[alpha[h] - 1, 0]
            if a > 0:
                m = np.empty(nn)
                F = np.empty(nn)
                for i in range(nn):
                    K11 = np.exp(-_pdist(s1[ind[i]], s1[ind[i]]) / a)
                    K12 = np.exp(-d[i, ind[i]] / a)
                    w = np.linalg.solve(K11, K12)
                    m[i] = w @ eta[ind[i], h]
                    F[i] = 1 - w @ K12
                res[:, h] = m + np.sqrt(F) * rng.standard_normal(nn)
            else:
                res[:, h] = rng.standard_normal(nn)
    elif method == "GPP":                                                     # :161-203
        sK = np.asarray(rL["sKnot"], dtype=np.float64)
        dss, dns, dnsOld = _pdist(sK, sK), _pdist(s2, sK), _pdist(s1, sK)
        for h in range(nf):
            a = alphapw[alpha[nf - 1] - 1, 0]                                  # R: ag = alpha[nf]
            if a > 0:
                Wns, W12, Wss = np.exp(-dns / a), np.exp(-dnsOld / a), np.exp(-dss / a)
                iWss = np.linalg.inv(Wss)
                dDn = 1 - ((Wns @ iWss) * Wns).sum(axis=1)
                idD = 1 / (1 - np.einsum("ik,kl,il->i", W12, iWss, W12))
                idDW12 = idD[:, None] * W12
                iF = np.linalg.inv(Wss + W12.T @ idDW12)
                LiF = np.linalg.cholesky(iF).T                                 # chol(): upper
                mu = iF @ idDW12.T @ eta[:, h] + LiF @ rng.standard_normal(sK.shape[0])
                res[:, h] = Wns @ mu + np.sqrt(dDn) * rng.standard_normal(nn)
            else:
                res[:, h] = rng.standard_normal(nn)
    else:
        raise ValueError(f"unknown spatialMethod {method!r}")
    return res


def predict(hM, post=None, X=None, studyDesign=None, Yc=None, mcmcStep=1, expected=False, predictEtaMean=False,
            seed=None, device=0, predictEtaMeanField=False):
    """predict.Hmsc (R/predict.R): a list of ny x ns arrays, one per posterior sample.  With Yc
    (conditional prediction, :191-202) each sample's latent factors are first updated given the
    observed part of Yc by updateZ / (updateEta, updateZ) x mcmcStep on the device."""
    post = poolMcmcChains(hM.postList) if post is None else post
    X = np.asarray(hM.X if X is None else X, dtype=np.float64)
    nyN = X.shape[0]
    studyDesign = hM.studyDesign if studyDesign is None else studyDesign
    if Yc is not None:
        Yc = np.asarray(Yc, dtype=np.float64)
        if Yc.shape[1] != hM.ns:
            raise ValueError("hMsc.predict: number of columns in Yc must be equal to ns")
        if Yc.shape[0] != nyN:
            raise ValueError("hMsc.predict: number of rows in Yc and X must be equal")
    rng = np.random.default_rng(seed)
    S = len(post)
    keep = []
    a = L.hmsc_predict_args()
    a.ny, a.ns, a.nc, a.nr, a.nsamples = nyN, hM.ns, X.shape[1], hM.nr, S
    a.expected = 1 if expected else 0
    a.seed = int(rng.integers(1, 2 ** 62)) if seed is None else int(seed)
    a.device = device
    a.X = L.colmajor_ptr(X, keep)
    a.Beta = L.fptr(_stack(keep, [np.asarray(s["Beta"]).reshape(-1, order="F") for s in post]))
    a.sigma = L.fptr(_stack(keep, [np.asarray(s["sigma"], dtype=np.float64) for s in post]))
    a.family = L.colmajor_ptr(hM.distr[:, 0], keep, np.int32)
    a.YScalePar = L.colmajor_ptr(hM.YScalePar, keep)
    if hM.nr:
        # a covariate-dependent level goes to the kernel as one level per column of rL$x with
        # Eta[q, ] * x[q, k] of the prediction units (R/predict.R:171-176: LRan = sum_k
        # (Eta[dfPiNew,] * x[dfPiNew, k]) %*% Lambda[,,k])
        ndev = sum(max(int(rl.xDim or 0), 1) for rl in hM.rL)
        if ndev > L.MAX_LEVELS:
            raise ValueError(f"predict: at most {L.MAX_LEVELS} device levels")
        PiNew = np.zeros((nyN, ndev), dtype=np.int32)
        nps, nfs = [], []
        d = 0
        for r, name in enumerate(hM.rLNames):
            raw = studyDesign[name]
            col = np.asarray(raw).astype(str)
            unitsPred = _levels(raw)
            units = _levels(hM.dfPi[name])
            etas = predictLatentFactor(unitsPred, units, [s["Eta"][r] for s in post], hM.rL[r],
                                       predictMean=predictEtaMean, rng=rng,
                                       postAlpha=[s["Alpha"][r] for s in post] if hM.rL[r].sDim else None,
                                       predictMeanField=predictEtaMeanField)
            if Yc is not None and np.any(~np.isnan(Yc)):
                if r == 0:
                    cond = _conditional_etas(hM, post, X, studyDesign, Yc, mcmcStep, rng, device)
                etas = [c[r] for c in cond]
            nf = max(e.shape[1] for e in etas)
            lams = [np.asarray(s["Lambda"][r]) for s in post]
            etas = [np.pad(e, ((0, 0), (0, nf - e.shape[1]))) for e in etas]      # nf may vary (updateNf)
            lams = [np.pad(lm, ((0, nf - lm.shape[0]),) + ((0, 0),) * (lm.ndim - 1)) for lm in lams]
            idx = {u: k for k, u in enumerate(unitsPred)}
            xd = int(hM.rL[r].xDim or 0)
            xp = _x_rows(hM, r, unitsPred) if xd else None
            for k in range(max(xd, 1)):
                PiNew[:, d] = [idx[v] + 1 for v in col]
                ek = etas if not xd else [e * xp[:, k:k + 1] for e in etas]
                lk = lams if not xd else [lm[:, :, k] for lm in lams]
                a.Eta[d] = L.fptr(_stack(keep, [e.reshape(-1, order="F") for e in ek]))
                a.Lambda[d] = L.fptr(_stack(keep, [lm.reshape(-1, order="F") for lm in lk]))
                nps.append(len(unitsPred))
                nfs.append(nf)
                d += 1
        a.nr = ndev
        a.Pi = L.colmajor_ptr(PiNew, keep, np.int32)
        a.np = L.colmajor_ptr(nps, keep, np.int32)
        a.nf = L.colmajor_ptr(nfs, keep, np.int32)
    out = np.empty(S * nyN * hM.ns)
    L.check(L.lib().hmsc_predict(C.byref(a), L.fptr(out)))
    out = out.reshape(S, hM.ns, nyN).transpose(0, 2, 1)
    return [out[k] for k in range(S)]


def _x_rows(hM, r, units):
    """rL$x rows of the given unit names (R indexes rL$x by unit name, R/predict.R:174); unnamed
    rows are the fitted units in order."""
    rl = hM.rL[r]
    x = np.asarray(rl.x, dtype=np.float64)
    names = [str(i) for i in rl.x.index] if hasattr(rl.x, "index") else None
    if names is None:
        fitted = _levels(hM.dfPi[hM.rLNames[r]])
        pos = {u: k for k, u in enumerate(fitted)}
        if any(u not in pos for u in units) or x.shape[0] != len(fitted):
            raise ValueError(f"predict: covariates of new units of level {hM.rLNames[r]} are needed: give xData "
                             f"as a DataFrame whose index names every unit")
    else:
        pos = {n: k for k, n in enumerate(names)}
        missing = [u for u in units if str(u) not in pos]
        if missing:
            raise ValueError(f"predict: no xData rows for units {missing[:5]} of level {hM.rLNames[r]}")
    return x[[pos[str(u)] for u in units]]


def _conditional_etas(hM, post, X, studyDesign, Yc, mcmcStep, rng, device):
    """R/predict.R:191-202: per sample, Z = L; Z = updateZ(Yc); then mcmcStep x (updateEta,
    updateZ), all with the sample's Beta, sigma, Lambda fixed -- the device updaters of a chain
    built on (Yc, X) in R's unscaled space (X and Beta as `post` holds them)."""
    from .model import Hmsc
    from .sampler import Chain, level_lran
    rl = {name: hM.rL[r] for r, name in enumerate(hM.rLNames)}
    sd = studyDesign.reset_index(drop=True) if hasattr(studyDesign, "reset_index") else studyDesign
    hMc = Hmsc(Y=Yc, X=X, XScale=False, YScale=False, distr=hM.distr, studyDesign=sd, ranLevels=rl,
               covNames=list(hM.covNames), spNames=list(hM.spNames))
    ch = Chain(hMc, int(rng.integers(1, 2 ** 62)), device=device, updater={"GammaEta": False})
    out = []
    try:
        ch.init()
        units = [_levels(hM.dfPi[name]) for name in hM.rLNames]
        for k, sam in enumerate(post):
            etas = []
            for r, name in enumerate(hM.rLNames):
                etas.append(predictLatentFactor(_levels(sd[name]), units[r], [sam["Eta"][r]], hM.rL[r], rng=rng,
                                                postAlpha=[sam["Alpha"][r]] if hM.rL[r].sDim else None)[0])
            L = X @ sam["Beta"]
            for r in range(hM.nr):
                xr = _x_rows(hM, r, _levels(sd[hM.rLNames[r]])) if hM.rL[r].xDim else None
                L = L + level_lran(etas[r], sam["Lambda"][r], hMc.Pi[:, r] - 1, xr)
            # the sample's spatial scales condition the spatial levels' updateEta prior
            # (R/predict.R:185 passes Alpha = sam$Alpha)
            ch.set_state(dict(Beta=sam["Beta"], sigma=np.asarray(sam["sigma"]), Eta=etas,
                              Lambda=[np.asarray(lm) for lm in sam["Lambda"]], Z=L,
                              Alpha=[np.asarray(a, dtype=np.int64).ravel() for a in sam["Alpha"]]))
            it = 1 + k * (2 * mcmcStep + 1)
            ch.update("Z", it)
            for m in range(mcmcStep):
                ch.update("Eta", it + 1 + 2 * m)
                ch.update("Z", it + 2 + 2 * m)
            out.append(ch.get_state(with_z=False)["Eta"])
    finally:
        ch.close()
    return out


def _stack(keep, arrays):
    flat = np.ascontiguousarray(np.concatenate(arrays).astype(np.float64)) if arrays else np.zeros(1)
    keep.append(flat)
    return flat


def computePredictedValues(hM, partition=None, start=1, thin=1, Yc=None, mcmcStep=1, expected=True,
                           initPar=None, nParallel=1, nChains=None, updater=None, verbose=None, seed=None):
    """R/computePredictedValues.R:66-142: ny x ns x predN.  Without a partition, the fitted
    model's own predictions; with one, K-fold cross-validation refits (sampleMcmc on the
    training rows with the fitted run's samples / transient / thin, predictions for the
    held-out rows)."""
    if partition is None:
        post = poolMcmcChains(hM.postList, start=start, thin=thin)
        pred = predict(hM, post=post, Yc=Yc, mcmcStep=mcmcStep, expected=expected, seed=seed)
        return np.stack(pred, axis=2)
    partition = np.asarray(partition)
    nfolds = len(np.unique(partition))
    nChains = len(hM.postList) if nChains is None else nChains
    postN = hM.samples * nChains
    out = np.full((hM.ny, hM.ns, postN), np.nan)
    for k in np.unique(partition):
        train, val = partition != k, partition == k
        hM1 = _cv_refit(hM, train, k, seed, nChains, updater, initPar, nParallel)
        post = poolMcmcChains(hM1.postList, start=start)
        sdv = None if hM.studyDesign is None else hM.studyDesign.loc[val].reset_index(drop=True)
        pred = predict(hM1, post=post, X=hM.X[val], studyDesign=sdv, Yc=None if Yc is None else np.asarray(Yc)[val],
                       mcmcStep=mcmcStep, expected=expected, seed=seed)
        out[val] = np.stack(pred, axis=2)
    del nfolds
    return out


def _cv_fold_model(hM, train):
    """R/computePredictedValues.R:92-116: the model on the training rows, with the full
    model's scalings."""
    from .model import Hmsc
    sd = None if hM.studyDesign is None else hM.studyDesign.loc[train].reset_index(drop=True)
    rl = {name: hM.ranLevels[name] for name in hM.rLNames} if hM.nr else None
    hM1 = Hmsc(Y=hM.Y[train], X=hM.X[train], Tr=hM.Tr, distr=hM.distr, C=hM.C,                   # :92
               studyDesign=sd, ranLevels=rl, covNames=list(hM.covNames), spNames=list(hM.spNames))
    # :93-94 calls setPriors(hM1, V0 = hM$V0, ...) without assigning its result, so the refit
    # keeps Hmsc()'s default priors (the random levels' priors travel with ranLevels); the
    # scalings are the full model's (:95-116)
    hM1.YScalePar = hM.YScalePar
    hM1.YScaled = (hM1.Y - hM1.YScalePar[0][None, :]) / hM1.YScalePar[1][None, :]
    hM1.XInterceptInd = hM.XInterceptInd
    hM1.XScalePar = hM.XScalePar
    hM1.XScaled = (np.asarray(hM1.X, dtype=np.float64) - hM1.XScalePar[0][None, :]) / hM1.XScalePar[1][None, :]
    hM1.TrInterceptInd = hM.TrInterceptInd
    hM1.TrScalePar = hM.TrScalePar
    hM1.TrScaled = (np.asarray(hM1.Tr, dtype=np.float64) - hM1.TrScalePar[0][None, :]) / hM1.TrScalePar[1][None, :]
    return hM1


def cv_fold_seed(seed, k):
    """Seed of fold k's refit: R draws the refit's chain seeds from its global RNG; here a given
    predict seed fixes them per fold (None: fresh seeds)."""
    return None if seed is None else int(np.random.default_rng([int(seed), int(k)]).integers(1, 2 ** 62))


def _cv_refit(hM, train, k, seed, nChains, updater, initPar, nParallel):
    """R/computePredictedValues.R:117: sampleMcmc of the fold model with the fitted run's
    samples / transient / thin / adaptNf."""
    from .sampler import sampleMcmc
    return sampleMcmc(_cv_fold_model(hM, train), samples=hM.samples, thin=hM.thin, transient=hM.transient,
                      nChains=nChains, adaptNf=getattr(hM, "adaptNf", None), updater=updater, initPar=initPar,
                      verbose=0, nParallel=nParallel, seed=cv_fold_seed(seed, k))


def _auc(y, p):
    """pROC::auc(levels=c(0,1), direction="<"): Mann-Whitney with average ranks for ties."""
    r = stats.rankdata(p)
    n1 = np.sum(y == 1)
    n0 = np.sum(y == 0)
    return (np.sum(r[y == 1]) - n1 * (n1 + 1) / 2) / (n1 * n0)


def evaluateModelFit(hM, predY):
    """R/evaluateModelFit.R: RMSE for all species; R2 (normal); AUC and TjurR2 (probit);
    SR2, O.AUC, O.TjurR2, O.RMSE, C.SR2, C.RMSE (Poisson)."""
    Y = np.asarray(hM.Y, dtype=np.float64)
    fam = hM.distr[:, 0]
    m = np.full((hM.ny, hM.ns), np.nan)
    with np.errstate(all="ignore"):
        pois = fam == 3
        if pois.any():
            m[:, pois] = np.nanmedian(predY[:, pois, :], axis=2)
        if (~pois).any():
            m[:, ~pois] = np.nanmean(predY[:, ~pois, :], axis=2)

    def rmse(Yc, P):
        return np.sqrt(np.nanmean((Yc - P) ** 2, axis=0))

    def r2(Yc, P, method="pearson"):
        out = np.full(Yc.shape[1], np.nan)
        for j in range(Yc.shape[1]):
            ok = ~np.isnan(Yc[:, j]) & ~np.isnan(P[:, j])
            if ok.sum() > 1:
                if method == "spearman":
                    co = stats.spearmanr(Yc[ok, j], P[ok, j])[0]
                else:
                    co = np.corrcoef(Yc[ok, j], P[ok, j])[0, 1]
                out[j] = np.sign(co) * co ** 2
        return out

    def auc(Yc, P):
        Yb = np.where(np.isnan(Yc), np.nan, (Yc > 0).astype(float))
        out = np.full(Yc.shape[1], np.nan)
        for j in range(Yc.shape[1]):
            sel = ~np.isnan(Yb[:, j])
            if len(np.unique(Yb[sel, j])) == 2:
                out[j] = _auc(Yb[sel, j], P[sel, j])
        return out

    def tjur(Yc, P):
        return np.array([np.mean(P[Yc[:, j] == 1, j]) - np.mean(P[Yc[:, j] == 0, j]) for j in range(Yc.shape[1])])

    res = dict(RMSE=rmse(Y, m))
    sel = fam == 1
    if sel.any():
        res["R2"] = np.full(hM.ns, np.nan)
        res["R2"][sel] = r2(Y[:, sel], m[:, sel])
    sel = fam == 2
    if sel.any():
        res["AUC"] = np.full(hM.ns, np.nan)
        res["TjurR2"] = np.full(hM.ns, np.nan)
        res["AUC"][sel] = auc(Y[:, sel], m[:, sel])
        res["TjurR2"][sel] = tjur(Y[:, sel], m[:, sel])
    sel = fam == 3
    if sel.any():
        Ys, ms = Y[:, sel], m[:, sel]
        res["SR2"] = np.full(hM.ns, np.nan)
        res["SR2"][sel] = r2(Ys, ms, method="spearman")
        Yo = np.where(np.isnan(Ys), np.nan, (Ys > 0).astype(float))
        pO = np.nanmean((predY[:, sel, :] > 0).astype(float), axis=2)
        for key, val in (("O.AUC", auc(Yo, pO)), ("O.TjurR2", tjur(Yo, pO)), ("O.RMSE", rmse(Yo, pO))):
            res[key] = np.full(hM.ns, np.nan)
            res[key][sel] = val
        with np.errstate(all="ignore"):
            mc = ms / pO                                    # mPredCY = mPredY / mPredO  (:150)
        Yc = np.where(Ys == 0, np.nan, Ys)                  # CY[CY == 0] = NA  (:151-152)
        res["C.SR2"] = np.full(hM.ns, np.nan)
        res["C.RMSE"] = np.full(hM.ns, np.nan)
        res["C.SR2"][sel] = r2(Yc, mc, method="spearman")
        res["C.RMSE"][sel] = rmse(Yc, mc)
    return res
