"""computeDataParameters — R/computeDataParameters.R:16-205 (host precompute, once per fit).

Phylogeny grid over rhopw (Qg/iQg/RQg/detQg, :19-39; identity when C is NULL, :40-45)
and the spatial grids over alphapw: "Full" (Wg/iWg/RiWg/detWg, :53-81), "NNGP"
(sparse Vecchia precision iWg = RiWg' RiWg, detWg, :82-136) and "GPP" (predictive-process
idDg/idDW12g/Fg/iFg/detDg, :138-194).  Arrays are returned in R's layout ([np, np, grid]
etc.).  For NNGP and GPP the dense precision of the level's prior is returned beside R's
own fields as iWg / RiWg / detWg (RiWg' RiWg = iWg): the device runs every spatial method
through the one dense (np nf)^2 updateEta / updateAlpha path (DESIGN.md §4 "Spatial
levels"), and for GPP

    iW = diag(idD) - idDW12 iF idDW12' = W^-1  (Woodbury on W = D + W12 iW22 W12'),
    det W = detD,

computed as iW = RiW' RiW with RiW = chol(W)^-1 (lower triangular, like NNGP's factor),

which is exactly the prior R/updateEta.R:148-196 and R/updateAlpha.R:35-75 condition on.
"""
import numpy as np
from scipy.linalg import solve_triangular


def _chol_upper(A):
    return np.linalg.cholesky(A).T


def _chol2inv(R):
    Ri = solve_triangular(R, np.eye(R.shape[0]), lower=False)
    return Ri @ Ri.T


def computeDataParameters(hM):
    par = {}
    ns = hM.ns
    if hM.C is not None:
        rhopw = hM.rhopw
        g = rhopw.shape[0]
        Qg = np.empty((ns, ns, g))
        iQg = np.empty((ns, ns, g))
        RQg = np.empty((ns, ns, g))
        detQg = np.empty(g)
        iC = _chol2inv(_chol_upper(hM.C)) if np.any(rhopw[:, 0] < 0) else None
        for k in range(g):
            rho = rhopw[k, 0]
            rhoC = rho * hM.C if rho >= 0 else (-rho) * iC
            Q = rhoC + (1 - abs(rho)) * np.eye(ns)
            RQ = _chol_upper(Q)
            Qg[:, :, k], iQg[:, :, k], RQg[:, :, k] = Q, _chol2inv(RQ), RQ
            detQg[k] = 2 * np.sum(np.log(np.diag(RQ)))
    else:
        Qg = np.eye(ns)[:, :, None]
        iQg = np.eye(ns)[:, :, None]
        RQg = np.eye(ns)[:, :, None]
        detQg = np.array([0.0])
    par.update(Qg=Qg, iQg=iQg, RQg=RQg, detQg=detQg)
    par["rLPar"] = spatialDataParameters(hM)
    return par


def spatialDataParameters(hM, skip=None, gpp_dense=True):
    """rLPar of R/computeDataParameters.R:47-196 ({} for non-spatial levels and for levels
    with skip[r] true).  gpp_dense=False leaves out the dense np^2 iWg / RiWg of GPP levels
    (the device samples them in R's low-rank form from idDg / idDW12g / Fg / iFg)."""
    rLPar = []
    for r, rl in enumerate(hM.rL or []):
        if not rl.sDim or (skip is not None and skip[r]):
            rLPar.append({})
            continue
        method = rl.spatialMethod
        if method == "NNGP":
            rLPar.append(_nngp_grid(hM, r, rl))
            continue
        if method == "GPP":
            rLPar.append(_gpp_grid(hM, r, rl, dense=gpp_dense))
            continue
        if method != "Full":
            raise ValueError(f"computeDataParameters: unknown spatialMethod {method!r}")
        if rl.distMat is None:
            s = rl.s[_level_order(hM, r, rl)]
            d = np.sqrt(((s[:, None, :] - s[None, :, :]) ** 2).sum(-1))
        else:
            idx = _level_order(hM, r, rl)
            d = rl.distMat[np.ix_(idx, idx)]
        alphapw = rl.alphapw
        npr = d.shape[0]
        G = alphapw.shape[0]
        Wg = np.empty((npr, npr, G))
        iWg = np.empty_like(Wg)
        RiWg = np.empty_like(Wg)
        detWg = np.empty(G)
        for k in range(G):
            a = alphapw[k, 0]
            W = np.eye(npr) if a == 0 else np.exp(-d / a)
            RW = _chol_upper(W)
            iW = _chol2inv(RW)
            Wg[:, :, k], iWg[:, :, k], RiWg[:, :, k] = W, iW, _chol_upper(iW)
            detWg[k] = 2 * np.sum(np.log(np.diag(RW)))
        rLPar.append(dict(Wg=Wg, iWg=iWg, RiWg=RiWg, detWg=detWg))
    return rLPar


def knn_index(s, k):
    """FNN::get.knn(s, k)$nn.index (exact Euclidean k nearest neighbours, self excluded),
    0-based; ties broken by the lower index."""
    n = s.shape[0]
    if not 0 < k < n:
        raise ValueError("NNGP: nNeighbours must be positive and smaller than the number of units")
    d = ((s[:, None, :] - s[None, :, :]) ** 2).sum(-1)
    d[np.arange(n), np.arange(n)] = np.inf
    return np.argsort(d, axis=1, kind="stable")[:, :k]


def _nngp_grid(hM, r, rl):
    """R/computeDataParameters.R:82-136: Vecchia factor RiW = diag(D^-1/2)(I - A) over the
    nNeighbours (default 10) nearest earlier units, iW = RiW' RiW, detW = sum(log D)."""
    if rl.distMat is not None:
        raise ValueError("computeDataParameters: Nearest neighbours not available for distance matrices")
    k = int(rl.nNeighbours) if rl.nNeighbours is not None else 10
    s = np.asarray(rl.s, dtype=np.float64)[_level_order(hM, r, rl)]
    npr = s.shape[0]
    indNN = np.sort(knn_index(s, k), axis=1)                       # :93-94
    prev = [indNN[i][indNN[i] < i] for i in range(npr)]          # :97-104
    alphapw = rl.alphapw
    G = alphapw.shape[0]
    iWg = np.empty((npr, npr, G))
    RiWg = np.empty_like(iWg)
    detWg = np.empty(G)
    for g in range(G):
        a = alphapw[g, 0]
        if a == 0:                                                # :107-110
            RiW = np.eye(npr)
            detW = 0.0
        else:
            D = np.ones(npr)
            A = np.zeros((npr, npr))
            for i in range(1, npr):                               # :115-123
                ind = prev[i]
                if ind.size == 0:
                    continue
                pts = s[np.r_[ind, i]]
                Kp = np.exp(-np.sqrt(((pts[:, None, :] - pts[None, :, :]) ** 2).sum(-1)) / a)
                v = np.linalg.solve(Kp[:-1, :-1], Kp[:-1, -1])
                D[i] = Kp[-1, -1] - Kp[-1, :-1] @ v
                A[i, ind] = v
            RiW = (D ** -0.5)[:, None] * (np.eye(npr) - A)        # :124-127
            detW = float(np.sum(np.log(D)))                       # :129
        iWg[:, :, g] = RiW.T @ RiW                                 # :128
        RiWg[:, :, g] = RiW
        detWg[g] = detW
    return dict(iWg=iWg, RiWg=RiWg, detWg=detWg)


def _gpp_grid(hM, r, rl, dense=True):
    """R/computeDataParameters.R:138-194 (predictive process over the knots sKnot), plus
    (dense=True) the dense precision iWg / RiWg / detWg of the same prior (module docstring;
    the device samples GPP levels from the low-rank arrays and needs none of it)."""
    if rl.distMat is not None:
        raise ValueError("computeDataParameters: predictive gaussian process not available for distance matrices")
    sKnot = rl["sKnot"] if "sKnot" in rl.names() else None
    if sKnot is None:
        raise ValueError("computeDataParameters: GPP level needs sKnot (see constructKnots)")
    sKnot = np.asarray(sKnot, dtype=np.float64)
    s = np.asarray(rl.s, dtype=np.float64)[_level_order(hM, r, rl)]
    npr, nK = s.shape[0], sKnot.shape[0]
    di12 = np.sqrt(((s[:, None, :] - sKnot[None, :, :]) ** 2).sum(-1))     # :146-153
    di22 = np.sqrt(((sKnot[:, None, :] - sKnot[None, :, :]) ** 2).sum(-1))  # :155
    alphapw = rl.alphapw
    G = alphapw.shape[0]
    idDg = np.empty((npr, G))
    idDW12g = np.empty((npr, nK, G))
    Fg = np.empty((nK, nK, G))
    iFg = np.empty((nK, nK, G))
    detDg = np.empty(G)
    iWg = np.empty((npr, npr, G)) if dense else None
    RiWg = np.empty_like(iWg) if dense else None
    for g in range(G):
        a = alphapw[g, 0]
        if a == 0:
            W22, W12 = np.eye(nK), np.zeros((npr, nK))
        else:
            W22, W12 = np.exp(-di22 / a), np.exp(-di12 / a)
        iW22 = np.linalg.inv(W22)                                   # :172
        dD = 1.0 - np.einsum("ik,kl,il->i", W12, iW22, W12)       # :173-174
        liW22 = np.linalg.cholesky(iW22)                            # :176
        idD = 1.0 / dD
        idDW12 = idD[:, None] * W12                                 # :179-180
        F = W22 + W12.T @ idDW12                                    # :181
        iF = np.linalg.inv(F)
        tmp2 = W12 @ liW22
        DS = tmp2.T @ (idD[:, None] * tmp2) + np.eye(nK)            # :184
        detD = float(np.sum(np.log(dD)) + 2 * np.sum(np.log(np.diag(np.linalg.cholesky(DS)))))
        idDg[:, g], idDW12g[:, :, g], Fg[:, :, g], iFg[:, :, g], detDg[g] = idD, idDW12, F, iF, detD
        if not dense:
            continue
        # dense precision through W itself (unit diagonal): W = L L', RiW = L^-1 (lower),
        # iW = RiW' RiW.  Equal to diag(idD) - idDW12 iF idDW12' but without its cancellation
        # when a unit sits on a knot (dD -> 0, idD -> inf while W stays well conditioned)
        W = W12 @ iW22 @ W12.T
        W = 0.5 * (W + W.T)
        W[np.diag_indices(npr)] = 1.0
        try:
            LW = np.linalg.cholesky(W)
        except np.linalg.LinAlgError:
            raise ValueError(f"computeDataParameters, GPP: W at alphapw[{g + 1}] is not positive definite") from None
        RiW = solve_triangular(LW, np.eye(npr), lower=True)
        RiWg[:, :, g] = RiW
        iWg[:, :, g] = RiW.T @ RiW
    return dict(idDg=idDg, idDW12g=idDW12g, Fg=Fg, iFg=iFg, detDg=detDg,
                iWg=iWg, RiWg=RiWg, detWg=detDg.copy())


def constructKnots(sData, nKnots=None, knotDist=None, minKnotDist=None):
    """R/constructKnots.R:26-49: regular grid over the bounding box of sData (first axis
    fastest, as expand.grid), keeping knots closer than minKnotDist (default 2 knotDist) to
    the nearest data point."""
    if nKnots is not None and knotDist is not None:
        raise ValueError("constructKnots: nKnots and knotDist cannot both be specified")
    s = np.asarray(sData, dtype=np.float64)
    mins, maxs = s.min(axis=0), s.max(axis=0)
    if knotDist is None:
        knotDist = float(np.min(maxs - mins)) / (10 if nKnots is None else nKnots)
    axes = [np.arange(mins[d], maxs[d] + 1e-10 * max(1.0, abs(maxs[d])), knotDist) for d in range(s.shape[1])]
    mesh = np.meshgrid(*axes, indexing="ij")
    sKnot = np.column_stack([m.ravel(order="F") for m in mesh])
    dist = np.sqrt(((sKnot[:, None, :] - s[None, :, :]) ** 2).sum(-1)).min(axis=1)
    if minKnotDist is None:
        minKnotDist = 2 * knotDist
    return sKnot[dist < minKnotDist]


def _level_order(hM, r, rl):
    """Rows of rl$s in levels(dfPi[,r]) order (R indexes s by unit names,
    R/computeDataParameters.R:56,92,142); unnamed coordinates are taken in that order."""
    names = rl["sNames"] if "sNames" in rl.names() else None
    if names is None:
        return np.arange(rl.s.shape[0] if rl.s is not None else rl.distMat.shape[0])
    from .model import _factor_levels
    levels = _factor_levels(hM.dfPi[hM.rLNames[r]])
    pos = {str(n): k for k, n in enumerate(names)}
    missing = [lv for lv in levels if str(lv) not in pos]
    if missing:
        raise ValueError(f"spatial level {hM.rLNames[r]}: no coordinates for units {missing[:5]}")
    return np.array([pos[str(lv)] for lv in levels])
