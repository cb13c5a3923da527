"""computeDataParameters — R/computeDataParameters.R:16-205 (host precompute, once per fit).

Phylogeny grid over rhopw (Qg/iQg/RQg/detQg, :19-39; identity when C is NULL, :40-45)
and the spatial "Full" grid over alphapw (Wg/iWg/RiWg/detWg, :53-81).  Arrays are
returned in R's layout ([ns, ns, grid] etc.).  NNGP / GPP grids belong to the
spatial 'next' row.
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


def spatialDataParameters(hM):
    """rLPar of R/computeDataParameters.R:47-81 (spatial 'Full' levels; {} for the others)."""
    rLPar = []
    for r, rl in enumerate(hM.rL or []):
        if not rl.sDim:
            rLPar.append({})
            continue
        method = rl.spatialMethod
        if method != "Full":
            raise NotImplementedError(f"spatial method {method} is a 'next' row (SURVEY.md §8 f2)")
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


def _level_order(hM, r, rl):
    """Rows of rl$s in levels(dfPi[,r]) order (R indexes s by unit names)."""
    names = rl["sNames"] if "sNames" in rl.names() and rl["sNames"] is not None else None
    levels = hM["dfPiLevels"][r] if "dfPiLevels" in hM.names() and hM["dfPiLevels"] is not None else None
    if names is None or levels is None:
        return np.arange(rl.s.shape[0] if rl.s is not None else rl.distMat.shape[0])
    pos = {str(n): k for k, n in enumerate(names)}
    return np.array([pos[str(lv)] for lv in levels])
