"""Posterior output layout and diagnostics (host side).

* ``convertToCodaObject`` — R/convertToCodaObject.r:36-290: the parameter naming
  and vectorisation order of the reference's coda objects ("B[cov (C1), sp (S1)]",
  Beta as.vector covariate-fastest, Lambda as.vector(t(.)) species-fastest,
  Omega = crossprod(Lambda)), returned as ``{name: [chain arrays (samples, p)]}``
  plus ``{name: column names}``.
* ``effectiveSize`` — coda::effectiveSize (spectrum0.ar: AR order by AIC via Yule-Walker,
  R's ar.yw.default) on the device (post.hip), used for the Beta ESS/sec metric;
  ``gelman_diag`` — coda::gelman.diag(multivariate=FALSE) on the host (m x p numbers).
* ``computeVariancePartitioning``, ``computeAssociations``, ``getPostEstimate(.., "Omega")``
  — their loops over posterior samples on the device (post.hip); checkers in
  oracle/post_oracle.py.
* ``poolMcmcChains``, ``getPostEstimate``, ``computeWAIC`` — R/poolMcmcChains.R,
  R/getPostEstimate.R, R/computeWAIC.R:25-131 (normal and probit columns).
"""
import numpy as np
from scipy import stats
from scipy.special import log_ndtr

from . import _lib as L


def poolMcmcChains(postList, start=1, thin=1):
    out = []
    for chain in postList:
        out.extend(chain[start - 1::thin])
    return out


def convertToCodaObject(hM, start=1, spNamesNumbers=(True, True), covNamesNumbers=(True, True),
                        trNamesNumbers=(True, True), Beta=True, Gamma=True, V=True, Sigma=True, Rho=True,
                        Eta=True, Lambda=True, Alpha=True, Omega=True, Psi=True, Delta=True):
    """R/convertToCodaObject.r:36-290: per chain, one (samples, P) matrix per parameter and
    its column names (the coda mcmc.list layout)."""
    def nm(names, numbers, prefix):                                        # :54-92
        res = []
        for k, n in enumerate(names):
            parts = []
            if numbers[0]:
                parts.append(str(n))
            if numbers[1]:
                parts.append(f"({prefix}{k + 1})")
            res.append(" ".join(parts))
        return res

    sp = nm(hM.spNames, spNamesNumbers, "S")
    cov = nm(hM.covNames, covNamesNumbers, "C")
    tr = nm(hM.trNames, trNamesNumbers, "T")
    out, cols = {}, {}
    chains = [c[start - 1:] for c in hM.postList]
    if Beta:                                                                # :131-135
        out["Beta"] = [np.stack([s["Beta"].reshape(-1, order="F") for s in c]) for c in chains]
        cols["Beta"] = [f"B[{cv}, {s}]" for s in sp for cv in cov]
    if Gamma:
        out["Gamma"] = [np.stack([s["Gamma"].reshape(-1, order="F") for s in c]) for c in chains]
        cols["Gamma"] = [f"G[{cv}, {t}]" for t in tr for cv in cov]
    if V:
        out["V"] = [np.stack([s["V"].reshape(-1, order="F") for s in c]) for c in chains]
        cols["V"] = [f"V[{c1}, {c2}]" for c2 in cov for c1 in cov]
    if Sigma:
        out["Sigma"] = [np.stack([np.asarray(s["sigma"]) for s in c]) for c in chains]
        cols["Sigma"] = [f"Sig[{s}]" for s in sp]
    if Rho and hM.C is not None:
        out["Rho"] = [np.array([[s["rho"]] for s in c]) for c in chains]
        cols["Rho"] = ["Rho"]
    for r in range(hM.nr):
        nfMax = max(c[0]["Lambda"][r].shape[0] for c in chains)
        if Eta:                                                             # :171-176
            units = list(_levels(hM.dfPi[hM.rLNames[r]])) if hM.dfPi is not None else \
                [str(q + 1) for q in range(int(hM.np[r]))]
            out.setdefault("Eta", []).append(
                [np.stack([_pad_cols(s["Eta"][r], nfMax).reshape(-1, order="F") for s in c]) for c in chains])
            cols.setdefault("Eta", []).append(
                [f"Eta{r + 1}[{u}, factor{h + 1}]" for h in range(nfMax) for u in units])
        if Lambda:                                                          # :178-183 as.vector(t(Lambda))
            out.setdefault("Lambda", []).append(
                [np.stack([_pad_rows(s["Lambda"][r], nfMax).T.reshape(-1, order="F") for s in c]) for c in chains])
            cols.setdefault("Lambda", []).append(
                [f"Lambda{r + 1}[{s}, factor{h + 1}]" for h in range(nfMax) for s in sp])
        if Omega:                                                           # :184-188 crossprod(Lambda)
            out.setdefault("Omega", []).append(
                [np.stack([(s["Lambda"][r].T @ s["Lambda"][r]).reshape(-1, order="F") for s in c]) for c in chains])
            cols.setdefault("Omega", []).append([f"Omega{r + 1}[{a}, {b}]" for b in sp for a in sp])
        if Alpha:                                                           # :189-195 alphapw[Alpha, 1], 0-padded
            apw = np.asarray(hM.rL[r].alphapw)[:, 0] if hM.rL[r].sDim else None
            rows = []
            for c in chains:
                m = np.zeros((len(c), nfMax))
                for k, smp in enumerate(c):
                    a = np.asarray(smp["Alpha"][r], dtype=np.int64).ravel()
                    m[k, :len(a)] = apw[a - 1] if apw is not None else 0.0
                rows.append(m)
            out.setdefault("Alpha", []).append(rows)
            cols.setdefault("Alpha", []).append([f"Alpha{r + 1}[factor{h + 1}]" for h in range(nfMax)])
        if Psi:                                                             # :197-203
            out.setdefault("Psi", []).append(
                [np.stack([_pad_rows(s["Psi"][r], nfMax).T.reshape(-1, order="F") for s in c]) for c in chains])
            cols.setdefault("Psi", []).append([f"Psi{r + 1}[{s}, factor{h + 1}]" for h in range(nfMax) for s in sp])
        if Delta:                                                           # :205-210 0-padded
            out.setdefault("Delta", []).append(
                [np.stack([_pad_rows(s["Delta"][r], nfMax, fill=0.0).reshape(-1) for s in c]) for c in chains])
            cols.setdefault("Delta", []).append([f"Delta{r + 1}[factor{h + 1}]" for h in range(nfMax)])
    return out, cols


def _levels(col):
    """levels(hM$dfPi[, r]): the rule hM$Pi was built with (model._factor_levels)."""
    from .model import _factor_levels
    return [str(v) for v in _factor_levels(col)]


def _pad_rows(a, n, fill=0.0):
    a = np.atleast_2d(a)
    if a.shape[0] >= n:
        return a
    return np.vstack([a, np.full((n - a.shape[0], a.shape[1]), fill)])


def _pad_cols(a, n):
    if a.shape[1] >= n:
        return a
    return np.hstack([a, np.zeros((a.shape[0], n - a.shape[1]))])


# ---------------------------------------------------------------------------
# coda::effectiveSize on the device (hmsc_effective_size, post.hip; the numpy restatement
# of spectrum0.ar with R's ar.yw.default is the checker in oracle/post_oracle.py)
# ---------------------------------------------------------------------------
def _device():
    """The device post-processing runs on: HMSC_POST_DEVICE, else 0."""
    import os
    return int(os.environ.get("HMSC_POST_DEVICE", "0"))


def spectrum0_ar(x, device=None):
    """coda::spectrum0.ar for every column of x (n, p): (spec, AR order), on the device.
    spec follows from the ESS: spec = n var / ESS (0 for a constant column)."""
    x = np.asarray(x, dtype=np.float64)
    if x.ndim == 1:
        x = x[:, None]
    ess, order = _ess_device(x, device)
    var = x.var(axis=0, ddof=1)
    with np.errstate(divide="ignore", invalid="ignore"):
        spec = np.where(ess == 0, 0.0, x.shape[0] * var / ess)
    return spec, order


def _ess_device(x, device=None):
    n, p = x.shape
    xf = np.asfortranarray(x)
    ess = np.zeros(p)
    order = np.zeros(p, dtype=np.int32)
    L.check(L.lib().hmsc_effective_size(_device() if device is None else int(device), n, p,
                                        xf.ctypes.data_as(L.dp), L.fptr(ess), L.iptr(order)))
    return ess, order


def effectiveSize(chains, device=None):
    """coda::effectiveSize for an mcmc.list: per-chain n var / spec0 (device), summed over chains."""
    if isinstance(chains, np.ndarray):
        chains = [chains]
    total = 0.0
    for x in chains:
        x = np.asarray(x, dtype=np.float64)
        if x.ndim == 1:
            x = x[:, None]
        total = total + _ess_device(x, device)[0]
    return total


def gelman_diag(chains, confidence=0.95):
    """coda::gelman.diag(multivariate=FALSE): point estimate and upper CI of the PSRF."""
    X = np.stack([np.asarray(c, dtype=np.float64) for c in chains])      # (m, n, p)
    m, n, p = X.shape
    xbar = X.mean(axis=1)
    s2 = X.var(axis=1, ddof=1)
    W = s2.mean(axis=0)
    B = n * xbar.var(axis=0, ddof=1)
    muhat = xbar.mean(axis=0)
    var_w = s2.var(axis=0, ddof=1) / m
    var_b = (2 * B ** 2) / (m - 1)
    cov = lambda a, b: ((a - a.mean(0)) * (b - b.mean(0))).sum(0) / (m - 1)   # noqa: E731
    cov_wb = (n / m) * (cov(s2, xbar ** 2) - 2 * muhat * cov(s2, xbar))
    V = (n - 1) * W / n + (1 + 1 / m) * B / n
    var_V = ((n - 1) ** 2 * var_w + (1 + 1 / m) ** 2 * var_b + 2 * (n - 1) * (1 + 1 / m) * cov_wb) / n ** 2
    with np.errstate(divide="ignore", invalid="ignore"):
        df_V = 2 * V ** 2 / var_V
        df_adj = (df_V + 3) / (df_V + 1)
        W_df = 2 * W ** 2 / var_w
        R2_fixed = (n - 1) / n
        R2_random = (1 + 1 / m) * (1 / n) * (B / W)
        point = np.sqrt(df_adj * (R2_fixed + R2_random))
        upper = np.sqrt(df_adj * (R2_fixed + stats.f.ppf((1 + confidence) / 2, m - 1, W_df) * R2_random))
    return point, upper


def getPostEstimate(hM, parName, r=1, x=None, q=(), chainIndex=None, start=1):
    """R/getPostEstimate.R: posterior mean and support (P(>0)) of Beta/Gamma/V/Sigma/Omega."""
    postList = hM.postList if chainIndex is None else [hM.postList[i] for i in chainIndex]
    post = poolMcmcChains(postList, start=start)
    if parName == "Omega" and not q:   # mean and supports summed on the device (hmsc_post_omega)
        o = _omega_device(post, r - 1, hM.ns)
        return dict(mean=o["mean_omega"], support=o["support"], supportNeg=o["support_neg"])
    if parName == "Omega":
        vals = np.stack([s["Lambda"][r - 1].T @ s["Lambda"][r - 1] for s in post])
    elif parName == "Sigma":
        vals = np.stack([np.asarray(s["sigma"]) for s in post])
    else:
        vals = np.stack([np.asarray(s[parName]) for s in post])
    res = dict(mean=vals.mean(axis=0), support=(vals > 0).mean(axis=0), supportNeg=(vals < 0).mean(axis=0))
    if q:
        res["q"] = np.quantile(vals, q, axis=0)
    return res


def computeWAIC(hM, ghN=11):
    """R/computeWAIC.R:25-131.  Poisson columns integrate the lognormal intensity with
    ghN-point Gauss-Hermite quadrature (:108-118); ``dpois(Y, exp(gX))`` there recycles the
    whole ny x ns Y column-major against the ny x cN x ghN node array, which is reproduced
    as written (it only equals the per-cell likelihood when every species is Poisson)."""
    post = poolMcmcChains(hM.postList)
    Y, X, Pi = hM.Y, hM.X, hM.Pi
    fam = hM.distr[:, 0]
    normal, probit, pois = fam == 1, fam == 2, fam == 3
    if pois.any():
        gx, gw = np.polynomial.hermite.hermgauss(ghN)   # statmod::gauss.quad(kind="hermite")
        cN = int(pois.sum())
        ii, cc, gg = np.meshgrid(np.arange(hM.ny), np.arange(cN), np.arange(ghN), indexing="ij")
        Yrec = Y.ravel(order="F")[(ii + hM.ny * cc + hM.ny * cN * gg) % Y.size]
    na = np.isnan(Y)
    vals = []
    from .sampler import level_lran, x_unit_order
    xs = [x_unit_order(hM, r, rl) if rl.xDim else None for r, rl in enumerate(hM.rL or [])]
    for s in post:
        E = X @ s["Beta"]
        for r in range(hM.nr):
            E = E + level_lran(s["Eta"][r], s["Lambda"][r], Pi[:, r] - 1, xs[r])
        std = np.asarray(s["sigma"]) ** -0.5
        Lr = np.zeros(hM.ny)
        if normal.any():
            t = stats.norm.logpdf(Y[:, normal], loc=E[:, normal], scale=std[normal][None, :])
            t[na[:, normal]] = 0
            Lr += t.sum(axis=1)
        if probit.any():
            pz0 = log_ndtr(-E[:, probit])
            pz1 = log_ndtr(E[:, probit])
            Yp = Y[:, probit]
            t = pz1 * Yp + pz0 * (1 - Yp)
            t[na[:, probit]] = 0
            Lr += t.sum(axis=1)
        if pois.any():
            gX = E[:, pois][:, :, None] + np.sqrt(2.0) * gx[None, None, :] * std[pois][None, :, None]
            like = stats.poisson.pmf(Yrec, np.exp(gX))
            t = np.log(np.sum(like * gw[None, None, :], axis=2) / np.sqrt(np.pi))
            t[na[:, pois]] = 0
            Lr += t.sum(axis=1)
        vals.append(Lr)
    val = np.stack(vals)
    Bl = -np.log(np.mean(np.exp(val), axis=0))
    Vv = val.var(axis=0, ddof=1)
    return float(np.mean(Bl + Vv))


def computeVariancePartitioning(hM, group=None, groupnames=None, start=1, device=None):
    """R/computeVariancePartitioning.R:37-204 (X a matrix, na.ignore=FALSE), the loop over
    samples on the device (hmsc_variance_partitioning, post.hip).

    Reproduces the reference's loop ``for (i in 1:hM$samples)`` over the *pooled* list
    (:125), i.e. with nChains > 1 only the first chain's samples enter (SURVEY.md
    Appendix B quirk 4).  Returns dict(vals (ngroups+nr, ns), R2T=dict(Beta, Y), group,
    groupnames, rownames).
    """
    ns, nc, nr = hM.ns, hM.nc, hM.nr
    if group is None:                                                      # :42-51
        if nc > 1:
            group = np.r_[1, np.arange(1, nc)]
            groupnames = list(hM.covNames[1:nc])
        else:
            group = np.array([1])
            groupnames = [hM.covNames[0]]
    group = np.asarray(group)
    ngroups = int(group.max())
    X = np.asarray(hM.X, dtype=np.float64)
    Tr = np.asarray(hM.Tr, dtype=np.float64)
    cM = np.cov(X, rowvar=False).reshape(nc, nc)                           # :66
    post = poolMcmcChains(hM.postList, start=start)[:hM.samples]            # :125 (quirk above)
    S = len(post)
    keep = []
    a = L.hmsc_vp_args()
    a.device = _default_device_of(device)
    a.ny, a.ns, a.nc, a.nt, a.S, a.ngroups, a.nr = hM.ny, ns, nc, Tr.shape[1], S, ngroups, nr
    a.group = L.colmajor_ptr(group.astype(np.int32), keep, np.int32)
    a.X = L.colmajor_ptr(X, keep)
    a.Tr = L.colmajor_ptr(Tr, keep)
    a.cM = L.colmajor_ptr(cM, keep)
    a.Beta = L.fptr(_flat(keep, [np.asarray(s_["Beta"], dtype=np.float64) for s_ in post]))
    a.Gamma = L.fptr(_flat(keep, [np.asarray(s_["Gamma"], dtype=np.float64) for s_ in post]))
    nfs = np.zeros((max(1, nr), S), dtype=np.int32)
    for r in range(nr):
        nfm = max(int(np.asarray(s_["Lambda"][r]).shape[0]) for s_ in post)
        lam = np.zeros((S, nfm, ns))
        for k, s_ in enumerate(post):
            l_ = np.asarray(s_["Lambda"][r], dtype=np.float64)
            nfs[r, k] = l_.shape[0]
            lam[k, :l_.shape[0]] = l_
        a.nfmax[r] = nfm
        a.Lambda[r] = L.fptr(_flat(keep, list(lam)))
    a.nf = L.iptr(_keep(keep, np.ascontiguousarray(nfs.ravel())))
    slot = nc + 1 + ns * (1 + nr + ngroups)
    out = np.zeros(slot)
    L.check(L.lib().hmsc_variance_partitioning(L.C.byref(a), L.fptr(out)))
    R2T_Beta, R2T_Y = out[:nc], float(out[nc])
    fixed = out[nc + 1:nc + 1 + ns]
    random = out[nc + 1 + ns:nc + 1 + ns * (1 + nr)].reshape(nr, ns).T
    fixedsplit = out[nc + 1 + ns * (1 + nr):].reshape(ngroups, ns).T
    vals = np.zeros((ngroups + nr, ns))                                    # :180-187
    for g in range(ngroups):
        vals[g] = fixed * fixedsplit[:, g]
    for r in range(nr):
        vals[ngroups + r] = random[:, r]
    rl = list(getattr(hM, "rLNames", None) or [f"level{r + 1}" for r in range(nr)])
    return dict(vals=vals, R2T=dict(Beta=R2T_Beta, Y=R2T_Y), group=group, groupnames=groupnames,
                rownames=list(groupnames) + [f"Random: {n}" for n in rl])


def _keep(keep, arr):
    keep.append(arr)
    return arr


def _flat(keep, mats):
    """Samples stacked as consecutive column-major matrices (the C side's S x (m x n))."""
    return _keep(keep, np.ascontiguousarray(np.concatenate([np.asarray(m_).ravel(order="F") for m_ in mats])))


def _default_device_of(device):
    return _device() if device is None else int(device)


def computeAssociations(hM, start=1, thin=1, device=None):
    """R/computeAssociations.R: per random level, dict(mean, support) of
    cov2cor(crossprod(Lambda)) over the pooled samples, on the device (hmsc_post_omega)."""
    post = poolMcmcChains(hM.postList, start=start, thin=thin)
    out = []
    for r in range(hM.nr):
        res = _omega_device(post, r, hM.ns, device)
        out.append(dict(mean=res["mean_cor"], support=res["support"]))
    return out


def _omega_device(post, r, ns, device=None):
    S = len(post)
    nfm = max(int(np.asarray(s_["Lambda"][r]).shape[0]) for s_ in post)
    lam = np.zeros((S, ns, nfm))   # C order (S, ns, nfm) = each sample nfm x ns column-major
    nf = np.zeros(S, dtype=np.int32)
    for k, s_ in enumerate(post):
        l_ = np.asarray(s_["Lambda"][r], dtype=np.float64)
        nf[k] = l_.shape[0]
        lam[k, :, :l_.shape[0]] = l_.T
    outs = {k: np.zeros((ns, ns), order="F") for k in ("mean_cor", "support", "support_neg", "mean_omega")}
    L.check(L.lib().hmsc_post_omega(_default_device_of(device), S, ns, nfm, L.iptr(nf), L.fptr(lam),
                                    *[outs[k].ctypes.data_as(L.dp) for k in ("mean_cor", "support", "support_neg",
                                                                             "mean_omega")]))
    return outs
