"""Posterior output layout and diagnostics (host side).

* ``convertToCodaObject`` — R/convertToCodaObject.r:36-290: the parameter naming
  and vectorisation order of the reference's coda objects ("B[cov (C1), sp (S1)]",
  Beta as.vector covariate-fastest, Lambda as.vector(t(.)) species-fastest,
  Omega = crossprod(Lambda)), returned as ``{name: [chain arrays (samples, p)]}``
  plus ``{name: column names}``.
* ``effectiveSize`` / ``gelman_diag`` — restatements of coda::effectiveSize
  (spectrum0.ar: AR order by AIC via Yule-Walker, R's ar.yw.default) and
  coda::gelman.diag(multivariate=FALSE), used for the Beta ESS/sec metric.
* ``poolMcmcChains``, ``getPostEstimate``, ``computeWAIC`` — R/poolMcmcChains.R,
  R/getPostEstimate.R, R/computeWAIC.R:25-131 (normal and probit columns).
"""
import numpy as np
from scipy import stats
from scipy.special import log_ndtr


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
# coda::effectiveSize restated (spectrum0.ar with R's ar.yw.default)
# ---------------------------------------------------------------------------
def spectrum0_ar(x):
    """Spectral density at zero for every column of x (n, p) — coda::spectrum0.ar."""
    x = np.asarray(x, dtype=np.float64)
    if x.ndim == 1:
        x = x[:, None]
    n, p = x.shape
    z = np.arange(1, n + 1, dtype=np.float64)
    zc = z - z.mean()
    xc = x - x.mean(axis=0)
    beta = (zc @ xc) / (zc @ zc)
    resid = xc - np.outer(zc, beta)
    rsd = resid.std(axis=0, ddof=1)
    scale = np.maximum(np.abs(x).max(axis=0), 1e-300)
    const = rsd <= 1.5e-8 * scale                                          # all.equal(sd(resid), 0)
    order_max = int(min(n - 1, np.floor(10 * np.log10(n))))
    # autocovariances with denominator n (acf type="covariance", demean=TRUE)
    r = np.empty((order_max + 1, p))
    for k in range(order_max + 1):
        r[k] = np.sum(xc[: n - k] * xc[k:], axis=0) / n
    r0 = np.where(r[0] > 0, r[0], 1.0)
    # Levinson-Durbin (R's eureka) for all orders
    vars_ = np.empty((order_max + 1, p))
    vars_[0] = r0
    coefs = np.zeros((order_max + 1, order_max + 1, p))
    a = np.zeros((order_max + 1, p))
    v = r0.copy()
    for m in range(1, order_max + 1):
        acc = r[m] - np.sum(a[1:m] * r[m - 1:0:-1], axis=0) if m > 1 else r[m].copy()
        k = acc / v
        a_new = a.copy()
        a_new[m] = k
        if m > 1:
            a_new[1:m] = a[1:m] - k * a[m - 1:0:-1]
        a = a_new
        v = v * (1 - k * k)
        vars_[m] = v
        coefs[m, 1:m + 1] = a[1:m + 1]
    with np.errstate(divide="ignore", invalid="ignore"):
        xaic = n * np.log(vars_) + 2 * np.arange(order_max + 1)[:, None] + 2.0
    order = np.argmin(xaic, axis=0)
    cols = np.arange(p)
    var_pred = vars_[order, cols] * n / (n - (order + 1))
    ar_sum = np.array([coefs[order[j], 1:order[j] + 1, j].sum() for j in range(p)])
    spec = var_pred / (1 - ar_sum) ** 2
    spec[const] = 0.0
    return spec, order


def effectiveSize(chains):
    """coda::effectiveSize for an mcmc.list: per-chain n*var/spec0, summed over chains."""
    if isinstance(chains, np.ndarray):
        chains = [chains]
    total = 0.0
    for x in chains:
        x = np.asarray(x, dtype=np.float64)
        if x.ndim == 1:
            x = x[:, None]
        spec, _ = spectrum0_ar(x)
        var = x.var(axis=0, ddof=1)
        with np.errstate(divide="ignore", invalid="ignore"):
            ess = np.where(spec == 0, 0.0, x.shape[0] * var / spec)
        total = total + ess
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
    for s in post:
        E = X @ s["Beta"]
        for r in range(hM.nr):
            E = E + s["Eta"][r][Pi[:, r] - 1] @ s["Lambda"][r]
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


def computeVariancePartitioning(hM, group=None, groupnames=None, start=1):
    """R/computeVariancePartitioning.R:37-204 (X a matrix, na.ignore=FALSE).

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
    X, Tr = hM.X, hM.Tr
    cM = np.cov(X, rowvar=False).reshape(nc, nc)                           # :66
    post = poolMcmcChains(hM.postList, start=start)
    S = hM.samples
    fixed = np.zeros(ns)
    fixedsplit = np.zeros((ns, ngroups))
    random = np.zeros((ns, nr))
    R2T_Y = 0.0
    R2T_Beta = np.zeros(nc)
    for i in range(S):                                                     # :125
        s = post[i]
        Beta = s["Beta"]
        mu = (Tr @ s["Gamma"].T).T                                         # gemu :100-103
        for k in range(nc):                                                # :126-128
            R2T_Beta[k] += np.corrcoef(Beta[k], mu[k])[0, 1] ** 2
        f = X @ Beta                                                       # getf :87-97
        a = X @ mu                                                         # geta :75-84
        a = a - a.mean(axis=1, keepdims=True)
        f = f - f.mean(axis=1, keepdims=True)
        res1 = np.sum((np.sum(a * f, axis=1) / (ns - 1)) ** 2)            # :139-141
        res2 = np.sum((np.sum(a * a, axis=1) / (ns - 1)) * (np.sum(f * f, axis=1) / (ns - 1)))
        R2T_Y += res1 / res2
        fixed1 = np.einsum("kj,kl,lj->j", Beta, cM, Beta)                  # :142-146
        fixedsplit1 = np.zeros((ns, ngroups))
        for g in range(1, ngroups + 1):                                    # :147-151
            sel = group == g
            fixedsplit1[:, g - 1] = np.einsum("kj,kl,lj->j", Beta[sel], cM[np.ix_(sel, sel)], Beta[sel])
        random1 = np.zeros((ns, nr))
        for r in range(nr):                                                # :154-160
            lam = s["Lambda"][r]
            random1[:, r] = np.sum(lam * lam, axis=0)
        if nr > 0:                                                         # :161-170
            tot = fixed1 + random1.sum(axis=1)
            fixed += fixed1 / tot
            random += random1 / tot[:, None]
        else:
            fixed += 1.0
        fixedsplit += fixedsplit1 / fixedsplit1.sum(axis=1, keepdims=True)  # :171-173
    fixed /= S
    random /= S
    fixedsplit /= S
    vals = np.zeros((ngroups + nr, ns))                                    # :180-187
    for g in range(ngroups):
        vals[g] = fixed * fixedsplit[:, g]
    for r in range(nr):
        vals[ngroups + r] = random[:, r]
    rl = list(getattr(hM, "rLNames", None) or [f"level{r + 1}" for r in range(nr)])
    return dict(vals=vals, R2T=dict(Beta=R2T_Beta / S, Y=R2T_Y / S), group=group, groupnames=groupnames,
                rownames=list(groupnames) + [f"Random: {n}" for n in rl])
