"""Post-sampling statistics restated in numpy -- TEST INFRASTRUCTURE (the checker of
hmsc_amd/csrc/post.hip), imported only by tests/, the fixture generators and bench.py's
cpu_baseline leg; the product (hmsc_amd.post) computes these on the device.

* spectrum0_ar / effectiveSize: coda::effectiveSize (spectrum0.ar with R's ar.yw.default:
  AR order by AIC up to min(n - 1, 10 log10 n), Yule-Walker by Levinson-Durbin); coda is not
  vendored in the reference (DESCRIPTION:27-48, version unpinned): parity with coda itself is
  unpinned, the restatement follows its published algorithm.
* computeVariancePartitioning: R/computeVariancePartitioning.R:37-204 line by line.
* computeAssociations: R/computeAssociations.R (mean and support of cov2cor(crossprod(Lambda))).
"""
import numpy as np


def poolMcmcChains(postList, start=1, thin=1):
    """R/poolMcmcChains.R."""
    out = []
    for ch in postList:
        out.extend(ch[start - 1::thin])
    return out


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


def computeAssociations(hM, start=1, thin=1):
    """R/computeAssociations.R: per level, mean and support (P(> 0)) of
    cov2cor(crossprod(Lambda_s)) over the pooled samples (the diagonal exactly 1)."""
    post = poolMcmcChains(hM.postList, start=start, thin=thin)
    out = []
    for r in range(hM.nr):
        cs = []
        for s in post:
            om = s["Lambda"][r].T @ s["Lambda"][r]
            d = 1.0 / np.sqrt(np.diag(om))
            c = om * d[:, None] * d[None, :]
            np.fill_diagonal(c, 1.0)
            cs.append(c)
        cs = np.stack(cs)
        out.append(dict(mean=cs.mean(axis=0), support=(cs > 0).mean(axis=0)))
    return out
