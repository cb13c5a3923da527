"""ORACLE — test infrastructure only.

CPU restatement (numpy, fp64) of the reference's Gibbs sweep for Hmsc 3.0-4
(taddallas/HMSC).  Each function follows one R updater line by line and cites
it; randomness follows the counter contract of ``oracle/rng.py`` (== the device
``hmsc_amd/csrc/rng.h``), so given the same state and chain seed the HIP
updaters must reproduce these draws to fp64 rounding.

Imported only by ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg — never by the product path (``hmsc_amd``).

Parity status: pinned by the reference's own deterministic known answers
(computeDataParameters sums, WAIC, scaling, shapes — tests/test_oracle_golden.py)
and statistically by the TD$m golden posterior; the reference's RNG-dependent
``round(sum(.))`` test values depend on R's Mersenne-Twister + truncnorm /
MCMCpack / BayesLogit bitstreams and are not reproducible.

State dict keys (mirror R's parList, R/computeInitialParameters.R:256-270):
  Gamma (nc,nt)  iV (nc,nc)  Beta (nc,ns)  iSigma (ns,)  rho (int, 1-based)
  Eta [r] (np_r,nf_r)  Lambda [r] (nf_r,ns)  Psi [r] (nf_r,ns)  Delta [r] (nf_r,)
  Alpha [r] (nf_r,) int 1-based   Z (ny,ns)
Model dict keys (the hM fields the sampler consumes):
  X (ny,nc)  Y (ny,ns) NaN=NA  Tr (ns,nt)  Pi (ny,nr) 1-based  distr (ns,4)
  V0 f0 mGamma UGamma aSigma bSigma  rL [dict(nu,a1,b1,a2,b2,nfMin,nfMax,sDim,xDim)]
  C (or None), iQg/RQg/detQg (from compute_data_parameters), rhopw
"""
import numpy as np
from scipy.linalg import solve_triangular

from . import rng as R


def chol_upper(A):
    """R's chol(): upper-triangular R with R'R = A."""
    return np.linalg.cholesky(A).T


def chol2inv(Rm):
    """R's chol2inv(R) = (R'R)^-1."""
    Ri = solve_triangular(Rm, np.eye(Rm.shape[0]), lower=False)
    return Ri @ Ri.T


def backsolve(Rm, b, transpose=False):
    """R's backsolve(R, b[, transpose=TRUE])."""
    return solve_triangular(Rm, b, lower=False, trans=1 if transpose else 0)


# ---------------------------------------------------------------------------
# data parameters — R/computeDataParameters.R:16-45 (phylogeny grid / identity)
# ---------------------------------------------------------------------------
def compute_data_parameters(model):
    C = model.get("C")
    ns = model["Y"].shape[1]
    rhopw = model["rhopw"]
    if C is not None:
        nrho = rhopw.shape[0]
        Qg = np.empty((nrho, ns, ns))
        iQg = np.empty_like(Qg)
        RQg = np.empty_like(Qg)
        detQg = np.empty(nrho)
        iC = chol2inv(chol_upper(C)) if np.any(rhopw[:, 0] < 0) else None
        for g in range(nrho):                                  # :23-38
            rho = rhopw[g, 0]
            rhoC = rho * C if rho >= 0 else (-rho) * iC
            Q = rhoC + (1 - abs(rho)) * np.eye(ns)
            RQ = chol_upper(Q)
            Qg[g], iQg[g], RQg[g] = Q, chol2inv(RQ), RQ
            detQg[g] = 2 * np.sum(np.log(np.diag(RQ)))
    else:                                                      # :40-45
        Qg = np.eye(ns)[None]
        iQg = np.eye(ns)[None]
        RQg = np.eye(ns)[None]
        detQg = np.zeros(1)
    rLPar = []
    for rl in model.get("rL", []):                             # :47-196 spatial grids
        if not rl.get("sDim", 0):
            rLPar.append({})
            continue
        method = rl.get("spatialMethod", "Full")
        if method == "NNGP":
            rLPar.append(_nngp_data_parameters(rl))
            continue
        if method == "GPP":
            rLPar.append(_gpp_data_parameters(rl))
            continue
        d = rl["dist"]                                         # np x np, levels(dfPi) order
        alphapw = rl["alphapw"]
        npr, G = d.shape[0], alphapw.shape[0]
        iWg, RiWg, detWg = np.empty((G, npr, npr)), np.empty((G, npr, npr)), np.empty(G)
        for g in range(G):
            a = alphapw[g, 0]
            W = np.eye(npr) if a == 0 else np.exp(-d / a)
            RW = chol_upper(W)
            iW = chol2inv(RW)
            iWg[g], RiWg[g], detWg[g] = iW, chol_upper(iW), 2 * np.sum(np.log(np.diag(RW)))
        rLPar.append(dict(iWg=iWg, RiWg=RiWg, detWg=detWg))
    return dict(Qg=Qg, iQg=iQg, RQg=RQg, detQg=detQg, rLPar=rLPar)


def _nngp_data_parameters(rl):
    """R/computeDataParameters.R:82-136.  Neighbours: FNN::get.knn(s, k) (FNN 1.1.x, exact
    Euclidean kNN without the point itself; not vendored in the reference) restated by brute
    force, sorted ascending, only earlier units kept (:93-104).  Per grid point: A[i, nb] =
    K11^-1 k12, D[i] = 1 - k21 K11^-1 k12 (D = 1 for units without earlier neighbours),
    RiW = D^-1/2 (I - A), iW = RiW' RiW, detW = sum(log D); identity for alpha = 0."""
    s = np.asarray(rl["s"], dtype=np.float64)
    k = int(rl.get("nNeighbours") or 10)
    n = s.shape[0]
    nb = []
    for i in range(n):
        dist = [(float(np.sum((s[i] - s[j]) ** 2)), j) for j in range(n) if j != i]
        near = sorted(j for _, j in sorted(dist)[:k])
        nb.append([j for j in near if j < i])
    alphapw = rl["alphapw"]
    G = alphapw.shape[0]
    iWg, RiWg, detWg = np.empty((G, n, n)), np.empty((G, n, n)), np.zeros(G)
    for g in range(G):
        a = alphapw[g, 0]
        RiW = np.eye(n)
        if a != 0:
            for i in range(n):
                if not nb[i]:
                    continue
                pts = s[nb[i] + [i]]
                Kp = np.exp(-np.sqrt(((pts[:, None] - pts[None, :]) ** 2).sum(-1)) / a)
                v = np.linalg.solve(Kp[:-1, :-1], Kp[:-1, -1])
                Di = Kp[-1, -1] - Kp[-1, :-1] @ v
                RiW[i, :] = 0.0
                RiW[i, i] = 1.0
                RiW[i, nb[i]] = -v
                RiW[i, :] /= np.sqrt(Di)
                detWg[g] += np.log(Di)
        iWg[g], RiWg[g] = RiW.T @ RiW, RiW
    perm, bw = nngp_rcm(nb, n)
    return dict(iWg=iWg, RiWg=RiWg, detWg=detWg, nb=nb, perm=perm, bw_units=bw)


def nngp_rcm(nb, n):
    """The unit order in which the device factors an NNGP level's precision (hmsc_amd/csrc/
    nngp.hip, nngp_setup): reverse Cuthill-McKee on the graph whose edges join units that share a
    row of the Vecchia factor (the support {i} + nb[i] of row i), BFS from the unvisited unit of
    least degree (lowest index on ties), neighbours visited by increasing (degree, index), the
    visit order reversed.  Returns perm (perm[k] = unit at position k) and the bandwidth in
    units, max |pos[a] - pos[b]| over edges.  Not a reference function: R factors the sparse
    precision with CHOLMOD in its own order; any order gives the same conditional."""
    adj = [set() for _ in range(n)]
    for i in range(n):
        sup = [i] + list(nb[i])
        for a in sup:
            for b in sup:
                if a != b:
                    adj[a].add(b)
    adj = [sorted(a) for a in adj]
    deg = [len(a) for a in adj]
    seen = [False] * n
    order = []
    while len(order) < n:
        start = min((i for i in range(n) if not seen[i]), key=lambda i: (deg[i], i))
        seen[start] = True
        q, head = [start], 0
        while head < len(q):
            v = q[head]
            head += 1
            for u in sorted((u for u in adj[v] if not seen[u]), key=lambda u: (deg[u], u)):
                seen[u] = True
                q.append(u)
        order.extend(q)
    perm = np.array(order[::-1], dtype=np.int64)
    pos = np.empty(n, dtype=np.int64)
    pos[perm] = np.arange(n)
    bw = max((abs(int(pos[a]) - int(pos[b])) for a in range(n) for b in adj[a]), default=0)
    return perm, bw


def _gpp_data_parameters(rl):
    """R/computeDataParameters.R:138-194 literally (idDg, idDW12g, Fg, iFg, detDg), plus the
    dense prior precision iW = W^-1 = diag(idD) - idDW12 iF idDW12' (Woodbury on W = D + W12
    iW22 W12'), as RiW' RiW with the lower factor RiW = chol(W)^-1, and detW = detD, which the
    sweep's updateEta uses
    (_eta_spatial_full); gpp_eta_literal() restates R's own GPP updateEta and
    tests/test_oracle_spatial.py pins the two to the same posterior."""
    s = np.asarray(rl["s"], dtype=np.float64)
    sK = np.asarray(rl["sKnot"], dtype=np.float64)
    di12 = np.sqrt(((s[:, None] - sK[None, :]) ** 2).sum(-1))
    di22 = np.sqrt(((sK[:, None] - sK[None, :]) ** 2).sum(-1))
    alphapw = rl["alphapw"]
    G, n, nK = alphapw.shape[0], s.shape[0], sK.shape[0]
    out = dict(idDg=np.empty((G, n)), idDW12g=np.empty((G, n, nK)), Fg=np.empty((G, nK, nK)),
               iFg=np.empty((G, nK, nK)), detDg=np.empty(G), iWg=np.empty((G, n, n)), RiWg=np.empty((G, n, n)))
    for g in range(G):
        a = alphapw[g, 0]
        W22 = np.eye(nK) if a == 0 else np.exp(-di22 / a)
        W12 = np.zeros((n, nK)) if a == 0 else np.exp(-di12 / a)
        iW22 = np.linalg.solve(W22, np.eye(nK))
        dD = 1 - np.diag(W12 @ iW22 @ W12.T)
        liW22 = np.linalg.cholesky(iW22)
        idD = 1 / dD
        idDW12 = idD[:, None] * W12
        F = W22 + W12.T @ idDW12
        tmp2 = W12 @ liW22
        DS = tmp2.T @ (idD[:, None] * tmp2) + np.eye(nK)
        out["idDg"][g], out["idDW12g"][g], out["Fg"][g] = idD, idDW12, F
        out["iFg"][g] = np.linalg.solve(F, np.eye(nK))
        out["detDg"][g] = np.sum(np.log(dD)) + 2 * np.sum(np.log(np.diag(np.linalg.cholesky(DS))))
        W = W12 @ iW22 @ W12.T + np.diag(dD)                  # = D + W12 iW22 W12' (unit diagonal)
        RiW = np.linalg.inv(np.linalg.cholesky(0.5 * (W + W.T)))
        out["RiWg"][g] = np.tril(RiW)
        out["iWg"][g] = out["RiWg"][g].T @ out["RiWg"][g]
    out["detWg"] = out["detDg"]
    return out


def gpp_eta_literal(st, model, r, S, dp, xi1=None, xi2=None):
    """R/updateEta.R:148-196 as written: per-unit nf x nf blocks B0_i = Lam iSigma Lam' +
    diag(idD[i, alpha]), iA = blockdiag(B0_i^-1), H = Fmat - idD1W12' iA idD1W12, and
    eta = iA fS + iA W iRH iRH' W' iA fS + LiA xi1 + iA W iRH xi2 (xi1: np nf, xi2: nK nf
    normals; zero -> the posterior mean).  Returns (eta, posterior covariance)."""
    lam, iS = st["Lambda"][r], st["iSigma"]
    nf = lam.shape[0]
    par = dp["rLPar"][r]
    alpha = np.asarray(st["Alpha"][r], dtype=np.int64) - 1
    n = int(model["np"][r])
    nK = par["Fg"].shape[1]
    order = np.argsort(model["Pi"][:, r] - 1, kind="stable")
    fS = (S[order] @ (iS[:, None] * lam.T)).ravel(order="F")
    LSL = lam @ (iS[:, None] * lam.T)
    iA = np.zeros((n * nf, n * nf))
    LiA = np.zeros_like(iA)
    for i in range(n):
        idx = i + n * np.arange(nf)
        B1 = np.linalg.inv(LSL + np.diag(par["idDg"][alpha, i]))
        iA[np.ix_(idx, idx)] = B1
        LiA[np.ix_(idx, idx)] = np.linalg.cholesky(B1)
    Fmat = np.zeros((nK * nf, nK * nf))
    W = np.zeros((n * nf, nK * nf))
    for h in range(nf):
        Fmat[h * nK:(h + 1) * nK, h * nK:(h + 1) * nK] = par["Fg"][alpha[h]]
        W[h * n:(h + 1) * n, h * nK:(h + 1) * nK] = par["idDW12g"][alpha[h]]
    iAW = iA @ W
    H = Fmat - W.T @ iAW
    iRH = np.linalg.inv(chol_upper(H))
    tmp1 = iAW @ iRH
    eta = iA @ fS + tmp1 @ (tmp1.T @ fS)
    if xi1 is not None:
        eta = eta + LiA @ xi1 + tmp1 @ xi2
    return eta.reshape((n, nf), order="F"), iA + tmp1 @ tmp1.T


# ---------------------------------------------------------------------------
# linear predictor — R/updateZ.R:11-34 (repeated in updateEta/InvSigma/Gamma2)
# ---------------------------------------------------------------------------
def _xdim(model, r):
    return int(model["rL"][r].get("xDim", 0) or 0) if r < len(model.get("rL", [])) else 0


def _vlev(model, r):
    """The device level index of level r's first column block: a covariate-dependent level
    (xDim = ncr > 0) is ncr device levels sharing Eta (include/hmsc_amd.h etaShare / xScale),
    so the Philox level streams of level r start at sum_{r' < r} max(xDim_r', 1); = r without
    covariate-dependent levels."""
    return sum(max(_xdim(model, q), 1) for q in range(r))


def _prior(rl, name, k):
    """rL$nu / a1 / b1 / a2 / b2: scalars, or one per column of rL$x
    (R/setPriors.HmscRandomLevel.R:21-80)."""
    v = np.atleast_1d(np.asarray(rl[name], dtype=np.float64))
    return float(v[k] if v.size > 1 else v[0])


def eta_full(st, model, r):
    """Eta[Pi,] or, for a covariate-dependent level, [Eta[Pi,] * x[dfPi, k] for k] (the
    EtaFull / EtaSt columns of R/updateBetaLambda.R:21-36; x rows in unit order)."""
    E = st["Eta"][r][model["Pi"][:, r] - 1, :]
    xd = _xdim(model, r)
    if not xd:
        return E
    x = np.asarray(model["rL"][r]["x"], dtype=np.float64)[model["Pi"][:, r] - 1]
    return np.concatenate([E * x[:, k:k + 1] for k in range(xd)], axis=1)


def lambda_rows(lam):
    """Lambda[[r]] as BetaLambda rows: the matrix itself, or for an nf x ns x ncr array the
    ncr slices stacked (row f + nf k, R/updateBetaLambda.R:42-53,150-154)."""
    lam = np.asarray(lam)
    return lam if lam.ndim == 2 else np.concatenate([lam[:, :, k] for k in range(lam.shape[2])], axis=0)


def l_ran(st, model, r):
    return eta_full(st, model, r) @ lambda_rows(st["Lambda"][r])


def linear_predictor(st, model):
    E = model["X"] @ st["Beta"]
    for r in range(model["Pi"].shape[1]):
        E = E + l_ran(st, model, r)
    return E


# ---------------------------------------------------------------------------
# updateZ — R/updateZ.R:4-94 (normal :40-41, probit :43-63, NA :92)
# ---------------------------------------------------------------------------
POIS_R = 1e3   # Poisson as the limit of the negative binomial, R/updateZ.R:68


def pg_moments(b, c):
    """Mean and variance of the Polya-Gamma PG(b, c) (Polson, Scott & Windle 2013, eqs. in
    section 2.2): E = b tanh(c/2) / (2c), Var = b (sinh c - c) sech^2(c/2) / (4 c^3), written
    as b (2 tanh(x/2) - x sech^2(x/2)) / (4 x^3) for x = |c| >= 1 and as its Taylor series
    below 1 (no cancellation, no overflow).  Same formulas as rng.h pg_moments."""
    x = np.abs(np.asarray(c, dtype=np.float64))
    x2 = x * x
    with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
        m = np.where(x < 1e-4, 0.25 - x2 / 48.0, np.tanh(0.5 * x) / (2.0 * x))
        # (sinh x - x) / x^3 = sum_k x^(2k) / (2k+3)!
        q = 1.0 + x2 / 272.0
        for d in (210.0, 156.0, 110.0, 72.0, 42.0, 20.0):
            q = 1.0 + x2 / d * q
        q = q / 6.0
        ch = np.cosh(0.5 * x)
        sech2 = 1.0 / (ch * ch)
        v_small = q * sech2 / 4.0
        v_big = (2.0 * np.tanh(0.5 * x) - x * sech2) / (4.0 * x2 * x)
        v = np.where(x < 1.0, v_small, v_big)
    return b * m, b * v


def poisson_z_draw(y, e, sd, zprev, u1, u2, zero_noise=False):
    """Poisson Z (R/updateZ.R:65-90): omega ~ PG(y + r, zPrev - log r), r = 1000; then
    Z ~ N(sigmaZ ((y - r)/2 + prec (E - log r)) + log r, sigmaZ), sigmaZ = 1/(prec + omega).
    BayesLogit's rpg draws PG(h, z) for h > 170 -- always here, h >= 1000 -- as the normal
    with the PG mean and variance (PolyaGammaHybrid::draw, BayesLogit 2.x; the package is
    unvendored and unpinned, DESCRIPTION:33), so omega = m + sqrt(v) Phi^-1(u1)."""
    lr = np.log(POIS_R)
    m, v = pg_moments(y + POIS_R, zprev - lr)
    omega = m if zero_noise else m + np.sqrt(v) * R.qnorm_as241(u1.ravel()).reshape(u1.shape)
    prec = sd ** -2.0
    sigz = 1.0 / (prec + omega)
    muz = sigz * ((y - POIS_R) / 2.0 + prec * (e - lr)) + lr
    if zero_noise:
        return muz
    return muz + np.sqrt(sigz) * R.qnorm_as241(u2.ravel()).reshape(u2.shape)


def update_z(st, model, rng, it, Y=None, zero_noise=False):
    Y = model["Y"] if Y is None else Y
    ny, ns = Y.shape
    E = linear_predictor(st, model)
    sd = st["iSigma"] ** -0.5
    # one Philox block per (site, species quad 4q .. 4q + 3); species 4q + k takes word k as the
    # uniform (w + 1/2) 2^-32 (rng.h contract, z_wave_kernel)
    j = np.arange(ns)
    idx = (np.arange(ny)[:, None] + ny * (j[None, :] >> 2)).astype(np.uint64)
    fam = model["distr"][:, 0]
    na = np.isnan(Y)
    Z = np.empty((ny, ns))
    normal_cols = fam == 1
    Z[:, normal_cols] = Y[:, normal_cols]
    w4 = rng.words(idx, 0, R.S_Z, it)
    u = R.u32o(np.choose(np.broadcast_to((j & 3)[None, :], idx.shape), w4))
    s = np.where(Y == 1, 1.0, -1.0)
    alpha = -s * E / sd[None, :]
    w = R.trunc_normal_lower(alpha, u)
    zp = E + sd[None, :] * s * w
    probit_cols = fam == 2
    Z[:, probit_cols] = zp[:, probit_cols]
    pois_cols = fam == 3
    if pois_cols.any():   # R/updateZ.R:65-90
        jp = np.nonzero(pois_cols)[0]
        Zprev = st["Z"][:, jp] if "Z" in st else E[:, jp]   # init: Z = LFix + LRan (computeInitialParameters.R:250-254)
        cell = (np.arange(ny)[:, None] + ny * jp[None, :]).astype(np.uint64)
        u1, u2 = rng.uniforms(cell, 0, R.S_ZPOIS, it)
        Z[:, jp] = poisson_z_draw(Y[:, jp], E[:, jp], sd[jp][None, :], Zprev, u1, u2,
                                  zero_noise)
    if na.any():   # R/updateZ.R:92: N(E, sd), drawn by inversion of the same uniform
        nz = E - sd[None, :] * R.qnorm_as241(u.ravel()).reshape(u.shape)
        Z[na] = nz[na]
    return Z


# ---------------------------------------------------------------------------
# updateBetaLambda — R/updateBetaLambda.R:8-157
# ---------------------------------------------------------------------------
def _xeta_and_prior(st, model):
    nr = model["Pi"].shape[1]
    X = model["X"]
    cols = [X] + [eta_full(st, model, r) for r in range(nr)]          # :21-41
    XEta = np.concatenate(cols, axis=1)
    ns = model["Y"].shape[1]
    pl = []
    for r in range(nr):                                               # :42-53
        if _xdim(model, r):   # tau = apply(delta, 2, cumprod) per column k, psiSt rows f + nf k
            tau = np.cumprod(st["Delta"][r], axis=0)
            pl.append(lambda_rows(st["Psi"][r] * tau[:, None, :]))
            continue
        tau = np.cumprod(st["Delta"][r])
        pl.append(st["Psi"][r] * tau[:, None])
    priorLambda = np.concatenate(pl, axis=0) if pl else np.zeros((0, ns))
    return XEta, priorLambda


def beta_lambda_moments(st, model, data_par=None):
    """Per-species precision iU_j and mean m_j of the C=NULL branch (:76-123)."""
    Y, Z = model["Y"], st["Z"]
    nc = model["X"].shape[1]
    ns = Y.shape[1]
    XEta, priorLambda = _xeta_and_prior(st, model)
    K = XEta.shape[1]
    Mu = np.concatenate([st["Gamma"] @ model["Tr"].T, np.zeros((K - nc, ns))])   # :62
    iS = st["iSigma"]
    Yx = ~np.isnan(Y)
    precs = np.empty((ns, K, K))
    means = np.empty((K, ns))
    G = XEta.T @ XEta                                                  # :65
    XS = XEta.T @ Z                                                    # :66
    for j in range(ns):
        P = np.zeros((K, K))
        P[:nc, :nc] = st["iV"]                                         # :83-84
        P[np.diag_indices(K)] = np.concatenate([np.diag(st["iV"]), priorLambda[:, j]])  # :89
        if Yx[:, j].all():
            iU = P + G * iS[j]                                         # :92
            isXTS = XS[:, j] * iS[j]
        else:                                                          # :103-117
            o = Yx[:, j]
            iU = P + (XEta[o].T @ XEta[o]) * iS[j]
            isXTS = (XEta[o].T @ Z[o, j]) * iS[j]
        precs[j] = iU
        means[:, j] = np.linalg.solve(iU, P @ Mu[:, j] + isXTS)        # :98-100
    return precs, means


def update_beta_lambda(st, model, rng, it, data_par=None, zero_noise=False):
    nc = model["X"].shape[1]
    ns = model["Y"].shape[1]
    nr = model["Pi"].shape[1]
    if model.get("C") is not None:
        BL = _beta_lambda_phylo(st, model, rng, it, data_par, zero_noise)
    else:
        precs, means = beta_lambda_moments(st, model)
        K = means.shape[0]
        BL = np.empty((K, ns))
        for j in range(ns):
            RiU = chol_upper(precs[j])                                 # :98
            xi = np.zeros(K) if zero_noise else rng.normal(j, np.arange(K), R.S_BETALAMBDA, it)
            BL[:, j] = means[:, j] + backsolve(RiU, xi)                # :101
    Beta = BL[:nc].copy()                                              # :148
    Lambda = []
    off = nc
    for r in range(nr):                                                # :149-155
        nf = st["Lambda"][r].shape[0]
        xd = _xdim(model, r)
        if xd:  # aperm(array(rows, c(nf, ncr, ns)), c(1, 3, 2))
            Lambda.append(BL[off:off + nf * xd].reshape(xd, nf, ns).transpose(1, 2, 0).copy())
            off += nf * xd
            continue
        Lambda.append(BL[off:off + nf].copy())
        off += nf
    return Beta, Lambda


def _beta_lambda_phylo(st, model, rng, it, data_par, zero_noise):
    """Dense branch with phylogeny, R/updateBetaLambda.R:124-147 (species-fastest vec)."""
    Z = st["Z"]
    nc = model["X"].shape[1]
    ns = Z.shape[1]
    XEta, priorLambda = _xeta_and_prior(st, model)
    K = XEta.shape[1]
    iQ = data_par["iQg"][st["rho"] - 1]
    Mu = np.concatenate([st["Gamma"] @ model["Tr"].T, np.zeros((K - nc, ns))])
    iS = st["iSigma"]
    G = XEta.T @ XEta
    isXTS = (XEta.T @ Z) * iS[None, :]
    P = np.zeros((K * ns, K * ns))
    P[:nc * ns, :nc * ns] = np.kron(st["iV"], iQ)                      # :126
    P[nc * ns:, nc * ns:] = np.diag(priorLambda.reshape(-1))           # Diagonal(x=t(priorLambda))
    RiU = chol_upper(np.kron(G, np.diag(iS)) + P)                      # :129
    m1 = backsolve(RiU, P @ Mu.reshape(-1) + isXTS.reshape(-1), transpose=True)   # :145
    xi = np.zeros(K * ns) if zero_noise else \
        rng.normal(np.tile(np.arange(ns), K), np.repeat(np.arange(K), ns), R.S_BETALAMBDA, it)
    return backsolve(RiU, m1 + xi).reshape(K, ns)                      # :146 byrow=TRUE


# ---------------------------------------------------------------------------
# Wishart (MCMCpack::rwish restated) — Bartlett construction, upper Z
# ---------------------------------------------------------------------------
def rwish(v, S, rng, it, s_diag, s_off, zero_noise=False):
    p = S.shape[0]
    CC = chol_upper(S)
    Zm = np.zeros((p, p))
    df = v - np.arange(p)                                              # v:(v-p+1)
    Zm[np.diag_indices(p)] = np.sqrt(2.0 * rng.gamma_std(np.arange(p), s_diag, it, df / 2.0))
    iu = np.triu_indices(p, 1)
    if p > 1 and not zero_noise:
        Zm[iu] = rng.normal(iu[0] + p * iu[1], 0, s_off, it)
    ZC = Zm @ CC
    return ZC.T @ ZC


# ---------------------------------------------------------------------------
# updateGammaV — R/updateGammaV.R:4-34
# ---------------------------------------------------------------------------
def update_gamma_v(st, model, rng, it, data_par=None, zero_noise=False):
    Beta, Gamma, Tr = st["Beta"], st["Gamma"], model["Tr"]
    ns, nc, nt = Beta.shape[1], Beta.shape[0], Tr.shape[1]
    if model.get("C") is None:                                         # :10-12
        iQ = RQ = None
    else:
        iQ = data_par["iQg"][st["rho"] - 1]
        RQ = data_par["RQg"][st["rho"] - 1]
    E = Beta - Gamma @ Tr.T                                            # :16-17
    A = E @ E.T if iQ is None else E @ (iQ @ E.T)                      # :18 (identity special-cased)
    Vn = chol2inv(chol_upper(A + model["V0"]))                         # :19
    iV = rwish(model["f0"] + ns, Vn, rng, it, R.S_WISHART_DIAG, R.S_WISHART_OFF)   # :20
    iUGamma = np.linalg.inv(model["UGamma"])
    TrQ = Tr if RQ is None else backsolve(RQ, Tr, transpose=True)
    RG = chol_upper(iUGamma + np.kron(TrQ.T @ TrQ, iV))                # :29
    QTr = Tr if iQ is None else iQ @ Tr
    rhs = iUGamma @ model["mGamma"] + ((iV @ Beta) @ QTr).reshape(-1, order="F")
    mg = chol2inv(RG) @ rhs                                            # :30
    xi = np.zeros(nc * nt) if zero_noise else rng.normal(np.arange(nc * nt), 0, R.S_GAMMAV, it)
    Gamma = (mg + backsolve(RG, xi)).reshape(nc, nt, order="F")        # :31
    return Gamma, iV


def gamma_v_moments(st, model, iV):
    """Gamma conditional mean/precision given the new iV (C=NULL)."""
    Beta, Tr = st["Beta"], model["Tr"]
    iUGamma = np.linalg.inv(model["UGamma"])
    prec = iUGamma + np.kron(Tr.T @ Tr, iV)
    rhs = iUGamma @ model["mGamma"] + ((iV @ Beta) @ Tr).reshape(-1, order="F")
    return prec, np.linalg.solve(prec, rhs)


# ---------------------------------------------------------------------------
# updateGamma2 — R/updateGamma2.R:6-60 (acts only if C is NULL and all iSigma==1)
# ---------------------------------------------------------------------------
def gamma2_moments(st, model):
    X, Tr, iV = model["X"], model["Tr"], st["iV"]
    nc, nt = X.shape[1], Tr.shape[1]
    S = st["Z"].copy()
    for r in range(model["Pi"].shape[1]):                              # :20-33
        S -= l_ran(st, model, r)
    inv = lambda A: chol2inv(chol_upper(A))                            # noqa: E731
    cholL = lambda A: chol_upper(A).T                                  # noqa: E731
    iUGamma = np.linalg.inv(model["UGamma"])
    iV0 = iUGamma[:nc, :nc]                                            # :37
    V0 = inv(iV0)
    XX = X.T @ X
    TT = Tr.T @ Tr
    iP = inv(iV + XX)
    LiP = cholL(iP)
    t1 = iV @ LiP
    Rm = inv(np.kron(np.eye(nt), iV0) + np.kron(TT, iV - t1 @ t1.T))   # :44
    LR = cholL(Rm)
    XZT = X.T @ (S @ Tr)                                               # :46
    iPXZT = iP @ XZT
    tmp = np.kron(TT, V0 @ XX @ iP @ iV)
    muG = (V0 @ (XZT - XX @ iPXZT)).reshape(-1, order="F") - tmp @ Rm @ (iV @ iPXZT).reshape(-1, order="F")
    V0Xt = V0 @ X.T
    t2 = V0 @ XX @ LiP
    t3 = tmp @ LR
    SigmaG = np.kron(np.eye(nt), V0) - np.kron(TT, V0Xt @ V0Xt.T - t2 @ t2.T) + t3 @ t3.T   # :50
    return muG, SigmaG


def update_gamma2(st, model, rng, it, zero_noise=False):
    if model.get("C") is not None or not np.all(st["iSigma"] == 1):  # :35-36
        return st["Gamma"]
    nc, nt = model["X"].shape[1], model["Tr"].shape[1]
    muG, SigmaG = gamma2_moments(st, model)
    LS = chol_upper(SigmaG).T
    xi = np.zeros(nc * nt) if zero_noise else rng.normal(np.arange(nc * nt), 0, R.S_GAMMA2, it)
    return (muG + LS @ xi).reshape(nc, nt, order="F")                 # :53-54


# ---------------------------------------------------------------------------
# updateLambdaPriors — R/updateLambdaPriors.R:3-53 (matrix branch :21-33)
# ---------------------------------------------------------------------------
def update_lambda_priors(st, model, rng, it):
    Psi, Delta = [], []
    ns = model["Y"].shape[1]
    for r, rl in enumerate(model["rL"]):
        if _xdim(model, r):
            p, d = _lambda_priors_x(st, model, rng, it, r)
            Psi.append(p)
            Delta.append(d)
            continue
        nu, a1, b1, a2, b2 = rl["nu"], rl["a1"], rl["b1"], rl["a2"], rl["b2"]
        v = _vlev(model, r)
        delta = st["Delta"][r].astype(np.float64).copy()
        lam = st["Lambda"][r]
        nf = lam.shape[0]
        tau = np.cumprod(delta)                                        # :17
        lam2 = lam ** 2
        aPsi = nu / 2 + 0.5
        bPsi = nu / 2 + 0.5 * lam2 * tau[:, None]                      # :22
        hh, jj = np.meshgrid(np.arange(nf), np.arange(ns), indexing="ij")
        psi = rng.gamma(hh + nf * jj, R.S_PSI + R.LEVEL_STRIDE * v, it, aPsi, bPsi)   # :23
        M = psi * lam2
        rs = M.sum(axis=1)
        ad = a1 + 0.5 * ns * nf                                        # :25
        bd = b1 + 0.5 * np.sum(tau * rs) / delta[0]                    # :26
        delta[0] = rng.gamma(0, R.S_DELTA + R.LEVEL_STRIDE * v, it, ad, bd)
        for h in range(1, nf):                                         # :28-32
            tau = np.cumprod(delta)
            ad = a2 + 0.5 * ns * (nf - h)
            bd = b2 + 0.5 * np.sum(tau[h:] * rs[h:]) / delta[h]
            delta[h] = rng.gamma(h, R.S_DELTA + R.LEVEL_STRIDE * v, it, ad, bd)
        Psi.append(psi)
        Delta.append(delta)
    return Psi, Delta


def _lambda_priors_x(st, model, rng, it, r):
    """The array branch (R/updateLambdaPriors.R:34-48) for Lambda nf x ns x ncr: psi and the
    delta chain of column k are the matrix branch's on Lambda[,,k] with the priors' k-th entries
    (device level _vlev(r) + k).  R draws psi as rgamma(nf*ns*ncr, aPsi, bPsi) with the length-ncr
    nu recycled over the array's cells; with one nu for every column (the default, rep(3, xDim))
    that is nu[k]."""
    rl = model["rL"][r]
    lam = st["Lambda"][r]
    nf, ns, ncr = lam.shape
    psi = np.empty_like(lam)
    delta = np.asarray(st["Delta"][r], dtype=np.float64).reshape(nf, ncr).copy()
    for k in range(ncr):
        v = _vlev(model, r) + k
        nu = _prior(rl, "nu", k)
        d = delta[:, k]
        tau = np.cumprod(d)
        lam2 = lam[:, :, k] ** 2
        hh, jj = np.meshgrid(np.arange(nf), np.arange(ns), indexing="ij")
        psi[:, :, k] = rng.gamma(hh + nf * jj, R.S_PSI + R.LEVEL_STRIDE * v, it, nu / 2 + 0.5,
                                 nu / 2 + 0.5 * lam2 * tau[:, None])
        rs = (psi[:, :, k] * lam2).sum(axis=1)
        bd = _prior(rl, "b1", k) + 0.5 * np.sum(tau * rs) / d[0]
        d[0] = rng.gamma(0, R.S_DELTA + R.LEVEL_STRIDE * v, it, _prior(rl, "a1", k) + 0.5 * ns * nf, bd)
        for h in range(1, nf):
            tau = np.cumprod(d)
            bd = _prior(rl, "b2", k) + 0.5 * np.sum(tau[h:] * rs[h:]) / d[h]
            d[h] = rng.gamma(h, R.S_DELTA + R.LEVEL_STRIDE * v, it, _prior(rl, "a2", k) + 0.5 * ns * (nf - h), bd)
        delta[:, k] = d
    return psi, delta


# ---------------------------------------------------------------------------
# updateEta — R/updateEta.R:4-212, non-spatial xDim=0 branch (:42-92)
# ---------------------------------------------------------------------------
def eta_unit_moments(st, model, r, S):
    """Per-unit precision Q_q and mean mu_q for level r given residual S."""
    Y = model["Y"]
    lam = st["Lambda"][r]
    nf = lam.shape[0]
    iS = st["iSigma"]
    Pi_r = model["Pi"][:, r] - 1
    npr = st["Eta"][r].shape[0]
    Yx = ~np.isnan(Y)
    LamInvSigLam = (lam * iS[None, :]) @ lam.T                         # :45
    lamT = (lam * iS[None, :]).T                                       # lambda*iSigma, transposed
    # units whose rows are all observed share Q = I + n_q LamInvSigLam   (:46-57, :75-79)
    n_q = np.bincount(Pi_r, minlength=npr).astype(np.float64)
    Ssum = np.zeros((npr, S.shape[1]))
    np.add.at(Ssum, Pi_r, S)
    precs = np.eye(nf)[None, :, :] + LamInvSigLam[None, :, :] * n_q[:, None, None]
    bs = Ssum @ lamT
    has_na = np.zeros(npr, dtype=bool)
    np.logical_or.at(has_na, Pi_r, ~Yx.all(axis=1))
    for q in np.nonzero(has_na)[0]:                                    # :59-70 and :80-87
        Q = np.eye(nf)
        b = np.zeros(nf)
        for p in np.nonzero(Pi_r == q)[0]:
            w = iS * Yx[p]
            Q = Q + (lam * w[None, :]) @ lam.T
            b = b + (np.where(Yx[p], S[p], 0.0) * iS) @ lam.T
        precs[q] = Q
        bs[q] = b
    means = np.linalg.solve(precs, bs[:, :, None])[:, :, 0]
    return precs, means


def eta_unit_moments_x(st, model, r, S):
    """Covariate-dependent level (R/updateEta.R:93-108): per unit q, lambdaLocal =
    sum_k x[q, k] Lambda[,,k]; Q_q = I + sum_{rows p of q} lambdaLocal diag(iSigma Yx_p)
    lambdaLocal^T, mu_q = Q_q^-1 sum_p lambdaLocal diag(iSigma Yx_p) S_p."""
    Y = model["Y"]
    lam = st["Lambda"][r]
    nf = lam.shape[0]
    iS = st["iSigma"]
    Pi_r = model["Pi"][:, r] - 1
    npr = st["Eta"][r].shape[0]
    x = np.asarray(model["rL"][r]["x"], dtype=np.float64)
    Yx = ~np.isnan(Y)
    precs = np.empty((npr, nf, nf))
    means = np.empty((npr, nf))
    for q in range(npr):
        lL = np.tensordot(lam, x[q], axes=([2], [0]))                    # rowSums(lambda * x[q,], dims=2)
        Q = np.eye(nf)
        b = np.zeros(nf)
        for p in np.nonzero(Pi_r == q)[0]:
            w = iS * Yx[p]
            Q = Q + (lL * w[None, :]) @ lL.T
            b = b + (np.where(Yx[p], S[p], 0.0) * iS) @ lL.T
        precs[q] = Q
        means[q] = np.linalg.solve(Q, b)
    return precs, means


def _eta_spatial_full(st, model, r, S, dp, rng, it, zero_noise):
    """Spatial level, R/updateEta.R:115-147 ('Full'; 'NNGP' is the same code on a sparse
    iWg; 'GPP' goes to _eta_spatial_gpp, R's low-rank form): one dense (np nf)^2 system
    iUEta = bdiag(iWg[,,alpha_h]) + kron(Lam iSigma Lam', diag(colSums P)),
    fS = P'S (Lam diag(iSigma))', eta = R^-1 (R^-T vec(fS) + xi), R = chol(iUEta)."""
    lam, iS = st["Lambda"][r], st["iSigma"]
    nf = lam.shape[0]
    npr = int(model["np"][r])
    lPi = model["Pi"][:, r] - 1
    iWg = dp["rLPar"][r]["iWg"]
    alpha = np.asarray(st["Alpha"][r], dtype=np.int64)
    P = np.zeros((S.shape[0], npr))
    P[np.arange(S.shape[0]), lPi] = 1.0
    LamInvSigLam = (lam * np.sqrt(iS)[None, :]) @ (lam * np.sqrt(iS)[None, :]).T
    iU = np.kron(LamInvSigLam, np.diag(P.sum(axis=0)))
    for h in range(nf):
        iU[h * npr:(h + 1) * npr, h * npr:(h + 1) * npr] += iWg[alpha[h] - 1]
    fS = (P.T @ S) @ (lam * iS[None, :]).T
    xi = None if zero_noise else \
        rng.normal(np.arange(npr)[:, None], np.arange(nf)[None, :], R.S_ETA + R.LEVEL_STRIDE * _vlev(model, r), it).ravel(order="F")
    if model["rL"][r].get("spatialMethod", "Full") == "NNGP":
        # the device factors the sparse NNGP precision in RCM order, factors interleaved per unit
        # (index pos[q] nf + h, nngp.hip): eta = P' L^-T (L^-1 P vec(fS) + P xi), L L' = P iUEta P'
        # -- the same conditional, the noise of (unit q, factor h) as in R's order
        perm = dp["rLPar"][r]["perm"]
        ix = (perm[:, None] + npr * np.arange(nf)[None, :]).ravel()   # position-major, factor fastest
        Rm = chol_upper(iU[np.ix_(ix, ix)])
        tmp2 = backsolve(Rm, fS.ravel(order="F")[ix], transpose=True)
        if xi is not None:
            tmp2 = tmp2 + xi[ix]
        out = np.empty(npr * nf)
        out[ix] = backsolve(Rm, tmp2)
        return out.reshape((npr, nf), order="F")
    Rm = chol_upper(iU)
    tmp2 = backsolve(Rm, fS.ravel(order="F"), transpose=True)
    if xi is not None:
        tmp2 = tmp2 + xi
    return backsolve(Rm, tmp2).reshape((npr, nf), order="F")


GPP_XI2_SUB = 1024  # hmsc_amd/csrc/spatial.hip


def _eta_spatial_gpp(st, model, r, S, dp, rng, it, zero_noise):
    """'GPP' level (np == ny), R/updateEta.R:148-196 in R's own low-rank form
    (gpp_eta_literal): eta = iA fS + T (T' fS + xi2) + LiA xi1 with xi1 of unit i, factor h =
    normal(i, h, S_ETA + LEVEL_STRIDE r) and xi2 of knot k, factor h = normal(k,
    GPP_XI2_SUB + h, same stream), as the device draws them."""
    nf = st["Lambda"][r].shape[0]
    n = int(model["np"][r])
    nK = dp["rLPar"][r]["Fg"].shape[1]
    if zero_noise:
        return gpp_eta_literal(st, model, r, S, dp)[0]
    stream = R.S_ETA + R.LEVEL_STRIDE * _vlev(model, r)
    xi1 = rng.normal(np.arange(n)[:, None], np.arange(nf)[None, :], stream, it).ravel(order="F")
    xi2 = rng.normal(np.arange(nK)[:, None], GPP_XI2_SUB + np.arange(nf)[None, :], stream, it).ravel(order="F")
    return gpp_eta_literal(st, model, r, S, dp, xi1, xi2)[0]


def update_alpha(st, model, rng, it, data_par=None):
    """R/updateAlpha.R:3-86: v_gh = |RiWg[,,g] eta_h|^2 ('Full', 'NNGP'), or for 'GPP'
    eta_h' diag(idDg[,g]) eta_h - (eta' idDW12g iFg idDW12g' eta)_hh; log-likelihood
    log(alphapw[g,2]) - detWg[g]/2 - v_gh/2 (detDg for GPP), categorical draw by inverse CDF of the uniform
    (idx h, S_ALPHA + LEVEL_STRIDE r); rep(1, nf) for non-spatial levels (:81-82)."""
    out = []
    for r, rl in enumerate(model["rL"]):
        eta = st["Eta"][r]
        nf = eta.shape[1]
        if not rl.get("sDim", 0):
            out.append(np.ones(nf, dtype=np.int64))
            continue
        dp = data_par if data_par is not None else compute_data_parameters(model)
        par = dp["rLPar"][r]
        alphapw = rl["alphapw"]
        if rl.get("spatialMethod", "Full") == "GPP":                   # :35-49, :64-75
            G = alphapw.shape[0]
            v = np.empty((G, nf))
            det = par["detDg"]
            for g in range(G):
                t2 = eta.T @ par["idDW12g"][g]
                t4 = (t2 @ par["iFg"][g]) @ t2.T
                for h in range(nf):
                    v[g, h] = eta[:, h] @ eta[:, h] if alphapw[g, 0] == 0 else \
                        eta[:, h] @ (par["idDg"][g] * eta[:, h]) - t4[h, h]
        else:                                                          # :21-34, :56-63
            v = np.stack([np.sum((par["RiWg"][g] @ eta) ** 2, axis=0) for g in range(alphapw.shape[0])])
            det = par["detWg"]
        a = np.empty(nf, dtype=np.int64)
        for h in range(nf):
            like = np.log(alphapw[:, 1]) - 0.5 * det - 0.5 * v[:, h]
            like = np.exp(like - like.max())
            u = rng.uniforms(h, 0, R.S_ALPHA + R.LEVEL_STRIDE * _vlev(model, r), it)[0]
            a[h] = int(np.searchsorted(np.cumsum(like), u * like.sum(), side="right")) + 1
        out.append(a)
    return out


def update_eta(st, model, rng, it, zero_noise=False, data_par=None):
    nr = model["Pi"].shape[1]
    st = dict(st)
    Eta = list(st["Eta"])
    LFix = model["X"] @ st["Beta"]                                     # :11-20
    for r in range(nr):
        S = st["Z"] - LFix                                             # :31-37
        st["Eta"] = Eta
        for r2 in range(nr):
            if r2 != r:
                # (R's in-loop LRan refresh of a covariate-dependent level, :205, indexes x and
                # Lambda by the level number r instead of k; this is the form of :23-29)
                S = S - l_ran(st, model, r2)
        if model["rL"][r].get("sDim", 0) > 0:                          # :111-197
            dp = data_par if data_par is not None else compute_data_parameters(model)
            if model["rL"][r].get("spatialMethod", "Full") == "GPP":
                Eta[r] = _eta_spatial_gpp(st, model, r, S, dp, rng, it, zero_noise)
            else:
                Eta[r] = _eta_spatial_full(st, model, r, S, dp, rng, it, zero_noise)
            continue
        precs, means = eta_unit_moments_x(st, model, r, S) if _xdim(model, r) else eta_unit_moments(st, model, r, S)
        npr, nf = means.shape
        RiV = np.swapaxes(np.linalg.cholesky(precs), 1, 2)              # chol(): upper R, R'R = Q
        if zero_noise:
            xi = np.zeros((npr, nf))
        else:
            xi = rng.normal(np.arange(npr)[:, None], np.arange(nf)[None, :], R.S_ETA + R.LEVEL_STRIDE * _vlev(model, r), it)
        Eta[r] = means + np.linalg.solve(RiV, xi[:, :, None])[:, :, 0]  # backsolve(RiV, xi)  :56,69,90
    return Eta


# ---------------------------------------------------------------------------
# updateInvSigma — R/updateInvSigma.R:3-43
# ---------------------------------------------------------------------------
def update_inv_sigma(st, model, rng, it):
    distr = model["distr"]
    iS = st["iSigma"].copy()
    ind = distr[:, 1] == 1                                             # :4
    if ind.any():
        Y = model["Y"]
        Eps = st["Z"] - linear_predictor(st, model)                    # :31-34
        Yx = ~np.isnan(Y)
        shape = model["aSigma"] + Yx.sum(axis=0) / 2                   # :37-38
        rate = model["bSigma"] + np.sum(np.where(Yx, Eps, 0.0) ** 2, axis=0) / 2   # :39
        j = np.nonzero(ind)[0]
        iS[j] = rng.gamma(j, R.S_INVSIGMA, it, shape[j], rate[j])      # :40
    return iS


# ---------------------------------------------------------------------------
# updateNf — R/updateNf.R:3-70 (reproduces the setdiff(1:nf, logical) quirk, :56)
# ---------------------------------------------------------------------------
def update_nf(st, model, r, rng, it):
    rl = model["rL"][r]
    eta, lam, psi, delta, alpha = (st["Eta"][r], st["Lambda"][r], st["Psi"][r],
                                   st["Delta"][r], st["Alpha"][r])
    c0, c1, epsilon, prop = 1.0, 0.0005, 1e-3, 1.0                      # :10-13
    prob = 1 / np.exp(c0 + c1 * it)
    v0 = _vlev(model, r)
    stream = R.LEVEL_STRIDE * v0
    u = rng.uniforms(0, 0, R.S_NF + stream, it)[0]
    xd = _xdim(model, r)
    if u < prob:                                                       # :16
        ns = lam.shape[1]
        nf = lam.shape[0]
        npr = eta.shape[0]
        small = np.abs(lam) < epsilon
        smallProp = small.reshape(nf, -1).mean(axis=1)                 # rowMeans (over ns, and ncr)
        indRedundant = smallProp >= prop
        numRedundant = int(indRedundant.sum())
        if nf < rl["nfMax"] and it > 20 and numRedundant == 0 and np.all(smallProp < 0.995):
            nf += 1                                                    # :26-54
            eta = np.concatenate([eta, rng.normal(np.arange(npr), 0, R.S_NF_ETA + stream, it)[:, None]], axis=1)
            alpha = np.concatenate([alpha, [1]])
            if not xd:
                lam = np.concatenate([lam, np.zeros((1, ns))], axis=0)
                newpsi = rng.gamma(np.arange(ns), R.S_NF_PSI + stream, it, rl["nu"] / 2, rl["nu"] / 2)
                psi = np.concatenate([psi, newpsi[None, :]], axis=0)
                delta = np.concatenate([delta, [rng.gamma(0, R.S_NF_DELTA + stream, it, rl["a2"], rl["b2"])]])
            else:                                                      # :41-47, column k on level v0 + k
                lam = np.concatenate([lam, np.zeros((1, ns, xd))], axis=0)
                newpsi = np.stack([rng.gamma(np.arange(ns), R.S_NF_PSI + R.LEVEL_STRIDE * (v0 + k), it,
                                             _prior(rl, "nu", k) / 2, _prior(rl, "nu", k) / 2) for k in range(xd)], axis=1)
                psi = np.concatenate([psi, newpsi[None]], axis=0)
                newd = [rng.gamma(0, R.S_NF_DELTA + R.LEVEL_STRIDE * (v0 + k), it, _prior(rl, "a2", k),
                                  _prior(rl, "b2", k)) for k in range(xd)]
                delta = np.concatenate([delta, np.asarray(newd)[None, :]], axis=0)
        elif numRedundant > 0 and nf > rl["nfMin"]:                    # :55-68
            # setdiff(1:nf, indRedundant) with a logical vector: TRUE->1, FALSE->0,
            # so factor 1 is dropped whenever any factor is redundant (quirk kept).
            keep = [k for k in range(1, nf + 1) if k not in set(indRedundant.astype(int).tolist())]
            keep = np.array(keep) - 1
            eta, alpha, lam, psi, delta = eta[:, keep], alpha[keep], lam[keep], psi[keep], delta[keep]
    return eta, lam, alpha, psi, delta


# ---------------------------------------------------------------------------
# computeInitialParameters — R/computeInitialParameters.R:17-273 (initPar=NULL)
# ---------------------------------------------------------------------------
def compute_initial_parameters(model, rng, nf=None):
    it = 0
    X, Tr, distr = model["X"], model["Tr"], model["distr"]
    nc, nt, ns = X.shape[1], Tr.shape[1], Tr.shape[0]
    LU = np.linalg.cholesky(model["UGamma"])
    Gamma = (model["mGamma"] + LU @ rng.normal(np.arange(nc * nt), 0, R.S_INIT_GAMMA, it)).reshape(nc, nt, order="F")  # :85
    iV0 = np.linalg.inv(model["V0"])
    V = np.linalg.inv(rwish(model["f0"], iV0, rng, it, R.S_INIT_V_DIAG, R.S_INIT_V_OFF))   # :91 riwish
    Mu = Gamma @ Tr.T
    LV = np.linalg.cholesky(V)
    jj, kk = np.meshgrid(np.arange(ns), np.arange(nc))
    Beta = Mu + LV @ rng.normal(jj, kk, R.S_INIT_BETA, it)             # :97-101
    sigma = np.ones(ns)                                                # :111-126
    for j in range(ns):
        if distr[j, 1] == 1:
            sigma[j] = rng.gamma(j, R.S_INIT_SIGMA, it, model["aSigma"][j], model["bSigma"][j])
        elif distr[j, 0] == 3:
            sigma[j] = 1e-2
    Eta, Lambda, Psi, Delta, Alpha = [], [], [], [], []
    for r, rl in enumerate(model["rL"]):
        nfr = int(rl["nfMin"]) if nf is None else int(nf[r])
        v0 = _vlev(model, r)
        s = R.LEVEL_STRIDE * v0
        hh, jj2 = np.meshgrid(np.arange(nfr), np.arange(ns), indexing="ij")
        xd = _xdim(model, r)
        blocks = []
        for k in range(max(xd, 1)):  # covariate-dependent levels: column k of Delta / Psi / Lambda on device level v0 + k
            sk = R.LEVEL_STRIDE * (v0 + k)
            d = np.empty(nfr)
            d[0] = rng.gamma(0, R.S_INIT_DELTA + sk, it, _prior(rl, "a1", k), _prior(rl, "b1", k))   # :175,177
            if nfr > 1:
                d[1:] = rng.gamma(np.arange(1, nfr), R.S_INIT_DELTA + sk, it, _prior(rl, "a2", k), _prior(rl, "b2", k))
            nu = _prior(rl, "nu", k)
            psi = rng.gamma(hh + nfr * jj2, R.S_INIT_PSI + sk, it, nu / 2, nu / 2)  # :183,185
            tau = np.cumprod(d)
            lam = rng.normal(hh + nfr * jj2, 0, R.S_INIT_LAMBDA + sk, it) * np.sqrt(psi * tau[:, None]) ** -1  # :189-198
            blocks.append((d, psi, lam))
        if xd:
            d = np.stack([b[0] for b in blocks], axis=1)
            psi = np.stack([b[1] for b in blocks], axis=2)
            lam = np.stack([b[2] for b in blocks], axis=2)
        else:
            d, psi, lam = blocks[0]
        npr = int(model["np"][r])
        qq, kk2 = np.meshgrid(np.arange(npr), np.arange(nfr), indexing="ij")
        eta = rng.normal(qq, kk2, R.S_INIT_ETA + s, it)                # :207
        Eta.append(eta), Lambda.append(lam), Psi.append(psi), Delta.append(d)
        Alpha.append(np.ones(nfr, dtype=np.int64))
    st = dict(Gamma=Gamma, iV=np.linalg.inv(V), V=V, Beta=Beta, iSigma=1.0 / sigma, Eta=Eta,
              Lambda=Lambda, Psi=Psi, Delta=Delta, Alpha=Alpha, rho=1)
    st["Z"] = update_z(st, model, rng, it, Y=model.get("Yraw", model["Y"]))   # :254 uses hM$Y
    return st


# ---------------------------------------------------------------------------
# one sweep — R/sampleMcmc.R:219-306 (fixed block order)
# ---------------------------------------------------------------------------
def sweep(st, model, rng, it, updater=None, data_par=None, adapt_nf=None):
    up = updater or {}
    on = lambda name: up.get(name, True) is not False                  # noqa: E731  identical(x, FALSE)
    st = dict(st)
    nr = model["Pi"].shape[1]
    if on("Gamma2"):
        st["Gamma"] = update_gamma2(st, model, rng, it)
    if on("GammaEta"):
        st["Gamma"], st["Eta"] = update_gamma_eta(st, model, rng, it, data_par)
    if on("BetaLambda"):
        st["Beta"], st["Lambda"] = update_beta_lambda(st, model, rng, it, data_par)
    if on("GammaV"):
        st["Gamma"], st["iV"] = update_gamma_v(st, model, rng, it, data_par)
    if model.get("C") is not None and on("Rho"):
        st["rho"] = update_rho(st, model, rng, it, data_par)
    if on("LambdaPriors"):
        st["Psi"], st["Delta"] = update_lambda_priors(st, model, rng, it)
    if on("Eta"):
        st["Eta"] = update_eta(st, model, rng, it, data_par=data_par)
    if on("Alpha") and any(rl.get("sDim", 0) for rl in model["rL"]):
        st["Alpha"] = update_alpha(st, model, rng, it, data_par)
    if on("InvSigma"):
        st["iSigma"] = update_inv_sigma(st, model, rng, it)
    if on("Z"):
        st["Z"] = update_z(st, model, rng, it)
    for r in range(nr):                                                # :296-306
        if adapt_nf is not None and it <= adapt_nf[r]:
            e, l, a, p, d = update_nf(st, model, r, rng, it)
            st["Eta"] = list(st["Eta"]); st["Eta"][r] = e
            st["Lambda"] = list(st["Lambda"]); st["Lambda"][r] = l
            st["Alpha"] = list(st["Alpha"]); st["Alpha"][r] = a
            st["Psi"] = list(st["Psi"]); st["Psi"][r] = p
            st["Delta"] = list(st["Delta"]); st["Delta"][r] = d
    return st


# ---------------------------------------------------------------------------
# updateGammaEta — R/updateGammaEta.R:7-206 (non-spatial levels, xDim = 0)
# Gamma and Eta_r given Z with Beta integrated out, level by level; Beta is drawn as an
# auxiliary and discarded (the function returns only Gamma and Eta).  Randomness: Beta's
# rnorm(nc*ns) is normal(c + nc*j, 0, S_GE_BETA), Gamma's normal(c + nc*t, 0, S_GE_GAMMA),
# Eta's rnorm(ny*nf) / rnorm(np*nf) normal(row i (np == ny) or unit p, h, S_GE_ETA), each
# plus LEVEL_STRIDE * r.
# ---------------------------------------------------------------------------
def _spatial_pieces(st, model, r, S, dp):
    X, Tr = model["X"], model["Tr"]
    lam, idv = st["Lambda"][r], st["iSigma"]
    ny = X.shape[0]
    npr = int(model["np"][r])
    P = np.zeros((ny, npr))
    P[np.arange(ny), model["Pi"][:, r] - 1] = 1.0
    alpha = np.asarray(st["Alpha"][r], dtype=np.int64) - 1
    iWg = dp["rLPar"][r]["iWg"]
    iK = np.zeros((npr * lam.shape[0],) * 2)
    for h, a in enumerate(alpha):
        iK[h * npr:(h + 1) * npr, h * npr:(h + 1) * npr] = iWg[a]
    return X, Tr, lam, idv, P, iK


def gamma_eta_spatial_literal(st, model, r, S, dp, iQ, iV, U, iU, iA):
    """R/updateGammaEta.R:139-194 ('Full' spatial level) as written: the mean (mg, me)
    through W = iK + kron(Lam iD Lam', P'P), M = iA + kron(iD, X'X) - ..., and the joint
    precision iG = bdiag(iU, iK) + iG2 - iG3 of (vec Gamma, vec Eta).  K = bdiag(Wg) is
    applied as a solve with iK (K = iK^-1).  Returns (m, iG)."""
    X, Tr, lam, idv, P, iK = _spatial_pieces(st, model, r, S, dp)
    nc, nt, ns = X.shape[1], Tr.shape[1], S.shape[1]
    XtX, XtS = X.T @ X, X.T @ S
    LamiD = lam * idv[None, :]
    LamiDLam = (lam * np.sqrt(idv)[None, :]) @ (lam * np.sqrt(idv)[None, :]).T
    iDT = idv[:, None] * Tr
    iD05T = np.sqrt(idv)[:, None] * Tr
    iD05Lamt = np.sqrt(idv)[:, None] * lam.T
    PtX = P.T @ X
    PtP = np.diag(P.sum(axis=0))
    LamiDLam_PtP = np.kron(LamiDLam, PtP)                                    # :145
    LamiD_PtX = np.kron(LamiD, PtX)
    LamiDT_PtX = np.kron(LamiD @ Tr, PtX)
    iDT_XtX = np.kron(iDT, XtX)
    RW = chol_upper(iK + LamiDLam_PtP)                                       # :160-161
    iLW = backsolve(RW, LamiD_PtX, transpose=True)                           # :163
    iDL = iLW.T @ iLW
    RM = chol_upper(iA + np.kron(np.diag(idv), XtX) - iDL)                  # :165-166
    mg10 = (XtS @ iDT).ravel(order="F")                                      # :168
    mg21 = ((P.T @ S) @ LamiD.T).ravel(order="F")
    mg22 = backsolve(RW, backsolve(RW, mg21, transpose=True))
    mg20 = LamiDT_PtX.T @ mg22
    mg31 = (XtS * idv[None, :]).ravel(order="F") - LamiD_PtX.T @ mg22
    mg32 = backsolve(RM, backsolve(RM, mg31, transpose=True))
    tmp1 = iDT_XtX - iDL @ np.kron(Tr, np.eye(nc))                           # :174
    mg = U @ (mg10 - mg20 - tmp1.T @ mg32)                                   # :175-176
    me20 = LamiDLam_PtP @ mg22                                               # :178-181
    me30 = LamiD_PtX @ mg32 - LamiDLam_PtP @ backsolve(RW, iLW @ mg32)
    me = np.linalg.solve(iK, mg21 - me20 - me30)
    H = np.kron(iQ, iV) + np.kron(np.diag(idv), XtX)                         # :183
    nE = iK.shape[0]
    iG1 = np.zeros((nc * nt + nE,) * 2)
    iG1[:nc * nt, :nc * nt] = iU
    iG1[nc * nt:, nc * nt:] = iK
    Gm = np.hstack([np.kron(iD05T, X), np.kron(iD05Lamt, P)])                # :185
    tmp = backsolve(chol_upper(H), np.hstack([iDT_XtX, LamiD_PtX.T]), transpose=True)
    return np.r_[mg, me], iG1 + Gm.T @ Gm - tmp.T @ tmp


def gamma_eta_spatial_natural(st, model, r, S, dp, iQ, iV, iU):
    """The same joint conditional in natural form, as the device computes it
    (hmsc_amd/csrc/gamma_eta.hip gamma_eta_spatial_kernel): with H = kron(iQ, iV) +
    kron(iD, X'X) and C = [kron(iD Tr, X'X), t(kron(Lam iD, P'X))] (the Woodbury factors of
    the B-integrated likelihood), mean = iG^-1 (c0 - C' H^-1 vec(X'S iD)),
    c0 = [vec(X'S iD Tr); vec(P'S iD Lam')].  Returns (m, iG)."""
    X, Tr, lam, idv, P, iK = _spatial_pieces(st, model, r, S, dp)
    nc, nt = X.shape[1], Tr.shape[1]
    XtX, XtS = X.T @ X, X.T @ S
    LamiD = lam * idv[None, :]
    LH = np.linalg.cholesky(np.kron(iQ, iV) + np.kron(np.diag(idv), XtX))
    C = np.hstack([np.kron(idv[:, None] * Tr, XtX), np.kron(LamiD, P.T @ X).T])
    tmp = solve_triangular(LH, C, lower=True)
    y = solve_triangular(LH, (XtS * idv[None, :]).ravel(order="F"), lower=True)
    c0 = np.r_[(XtS @ (idv[:, None] * Tr)).ravel(order="F"), ((P.T @ S) @ LamiD.T).ravel(order="F")]
    Gm = np.hstack([np.kron(np.sqrt(idv)[:, None] * Tr, X), np.kron(np.sqrt(idv)[:, None] * lam.T, P)])
    iG = Gm.T @ Gm - tmp.T @ tmp
    iG[:nc * nt, :nc * nt] += iU
    iG[nc * nt:, nc * nt:] += iK
    return np.linalg.solve(iG, c0 - tmp.T @ y), iG


def update_gamma_eta(st, model, rng, it, data_par=None, zero_noise=False):
    X, Tr, Pi, Z = model["X"], model["Tr"], model["Pi"], st["Z"]
    ny, ns = Z.shape
    nc, nt, nr = X.shape[1], Tr.shape[1], Pi.shape[1]
    dp = data_par if data_par is not None else compute_data_parameters(model)
    g = st.get("rho", 1) - 1 if model.get("C") is not None else 0
    Q, iQ, RQ = dp["Qg"][g], dp["iQg"][g], dp["RQg"][g]
    iV = st["iV"]
    V = chol2inv(chol_upper(iV))
    U = model["UGamma"]
    iU = chol2inv(chol_upper(U))
    idv = st["iSigma"]
    lam_all = st["Lambda"]
    LRan = [eta_full(st, model, r) @ lam_all[r] for r in range(nr)]          # :15-26
    Eta = [e.copy() for e in st["Eta"]]
    Gamma = st["Gamma"]
    XtX = X.T @ X
    KT = np.kron(Tr, np.eye(nc))
    A = KT @ U @ KT.T + np.kron(Q, V)                                         # :32
    iA = chol2inv(chol_upper(A))                                              # :33

    def nrm(idx, sub, stream, shape):
        if zero_noise:
            return np.zeros(shape)
        return rng.normal(idx, sub, stream, it).reshape(shape, order="F")

    for r in range(nr):
        rl = model["rL"][r]
        if rl.get("xDim", 0):
            raise NotImplementedError("updateGammaEta: covariate-dependent levels (SURVEY.md §8 f2)")
        s = R.LEVEL_STRIDE * r
        S = Z - sum(LRan[q] for q in range(nr) if q != r) if nr > 1 else Z  # :37-42
        if rl.get("sDim", 0):                                                 # :139-198
            if rl.get("spatialMethod", "Full") != "Full":
                raise ValueError("updataGammaEta: no method implemented yet for NNGP / GPP with GammaEta updater")
            mvec, iG = gamma_eta_spatial_literal(st, model, r, S, dp, iQ, iV, U, iU, iA)
            D2 = iG.shape[0]
            RG = chol_upper(iG)
            ge = mvec + backsolve(RG, nrm(np.arange(D2), 0, R.S_GE_GAMMA + s, D2))   # :193-194
            Gamma = ge[:nc * nt].reshape((nc, nt), order="F")
            Eta[r] = ge[nc * nt:].reshape((int(model["np"][r]), -1), order="F")
            LRan[r] = Eta[r][Pi[:, r] - 1] @ lam_all[r]
            continue
        lam = lam_all[r]
        nf = lam.shape[0]
        lPi = Pi[:, r] - 1
        npr = int(model["np"][r])
        LamiD = lam * idv[None, :]
        LamiDLam = (lam * np.sqrt(idv)[None, :]) @ (lam * np.sqrt(idv)[None, :]).T
        XtS = X.T @ S
        mb10 = (XtS * idv[None, :]).ravel(order="F")
        jj, cc = np.meshgrid(np.arange(ns), np.arange(nc))
        xi_b = nrm((cc + nc * jj).ravel(order="F"), 0, R.S_GE_BETA + s, nc * ns)
        if npr == ny:                                                         # :51-75
            W0 = LamiDLam + np.eye(nf)
            RW0 = chol_upper(W0)
            iW0 = chol2inv(RW0)
            iLW0LamiD = backsolve(RW0, LamiD, transpose=True)
            tmp1 = np.diag(idv) - iLW0LamiD.T @ iLW0LamiD
            K1 = np.kron(tmp1, XtX)
            M = iA + K1
            RM = chol_upper(M)
            mb20 = ((XtS @ LamiD.T) @ iW0 @ LamiD).ravel(order="F")
            mb31 = backsolve(RM, backsolve(RM, mb10 - mb20, transpose=True))
            mb30 = K1 @ mb31
            mb = A @ (mb10 - mb20 - mb30)
            Beta = (mb + backsolve(RM, xi_b)).reshape((nc, ns), order="F")
        else:                                                                 # :76-150
            P = np.zeros((ny, npr))
            P[np.arange(ny), lPi] = 1.0
            PtX = P.T @ X
            colSumP = P.sum(axis=0)
            iWs, LiWs = [], []
            for q in range(npr):
                Wp = np.eye(nf) + colSumP[q] * LamiDLam
                RWp = chol_upper(Wp)
                iWs.append(chol2inv(RWp))
                LiWs.append(np.linalg.solve(RWp, np.eye(nf)))
            # W, iW, LiW are block-diagonal in the (p + np h) ordering of vec(np x nf)
            LiW = np.zeros((nf * npr, nf * npr))
            iW = np.zeros((nf * npr, nf * npr))
            for q in range(npr):
                ix = q + npr * np.arange(nf)
                LiW[np.ix_(ix, ix)] = LiWs[q]
                iW[np.ix_(ix, ix)] = iWs[q]
            LamiD_PtX = np.kron(LamiD, PtX)
            iLW = LiW.T @ LamiD_PtX
            tmp1 = np.kron(np.diag(idv), XtX) - iLW.T @ iLW
            M = iA + tmp1
            RM = chol_upper(M)
            mb21 = ((P.T @ S) @ LamiD.T).ravel(order="F")
            mb22 = iW @ mb21
            mb20 = (PtX.T @ mb22.reshape((npr, nf), order="F") @ LamiD).ravel(order="F")
            mb31 = backsolve(RM, backsolve(RM, mb10 - mb20, transpose=True))
            mb30 = tmp1 @ mb31
            mb = A @ (mb10 - mb20 - mb30)
            Beta = (mb + backsolve(RM, xi_b)).reshape((nc, ns), order="F")
        # Gamma | Beta  (:66-69 / :130-133)
        TQT = backsolve(RQ, Tr, transpose=True)
        RG = chol_upper(iU + np.kron(TQT.T @ TQT, iV))
        mg = chol2inv(RG) @ ((iV @ Beta) @ (iQ @ Tr)).ravel(order="F")
        tt, cg = np.meshgrid(np.arange(nt), np.arange(nc))
        xi_g = nrm((cg + nc * tt).ravel(order="F"), 0, R.S_GE_GAMMA + s, nc * nt)
        Gamma = (mg + backsolve(RG, xi_g)).reshape((nc, nt), order="F")
        # Eta | Beta, S
        S1 = S - X @ Beta
        if npr == ny:                                                         # :71-74
            me = S1 @ LamiD.T @ iW0
            hh, ii = np.meshgrid(np.arange(nf), np.arange(ny))
            xi = nrm(ii.ravel(order="F"), hh.ravel(order="F"), R.S_GE_ETA + s, (ny, nf))
            E = np.empty((ny, nf))
            E[lPi, :] = me + backsolve(RW0, xi.T).T
            Eta[r] = E
        else:                                                                 # :136-146
            PtS1 = P.T @ S1
            me10 = (PtS1 @ LamiD.T).ravel(order="F")
            me21 = iW @ me10
            me20 = (np.diag(colSumP) @ me21.reshape((npr, nf), order="F") @ LamiDLam).ravel(order="F")
            me = me10 - me20
            hh, qq = np.meshgrid(np.arange(nf), np.arange(npr))
            xi = nrm(qq.ravel(order="F"), hh.ravel(order="F"), R.S_GE_ETA + s, nf * npr)
            Eta[r] = (me + LiW @ xi).reshape((npr, nf), order="F")
        LRan[r] = Eta[r][lPi, :] @ lam                                        # :201
    return Gamma, Eta


# ---------------------------------------------------------------------------
# updateRho — R/updateRho.R:1-25 (phylogeny grid; categorical by inverse CDF)
# ---------------------------------------------------------------------------
def update_rho(st, model, rng, it, data_par):
    Beta, Gamma, iV, Tr = st["Beta"], st["Gamma"], st["iV"], model["Tr"]
    rhopw = model["rhopw"]
    nc = Beta.shape[0]
    E = (Beta - Gamma @ Tr.T).T
    RiV = chol_upper(iV)
    E = E @ RiV.T                                                      # tcrossprod(E, RiV)
    v = np.array([np.sum(backsolve(data_par["RQg"][g], E, transpose=True) ** 2)
                  for g in range(rhopw.shape[0])])
    logLike = np.log(rhopw[:, 1]) - 0.5 * nc * data_par["detQg"] - 0.5 * v
    like = np.exp(logLike - logLike.max())
    u = rng.uniforms(0, 0, R.S_RHO, it)[0]
    return int(np.searchsorted(np.cumsum(like), u * like.sum(), side="right")) + 1


# ---------------------------------------------------------------------------
# predict.Hmsc per-sample loop — R/predict.R:143-229 (device: hmsc_amd/csrc/predict.hip)
# ---------------------------------------------------------------------------
S_PREDICT = 30


def _rpois_ptrs(lam, rng, cell, s):
    """numpy's PTRS (Hormann 1993) for lam >= 10, sequential inversion below; trial t uses
    the uniforms of (cell, 1 + t, S_PREDICT, s) -- the rpois of R/predict.R:216 restated with
    the Philox counter contract."""
    if not lam > 0:
        return 0.0
    if lam < 10:
        u = rng.uniforms(cell, 1, S_PREDICT, s)[0]
        p = c = np.exp(-lam)
        k = 0
        while u > c and k < 1000:
            k += 1
            p *= lam / k
            c += p
        return float(k)
    from math import floor, lgamma, log, sqrt
    slam, loglam = sqrt(lam), log(lam)
    b = 0.931 + 2.53 * slam
    a = -0.059 + 0.02483 * b
    invalpha = 1.1239 + 1.1328 / (b - 3.4)
    vr = 0.9277 - 3.6224 / (b - 2.0)
    for t in range(256):
        ua, ub = rng.uniforms(cell, 1 + t, S_PREDICT, s)
        U, V = float(ua) - 0.5, float(ub)
        us = 0.5 - abs(U)
        k = floor((2 * a / us + b) * U + lam + 0.43)
        if us >= 0.07 and V <= vr:
            return float(k)
        if k < 0 or (us < 0.013 and V > us):
            continue
        if log(V) + log(invalpha) - log(a / (us * us) + b) <= -lam + k * loglam - lgamma(k + 1.0):
            return float(k)
    return float(floor(lam))


def predict_samples(X, post, PiNew, family, YScalePar, expected, rng):
    """post: list of dict(Beta nc x ns, sigma ns, Eta [np_r x nf_r] (prediction units),
    Lambda [nf_r x ns]); PiNew ny x nr (1-based).  Returns the list of ny x ns predictions."""
    from scipy.special import ndtr
    ny, ns = X.shape[0], post[0]["Beta"].shape[1]
    out = []
    cells = (np.arange(ny)[:, None] + ny * np.arange(ns)[None, :]).astype(np.uint64)
    for s, sam in enumerate(post):
        L = X @ sam["Beta"]
        for r in range(PiNew.shape[1]):
            L = L + sam["Eta"][r][PiNew[:, r] - 1] @ sam["Lambda"][r]
        sg = np.asarray(sam["sigma"], dtype=np.float64)
        if expected:
            Z = L.copy()
            Z[:, family == 2] = ndtr(L[:, family == 2])
            Z[:, family == 3] = np.exp(L[:, family == 3] + sg[family == 3] / 2)
        else:
            Z = L + np.sqrt(sg)[None, :] * rng.normal(cells, 0, S_PREDICT, s)
            Z[:, family == 2] = (Z[:, family == 2] > 0).astype(float)
            for j in np.nonzero(family == 3)[0]:
                Z[:, j] = [_rpois_ptrs(float(np.exp(Z[i, j])), rng, int(cells[i, j]), s) for i in range(ny)]
        m, sd = YScalePar[0], YScalePar[1]
        tr = (m != 0) | (sd != 1)
        Z[:, tr] = Z[:, tr] * sd[tr] + m[tr]
        out.append(Z)
    return out
