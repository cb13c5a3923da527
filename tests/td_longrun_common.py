"""Shared by tests/golden/make_td_longrun_fixture.py (CPU oracle side) and
tests/test_gpu_td_posterior.py (device side): the TD$m spec's long-run posterior summary.

TD$m (data-raw/simulateTestData.R:60-70) is sampled with the reference's default updater
set -- GammaEta on (its spatial 'Full' branch with phylogeny, R/updateGammaEta.R:139-198),
Rho, Alpha -- or with GammaEta off.  Every statistic is in the sampler's own (scaled)
parameterisation and invariant to the sign of a latent factor:
Beta (covariate-fastest), Gamma, V = iV^-1, rho (rhopw value), Omega_r = Lambda_r' Lambda_r
(upper triangle, both levels), and the spatial scale alphapw[Alpha] of both plot factors.
Per chain: mean, variance and coda::effectiveSize (hmsc_amd.post.effectiveSize, the
spectrum0.ar restatement); pooled: the mean of chain means and its Monte Carlo standard
error sqrt(sum_c var_c / ESS_c) / n_chains.
"""
import numpy as np

TRANSIENT = 1000
SAMPLES = 16000
N_CHAINS = 8
SEED0 = {"on": 7100, "off": 7200, "short": 50000}   # oracle chain c uses Rng(SEED0[mode] + c)
# the reference's own protocol for TD$m (data-raw/simulateTestData.R:70): 2 chains of
# transient 50 + samples 100; N_SHORT oracle chains give the sampling distribution of its means
SHORT_TRANSIENT, SHORT_SAMPLES, N_SHORT = 50, 100, 128
THIN_STORE = 40                     # thinned draws kept in the fixture (float32)


def names(hM):
    nc, nt, ns = hM.nc, hM.nt, hM.ns
    out = [f"Beta[{c},{j}]" for j in range(ns) for c in range(nc)]
    out += [f"Gamma[{c},{t}]" for t in range(nt) for c in range(nc)]
    iu = np.triu_indices(nc)
    out += [f"V[{a},{b}]" for a, b in zip(*iu)]
    out += ["rho"]
    ju = np.triu_indices(ns)
    for r in range(hM.nr):
        out += [f"Omega{r}[{a},{b}]" for a, b in zip(*ju)]
    for r in range(hM.nr):
        if hM.rL[r].sDim:
            out += [f"alpha{r}[{h}]" for h in range(int(hM.rL[r].nfMax))]
    return out


def param_rows(hM, Beta, Gamma, iV, rho_idx, Lambdas, Alphas):
    """(S, P) rows from per-sample arrays: Beta (S,nc,ns), Gamma (S,nc,nt), iV (S,nc,nc),
    rho_idx (S,) 1-based, Lambdas[r] (S,nf,ns), Alphas[r] (S,nf) 1-based grid indices."""
    S = Beta.shape[0]
    nc = hM.nc
    iu = np.triu_indices(nc)
    V = np.linalg.inv(iV)
    cols = [Beta.transpose(0, 2, 1).reshape(S, -1), Gamma.transpose(0, 2, 1).reshape(S, -1),
            V[:, iu[0], iu[1]], np.asarray(hM.rhopw)[np.asarray(rho_idx) - 1, 0][:, None]]
    ju = np.triu_indices(hM.ns)
    for lam in Lambdas:
        om = np.einsum("shi,shj->sij", lam, lam)
        cols.append(om[:, ju[0], ju[1]])
    for r, al in enumerate(Alphas):
        if hM.rL[r].sDim:
            cols.append(np.asarray(hM.rL[r].alphapw)[np.asarray(al) - 1, 0])
    return np.concatenate(cols, axis=1)


def chain_summary(rows):
    from oracle import post_oracle as P
    return dict(mean=rows.mean(0), var=rows.var(0, ddof=1), ess=P.effectiveSize(rows))


def pooled(means, variances, ess):
    """Mean of chain means and its Monte Carlo standard error (chains independent)."""
    n = means.shape[0]
    se = np.sqrt(np.sum(variances / np.maximum(ess, 1.0), axis=0)) / n
    return means.mean(0), se


def reference_rows(hM, postList):
    """The reference's stored TD$m$postList (combineParameters output: original X / Tr
    scale, R/combineParameters.R:1-58) mapped back to the sampler's scaled parameterisation,
    one (S, P) row block per chain: the inverse of combineParameters' un-scaling."""
    XS, TS = hM.XScalePar, hM.TrScalePar
    XI, TI = hM.XInterceptInd - 1, hM.TrInterceptInd - 1
    out = []
    for ch in postList:
        Bs, Gs, iVs = [], [], []
        for s in ch:
            B, G, V = (np.array(s[k], dtype=np.float64) for k in ("Beta", "Gamma", "V"))
            for k in range(hM.nc):                       # undo :12-26 (X scaling)
                m, sd = XS[0, k], XS[1, k]
                if m != 0 or sd != 1:
                    B[XI] += m * B[k]
                    G[XI] += m * G[k]
                    B[k] *= sd
                    G[k] *= sd
                    V[k, :] *= sd
                    V[:, k] *= sd
            for p in range(hM.nt):                       # undo :2-10 (Tr scaling)
                m, sd = TS[0, p], TS[1, p]
                if m != 0 or sd != 1:
                    G[:, TI] += m * G[:, p]
                    G[:, p] *= sd
            Bs.append(B), Gs.append(G), iVs.append(np.linalg.inv(V))
        rho_idx = np.array([int(np.argmin(np.abs(np.asarray(hM.rhopw)[:, 0] - s["rho"]))) + 1 for s in ch])
        lams = [np.stack([np.asarray(s["Lambda"][r]) for s in ch]) for r in range(hM.nr)]
        alphas = [np.stack([np.asarray(s["Alpha"][r]).ravel() for s in ch]).astype(np.int64) for r in range(hM.nr)]
        out.append(param_rows(hM, np.stack(Bs), np.stack(Gs), np.stack(iVs), rho_idx, lams, alphas))
    return out


def between_chain_t(means_a, means_b):
    """Welch t of two sets of independent chain means (per statistic): the standard error
    comes from the spread of the chain means themselves, which needs no ESS estimate."""
    na, nb = means_a.shape[0], means_b.shape[0]
    se = np.sqrt(means_a.var(0, ddof=1) / na + means_b.var(0, ddof=1) / nb)
    return (means_a.mean(0) - means_b.mean(0)) / np.maximum(se, 1e-300)
