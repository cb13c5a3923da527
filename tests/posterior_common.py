"""Shared by tests/golden/make_posterior_fixture.py (CPU oracle side) and
tests/test_gpu_posterior.py (GPU side): the models, chain lengths and the summary of a
set of chains (draws of Beta / Gamma / Omega, their means, sds, ESS, and the variance
partitioning)."""
import numpy as np

import hmsc_amd as H
from oracle import post_oracle as P

MODELS = {
    # probit with traits: Gamma2 acts (all iSigma == 1), GammaV, MGP priors, Eta
    "probit_traits": dict(ny=150, ns=12, nc=3, nf=2, nt=2, seed=21),
    # normal + probit species with NA cells: InvSigma acts, Gamma from GammaV only
    "mixed_na": dict(ny=120, ns=10, nc=3, nf=2, n_normal=3, na_frac=0.04, seed=22),
    # Poisson + lognormal Poisson + probit (Polya-Gamma updateZ, InvSigma on the lognormal ones)
    "poisson_mixed": dict(ny=120, ns=10, nc=3, nf=2, n_poisson=4, n_lognormal=3, seed=23),
}
# models that mix slowly record every THIN-th sweep (same number of recorded samples): with
# iSigma = 100 fixed for Poisson species (R/computeInitialParameters.R:122) Z moves little per
# sweep, so Beta's autocorrelation is long on both sides alike
THIN = {"poisson_mixed": 4}
N_CHAINS = 4
TRANSIENT = 200
SAMPLES = 1500
THIN_STORE = 6
START_SEED, START_SWEEPS = 999, 500   # every chain starts from this converged oracle state

STATE_KEYS = ("Gamma", "iV", "Beta", "iSigma", "Z", "Eta", "Lambda", "Psi", "Delta")


def pack_state(st, prefix):
    """state dict -> flat {prefix/key[/r]: array} for the npz fixture."""
    out = {}
    for k in STATE_KEYS:
        if isinstance(st[k], list):
            for r, a in enumerate(st[k]):
                out[f"{prefix}/{k}/{r}"] = np.asarray(a)
        else:
            out[f"{prefix}/{k}"] = np.asarray(st[k])
    return out


def unpack_state(npz, prefix, nr):
    st = {}
    for k in STATE_KEYS:
        if f"{prefix}/{k}" in npz:
            st[k] = np.array(npz[f"{prefix}/{k}"])
        else:
            st[k] = [np.array(npz[f"{prefix}/{k}/{r}"]) for r in range(nr)]
    st["Alpha"] = [np.ones(st["Lambda"][r].shape[0], dtype=np.int64) for r in range(nr)]
    st["rho"] = 1
    return st


def param_vector(rec):
    """(S, P): Beta (covariate-fastest), Gamma, upper triangle of Omega = Lambda' Lambda."""
    S = rec["Beta"].shape[0]
    lam = rec["Lambda0"]
    om = np.einsum("shi,shj->sij", lam, lam)
    iu = np.triu_indices(om.shape[1])
    return np.concatenate([rec["Beta"].reshape(S, -1, order="C").reshape(S, -1),
                           rec["Gamma"].reshape(S, -1), om[:, iu[0], iu[1]]], axis=1)


def variance_partitioning(hM, rec):
    """computeVariancePartitioning on one chain, after combineParameters' un-scaling."""
    S = rec["Beta"].shape[0]
    nf = rec["Lambda0"].shape[1]
    full = dict(Beta=rec["Beta"], Gamma=rec["Gamma"], iV=rec["iV"], iSigma=rec["iSigma"],
                rho=np.ones(S, dtype=np.int64), nf=[np.full(S, nf)],
                Eta0=np.zeros((S, hM.np[0], nf)), Lambda0=rec["Lambda0"], Psi0=np.ones_like(rec["Lambda0"]),
                Delta0=np.ones((S, nf)), Alpha0=np.ones((S, nf), dtype=np.int64))
    post = H.combine_parameters(full, hM)
    hM.postList = [post]
    hM.samples = S
    return P.computeVariancePartitioning(hM)["vals"]


def summarise(hM, chains):
    """chains: list of rec dicts (Beta (S,nc,ns), Gamma (S,nc,nt), iV, iSigma, Lambda0 (S,nf,ns))."""
    vecs = [param_vector(r) for r in chains]
    return dict(
        draws=np.stack([v[::THIN_STORE] for v in vecs]).astype(np.float32),
        mean=np.stack([v.mean(axis=0) for v in vecs]),
        sd=np.stack([v.std(axis=0, ddof=1) for v in vecs]),
        ess=np.stack([P.effectiveSize(v) for v in vecs]),
        vp=np.stack([variance_partitioning(hM, r) for r in chains]),
    )
