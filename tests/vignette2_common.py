"""Shared by tests/golden/make_vignette2_fixture.py (CPU oracle side) and
tests/test_gpu_vignette2.py (device side): BASELINE.json config 2, the models of
vignettes/vignette_2_multivariate_low.Rmd (hmsc_amd.workloads.vignette2), with the
reference's default updater set for each (R/sampleMcmc.R:124-152: GammaEta switches itself
off when nr == 0, and is ON for the sample-level model).

Per model: chains start from one converged oracle state, run TRANSIENT sweeps, then record
SAMPLES samples every THIN sweeps.  Statistics (scaled space, sign invariant): Beta
(covariate-fastest), Gamma, the upper triangle of V = iV^-1, sigma of the normal species,
and for a random level the upper triangle of Omega = Lambda' Lambda.
"""
import numpy as np

import hmsc_amd as H
from oracle import post_oracle as P

MODELS = ("linear", "mixed", "latent")
# updaters as the reference's defaults resolve them for each model (GammaEta off for nr == 0)
UPDATER = {"linear": {"GammaEta": False}, "mixed": {"GammaEta": False}, "latent": {}}
THIN = {"linear": 1, "mixed": 4, "latent": 1}
N_CHAINS = 4
TRANSIENT = 200
SAMPLES = 1500
THIN_STORE = 6
START_SEED, START_SWEEPS = 4321, 500

STATE_KEYS = ("Gamma", "iV", "Beta", "iSigma", "Z", "Eta", "Lambda", "Psi", "Delta")


def model(name):
    from hmsc_amd.workloads import vignette2
    return vignette2(name)


def pack_state(st, prefix, nr):
    out = {}
    for k in STATE_KEYS:
        v = st[k]
        if isinstance(v, list):
            for r in range(nr):
                out[f"{prefix}/{k}/{r}"] = np.asarray(v[r])
        else:
            out[f"{prefix}/{k}"] = np.asarray(v)
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


def param_vector(hM, rec):
    """(S, P) statistics of one chain; rec: Beta (S,nc,ns), Gamma (S,nc,nt), iV (S,nc,nc),
    iSigma (S,ns) and, for nr == 1, Lambda0 (S,nf,ns)."""
    S = rec["Beta"].shape[0]
    iu = np.triu_indices(hM.nc)
    V = np.linalg.inv(rec["iV"])
    normal = np.asarray(hM.distr)[:, 0] == 1
    cols = [rec["Beta"].transpose(0, 2, 1).reshape(S, -1), rec["Gamma"].transpose(0, 2, 1).reshape(S, -1),
            V[:, iu[0], iu[1]], 1.0 / rec["iSigma"][:, normal]]
    if hM.nr:
        lam = rec["Lambda0"]
        om = np.einsum("shi,shj->sij", lam, lam)
        ju = np.triu_indices(hM.ns)
        cols.append(om[:, ju[0], ju[1]])
    return np.concatenate(cols, axis=1)


def summarise(hM, chains):
    vecs = [param_vector(hM, r) for r in chains]
    return dict(draws=np.stack([v[::THIN_STORE] for v in vecs]).astype(np.float32),
                mean=np.stack([v.mean(axis=0) for v in vecs]),
                sd=np.stack([v.std(axis=0, ddof=1) for v in vecs]),
                ess=np.stack([P.effectiveSize(v) for v in vecs]))
