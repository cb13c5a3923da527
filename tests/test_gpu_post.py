"""Post-sampling statistics on the device (hmsc_amd/csrc/post.hip) against
their numpy restatements (oracle/post_oracle.py):
  * coda::effectiveSize (spectrum0.ar): the AR order the AIC picks, equal on >= 99.9 % of the
    columns, and the ESS to 1e-9 relative where the order agrees (orders can only differ on a
    near-tie of two AIC values, which summation order decides);
  * computeVariancePartitioning (R/computeVariancePartitioning.R:37-204) on TD$m's stored
    posterior and on a larger synthetic posterior: vals, R2T.Beta, R2T.Y to 1e-9;
  * computeAssociations (R/computeAssociations.R) and getPostEstimate(.., "Omega"): mean
    correlation / Omega to 1e-12, supports exactly.
"""
import numpy as np
import pytest

import hmsc_amd as H
from helpers import rel_err, synthetic_model
from oracle import post_oracle as P
from test_golden_td import M, td_model, td_postlist

pytestmark = pytest.mark.gpu


def _ar1(n, p, phi, seed):
    rng = np.random.default_rng(seed)
    e = rng.standard_normal((n, p))
    x = np.zeros((n, p))
    for t in range(1, n):
        x[t] = phi * x[t - 1] + e[t]
    return x


@pytest.mark.parametrize("n,p,phi", [(1000, 300, 0.6), (2000, 200, 0.95), (150, 50, 0.0)])
def test_effective_size_matches_restatement(n, p, phi):
    x = _ar1(n, p, phi, seed=n + p)
    x[:, 0] = 3.0                                   # a constant column: ESS 0 on both sides
    x[:, 1] = np.arange(n) * 1e-3 + 1.0             # a pure trend: ESS 0 (spec forced to 0)
    spec_o, ord_o = P.spectrum0_ar(x)
    ess_o = P.effectiveSize(x)
    spec_d, ord_d = H.spectrum0_ar(x)
    ess_d = H.effectiveSize(x)
    same = ord_o == ord_d
    assert np.mean(same) >= 0.999, np.nonzero(~same)
    assert ess_d[0] == 0.0 and ess_d[1] == 0.0
    ok = same & (ess_o > 0)
    assert rel_err(ess_d[ok], ess_o[ok]) < 1e-9


def test_effective_size_chains_sum():
    xs = [_ar1(800, 40, 0.7, seed=s) for s in (1, 2, 3)]
    np.testing.assert_allclose(H.effectiveSize(xs), P.effectiveSize(xs), rtol=1e-9)


def _td():
    hM = td_model()
    hM.postList = td_postlist(hM)
    hM.samples = M["n_samples"]
    return hM


def _synthetic_posterior(S=60, seed=3):
    hM = synthetic_model(ny=400, ns=70, nc=5, nf=3, nt=3, nr=2, units=[400, 50], seed=seed)
    rng = np.random.default_rng(seed)
    post = []
    for k in range(S):
        nf0 = 3 if k % 4 else 2            # ragged nf across samples (updateNf)
        post.append(dict(Beta=rng.standard_normal((hM.nc, hM.ns)), Gamma=rng.standard_normal((hM.nc, hM.nt)),
                         Lambda=[rng.standard_normal((nf0, hM.ns)), rng.standard_normal((3, hM.ns)) * 0.5]))
    hM.postList = [post[:S // 2], post[S // 2:]]
    hM.samples = S // 2
    return hM


@pytest.mark.parametrize("which", ["td", "synthetic"])
def test_variance_partitioning_matches_restatement(which):
    hM = _td() if which == "td" else _synthetic_posterior()
    d = H.computeVariancePartitioning(hM)
    o = P.computeVariancePartitioning(hM)
    assert rel_err(d["vals"], o["vals"]) < 1e-9
    assert rel_err(d["R2T"]["Beta"], o["R2T"]["Beta"]) < 1e-9
    assert abs(d["R2T"]["Y"] - o["R2T"]["Y"]) < 1e-9 * max(1.0, abs(o["R2T"]["Y"]))
    assert d["rownames"] == o["rownames"]
    np.testing.assert_allclose(d["vals"].sum(axis=0), 1.0, atol=1e-12)


@pytest.mark.parametrize("which", ["td", "synthetic"])
def test_associations_match_restatement(which):
    hM = _td() if which == "td" else _synthetic_posterior()
    d = H.computeAssociations(hM)
    o = P.computeAssociations(hM)
    for r in range(hM.nr):
        assert rel_err(d[r]["mean"], o[r]["mean"]) < 1e-12
        np.testing.assert_array_equal(d[r]["support"], o[r]["support"])
    est = H.getPostEstimate(hM, "Omega", r=1)
    pooled = H.poolMcmcChains(hM.postList)
    om = np.stack([s["Lambda"][0].T @ s["Lambda"][0] for s in pooled])
    assert rel_err(est["mean"], om.mean(axis=0)) < 1e-12
    np.testing.assert_array_equal(est["support"], (om > 0).mean(axis=0))
    np.testing.assert_array_equal(est["supportNeg"], (om < 0).mean(axis=0))


def test_associations_at_scale():
    """ns = 1000 species, nf = 10, 200 samples: 8 MB per Omega sample never leaves the device."""
    rng = np.random.default_rng(5)
    ns, S = 1000, 200
    hM = synthetic_model(ny=50, ns=20, nc=2, nf=2, seed=4)    # only nr / postList / ns are read
    hM.ns = ns
    post = [dict(Lambda=[rng.standard_normal((10, ns))]) for _ in range(S)]
    hM.postList = [post]
    d = H.computeAssociations(hM)[0]
    sub = [0, 17, 500, 999]
    lam = np.stack([p["Lambda"][0][:, sub] for p in post])
    om = np.einsum("shi,shj->sij", lam, lam)
    dd = np.sqrt(np.einsum("sii->si", om))
    c = om / dd[:, :, None] / dd[:, None, :]
    c[:, range(4), range(4)] = 1.0
    assert rel_err(d["mean"][np.ix_(sub, sub)], c.mean(axis=0)) < 1e-12
    np.testing.assert_array_equal(d["support"][np.ix_(sub, sub)], (c > 0).mean(axis=0))
