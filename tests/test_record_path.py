"""The per-sample record path pinned to the reference's stored TD$m (CPU only).

combineParameters (R/combineParameters.R:1-58) turns the sampler's scaled-space state into
the original-scale postList; TD$m$postList (data/TD.rda, 2 chains x 100 samples) is that
output.  The scaled-space samples it came from are not stored, so they are recovered here
WITHOUT combineParameters' own formulas: the linear predictor is invariant under the
reparametrisation, X beta = XScaled beta_s, so beta = M beta_s with M the exact solution of
X M = XScaled; likewise Tr = TrScaled P.  Then Beta_s = M^-1 Beta, Gamma_s = M^-1 Gamma P^T.
V is the one field the invariance does not fix: the reference rescales iV by the covariate
sd only (a quirk: no intercept term, so V is not the covariance of the un-scaled Beta), and
V_s = diag(sd) V diag(sd) restates that.  Pushing those through hmsc_amd.sampler.combine_parameters must give back
the stored postList (Beta, Gamma, V, sigma, rho) to rounding.

alignPosterior (R/alignPosterior.R:18-100): sign flips of a factor (Lambda row and Eta
column together) in some samples are repaired against the template chain's posterior mean
Lambda; a chain with fewer factors is padded (Lambda / Psi 0, Delta 1, Eta 0, Alpha 1 for a
spatial level, :57-68).
"""
import copy

import numpy as np

import hmsc_amd as H
from hmsc_amd.sampler import combine_parameters
from test_golden_td import td_model, td_postlist


def _scaled_record(hM, chain):
    """The sampler-side record arrays of one stored TD chain (rec layout of Chain.run)."""
    X, XS = np.asarray(hM.X, dtype=np.float64), np.asarray(hM.XScaled, dtype=np.float64)
    Tr, TS = np.asarray(hM.Tr, dtype=np.float64), np.asarray(hM.TrScaled, dtype=np.float64)
    Mx = np.linalg.lstsq(X, XS, rcond=None)[0]          # X Mx = XScaled   (beta = Mx beta_s)
    Pt = np.linalg.lstsq(TS, Tr, rcond=None)[0]         # TrScaled Pt = Tr  (Tr = TrScaled Pt)
    np.testing.assert_allclose(X @ Mx, XS, atol=1e-12)
    np.testing.assert_allclose(TS @ Pt, Tr, atol=1e-12)
    iM = np.linalg.inv(Mx)
    S = len(chain)
    # Beta = Gamma Tr^T = Gamma Pt^T TrS^T  and  Beta = Mx Beta_s  =>  Gamma_s = Mx^-1 Gamma Pt^T
    Beta = np.stack([iM @ s["Beta"] for s in chain])
    Gamma = np.stack([iM @ s["Gamma"] @ Pt.T for s in chain])
    # V: the reference only rescales iV (iV[k,] * s, iV[,k] * s, R/combineParameters.R:24-25),
    # with no intercept shift, so its stored V is diag(1/sd) V_s diag(1/sd), not Mx V_s Mx^T
    sd = np.where(np.asarray(hM.XScalePar)[1] != 0, np.asarray(hM.XScalePar)[1], 1.0)
    iV = np.stack([np.linalg.inv(np.diag(sd) @ s["V"] @ np.diag(sd)) for s in chain])
    rhopw = np.asarray(hM.rhopw)[:, 0]
    rho = np.array([int(np.argmin(np.abs(rhopw - s["rho"]))) + 1 for s in chain], dtype=np.int32)
    rec = dict(Beta=Beta, Gamma=Gamma, iV=iV, iSigma=np.stack([1.0 / s["sigma"] for s in chain]), rho=rho,
               nf=np.array([[s["Lambda"][r].shape[0] for s in chain] for r in range(hM.nr)]))
    for r in range(hM.nr):
        rec[f"Eta{r}"] = np.stack([s["Eta"][r] for s in chain])
        rec[f"Lambda{r}"] = np.stack([s["Lambda"][r] for s in chain])
        rec[f"Psi{r}"] = np.stack([s["Psi"][r] for s in chain])
        rec[f"Delta{r}"] = np.stack([np.asarray(s["Delta"][r]).ravel() for s in chain])
        rec[f"Alpha{r}"] = np.stack([np.asarray(s["Alpha"][r]).ravel() for s in chain]).astype(np.int64)
    assert Beta.shape == (S, hM.nc, hM.ns)
    return rec


def test_combine_parameters_reproduces_td_postlist():
    hM = td_model()
    stored = td_postlist(hM)
    # the reparametrisation is not the identity on TD (x1 and T1 are centred and scaled)
    assert np.any(np.asarray(hM.XScalePar)[:, 1] != [0, 1]) and np.any(np.asarray(hM.TrScalePar)[:, 1] != [0, 1])
    for chain in stored:
        post = combine_parameters(_scaled_record(hM, chain), hM)
        assert len(post) == len(chain) and list(post[0].keys()) == list(chain[0].keys())
        for got, ref in zip(post, chain):
            for k in ("Beta", "Gamma", "V", "sigma"):
                np.testing.assert_allclose(got[k], ref[k], rtol=1e-9, atol=1e-10, err_msg=k)
            assert got["rho"] == ref["rho"]
            for r in range(hM.nr):
                np.testing.assert_array_equal(got["Lambda"][r], ref["Lambda"][r])
                np.testing.assert_array_equal(got["Eta"][r], ref["Eta"][r])
                assert got["Delta"][r].shape == (ref["Lambda"][r].shape[0], 1)


def test_combine_parameters_intercept_shift_is_exact_on_the_linear_predictor():
    """R/combineParameters.R:15-28 in effect: XScaled B_s == X combine(B_s) for any B_s."""
    hM = td_model()
    rng = np.random.default_rng(3)
    S = 7
    rec = _scaled_record(hM, td_postlist(hM)[0][:S])
    rec["Beta"] = rng.standard_normal(rec["Beta"].shape)
    post = combine_parameters(rec, hM)
    for k in range(S):
        np.testing.assert_allclose(np.asarray(hM.X) @ post[k]["Beta"], np.asarray(hM.XScaled) @ rec["Beta"][k],
                                   atol=1e-12)


def _aligned_td():
    hM = td_model()
    hM.postList = td_postlist(hM)
    for _ in range(5):                       # R/sampleMcmc.R:365-369: a fixed point afterwards
        H.alignPosterior(hM)
    return hM


def test_align_posterior_repairs_flipped_factors():
    hM = _aligned_td()
    ref = copy.deepcopy(hM.postList)
    H.alignPosterior(hM)                     # a fixed point: nothing moves
    for c in range(2):
        for s0, s1 in zip(ref[c], hM.postList[c]):
            for r in range(hM.nr):
                np.testing.assert_array_equal(s0["Lambda"][r], s1["Lambda"][r])
    rng = np.random.default_rng(11)
    flipped = []
    for j, s in enumerate(hM.postList[1]):  # chain 2 (the template is chain 1: equal nf)
        for r in range(hM.nr):
            for k in range(s["Lambda"][r].shape[0]):
                if rng.random() < 0.5:
                    s["Lambda"][r] = s["Lambda"][r].copy()
                    s["Eta"][r] = s["Eta"][r].copy()
                    s["Lambda"][r][k] *= -1
                    s["Eta"][r][:, k] *= -1
                    flipped.append((j, r, k))
    assert len(flipped) > 100
    H.alignPosterior(hM)
    for j, s in enumerate(hM.postList[1]):
        for r in range(hM.nr):
            np.testing.assert_array_equal(s["Lambda"][r], ref[1][j]["Lambda"][r])
            np.testing.assert_array_equal(s["Eta"][r], ref[1][j]["Eta"][r])


def test_align_posterior_pads_fewer_factors():
    """A chain with nf = 1 at level 2 (the spatial plot level) next to one with nf = 2."""
    hM = _aligned_td()
    r = 1
    assert hM.rL[r].sDim
    for s in hM.postList[1]:
        s["Lambda"][r] = s["Lambda"][r][:1].copy()
        s["Psi"][r] = s["Psi"][r][:1].copy()
        s["Delta"][r] = np.asarray(s["Delta"][r])[:1].copy()
        s["Eta"][r] = s["Eta"][r][:, :1].copy()
        s["Alpha"][r] = np.asarray(s["Alpha"][r]).ravel()[:1].copy()
    keep = [s["Lambda"][r][0].copy() for s in hM.postList[1]]
    H.alignPosterior(hM)
    for j, s in enumerate(hM.postList[1]):
        assert s["Lambda"][r].shape == (2, hM.ns) and s["Psi"][r].shape == (2, hM.ns)
        np.testing.assert_array_equal(np.abs(s["Lambda"][r][0]), np.abs(keep[j]))
        np.testing.assert_array_equal(s["Lambda"][r][1], 0.0)
        np.testing.assert_array_equal(s["Psi"][r][1], 0.0)
        assert np.asarray(s["Delta"][r]).shape == (2, 1) and np.asarray(s["Delta"][r])[1, 0] == 1.0
        assert s["Eta"][r].shape == (10, 2) and np.all(s["Eta"][r][:, 1] == 0.0)
        assert list(np.asarray(s["Alpha"][r]).ravel()[1:]) == [1]
    # the template (max nf) is chain 1; its samples are untouched by the padding
    assert all(s["Lambda"][r].shape == (2, hM.ns) for s in hM.postList[0])
