"""Known answers from the reference's own tests, on the TD fixture (data/TD.rda).

tests/testthat/test-initialParameters.R:137-186 (computeDataParameters sums),
tests/testthat/test-WAIC.R:3-6 (WAIC), tests/testthat/test-setHmsc.R:166-189 (the TD
model rebuilt from its inputs equals TD$m), tests/testthat/test-sampling.R:164-169
(object / sample sizes).  CPU only.
"""
import json
import os

import numpy as np
import pandas as pd
import pytest

import hmsc_amd as H
from oracle import post_oracle as P

HERE = os.path.dirname(os.path.abspath(__file__))
D = np.load(os.path.join(HERE, "golden", "td.npz"))
M = json.load(open(os.path.join(HERE, "golden", "td_meta.json")))


def td_model():
    """Hmsc(Y=TD$Y, XData=TD$X, XFormula=~x1+x2, TrData=TD$Tr, TrFormula=~T1+T2, phylo C,
    ranLevels=list(sample=rL2, plot=rL1), studyDesign) — data-raw/simulateTestData.R:60-68."""
    ny = M["ny"]
    XData = pd.DataFrame({"x1": D["x1"], "x2": pd.Categorical(["o"] * (ny // 2) + ["c"] * (ny // 2))})
    TrData = pd.DataFrame({"T1": D["Tr"][:, 1], "T2": pd.Categorical(np.where(D["Tr"][:, 2] == 1, "B", "A"))})
    sd = pd.DataFrame({"sample": pd.Categorical([str(i) for i in range(1, ny + 1)],
                                                categories=[str(i) for i in range(1, ny + 1)]),
                       "plot": pd.Categorical([str(v) for v in M["studyDesign_plot"]],
                                              categories=M["studyDesign_plot_levels"])})
    rL2 = H.HmscRandomLevel(units=sd["sample"])
    H.setPriors(rL2, nfMax=2, nfMin=2)
    rL1 = H.HmscRandomLevel(sData=D["xycoords"])
    H.setPriors(rL1, nfMax=2, nfMin=2)
    return H.Hmsc(Y=D["Y"], XData=XData, XFormula="~x1+x2", TrData=TrData, TrFormula="~T1+T2", C=D["C"],
                  ranLevels={"sample": rL2, "plot": rL1}, studyDesign=sd, distr="probit",
                  spNames=M["spNames"])


def td_postlist(hM):
    post = []
    for c in range(M["n_chains"]):
        chain = []
        for k in range(M["n_samples"]):
            s = dict(Beta=D[f"post_Beta_c{c}"][k], wRRR=None, Gamma=D[f"post_Gamma_c{c}"][k], V=D[f"post_V_c{c}"][k],
                     rho=float(D[f"post_rho_c{c}"][k][0]), sigma=D[f"post_sigma_c{c}"][k],
                     Eta=[D[f"post_Eta{r}_c{c}"][k] for r in range(2)],
                     Lambda=[D[f"post_Lambda{r}_c{c}"][k] for r in range(2)],
                     Alpha=[D[f"post_Alpha{r}_c{c}"][k] for r in range(2)],
                     Psi=[D[f"post_Psi{r}_c{c}"][k] for r in range(2)],
                     Delta=[D[f"post_Delta{r}_c{c}"][k] for r in range(2)], PsiRRR=None, DeltaRRR=None)
            chain.append(s)
        post.append(chain)
    return post


def test_model_rebuilt_equals_td_m():
    """test-setHmsc.R:166-189: rebuilding TD$m from its inputs gives the same scaled data."""
    hM = td_model()
    np.testing.assert_allclose(hM.XScaled, D["XScaled"], rtol=1e-12, atol=1e-14)
    np.testing.assert_allclose(hM.XScalePar, D["XScalePar"], rtol=1e-12, atol=1e-14)
    np.testing.assert_allclose(hM.TrScaled, D["TrScaled"], rtol=1e-12, atol=1e-14)
    np.testing.assert_allclose(hM.TrScalePar, D["TrScalePar"], rtol=1e-12, atol=1e-14)
    np.testing.assert_array_equal(hM.Pi, D["Pi"])
    np.testing.assert_array_equal(hM.distr, D["distr"])
    assert hM.covNames == M["covNames"] and hM.trNames == M["trNames"]
    assert hM.XInterceptInd == M["XInterceptInd"] and hM.TrInterceptInd == M["TrInterceptInd"]
    np.testing.assert_allclose(hM.rhopw, D["rhopw"])
    np.testing.assert_allclose(hM.rL[1].alphapw, D["alphapw_1"], rtol=1e-12)
    assert list(hM.np) == M["np"]
    assert len(hM) == M["n_hM_fields"] == 72
    assert hM.names() == M["hM_fields"]


def test_compute_data_parameters_known_sums():
    """test-initialParameters.R:144-186."""
    hM = td_model()
    par = H.computeDataParameters(hM)
    k = M["known"]
    assert len(par) == 5
    assert len(par["rLPar"][0]) == 0 and len(par["rLPar"][1]) == 4
    assert par["Qg"].shape == (4, 4, 101)
    assert round(par["detQg"].sum()) == k["sum_detQg_round"]
    assert round(par["Qg"].sum()) == k["sum_Qg_round"]
    assert round(par["iQg"].sum()) == k["sum_iQg_round"]
    assert round(par["RQg"].sum()) == k["sum_RQg_round"]
    sp = par["rLPar"][1]
    assert sp["Wg"].shape == (10, 10, 101)
    assert round(sp["detWg"].sum()) == k["sum_detWg_round"]
    assert round(sp["Wg"].sum()) == k["sum_Wg_round"]
    assert round(sp["iWg"].sum()) == k["sum_iWg_round"]
    assert round(sp["RiWg"].sum()) == k["sum_RiWg_round"]


def test_compute_data_parameters_no_phylogeny():
    """test-initialParameters.R:157-174: identity Q grid and no spatial parameters."""
    hM = H.Hmsc(Y=np.arange(1, 21, dtype=float).reshape(10, 2, order="F"),
                X=np.arange(1, 21, dtype=float).reshape(10, 2, order="F"))
    par = H.computeDataParameters(hM)
    assert par["detQg"][0] == 0
    np.testing.assert_array_equal(par["Qg"][:, :, 0], np.eye(2))
    np.testing.assert_array_equal(par["iQg"][:, :, 0], np.eye(2))
    np.testing.assert_array_equal(par["RQg"][:, :, 0], np.eye(2))
    assert len(par["rLPar"]) == 0


def test_waic_known_answer():
    """test-WAIC.R:4: round(computeWAIC(TD$m), 1) == 0.8."""
    hM = td_model()
    hM.postList = td_postlist(hM)
    w = H.computeWAIC(hM)
    assert round(w, 1) == M["known"]["WAIC_round1"]


def test_golden_posterior_layout_and_means():
    hM = td_model()
    hM.postList = td_postlist(hM)
    assert len(hM.postList[0][0]) == M["known"]["len_postList_sample"] == 13
    post = H.poolMcmcChains(hM.postList)
    mean_beta = np.mean([s["Beta"] for s in post], axis=0)
    np.testing.assert_allclose(mean_beta, [[-2.388, 0.687, -0.444, -1.604], [0.682, 2.039, 2.305, 1.174],
                                           [0.007, 0.392, -0.955, -0.975]], atol=5e-4)
    mp, cols = H.convertToCodaObject(hM)
    assert mp["Beta"][0].shape == (100, 12)
    sp = M["spNames"]
    assert cols["Beta"][:2] == [f"B[(Intercept) (C1), {sp[0]} (S1)]", f"B[x1 (C2), {sp[0]} (S1)]"]
    assert mp["Lambda"][0][0].shape == (100, 8) and cols["Lambda"][0][1] == f"Lambda1[{sp[1]} (S2), factor1]"
    assert mp["Omega"][1][0].shape == (100, 16)
    est = H.getPostEstimate(hM, "Beta")
    np.testing.assert_allclose(est["mean"], mean_beta)


def test_align_posterior_is_idempotent_on_aligned_chains():
    hM = td_model()
    hM.postList = td_postlist(hM)
    before = np.stack([s["Lambda"][0] for s in hM.postList[1]])
    H.alignPosterior(hM)
    after = np.stack([s["Lambda"][0] for s in hM.postList[1]])
    # the fitted TD$m was aligned by sampleMcmc (5 passes): nothing flips again
    np.testing.assert_allclose(np.abs(after), np.abs(before))
    flips = np.mean(np.sign(after) != np.sign(before))
    assert flips < 0.05


def test_effective_size_ar1():
    """coda::effectiveSize restated (oracle/post_oracle.py, the device version's checker):
    AR(1) with phi has ESS ~ n (1 - phi) / (1 + phi)."""
    rng = np.random.default_rng(0)
    n, phi = 20000, 0.6
    e = rng.standard_normal((n, 3))
    x = np.zeros((n, 3))
    for t in range(1, n):
        x[t] = phi * x[t - 1] + e[t]
    ess = P.effectiveSize(x)
    expect = n * (1 - phi) / (1 + phi)
    assert np.all(np.abs(ess / expect - 1) < 0.1)
    point, upper = H.gelman_diag([x[:10000], x[10000:]])
    assert np.all(point < 1.05) and np.all(upper >= point)


def test_variance_partitioning_td():
    """computeVariancePartitioning(TD$m) restated (oracle/post_oracle.py; the roxygen example,
    tests/Examples/Hmsc-Ex.Rout.save:181, values not printed there: structure only).
    Fixed groups + random levels partition each species' explained variance."""
    hM = td_model()
    hM.postList = td_postlist(hM)
    hM.samples = M["n_samples"]
    VP = P.computeVariancePartitioning(hM)
    assert VP["vals"].shape == (hM.nc - 1 + hM.nr, hM.ns)
    np.testing.assert_allclose(VP["vals"].sum(axis=0), 1.0, atol=1e-12)
    assert np.all(VP["vals"] >= 0)
    assert np.all((VP["R2T"]["Beta"] >= 0) & (VP["R2T"]["Beta"] <= 1)) and 0 <= VP["R2T"]["Y"] <= 1
    assert VP["rownames"][-2:] == ["Random: sample", "Random: plot"]


def test_coda_name_flags_follow_r():
    """convertToCodaObject's *NamesNumbers flags (R/convertToCodaObject.r:54-92): [1] adds
    the name, [2] adds '(S%d)', joined by a space; Delta / Alpha are 0-padded; Eta columns
    are named by unit."""
    hM = td_model()
    hM.postList = td_postlist(hM)
    sp = M["spNames"]
    _, c = H.convertToCodaObject(hM, spNamesNumbers=(True, False), covNamesNumbers=(False, True))
    assert c["Beta"][0] == f"B[(C1), {sp[0]}]"
    _, c = H.convertToCodaObject(hM, spNamesNumbers=(False, True), covNamesNumbers=(True, False))
    assert c["Beta"][1] == "B[x1, (S1)]"
    mp, c = H.convertToCodaObject(hM)
    assert c["Beta"][0] == f"B[(Intercept) (C1), {sp[0]} (S1)]"
    assert c["Eta"][1][0] == "Eta2[1, factor1]" and c["Alpha"][1] == ["Alpha2[factor1]", "Alpha2[factor2]"]
    a = mp["Alpha"][1][0]
    assert a.shape == (100, 2) and np.all(np.isin(a, hM.rL[1].alphapw[:, 0]))
