"""End to end with spatial levels through the R-mirroring API:
sampleMcmc on Full (default updater set, so updateGammaEta's spatial branch runs, as TD$m
does), NNGP and GPP levels; R's stop for NNGP / GPP with the GammaEta updater
(R/updateGammaEta.R:153-158); predict at new spatial units (predictLatentFactor kriging on
the host, linear predictor on the device).  Coordinates come as a DataFrame whose index
names the units (R's rownames(sData)), covering the fitted units and 6 new ones."""
import numpy as np
import pandas as pd
import pytest

from helpers import H

pytestmark = pytest.mark.gpu


def _spatial_model(method, ny=60, ns=5, seed=3):
    rng = np.random.default_rng(seed)
    xy = rng.random((ny + 6, 2))
    names = [f"s{k:03d}" for k in range(ny + 6)]
    field = np.sin(4 * xy[:, 0]) + np.cos(3 * xy[:, 1])
    X = np.column_stack([np.ones(ny), rng.standard_normal(ny)])
    lam = rng.standard_normal(ns)
    L = X @ rng.normal(0, 0.5, (2, ns)) + field[:ny, None] * lam[None, :]
    Y = (L + rng.standard_normal((ny, ns)) > 0).astype(float)
    kw = {}
    if method == "NNGP":
        kw = dict(nNeighbours=8)
    if method == "GPP":
        # knots shifted off the sampling sites: a knot on a site makes dD = 1 - w12' iW22 w12
        # vanish there (idD ~ 1e15), degenerate in R's GPP as well
        kw = dict(sKnot=H.constructKnots(xy[:ny], nKnots=4) + 0.037)
    rl = H.HmscRandomLevel(sData=pd.DataFrame(xy, index=names), sMethod=method, **kw)
    H.setPriors(rl, nfMin=2, nfMax=2)
    sd = pd.DataFrame({"plot": names[:ny]})
    hM = H.Hmsc(Y=Y, X=X, covNames=["(Intercept)", "x1"], distr="probit", studyDesign=sd,
                ranLevels={"plot": rl})
    return hM, names


@pytest.mark.parametrize("method", ["Full", "NNGP", "GPP"])
def test_sample_and_predict_new_units(method):
    hM, names = _spatial_model(method)
    upd = {} if method == "Full" else {"GammaEta": False}
    hM = H.sampleMcmc(hM, samples=20, transient=30, thin=1, nChains=1, updater=upd, seed=9, verbose=0)
    post = H.poolMcmcChains(hM.postList)
    assert len(post) == 20
    a = np.stack([s["Alpha"][0] for s in post])
    assert np.all(a >= 1) and np.all(a <= hM.rL[0].alphapw.shape[0])
    assert all(np.all(np.isfinite(s["Beta"])) for s in post)
    new = names[-6:]
    sd = pd.DataFrame({"plot": new})
    Xn = np.column_stack([np.ones(6), np.zeros(6)])
    pred = H.predict(hM, post=post, X=Xn, studyDesign=sd, expected=True, seed=4)
    P = np.stack(pred)
    assert P.shape == (20, 6, hM.ns) and np.all((P >= 0) & (P <= 1))


def test_nngp_with_gamma_eta_stops_like_r():
    hM, _ = _spatial_model("NNGP")
    with pytest.raises(Exception, match="GammaEta"):
        H.sampleMcmc(hM, samples=2, transient=0, nChains=1, seed=1, verbose=0)
