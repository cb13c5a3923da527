"""Host logic of the post-sampling path: evaluateModelFit's measures
(R/evaluateModelFit.R) against independent implementations, and predictLatentFactor's unit
bookkeeping (R/predictLatentFactor.R:1-30).  No GPU: predict itself is tested in
tests/test_gpu_predict.py."""
import numpy as np
import pytest
from sklearn.metrics import roc_auc_score

from helpers import H, synthetic_model
from hmsc_amd.predict import _auc, evaluateModelFit, predictLatentFactor


def test_auc_matches_sklearn_with_ties():
    rng = np.random.default_rng(0)
    y = (rng.random(300) < 0.4).astype(float)
    p = np.round(rng.random(300) + 0.3 * y, 2)   # ties on purpose
    assert abs(_auc(y, p) - roc_auc_score(y, p)) < 1e-12


def test_evaluate_model_fit_probit_and_normal():
    hM = synthetic_model(ny=80, ns=6, nc=2, nf=1, n_normal=2, seed=3)
    rng = np.random.default_rng(1)
    predY = np.clip(np.nan_to_num(hM.Y)[:, :, None] * 0.6 + 0.2 * rng.random((80, 6, 5)), 0, None)
    mf = evaluateModelFit(hM, predY)
    m = predY.mean(axis=2)
    Y = hM.Y
    assert np.allclose(mf["RMSE"], np.sqrt(np.mean((Y - m) ** 2, axis=0)))
    for j in range(2):
        co = np.corrcoef(Y[:, j], m[:, j])[0, 1]
        assert abs(mf["R2"][j] - np.sign(co) * co ** 2) < 1e-12
    for j in range(2, 6):
        assert abs(mf["AUC"][j] - roc_auc_score(Y[:, j], m[:, j])) < 1e-12
        assert abs(mf["TjurR2"][j] - (m[Y[:, j] == 1, j].mean() - m[Y[:, j] == 0, j].mean())) < 1e-12
    assert np.isnan(mf["AUC"][0]) and np.isnan(mf["R2"][3])


def test_evaluate_model_fit_poisson_measures():
    hM = synthetic_model(ny=60, ns=3, nc=2, nf=1, n_poisson=3, seed=4)
    rng = np.random.default_rng(2)
    predY = rng.poisson(np.nan_to_num(hM.Y)[:, :, None] + 0.5, size=(60, 3, 7)).astype(float)
    mf = evaluateModelFit(hM, predY)
    med = np.median(predY, axis=2)
    assert np.allclose(mf["RMSE"], np.sqrt(np.mean((hM.Y - med) ** 2, axis=0)))
    pO = (predY > 0).mean(axis=2)
    Yo = (hM.Y > 0).astype(float)
    for j in range(3):
        assert abs(mf["O.AUC"][j] - roc_auc_score(Yo[:, j], pO[:, j])) < 1e-12
        assert abs(mf["O.RMSE"][j] - np.sqrt(np.mean((Yo[:, j] - pO[:, j]) ** 2))) < 1e-12
    assert set(mf) >= {"SR2", "O.TjurR2", "C.SR2", "C.RMSE"}


def test_predict_latent_factor_units():
    post = [np.arange(6.0).reshape(3, 2), 10 + np.arange(6.0).reshape(3, 2)]
    rl = H.HmscRandomLevel(units=["a", "b", "c"])
    out = predictLatentFactor(["b", "z", "a"], ["a", "b", "c"], post, rl, predictMean=True)
    assert np.array_equal(out[0], np.array([[2.0, 3.0], [0.0, 0.0], [0.0, 1.0]]))
    assert np.array_equal(out[1][0], [12.0, 13.0])
    draws = predictLatentFactor(["z", "y"], ["a"], post[:1], rl, rng=np.random.default_rng(0))
    assert draws[0].shape == (2, 2) and np.all(draws[0] != 0)


def _spatial_rl(method, s_df, **kw):
    rl = H.HmscRandomLevel(sData=s_df, sMethod=method, **kw)
    H.setPriors(rl, nfMin=2, nfMax=2)
    return rl


@pytest.mark.parametrize("method", ["Full", "NNGP", "GPP"])
def test_predict_latent_factor_spatial(method):
    """R/predictLatentFactor.R:59-204: new units of a spatial level are kriged; a new unit at
    (almost) the location of a fitted one inherits its Eta under a smooth kernel."""
    import pandas as pd
    from hmsc_amd.dataparams import constructKnots
    rng = np.random.default_rng(1)
    xy = rng.random((30, 2))
    names = [f"p{k:02d}" for k in range(30)]
    xy_new = xy[:3] + 1e-6
    df = pd.DataFrame(np.vstack([xy, xy_new]), index=names + ["n0", "n1", "n2"])
    kw = dict(nNeighbours=5) if method == "NNGP" else dict(sKnot=constructKnots(xy, nKnots=6)) if method == "GPP" else {}
    rl = _spatial_rl(method, df, **kw)
    eta = np.column_stack([np.sin(4 * xy[:, 0]), np.cos(3 * xy[:, 1])])
    alpha = np.array([60, 80])                   # long range: W ~ smooth, kriging ~ interpolation
    unitsPred = ["n0", "p05", "n1", "n2"]
    mean = predictLatentFactor(unitsPred, names, [eta], rl, predictMean=True, postAlpha=[alpha])[0]
    assert np.allclose(mean[1], eta[5])
    assert np.allclose(mean[[0, 2, 3]], eta[:3], atol=1e-3)
    draws = predictLatentFactor(unitsPred, names, [eta] * 200, rl, postAlpha=[alpha] * 200,
                                rng=np.random.default_rng(2))
    d = np.stack(draws)
    assert np.allclose(d[:, 1], eta[5])
    if method != "GPP":                          # GPP's knot approximation leaves a nugget
        assert np.abs(d[:, [0, 2, 3]].mean(0) - eta[:3]).max() < 1e-2
    assert np.all(np.isfinite(d))
    mf = predictLatentFactor(unitsPred, names, [eta], rl, predictMeanField=True, postAlpha=[alpha],
                             rng=np.random.default_rng(3))[0]
    assert np.allclose(mf[[0, 2, 3]], eta[:3], atol=1e-2)
    with pytest.raises(ValueError):
        predictLatentFactor(unitsPred, names, [eta], rl, predictMean=True, predictMeanField=True, postAlpha=[alpha])


def test_predict_latent_factor_distmat_equals_coordinates():
    """A spatial level given by distances (R/predictLatentFactor.R:69-70,100): rL$distMat rows by
    unit name replace dist(rL$s); with the distances of the same coordinates the kriged Eta of
    new units is the sData level's draw for draw ('Full', predictMean, predictMeanField)."""
    import pandas as pd
    rng = np.random.default_rng(4)
    xy = rng.random((25, 2))
    names = [f"p{k:02d}" for k in range(25)]
    xy_all = np.vstack([xy, xy[:2] + 0.03])
    all_names = names + ["n0", "n1"]
    D = np.sqrt(((xy_all[:, None, :] - xy_all[None, :, :]) ** 2).sum(-1))
    rl_s = _spatial_rl("Full", pd.DataFrame(xy_all, index=all_names))
    order = np.random.default_rng(5).permutation(len(all_names))   # distMat rows in another order
    dm = pd.DataFrame(D[np.ix_(order, order)], index=[all_names[k] for k in order])
    rl_d = H.HmscRandomLevel(distMat=dm)
    H.setPriors(rl_d, nfMin=2, nfMax=2)
    H.setPriors(rl_d, alphapw=rl_s.alphapw)
    eta = np.column_stack([np.sin(3 * xy[:, 0]), xy[:, 1]])
    alpha = np.array([30, 50])
    up = ["n0", "p03", "n1"]
    for kw in (dict(predictMean=True), dict(predictMeanField=True), {}):
        a = predictLatentFactor(up, names, [eta], rl_s, postAlpha=[alpha], rng=np.random.default_rng(6), **kw)[0]
        b = predictLatentFactor(up, names, [eta], rl_d, postAlpha=[alpha], rng=np.random.default_rng(6), **kw)[0]
        np.testing.assert_allclose(b, a, rtol=1e-12, atol=1e-12)
    rl_n = H.HmscRandomLevel(distMat=dm, sMethod="NNGP")
    H.setPriors(rl_n, nfMin=2, nfMax=2)
    with pytest.raises(ValueError, match="needs coordinates"):
        predictLatentFactor(up, names, [eta], rl_n, postAlpha=[alpha])
