"""Host side of covariate-dependent levels (CPU only): R's level -> the C ABI's device levels
(include/hmsc_amd.h etaShare / xScale; hmsc_amd/sampler.py LevelMap, ModelBuffers), per-column
priors (R/setPriors.HmscRandomLevel.R:21-80), and R's array layouts through combineParameters and
alignPosterior."""
import ctypes as C

import numpy as np
import pytest

import hmsc_amd as H
from helpers import synthetic_model
from hmsc_amd.sampler import LevelMap, ModelBuffers, alignPosterior, combine_parameters, x_unit_order


def _arr(ptr, n, dt=np.float64):
    return np.ctypeslib.as_array(ptr, shape=(n,)).astype(dt)


def test_level_expansion_in_the_c_struct():
    hM = synthetic_model(ny=60, ns=5, nc=3, nf=2, nr=2, units=[20, 60], x_dim=3, seed=2)
    H.setPriors(hM.rL[0], a1=[10.0, 20.0, 30.0])
    lm = LevelMap(hM)
    assert lm.groups == [[0, 1, 2], [3]] and lm.ndev == 4 and lm.xdim == [3, 0]
    buf = ModelBuffers(hM)
    m = buf.struct
    assert m.nr == 4
    assert _arr(m.etaShare, 4, np.int32).tolist() == [0, 0, 0, 3]
    assert _arr(m.a1, 4).tolist() == [10.0, 20.0, 30.0, 50.0]
    assert _arr(m.nfMin, 4, np.int32).tolist() == [2, 2, 2, 2]
    Pi = _arr(m.Pi, 60 * 4, np.int32).reshape(60, 4, order="F")
    assert (Pi[:, 0] == Pi[:, 1]).all() and (Pi[:, 0] == Pi[:, 2]).all() and (Pi[:, 3] == hM.Pi[:, 1]).all()
    x = x_unit_order(hM, 0, hM.rL[0])
    for k in range(3):
        np.testing.assert_array_equal(_arr(m.xScale[k], 20), x[:, k])
    assert not m.xScale[3]
    assert _arr(m.xDim, 4, np.int32).tolist() == [0, 0, 0, 0]


def test_x_rows_follow_unit_names():
    """rL$x is indexed by unit name (rL$x[as.character(dfPi[,r]), k]): shuffled rows come back
    in the unit order of Eta."""
    import pandas as pd
    hM = synthetic_model(ny=40, ns=4, nc=2, nf=1, units=[8], x_dim=2, seed=4)
    x0 = x_unit_order(hM, 0, hM.rL[0])
    df = hM.rL[0].x
    hM.rL[0].x = df.iloc[np.random.default_rng(1).permutation(8)]
    np.testing.assert_array_equal(x_unit_order(hM, 0, hM.rL[0]), x0)
    with pytest.raises(ValueError, match="length of nu"):
        H.setPriors(hM.rL[0], nu=[1.0, 2.0, 3.0])


def test_combine_and_align_keep_r_layouts():
    hM = synthetic_model(ny=40, ns=6, nc=2, nf=2, units=[10], x_dim=2, seed=5)
    S, nf, ns = 4, 2, 6
    rng = np.random.default_rng(0)
    rec = dict(Beta=rng.standard_normal((S, 2, ns)), Gamma=rng.standard_normal((S, 2, 1)),
               iV=np.tile(np.eye(2), (S, 1, 1)), iSigma=np.ones((S, ns)), rho=np.ones(S, dtype=np.int32),
               nf=np.full((1, S), nf), Eta0=rng.standard_normal((S, 10, 3)),
               Lambda0=rng.standard_normal((S, 3, ns, 2)), Psi0=np.ones((S, 3, ns, 2)),
               Delta0=np.ones((S, 3, 2)), Alpha0=np.ones((S, 3), dtype=np.int64))
    post = combine_parameters(rec, hM)
    assert post[0]["Lambda"][0].shape == (nf, ns, 2) and post[0]["Delta"][0].shape == (nf, 2)
    # a chain whose factor 1 has the opposite sign everywhere is flipped back, Eta column too
    other = [dict(s, Lambda=[-s["Lambda"][0]], Eta=[-s["Eta"][0]], Psi=list(s["Psi"]), Delta=list(s["Delta"]))
             for s in post]
    hM.postList = [post, other]
    alignPosterior(hM)
    np.testing.assert_allclose(hM.postList[1][0]["Lambda"][0], post[0]["Lambda"][0])
    np.testing.assert_allclose(hM.postList[1][0]["Eta"][0], post[0]["Eta"][0])
