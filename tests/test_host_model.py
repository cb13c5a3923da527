"""Host API mirror of Hmsc()/HmscRandomLevel()/setPriors() — the reference's model-spec tests
(tests/testthat/test-setHmsc.R, test-setPriors.R, test-setRL.R) restated.  CPU only."""
import math

import numpy as np
import pandas as pd
import pytest

import hmsc_amd as H


def M(a, nrow, ncol):
    return np.asarray(a, dtype=float).reshape(nrow, ncol, order="F")


def test_y_scaling():
    """test-setHmsc.R:105-122."""
    m = H.Hmsc(Y=M(range(1, 21), 10, 2), X=M(range(1, 11), 10, 1))
    np.testing.assert_allclose(m.YScaled.mean(0), [11 / 2, 31 / 2])
    m = H.Hmsc(Y=M(range(1, 21), 10, 2), X=M(range(1, 11), 10, 1), YScale=True)
    np.testing.assert_allclose(m.YScaled.mean(0), [0, 0], atol=1e-14)
    np.testing.assert_allclose(np.round(m.YScalePar), [[6, 16], [3, 3]])
    m = H.Hmsc(Y=M(range(1, 21), 10, 2), X=M(range(1, 11), 10, 1), YScale=True, distr=["normal", "probit"])
    np.testing.assert_allclose(m.YScaled.mean(0), [0, 31 / 2], atol=1e-14)
    np.testing.assert_allclose(np.round(m.YScalePar), [[6, 0], [3, 1]])
    m = H.Hmsc(Y=M(range(1, 21), 10, 2), X=M(range(1, 11), 10, 1), YScale=True,
               distr=["poisson", "lognormal poisson"])
    np.testing.assert_allclose(m.YScaled.mean(0), [11 / 2, 31 / 2])


def test_x_scaling():
    """test-setHmsc.R:123-135."""
    m = H.Hmsc(Y=M(range(1, 11), 10, 1), X=M(range(1, 11), 10, 1))
    assert round(m.XScaled.mean()) == 1
    np.testing.assert_allclose(np.round(m.XScalePar).ravel(), [0, 7])
    m = H.Hmsc(Y=M(range(1, 11), 10, 1), X=M(range(1, 11), 10, 1), XScale=False)
    assert m.XScaled.mean() == 5.5
    m = H.Hmsc(Y=M(range(1, 11), 10, 1), XData=pd.DataFrame({"x1": np.arange(1, 11)}), XFormula="~x1")
    np.testing.assert_allclose(m.X.mean(0), [1, 5.5])
    np.testing.assert_allclose(m.XScaled.mean(0), [1, 0], atol=1e-14)
    np.testing.assert_allclose(np.round(m.XScalePar), [[0, 6], [1, 3]])


def test_trait_scaling():
    """test-setHmsc.R:136-147."""
    Traits = M([1, 1, 2, 23], 2, 2)
    m = H.Hmsc(Y=M(range(1, 21), 10, 2), X=M(range(1, 11), 10, 1),
               TrData=pd.DataFrame({"Intercept": Traits[:, 0], "x1": Traits[:, 1]}), TrFormula="~ x1")
    np.testing.assert_allclose(m.Tr, Traits)
    np.testing.assert_allclose(np.round(m.TrScaled.mean(0)), [1, 0])
    np.testing.assert_allclose(np.round(m.TrScalePar), [[0, 12], [1, 15]])
    m = H.Hmsc(Y=M(range(1, 21), 10, 2), X=M(range(1, 11), 10, 1), Tr=Traits, TrScale=False)
    np.testing.assert_allclose(m.TrScaled, Traits)


def test_distr_codes():
    """test-setHmsc.R:150-161."""
    m = H.Hmsc(Y=M(range(1, 21), 5, 4), X=M(range(1, 6), 5, 1),
               distr=["probit", "poisson", "normal", "lognormal poisson"])
    assert list(m.distr[:, 0]) == [2, 3, 1, 3]
    assert list(m.distr[:, 1]) == [0, 0, 1, 1]
    with pytest.raises(ValueError, match="some of the distributions ill defined"):
        H.Hmsc(Y=M(range(1, 11), 5, 2), X=M(range(1, 6), 5, 1), distr=["probit", "logit"])


def test_argument_errors():
    """test-setHmsc.R error messages."""
    with pytest.raises(ValueError, match="must be a matrix"):
        H.Hmsc(Y=np.arange(10.0), X=M(range(1, 11), 10, 1))
    with pytest.raises(ValueError, match="number of rows in X"):
        H.Hmsc(Y=M(range(1, 11), 10, 1), X=M(range(1, 10), 9, 1))
    with pytest.raises(ValueError, match="only single of XData and X"):
        H.Hmsc(Y=M(range(1, 11), 10, 1), X=M(range(1, 11), 10, 1), XData=pd.DataFrame({"a": np.arange(10)}))
    rl = H.HmscRandomLevel(units=np.arange(10))
    with pytest.raises(ValueError, match="number of rows in studyDesign"):
        H.Hmsc(Y=M(range(1, 11), 10, 1), X=M(range(1, 11), 10, 1), ranLevels={"sample": rl},
               studyDesign=pd.DataFrame({"sample": np.arange(9)}))
    with pytest.raises(ValueError, match="studyDesign must contain named columns"):
        H.Hmsc(Y=M(range(1, 11), 10, 1), X=M(range(1, 11), 10, 1), ranLevels={"unit": rl},
               studyDesign=pd.DataFrame({"sample": np.arange(10)}))


def test_priors_defaults_and_checks():
    """R/setPriors.Hmsc.R:28-101 defaults; test-setPriors.R."""
    m = H.Hmsc(Y=M(range(1, 21), 10, 2), X=np.column_stack([np.ones(10), np.arange(10.0)]))
    assert np.array_equal(m.V0, np.eye(2)) and m.f0 == 3 and np.all(m.mGamma == 0)
    assert np.array_equal(m.UGamma, np.eye(2)) and np.all(m.aSigma == 1) and np.all(m.bSigma == 5)
    assert m.rhopw.shape == (101, 2) and m.rhopw[0, 1] == 0.5
    with pytest.raises(ValueError, match="f0 must be greater"):
        H.setPriors(m, f0=1)
    with pytest.raises(ValueError, match="V0 must be a positive definite"):
        H.setPriors(m, V0=np.eye(3))
    with pytest.raises(ValueError, match="no phylogenic relationship"):
        H.setPriors(m, rhopw=np.ones((3, 2)))


def test_random_level():
    """R/HmscRandomLevel.R + test-setRL.R: defaults and nf truncation."""
    rl = H.HmscRandomLevel(units=["a", "b", "c", "a"])
    assert rl.pi == ["a", "b", "c"] and rl.N == 4 and rl.sDim == 0
    assert (rl.nu, rl.a1, rl.b1, rl.a2, rl.b2) == (3, 50, 1, 50, 1)
    assert math.isinf(rl.nfMax) and rl.nfMin == 2
    with pytest.raises(ValueError, match="At least one argument"):
        H.HmscRandomLevel()
    with pytest.raises(ValueError, match="nfMin must be not greater than nfMax"):
        H.setPriors(H.HmscRandomLevel(N=5), nfMax=2, nfMin=3)
    sp = H.HmscRandomLevel(sData=np.array([[0, 0], [3, 4.0]]))
    assert sp.sDim == 2 and sp.alphapw.shape == (101, 2) and sp.alphapw[-1, 0] == pytest.approx(5.0)
    m = H.Hmsc(Y=M(range(1, 21), 10, 2), X=M(range(1, 11), 10, 1), ranLevels={"u": H.HmscRandomLevel(N=10)},
               studyDesign=pd.DataFrame({"u": np.arange(10)}))
    assert m.rL[0].nfMax == 2 and m.rL[0].nfMin == 2     # truncateNumberOfFactors: nfMax = min(nfMax, ns)
    assert m.nr == 1 and list(m.np) == [10] and m.Pi[:, 0].tolist() == list(range(1, 11))


def test_sample_mcmc_argument_checks():
    """R/sampleMcmc.R:72-80 (checked before any device work)."""
    m = H.Hmsc(Y=M(range(1, 21), 10, 2), X=M(range(1, 11), 10, 1), distr="normal")
    with pytest.raises(ValueError, match="no less than any element of adaptNf"):
        H.sampleMcmc(m, samples=10, transient=5, adaptNf=[6])
    with pytest.raises(NotImplementedError):
        H.sampleMcmc(m, samples=10, fromPrior=True)
