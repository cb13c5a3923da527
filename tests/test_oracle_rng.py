"""The shared randomness contract (oracle/rng.py == hmsc_amd/csrc/rng.h) on CPU."""
import numpy as np
import pytest
from scipy import stats
from scipy.special import ndtri

from oracle.rng import Rng, philox4x32_10, qnorm_as241, trunc_normal_lower


@pytest.mark.parametrize("ctr,key,expect", [
    ((0, 0, 0, 0), (0, 0), (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
    ((0xffffffff,) * 4, (0xffffffff,) * 2, (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
    ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
     (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1)),
])
def test_philox_known_answers(ctr, key, expect):
    """Random123 philox4x32_10 KAT vectors."""
    out = philox4x32_10(*ctr, *key)
    assert tuple(int(x) for x in out) == expect


def test_qnorm_as241_accuracy():
    p = np.concatenate([np.logspace(-300, -1, 3000), np.linspace(1e-3, 1 - 1e-3, 5000), 1 - np.logspace(-15, -1, 500)])
    a, b = qnorm_as241(p), ndtri(p)
    assert np.max(np.abs(a - b) / np.maximum(np.abs(b), 1e-300)) < 5e-15


def test_uniforms_open_interval_and_independence():
    r = Rng(42)
    a, b = r.uniforms(np.arange(200000), 0, 12, 3)
    assert a.min() > 0 and a.max() < 1 and b.min() > 0 and b.max() < 1
    assert stats.kstest(a, "uniform").pvalue > 1e-3
    assert abs(np.corrcoef(a, b)[0, 1]) < 0.01
    c, _ = r.uniforms(np.arange(200000), 0, 12, 4)   # next sweep: a different stream
    assert abs(np.corrcoef(a, c)[0, 1]) < 0.01


def test_normal_distribution():
    x = Rng(7).normal(np.arange(200000), 0, 22, 5)
    assert stats.kstest(x, "norm").pvalue > 1e-3


@pytest.mark.parametrize("shape", [0.3, 1.0, 2.5, 50.0, 5000.0])
def test_gamma_distribution(shape):
    g = Rng(9).gamma_std(np.arange(100000), 20, 1, shape)
    assert stats.kstest(g, "gamma", args=(shape,)).pvalue > 1e-3


@pytest.mark.parametrize("alpha", [-6.0, -1.0, 0.0, 0.7, 3.0, 9.0, 30.0])
def test_truncated_normal(alpha):
    u = Rng(11).uniforms(np.arange(100000), 0, 12, 2)[0]
    x = trunc_normal_lower(np.full(u.shape, alpha), u)
    assert np.all(x >= alpha)
    if alpha <= 9:
        d = stats.truncnorm(alpha, np.inf)
        assert stats.kstest(x, d.cdf).pvalue > 1e-3
    else:
        # deep tail: (x - alpha) * alpha ~ Exp(1) to O(1/alpha^2)
        assert abs(np.mean((x - alpha) * alpha) - 1.0) < 0.02
