"""ORACLE — test infrastructure only (never imported by the product path).

numpy restatement of the counter-based randomness contract of
``hmsc_amd/csrc/rng.h``: Philox4x32-10 (Salmon et al., SC'11; Random123 KAT
vectors checked in tests/test_oracle_rng.py), 53-bit open-interval uniforms,
Box-Muller normals, Marsaglia-Tsang gammas, inverse-CDF one-sided truncated
normals.  It stands in for the unvendored samplers the reference calls:
stats::rnorm / rgamma (R/updateLambdaPriors.R:23-32, R/updateInvSigma.R:40),
truncnorm::rtruncnorm (R/updateZ.R:59), MCMCpack::rwish (R/updateGammaV.R:21).
Those libraries are not present here (R is absent); the restated algorithms are
the published ones, and parity with the reference is pinned at the level of
conditional moments and posterior distributions, not R's RNG bitstream.
"""
import numpy as np
from scipy.special import erfc, erfcinv

M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = 0x9E3779B9, 0xBB67AE85
MASK = np.uint64(0xFFFFFFFF)

# stream ids — must match enum Stream in rng.h
S_GAMMA2 = 1
S_BETALAMBDA = 3
S_WISHART_DIAG = 4
S_WISHART_OFF = 5
S_GAMMAV = 6
S_RHO = 7
S_INVSIGMA = 11
S_Z = 12
S_PSI = 20
S_DELTA = 21
S_ETA = 22
S_ALPHA = 23
S_NF = 24
S_NF_ETA = 25
S_NF_PSI = 26
S_NF_DELTA = 27
S_INIT_GAMMA = 40
S_INIT_V_DIAG = 41
S_INIT_V_OFF = 42
S_INIT_BETA = 43
S_INIT_SIGMA = 44
S_INIT_DELTA = 50
S_INIT_PSI = 51
S_INIT_LAMBDA = 52
S_INIT_ETA = 53
LEVEL_STRIDE = 256
GAMMA_BOOST_SUB = 0xFFFF0000
GAMMA_MAX_TRIALS = 64


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Vectorised Philox4x32-10 over broadcastable uint32 counter arrays."""
    c0, c1, c2, c3 = [np.asarray(c, dtype=np.uint64) & MASK for c in (c0, c1, c2, c3)]
    c0, c1, c2, c3 = np.broadcast_arrays(c0, c1, c2, c3)
    k0 = int(k0) & 0xFFFFFFFF
    k1 = int(k1) & 0xFFFFFFFF
    for _ in range(10):
        p0 = M0 * c0
        p1 = M1 * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & MASK
        hi1, lo1 = p1 >> np.uint64(32), p1 & MASK
        c0, c1, c2, c3 = hi1 ^ c1 ^ np.uint64(k0), lo1, hi0 ^ c3 ^ np.uint64(k1), lo0
        k0 = (k0 + W0) & 0xFFFFFFFF
        k1 = (k1 + W1) & 0xFFFFFFFF
    return c0, c1, c2, c3


def u53(hi, lo):
    return ((hi >> np.uint64(5)).astype(np.float64) * 67108864.0
            + (lo >> np.uint64(6)).astype(np.float64) + 0.5) * (1.0 / 9007199254740992.0)


class Rng:
    """Key = one chain's 64-bit seed; ``iter`` = sweep number (0 for initialisation)."""

    def __init__(self, seed):
        seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        self.k0 = seed & 0xFFFFFFFF
        self.k1 = seed >> 32

    def uniforms(self, idx, sub, stream, it):
        x, y, z, w = philox4x32_10(idx, sub, stream, it, self.k0, self.k1)
        return u53(x, y), u53(z, w)

    def normal(self, idx, sub, stream, it):
        a, b = self.uniforms(idx, sub, stream, it)
        return np.sqrt(-2.0 * np.log(a)) * np.cos(6.283185307179586 * b)

    def gamma_std(self, idx, stream, it, shape):
        """Marsaglia-Tsang Gamma(shape, 1), elementwise over ``idx``/``shape``."""
        idx = np.asarray(idx, dtype=np.uint64)
        shape = np.asarray(shape, dtype=np.float64)
        idx, shape = np.broadcast_arrays(idx, shape)
        a = np.where(shape < 1.0, shape + 1.0, shape)
        d = a - 1.0 / 3.0
        c = 1.0 / np.sqrt(9.0 * d)
        out = d.copy()
        done = np.zeros(idx.shape, dtype=bool)
        for t in range(GAMMA_MAX_TRIALS):
            if done.all():
                break
            x = self.normal(idx, 2 * t, stream, it)
            v = 1.0 + c * x
            ok = v > 0.0
            v3 = np.where(ok, v, 1.0) ** 3
            u = self.uniforms(idx, 2 * t + 1, stream, it)[0]
            with np.errstate(invalid="ignore", divide="ignore"):
                acc = ok & (np.log(u) < 0.5 * x * x + d - d * v3 + d * np.log(v3))
            newly = acc & ~done
            out = np.where(newly, d * v3, out)
            done |= acc
        boost = shape < 1.0
        if boost.any():
            u = self.uniforms(idx, GAMMA_BOOST_SUB, stream, it)[0]
            out = np.where(boost, out * u ** (1.0 / shape), out)
        return out

    def gamma(self, idx, stream, it, shape, rate):
        return self.gamma_std(idx, stream, it, shape) / np.asarray(rate, dtype=np.float64)


def trunc_normal_lower(alpha, u):
    """Standard normal truncated to [alpha, inf) by upper-tail inversion (rng.h)."""
    alpha = np.asarray(alpha, dtype=np.float64)
    with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
        t = u * erfc(alpha * 0.7071067811865476)
        x = 1.4142135623730951 * erfcinv(t)
        tail = alpha - np.log(u) / np.where(alpha == 0, 1.0, alpha)
    return np.where(alpha > 25.0, tail, x)
