"""ORACLE — test infrastructure only (never imported by the product path).

numpy restatement of the counter-based randomness contract of
``hmsc_amd/csrc/rng.h``: Philox4x32-10 (Salmon et al., SC'11; Random123 KAT
vectors checked in tests/test_oracle_rng.py), 53-bit open-interval uniforms,
inverse-CDF normals, Marsaglia-Tsang gammas, inverse-CDF one-sided truncated
normals.  It stands in for the unvendored samplers the reference calls:
stats::rnorm / rgamma (R/updateLambdaPriors.R:23-32, R/updateInvSigma.R:40),
truncnorm::rtruncnorm (R/updateZ.R:59), MCMCpack::rwish (R/updateGammaV.R:21).
Those libraries are not present here (R is absent); the restated algorithms are
the published ones, and parity with the reference is pinned at the level of
conditional moments and posterior distributions, not R's RNG bitstream.
"""
import numpy as np
from scipy.special import erfc

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
S_GE_BETA = 8
S_GE_GAMMA = 9
S_GE_ETA = 10
S_INVSIGMA = 11
S_Z = 12
S_ZPOIS = 13
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


def u32o(w):
    """Open-interval uniform from one 32-bit word, (w + 1/2) 2^-32 (rng.h u32o, exact in
    double): updateZ's uniforms, at the resolution of R's own unif_rand (Mersenne-Twister)."""
    return (np.asarray(w, dtype=np.uint64).astype(np.float64) + 0.5) * (1.0 / 4294967296.0)


class Rng:
    """Key = one chain's 64-bit seed; ``iter`` = sweep number (0 for initialisation)."""

    def __init__(self, seed):
        seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        self.k0 = seed & 0xFFFFFFFF
        self.k1 = seed >> 32

    def uniforms(self, idx, sub, stream, it):
        x, y, z, w = philox4x32_10(idx, sub, stream, it, self.k0, self.k1)
        return u53(x, y), u53(z, w)

    def words(self, idx, sub, stream, it):
        """The block's four 32-bit words (uint64 arrays)."""
        return philox4x32_10(idx, sub, stream, it, self.k0, self.k1)

    def normal(self, idx, sub, stream, it):
        """Standard normal by inversion of the first uniform of the (idx, sub) block
        (R's own default rnorm method, INVERSION)."""
        a, _ = self.uniforms(idx, sub, stream, it)
        return qnorm_as241(a)

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
            vv = np.where(ok, v, 1.0)
            v3 = vv * vv * vv  # same rounding as rng.h (v*v*v)
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


def qnorm_as241(p):
    """Phi^-1(p): Wichura (1988) AS241 PPND16, the algorithm of R's qnorm (rng.h mirror)."""
    p = np.asarray(p, dtype=np.float64)
    q = p - 0.5
    out = np.empty_like(p)
    c = np.abs(q) <= 0.425
    r = 0.180625 - q[c] * q[c]
    num = (((((((2.5090809287301226727e+3 * r + 3.3430575583588128105e+4) * r + 6.7265770927008700853e+4) * r
                + 4.5921953931549871457e+4) * r + 1.3731693765509461125e+4) * r + 1.9715909503065514427e+3) * r
            + 1.3314166789178437745e+2) * r + 3.3871328727963666080e0)
    den = (((((((5.2264952788528545610e+3 * r + 2.8729085735721942674e+4) * r + 3.9307895800092710610e+4) * r
                + 2.1213794301586595867e+4) * r + 5.3941960214247511077e+3) * r + 6.8718700749205790830e+2) * r
            + 4.2313330701600911252e+1) * r + 1.0)
    out[c] = q[c] * num / den
    t = ~c
    if t.any():
        qt, pt = q[t], p[t]
        rr = np.sqrt(-np.log(np.where(qt < 0, pt, 1.0 - pt)))
        lo = rr <= 5.0
        r1 = rr - 1.6
        n1 = (((((((7.74545014278341407640e-4 * r1 + 2.27238449892691845833e-2) * r1 + 2.41780725177450611770e-1) * r1
                  + 1.27045825245236838258e0) * r1 + 3.64784832476320460504e0) * r1 + 5.76949722146069140550e0) * r1
               + 4.63033784615654529590e0) * r1 + 1.42343711074968357734e0)
        d1 = (((((((1.05075007164441684324e-9 * r1 + 5.47593808499534494600e-4) * r1 + 1.51986665636164571966e-2) * r1
                  + 1.48103976427480074590e-1) * r1 + 6.89767334985100004550e-1) * r1 + 1.67638483018380384940e0) * r1
               + 2.05319162663775882187e0) * r1 + 1.0)
        r2 = rr - 5.0
        n2 = (((((((2.01033439929228813265e-7 * r2 + 2.71155556874348757815e-5) * r2 + 1.24266094738807843860e-3) * r2
                  + 2.65321895265761230930e-2) * r2 + 2.96560571828504891230e-1) * r2 + 1.78482653991729133580e0) * r2
               + 5.46378491116411436990e0) * r2 + 6.65790464350110377720e0)
        d2 = (((((((2.04426310338993978564e-15 * r2 + 1.42151175831644588870e-7) * r2 + 1.84631831751005468180e-5) * r2
                  + 7.86869131145613259100e-4) * r2 + 1.48753612908506148525e-2) * r2 + 1.36929880922735805310e-1) * r2
               + 5.99832206555887937690e-1) * r2 + 1.0)
        val = np.where(lo, n1 / d1, n2 / d2)
        out[t] = np.where(qt < 0, -val, val)
    return out


def trunc_normal_lower(alpha, u):
    """Standard normal truncated to [alpha, inf) by upper-tail inversion (rng.h):
    x = -qnorm(u * Phic(alpha)), exponential tail beyond alpha > 25."""
    alpha, u = np.broadcast_arrays(np.asarray(alpha, dtype=np.float64), np.asarray(u, dtype=np.float64))
    with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
        p = u * (0.5 * erfc(alpha * 0.7071067811865476))
        x = -qnorm_as241(p.ravel()).reshape(p.shape)
        tail = alpha - np.log(u) / np.where(alpha == 0, 1.0, alpha)
    return np.where(alpha > 25.0, tail, x)
