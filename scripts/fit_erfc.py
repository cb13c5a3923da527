"""Fit the polynomial used by the device erfc (hmsc_amd/csrc/rng.h, erfc_fast).

For z >= 0, erfc(z) = t exp(-z^2) exp(g(t)), t = 2 / (2 + z); g is smooth on t in (0, 1]
and is interpolated at the DEG+1 Chebyshev nodes of x = 2t - 1 (reference values from
mpmath, 40 digits), then converted to monomials in x (Horner; the coefficients stay below
0.68 so the conversion is well conditioned).  exp(-z^2) is taken of the rounded square and
the rounding error of z*z (an fma) is folded into the second exponential, so the result
keeps ~1e-15 relative accuracy out to z = 18.  Prints the coefficients (Horner order,
highest degree first) and the max relative error against mpmath.
"""
import mpmath as mp
import numpy as np
from numpy.polynomial import chebyshev as C

DEG = 20
mp.mp.dps = 40


def g(x):
    t = (mp.mpf(x) + 1) / 2
    z = 2 / t - 2
    return mp.log(mp.erfc(z)) + z * z - mp.log(t)


def two_prod(a, b):
    p = a * b
    A = a * 134217729.0
    ah = A - (A - a)
    al = a - ah
    B = b * 134217729.0
    bh = B - (B - b)
    bl = b - bh
    return p, ((ah * bh - p) + ah * bl + al * bh) + al * bl


if __name__ == "__main__":
    k = np.arange(DEG + 1)
    xn = np.cos(np.pi * (k + 0.5) / (DEG + 1))
    mono = C.cheb2poly(C.chebfit(xn, np.array([float(g(v)) for v in xn]), DEG))[::-1]
    z = np.concatenate([np.linspace(0, 18, 4001), np.geomspace(1e-10, 18, 2001)])
    t = 2 / (2 + z)
    x = 2 * t - 1
    gx = np.zeros_like(x)
    for a in mono:
        gx = gx * x + a
    zz, err = two_prod(z, z)
    approx = t * np.exp(-zz) * np.exp(gx - err)
    ref = np.array([float(mp.erfc(mp.mpf(v))) for v in z])
    print("max rel err", np.max(np.abs(approx / ref - 1)))
    print("{" + ", ".join(repr(float(v)) for v in mono) + "}")
