"""Fit the division-free normal quantile used by the device truncated-normal draw
(hmsc_amd/csrc/rng.h, qnorm_fast).

Phi^-1(p) = y F(w),   y = 2p - 1,   w = -log(4 p (1 - p))       (Giles 2010 form)
  region A  w in [0, 6.25]         F = polyA(w - 3.125)
  region B  w in [6.25, 16]        F = polyB(sqrt(w) - 3.25)
  region C  w >= 16 (p < 2.8e-8, rare)   AS241's tail branch (rng.h qnorm_as241_tail)
Reference values from mpmath at 40 digits.  Prints monomial coefficients (Horner order,
highest first) and the max relative error of a float64 Horner evaluation against
scipy's ndtri on dense p grids.
"""
import sys

import mpmath as mp
import numpy as np
from scipy.special import ndtri

mp.mp.dps = 40


def F_of_w(w):
    """Phi^-1(p) / (2p - 1) at the lower root p of 4 p (1 - p) = exp(-w)."""
    w = mp.mpf(w)
    e = mp.exp(-w)
    p = e / (2 * (1 + mp.sqrt(-mp.expm1(-w))))
    if w < 1:
        y = mp.sqrt(-mp.expm1(-w))
        return mp.sqrt(2) * mp.erfinv(y) / y
    x0 = -mp.sqrt(2 * w)
    lp = mp.log(p)
    x = mp.findroot(lambda x: mp.log(mp.erfc(-x / mp.sqrt(2)) / 2) - lp, x0)
    return x / (2 * p - 1)


def fit(var_to_w, lo, hi, deg, center=0.0):
    """Least squares on Chebyshev nodes of the fit variable v in [lo, hi]; returns monomial
    coefficients in (v - center), highest degree first."""
    n = 4 * deg + 40
    k = np.arange(n)
    xs = np.cos(np.pi * (k + 0.5) / n)
    vs = [mp.mpf(lo) + (mp.mpf(hi) - lo) * (mp.mpf(x) + 1) / 2 for x in xs]
    fs = [F_of_w(var_to_w(v)) for v in vs]
    # solve the least-squares problem in extended precision, basis (v - center)^j scaled
    half = (mp.mpf(hi) - lo) / 2
    A = mp.matrix(n, deg + 1)
    b = mp.matrix(n, 1)
    for i, v in enumerate(vs):
        t = (v - center) / half
        for j in range(deg + 1):
            A[i, j] = t ** j
        b[i] = fs[i]
    # relative weighting
    for i in range(n):
        wgt = 1 / fs[i]
        for j in range(deg + 1):
            A[i, j] *= wgt
        b[i] *= wgt
    coef = mp.lu_solve(A.T * A, A.T * b)
    return [float(coef[j] / half ** j) for j in range(deg, -1, -1)]


def horner(c, t):
    r = np.full_like(t, c[0])
    for a in c[1:]:
        r = r * t + a
    return r


def qnorm_fast(p, cA, cB):
    from scipy.special import ndtri as as241_stand_in  # region C is AS241 on the device
    p = np.asarray(p, dtype=np.float64)
    y = 2.0 * p - 1.0
    w = -np.log(4.0 * p * (1.0 - p))
    s = np.sqrt(w)
    out = np.where(w < 6.25, y * horner(cA, w - 3.125), y * horner(cB, s - 3.25))
    return np.where(w < 16.0, out, as241_stand_in(p))


if __name__ == "__main__":
    degA, degB = (int(a) for a in sys.argv[1:3]) if len(sys.argv) > 2 else (18, 14)
    cA = fit(lambda v: v, 0.0, 6.25, degA, center=3.125)
    cB = fit(lambda v: v * v, 2.5, 4.0, degB, center=3.25)
    rng = np.random.default_rng(0)
    p = np.concatenate([rng.random(2_000_000), np.geomspace(1e-170, 0.5, 400_000), 1 - np.geomspace(1e-16, 0.5, 200_000)])
    ref = ndtri(p)
    got = qnorm_fast(p, cA, cB)
    rel = np.abs(got - ref) / np.maximum(np.abs(ref), 1e-300)
    rel[p == 0.5] = 0.0
    print("max rel err vs ndtri", rel.max(), "at p =", p[np.argmax(rel)])
    for name, c in (("A", cA), ("B", cB)):
        print(f"constexpr double QN_{name}[{len(c)}] = {{" + ", ".join(repr(v) for v in c) + "};")
