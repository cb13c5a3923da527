"""Fit the Chebyshev expansion used by the device erfc (hmsc_amd/csrc/rng.h, erfc_cheb).

For z >= 0, erfc(z) = t exp(-z^2 + g(t)) with t = 2 / (2 + z); g is smooth on t in (0, 1]
and is interpolated at the degree+1 Chebyshev nodes of x = 2t - 1.  The reference values
come from scipy's erfcx (log erfc(z) = log erfcx(z) - z^2, no underflow).  Prints the
coefficients (C initialiser) and the max relative error on z in [0, 18].
"""
import numpy as np
from numpy.polynomial import chebyshev as C
from scipy.special import erfc, erfcx

DEG = 24


def g_of_x(x):
    t = (x + 1) / 2
    z = 2 / t - 2
    return np.log(erfcx(z)) - np.log(t)


k = np.arange(DEG + 1)
xn = np.cos(np.pi * (k + 0.5) / (DEG + 1))
c = C.chebfit(xn, g_of_x(xn), DEG)
z = np.concatenate([np.linspace(0, 18, 400001), np.geomspace(1e-10, 18, 40001)])
t = 2 / (2 + z)
approx = t * np.exp(-z * z + C.chebval(2 * t - 1, c))
print("max rel err", np.max(np.abs(approx / erfc(z) - 1)))
print("{" + ", ".join(repr(float(v)) for v in c) + "}")
