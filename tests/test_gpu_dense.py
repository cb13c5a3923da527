"""The blocked multi-workgroup fp64 Cholesky and triangular solves (hmsc_amd/csrc/dense.hip:
64-column panels, MFMA trailing update) against numpy, at sizes that are and are not
multiples of the panel width, and a non-positive-definite matrix."""
import numpy as np
import pytest

from helpers import H, rel_err
from hmsc_amd import _lib as L

pytestmark = pytest.mark.gpu


def _spd(n, seed):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((n, n + 5))
    return X @ X.T / n + np.eye(n)


def _run(A, b):
    A = np.asfortranarray(A.copy())
    b = None if b is None else b.copy()
    info = np.zeros(1, dtype=np.int32)
    L.check(L.lib().hmsc_dense_chol_solve(0, L.fptr(A), A.shape[0], L.fptr(b) if b is not None else None,
                                          L.iptr(info)))
    return np.tril(A), b, int(info[0])


@pytest.mark.parametrize("n", [5, 64, 100, 777, 2500])
def test_blocked_cholesky_and_solves(n):
    A = _spd(n, n)
    b = np.random.default_rng(1).standard_normal(n)
    Lm, x, info = _run(A, b)
    assert info == 0
    assert rel_err(Lm, np.linalg.cholesky(A)) < 1e-12
    assert rel_err(x, np.linalg.solve(A, b)) < 1e-10


def test_blocked_cholesky_flags_indefinite():
    A = _spd(300, 3)
    A[200, 200] = -5.0
    _, _, info = _run(A, None)
    assert info == 1


def _grid_device(np_, coords=None, dist=None, alphas=None):
    G = len(alphas)
    iW = np.zeros((np_, np_, G), order="F")
    RiW = np.zeros((np_, np_, G), order="F")
    det = np.zeros(G)
    c = None if coords is None else np.asfortranarray(coords, dtype=np.float64)
    d = None if dist is None else np.asfortranarray(dist, dtype=np.float64)
    L.check(L.lib().hmsc_spatial_full_grid(0, np_, 0 if c is None else c.shape[1], L.fptr(c) if c is not None else None,
                                           L.fptr(d) if d is not None else None, G,
                                           L.fptr(np.asarray(alphas, dtype=np.float64)), L.fptr(iW), L.fptr(RiW),
                                           L.fptr(det)))
    return iW, RiW, det


@pytest.mark.parametrize("n", [40, 64, 200, 650])
def test_device_full_grid_matches_compute_data_parameters(n):
    """hmsc_spatial_full_grid (chol + trtri + lauum on the matrix cores) against the host
    restatement of R/computeDataParameters.R:53-81: iW, detW, and RiW' RiW = iW with RiW
    lower triangular; alpha = 0 gives the identity."""
    rng = np.random.default_rng(n)
    s = rng.random((n, 2))
    alphas = np.array([0.0, 0.02, 0.05, 0.1])
    iW, RiW, det = _grid_device(n, coords=s, alphas=alphas)
    d = np.sqrt(((s[:, None, :] - s[None, :, :]) ** 2).sum(-1))
    for g, a in enumerate(alphas):
        W = np.eye(n) if a == 0 else np.exp(-d / a)
        tol = max(1e-12, 100 * np.finfo(float).eps * np.linalg.cond(W))
        assert rel_err(iW[:, :, g], np.linalg.inv(W)) < tol, (g, a)
        assert np.array_equal(iW[:, :, g], iW[:, :, g].T)
        assert abs(det[g] - np.linalg.slogdet(W)[1]) < 1e-9 * max(1.0, abs(det[g]))
        assert np.all(np.triu(RiW[:, :, g], 1) == 0)
        assert rel_err(RiW[:, :, g], np.linalg.inv(np.linalg.cholesky(W))) < tol
        assert rel_err(RiW[:, :, g].T @ RiW[:, :, g], iW[:, :, g]) < 1e-12
    # distance-matrix input is the same grid
    iW2, RiW2, det2 = _grid_device(n, dist=d, alphas=alphas)
    assert rel_err(iW2, iW) < 1e-12 and rel_err(det2, det) < 1e-12


def test_device_full_grid_chain_matches_host_grid():
    """A 'Full' chain whose grid the device built and one given computeDataParameters' arrays
    sample the same Eta / Alpha path (the quadratic forms agree to rounding)."""
    from helpers import synthetic_model
    import hmsc_amd as HA
    hM = synthetic_model(ny=120, ns=4, nc=2, nf=2, nr=1, spatial=[0], seed=81, alpha_n=12)
    out = []
    for grid in ("device", "host"):
        ch = HA.Chain(hM, 17, device=0, spatial_grid=grid)
        ch.init([2])
        rec = ch.run(transient=0, samples=30, thin=1)
        out.append((rec["Eta0"], rec["Alpha0"]))
        ch.close()
    assert np.array_equal(out[0][1], out[1][1])
    assert rel_err(out[0][0], out[1][0]) < 1e-8
