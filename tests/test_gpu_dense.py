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
