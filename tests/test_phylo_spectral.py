"""CPU check of the spectral form of the phylogeny grid (hmsc_amd/csrc/phylo.hip) against the
oracle's literal restatement of R/computeDataParameters.R:19-39 and R/updateRho.R:14-17.

With C = U diag(d) U^T, Q_g = U diag(q_g) U^T and every quantity the sampler takes from the
grid follows from U and q: iQg, logdet Q_g, and updateRho's v_g = |RQ_g^-T E RiV^T|^2.
"""
import numpy as np

from helpers import O, phylo_corr


def _spectral(C, rhopw):
    d, U = np.linalg.eigh(C)
    rho = rhopw[:, 0][:, None]
    q = np.where(rho >= 0, rho * d[None, :] + 1 - rho, -rho / d[None, :] + 1 + rho)
    return U, q


def test_grid_matches_dense_restatement():
    ns = 9
    C = phylo_corr(ns, seed=3)
    rhopw = np.column_stack([np.linspace(-0.5, 1.0, 31), np.full(31, 1 / 31)])
    dp = O.compute_data_parameters(dict(Y=np.zeros((2, ns)), C=C, rhopw=rhopw))
    U, q = _spectral(C, rhopw)
    for g in range(rhopw.shape[0]):
        iQ = (U / q[g]) @ U.T
        np.testing.assert_allclose(iQ, dp["iQg"][g], rtol=0, atol=1e-10 * np.abs(dp["iQg"][g]).max())
        np.testing.assert_allclose(np.log(q[g]).sum(), dp["detQg"][g], rtol=1e-12, atol=1e-12)


def test_rho_quadratic_form_matches_backsolves():
    rng = np.random.default_rng(5)
    ns, nc, nt = 12, 3, 2
    C = phylo_corr(ns, seed=5)
    rhopw = np.column_stack([np.arange(101) / 100, np.r_[0.5, np.full(100, 0.005)]])
    dp = O.compute_data_parameters(dict(Y=np.zeros((2, ns)), C=C, rhopw=rhopw))
    Beta = rng.standard_normal((nc, ns))
    Gamma = rng.standard_normal((nc, nt))
    Tr = rng.standard_normal((ns, nt))
    A = rng.standard_normal((nc, nc))
    iV = A @ A.T + nc * np.eye(nc)
    E = (Beta - Gamma @ Tr.T).T @ O.chol_upper(iV).T
    v_ref = np.array([np.sum(O.backsolve(dp["RQg"][g], E, transpose=True) ** 2) for g in range(101)])
    U, q = _spectral(C, rhopw)
    Et = (Beta - Gamma @ Tr.T) @ U                     # nc x ns, = Bt - Gamma Tt^T
    s = np.einsum("ci,cd,di->i", Et, iV, Et)
    v = (s[None, :] / q).sum(axis=1)
    np.testing.assert_allclose(v, v_ref, rtol=1e-11)
