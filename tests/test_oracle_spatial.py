"""NNGP and GPP spatial levels on the host and in the oracle, no GPU.

The device runs every spatial method through one dense (np nf)^2 updateEta / updateAlpha
path on the prior precision of the alphapw grid.  These tests pin that
reduction: the product grid (hmsc_amd/dataparams.py) equals the oracle restatement of
R/computeDataParameters.R:82-194; the NNGP factor reproduces iWg; the GPP precision is the
inverse of W = D + W12 iW22 W12' with detDg = log det W; and R's own GPP updateEta
(R/updateEta.R:148-196, oracle gpp_eta_literal) has the same posterior mean and covariance
as the dense system, and R's GPP updateAlpha statistic equals |RiWg eta_h|^2.
FNN::get.knn is restated by brute force (parity unpinned against FNN itself: it is not in
the reference and R is not installed; exact kNN is unique for continuous coordinates)."""
import numpy as np
import pytest

from helpers import H, O, oracle_model, rel_err, synthetic_model
from hmsc_amd import dataparams as DPm


def _model(method, **kw):
    base = dict(ny=40, ns=6, nc=2, nf=2, nr=1, spatial=[0], seed=52, spatial_method=method, n_neighbours=5)
    base.update(kw)
    return synthetic_model(**base)


@pytest.fixture(scope="module", params=["NNGP", "GPP"])
def grids(request):
    hM = _model(request.param)
    m = oracle_model(hM)
    return request.param, hM, m, DPm.spatialDataParameters(hM)[0], O.compute_data_parameters(m)


def test_product_grid_matches_oracle(grids):
    meth, hM, m, prod, dp = grids
    orc = dp["rLPar"][0]
    G = prod["iWg"].shape[2]
    for g in range(G):
        assert rel_err(prod["iWg"][:, :, g], orc["iWg"][g]) < 1e-11, (meth, g)
        assert rel_err(prod["RiWg"][:, :, g], orc["RiWg"][g]) < 1e-9, (meth, g)
    assert rel_err(prod["detWg"], orc["detWg"]) < 1e-12
    if meth == "GPP":
        for k in ("idDW12g", "Fg", "iFg"):
            assert rel_err(np.moveaxis(prod[k], 2, 0), orc[k]) < 1e-11, k
        assert rel_err(prod["idDg"].T, orc["idDg"]) < 1e-12


def test_factor_reproduces_precision(grids):
    meth, hM, m, prod, dp = grids
    for g in (0, 5, 50, 100):
        R = prod["RiWg"][:, :, g]
        assert rel_err(R.T @ R, prod["iWg"][:, :, g]) < 1e-10, (meth, g)
    assert np.array_equal(prod["iWg"][:, :, 0], np.eye(hM.np[0]))     # alpha = 0: independent units
    assert prod["detWg"][0] == 0.0


def test_nngp_structure():
    hM = _model("NNGP")
    prod = DPm.spatialDataParameters(hM)[0]
    s = np.asarray(hM.rL[0].s)
    nn = DPm.knn_index(s, 5)
    R = prod["RiWg"][:, :, 30]
    for i in range(s.shape[0]):       # row i of the Vecchia factor touches only i and its earlier neighbours
        allowed = set(nn[i][nn[i] < i]) | {i}
        assert set(np.nonzero(R[i])[0]) <= allowed
    assert np.allclose(np.triu(R, 1), 0.0)
    # NNGP with every earlier unit as a neighbour is the exact Full precision
    hF = _model("NNGP", n_neighbours=39)
    full = _model("Full")
    a = DPm.spatialDataParameters(hF)[0]
    b = DPm.spatialDataParameters(full)[0]
    for g in (3, 40, 100):
        assert rel_err(a["iWg"][:, :, g], b["iWg"][:, :, g]) < 1e-7, g
        assert abs(a["detWg"][g] - b["detWg"][g]) < 1e-7 * max(1, abs(b["detWg"][g]))


def test_gpp_precision_is_inverse_covariance():
    hM = _model("GPP")
    prod = DPm.spatialDataParameters(hM)[0]
    s = np.asarray(hM.rL[0].s)
    sK = np.asarray(hM.rL[0]["sKnot"])
    d12 = np.sqrt(((s[:, None] - sK[None]) ** 2).sum(-1))
    d22 = np.sqrt(((sK[:, None] - sK[None]) ** 2).sum(-1))
    for g in (4, 30, 80):
        a = hM.rL[0].alphapw[g, 0]
        W12, W22 = np.exp(-d12 / a), np.exp(-d22 / a)
        Q = W12 @ np.linalg.solve(W22, W12.T)
        W = Q + np.diag(1 - np.diag(Q))
        assert rel_err(prod["iWg"][:, :, g] @ W, np.eye(s.shape[0])) < 1e-8, g
        assert abs(prod["detWg"][g] - np.linalg.slogdet(W)[1]) < 1e-8 * max(1, abs(prod["detWg"][g]))


def _state(m, dp, seed=9):
    from oracle.rng import Rng
    rng = Rng(seed)
    st = O.compute_initial_parameters(m, rng)
    st["Alpha"] = [np.array([9, 25])]
    xy = m["rL"][0]["s"]
    st["Eta"] = [np.column_stack([np.sin(3 * xy[:, 0]) + xy[:, 1], np.cos(2 * xy[:, 1])])]
    return st


def test_gpp_literal_eta_equals_dense_posterior():
    hM = _model("GPP")
    m = oracle_model(hM)
    dp = O.compute_data_parameters(m)
    st = _state(m, dp)
    S = st["Z"] - m["X"] @ st["Beta"]
    mean_lit, cov_lit = O.gpp_eta_literal(st, m, 0, S, dp)
    mean_dense = O._eta_spatial_full(st, m, 0, S, dp, None, 0, True)
    assert rel_err(mean_lit, mean_dense) < 1e-9
    # dense posterior precision: bdiag(iWg[alpha_h]) + kron(Lam iSigma Lam', I)
    lam, iS = st["Lambda"][0], st["iSigma"]
    n, nf = mean_dense.shape
    P = np.kron(lam @ (iS[:, None] * lam.T), np.eye(n))
    for h in range(nf):
        P[h * n:(h + 1) * n, h * n:(h + 1) * n] += dp["rLPar"][0]["iWg"][st["Alpha"][0][h] - 1]
    assert rel_err(cov_lit @ P, np.eye(n * nf)) < 1e-8


@pytest.mark.parametrize("method", ["NNGP", "GPP"])
def test_alpha_statistic(method):
    hM = _model(method)
    m = oracle_model(hM)
    dp = O.compute_data_parameters(m)
    st = _state(m, dp)
    from oracle.rng import Rng
    a = O.update_alpha(st, m, Rng(3), 11, dp)[0]
    # the dense statistic the device evaluates gives the same draw
    m2 = oracle_model(hM)
    m2["rL"][0]["spatialMethod"] = "Full"
    b = O.update_alpha(st, m2, Rng(3), 11, dp)[0]
    assert np.array_equal(a, b) and np.all(a >= 1)


def test_construct_knots():
    rng = np.random.default_rng(0)
    s = rng.random((200, 2)) * [2.0, 1.0]
    k = DPm.constructKnots(s, nKnots=5)
    step = (s[:, 1].max() - s[:, 1].min()) / 5
    assert k.shape[1] == 2 and k.shape[0] > 20
    assert np.allclose(np.diff(np.unique(k[:, 0])), step)
    assert k[1, 0] > k[0, 0] and k[1, 1] == k[0, 1]          # expand.grid: first axis fastest
    with pytest.raises(ValueError):
        DPm.constructKnots(s, nKnots=5, knotDist=0.1)


def test_model_buffers_accept_nngp_gpp():
    from hmsc_amd.sampler import ModelBuffers, SPATIAL_CODE
    for meth in ("NNGP", "GPP"):
        b = ModelBuffers(_model(meth))
        assert b.struct.spatialMethod[0] == SPATIAL_CODE[meth]


@pytest.mark.parametrize("kw", [
    dict(ny=50, ns=4, nc=3, nf=2, nr=2, units=[50, 10], spatial=[1], seed=51, alpha_n=30, nt=2),
    dict(ny=30, ns=5, nc=2, nf=2, nr=1, spatial=[0], seed=52)])
def test_spatial_gamma_eta_natural_form_equals_literal(kw):
    """R/updateGammaEta.R:139-194's mean chain (mg, me) equals iG^-1 (c0 - C'H^-1 s), the
    natural form the device kernel evaluates; both use the same iG."""
    from oracle.rng import Rng
    hM = synthetic_model(**kw)
    m = oracle_model(hM)
    dp = O.compute_data_parameters(m)
    st = O.compute_initial_parameters(m, Rng(5))
    r = [k for k, rl in enumerate(m["rL"]) if rl["sDim"]][0]
    st["Alpha"] = list(st["Alpha"])
    st["Alpha"][r] = np.array([7, 12])
    S = st["Z"] - sum(O.l_ran(st, m, q) for q in range(len(m["rL"])) if q != r)
    iQ, Q = dp["iQg"][0], dp["Qg"][0]
    iV = st["iV"]
    V = O.chol2inv(O.chol_upper(iV))
    U = m["UGamma"]
    iU = O.chol2inv(O.chol_upper(U))
    KT = np.kron(m["Tr"], np.eye(m["X"].shape[1]))
    iA = O.chol2inv(O.chol_upper(KT @ U @ KT.T + np.kron(Q, V)))
    m1, g1 = O.gamma_eta_spatial_literal(st, m, r, S, dp, iQ, iV, U, iU, iA)
    m2, g2 = O.gamma_eta_spatial_natural(st, m, r, S, dp, iQ, iV, iU)
    assert rel_err(g1, g2) < 1e-12
    assert rel_err(m1, m2) < 1e-10


def test_gpp_knot_on_a_site():
    """A knot (almost) on a sampling unit makes dD ~ 0 there (idD huge in R's form, where
    diag(idD) - idDW12 iF idDW12' loses digits to cancellation); the dense precision, built from
    W = D + W12 iW22 W12' itself, stays accurate.  (Exactly on a site, R's own DS / F are
    infinite and R fails too.)"""
    hM = _model("GPP")
    rl = hM.rL[0]
    s = np.asarray(rl.s)
    rl["sKnot"] = np.vstack([np.asarray(rl["sKnot"]), s[7] + 1e-6])
    prod = DPm.spatialDataParameters(hM)[0]
    sK = np.asarray(rl["sKnot"])
    d12 = np.sqrt(((s[:, None] - sK[None]) ** 2).sum(-1))
    d22 = np.sqrt(((sK[:, None] - sK[None]) ** 2).sum(-1))
    for g in (10, 60):
        a = rl.alphapw[g, 0]
        Q = np.exp(-d12 / a) @ np.linalg.solve(np.exp(-d22 / a), np.exp(-d12 / a).T)
        W = Q + np.diag(1 - np.diag(Q))
        assert np.all(np.isfinite(prod["iWg"][:, :, g]))
        assert rel_err(prod["iWg"][:, :, g] @ W, np.eye(s.shape[0])) < 1e-6, g


def test_model_buffers_full_grid_routing():
    """'Full' levels hand their coordinates (unit order) to the device by default and
    computeDataParameters' arrays with spatial_grid='host'; NNGP its coordinates and
    nNeighbours (the library builds the sparse Vecchia factor), GPP R's low-rank arrays (nKnots,
    idDg, idDW12g, Fg, iFg, detDg); neither passes an np^2 array."""
    from hmsc_amd.sampler import ModelBuffers
    hM = _model("Full")
    b = ModelBuffers(hM)
    m = b.struct
    assert bool(m.sCoord[0]) and not bool(m.iWg[0]) and not bool(m.distMat[0])
    assert m.sDim[0] == hM.rL[0].s.shape[1]
    h = ModelBuffers(hM, spatial_grid="host").struct
    assert bool(h.iWg[0]) and bool(h.RiWg[0]) and not bool(h.sCoord[0])
    g = ModelBuffers(_model("GPP")).struct
    assert not bool(g.iWg[0]) and not bool(g.RiWg[0]) and not bool(g.sCoord[0])
    assert g.nKnots[0] > 0 and all(bool(getattr(g, f)[0]) for f in ("idDg", "idDW12g", "Fg", "iFg", "detDg"))
    n = ModelBuffers(_model("NNGP")).struct
    assert not bool(n.iWg[0]) and not bool(n.RiWg[0]) and bool(n.sCoord[0])
    assert n.nNeighbours[0] == int(_model("NNGP").rL[0].nNeighbours or 10)
    assert m.struct_size == n.struct_size > 0
    with pytest.raises(ValueError):
        ModelBuffers(hM, spatial_grid="cpu")
