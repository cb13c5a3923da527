"""Config 5 diagnostics on the GPU box: (a) the device 'Full' alphapw grid
(hmsc_spatial_full_grid) against numpy at a large np for a few alphas; (b) the alpha trace of
a 'Full' and a 'GPP' chain of spatial_vignette4 at ny = --ny.  Prints one JSON line."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import hmsc_amd as H  # noqa: E402
from hmsc_amd import _lib as L  # noqa: E402


def grid_check(npts, alphas, seed=3):
    rng = np.random.default_rng(seed)
    xy = rng.random((npts, 2))
    G = len(alphas)
    iW = np.zeros(npts * npts * G)
    RiW = np.zeros(npts * npts * G)
    det = np.zeros(G)
    crd = np.asfortranarray(xy).ravel(order="F")
    t0 = time.time()
    L.check(L.lib().hmsc_spatial_full_grid(0, npts, 2, L.fptr(crd), None, G, L.fptr(np.asarray(alphas, float)),
                                           L.fptr(iW), L.fptr(RiW), L.fptr(det)))
    t_dev = time.time() - t0
    d = np.sqrt(((xy[:, None, :] - xy[None, :, :]) ** 2).sum(-1))
    out = []
    for g, a in enumerate(alphas):
        W = np.exp(-d / a) if a > 0 else np.eye(npts)
        Lc = np.linalg.cholesky(W)
        det_ref = 2 * np.sum(np.log(np.diag(Lc)))
        R = RiW[g * npts * npts:(g + 1) * npts * npts].reshape(npts, npts, order="F")
        I = iW[g * npts * npts:(g + 1) * npts * npts].reshape(npts, npts, order="F")
        # R = chol(W)^-1 (lower): R W R^T = I and R^T R = iW
        e1 = float(np.max(np.abs(R @ W @ R.T - np.eye(npts))))
        e2 = float(np.max(np.abs(R.T @ R - I)) / np.max(np.abs(I)))
        v = rng.standard_normal(npts)
        q_dev = float(np.sum((R @ v) ** 2))
        q_ref = float(v @ np.linalg.solve(W, v))
        out.append(dict(alpha=a, det_dev=float(det[g]), det_ref=float(det_ref), RWRt_minus_I=e1, RtR_vs_iW=e2,
                        quad_dev=q_dev, quad_ref=q_ref, cond=float(np.linalg.cond(W)) if npts <= 3000 else None))
    return dict(np=npts, t_device_s=round(t_dev, 2), grid=out)


def alpha_trace(ny, method, sweeps):
    from hmsc_amd.workloads import spatial_vignette4
    hM = spatial_vignette4(ny=ny, method=method)
    ch = H.Chain(hM, 4242, device=0, updater={"GammaEta": False})
    ch.init([1])
    rec = ch.run(transient=0, samples=sweeps, thin=1, adaptNf=[0])
    ch.close()
    a = rec["Alpha0"][:, 0]
    vals = np.asarray(hM.rL[0].alphapw)[a - 1, 0]
    lam = rec["Lambda0"][:, 0, :]
    return dict(method=method, alpha_index_first20=a[:20].tolist(), alpha_index_last20=a[-20:].tolist(),
                alpha_value_mean_last_half=float(vals[sweeps // 2:].mean()),
                frac_index1=float(np.mean(a == 1)), lambda_mean_last_half=lam[sweeps // 2:].mean(0).tolist())


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--np", type=int, default=2500)
    p.add_argument("--ny", type=int, default=5000)
    p.add_argument("--sweeps", type=int, default=300)
    a = p.parse_args()
    res = dict(grid=grid_check(a.np, [0.05, 0.35, 1.0, 1.41]))
    print(json.dumps(res), flush=True)
    res["traces"] = [alpha_trace(a.ny, m, a.sweeps) for m in ("GPP", "Full")]
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
