"""Config-5 long chains on the GPU box (vignette_4 at ny = 5000): 'Full' from the default
initial state (Alpha = 1), 'GPP' (25 knots) from the same, and 'Full' started from the GPP
chain's final state; alpha index trajectories (recorded path).  One JSON line."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import hmsc_amd as H  # noqa: E402
from hmsc_amd.workloads import spatial_vignette4  # noqa: E402


def chain(method, ny, n, state=None, seed=4242):
    hM = spatial_vignette4(ny=ny, method=method)
    ch = H.Chain(hM, seed, device=0, updater={"GammaEta": False})
    ch.init([1])
    if state is not None:
        ch.set_state(state)
    rec = ch.run(transient=0, samples=n, thin=1, adaptNf=[0], iter0=0, record=True)
    st = ch.get_state()
    ch.close()
    a = rec["Alpha0"][:, 0].astype(int)
    return hM, a, st


def summary(hM, a):
    grid = np.asarray(hM.rL[0].alphapw)[:, 0]
    h = a[len(a) // 2:]
    return dict(first=a[:30].tolist(), last=a[-30:].tolist(), max=int(a.max()), frac1=float(np.mean(a == 1)),
                mean_index_2nd_half=float(h.mean()), mean_alpha_2nd_half=float(grid[h - 1].mean()))


def main():
    ny = int(sys.argv[1]) if len(sys.argv) > 1 else 5000
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 400
    out = {"ny": ny, "sweeps": n}
    hM, a, _ = chain("Full", ny, n)
    out["full_from_init"] = summary(hM, a)
    print(json.dumps(out), flush=True)
    hM, a, st = chain("GPP", ny, n)
    out["gpp_from_init"] = summary(hM, a)
    print(json.dumps(out), flush=True)
    keep = {k: st[k] for k in ("Beta", "Gamma", "iV", "iSigma", "Eta", "Lambda", "Psi", "Delta", "Alpha", "Z")}
    hM, a, _ = chain("Full", ny, n, state=keep)
    out["full_from_gpp_state"] = summary(hM, a)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
