"""Config-5 chain diagnostics on the GPU box: a 'Full' spatial_vignette4 chain at several ny,
(a) eager sweeps with get_state after each (device state), (b) a recorded hmsc_run of the same
chain (record path), printing alpha indices, |Eta| and Lambda.  One JSON line per ny."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import hmsc_amd as H  # noqa: E402
from hmsc_amd.workloads import spatial_vignette4  # noqa: E402


def main():
    sizes = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "1000,1100,2100,5000").split(",")]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    for ny in sizes:
        hM = spatial_vignette4(ny=ny, method="Full")
        ch = H.Chain(hM, 4242, device=0, updater={"GammaEta": False})
        ch.init([1])
        tr = []
        for it in range(1, n + 1):
            ch.sweep(it)
            g = ch.get_state(with_z=False)
            tr.append((int(g["Alpha"][0][0]), float(np.linalg.norm(g["Eta"][0])), g["Lambda"][0][0].round(3).tolist()))
        rec = ch.run(transient=0, samples=n, thin=1, adaptNf=[0], iter0=n)
        ch.close()
        out = dict(ny=ny, eager_alpha=[t[0] for t in tr], eager_eta_norm=[round(t[1], 2) for t in tr[::5]],
                   eager_lambda_last=tr[-1][2], rec_alpha=rec["Alpha0"][:, 0].tolist(),
                   rec_eta_norm=[round(float(np.linalg.norm(e)), 2) for e in rec["Eta0"][::5]])
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
