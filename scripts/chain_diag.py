"""Per-chain diagnostics for the probit_traits posterior model (GPU side)."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import hmsc_amd as H
from helpers import synthetic_model
from posterior_common import MODELS, param_vector, TRANSIENT, SAMPLES
name = sys.argv[1] if len(sys.argv) > 1 else "probit_traits"
hM = synthetic_model(**MODELS[name])
out = {}
for c in range(8):
    ch = H.Chain(hM, 1 + c, device=0, updater={"GammaEta": False})
    ch.init()
    rec = ch.run(transient=0, samples=TRANSIENT + SAMPLES, thin=1, adaptNf=[0])
    ch.close()
    v = param_vector(dict(Beta=rec["Beta"], Gamma=rec["Gamma"], Lambda0=rec["Lambda0"][:, :2, :]))
    out[f"v{c}"] = v.astype(np.float32)
    out[f"delta{c}"] = rec["Delta0"]
    out[f"isig{c}"] = rec["iSigma"]
np.savez(os.path.join(ROOT, "gpurun_out", f"chain_diag_{name}.npz"), **out)
print("ok")
