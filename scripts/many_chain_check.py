"""Chain-mean spread of one parameter over many GPU chains (diagnostic for slow modes)."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import hmsc_amd as H
from helpers import synthetic_model
from posterior_common import MODELS, param_vector, TRANSIENT, SAMPLES
hM = synthetic_model(**MODELS["probit_traits"])
res = []
for c in range(24):
    ch = H.Chain(hM, 100 + c, device=0, updater={"GammaEta": False})
    ch.init()
    rec = ch.run(transient=TRANSIENT, samples=SAMPLES, thin=1, adaptNf=[0])
    ch.close()
    v = param_vector(dict(Beta=rec["Beta"], Gamma=rec["Gamma"], Lambda0=rec["Lambda0"][:, :2, :]))
    res.append(v.mean(axis=0))
np.save(os.path.join(ROOT, "gpurun_out", "many_gpu_means.npy"), np.stack(res))
print("ok")
