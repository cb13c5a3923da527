"""Dump the GPU chain state after every sweep (for trajectory comparison with the oracle)."""
import os, sys, pickle
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import hmsc_amd as H
from helpers import synthetic_model
from posterior_common import MODELS
name, seed, n = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
hM = synthetic_model(**MODELS[name])
ch = H.Chain(hM, seed, device=0, updater={"GammaEta": False})
ch.init()
states = [ch.get_state()]
for it in range(1, n + 1):
    ch.sweep(it)
    states.append(ch.get_state())
ch.close()
np.save(os.path.join(ROOT, "gpurun_out", f"traj_{name}_{seed}.npy"), np.array(states, dtype=object), allow_pickle=True)
print("ok")
