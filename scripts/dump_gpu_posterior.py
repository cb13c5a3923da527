"""Dump the GPU side of tests/test_gpu_posterior.py (summaries per model) to gpurun_out/."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from helpers import synthetic_model  # noqa: E402
from posterior_common import MODELS, summarise, unpack_state  # noqa: E402
import test_gpu_posterior as T  # noqa: E402

out = {}
for name in MODELS:
    hM = synthetic_model(**MODELS[name])
    for k, v in summarise(hM, T.gpu_chains(hM, unpack_state(T.FIX, f"{name}/start", hM.nr))).items():
        out[f"{name}/{k}"] = v
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez(os.path.join(ROOT, "gpurun_out", "gpu_posterior.npz"), **out)
print("ok")
