"""The species-sharded chain from two processes on one GPU: torch.distributed
.run starts two ranks (tests/mgpu_worker.py --mode sharded --transport host --same-device),
each a hmsc_create_sharded_host state whose all-reduce callback sums over gloo.  Every rank
runs eager sweeps and then a recorded hmsc_run through the sweep graphs (segments split at the
all-reduces); the ranks' blocks must follow the unsharded chain of the same key, computed in
this process, to reduction-order rounding, and their redundant draws must agree bit for bit."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from helpers import H, rel_err, synthetic_model

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)
from mgpu_worker import MODELS  # noqa: E402


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("model", ["mid", "na"])
def test_two_processes_gloo_one_gpu(tmp_path, model):
    sweeps, run = 3, 8
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(HERE, "mgpu_worker.py"),
           "--mode", "sharded", "--transport", "host", "--same-device", "--model", model,
           "--sweeps", str(sweeps), "--recorded", str(run), "--out", str(tmp_path)]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="2")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=420)
    assert r.returncode == 0, r.stderr[-4000:]
    hM = synthetic_model(**MODELS[model])
    full = H.Chain(hM, 97531, device=0, updater={"GammaEta": False})
    full.init()
    for it in range(1, sweeps + 1):
        full.sweep(it)
    rec = full.run(transient=0, samples=run, thin=1, adaptNf=[0], iter0=sweeps, record=True)
    g = full.get_state()
    full.close()
    parts = [np.load(tmp_path / f"rank{k}.npz") for k in range(2)]
    covered = 0
    for k, p in enumerate(parts):
        a, n = int(p["sp0"]), int(p["nsl"])
        covered += n
        assert int(p["device"]) == 0
        assert rel_err(p["Beta"], g["Beta"][:, a:a + n]) < 1e-8, (k, "Beta")
        assert rel_err(p["Lambda"], g["Lambda"][0][:, a:a + n]) < 1e-8, (k, "Lambda")
        assert rel_err(p["Z"], g["Z"][:, a:a + n]) < 1e-8, (k, "Z")
        assert rel_err(p["rec_beta"], rec["Beta"][:, :, a:a + n]) < 1e-8, (k, "recorded Beta")
        for key in ("Gamma", "iV", "Eta", "Delta"):
            ref = g[key] if key in ("Gamma", "iV") else g[key][0]
            assert rel_err(p[key], ref) < 1e-8, (k, key)
            np.testing.assert_array_equal(p[key], parts[0][key])   # the redundant draws agree
        assert p["graph"][0] == 1, "the sweep graphs were not built"
        assert p["ar_calls"][2] == 2, p["ar_calls"]                # two all-reduces per sweep
        # every all-reduce went through the gloo callback: init + 3 eager sweeps + the run
        assert int(p["callbacks"]) == int(p["ar_calls"][0])
    assert covered == hM.ns
