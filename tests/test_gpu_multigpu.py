"""The multi-GPU paths on real devices, when at least 2 GPUs are visible;
skipped on a one-GPU box (tests/test_gpu_sharded.py runs the same sharded chain there with a
host transport, tests/test_distributed_gloo.py the decomposition on CPU).

  * species-sharded chain: 2 ranks (torch.distributed.run, one process per GPU) through
    hmsc_create_sharded with an RCCL communicator; the all-reduced chain must follow the
    unsharded chain of the same key to 1e-8 (reduction order only);
  * independent chains: rank r's chain equals, bit for bit, the same key run on device 0 by
    this process (the Philox stream does not depend on the device);
  * bench.py --gpus 2 in both modes prints one JSON line with n_gpus = 2.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from hmsc_amd import _lib as L
from helpers import H, rel_err, synthetic_model

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _ndev():
    n = np.zeros(1, dtype=np.int32)
    try:
        L.check(L.lib().hmsc_device_count(L.iptr(n)))
    except L.HmscNativeError:   # no device at all (the CPU container): the tests skip
        return 0
    return int(n[0])


needs2 = pytest.mark.skipif(_ndev() < 2, reason="needs >= 2 GPUs (the driver's multi-GPU node)")


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _torchrun(args, timeout=300):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port())] + args
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-4000:]
    return r.stdout


def _reference(seed, sweeps=5):
    hM = synthetic_model(ny=300, ns=41, nc=4, nf=3, seed=61)
    ch = H.Chain(hM, seed, device=0, updater={"GammaEta": False})
    ch.init()
    for it in range(1, sweeps + 1):
        ch.sweep(it)
    g = ch.get_state()
    ch.close()
    return g


@needs2
def test_sharded_chain_rccl(tmp_path):
    _torchrun([os.path.join(HERE, "mgpu_worker.py"), "--mode", "sharded", "--out", str(tmp_path)])
    full = _reference(97531)
    covered = 0
    for r in range(2):
        p = np.load(tmp_path / f"rank{r}.npz")
        assert int(p["device"]) == r
        a, n = int(p["sp0"]), int(p["nsl"])
        covered += n
        assert rel_err(p["Beta"], full["Beta"][:, a:a + n]) < 1e-8, r
        assert rel_err(p["Lambda"], full["Lambda"][0][:, a:a + n]) < 1e-8, r
        assert rel_err(p["Z"], full["Z"][:, a:a + n]) < 1e-8, r
        for k in ("Gamma", "iV"):
            assert rel_err(p[k], full[k]) < 1e-8, (r, k)
    assert covered == 41


@needs2
def test_independent_chains_one_per_gpu(tmp_path):
    _torchrun([os.path.join(HERE, "mgpu_worker.py"), "--mode", "chains", "--out", str(tmp_path)])
    for r in range(2):
        p = np.load(tmp_path / f"rank{r}.npz")
        ref = _reference(97531 + 7919 * r)
        for k in ("Beta", "Gamma", "iV", "Z"):
            np.testing.assert_array_equal(p[k], ref[k], err_msg=f"rank {r} {k}")


@needs2
@pytest.mark.parametrize("mode", ["chains", "sharded"])
def test_bench_two_gpus(mode):
    out = _torchrun([os.path.join(ROOT, "bench.py"), "--gpus", "2", "--mode", mode, "--steps", "20",
                     "--warmup", "5", "--ess-samples", "1000", "--no-cpu"], timeout=600)
    line = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(line) == 1, out
    res = json.loads(line[0])
    assert res["n_gpus"] == 2 and res["value"] > 0
    assert res["scaling"] == ("weak" if mode == "chains" else "strong")
