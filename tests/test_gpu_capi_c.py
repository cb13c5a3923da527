"""The R .Call shim of INTEGRATION.md, as plain C compiled with gcc against
include/hmsc_amd.h (tests/capi/shim_run.c, built by hmsc_amd.build), run on the GPU for the
TD spec (phylogeny + spatial 'Full' plot level + sample level, the reference's default
updaters): it fills hmsc_model from R's hM fields -- rhopw, eigen(C), alphapw and the
unit-ordered coordinates included -- and runs hmsc_create / hmsc_init_state / hmsc_run.
Its recorded chain must equal, bit for bit, the same chain run through this repository's
own binding (hmsc_amd/_lib.py): the two marshal the same model the same way."""
import os
import subprocess
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "capi"))
from model_io import read_results, write_model  # noqa: E402

import hmsc_amd as H  # noqa: E402
from hmsc_amd.sampler import updater_mask  # noqa: E402
from test_golden_td import td_model  # noqa: E402

pytestmark = pytest.mark.gpu
SHIM = os.path.join(HERE, "capi", "shim_run")


def test_c_shim_td_matches_python_binding(tmp_path):
    assert os.path.exists(SHIM), "tests/capi/shim_run not built (python -m hmsc_amd.build)"
    hM = td_model()
    model = str(tmp_path / "td_model.bin")
    out = str(tmp_path / "td_out.bin")
    write_model(hM, model)
    seed, transient, S = 4242, 20, 30
    mask = updater_mask(None)
    p = subprocess.run([SHIM, model, out, str(seed), str(mask), str(transient), str(S)], capture_output=True,
                       text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    res = read_results(out)
    ch = H.Chain(hM, seed, device=0, mask=mask)
    ch.init([int(rl.nfMin) for rl in hM.rL])
    rec = ch.run(transient=transient, samples=S, thin=1, adaptNf=[0] * hM.nr)
    ch.close()
    nc, ns, nt = hM.nc, hM.ns, hM.nt
    np.testing.assert_array_equal(res["Beta"].reshape(S, ns, nc).transpose(0, 2, 1), rec["Beta"])
    np.testing.assert_array_equal(res["Gamma"].reshape(S, nt, nc).transpose(0, 2, 1), rec["Gamma"])
    np.testing.assert_array_equal(res["iV"].reshape(S, nc, nc).transpose(0, 2, 1), rec["iV"])
    np.testing.assert_array_equal(res["rho"], rec["rho"])
    for r in range(hM.nr):
        nfm = int(hM.rL[r].nfMax)
        np.testing.assert_array_equal(res[f"Lambda{r}"].reshape(S, ns, nfm).transpose(0, 2, 1), rec[f"Lambda{r}"])
        np.testing.assert_array_equal(res[f"Eta{r}"].reshape(S, nfm, int(hM.np[r])).transpose(0, 2, 1),
                                      rec[f"Eta{r}"])
        np.testing.assert_array_equal(res[f"Alpha{r}"].reshape(S, nfm), rec[f"Alpha{r}"])
    # the chain moved (rho and the spatial scale are drawn, Beta varies)
    assert np.unique(res["rho"]).size > 1 and np.std(rec["Beta"][:, 0, 0]) > 0
