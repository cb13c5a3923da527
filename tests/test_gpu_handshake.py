"""Every bounded in-launch spin reports instead of continuing silently.

The sync-free triangular solve (dense.hip trsv_sf_kernel) and the blocked Cholesky's fused
panel step (chol_update_kernel) wait on flags raised by other workgroups of the same launch.
A wait that outlasts its time bound raises a bit in the chain's handshake error word; the host
turns it into a distinct error (-5, "... handshake timed out ...") at the next hmsc_run /
hmsc_sync / hmsc_get_state, never a "not positive definite" and never silent samples.  The
tests corrupt one handshake through the C ABI (hmsc_debug_poison) before a phylogeny
BetaLambda update on the blocked path ((nc + nf) ns > 1024), which runs both waits.

The second half runs the dense / phylogeny parity with each of the fallback switches
(HMSC_NO_CHOL_PANEL_FUSION, HMSC_NO_CHOL_DIAG_FUSION, HMSC_NO_TRSV_SF; read once per process)
in a fresh child process, so the non-default launch sequences stay covered."""
import os
import subprocess
import sys

import numpy as np
import pytest

from helpers import H, ROOT, phylo_corr, synthetic_model
from hmsc_amd._lib import HmscNativeError

pytestmark = pytest.mark.gpu


def _blocked_phylo_chain():
    hM = synthetic_model(ny=120, ns=300, nc=3, nf=2, seed=71, C=phylo_corr(300, seed=71))
    ch = H.Chain(hM, 9, device=0, updater={"GammaEta": False})
    ch.init()
    return ch


@pytest.mark.parametrize("what", ["trsv_ticket", "chol_publish"])
def test_poisoned_handshake_is_reported(what):
    ch = _blocked_phylo_chain()
    ch.update("BetaLambda", 1)
    ch.sync()                                    # clean: no flag raised
    ch.debug_poison(what)
    ch.update("BetaLambda", 2)
    with pytest.raises(HmscNativeError, match=r"handshake.*timed out") as ei:
        ch.sync()
    assert "error -5" in str(ei.value)
    assert "not positive definite" not in str(ei.value)
    # reported once: the error words are cleared, so the state can be read to diagnose it
    st = ch.get_state(with_z=False)
    assert np.all(np.isfinite(st["Gamma"]))
    ch.close()


def test_poisoned_handshake_fails_the_run():
    ch = _blocked_phylo_chain()
    ch.debug_poison("trsv_ticket")
    with pytest.raises(HmscNativeError, match=r"handshake.*timed out"):
        ch.run(transient=1, samples=1, thin=1)
    ch.close()


_CHILD = r"""
import sys
sys.path.insert(0, {root!r}); sys.path.insert(0, {tests!r})
import numpy as np
from helpers import H, O, oracle_model, phylo_corr, rel_err, synthetic_model
from oracle.rng import Rng
from hmsc_amd import _lib
# the blocked Cholesky and both solves on one host system
rng = np.random.default_rng(3)
n = 700
A0 = rng.standard_normal((n, n)); A0 = A0 @ A0.T / n + np.eye(n)
b0 = rng.standard_normal(n)
A = np.asfortranarray(A0.copy()); b = b0.copy(); info = np.zeros(1, dtype=np.int32)
L = _lib.lib()
_lib.check(L.hmsc_dense_chol_solve(0, _lib.fptr(A), n, _lib.fptr(b), _lib.iptr(info)))
assert info[0] == 0
assert rel_err(b, np.linalg.solve(A0, b0)) < 1e-10, rel_err(b, np.linalg.solve(A0, b0))
# the phylogeny BetaLambda system on the blocked path, moments against the oracle
hM = synthetic_model(ny=120, ns=300, nc=3, nf=2, seed=72, C=phylo_corr(300, seed=72))
m = oracle_model(hM); dp = O.compute_data_parameters(m)
up = {{"GammaEta": False}}
r = Rng(5); st = O.compute_initial_parameters(m, r); st = O.sweep(st, m, r, 1, updater=up, data_par=dp)
ch = H.Chain(hM, 5, device=0, updater=up); ch.init(); ch.set_state(st); ch.set_noise_mode(1)
ch.update("BetaLambda", 2)
g = ch.get_state(with_z=False)
BL = O._beta_lambda_phylo(st, m, Rng(5), 2, dp, zero_noise=True)
e = rel_err(g["Beta"], BL[:hM.nc])
assert e < 1e-10, e
ch.close()
print("child ok")
"""


@pytest.mark.parametrize("switch", ["HMSC_NO_CHOL_PANEL_FUSION", "HMSC_NO_CHOL_DIAG_FUSION", "HMSC_NO_TRSV_SF"])
def test_dense_fallback_paths_in_fresh_process(switch):
    env = dict(os.environ)
    env[switch] = "1"
    code = _CHILD.format(root=ROOT, tests=os.path.join(ROOT, "tests"))
    p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0 and "child ok" in p.stdout, (p.stdout[-2000:], p.stderr[-2000:])
