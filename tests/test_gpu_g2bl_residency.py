"""The fused Gamma2 + BetaLambda launch at species counts whose grid does not fit the device's
resident workgroup slots.  Workgroup 0 waits for Gamma2's species-block
partials and every BetaLambda workgroup waits for workgroup 0, so the partials on trailing
workgroups are only safe when the whole grid is resident; above that the launch puts the
partials ahead of the first BetaLambda bodies (dispatched before any waiter), and when even
those do not fit beside workgroup 0 the sweep takes the unfused Gamma2 and BetaLambda
launches.  ns = 2400 (1 + 600 + 300 workgroups against 2 x 256 slots: partials ahead) and
4800 (600 partial workgroups: unfused) run three sweeps eagerly and then graph replays, and
follow the oracle (R/updateGamma2.R, R/updateBetaLambda.R)."""
import numpy as np
import pytest

from helpers import O, oracle_model, rel_err, synthetic_model
from hmsc_amd.sampler import Chain
from oracle.rng import Rng

pytestmark = pytest.mark.gpu
UP = {"GammaEta": False}


@pytest.mark.parametrize("ns", [2400, 4800])
def test_fused_launch_beyond_resident_slots(ns):
    hM = synthetic_model(ny=160, ns=ns, nc=4, nf=3, seed=11)
    m = oracle_model(hM)
    seed = 777
    ch = Chain(hM, seed, device=0, updater=UP)
    ch.init()
    rng = Rng(seed)
    o = O.compute_initial_parameters(m, rng)
    for it in range(1, 4):
        ch.sweep(it)
        o = O.sweep(o, m, rng, it, updater=UP)
    lay = ch.debug_get("g2bl", 2)
    if ns == 2400:
        assert lay[1] > 0, "the fused Gamma2 + BetaLambda launch did not run"
        assert lay[0] == 0, "a grid beyond the resident slots must not use trailing partial workgroups"
    else:
        assert lay[1] == 0, "600 partial workgroups cannot be resident beside workgroup 0: unfused path"
    g = ch.get_state()
    for k in ("Beta", "Gamma", "iV", "Z"):
        assert rel_err(g[k], o[k]) < 1e-7, (k, rel_err(g[k], o[k]))
    # recorded graph replays of the same launch: finite, and the chain keeps running
    rec = ch.run(transient=0, samples=40, thin=1, iter0=4)
    assert np.all(np.isfinite(rec["Beta"])) and rec["Beta"].shape == (40, hM.nc, ns)
    ch.close()


def test_config4_keeps_trailing_partials():
    """At config 4's 1,000 species (1 + 250 + 125 workgroups) the trailing layout stays on."""
    from hmsc_amd.workloads import synthetic_probit
    hM = synthetic_probit(ny=2000)
    ch = Chain(hM, 5, device=0, updater=UP)
    ch.init()
    ch.sweep(1)
    lay = ch.debug_get("g2bl", 2)
    ch.close()
    assert lay[0] == 1 and lay[1] == 376, lay
