"""TD$m's default updater set on the CPU oracle, long runs (tests/golden/td_longrun.npz,
generator tests/golden/make_td_longrun_fixture.py), CPU only.

1. GammaEta on and off are two samplers of one posterior (R/updateGammaEta.R:7-206 draws
   Gamma and Eta with Beta integrated out; without it Gamma comes from updateGammaV alone):
   their long-run means agree within Monte Carlo error on Beta, Gamma, V, rho, Omega of both
   levels and the spatial scales.  The standard errors are between-chain (8 independent
   chains per side), so they do not rest on an ESS estimate of sticky chains.
2. The reference's stored TD$m$postList (2 chains x 100 samples after a 50-sweep transient,
   data-raw/simulateTestData.R:70) is a typical outcome of that same short protocol: against
   the distribution of 2-chain means of 64 oracle protocol replicates its Beta / Gamma / rho
   means are within 3 sd each, chi-square within its degrees of freedom.
3. ... and that protocol does not reach the posterior: its replicated mean sits many Monte
   Carlo standard errors from the long-run mean on several Beta / Gamma entries -- which is
   why the reference's stored means differ from a long run (VERDICT r01 "What's weak" #1).
"""
import os

import numpy as np
import pytest

from td_longrun_common import between_chain_t, reference_rows
from test_golden_td import td_model, td_postlist

HERE = os.path.dirname(os.path.abspath(__file__))
F = os.path.join(HERE, "golden", "td_longrun.npz")
pytestmark = pytest.mark.skipif(not os.path.exists(F), reason="td_longrun.npz not generated")


def _load():
    return np.load(F)


def test_gamma_eta_on_off_same_posterior():
    D = _load()
    t = between_chain_t(D["on/mean"], D["off/mean"])
    names = list(D["names"])
    worst = int(np.argmax(np.abs(t)))
    # 50 statistics, Welch t on 8 + 8 chains: |t| < 4 for all of them at family level ~1 %
    assert np.max(np.abs(t)) < 4.0, (names[worst], t[worst])
    assert np.mean(np.abs(t) > 2.0) < 0.2


def _ref_means(hM):
    rows = reference_rows(hM, td_postlist(hM))
    return np.mean([r.mean(0) for r in rows], axis=0)


def test_reference_posterior_is_a_short_protocol_outcome():
    D = _load()
    hM = td_model()
    names = list(D["names"])
    sel = [i for i, n in enumerate(names) if n.startswith(("Beta", "Gamma", "rho"))]
    sh = D["short/means"]
    pairs = 0.5 * (sh[0::2] + sh[1::2])          # the reference ran 2 chains
    ref = _ref_means(hM)
    z = (ref - pairs.mean(0)) / pairs.std(0, ddof=1)
    assert np.max(np.abs(z[sel])) < 3.0, [(names[i], z[i]) for i in sel]
    chi2 = float(np.sum(z[sel] ** 2))
    assert chi2 < 2.0 * len(sel), chi2             # ~8 observed on 22 statistics


def test_short_protocol_does_not_reach_the_posterior():
    D = _load()
    names = list(D["names"])
    sh = D["short/means"]
    on = D["on/mean"]
    t = between_chain_t(sh, on)
    beta_gamma = [i for i, n in enumerate(names) if n.startswith(("Beta", "Gamma"))]
    assert np.sum(np.abs(t[beta_gamma]) > 5.0) >= 3, t[beta_gamma]
