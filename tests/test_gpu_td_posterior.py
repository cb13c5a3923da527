"""TD$m's exact spec on the device against the reference's own posterior (SURVEY.md §8 (d)
config 1): two random levels (sample, spatial 'Full' plot level), phylogeny C, traits, and
the reference's default updater set -- so updateGammaEta's spatial branch with phylogeny,
updateRho and updateAlpha all run.  The golden side is TD$m$postList as the reference
stored it (2 chains x 100 samples, tests/golden/td.npz).  Posterior means of Beta, Gamma
and rho are compared under the reference's own (short, unconverged) run protocol; a second
test checks that GammaEta on / off sample one posterior (long runs, AR(1) effective sizes)."""
import numpy as np
import pytest

import hmsc_amd as H
from test_golden_td import td_model, td_postlist

pytestmark = pytest.mark.gpu


def _summ(chains, key):
    """Pooled mean and its standard error with an AR(1) effective size per chain,
    n (1 - rho1) / (1 + rho1): the reference's chains are short and sticky (lag-1
    autocorrelation up to 0.9 on Beta, 100 samples each)."""
    arrs = [np.stack([np.asarray(s[key], dtype=np.float64).ravel() for s in ch]) for ch in chains]
    a = np.concatenate(arrs)
    ess = 0.0
    for x in arrs:
        xc = x - x.mean(0)
        v = np.maximum((xc ** 2).mean(0), 1e-300)
        r1 = np.clip((xc[1:] * xc[:-1]).mean(0) / v, -0.5, 0.99)
        ess = ess + x.shape[0] * (1 - r1) / (1 + r1)
    return a.mean(0), a.std(0, ddof=1) / np.sqrt(ess)


def test_td_reference_protocol_covers_reference_posterior():
    """TD$m was fitted with transient=50, samples=100, thin=1, nChains=2
    (data-raw/simulateTestData.R:70): too short to converge (its two chains' Beta means differ
    by up to 1.2 posterior sd), so its pooled mean is compared with the sampling distribution
    of the same protocol on the device: 32 chains run exactly so, and the reference's
    2-chain mean must lie within 4 sd of the distribution of 2-chain means."""
    ref = td_model()
    ref.postList = td_postlist(ref)
    hM = H.sampleMcmc(td_model(), samples=100, transient=50, thin=1, nChains=32, seed=31, verbose=0)
    for key in ("Beta", "Gamma", "rho"):
        cm = np.stack([np.mean([np.asarray(s[key], dtype=np.float64).ravel() for s in ch], axis=0)
                       for ch in hM.postList])                           # per-chain means
        rm = np.mean([np.asarray(s[key], dtype=np.float64).ravel() for ch in ref.postList for s in ch], axis=0)
        z = (rm - cm.mean(0)) / (cm.std(0, ddof=1) / np.sqrt(2) + 1e-12)
        print(key, "ref", np.round(rm, 3), "device", np.round(cm.mean(0), 3), "z", np.round(z, 2))
        assert np.all(np.isfinite(cm)) and np.max(np.abs(z)) < 4.0, (key, z)
    a = np.stack([s["Alpha"][1] for ch in hM.postList for s in ch])
    assert np.all(a >= 1) and np.all(a <= hM.rL[1].alphapw.shape[0])


def test_td_gamma_eta_on_off_agree():
    """The same posterior with and without the joint updateGammaEta step (both are valid
    Gibbs samplers of one posterior): Beta / Gamma means within Monte Carlo error."""
    on = H.sampleMcmc(td_model(), samples=500, transient=500, thin=2, nChains=4, seed=41, verbose=0)
    off = H.sampleMcmc(td_model(), samples=500, transient=500, thin=2, nChains=4, seed=42, verbose=0,
                       updater={"GammaEta": False})
    for key in ("Beta", "Gamma"):
        m1, s1 = _summ(on.postList, key)
        m2, s2 = _summ(off.postList, key)
        z = (m1 - m2) / np.sqrt(s1 ** 2 + s2 ** 2)
        print(key, "on", np.round(m1, 3), "off", np.round(m2, 3), "z", np.round(z, 2))
        assert np.max(np.abs(z)) < 4.0, (key, z)
