"""Run-to-run reproducibility (SURVEY.md §2.3 "Reproducibility invariant"): every draw is a
function of (seed, chain, sweep, element) through the Philox counters, and every reduction on
the device is a fixed-order slab or tree sum (no floating-point atomics: the only device
atomics are the Cholesky failure flag and the integer launch-timer min / max).  So the same
call twice gives the same bits, whether the chains run one after another or concurrently on
one device (nParallel), and conditional prediction (predict(Yc=...), R/predict.R:181-198)
repeats exactly."""
import numpy as np
import pytest

from helpers import H, synthetic_model

pytestmark = pytest.mark.gpu


def _model():
    return synthetic_model(ny=90, ns=9, nc=3, nf=2, nr=2, units=[90, 15], n_normal=2, n_poisson=3, seed=61,
                           yscale=True)


def _fit(nParallel):
    return H.sampleMcmc(_model(), samples=12, transient=20, thin=2, nChains=2, nParallel=nParallel,
                        updater={"GammaEta": False}, seed=5, verbose=0)


def _same_post(a, b):
    for ca, cb in zip(a.postList, b.postList):
        for sa, sb in zip(ca, cb):
            for k in ("Beta", "Gamma", "V", "sigma"):
                np.testing.assert_array_equal(sa[k], sb[k], err_msg=k)
            for r in range(len(sa["Eta"])):
                np.testing.assert_array_equal(sa["Eta"][r], sb["Eta"][r])
                np.testing.assert_array_equal(sa["Lambda"][r], sb["Lambda"][r])


@pytest.fixture(scope="module")
def fits():
    return _fit(2), _fit(2), _fit(1)


def test_sample_mcmc_bitwise_repeatable(fits):
    a, b, _ = fits
    _same_post(a, b)


def test_chains_independent_of_nparallel(fits):
    a, _, c = fits     # concurrent chains (two host threads, one device) vs one after another
    _same_post(a, c)


def test_conditional_prediction_repeatable(fits):
    hM = fits[0]
    post = H.poolMcmcChains(hM.postList)[:6]
    probit = np.nonzero(hM.distr[:, 0] == 2)[0]
    Yc = np.full((hM.ny, hM.ns), np.nan)
    Yc[:, probit] = hM.Y[:, probit]
    p1 = np.stack(H.predict(hM, post=post, Yc=Yc, mcmcStep=3, expected=True, seed=11), axis=2)
    p2 = np.stack(H.predict(hM, post=post, Yc=Yc, mcmcStep=3, expected=True, seed=11), axis=2)
    np.testing.assert_array_equal(p1, p2)


def test_two_chains_one_device_fused_path_with_graphs():
    """with nParallel = 2 on one device the two chains' streams may share hardware
    queues, so the device-side joins of edge-free sweep graphs could wait on each other in a
    cycle.  A second live chain on the device makes every chain capture with graph edges
    (capi.cpp live_chains): at a size where the fused BetaLambda launch fills the CUs (ns =
    1000: 251 workgroups) and long enough for graph replays, both chains finish, and each equals
    the same chain run alone."""
    from hmsc_amd.workloads import synthetic_probit
    hM = synthetic_probit(ny=2000, ns=1000, nc=6, nf=4)
    fit2 = H.sampleMcmc(hM, samples=60, transient=10, thin=1, nChains=2, nParallel=2,
                        updater={"GammaEta": False}, seed=9, verbose=0, alignPost=False)
    hM1 = synthetic_probit(ny=2000, ns=1000, nc=6, nf=4)
    fit1 = H.sampleMcmc(hM1, samples=60, transient=10, thin=1, nChains=2, nParallel=1,
                        updater={"GammaEta": False}, seed=9, verbose=0, alignPost=False)
    _same_post(fit2, fit1)


@pytest.mark.parametrize("env", ["HMSC_XZ_FOLD", "HMSC_NO_TAIL_DEFER", "HMSC_NO_SIDE_GATE", "HMSC_G2_PART_INLINE",
                                 "HMSC_NO_PSI_PRE", "HMSC_NO_BL_PREDRAW", "HMSC_TAIL_DEFER_LEVELS"])
def test_launch_variants_bitwise(env, monkeypatch):
    """Launch-structure variants give the same bits: XZ read from updateZ's chunk partials by the
    fused Gamma2 + BetaLambda launch (HMSC_XZ_FOLD, with the record pack in the z launch) or
    reduced first (default), Gamma2's species-block partials on workgroups of their own (default)
    or ahead of the first BetaLambda bodies (HMSC_G2_PART_INLINE), the BetaLambda tail's two
    reduction levels deferred to the Eta launch (default), only the last (HMSC_TAIL_DEFER_LEVELS=1)
    or neither, the next sweep's BetaLambda draws made by the Eta launch (default) or in the
    BetaLambda prologue (HMSC_NO_BL_PREDRAW), and the previous sweep's side chain awaited
    by the reduction launch after updateZ (default) or polled by the fused launch itself
    (HMSC_NO_SIDE_GATE), and the BetaLambda tail's psi gamma variates drawn ahead by the bodies
    (default) or in the tail (HMSC_NO_PSI_PRE).  A probit-only model (the fused paths), recorded
    graph sweeps."""
    def fit():
        hM = synthetic_model(ny=300, ns=60, nc=4, nf=3, seed=17)
        return H.sampleMcmc(hM, samples=30, transient=40, thin=1, nChains=1, updater={"GammaEta": False},
                            seed=9, verbose=0)
    base = fit()
    monkeypatch.setenv(env, "1")
    _same_post(base, fit())
