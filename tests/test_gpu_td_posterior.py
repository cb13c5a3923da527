"""TD$m's exact spec on the device: two random levels (sample,
spatial 'Full' plot level), phylogeny C, traits, and the reference's default updater set --
so updateGammaEta's spatial branch with phylogeny, updateRho and updateAlpha all run.

1. Long runs against the CPU oracle's long runs (tests/golden/td_longrun.npz): 8 device
   chains per updater set (GammaEta on = the reference default, and off), their chain means
   of Beta, Gamma, V, rho, Omega (both levels) and the spatial scales against the oracle's 8
   chains, Welch t on between-chain standard errors (no ESS estimate involved).
2. The reference's own stored posterior (TD$m$postList: 2 chains x 100 samples after a
   50-sweep transient, data-raw/simulateTestData.R:70) against the device run under that
   same protocol (64 chains): the reference is a typical 2-chain outcome of it.
   tests/test_golden_td_longrun.py shows with the oracle that this protocol has not
   converged (its replicated means sit many standard errors from the long-run means), which
   is why the reference's stored means differ from a long run.
"""
import os
import threading

import numpy as np
import pytest

import hmsc_amd as H
from td_longrun_common import between_chain_t, param_rows, reference_rows
from test_golden_td import td_model, td_postlist

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
FIX = os.path.join(HERE, "golden", "td_longrun.npz")

DEV_TRANSIENT, DEV_SAMPLES, DEV_CHAINS = 500, 8000, 8


def _device_chain_rows(hM, seeds, updater, transient, samples, batch=8):
    """One device chain per seed: created and initialised on this thread, then run `batch`
    at a time concurrently (one stream each; the C calls release the GIL); returns each
    chain's (S, P) statistic rows."""
    out = [None] * len(seeds)
    err = []

    def work(c, ch):
        try:
            rec = ch.run(transient=transient, samples=samples, thin=1)
            lams = [rec[f"Lambda{r}"] for r in range(hM.nr)]
            alphas = [rec[f"Alpha{r}"] for r in range(hM.nr)]
            out[c] = param_rows(hM, rec["Beta"], rec["Gamma"], rec["iV"], rec["rho"], lams, alphas)
        except Exception as e:  # surfaced below
            err.append(e)

    for b0 in range(0, len(seeds), batch):
        idx = list(range(b0, min(len(seeds), b0 + batch)))
        chains = []
        for c in idx:
            ch = H.Chain(hM, int(seeds[c]), device=0, updater=updater)
            ch.init([int(rl.nfMin) for rl in hM.rL])
            chains.append(ch)
        th = [threading.Thread(target=work, args=(c, ch)) for c, ch in zip(idx, chains)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        for ch in chains:
            ch.close()
        if err:
            raise err[0]
    return out


@pytest.mark.parametrize("mode", ["on", "off"])
def test_td_long_run_matches_oracle(mode):
    D = np.load(FIX)
    hM = td_model()
    up = {} if mode == "on" else {"GammaEta": False}
    seeds = 910000 + 1000 * (mode == "off") + np.arange(DEV_CHAINS)
    rows = _device_chain_rows(hM, seeds, up, DEV_TRANSIENT, DEV_SAMPLES)
    dev = np.stack([r.mean(0) for r in rows])
    assert np.all(np.isfinite(dev))
    t = between_chain_t(dev, D[f"{mode}/mean"])
    names = list(D["names"])
    order = np.argsort(-np.abs(t))[:5]
    print(mode, "largest |t|:", [(names[i], round(float(t[i]), 2)) for i in order])
    assert np.max(np.abs(t)) < 4.0, [(names[i], float(t[i])) for i in order]


def test_td_reference_protocol_covers_reference_posterior():
    """64 device chains under the reference's protocol: the reference's 2-chain means of
    Beta, Gamma and rho lie within 3 sd of the distribution of 2-chain protocol means, and
    their chi-square is within its degrees of freedom."""
    hM = td_model()
    rows = _device_chain_rows(hM, 70000 + np.arange(64), {}, 50, 100)
    means = np.stack([r.mean(0) for r in rows])
    pairs = 0.5 * (means[0::2] + means[1::2])
    ref = np.mean([r.mean(0) for r in reference_rows(hM, td_postlist(hM))], axis=0)
    D = np.load(FIX)
    names = list(D["names"])
    sel = [i for i, n in enumerate(names) if n.startswith(("Beta", "Gamma", "rho"))]
    z = (ref - pairs.mean(0)) / pairs.std(0, ddof=1)
    print("z", {names[i]: round(float(z[i]), 2) for i in sel})
    assert np.max(np.abs(z[sel])) < 3.0
    assert float(np.sum(z[sel] ** 2)) < 2.0 * len(sel)
    # the device's protocol means agree with the oracle's protocol means (same algorithm)
    t = between_chain_t(means, D["short/means"])
    assert np.max(np.abs(t[sel])) < 4.0, t[sel]
