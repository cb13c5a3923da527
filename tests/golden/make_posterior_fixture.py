"""Generate tests/golden/posterior_small.npz: the CPU oracle's posterior on two small
synthetic models, the reference side of the distributional parity test
(tests/test_gpu_posterior.py, north star: "posterior means and variance partitioning must
match the CPU reference within Monte Carlo error, confirmed by KS / Gelman-Rubin checks on
Beta, Gamma and Omega").

The oracle (oracle/hmsc_oracle.py) restates the reference R updaters; R itself is not
installed here, so it stands in for the reference.  Chains are keyed 1000+c, disjoint
from any key the GPU test uses, so the two sides are independent samples of the same
posterior.  Every chain (both sides) starts from one converged oracle state (the prior
draw of computeInitialParameters can start a chain far in a heavy tail, from which it takes
thousands of sweeps to return, identically on both sides since they share the algorithm).
Stored per model: that start state, thinned draws (float32) of Beta, Gamma and the upper
triangle of Omega = Lambda' Lambda (scaled space), full-chain means / sds / ESS, and the
variance partitioning of each chain.

    python tests/golden/make_posterior_fixture.py      # ~3 minutes on 8 cores
"""
import os
import sys
from concurrent.futures import ProcessPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from posterior_common import (MODELS, N_CHAINS, SAMPLES, START_SEED, START_SWEEPS, THIN, TRANSIENT, pack_state,  # noqa: E402
                              summarise)


def start_state(name):
    import helpers
    from oracle import hmsc_oracle as O
    from oracle.rng import Rng
    hM = helpers.synthetic_model(**MODELS[name])
    m = helpers.oracle_model(hM)
    rng = Rng(START_SEED)
    st = O.compute_initial_parameters(m, rng)
    for it in range(1, START_SWEEPS + 1):
        st = O.sweep(st, m, rng, it, updater={"GammaEta": False})
    return name, st


def oracle_chain(args):
    name, c, st = args
    import helpers
    from oracle import hmsc_oracle as O
    from oracle.rng import Rng
    hM = helpers.synthetic_model(**MODELS[name])
    m = helpers.oracle_model(hM)
    rng = Rng(1000 + c)
    rec = {k: [] for k in ("Beta", "Gamma", "iV", "iSigma", "Lambda0")}
    thin = THIN.get(name, 1)
    for it in range(1, TRANSIENT + SAMPLES * thin + 1):
        st = O.sweep(st, m, rng, it, updater={"GammaEta": False})
        if it > TRANSIENT and (it - TRANSIENT) % thin == 0:
            rec["Beta"].append(st["Beta"].copy())
            rec["Gamma"].append(st["Gamma"].copy())
            rec["iV"].append(st["iV"].copy())
            rec["iSigma"].append(st["iSigma"].copy())
            rec["Lambda0"].append(st["Lambda"][0].copy())
    return name, c, {k: np.stack(v) for k, v in rec.items()}


def main():
    with ProcessPoolExecutor(max_workers=min(8, len(MODELS))) as ex:
        starts = dict(ex.map(start_state, list(MODELS)))
    jobs = [(name, c, starts[name]) for name in MODELS for c in range(N_CHAINS)]
    with ProcessPoolExecutor(max_workers=min(8, len(jobs))) as ex:
        res = list(ex.map(oracle_chain, jobs))
    out = {}
    for name in MODELS:
        out.update(pack_state(starts[name], f"{name}/start"))
    for name in MODELS:
        import helpers
        hM = helpers.synthetic_model(**MODELS[name])
        chains = [r for (n, c, r) in sorted(res, key=lambda t: t[1]) if n == name]
        summ = summarise(hM, chains)
        for k, v in summ.items():
            out[f"{name}/{k}"] = v
    np.savez_compressed(os.path.join(HERE, "posterior_small.npz"), **out)
    print({k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
