"""Generate tests/golden/vignette2_posterior.npz: the CPU oracle's posterior on the
vignette_2 models (BASELINE.json config 2; tests/vignette2_common.py), the reference side
of tests/test_gpu_vignette2.py.

The oracle (oracle/hmsc_oracle.py) restates the reference R updaters (R is not installed
here).  Oracle chains are keyed 1000+c, the GPU test's chains 1..8, so the two sides are
independent samples of one posterior; both start from the same converged oracle state.
The fixture is therefore oracle-relative (parity with the reference unpinned for these
posteriors: no output of the reference covers them); the oracle is pinned by the TD fixtures.

    python tests/golden/make_vignette2_fixture.py      # ~7 minutes on 8 cores
"""
import os
import sys
from concurrent.futures import ProcessPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from vignette2_common import (MODELS, N_CHAINS, SAMPLES, START_SEED, START_SWEEPS, THIN, TRANSIENT,  # noqa: E402
                              UPDATER, model, pack_state, summarise)


def start_state(name):
    import helpers
    from oracle import hmsc_oracle as O
    from oracle.rng import Rng
    m = helpers.oracle_model(model(name))
    rng = Rng(START_SEED)
    st = O.compute_initial_parameters(m, rng)
    for it in range(1, START_SWEEPS + 1):
        st = O.sweep(st, m, rng, it, updater=UPDATER[name])
    return name, st


def oracle_chain(args):
    name, c, st = args
    import helpers
    from oracle import hmsc_oracle as O
    from oracle.rng import Rng
    hM = model(name)
    m = helpers.oracle_model(hM)
    rng = Rng(1000 + c)
    keys = ("Beta", "Gamma", "iV", "iSigma") + (("Lambda0",) if hM.nr else ())
    rec = {k: [] for k in keys}
    for it in range(1, TRANSIENT + SAMPLES * THIN[name] + 1):
        st = O.sweep(st, m, rng, it, updater=UPDATER[name])
        if it > TRANSIENT and (it - TRANSIENT) % THIN[name] == 0:
            for k in keys:
                rec[k].append((st["Lambda"][0] if k == "Lambda0" else st[k]).copy())
    return name, c, {k: np.stack(v) for k, v in rec.items()}


def main():
    with ProcessPoolExecutor(max_workers=len(MODELS)) as ex:
        starts = dict(ex.map(start_state, MODELS))
    jobs = [(name, c, starts[name]) for name in MODELS for c in range(N_CHAINS)]
    with ProcessPoolExecutor(max_workers=8) as ex:
        res = list(ex.map(oracle_chain, jobs))
    out = {}
    for name in MODELS:
        hM = model(name)
        out.update(pack_state(starts[name], f"{name}/start", hM.nr))
        chains = [r for (n, c, r) in sorted(res, key=lambda t: t[1]) if n == name]
        for k, v in summarise(hM, chains).items():
            out[f"{name}/{k}"] = v
    np.savez_compressed(os.path.join(HERE, "vignette2_posterior.npz"), **out)


if __name__ == "__main__":
    main()
