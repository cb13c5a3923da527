"""Generate tests/golden/td_longrun.npz: the CPU oracle's long-run posterior of the TD$m
spec (data-raw/simulateTestData.R:60-70; two random levels -- sample and the spatial 'Full'
plot level --, phylogeny C, traits, probit), with the reference's default updater set
(GammaEta on, "on") and with updater GammaEta=FALSE ("off"), plus N_SHORT chains run under the
reference's own short protocol (transient 50, samples 100: "short/means", one row per chain).

The oracle (oracle/hmsc_oracle.py) restates the R updaters; R is not installed here, so it
stands in for the reference.  Both samplers target one posterior, so the "on"
and "off" summaries must agree within Monte Carlo error (tests/test_golden_td_longrun.py);
the device's chains are compared with the "on" summary in tests/test_gpu_td_posterior.py.
Chains start from computeInitialParameters (prior draws) like the reference and discard a
transient of TRANSIENT sweeps.

    python tests/golden/make_td_longrun_fixture.py      # ~8 minutes on 8 cores
"""
import os
import sys
from concurrent.futures import ProcessPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from td_longrun_common import (N_CHAINS, N_SHORT, SAMPLES, SEED0, SHORT_SAMPLES, SHORT_TRANSIENT, THIN_STORE,  # noqa: E402
                               TRANSIENT, chain_summary, names, param_rows)


def oracle_chain(args):
    mode, c = args
    if mode == "short":
        return mode, c, short_protocol_chain(c), None
    os.environ.setdefault("OMP_NUM_THREADS", "1")
    import helpers
    from oracle import hmsc_oracle as O
    from oracle.rng import Rng
    from test_golden_td import td_model
    hM = td_model()
    m = helpers.oracle_model(hM)
    dp = O.compute_data_parameters(m)
    rng = Rng(SEED0[mode] + c)
    up = {} if mode == "on" else {"GammaEta": False}
    st = O.compute_initial_parameters(m, rng)
    keep = {k: [] for k in ("Beta", "Gamma", "iV", "rho", "L0", "L1", "A0", "A1")}
    for it in range(1, TRANSIENT + SAMPLES + 1):
        st = O.sweep(st, m, rng, it, updater=up, data_par=dp)
        if it > TRANSIENT:
            keep["Beta"].append(st["Beta"]), keep["Gamma"].append(st["Gamma"]), keep["iV"].append(st["iV"])
            keep["rho"].append(st["rho"])
            keep["L0"].append(st["Lambda"][0]), keep["L1"].append(st["Lambda"][1])
            keep["A0"].append(st["Alpha"][0]), keep["A1"].append(st["Alpha"][1])
    k = {a: np.stack(v) for a, v in keep.items()}
    rows = param_rows(hM, k["Beta"], k["Gamma"], k["iV"], k["rho"], [k["L0"], k["L1"]], [k["A0"], k["A1"]])
    return mode, c, chain_summary(rows), rows[::THIN_STORE].astype(np.float32)


def short_protocol_chain(c):
    """The reference's own protocol for TD$m (transient=50, samples=100, thin=1,
    data-raw/simulateTestData.R:70): this chain's posterior-mean statistics."""
    import helpers
    from oracle import hmsc_oracle as O
    from oracle.rng import Rng
    from test_golden_td import td_model
    hM = td_model()
    m = helpers.oracle_model(hM)
    dp = O.compute_data_parameters(m)
    rng = Rng(SEED0["short"] + c)
    st = O.compute_initial_parameters(m, rng)
    keep = {k: [] for k in ("Beta", "Gamma", "iV", "rho", "L0", "L1", "A0", "A1")}
    for it in range(1, SHORT_TRANSIENT + SHORT_SAMPLES + 1):
        st = O.sweep(st, m, rng, it, data_par=dp)
        if it > SHORT_TRANSIENT:
            keep["Beta"].append(st["Beta"]), keep["Gamma"].append(st["Gamma"]), keep["iV"].append(st["iV"])
            keep["rho"].append(st["rho"])
            keep["L0"].append(st["Lambda"][0]), keep["L1"].append(st["Lambda"][1])
            keep["A0"].append(st["Alpha"][0]), keep["A1"].append(st["Alpha"][1])
    k = {a: np.stack(v) for a, v in keep.items()}
    return param_rows(hM, k["Beta"], k["Gamma"], k["iV"], k["rho"], [k["L0"], k["L1"]], [k["A0"], k["A1"]]).mean(0)


def main():
    from test_golden_td import td_model
    jobs = [(mode, c) for mode in ("on", "off") for c in range(N_CHAINS)] + [("short", c) for c in range(N_SHORT)]
    import multiprocessing as mp
    # spawn: fresh workers (a forked worker would share the parent's open td.npz handle)
    with ProcessPoolExecutor(max_workers=8, mp_context=mp.get_context("spawn")) as ex:
        res = list(ex.map(oracle_chain, jobs))
    out = {"names": np.array(names(td_model()))}
    for mode in ("on", "off"):
        rs = sorted([r for r in res if r[0] == mode], key=lambda t: t[1])
        for key in ("mean", "var", "ess"):
            out[f"{mode}/{key}"] = np.stack([r[2][key] for r in rs])
        out[f"{mode}/draws"] = np.stack([r[3] for r in rs])
    out["short/means"] = np.stack([r[2] for r in sorted([r for r in res if r[0] == "short"], key=lambda t: t[1])])
    out["meta"] = np.array([TRANSIENT, SAMPLES, N_CHAINS, THIN_STORE])
    np.savez_compressed(os.path.join(HERE, "td_longrun.npz"), **out)
    print({k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
