"""updateNf (R/updateNf.R:3-70) on the device against the oracle: a level with
nfMin < nfMax adapts its number of factors during the first adaptNf sweeps (add a factor
with probability exp(-1 - 0.0005 iter) when none is redundant and iter > 20, or drop one --
the reference's setdiff(1:nf, logical) quirk drops factor 1).  The
device keeps its buffers at nfMax and repacks on the host (capi.cpp update_nf); both sides
share the Philox stream, so nf must follow the same path sweep by sweep and the states
stay equal."""
import numpy as np
import pytest

from helpers import H, O, oracle_model, rel_err, synthetic_model
from oracle.rng import Rng

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("kw", [
    dict(ny=120, ns=15, nc=3, nf=3, nf_fit=None, seed=41),
    dict(ny=150, ns=12, nc=2, nf=2, nr=2, units=[150, 30], seed=42)])
def test_update_nf_tracks_oracle(kw):
    hM = synthetic_model(**kw)
    for rl in hM.rL:
        H.setPriors(rl, nfMin=2, nfMax=6)
    m = oracle_model(hM)
    seed = 1357
    up = {"GammaEta": False}
    ch = H.Chain(hM, seed, device=0, updater=up)
    ch.init([2] * hM.nr)
    rng = Rng(seed)
    o = O.compute_initial_parameters(m, rng, nf=[2] * hM.nr)
    nf_path_dev, nf_path_orc = [], []
    n_adapt = 60
    for it in range(1, n_adapt + 1):
        ch.sweep(it, adapt=True)
        o = O.sweep(o, m, rng, it, updater=up, adapt_nf=[n_adapt] * hM.nr)
        nf_path_dev.append(tuple(ch.nf()))
        nf_path_orc.append(tuple(l.shape[0] for l in o["Lambda"]))
    assert nf_path_dev == nf_path_orc
    assert len(set(nf_path_dev)) > 1, "nf never changed: the test did not exercise updateNf"
    g = ch.get_state()
    for r in range(hM.nr):
        assert g["Lambda"][r].shape == o["Lambda"][r].shape
        assert rel_err(g["Lambda"][r], o["Lambda"][r]) < 1e-6
        assert rel_err(g["Eta"][r], o["Eta"][r]) < 1e-6
        assert rel_err(g["Delta"][r], o["Delta"][r]) < 1e-6
    assert rel_err(g["Beta"], o["Beta"]) < 1e-6
    # the sampler keeps running at the adapted nf (graph replays after the adaptive phase)
    rec = ch.run(transient=0, samples=10, thin=1, adaptNf=[0] * hM.nr, iter0=n_adapt)
    assert np.all(rec["nf"] == np.array(nf_path_dev[-1])[:, None])
    ch.close()
