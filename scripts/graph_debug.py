"""Graph replay vs eager: state after plain sweeps and recorded samples, per sweeps-per-replay."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import hmsc_amd as H
from helpers import synthetic_model
hM = synthetic_model(ny=200, ns=30, nc=4, nf=3, nt=2, seed=12)
res = {}
for ng, per in (("1", "4"), ("0", "1"), ("0", "2"), ("0", "3"), ("0", "4")):
    os.environ["HMSC_NO_GRAPH"] = ng
    os.environ["HMSC_GRAPH_SWEEPS"] = per
    ch = H.Chain(hM, 77, device=0, updater={"GammaEta": False})
    ch.init()
    ch.run(transient=9, samples=0, adaptNf=[0], record=False)
    st = ch.get_state()
    print(ng, per, "graph", ch.debug_get("graph", 4))
    rec = ch.run(transient=0, samples=8, thin=1, adaptNf=[0], iter0=9)
    st2 = ch.get_state()
    res[(ng, per)] = (st["Beta"].copy(), rec["Beta"].copy(), st2["Beta"].copy())
    ch.close()
base = res[("1", "4")]
for k, v in res.items():
    print(k, "state-after-9", np.abs(v[0] - base[0]).max(), "rec per sample", [float(np.abs(v[1][i] - base[1][i]).max()) for i in range(8)],
          "state-after-17", np.abs(v[2] - base[2]).max())
# which eager sample does each graph sample match?
g = res[("0", "4")][1]
for i in range(8):
    print(i, [float(np.abs(g[i] - base[1][j]).max()) for j in range(8)])
