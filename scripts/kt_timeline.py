"""Per-sweep timeline of the synthetic config's graph-replayed sweep from the live launch
timers (hmsc_kernel_timing: each timed kernel's first start / last end per sweep, wall clock):
BetaLambda body, the fused launch's last reducer, Eta and Z, and the gaps between them."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import hmsc_amd as H  # noqa: E402
from hmsc_amd.workloads import synthetic_probit  # noqa: E402

KT_SLOTS, KT_N = 8192, 7
def _arg(name, default):
    return type(default)(sys.argv[sys.argv.index(name) + 1]) if name in sys.argv else default


# --sharded: the species-sharded chain on a one-rank RCCL communicator (the per-rank proxy of
# config 4's 8-way split with --ns 125); --ns: species count
hM = synthetic_probit(ns=_arg("--ns", 1000))
if "--sharded" in sys.argv:
    from hmsc_amd.sampler import comm_unique_id
    ch = H.Chain(hM, 1234567, device=0, updater={"GammaEta": False}, rank=0, nranks=1, comm_id=comm_unique_id())
else:
    ch = H.Chain(hM, 1234567, device=0, updater={"GammaEta": False})
ch.init([10])
ch.run(transient=100, samples=1, thin=1, adaptNf=[0], record=False)
ch.kernel_timing(True)
n = 400
if "--record" in sys.argv:  # every sweep recorded (the bench's timed region)
    ch.run(transient=0, samples=n, thin=1, adaptNf=[0], record=True, iter0=101)
else:
    ch.run(transient=n, samples=1, thin=1, adaptNf=[0], record=False, iter0=101)
kt = ch.debug_get("kt", KT_N * 2 * KT_SLOTS).reshape(KT_N, 2, KT_SLOTS)
its = np.arange(102 + 50, 101 + n)  # steady sweeps of the second run
names = ("z", "eta", "bl", "tail", "g2", "side")
st = {k: kt[i, 0, its % KT_SLOTS] for i, k in enumerate(names)}
en = {k: kt[i, 1, its % KT_SLOTS] for i, k in enumerate(names)}
nxt = (its + 1) % KT_SLOTS
tick_us = 0.01  # 100 MHz
rows = [
    ("Gamma2 wg0 start -> BL start", st["bl"] - st["g2"]),
    ("Gamma2 wg0 (wait + final)", en["g2"] - st["g2"]),
    ("BL body (first start -> last end)", en["bl"] - st["bl"]),
    ("BL end -> last reducer start", st["tail"] - en["bl"]),
    ("last reducer (sum + factor)", en["tail"] - st["tail"]),
    ("tail end -> Eta start", st["eta"] - en["tail"]),
    ("Eta", en["eta"] - st["eta"]),
    ("Eta end -> Z start", st["z"] - en["eta"]),
    ("Z", en["z"] - st["z"]),
    ("Z end -> next Gamma2 wg0 start", kt[4, 0, nxt] - en["z"]),
    ("side chain (start -> end)", en["side"] - st["side"]),
    ("side chain end -> next Gamma2 wg0 start", kt[4, 0, nxt] - en["side"]),
    ("BL end -> side chain start", st["side"] - en["bl"]),
    ("sweep (BL start -> next BL start)", kt[2, 0, nxt] - st["bl"]),
]
print("ar_calls", ch.debug_get("ar_calls", 4).tolist(), "graph", ch.debug_get("graph", 4).tolist())
for name, v in rows:
    if not np.all(np.isfinite(v)) or np.all(v == 0):
        continue
    v = v * tick_us
    print(f"{name:36s} median {np.median(v):8.2f} us  p10 {np.percentile(v, 10):8.2f}  p90 {np.percentile(v, 90):8.2f}")
