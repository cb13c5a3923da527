"""Read the HMSC_STAMP clock stamps of one sweep at the synthetic config (diagnostic
library: python -m hmsc_amd.build --stamps; run with HMSC_AMD_LIB=.../libhmsc_amd_stamps.so)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("HMSC_AMD_LIB", os.path.join(ROOT, "hmsc_amd", "libhmsc_amd_stamps.so"))
import hmsc_amd as H  # noqa: E402
from hmsc_amd.workloads import synthetic_probit  # noqa: E402

hM = synthetic_probit()
ch = H.Chain(hM, 1234567, device=0, updater={"GammaEta": False})
ch.init([10])
if "--graph" in sys.argv:  # the last sweep of a run of captured-graph replays
    ch.run(transient=300, samples=1, thin=1, record=False)
else:
    for it in range(1, 6):
        ch.sweep(it)
ch.sync()
st = ch.debug_get("stamps", 128)
groups = {"gammav_wave": range(0, 10), "delta": range(20, 22), "gamma2_final": range(30, 33), "eta_shared(block0)": range(40, 45), "eta_fused(block0)": range(50, 56),
          "beta_lambda(block0)": range(60, 65), "gammav_wave1": range(10, 15)}
v = np.array([st[i] for i in range(70, 77)])
print("gamma2_bl (10 ns ticks from workgroup 0's start): partial0 start", v[1] - v[0],
      "final start", v[2] - v[0], "final done", v[3] - v[0], "BL0 chol done", v[4] - v[0],
      "BL0 wait done", v[5] - v[0], "BL0 end", v[6] - v[0])
v = np.array([st[i] for i in range(70, 91)], dtype=np.float64)
t0 = v[0]
print("  tail (10 ns ticks from workgroup 0 start): BL0 side-wait done", v[14] - t0, "BL0 tail start", v[7] - t0,
      "group0 reducer", v[8] - t0, "final reducer", v[9] - t0, "final done", v[10] - t0)
print("  tail block0: draws done", v[15] - t0, "tile stored", v[16] - t0, "group0 tile stored", v[17] - t0,
      "final sums in", v[18] - t0)
print("  post_bl (side partials): start", v[19] - t0, "tails seen", v[20] - t0)
print("  side chain: start", v[11] - t0, "tails seen", v[12] - t0, "GammaV out", v[13] - t0, "(of the last sweep)")
v = np.array([st[i] for i in range(91, 98)], dtype=np.float64) - t0
print("  BL workgroup 40 (10 ns from workgroup 0 start): kernel entry %.0f body entry %.0f loads issued %.0f staged %.0f"
      " chol done %.0f Gamma seen %.0f end %.0f" % (v[6], v[0], v[1], v[2], v[3], v[4], v[5]))
v = np.array([st[i] for i in range(100, 106)], dtype=np.float64) - t0
print("  BL workgroup 40: tau done %.0f precision built %.0f rhs formed %.0f forward done %.0f transposed %.0f backward done %.0f" % tuple(v))
if "--parts" in sys.argv:  # Gamma2 partial workgroups: start / end (wall clock) from workgroup 0's start
    allst = np.array(ch.debug_get("stamps", 1024), dtype=np.float64)
    n = int(sys.argv[sys.argv.index("--parts") + 1])
    ps, pe = allst[700:700 + n] - t0, allst[860:860 + n] - t0
    print("  Gamma2 partials (10 ns): start min %.0f max %.0f  end min %.0f median %.0f max %.0f  longest %.0f" %
          (ps.min(), ps.max(), pe.min(), np.median(pe), pe.max(), (pe - ps).max()))
if "--blocks" in sys.argv:  # per-BetaLambda-workgroup body end (wall clock), from workgroup 0's start
    allst = ch.debug_get("stamps", 1024)
    e = np.array(allst[256:256 + 250], dtype=np.float64) - t0
    print("  BL body end per workgroup (10 ns): min %.0f median %.0f p90 %.0f max %.0f" % (e.min(), np.median(e), np.percentile(e, 90), e.max()))
    order = np.argsort(e)[::-1][:12]
    print("  latest workgroups:", [(int(b), int(e[b])) for b in order])
for name, idx in groups.items():
    v = np.array([st[i] for i in idx])
    d = np.diff(v)
    print(name, "total cycles", v[-1] - v[0], "segments", d.astype(np.int64).tolist())
