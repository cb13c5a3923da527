"""Short run for a rocprofv3 kernel trace: 60 sweeps without recording, then 60 with."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import hmsc_amd as H  # noqa: E402
from hmsc_amd.workloads import synthetic_probit  # noqa: E402

hM = synthetic_probit(ny=10000, ns=1000, nc=20, nf=10)
ch = H.Chain(hM, 1234567, device=0, updater={"GammaEta": False})
ch.init([10])
ch.run(transient=60, samples=0, adaptNf=[0], record=False)
ch.run(transient=0, samples=60, thin=1, adaptNf=[0], iter0=60, record=True)
ch.sync()
ch.close()
print("ok")
