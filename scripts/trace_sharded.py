"""The species-sharded chain (one rank, RCCL) of config 4 for a kernel trace: graphs prebuilt,
200 recorded sweeps (run under rocprofv3 --kernel-trace; scripts/trace_view.py-style analysis
of the per-dispatch CSV)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import hmsc_amd as H  # noqa: E402
from hmsc_amd.workloads import synthetic_probit  # noqa: E402

hM = synthetic_probit()
from hmsc_amd.sampler import comm_unique_id  # noqa: E402
cid = comm_unique_id()
ch = H.Chain(hM, 1234567, device=0, updater={"GammaEta": False}, rank=0, nranks=1, comm_id=cid)
ch.init([10])
ch.run(transient=0, samples=1, thin=1, adaptNf=[0], record=True)
ch.prepare_graphs(2)
ch.run(transient=0, samples=40, thin=1, adaptNf=[0], iter0=1, record=True)
ch.run(transient=0, samples=200, thin=1, adaptNf=[0], iter0=41, record=True)
ch.sync()
print("ar_calls", ch.debug_get("ar_calls", 4), "graph", ch.debug_get("graph", 4))
ch.close()
