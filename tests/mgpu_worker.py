"""Rank program of tests/test_gpu_multigpu.py and tests/test_gpu_sharded_procs.py, launched
by torch.distributed.run, one process per rank (never imported by pytest).

    --mode sharded  one chain, species-sharded over the ranks (two all-reduces per sweep,
                    kernels.hip "species-sharded sweep"):
                      --transport rccl  hmsc_create_sharded with an RCCL communicator (unique id
                                        broadcast over gloo), the all-reduces on RCCL over xGMI;
                      --transport host  hmsc_create_sharded_host, the all-reduces through a
                                        callback that sums over gloo (torch.distributed) -- the
                                        form that runs with every rank on one GPU (--same-device);
    --mode chains   independent chains, chain c = rank on device LOCAL_RANK (key seed + 7919 rank).
Each rank runs init + --sweeps eager sweeps, then --recorded sweeps through hmsc_run (sweep graphs,
recording every sweep), and writes its state and the recorded Beta to <out>/rank<r>.npz.
"""
import argparse
import os
import sys
from datetime import timedelta

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))

import hmsc_amd as H  # noqa: E402
from hmsc_amd import _lib as L  # noqa: E402

L.lib()  # the HIP library before torch (bench.py: torch bundles a libamdhip64 of the same soname)

from helpers import synthetic_model  # noqa: E402

MODELS = {"small": dict(ny=300, ns=41, nc=4, nf=3, seed=61),
          "mid": dict(ny=2000, ns=160, nc=6, nf=5, seed=72),
          "na": dict(ny=400, ns=50, nc=4, nf=3, na_frac=0.05, seed=73)}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--mode", choices=["sharded", "chains"], required=True)
    p.add_argument("--transport", choices=["rccl", "host"], default="rccl")
    p.add_argument("--same-device", action="store_true", help="every rank on GPU 0")
    p.add_argument("--model", choices=sorted(MODELS), default="small")
    p.add_argument("--out", required=True)
    p.add_argument("--sweeps", type=int, default=5)
    p.add_argument("--recorded", type=int, default=0)
    a = p.parse_args()
    import torch
    import torch.distributed as dist
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    local = 0 if a.same_device else int(os.environ.get("LOCAL_RANK", rank))
    dist.init_process_group("gloo", timeout=timedelta(seconds=120))
    hM = synthetic_model(**MODELS[a.model])
    up = {"GammaEta": False}
    n_ar = [0]
    if a.mode == "sharded" and a.transport == "host":
        def allreduce(x):  # x: the library's pinned staging buffer, summed in place over gloo
            n_ar[0] += 1
            dist.all_reduce(torch.from_numpy(x))
        ch = H.Chain(hM, 97531, device=local, updater=up, rank=rank, nranks=world, host_allreduce=allreduce)
    elif a.mode == "sharded":
        obj = [None]
        if rank == 0:
            buf = np.zeros(128, dtype=np.uint8)
            L.check(L.lib().hmsc_comm_unique_id(buf.ctypes.data))
            obj[0] = bytes(buf)
        dist.broadcast_object_list(obj, src=0)
        ch = H.Chain(hM, 97531, device=local, updater=up, rank=rank, nranks=world, comm_id=obj[0])
    else:
        ch = H.Chain(hM, 97531 + 7919 * rank, device=local, updater=up)
    ch.init()
    for it in range(1, a.sweeps + 1):
        ch.sweep(it)
    rec_beta = np.zeros(0)
    if a.recorded > 0:
        rec = ch.run(transient=0, samples=a.recorded, thin=1, adaptNf=[0], iter0=a.sweeps, record=True)
        rec_beta = rec["Beta"]
    g = ch.get_state()
    ar = ch.debug_get("ar_calls", 4)
    graph = ch.debug_get("graph", 4)
    ch.close()
    np.savez(os.path.join(a.out, f"rank{rank}.npz"), Beta=g["Beta"], Lambda=g["Lambda"][0], Z=g["Z"],
             Gamma=g["Gamma"], iV=g["iV"], iSigma=g["iSigma"], Eta=g["Eta"][0], Delta=g["Delta"][0],
             sp0=ch.sp0, nsl=ch.nsl, device=local, rec_beta=rec_beta, ar_calls=ar, graph=graph,
             callbacks=n_ar[0])
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
