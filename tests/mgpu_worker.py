"""Rank program of tests/test_gpu_multigpu.py, launched by torch.distributed.run, one rank per
GPU (never imported by pytest).

    --mode sharded  one chain, species-sharded over the ranks: hmsc_create_sharded with an RCCL
                    communicator (unique id broadcast over gloo), the all-reduces of
                    capi.cpp allreduce_sum on RCCL over xGMI;
    --mode chains   independent chains, chain c = rank on device LOCAL_RANK (key seed + 7919 rank).
Each rank runs init + --sweeps sweeps and writes its state to <out>/rank<r>.npz.
"""
import argparse
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))

import hmsc_amd as H  # noqa: E402
from hmsc_amd import _lib as L  # noqa: E402

L.lib()  # the HIP library before torch (bench.py: torch bundles a libamdhip64 of the same soname)

from helpers import synthetic_model  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--mode", choices=["sharded", "chains"], required=True)
    p.add_argument("--out", required=True)
    p.add_argument("--sweeps", type=int, default=5)
    a = p.parse_args()
    import torch.distributed as dist
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    dist.init_process_group("gloo")
    hM = synthetic_model(ny=300, ns=41, nc=4, nf=3, seed=61)
    up = {"GammaEta": False}
    if a.mode == "sharded":
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
    g = ch.get_state()
    ch.close()
    np.savez(os.path.join(a.out, f"rank{rank}.npz"), Beta=g["Beta"], Lambda=g["Lambda"][0], Z=g["Z"],
             Gamma=g["Gamma"], iV=g["iV"], iSigma=g["iSigma"], sp0=ch.sp0, nsl=ch.nsl, device=local)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
