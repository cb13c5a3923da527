"""Multi-process (gloo, world_size 2, CPU) checks of the multi-GPU decomposition.

The species-sharded single chain (RCCL inside hmsc_create_sharded)
splits species into contiguous blocks and all-reduces, once per updater, the
species-sums that couple the shards.  Here each rank computes its block's share of
those sums with the oracle's formulas and a gloo all_reduce must reproduce the
unsharded values — the same decomposition and block arithmetic the C library uses
(capi.cpp shard_range: whole species quads spread evenly over the ranks).  Chains mode needs no exchange;
its timing reduction (max over ranks) is checked too.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from helpers import O, oracle_model, synthetic_model
from oracle.rng import Rng


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def species_block(ns, rank, nranks):
    """capi.cpp shard_range (hmsc_shard_range): whole species quads (updateZ draws a quad from
    one Philox block), spread evenly."""
    quads = (ns + 3) // 4
    return min(ns, 4 * (quads * rank // nranks)), min(ns, 4 * (quads * (rank + 1) // nranks))


def sufficient_stats(st, m, sl):
    """The all-reduced quantities of one sharded sweep, restricted to species slice sl."""
    lam = np.concatenate(st["Lambda"], axis=0)[:, sl]
    iS = st["iSigma"][sl]
    Z = st["Z"][:, sl]
    BL = np.concatenate([st["Beta"]] + st["Lambda"], axis=0)[:, sl]
    E = st["Beta"][:, sl] - st["Gamma"] @ m["Tr"][sl].T
    psi = np.concatenate(st["Psi"], axis=0)[:, sl]
    return {
        "ZL": Z @ (lam * iS).T,                                  # updateEta numerator (R/updateEta.R:55)
        "CR": (BL * iS) @ lam.T,                                 # Lambda diag(iSigma) Lambda^T and cross terms (:45)
        "A": E @ E.T,                                            # updateGammaV E E^T (R/updateGammaV.R:18)
        "BTr": st["Beta"][:, sl] @ m["Tr"][sl],                  # (R/updateGammaV.R:30)
        "ZTr": Z @ m["Tr"][sl],                                  # updateGamma2 (R/updateGamma2.R:46)
        "psi_rs": (psi * lam ** 2).sum(axis=1),                  # updateLambdaPriors row sums (:24-26)
    }


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    hM = synthetic_model(ny=80, ns=13, nc=3, nf=2, seed=21)
    m = oracle_model(hM)
    st = O.compute_initial_parameters(m, Rng(5))
    a, b = species_block(hM.ns, rank, world)
    loc = sufficient_stats(st, m, slice(a, b))
    out = {}
    for k, v in loc.items():
        t = torch.from_numpy(np.ascontiguousarray(v, dtype=np.float64))
        dist.all_reduce(t)
        out[k] = t.numpy()
    full = sufficient_stats(st, m, slice(0, hM.ns))
    err = max(float(np.max(np.abs(out[k] - full[k])) / max(1e-300, np.max(np.abs(full[k])))) for k in full)
    t_run = torch.tensor([0.5 + rank], dtype=torch.float64)      # chains mode: job time = max over ranks
    dist.all_reduce(t_run, op=dist.ReduceOp.MAX)
    covered = torch.tensor([b - a], dtype=torch.int64)
    dist.all_reduce(covered)
    q.put((rank, err, float(t_run.item()), int(covered.item())))
    dist.destroy_process_group()


@pytest.mark.timeout(240)
def test_species_sharded_statistics_allreduce_gloo():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=200) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, err, tmax, covered in res:
        assert err < 1e-12, (rank, err)
        assert tmax == 1.5
        assert covered == 13


def test_species_blocks_partition():
    for ns in (1, 7, 1000, 1003):
        for n in (1, 2, 4, 8):
            if 4 * n > ns + 3:
                continue
            blocks = [species_block(ns, r, n) for r in range(n)]
            assert all(b > a for a, b in blocks)
            assert blocks[0][0] == 0 and blocks[-1][1] == ns
            assert all(blocks[i][1] == blocks[i + 1][0] for i in range(n - 1))
