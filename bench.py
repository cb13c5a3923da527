#!/usr/bin/env python
"""bench.py — Gibbs sweeps/sec + Beta ESS/sec on the synthetic probit JSDM
(BASELINE.json config 4: ny=10k sites, ns=1k species, nc=20, nf=10), MI355X.

A "step" is one Gibbs sweep of Hmsc's sampleMcmc (R/sampleMcmc.R:219-315, all
default updaters except GammaEta=FALSE as BASELINE.md §2 prescribes), including the
per-sample record (the reference records every sweep at thin=1).

    python bench.py [--gpus N --steps K --warmup W] [--mode chains|sharded]

N>1 runs one rank per GPU under torch.distributed.run.  Launched under torchrun (WORLD_SIZE set),
WORLD_SIZE must equal --gpus.  Launched plainly with --gpus N > 1, bench.py starts
`python -m torch.distributed.run --nproc-per-node N bench.py <same args>` as a child process
before anything touches the GPU, fails if fewer than N devices are visible, and exits with the
child's return code (rank 0's JSON line goes straight to stdout); --dry-launch prints that
command as JSON instead of running it.
  * chains  (default): one independent chain per GPU, no communication (the
    reference's PSOCK chain farm, R/sampleMcmc.R:329-345) -> weak scaling;
    value = total chain-sweeps/sec over all GPUs.
  * sharded: ONE chain, species sharded over the GPUs, RCCL all-reduce of the
    sufficient statistics inside the C library -> strong scaling.
Rank 0 prints one JSON line.  Beta ESS/sec = (coda ESS per sweep of a separate recorded run
of >= 1000 samples after the timed region) x the timed sweeps/sec.  The CPU baseline (rank 0,
N=1 only) times the compiled C++ restatement of the same sweep (oracle/cpu/hmsc_cpu.cpp,
validated against the numpy oracle) with chains = host cores, one thread per chain, on a
bounded sample (R is absent, so the reference itself cannot be timed: kind "port").
"""
import argparse
import json
import os
import platform
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import hmsc_amd as H  # noqa: E402
from hmsc_amd.workloads import synthetic_probit  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=1000)
    p.add_argument("--warmup", type=int, default=100)
    p.add_argument("--mode", choices=["chains", "sharded"], default="chains")
    p.add_argument("--workload", choices=["synthetic", "spatial", "phylo"], default="synthetic",
                   help="synthetic: config 4 (the metric); spatial: config 5, vignette_4 'Full' at --ny; "
                        "phylo: config 3, vignette_3 (phylogeny, traits, GammaEta) at --ns species")
    p.add_argument("--method", choices=["Full", "NNGP", "GPP"], default="Full",
                   help="config 5's spatial method (vignettes/vignette_4_spatial.Rmd:95-245)")
    p.add_argument("--spatial-start", choices=["gpp", "init"], default="gpp",
                   help="config 5 Full / NNGP: start from the state of 300 GPP sweeps (mixing) or from "
                        "computeInitialParameters (Alpha stuck at grid point 1 for hundreds of sweeps)")
    p.add_argument("--ny", type=int, default=10000)
    p.add_argument("--ns", type=int, default=1000)
    p.add_argument("--nc", type=int, default=20)
    p.add_argument("--nf", type=int, default=10)
    p.add_argument("--cpu-sweeps", type=int, default=3, help="sweeps per CPU chain in the baseline sample")
    p.add_argument("--ess-samples", type=int, default=2000, help="recorded sweeps of the separate ESS run")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--clock-warmup-s", type=float, default=0.5,
                   help="config 4: extra untimed sweeps until the warm-up has run this long (clock ramp)")
    p.add_argument("--cpu-oracle-sweeps", type=int, default=None,
                   help="configs 3 / 5: sweeps of the numpy restatement timed for cpu_baseline "
                        "(default 10 for config 3, 3 for config 5)")
    p.add_argument("--no-sharded-leg", action="store_true",
                   help="chains mode: skip the short species-sharded run reported beside the main line")
    p.add_argument("--sharded-leg-timeout", type=float, default=180.0)
    p.add_argument("--pmc-json", default=None,
                   help="rocprofv3 PMC summary (scripts/pmc_summary.py) the roofline's traffic / valu come from "
                        "(default: the newest profiles/rNN_sM_pmc.json)")
    p.add_argument("--kernel-stats", default=None,
                   help="rocprofv3 --kernel-trace --stats CSV the roofline's traced launch time comes from "
                        "(default: the newest profiles/rNN_sM_kernel_stats.csv)")
    p.add_argument("--dry-launch", action="store_true",
                   help="--gpus N > 1 without torchrun: print the child launch command (JSON) and exit")
    args = p.parse_args()
    if args.pmc_json is None:
        args.pmc_json = newest_profile("pmc.json")
    if args.kernel_stats is None:
        args.kernel_stats = newest_profile("kernel_stats.csv")
    return args


def newest_profile(suffix):
    """The newest round-evidence file profiles/rNN_sM_<suffix> (highest round, then session)."""
    import re
    best, key = None, None
    d = os.path.join(ROOT, "profiles")
    for f in os.listdir(d) if os.path.isdir(d) else []:
        m = re.fullmatch(r"r(\d+)_s(\d+)_" + re.escape(suffix), f)
        if m and (key is None or (int(m[1]), int(m[2])) > key):
            best, key = os.path.join(d, f), (int(m[1]), int(m[2]))
    return best or os.path.join(d, "missing_" + suffix)


def launch_command(args, argv, port):
    """The per-GPU rank launch for --gpus N > 1 started without torchrun: torch.distributed.run
    on this node, one process per GPU, rendezvous on 127.0.0.1 (the reference's counterpart is
    the PSOCK chain farm, R/sampleMcmc.R:329-345).  The ranks get the same arguments."""
    rest = [a for a in argv if a != "--dry-launch"]
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + rest


def visible_devices():
    """GPUs visible to this process, counted without initialising the GPU (torch.cuda's count
    reads the HIP_VISIBLE_DEVICES / ROCR masks and the device nodes; no HIP context is made, so
    the children own the devices)."""
    import torch
    return int(torch.cuda.device_count())


def maybe_launch_ranks(args):
    """None when this process is the run itself (torchrun rank, or N = 1); otherwise the exit
    code of the child torchrun that ran the N ranks."""
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is not None:
        if int(world_env) != args.gpus:
            sys.exit(f"bench.py: WORLD_SIZE={world_env} but --gpus {args.gpus}: launch one rank per GPU "
                     f"(--nproc-per-node {args.gpus}) or pass --gpus {world_env}")
        return None
    if args.gpus <= 1:
        return None
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = launch_command(args, sys.argv[1:], port)
    if args.dry_launch:
        print(json.dumps({"launch": cmd, "nproc_per_node": args.gpus, "mode": args.mode}), flush=True)
        return 0
    n = visible_devices()
    if n < args.gpus:
        print(f"bench.py: --gpus {args.gpus} asks for {args.gpus} GPUs but {n} visible: refusing to measure "
              f"fewer (nothing run)", file=sys.stderr, flush=True)
        return 3
    import subprocess
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this host driver (RCCL)
    return subprocess.call(cmd, env=env)


def main():
    args = parse()
    rc = maybe_launch_ranks(args)  # before any HIP call: the ranks are child processes
    if rc is not None:
        sys.exit(rc)
    if args.workload == "spatial":
        return main_spatial(args)
    if args.workload == "phylo":
        return main_phylo(args)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # Load the HIP library before torch: torch bundles its own libamdhip64 with the same
    # soname, and whichever is loaded first serves the whole process.  The sampler is built
    # against /opt/rocm's runtime, whose graph launches are several times cheaper on the host.
    H._lib.lib()
    import torch
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")

    def barrier():
        if dist is not None:
            dist.barrier()

    def sync(ch):
        ch.sync()  # every stream of the chain (torch runs nothing on the GPU here)

    hM = synthetic_probit(ny=args.ny, ns=args.ns, nc=args.nc, nf=args.nf)
    upd = {"GammaEta": False}
    if args.mode == "sharded":
        cid = _shared_comm_id(rank, dist)
        with _stdout_to_stderr():
            ch = H.Chain(hM, 1234567, device=local, updater=upd, rank=rank, nranks=world, comm_id=cid)
    else:
        ch = H.Chain(hM, 1234567 + 7919 * rank, device=local, updater=upd)
    ch.init([args.nf])
    # in-kernel launch timer (wall clock at every workgroup's start/finish, per sweep slot):
    # on before the graph is captured so the replays of the timed region carry it
    ch.kernel_timing(True)
    # warm-up: one eager sweep (the steady state the sweep graphs are captured from), then the
    # graphs are captured, instantiated and uploaded (hmsc_prepare_graphs) and the remaining
    # warm-up sweeps run as graph replays -- the same recorded replay path as the timed
    # region (host ring, unpack threads) -- whatever the warm-up length; output discarded
    graphs = False
    if args.warmup > 0:
        ch.run(transient=0, samples=1, thin=1, adaptNf=[0], record=True)
        graphs = ch.prepare_graphs(2)
    if args.warmup > 1:
        ch.run(transient=0, samples=args.warmup - 1, thin=1, adaptNf=[0], iter0=1, record=True)
    # clock ramp: a few warm-up sweeps are ~1 ms of GPU work, too short for the card to leave
    # its idle clocks (at --warmup 5 the timed sweeps ran 10 % slower per kernel than at
    # --warmup 100).  Untimed sweeps of the same chain are added until the warm-up has kept the
    # GPU busy for --clock-warmup-s; the timed region is unchanged (exactly --steps sweeps).
    sync(ch)
    extra, it_next = 0, args.warmup
    t_w = time.perf_counter()
    def more():  # rank 0 decides, so that a sharded chain's ranks run the same sweeps
        go = args.warmup > 0 and time.perf_counter() - t_w < args.clock_warmup_s
        if dist is not None:
            f = torch.tensor([1 if go else 0], dtype=torch.int32)
            dist.broadcast(f, src=0)
            go = bool(f.item())
        return go

    while more():
        ch.run(transient=0, samples=50, thin=1, adaptNf=[0], iter0=it_next, record=True)
        sync(ch)
        extra += 50
        it_next += 50
    barrier()
    sync(ch)
    ch.kernel_timing(True)  # clear: keep only the timed region's launches
    t0 = time.perf_counter()
    # timed region: every sweep is a replay of the captured per-sweep hipGraph (capi.cpp)
    rec = ch.run(transient=0, samples=args.steps, thin=1, adaptNf=[0], iter0=it_next, record=True)
    sync(ch)
    barrier()
    t_run = time.perf_counter() - t0
    live = {}
    for name in ("z", "eta", "betalambda"):
        tot_us, n = ch.kernel_timing_get(name)
        live[name] = dict(total_us=tot_us, launches=n, avg_us=tot_us / max(1, n))
    ch.kernel_timing(False)
    # per-kernel durations: HIP events around the launches of a short eager (un-captured)
    # run on the chain's own stream, after the timed region
    n_prof = min(args.steps, 50)
    ch.profile(True)
    ch.run(transient=n_prof, samples=0, adaptNf=[0], iter0=it_next + args.steps, record=False)
    sync(ch)
    kern = {}
    for name in ("z", "betalambda", "eta_unit", "sweep"):
        tot, n = ch.profile_get(name)
        kern[name] = dict(total_ms=tot, launches=n, avg_us=1e3 * tot / max(1, n))
    ch.profile(False)

    # Beta ESS (coda::effectiveSize restated) from a separate recorded run of >= 1000 sweeps
    # of the same chain after the timed region (Beta only), per sweep; x the timed rate below
    n_ess = max(1000, args.ess_samples)
    rec_ess = ch.run(transient=0, samples=n_ess, thin=1, adaptNf=[0], iter0=it_next + args.steps + n_prof,
                     record=True, fields=("Beta",))
    sync(ch)
    beta = rec_ess["Beta"].reshape(n_ess, -1)
    ess_local = H.effectiveSize(beta) / n_ess                   # ESS per sweep, per Beta entry
    del rec
    tmax = t_run
    if dist is not None:
        t = torch.tensor([t_run], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        tmax = float(t.item())
        gathered = [None] * world
        dist.all_gather_object(gathered, ess_local)
        if args.mode == "sharded":
            ess_all = np.concatenate(gathered)       # disjoint species blocks of one chain
        else:
            ess_all = np.sum(np.stack(gathered), axis=0)  # chains: per-sweep ESS adds over chains
    else:
        ess_all = ess_local
    ch.close()
    # the species-sharded form of config 4 over the same GPUs (chains runs only), guarded: if
    # its collectives do not finish within --sharded-leg-timeout, rank 0 still prints the main
    # line (with the leg marked timed out) and every rank exits
    lock, printed = threading.Lock(), [False]

    def finish(sharded):
        with lock:
            if printed[0]:
                return
            printed[0] = True
        if rank == 0:
            _finish_main(args, world, tmax, ess_all, ess_local, n_ess, live, kern, graphs, extra, hM, sharded)

    sharded = None
    if args.mode == "chains" and not args.no_sharded_leg:
        def fire():
            try:
                finish({"error": f"timed out after {args.sharded_leg_timeout:.0f} s"})
            finally:
                os._exit(0)
        timer = threading.Timer(args.sharded_leg_timeout, fire)
        timer.daemon = True
        timer.start()
        try:
            # (as many recorded sweeps as the main line, at least 200 and at most 1000)
            sharded = sharded_leg(hM, args, rank, world, local, dist, steps=max(200, min(args.steps, 1000)))
        except Exception as e:  # noqa: BLE001 -- reported beside the main line, not fatal to it
            sharded = {"error": str(e)[:400]}
        timer.cancel()
    finish(sharded)


def _finish_main(args, world, tmax, ess_all, ess_local, n_ess, live, kern, graphs, extra, hM, sharded):
    ny, ns = args.ny, args.ns
    sweeps = args.steps * (world if args.mode == "chains" else 1)
    value = sweeps / tmax
    per_chain_rate = args.steps / tmax                         # sweeps/s of each chain
    ess_rate_median = float(np.median(ess_all)) * per_chain_rate
    ess_rate_min = float(np.min(ess_all)) * per_chain_rate

    # roofline: the dominant kernel of the sweep, algorithmic bytes per launch
    algo_bytes = {
        # fused updateZ: writes Z (fp64) + reads the int8 Y code, ny*ns each (R/updateZ.R)
        "z": ny * (ns // (world if args.mode == "sharded" else 1)) * (8 + 1),
        # fused updateEta: reads Z once for S*diag(iSigma)*Lambda^T (R/updateEta.R:33-55)
        "eta": ny * (ns // (world if args.mode == "sharded" else 1)) * 8,
        # BetaLambda: XEta^T Z arrives precomputed from the z kernel; reads XZ + writes BL
        "betalambda": (ns // (world if args.mode == "sharded" else 1)) * (args.nc + args.nf) * 8 * 2,
    }
    # roofline: the dominant kernel, its average duration measured live on the timed
    # region's graph replays by the in-kernel wall-clock timer (hmsc_kernel_timing)
    roof_kernel = max(live, key=lambda k: live[k]["total_us"])
    avg_s = live[roof_kernel]["avg_us"] * 1e-6
    achieved = algo_bytes[roof_kernel] / avg_s / 1e9
    traffic, valu = None, None
    if os.path.exists(args.pmc_json):
        try:
            pmc = json.load(open(args.pmc_json))
            pref = {"z": "z_wave_kernel", "eta": "eta_fused_kernel", "betalambda": "beta_lambda_wave_kernel"}
            hit = [v for k, v in pmc.items() if k.startswith(pref[roof_kernel])]
            if hit:
                traffic = round(hit[0]["hbm_bytes_per_launch"])
                # VALU issue floor: every VALU instruction of the launch at the fp64 issue cost
                # (4 cycles per wave instruction on a SIMD-32, MI355X_MICROARCH.md) over the
                # 1024 SIMDs at 2.4 GHz; frac = floor / the measured launch duration
                ni = hit[0].get("SQ_INSTS_VALU")
                if ni:
                    floor_us = ni * 4.0 / 1024 / 2.4e9 * 1e6
                    valu = {"bound": "valu", "valu_insts_per_launch": round(ni), "issue_floor_us": round(floor_us, 2),
                            "frac": round(floor_us / live[roof_kernel]["avg_us"], 4),
                            "source": os.path.relpath(args.pmc_json, ROOT)}
        except Exception:
            traffic, valu = None, None

    traced = traced_launch(args.kernel_stats, roof_kernel)
    if traced is not None:
        traced["achieved"] = round(algo_bytes[roof_kernel] / (traced["avg_us"] * 1e-6) / 1e9, 1)
        traced["frac"] = round(traced["achieved"] / HBM_PEAK_GBS, 4)
        if valu is not None:
            valu["frac_traced"] = round(valu["issue_floor_us"] / traced["avg_us"], 4)

    cpu = None
    if world == 1 and not args.no_cpu:
        cpu = cpu_baseline(hM, args, float(np.median(ess_local)))

    out = {
        "metric": "Gibbs sweeps/sec + Beta ESS/sec at ny=10k, ns=1k, nf=10; 1/2/4/8 MI355X",
        "value": round(value, 3),
        "unit": "sweeps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * tmax / args.steps, 4),
        "higher_is_better": True,
        "scaling": "weak" if args.mode == "chains" else "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (BASELINE.md §2 generator, seed 20261015)",
        "config": {"workload": f"synthetic probit JSDM ny={ny} ns={ns} nc={args.nc} nf={args.nf}, "
                               f"1 sample-level random level, updater GammaEta=FALSE, record every sweep",
                   "ny": ny, "ns": ns, "nc": args.nc, "nf": args.nf,
                   "parallelism": (f"{world} independent chains, one per GPU" if args.mode == "chains"
                                   else f"1 chain species-sharded over {world} GPUs (RCCL)")},
        "beta_ess_per_s": {"median": round(ess_rate_median, 3), "min": round(ess_rate_min, 3),
                           "n_beta": int(ess_all.size), "ess_per_sweep_median": float(np.median(ess_all)),
                           "ess_run": f"separate recorded run of {n_ess} sweeps after the timed region (coda "
                                      f"effectiveSize restated); ESS/s = ESS per sweep x timed sweeps/s"},
        "roofline": {"kernel": roof_kernel, "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "traffic_source": (os.path.relpath(args.pmc_json, ROOT) + " (rocprofv3 PMC passes, FETCH_SIZE x 2 "
                                        "+ WRITE_SIZE per launch)") if traffic else None,
                     "algorithmic_bytes_per_launch": algo_bytes[roof_kernel],
                     "avg_launch_us": round(live[roof_kernel]["avg_us"], 3),
                     "timed_launches": live[roof_kernel]["launches"],
                     "timer": "in-kernel wall clock (s_memrealtime, 100 MHz) over the timed region's graph replays",
                     "valu": valu,
                     "traced": traced,
                     "sweep_level": {"algorithmic_bytes_per_sweep": ny * ns * 25,
                                     "achieved": round(ny * ns * 25 * per_chain_rate / 1e9, 1),
                                     "frac": round(ny * ns * 25 * per_chain_rate / 1e9 / HBM_PEAK_GBS, 4),
                                     "note": "SURVEY 8(d): 3 fp64 Z touches + 1 B Y per cell per sweep"}},
        "graphs_prebuilt": graphs,
        "clock_warmup_sweeps": extra,
        "kernels_live_us": {k: round(v["avg_us"], 3) for k, v in live.items()},
        "kernels_eager_events_us": {k: round(v["avg_us"], 2) for k, v in kern.items()},
        "cpu_baseline": cpu,
        "sharded_chain": sharded,
    }
    print(json.dumps(out), flush=True)


KERNEL_PREFIX = {"z": "z_wave_kernel", "eta": "eta_fused_kernel", "betalambda": "gamma2_bl_kernel"}


def traced_launch(csv_path, kernel):
    """The dominant kernel's average launch duration from a committed rocprofv3 --kernel-trace
    --stats summary (the traced figure beside the live in-kernel timer's)."""
    import csv
    if not csv_path or not os.path.exists(csv_path):
        return None
    try:
        for r in csv.DictReader(open(csv_path)):
            if r["Name"].replace("void ", "").replace("hmsc::", "").startswith(KERNEL_PREFIX[kernel]):
                return {"avg_us": round(float(r["AverageNs"]) / 1e3, 3), "calls": int(r["Calls"]),
                        "source": os.path.relpath(csv_path, ROOT) + " (rocprofv3 --kernel-trace --stats)"}
    except Exception:  # noqa: BLE001 -- evidence is informative; the live timer is the measurement
        return None
    return None


class _stdout_to_stderr:
    """RCCL prints its version banner on stdout when the first communicator is made; the
    driver reads bench.py's stdout as ONE JSON line, so the RCCL setup writes to stderr."""

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)

    def __exit__(self, *exc):
        sys.stdout.flush()
        os.dup2(self.saved, 1)
        os.close(self.saved)
        return False


def _shared_comm_id(rank, dist):
    """An RCCL unique id made by rank 0 and broadcast over gloo (hmsc_comm_unique_id)."""
    from hmsc_amd.sampler import comm_unique_id
    with _stdout_to_stderr():
        cid = comm_unique_id() if rank == 0 else None
    obj = [cid]
    if dist is not None:
        dist.broadcast_object_list(obj, src=0)
    return obj[0]


def sharded_leg(hM, args, rank, world, local, dist, steps=200, warmup=40):
    """Config 4's other form on the same GPUs: ONE chain species-sharded over the `world` ranks
    (RCCL; at world = 1 a 1-rank communicator), two all-reduces per sweep captured in the sweep
    graphs (kernels.hip "species-sharded sweep").  A short timed run after the main measurement,
    reported beside it (strong scaling: the same ns = 1000 species over more GPUs)."""
    import torch
    cid = _shared_comm_id(rank, dist)
    with _stdout_to_stderr():
        ch = H.Chain(hM, 1234567, device=local, updater={"GammaEta": False}, rank=rank, nranks=world, comm_id=cid)
    ch.init([args.nf])
    ch.run(transient=0, samples=1, thin=1, adaptNf=[0], record=True)
    ch.prepare_graphs(2)
    # warm-up: at least `warmup` recorded sweeps, and at least 0.5 s of them (a new sharded
    # chain's first ~150 replayed sweeps ran ~40 % slower than its steady state, r06 traces);
    # rank 0 decides so every rank runs the same sweeps
    it, t_w = 1, time.perf_counter()
    while True:
        ch.run(transient=0, samples=warmup, thin=1, adaptNf=[0], iter0=it, record=True)
        ch.sync()
        it += warmup
        go = time.perf_counter() - t_w < 0.5
        if dist is not None:
            f = torch.tensor([1 if go else 0], dtype=torch.int32)
            dist.broadcast(f, src=0)
            go = bool(f.item())
        if not go:
            break
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    # (the record is kept past the timed region, as the main line's is: dropping ~0.2 GB of
    # arrays inside it unmapped their pages within the bracket -- ~60 us a sweep at 200 steps,
    # scripts/sharded_diag.py)
    rec = ch.run(transient=0, samples=steps, thin=1, adaptNf=[0], iter0=it, record=True)
    ch.sync()
    if dist is not None:
        dist.barrier()
    t = time.perf_counter() - t0
    del rec
    if dist is not None:
        tt = torch.tensor([t], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t = float(tt.item())
    ar = ch.debug_get("ar_calls", 4)
    graph = ch.debug_get("graph", 4)
    nsl = ch.nsl
    ch.close()
    return {"value": round(steps / t, 3), "unit": "sweeps/s", "ms_per_step": round(1e3 * t / steps, 4),
            "steps": steps, "warmup": it - 1, "ranks": world, "species_per_rank": nsl, "scaling": "strong",
            "allreduces_per_sweep": int(ar[2]), "graphs": bool(graph[0]),
            "transport": f"RCCL ({world}-rank communicator)",
            "note": "one chain, species-sharded over the GPUs, recording every sweep (beside the main line, "
                    "which is the chains form)"}


def main_spatial(args):
    """BASELINE.json config 5 (vignette_4 spatial, 'Full' GP latent factor) at ny = --ny
    (default 5000 when --ny is left at the config-4 value): ns=5, nc=2, nf=1, probit,
    updater GammaEta=FALSE (vignettes/vignette_4_spatial.Rmd:124).  One chain per GPU.  The
    alphapw grid (101 x ny^2 iW and RiW, 2 x 20 GB at ny=5k) is built on the device at chain
    creation (setup_s, outside the timed region).  Each sweep solves the (ny nf)^2 Eta system
    with the blocked Cholesky on the matrix cores and streams the grid once for updateAlpha;
    the roofline object prices the Cholesky (n^3 / 3 fp64 flops) against the fp64 matrix peak.
    --method GPP: the same model on the constructKnots(knotDist=0.2, minKnotDist=0.4) knots
    (:177-228), sampled in R's low-rank form (no np^2 array); the roofline prices updateAlpha's
    stream of the predictive-process grid (idDW12g + idDg, np (nK + 1) nalpha doubles) against HBM."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    H._lib.lib()
    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")
    from hmsc_amd.workloads import spatial_vignette4
    ny = 5000 if args.ny == 10000 else args.ny
    hM = spatial_vignette4(ny=ny, method=args.method)
    t0 = time.perf_counter()
    start_state = None
    if args.method != "GPP" and args.spatial_start == "gpp":
        # the timed chain starts where a chain mixes, not at Alpha = grid point 1: from
        # Alpha = 1 the Full / NNGP chain's Eta is drawn under the independent prior and
        # updateAlpha keeps it there for hundreds of sweeps at this ny (tests/
        # test_gpu_config5_chain.py), so the state of 300 sweeps of the same model on GPP
        # (R's predictive-process form, ~0.1 s) is handed over first, outside the timed region
        hG = spatial_vignette4(ny=ny, method="GPP")
        cg = H.Chain(hG, 4241 + 7919 * rank, device=local, updater={"GammaEta": False})
        cg.init([1])
        cg.run(transient=300, samples=0, thin=1, adaptNf=[0], record=False)
        sg = cg.get_state()
        cg.close()
        start_state = {k: sg[k] for k in ("Beta", "Gamma", "iV", "iSigma", "Eta", "Lambda", "Psi", "Delta",
                                          "Alpha", "Z")}
    ch = H.Chain(hM, 4242 + 7919 * rank, device=local, updater={"GammaEta": False})
    ch.init([1])
    if start_state is not None:
        ch.set_state(start_state)
    ch.sync()
    setup = time.perf_counter() - t0
    ch.run(transient=0, samples=args.warmup, thin=1, adaptNf=[0], record=True)
    ch.sync()
    ch.prepare_graphs(args.warmup + 1)
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    rec = ch.run(transient=0, samples=args.steps, thin=1, adaptNf=[0], iter0=args.warmup, record=True)
    ch.sync()
    if dist is not None:
        dist.barrier()
    t_run = time.perf_counter() - t0
    alpha_mean = float(np.mean(rec["Alpha0"]))
    del rec
    n_prof = min(args.steps, 20)
    ch.profile(True)
    ch.run(transient=n_prof, samples=0, adaptNf=[0], iter0=args.warmup + args.steps, record=False)
    ch.sync()
    kern = {}
    for name in ("eta_spatial", "chol", "alpha", "z", "betalambda", "sweep"):
        tot, n = ch.profile_get(name)
        kern[name] = dict(total_ms=tot, launches=n, avg_us=1e3 * tot / max(1, n))
    ch.profile(False)
    nngp_bw = int(ch.debug_get("nngp_bw0", 1)[0]) if args.method == "NNGP" else None
    ch.close()
    tmax = t_run
    if dist is not None:
        t = torch.tensor([t_run], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        tmax = float(t.item())
    if rank != 0:
        return
    N = ny  # np * nf
    chol_flops = N ** 3 / 3.0
    chol_s = kern["chol"]["avg_us"] * 1e-6
    peak_tf = 78.6
    achieved = chol_flops / max(chol_s, 1e-12) / 1e12
    grid_bytes = 101 * ny * ny * 8 / 2  # lower-triangular RiW_g streamed once per sweep
    alpha_s = kern["alpha"]["avg_us"] * 1e-6
    if args.method == "GPP":
        nK = int(hM.rL[0]["sKnot"].shape[0])
        gpp_bytes = 101 * ny * (nK + 1) * 8
        roof = {"kernel": "updateAlpha's GPP statistic (gpp_alpha_kernel): idDW12g and idDg streamed once per sweep",
                "bound": "hbm", "achieved": round(gpp_bytes / max(alpha_s, 1e-12) / 1e9, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(gpp_bytes / max(alpha_s, 1e-12) / 1e9 / HBM_PEAK_GBS, 4),
                "traffic": None, "algorithmic_bytes_per_launch": gpp_bytes,
                "avg_launch_us": round(kern["alpha"]["avg_us"], 1), "n_knots": nK,
                "timer": "HIP events on the chain stream around the updater (eager sweeps)"}
        workload = (f"vignette_4 spatial 'GPP' ny={ny} ns=5 nc=2 nf=1, {nK} knots (knotDist 0.2), "
                    f"101-point alphapw grid, R's low-rank updateEta, updater GammaEta=FALSE, record every sweep")
    elif args.method == "NNGP":
        # band Cholesky of the NNGP precision in RCM order: sum over columns of (band rows)^2
        bw = nngp_bw  # nf = 1: the matrix bandwidth is the unit bandwidth
        flops = float(N) * bw * bw
        roof = {"kernel": "band Cholesky of the NNGP Eta precision in RCM order (chol_diag/panel/update on the band)",
                "bound": "mfma", "achieved": round(flops / max(chol_s, 1e-12) / 1e12, 3), "peak": peak_tf,
                "unit": "TFLOP/s", "frac": round(flops / max(chol_s, 1e-12) / 1e12 / peak_tf, 5), "traffic": None,
                "algorithmic_flops_per_launch": flops, "bandwidth": bw, "avg_launch_us": round(kern["chol"]["avg_us"], 1),
                "timer": "HIP events on the chain stream around each factorization (eager sweeps)",
                "note": "latency bound: ceil(np / 64) dependent diagonal-block steps"}
        workload = (f"vignette_4 spatial 'NNGP' ny={ny} ns=5 nc=2 nf=1, 10 nearest neighbours, sparse Vecchia "
                    f"factor over the 101-point alphapw grid, updater GammaEta=FALSE, record every sweep")
    else:
        roof = {"kernel": "blocked Cholesky of the (np nf)^2 Eta precision (chol_diag/panel/update)",
                "bound": "mfma", "achieved": round(achieved, 2), "peak": peak_tf, "unit": "TFLOP/s",
                "frac": round(achieved / peak_tf, 4), "traffic": None,
                "algorithmic_flops_per_launch": chol_flops, "avg_launch_us": round(kern["chol"]["avg_us"], 1),
                "timer": "HIP events on the chain stream around each factorization (eager sweeps)",
                "alpha_grid": {"bytes_per_sweep": grid_bytes, "avg_us": round(kern["alpha"]["avg_us"], 1),
                               "achieved_GBs": round(grid_bytes / max(alpha_s, 1e-12) / 1e9, 1),
                               "peak_GBs": HBM_PEAK_GBS}}
        workload = (f"vignette_4 spatial 'Full' ny={ny} ns=5 nc=2 nf=1, 101-point alphapw grid, "
                    f"updater GammaEta=FALSE, record every sweep")
    out = {
        "metric": "Gibbs sweeps/sec, config 5 (vignette_4 spatial %s) at ny=%d" % (args.method, ny),
        "value": round(world * args.steps / tmax, 3), "unit": "sweeps/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(1e3 * tmax / args.steps, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (vignette_4 generator scaled to ny, seed 20261015)",
        "config": {"workload": workload,
                   "ny": ny, "ns": 5, "nc": 2, "nf": 1, "parallelism": f"{world} independent chains, one per GPU"},
        "setup_s": round(setup, 2),
        "roofline": roof,
        "kernels_eager_events_us": {k: round(v["avg_us"], 1) for k, v in kern.items()},
        "alpha_posterior_mean_index": round(alpha_mean, 2),
        "start": ("state of 300 GPP sweeps of the same model (Alpha index %s)" % (
            start_state["Alpha"][0].tolist() if start_state is not None else None)) if start_state is not None
                 else "computeInitialParameters (Alpha = grid point 1)",
        "cpu_baseline": None if (args.no_cpu or world > 1) else cpu_baseline_oracle(
            hM, {"GammaEta": False}, [1], args.cpu_oracle_sweeps or 3, f"vignette_4 '{args.method}' ny={ny}"),
    }
    print(json.dumps(out), flush=True)


def main_phylo(args):
    """BASELINE.json config 3: vignette_3 (vignettes/vignette_3_multivariate_high.Rmd:42-128)
    scaled to --ns species (default 300 when --ns is left at the config-4 value): ny=200, nc=4,
    nt=3, coalescent phylogeny, normal species, one sample-level level with nfMax=15, the
    reference's default updater set (GammaEta and Rho on; R/sampleMcmc.R:124-152 keeps both).
    One chain per GPU (the vignette's nChains).  Warm-up = transient with updateNf adaptation
    (adaptNf = transient, R's default), then the timed sweeps with recording.  Per sweep the
    dense phylogeny BetaLambda ((nc+nf) ns)^2 system and updateGammaEta's (nc ns)^2 systems run
    on the blocked fp64 Cholesky (dense.hip); the roofline prices BetaLambda's factorization
    ((nc+nf) ns)^3 / 3 flops against the fp64 matrix peak."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    H._lib.lib()
    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")
    from hmsc_amd.workloads import vignette3_phylo
    ns = 300 if args.ns == 1000 else args.ns
    hM = vignette3_phylo(ns=ns)
    t0 = time.perf_counter()
    ch = H.Chain(hM, 4242 + 7919 * rank, device=local, updater={})
    ch.init([int(hM.rL[0].nfMin)])
    ch.sync()
    setup = time.perf_counter() - t0
    ch.run(transient=args.warmup, samples=0, thin=1, adaptNf=[args.warmup], record=False)
    ch.sync()
    nf = int(ch.nf()[0])
    ch.prepare_graphs(args.warmup + 1)
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    rec = ch.run(transient=0, samples=args.steps, thin=1, adaptNf=[0], iter0=args.warmup, record=True)
    ch.sync()
    if dist is not None:
        dist.barrier()
    t_run = time.perf_counter() - t0
    rho_mean = float(np.mean(rec["rho"]))
    del rec
    n_prof = min(args.steps, 20)
    ch.profile(True)
    ch.run(transient=n_prof, samples=0, adaptNf=[0], iter0=args.warmup + args.steps, record=False)
    ch.sync()
    kern = {}
    for name in ("betalambda", "gamma_eta", "rho", "eta_unit", "z", "sweep"):
        tot, n = ch.profile_get(name)
        kern[name] = dict(total_ms=tot, launches=n, avg_us=1e3 * tot / max(1, n))
    ch.profile(False)
    ch.close()
    tmax = t_run
    if dist is not None:
        t = torch.tensor([t_run], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        tmax = float(t.item())
    if rank != 0:
        return
    N = (hM.nc + nf) * ns
    flops = N ** 3 / 3.0
    bl_s = kern["betalambda"]["avg_us"] * 1e-6
    peak_tf = 78.6
    achieved = flops / max(bl_s, 1e-12) / 1e12
    out = {
        "metric": "Gibbs sweeps/sec, config 3 (vignette_3 phylogeny + traits, default updaters) at ns=%d" % ns,
        "value": round(world * args.steps / tmax, 3), "unit": "sweeps/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(1e3 * tmax / args.steps, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (vignette_3 generator scaled to ns, coalescent phylogeny, seed 20261015)",
        "config": {"workload": f"vignette_3 ny=200 ns={ns} nc=4 nt=3 normal, phylogeny C, sample level nfMax=15 "
                               f"(nf={nf} after adaptation), default updaters incl. GammaEta and Rho, record every sweep",
                   "ny": 200, "ns": ns, "nc": 4, "nt": 3, "nf": int(nf),
                   "parallelism": f"{world} independent chains, one per GPU"},
        "setup_s": round(setup, 2),
        "roofline": {"kernel": "phylogeny BetaLambda: blocked Cholesky of the ((nc+nf) ns)^2 precision + solves",
                     "bound": "mfma", "achieved": round(achieved, 2), "peak": peak_tf, "unit": "TFLOP/s",
                     "frac": round(achieved / peak_tf, 4), "traffic": None,
                     "algorithmic_flops_per_launch": flops, "avg_launch_us": round(kern["betalambda"]["avg_us"], 1),
                     "timer": "HIP events on the chain stream around the updater (eager sweeps)"},
        "kernels_eager_events_us": {k: round(v["avg_us"], 1) for k, v in kern.items()},
        "rho_posterior_mean_index": round(rho_mean, 2),
        "cpu_baseline": None if (args.no_cpu or world > 1) else cpu_baseline_oracle(
            hM, {}, [nf], args.cpu_oracle_sweeps or 10, f"vignette_3 ns={ns} nf={nf}, default updaters"),
    }
    print(json.dumps(out), flush=True)


def _cpu_model():
    model = platform.processor() or platform.machine()
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return model


def cpu_baseline_oracle(hM, updater, nf, n_sweeps, what):
    """Configs 3 and 5: the numpy restatement of the reference's sweep (oracle/hmsc_oracle.py,
    the parity checker of the device path) timed on the host: compute_data_parameters and the
    initial state once (untimed, reported as setup_s), then n_sweeps full sweeps of one chain
    at the device chain's nf; multi-threaded only through numpy's BLAS/LAPACK (cores = its
    thread count).  The C++ port of config 4 covers neither the phylogeny nor the spatial
    levels, so this leg is the numpy one ("port", the reference's R being absent)."""
    from oracle import hmsc_oracle as O
    from oracle.rng import Rng
    m = dict(X=hM.XScaled, Y=hM.YScaled, Yraw=hM.Y, Tr=hM.TrScaled, Pi=hM.Pi, np=hM.np, distr=hM.distr,
             V0=hM.V0, f0=hM.f0, mGamma=hM.mGamma, UGamma=hM.UGamma, aSigma=hM.aSigma, bSigma=hM.bSigma,
             rhopw=hM.rhopw, C=hM.C,
             rL=[dict(nu=rl.nu, a1=rl.a1, b1=rl.b1, a2=rl.a2, b2=rl.b2, nfMin=rl.nfMin, nfMax=rl.nfMax,
                      sDim=rl.sDim, xDim=rl.xDim) for rl in (hM.rL or [])])
    for r, (d, rl) in enumerate(zip(m["rL"], hM.rL or [])):
        if rl.sDim:
            # rows of rl$s in levels(dfPi[,r]) order, the unit order of Eta (R indexes s by
            # the unit names, R/computeDataParameters.R:56,92,142)
            from hmsc_amd.dataparams import _level_order
            xy = np.asarray(rl.s, dtype=np.float64)[_level_order(hM, r, rl)]
            d.update(spatialMethod=rl.spatialMethod, alphapw=np.asarray(rl.alphapw, dtype=np.float64),
                     dist=np.sqrt(((xy[:, None, :] - xy[None, :, :]) ** 2).sum(-1)), s=xy,
                     nNeighbours=rl.nNeighbours, sKnot=rl["sKnot"] if "sKnot" in rl.names() else None)
    try:
        from threadpoolctl import threadpool_info
        cores = max([int(i.get("num_threads", 1)) for i in threadpool_info() if i.get("user_api") == "blas"] or [1])
    except Exception:  # noqa: BLE001 -- thread count is informative only
        cores = 1
    import threading
    done = threading.Event()

    def heartbeat():  # minutes of host work: keep the job's output alive
        while not done.wait(30.0):
            print(f"[bench] cpu_baseline ({what}): {time.perf_counter() - t0:.0f} s", file=sys.stderr, flush=True)

    t0 = time.perf_counter()
    threading.Thread(target=heartbeat, daemon=True).start()
    rng = Rng(1234567)
    dp = O.compute_data_parameters(m)
    st = O.compute_initial_parameters(m, rng, nf=list(nf))
    setup = time.perf_counter() - t0
    t0 = time.perf_counter()
    for it in range(1, n_sweeps + 1):
        st = O.sweep(st, m, rng, it, updater=updater, data_par=dp)
    sec = time.perf_counter() - t0
    done.set()
    del dp, st
    return {"value": round(n_sweeps / sec, 5), "unit": "sweeps/s", "cores": cores, "kind": "port",
            "sample": f"{n_sweeps} full sweeps of one chain of the numpy restatement (oracle/hmsc_oracle.py) "
                      f"at {what}, {sec:.1f} s wall after {setup:.1f} s of untimed setup "
                      f"(data parameters + initial state); BLAS threads {cores}; {_cpu_model()}",
            "setup_s": round(setup, 1)}


def cpu_baseline(hM, args, ess_per_sweep):
    """The compiled C++ restatement of the same sweep (oracle/cpu/hmsc_cpu.cpp; equal to the
    numpy oracle to fp64 rounding, tests/test_oracle_cpu_port.py), chains = host cores, one
    thread per chain, timed on a bounded sample: args.cpu_sweeps sweeps of every chain after
    its initialisation (R is absent, so this stands in for sampleMcmc with
    nChains = nParallel = cores, labelled "port")."""
    from oracle import cpu_port
    m = dict(X=hM.XScaled, Y=hM.YScaled, Yraw=hM.Y, Tr=hM.TrScaled, Pi=hM.Pi, np=hM.np, distr=hM.distr,
             V0=hM.V0, f0=hM.f0, mGamma=hM.mGamma, UGamma=hM.UGamma, aSigma=hM.aSigma, bSigma=hM.bSigma,
             rL=[dict(nu=rl.nu, a1=rl.a1, b1=rl.b1, a2=rl.a2, b2=rl.b2, nfMin=rl.nfMin, nfMax=rl.nfMax)
                 for rl in hM.rL])
    cores = min(os.cpu_count() or 1, int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or os.cpu_count() or 1, 64)
    _, sec = cpu_port.run(m, 1234567, n_sweeps=args.cpu_sweeps, nchains=cores, iter0=0, gamma2=True)
    rate = cores * args.cpu_sweeps / sec
    model = _cpu_model()
    return {"value": round(rate, 4), "unit": "sweeps/s", "cores": cores, "kind": "port",
            "sample": f"{cores} chains x {args.cpu_sweeps} full sweeps of the C++ restatement (oracle/cpu/hmsc_cpu.cpp, "
                      f"one thread per chain) at ny={args.ny} ns={args.ns} nc={args.nc} nf={args.nf}, "
                      f"{sec:.1f} s wall; {model}",
            "per_chain_sweeps_per_s": round(args.cpu_sweeps / sec, 4),
            "beta_ess_per_s_median_est": round(rate * ess_per_sweep, 5)}


if __name__ == "__main__":
    main()
