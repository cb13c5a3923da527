"""GPU-box diagnostic: where a one-rank RCCL sharded chain's bench-leg time goes.  The chain as
bench.py's sharded leg builds it (config 4), warmed up, then timed runs of 200 and 1000 recorded
sweeps and 200 unrecorded ones, each with the library's host timer (HMSC_DIAG_TIMING=1 prints
setup / enqueue / device-done / unpack per run on stderr); the unsharded chain's same runs beside."""
import os
import sys
import time

os.environ.setdefault("HMSC_DIAG_TIMING", "1")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import hmsc_amd as H  # noqa: E402
from hmsc_amd.sampler import comm_unique_id  # noqa: E402


def timed(ch, it, n, record, keep=True):
    t0 = time.perf_counter()
    rec = ch.run(transient=0 if record else n, samples=n if record else 0, thin=1, adaptNf=[0], iter0=it, record=record)
    if not keep:
        del rec  # (freed inside the bracket: the record's pages unmapped there)
    ch.sync()
    t = time.perf_counter() - t0
    rec = None
    return t


def main():
    sys.argv = [sys.argv[0], "--no-cpu"]
    args = bench.parse()
    hM = bench.synthetic_probit(ny=args.ny, ns=args.ns, nc=args.nc, nf=args.nf)
    for sharded in (True, False):
        kw = dict(rank=0, nranks=1, comm_id=comm_unique_id()) if sharded else {}
        ch = H.Chain(hM, 1234567, device=0, updater={"GammaEta": False}, **kw)
        ch.init([args.nf])
        ch.run(transient=0, samples=1, thin=1, adaptNf=[0], record=True)
        ch.prepare_graphs(2)
        it = 2
        t_w = time.perf_counter()
        while time.perf_counter() - t_w < 1.0:
            ch.run(transient=0, samples=40, thin=1, adaptNf=[0], iter0=it, record=True)
            ch.sync()
            it += 40
        for n, rec, keep in ((200, True, False), (200, True, True), (1000, True, True), (200, False, True),
                             (1000, False, True)):
            print(f"[diag] {'sharded' if sharded else 'unsharded'} {n} {'rec' if rec else 'norec'}", file=sys.stderr, flush=True)
            t = timed(ch, it, n, rec, keep)
            it += n
            print(f"{'sharded' if sharded else 'unsharded'} n={n} record={rec} kept={keep}: {1e6 * t / n:.1f} us/sweep "
                  f"({n / t:.0f} sweeps/s)", flush=True)
        ch.close()


if __name__ == "__main__":
    main()
