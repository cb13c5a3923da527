"""Build recipe for the in-tree C-ABI library ``hmsc_amd/libhmsc_amd.so`` (gfx950).

    python -m hmsc_amd.build          # or __graft_entry__.build()

hipcc compiles the HIP kernels and the C ABI for --offload-arch=gfx950 and links
RCCL (species-sharded chains).  No CPU fallback is built: the product path needs
this library and fails loudly without it.

Staleness is decided by content, not by mtime: every object records a hash of its
source, the headers, the compiler flags and the hipcc version next to it
(``*.o.sha``), so a tree copied to another machine (whose mtimes say nothing) is
recompiled exactly when something that goes into the object differs.
"""
import hashlib
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libhmsc_amd.so")
SOURCES = ["kernels.hip", "zdraw.hip", "dense.hip", "phylo.hip", "gamma_eta.hip", "spatial.hip", "predict.hip", "post.hip",
           "capi.cpp"]
HEADERS = ["common.h", "rng.h", "state.h", "wave_la.h", "z_kernel.h", "z_tables.h", "record.h", os.path.join("..", "..", "include", "hmsc_amd.h")]
ARCH = os.environ.get("HMSC_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["-O3", "-fPIC", "-std=c++17", "-pthread", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-function",
         "-Wno-unused-variable", "-Wno-unused-but-set-variable"]
# per-source extra flags: the z kernel's inlined draw keeps its polynomial constants at their
# uses (MachineLICM would hoist ~60 f64 constants out of the site loop and spill them)
EXTRA = {"zdraw.hip": ["-mllvm", "-disable-machine-licm"]}


def _hipcc_version():
    try:
        return subprocess.run([HIPCC, "--version"], capture_output=True, text=True, timeout=60).stdout
    except Exception:  # pragma: no cover
        return "unknown"


def _digest(paths, extra):
    h = hashlib.sha256()
    for p in paths:
        with open(p, "rb") as f:
            h.update(p.encode() + b"\0" + f.read())
    h.update("\0".join(extra).encode())
    return h.hexdigest()


def source_digest():
    """Hash of the library's sources and headers (content only).  The link step writes it next
    to the library (``libhmsc_amd.so.src``) and ``_lib.lib()`` refuses a library whose stamp
    does not match the sources beside it (a stale library pushed with newer sources)."""
    paths = [os.path.join(CSRC, f) for f in SOURCES + HEADERS]
    h = hashlib.sha256()
    for p in paths:
        with open(p, "rb") as f:
            h.update(os.path.basename(p).encode() + b"\0" + f.read())
    return h.hexdigest()


def _fresh(target, digest):
    stamp = target + ".sha"
    if not (os.path.exists(target) and os.path.exists(stamp)):
        return False
    with open(stamp) as f:
        return f.read().strip() == digest


def _stamp(target, digest):
    with open(target + ".sha", "w") as f:
        f.write(digest + "\n")


def build(force=False, verbose=True, stamps=False, jobs=None):
    """stamps=True builds the diagnostic library libhmsc_amd_stamps.so (HMSC_STAMP clock
    stamps in the kernels; select it with HMSC_AMD_LIB=...)."""
    lib = LIB.replace(".so", "_stamps.so") if stamps else LIB
    flags = FLAGS + (["-DHMSC_STAMPS"] if stamps else [])
    hdrs = [os.path.join(CSRC, h) for h in HEADERS]
    ver = _hipcc_version()
    todo, objs, digests = [], [], []
    for src in SOURCES:
        path = os.path.join(CSRC, src)
        obj = os.path.join(CSRC, os.path.splitext(src)[0] + ("_stamps.o" if stamps else ".o"))
        cmd = [HIPCC] + flags + EXTRA.get(src, []) + ["-x", "hip", "-c", path, "-o", obj]
        dg = _digest([path] + hdrs, cmd + [ver])
        objs.append(obj)
        digests.append(dg)
        if force or not _fresh(obj, dg):
            todo.append((cmd, obj, dg))

    def compile_one(job):
        cmd, obj, dg = job
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.check_call(cmd)
        _stamp(obj, dg)

    with ThreadPoolExecutor(max_workers=jobs or min(8, max(1, len(todo)))) as ex:
        list(ex.map(compile_one, todo))
    link = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", lib] + objs + \
           ["-pthread", "-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"]
    ldg = hashlib.sha256(("\0".join(digests + link)).encode()).hexdigest()
    if force or todo or not _fresh(lib, ldg):
        if verbose:
            print(" ".join(link), flush=True)
        subprocess.check_call(link)
        _stamp(lib, ldg)
    with open(lib + ".src", "w") as f:
        f.write(source_digest() + "\n")
    if not stamps:
        build_shim(force=force, verbose=verbose)
    return lib


def build_shim(force=False, verbose=True):
    """tests/capi/shim_run: the INTEGRATION.md .Call shim as a plain C program, gcc against
    include/hmsc_amd.h, linked to the in-tree library (tests/test_gpu_capi_c.py)."""
    root = os.path.dirname(HERE)
    src = os.path.join(root, "tests", "capi", "shim_run.c")
    out = os.path.join(root, "tests", "capi", "shim_run")
    if not os.path.exists(src):
        return None
    cmd = ["gcc", "-std=c99", "-O2", "-Wall", "-Wextra", "-I", os.path.join(root, "include"), src, "-L", HERE,
           "-lhmsc_amd", "-Wl,-rpath,$ORIGIN/../../hmsc_amd", "-o", out]
    dg = _digest([src, os.path.join(root, "include", "hmsc_amd.h")], cmd)
    if force or not _fresh(out, dg):
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.check_call(cmd)
        _stamp(out, dg)
    return out


if __name__ == "__main__":
    build(force="--force" in sys.argv, stamps="--stamps" in sys.argv)
