"""Build recipe for the in-tree C-ABI library ``hmsc_amd/libhmsc_amd.so`` (gfx950).

    python -m hmsc_amd.build          # or __graft_entry__.build()

hipcc compiles the HIP kernels and the C ABI for --offload-arch=gfx950 and links
RCCL (species-sharded chains).  No CPU fallback is built: the product path needs
this library and fails loudly without it.
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libhmsc_amd.so")
SOURCES = ["kernels.hip", "phylo.hip", "gamma_eta.hip", "spatial.hip", "predict.hip", "capi.cpp"]
HEADERS = ["common.h", "rng.h", "state.h", "wave_la.h", "z_kernel.h", os.path.join("..", "..", "include", "hmsc_amd.h")]
ARCH = os.environ.get("HMSC_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["-O3", "-fPIC", "-std=c++17", "-pthread", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-function",
         "-Wno-unused-variable", "-Wno-unused-but-set-variable"]


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build(force=False, verbose=True, stamps=False):
    """stamps=True builds the diagnostic library libhmsc_amd_stamps.so (HMSC_STAMP clock
    stamps in the kernels; select it with HMSC_AMD_LIB=...)."""
    lib = LIB.replace(".so", "_stamps.so") if stamps else LIB
    flags = FLAGS + (["-DHMSC_STAMPS"] if stamps else [])
    objs = []
    hdrs = [os.path.join(CSRC, h) for h in HEADERS]
    for src in SOURCES:
        path = os.path.join(CSRC, src)
        obj = os.path.join(CSRC, os.path.splitext(src)[0] + ("_stamps.o" if stamps else ".o"))
        objs.append(obj)
        if force or _stale(obj, [path] + hdrs):
            cmd = [HIPCC] + flags + ["-x", "hip", "-c", path, "-o", obj]
            if verbose:
                print(" ".join(cmd), flush=True)
            subprocess.check_call(cmd)
    if force or _stale(lib, objs):
        cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", lib] + objs + \
              ["-pthread", "-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.check_call(cmd)
    return lib


if __name__ == "__main__":
    build(force="--force" in sys.argv, stamps="--stamps" in sys.argv)
