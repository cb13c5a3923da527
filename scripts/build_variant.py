"""Build an A/B variant of the library: the given sources recompiled with extra flags (e.g.
-DZ_MIN_BLOCKS=3), linked with the in-tree objects of the rest, as hmsc_amd/libab_<name>.so
(select it with HMSC_AMD_LIB; scripts/ab_lib.sh).  usage:
    python scripts/build_variant.py NAME SRC[,SRC...] FLAG [FLAG ...]"""
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hmsc_amd import build as B  # noqa: E402


def main():
    name, srcs, flags = sys.argv[1], sys.argv[2].split(","), sys.argv[3:]
    B.build(verbose=False)
    objs = []
    for src in B.SOURCES:
        base = os.path.splitext(src)[0]
        if src in srcs:
            obj = os.path.join(B.CSRC, f"{base}_ab_{name}.o")
            cmd = [B.HIPCC] + B.FLAGS + B.EXTRA.get(src, []) + flags + ["-x", "hip", "-c", os.path.join(B.CSRC, src), "-o", obj]
            print(" ".join(cmd), flush=True)
            subprocess.check_call(cmd)
        else:
            obj = os.path.join(B.CSRC, base + ".o")
        objs.append(obj)
    lib = os.path.join(B.HERE, f"libab_{name}.so")
    subprocess.check_call([B.HIPCC, "-shared", "-fPIC", f"--offload-arch={B.ARCH}", "-o", lib] + objs +
                          ["-pthread", "-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"])
    print(lib)


if __name__ == "__main__":
    main()
