"""ORACLE / CPU BASELINE — test and measurement infrastructure only (never imported by the
product path).  ctypes front of oracle/cpu/hmsc_cpu.cpp (libhmsc_cpu.so): the compiled C++
restatement of the config-4-class sweep that bench.py times as its CPU baseline, chains =
cores, one thread per chain."""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "cpu", "hmsc_cpu.cpp")
LIB = os.path.join(HERE, "libhmsc_cpu.so")
CMD = ["g++", "-O3", "-march=x86-64-v3", "-fPIC", "-shared", "-pthread", SRC, "-o", LIB]
_lib = None


def build(verbose=False):
    import subprocess
    if verbose:
        print(" ".join(CMD), flush=True)
    subprocess.check_call(CMD)
    return LIB


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        _lib = C.CDLL(LIB)
        _lib.hmsc_cpu_last_error.restype = C.c_char_p
    return _lib


def _f(a):
    return np.asfortranarray(np.asarray(a, dtype=np.float64))


def run(m, seed, n_sweeps, nchains=1, iter0=0, gamma2=True):
    """m: oracle model dict (tests/helpers.oracle_model) with one non-spatial level.
    Returns (chain 0's final state dict, seconds of the sweeps over all chains)."""
    X, Y, Tr = _f(m["X"]), _f(m["Y"]), _f(m["Tr"])
    Yraw = _f(m.get("Yraw", m["Y"]))
    ny, nc = X.shape
    ns, nt = Tr.shape
    rl = m["rL"][0]
    nf = int(rl["nfMin"])
    npr = int(m["np"][0])
    Pi = np.ascontiguousarray(m["Pi"][:, 0], dtype=np.int32)
    fam = np.ascontiguousarray(m["distr"][:, 0], dtype=np.int32)
    var = np.ascontiguousarray(m["distr"][:, 1], dtype=np.int32)
    pri = np.array([m["f0"], rl["nu"], rl["a1"], rl["b1"], rl["a2"], rl["b2"]], dtype=np.float64)
    keep = [X, Y, Yraw, Tr, Pi, fam, var, pri]
    V0, UG, mG, aS, bS = (_f(m[k]) for k in ("V0", "UGamma", "mGamma", "aSigma", "bSigma"))
    keep += [V0, UG, mG, aS, bS]
    out = dict(Beta=np.zeros((nc, ns), order="F"), Gamma=np.zeros((nc, nt), order="F"),
               iV=np.zeros((nc, nc), order="F"), Lambda=np.zeros((nf, ns), order="F"),
               Eta=np.zeros((npr, nf), order="F"), Psi=np.zeros((nf, ns), order="F"), Delta=np.zeros(nf),
               Z=np.zeros((ny, ns), order="F"), iSigma=np.zeros(ns))
    sec = C.c_double(0.0)
    p = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
    L = lib()
    rc = L.hmsc_cpu_run(C.c_int(ny), C.c_int(ns), C.c_int(nc), C.c_int(nt), C.c_int(npr), C.c_int(nf),
                        p(X), p(Y), p(Yraw), p(Tr), p(Pi), p(fam), p(var), p(V0), p(UG), p(mG), p(aS), p(bS), p(pri),
                        C.c_uint64(int(seed)), C.c_int(nchains), C.c_int(n_sweeps), C.c_int(iter0),
                        C.c_int(1 if gamma2 else 0), *[p(out[k]) for k in
                                                        ("Beta", "Gamma", "iV", "Lambda", "Eta", "Psi", "Delta", "Z",
                                                         "iSigma")], C.byref(sec))
    del keep
    if rc != 0:
        raise RuntimeError("hmsc_cpu_run: " + L.hmsc_cpu_last_error().decode())
    return out, sec.value
