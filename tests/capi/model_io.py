"""Binary model files for the C-ABI shim test (tests/capi/shim_run.c).

``write_model(hM, path)`` writes the hM fields the R ``.Call`` shim of INTEGRATION.md hands
to ``hmsc_model`` -- as R holds them (column-major, NA as NaN, 1-based Pi), plus what R
computes on its side of the boundary: ``eigen(hM$C, symmetric=TRUE)`` and, per spatial
'Full' level, the unit-ordered coordinates and ``alphapw``.  Format: a sequence of
records ``int32 name_len | name | int32 kind (0 = float64, 1 = int32) | int64 n | data``.
"""
import struct

import numpy as np


def _f(a):
    return np.asfortranarray(np.asarray(a, dtype=np.float64)).ravel(order="F")


def _i(a):
    return np.asfortranarray(np.asarray(a, dtype=np.int32)).ravel(order="F")


def model_arrays(hM):
    from hmsc_amd.dataparams import _level_order
    rl = hM.rL or []
    out = {
        "dims": _i([hM.ny, hM.ns, hM.nc, hM.nt, hM.nr]),
        "Y": _f(hM.YScaled), "Yraw": _f(hM.Y), "X": _f(hM.XScaled), "Tr": _f(hM.TrScaled),
        "Pi": _i(hM.Pi if hM.nr else np.zeros((hM.ny, 1))), "np": _i(hM.np if hM.nr else [0]),
        "distr": _i(hM.distr), "V0": _f(hM.V0), "f0": _f([hM.f0]), "mGamma": _f(hM.mGamma),
        "UGamma": _f(hM.UGamma), "aSigma": _f(hM.aSigma), "bSigma": _f(hM.bSigma),
    }
    for k in ("nu", "a1", "b1", "a2", "b2"):
        out[k] = _f([float(r[k]) for r in rl] or [0.0])
    cap = lambda v: hM.ns if v == float("inf") else int(v)  # noqa: E731
    out["nfMin"] = _i([int(r.nfMin) for r in rl] or [0])
    out["nfMax"] = _i([cap(r.nfMax) for r in rl] or [0])
    out["sDim"] = _i([(r.s.shape[1] if r.s is not None else 1) if r.sDim else 0 for r in rl] or [0])
    out["spatialMethod"] = _i([{"Full": 1, "NNGP": 2, "GPP": 3}[r.spatialMethod] if r.sDim else 0 for r in rl] or [0])
    out["nalpha"] = _i([r.alphapw.shape[0] if r.sDim else 0 for r in rl] or [0])
    for r, lv in enumerate(rl):
        if lv.sDim:
            if lv.spatialMethod == "GPP" or lv.distMat is not None:
                raise NotImplementedError("the shim test marshals 'Full' / 'NNGP' levels given by coordinates")
            out[f"alphapw{r}"] = _f(lv.alphapw)
            out[f"sCoord{r}"] = _f(np.asarray(lv.s, dtype=np.float64)[_level_order(hM, r, lv)])
    if any(lv.sDim and lv.spatialMethod == "NNGP" for lv in rl):
        out["nNeighbours"] = _i([int(lv.nNeighbours or 10) if lv.sDim and lv.spatialMethod == "NNGP" else 0
                                 for lv in rl])
    if hM.C is not None:
        Cm = np.asarray(hM.C, dtype=np.float64)
        d, U = np.linalg.eigh(Cm)  # R: e = eigen(hM$C, symmetric = TRUE)
        out["C"] = _f(Cm)
        out["rhopw"] = _f(hM.rhopw)
        out["C_vectors"] = _f(U)
        out["C_values"] = _f(d)
    return out


def write_model(hM, path):
    with open(path, "wb") as f:
        for name, a in model_arrays(hM).items():
            kind = 1 if a.dtype == np.int32 else 0
            nb = name.encode()
            f.write(struct.pack("<i", len(nb)) + nb + struct.pack("<iq", kind, a.size))
            f.write(a.tobytes())


def read_results(path):
    """The shim program's output: the same record format (float64 / int32 arrays)."""
    res = {}
    with open(path, "rb") as f:
        data = f.read()
    p = 0
    while p < len(data):
        (ln,) = struct.unpack_from("<i", data, p)
        p += 4
        name = data[p:p + ln].decode()
        p += ln
        kind, n = struct.unpack_from("<iq", data, p)
        p += 12
        dt = np.int32 if kind == 1 else np.float64
        res[name] = np.frombuffer(data, dtype=dt, count=n, offset=p).copy()
        p += n * np.dtype(dt).itemsize
    return res
