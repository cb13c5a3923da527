"""``sampleMcmc`` — host mirror of R/sampleMcmc.R:68-372 over the MI355X sampler.

The R-side logic the reference keeps around its sweep loop stays here (argument
checks, per-chain ``initSeed``, updater auto-disable, ``combineParameters``
back-transform, ``alignPosterior`` x5, hM bookkeeping); the sweep loop itself
(:219-325) runs on the GPU through the C ABI (``Chain``).  Independent chains
run one per GPU, concurrently (threads; the C calls release the GIL), which is
the MI355X form of the reference's PSOCK chain farm (:329-345).
"""
import ctypes as C
import math
import threading
import warnings

import numpy as np

from . import _lib as L
from .model import Hmsc


def _r_bool_on(updater, name):
    """R: ``!identical(updater$NAME, FALSE)`` (only a literal FALSE disables)."""
    v = (updater or {}).get(name, None)
    return not (v is False)


def _finite_int(v, cap):
    return int(min(cap, v)) if not (isinstance(v, float) and math.isinf(v)) else int(cap)


# include/hmsc_amd.h spatialMethod codes.  'Full' levels reach the device as their
# coordinates (or distances), from which the library builds the alphapw grid of dense prior
# precisions; 'NNGP' as coordinates + nNeighbours, kept in the sparse Vecchia form (per grid
# point the k neighbour weights and conditional variances, spatial.hip setup_nngp_level);
# 'GPP' as R's low-rank predictive-process arrays (hmsc_amd/dataparams.py)
SPATIAL_CODE = {"Full": 1, "NNGP": 2, "GPP": 3}


def x_unit_order(hM, r, rl):
    """rL$x in the unit order of Eta (levels(dfPi[,r])): R indexes it by unit name,
    rL$x[as.character(dfPi[,r]), k] (R/updateZ.R:27); unnamed rows are taken in that order."""
    x = np.asarray(rl.x, dtype=np.float64)
    names = [str(i) for i in rl.x.index] if hasattr(rl.x, "index") else None
    from .model import _factor_levels
    levels = _factor_levels(hM.dfPi[hM.rLNames[r]])
    if names is None:
        if x.shape[0] != len(levels):
            raise ValueError(f"level {hM.rLNames[r]}: xData has {x.shape[0]} rows for {len(levels)} units; "
                             f"give it as a DataFrame whose index names the units")
        return x
    pos = {n: k for k, n in enumerate(names)}
    missing = [lv for lv in levels if str(lv) not in pos]
    if missing:
        raise ValueError(f"level {hM.rLNames[r]}: no xData rows for units {missing[:5]}")
    return x[[pos[str(lv)] for lv in levels]]


def level_lran(eta, lam, rows, x=None):
    """LRan of one level for the rows' units (0-based): Eta[Pi,] %*% Lambda, or for a
    covariate-dependent level sum_k (Eta[Pi,] * x[Pi, k]) %*% Lambda[,,k] (R/updateZ.R:24-29,
    R/computeWAIC.R:66-70, R/predict.R:171-176); x in the units' order of eta."""
    lam = np.asarray(lam)
    if lam.ndim == 2:
        return eta[rows] @ lam
    return sum((eta[rows] * x[rows, k:k + 1]) @ lam[:, :, k] for k in range(lam.shape[2]))


class LevelMap:
    """R's random levels -> the device levels of the C ABI.  A covariate-dependent level
    (rL$xDim = ncr > 0) is ncr consecutive device levels sharing its units and Eta, device level
    k scaling its XEta columns by rL$x[, k] and holding Lambda[,,k], Psi[,,k], Delta[,k]
    (include/hmsc_amd.h etaShare / xScale); every other level is one device level."""

    def __init__(self, hM):
        self.groups, self.xdim = [], []
        d = 0
        for rl in hM.rL or []:
            xd = int(rl.xDim or 0)
            n = max(xd, 1)
            self.groups.append(list(range(d, d + n)))
            self.xdim.append(xd)
            d += n
        self.ndev = d
        if d > L.MAX_LEVELS:
            raise ValueError(f"this build holds at most {L.MAX_LEVELS} device levels (a covariate-dependent level "
                             f"counts one per column of xData); the model needs {d}")
        self.owner = [r for r, g in enumerate(self.groups) for _ in g]     # device level -> R level
        self.col = [k for g in self.groups for k in range(len(g))]         # device level -> column of rL$x

    def expand(self, per_level):
        """A per-R-level list -> per device level."""
        return [per_level[self.owner[d]] for d in range(self.ndev)]


def _prior_k(rl, name, k):
    v = np.atleast_1d(np.asarray(rl[name], dtype=np.float64))
    return float(v[k] if v.size > 1 else v[0])


class ModelBuffers:
    """Column-major copies of the hM fields the sampler consumes (the marshalling the
    R ``.Call`` shim would do), kept alive for the lifetime of the C struct."""

    def __init__(self, hM, spatial_grid="device"):
        """spatial_grid: "device" hands 'Full' levels' coordinates / distances to the library,
        which builds the alphapw grid on the GPU; "host" passes computeDataParameters'
        arrays (hmsc_amd/dataparams.py) as R's shim could."""
        if spatial_grid not in ("device", "host"):
            raise ValueError("spatial_grid must be 'device' or 'host'")
        for rl in hM.rL or []:
            if rl.sDim and rl.spatialMethod not in SPATIAL_CODE:
                raise ValueError(f"unknown spatialMethod {rl.spatialMethod!r}")
            if rl.xDim and rl.sDim:
                raise ValueError("a covariate-dependent level cannot also be spatial here (the spatial branches "
                                 "of R/updateEta.R take Lambda as a matrix)")
        self.lm = lm = LevelMap(hM)
        self.keep = []
        k = self.keep
        m = L.hmsc_model()
        m.ny, m.ns, m.nc, m.nt, m.nr = hM.ny, hM.ns, hM.nc, hM.nt, lm.ndev
        m.Y = L.colmajor_ptr(hM.YScaled, k)
        m.Yraw = L.colmajor_ptr(hM.Y, k)
        m.X = L.colmajor_ptr(hM.XScaled, k)
        m.Tr = L.colmajor_ptr(hM.TrScaled, k)
        m.Pi = L.colmajor_ptr(hM.Pi[:, lm.owner] if hM.nr else np.zeros((hM.ny, 1)), k, np.int32)
        m.np = L.colmajor_ptr([int(hM.np[r]) for r in lm.owner] if hM.nr else [0], k, np.int32)
        m.distr = L.colmajor_ptr(hM.distr, k, np.int32)
        m.V0 = L.colmajor_ptr(hM.V0, k)
        m.f0 = float(hM.f0)
        m.mGamma = L.colmajor_ptr(hM.mGamma, k)
        m.UGamma = L.colmajor_ptr(hM.UGamma, k)
        m.aSigma = L.colmajor_ptr(hM.aSigma, k)
        m.bSigma = L.colmajor_ptr(hM.bSigma, k)
        rl = hM.rL or []
        # priors per device level: column k of a covariate-dependent level takes entry k of
        # rL$nu / a1 / b1 / a2 / b2 (R/setPriors.HmscRandomLevel.R:21-80)
        vec = lambda name: L.colmajor_ptr([_prior_k(rl[lm.owner[d]], name, lm.col[d])  # noqa: E731
                                           for d in range(lm.ndev)] or [0.0], k)
        m.nu, m.a1, m.b1, m.a2, m.b2 = vec("nu"), vec("a1"), vec("b1"), vec("a2"), vec("b2")
        self.nfMax = [_finite_int(r.nfMax, hM.ns) for r in rl]
        self.nfMin = [int(r.nfMin) for r in rl]
        m.nfMin = L.colmajor_ptr(lm.expand(self.nfMin) or [0], k, np.int32)
        m.nfMax = L.colmajor_ptr(lm.expand(self.nfMax) or [0], k, np.int32)
        if any(lm.xdim):
            m.etaShare = L.colmajor_ptr([lm.groups[lm.owner[d]][0] for d in range(lm.ndev)], k, np.int32)
            for r, g in enumerate(lm.groups):
                if lm.xdim[r]:
                    x = x_unit_order(hM, r, rl[r])
                    for kk, d in enumerate(g):
                        m.xScale[d] = L.colmajor_ptr(np.ascontiguousarray(x[:, kk]), k)
        sdim = [(r.s.shape[1] if r.s is not None else 1) if r.sDim else 0 for r in rl]
        m.sDim = L.colmajor_ptr(lm.expand(sdim) or [0], k, np.int32)
        m.spatialMethod = L.colmajor_ptr(lm.expand([SPATIAL_CODE[r.spatialMethod] if r.sDim else 0 for r in rl]) or [0],
                                         k, np.int32)
        dev = lambda r: lm.groups[r][0]  # noqa: E731  (the device level of a spatial R level)
        if any(sdim):
            # computeDataParameters' alphapw grid (R/computeDataParameters.R:53-81); the R shim
            # would pass dataParList$rLPar[[r]]$iWg / RiWg / detWg
            from .dataparams import _level_order, spatialDataParameters
            # 'Full' (spatial_grid="device") and 'NNGP' levels hand over their coordinates: the
            # library builds the Full grid on the device and the NNGP Vecchia factor itself
            on_device = [bool(lv.sDim) and ((spatial_grid == "device" and lv.spatialMethod == "Full")
                                            or lv.spatialMethod == "NNGP") for lv in rl]
            rlp = spatialDataParameters(hM, skip=on_device, gpp_dense=False)
            m.nNeighbours = L.colmajor_ptr(lm.expand([int(lv.nNeighbours or 10) if lv.sDim and lv.spatialMethod == "NNGP"
                                                      else 0 for lv in rl]), k, np.int32)
            m.nalpha = L.colmajor_ptr(lm.expand([r.alphapw.shape[0] if r.sDim else 0 for r in rl]), k, np.int32)
            m.nKnots = L.colmajor_ptr(lm.expand([rlp[r]["Fg"].shape[0] if lv.sDim and lv.spatialMethod == "GPP" else 0
                                                 for r, lv in enumerate(rl)]), k, np.int32)
            for r, lv in enumerate(rl):
                if not lv.sDim:
                    continue
                m.alphapw[dev(r)] = L.colmajor_ptr(np.asarray(lv.alphapw, dtype=np.float64), k)
                if on_device[r]:
                    idx = _level_order(hM, r, lv)
                    if lv.spatialMethod == "NNGP" and lv.distMat is not None:
                        raise ValueError("computeDataParameters: Nearest neighbours not available for distance matrices")
                    if lv.distMat is None:
                        m.sCoord[dev(r)] = L.colmajor_ptr(np.asarray(lv.s, dtype=np.float64)[idx], k)
                    else:
                        m.distMat[dev(r)] = L.colmajor_ptr(lv.distMat[np.ix_(idx, idx)], k)
                elif lv.spatialMethod == "GPP":  # R's low-rank arrays (include/hmsc_amd.h)
                    for f in ("idDg", "idDW12g", "Fg", "iFg", "detDg"):
                        getattr(m, f)[dev(r)] = L.colmajor_ptr(rlp[r][f], k)
                else:
                    m.iWg[dev(r)] = L.colmajor_ptr(rlp[r]["iWg"], k)
                    m.RiWg[dev(r)] = L.colmajor_ptr(rlp[r]["RiWg"], k)
                    m.detWg[dev(r)] = L.colmajor_ptr(rlp[r]["detWg"], k)
        m.xDim = L.colmajor_ptr([0] * max(1, lm.ndev), k, np.int32)
        m.C = None
        if hM.C is not None:
            # computeDataParameters' rho grid in spectral form (include/hmsc_amd.h): the
            # R shim would pass eigen(hM$C, symmetric=TRUE)
            Cm = np.asarray(hM.C, dtype=np.float64)
            d, U = np.linalg.eigh(Cm)
            rhopw = np.asarray(hM.rhopw, dtype=np.float64)
            m.C = L.colmajor_ptr(Cm, k)
            m.nrho = rhopw.shape[0]
            m.rhopw = L.colmajor_ptr(rhopw, k)
            m.C_vectors = L.colmajor_ptr(U, k)
            m.C_values = L.colmajor_ptr(d, k)
        self.struct = m


def updater_mask(updater):
    mask = 0
    for name, bit in L.UP.items():
        if _r_bool_on(updater, name):
            mask |= bit
    return mask


def shard_range(ns, rank, nranks):
    """(sp0, nsl): the species block of `rank` in a species-sharded chain (hmsc_shard_range,
    the one formula the C library also uses)."""
    a = np.zeros(1, dtype=np.int32)
    b = np.zeros(1, dtype=np.int32)
    L.check(L.lib().hmsc_shard_range(int(ns), int(rank), int(nranks), L.iptr(a), L.iptr(b)))
    return int(a[0]), int(b[0])


def comm_unique_id():
    """A fresh RCCL unique id (hmsc_comm_unique_id, 128 bytes): one rank creates it and every
    rank of a species-sharded chain passes it to Chain(..., comm_id=...)."""
    buf = np.zeros(128, dtype=np.uint8)
    L.check(L.lib().hmsc_comm_unique_id(buf.ctypes.data))
    return bytes(buf)


class Chain:
    """One chain's device-resident state (hmsc_create ... hmsc_destroy)."""

    def __init__(self, hM, seed, device=0, updater=None, rank=0, nranks=1, comm_id=None, mask=None,
                 host_allreduce=None, spatial_grid="device", nf_capacity="warn"):
        """A species-sharded chain (rank of nranks, two all-reduces per sweep) is created when
        comm_id (an RCCL unique id, hmsc_comm_unique_id) or host_allreduce is given -- also at
        nranks = 1, where it runs the sharded kernels and collectives on one GPU.
        host_allreduce: a callable f(x) that replaces the float64 array x by its sum over all
        ranks, in place (hmsc_create_sharded_host; RCCL is not used).
        spatial_grid: where a 'Full' level's alphapw grid is evaluated (ModelBuffers).
        nf_capacity: what to do when a level's nfMax exceeds what the device holds (K = nc +
        sum(nf) <= 128, hmsc_get_nf_cap): "warn" (hold nfMax at the capacity; the chain stops
        with an error only if updateNf must grow a level past it), "error" (refuse the model
        here) or "ignore" (hold it at the capacity silently)."""
        if nf_capacity not in ("warn", "error", "ignore"):
            raise ValueError("nf_capacity must be 'warn', 'error' or 'ignore'")
        self.hM = hM
        self.lib = L.lib()
        self.buf = ModelBuffers(hM, spatial_grid=spatial_grid)
        self.mask = updater_mask(updater) if mask is None else mask
        h = C.c_void_p()
        if nranks > 1 and host_allreduce is None and comm_id is None:
            raise ValueError("a species-sharded chain needs comm_id (RCCL) or host_allreduce")
        if host_allreduce is not None:
            def _cb(ptr, n, ctx):
                try:
                    host_allreduce(np.ctypeslib.as_array(ptr, shape=(int(n),)))
                    return 0
                except Exception:  # reported by the library as a failed callback
                    return -1
            self._ar_cb = L.ALLREDUCE_FN(_cb)
            L.check(self.lib.hmsc_create_sharded_host(C.byref(self.buf.struct), C.c_uint64(int(seed)), device,
                                                      self.mask, rank, nranks, self._ar_cb, None, C.byref(h)))
        elif comm_id is not None:
            cid = C.create_string_buffer(bytes(comm_id), 128)
            L.check(self.lib.hmsc_create_sharded(C.byref(self.buf.struct), C.c_uint64(int(seed)), device,
                                                 self.mask, rank, nranks, cid, C.byref(h)))
        else:
            L.check(self.lib.hmsc_create(C.byref(self.buf.struct), C.c_uint64(int(seed)), device, self.mask,
                                         C.byref(h)))
        self.h = h
        self.lm = lm = self.buf.lm
        self.rank, self.nranks = rank, nranks
        self.sp0, self.nsl = shard_range(hM.ns, rank, nranks)
        dmax = lm.expand(self.buf.nfMax)
        cap = np.array(dmax + [0] * (L.MAX_LEVELS - len(dmax)), dtype=np.int32)
        if hasattr(self.lib, "hmsc_get_nf_cap"):  # (a pre-round-4 library strides records by nfMax)
            L.check(self.lib.hmsc_get_nf_cap(self.h, L.iptr(cap)))
        # factors each level's device buffers and record slots hold (K = nc + sum(nf) <= 128; the
        # capacity past every level's nfMin is shared between the levels)
        self.nf_cap_dev = [int(c) for c in cap[: lm.ndev]]
        self.nf_cap = [self.nf_cap_dev[g[0]] for g in lm.groups]
        short = [(r, self.buf.nfMax[r], c) for r, c in enumerate(self.nf_cap) if c < self.buf.nfMax[r]]
        if short:
            msg = ("nfMax " + ", ".join(f"{m} of level {r + 1} held as {c}" for r, m, c in short) +
                   ": this build holds K = nc + sum(nf) <= 128 latent dimensions")
            if nf_capacity == "error":
                self.close()
                raise ValueError(msg + "; set nfMax with setPriors (or pass nf_capacity='warn')")
            if nf_capacity == "warn" and rank == 0:
                import warnings
                warnings.warn(msg + "; the chain stops with an error only if updateNf must grow a level past "
                              "that", stacklevel=2)

    def close(self):
        if self.h:
            self.lib.hmsc_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- state
    def init(self, nf0=None):
        arr = None if nf0 is None else L.i32(self.lm.expand(list(nf0)))
        L.check(self.lib.hmsc_init_state(self.h, L.iptr(arr)))

    def init_z(self):
        """Z = updateZ(Y = hM$Y, ...) at the current state (R/computeInitialParameters.R:254)."""
        L.check(self.lib.hmsc_init_z(self.h))

    def nf(self):
        out = np.zeros(L.MAX_LEVELS, dtype=np.int32)
        L.check(self.lib.hmsc_get_nf(self.h, L.iptr(out)))
        return np.array([out[g[0]] for g in self.lm.groups], dtype=np.int32)

    def get_state(self, with_z=True):
        hM = self.hM
        nf = self.nf()
        ns = self.nsl
        st = dict(Gamma=np.zeros(hM.nc * hM.nt), iV=np.zeros(hM.nc * hM.nc), Beta=np.zeros(hM.nc * ns),
                  iSigma=np.zeros(ns))
        if with_z:
            st["Z"] = np.zeros(hM.ny * ns)
        p = L.hmsc_params()
        for key in st:
            setattr(p, key, L.fptr(st[key]))
        lm = self.lm
        lv = {f: [] for f in ("Eta", "Lambda", "Psi", "Delta", "Alpha")}
        for d in range(lm.ndev):
            r = lm.owner[d]
            lv["Eta"].append(np.zeros(int(hM.np[r]) * nf[r]))
            lv["Lambda"].append(np.zeros(nf[r] * ns))
            lv["Psi"].append(np.zeros(nf[r] * ns))
            lv["Delta"].append(np.zeros(nf[r]))
            lv["Alpha"].append(np.zeros(nf[r], dtype=np.int32))
            p.Eta[d] = L.fptr(lv["Eta"][d])
            p.Lambda[d] = L.fptr(lv["Lambda"][d])
            p.Psi[d] = L.fptr(lv["Psi"][d])
            p.Delta[d] = L.fptr(lv["Delta"][d])
            p.Alpha[d] = L.iptr(lv["Alpha"][d])
        L.check(self.lib.hmsc_get_state(self.h, C.byref(p)))
        out = dict(Gamma=st["Gamma"].reshape(hM.nc, hM.nt, order="F"),
                   iV=st["iV"].reshape(hM.nc, hM.nc, order="F"),
                   Beta=st["Beta"].reshape(hM.nc, ns, order="F"), iSigma=st["iSigma"], rho=int(p.rho))
        if with_z:
            out["Z"] = st["Z"].reshape(hM.ny, ns, order="F")
        def grp(f, r, shape):  # R's matrix, or for a covariate-dependent level the nf x ns x ncr array
            parts = [lv[f][d].reshape(shape, order="F") for d in lm.groups[r]]
            return np.stack(parts, axis=-1) if lm.xdim[r] else parts[0]
        g0 = [g[0] for g in lm.groups]
        out["Eta"] = [lv["Eta"][g0[r]].reshape(int(hM.np[r]), nf[r], order="F") for r in range(hM.nr)]
        out["Lambda"] = [grp("Lambda", r, (nf[r], ns)) for r in range(hM.nr)]
        out["Psi"] = [grp("Psi", r, (nf[r], ns)) for r in range(hM.nr)]
        out["Delta"] = [grp("Delta", r, (nf[r],)) for r in range(hM.nr)]
        out["Alpha"] = [lv["Alpha"][g0[r]].astype(np.int64) for r in range(hM.nr)]
        return out

    def set_state(self, st):
        """initPar-style override: any subset of Gamma, iV (or V), Beta, iSigma (or sigma),
        Eta, Lambda, Psi, Delta, Z (R/computeInitialParameters.R:82-227)."""
        hM = self.hM
        keep = []
        p = L.hmsc_params()
        st = dict(st)
        if "V" in st and "iV" not in st:
            st["iV"] = np.linalg.inv(st["V"])
        if "sigma" in st and "iSigma" not in st:
            st["iSigma"] = 1.0 / np.asarray(st["sigma"], dtype=np.float64)
        for key in ("Gamma", "iV", "Beta", "iSigma", "Z"):
            if st.get(key) is not None:
                setattr(p, key, L.colmajor_ptr(st[key], keep))
        if st.get("rho") is not None:
            p.rho = int(st["rho"])   # 1-based grid index, as parList$rho
        lm = self.lm
        for r in range(hM.nr):
            nf = 0
            for key in ("Eta", "Lambda", "Psi", "Delta"):
                v = st.get(key)
                if v is not None and v[r] is not None:
                    a = np.asarray(v[r], dtype=np.float64)
                    nf = a.shape[1] if key == "Eta" else a.shape[0]
                    for kk, d in enumerate(lm.groups[r]):
                        # a covariate-dependent level: slice k of Lambda / Psi (nf x ns x ncr) and
                        # column k of Delta (nf x ncr) to device level k of its group; Eta shared
                        part = a if (key == "Eta" or not lm.xdim[r]) else a[..., kk]
                        getattr(p, key)[d] = L.colmajor_ptr(part, keep)
            for d in lm.groups[r]:
                p.nf[d] = nf
            al = st.get("Alpha")
            if al is not None and al[r] is not None:   # initPar$Alpha: 1-based grid indices
                for d in lm.groups[r]:
                    p.Alpha[d] = L.colmajor_ptr(np.asarray(al[r]), keep, np.int32)
        L.check(self.lib.hmsc_set_state(self.h, C.byref(p)))

    # ---- sweeps
    def sweep(self, it, adapt=False):
        L.check(self.lib.hmsc_sweep(self.h, int(it), 1 if adapt else 0))

    def update(self, name, it):
        L.check(self.lib.hmsc_update(self.h, L.UP[name], int(it)))

    def set_noise_mode(self, mode):
        L.check(self.lib.hmsc_set_noise_mode(self.h, int(mode)))

    def sync(self):
        L.check(self.lib.hmsc_sync(self.h))

    def prepare_graphs(self, it):
        """Capture the steady-state sweep graphs now (hmsc_prepare_graphs), so a timed
        run() starts replaying at once; True when they exist afterwards."""
        built = np.zeros(1, dtype=np.int32)
        L.check(self.lib.hmsc_prepare_graphs(self.h, int(it), L.iptr(built)))
        return bool(built[0])

    PROF_IDS = dict(z=0, zl=1, betalambda=2, eta_unit=3, sweep=4, eta_spatial=5, chol=6, alpha=7, gamma_eta=8, rho=9)

    def profile(self, enable=True):
        L.check(self.lib.hmsc_profile(self.h, 1 if enable else 0))

    def profile_get(self, name):
        t = np.zeros(1)
        n = np.zeros(1, dtype=np.int32)
        L.check(self.lib.hmsc_profile_get(self.h, self.PROF_IDS[name], L.fptr(t), L.iptr(n)))
        return float(t[0]), int(n[0])

    KT_IDS = dict(z=0, eta=1, betalambda=2, bl_tail=3, gamma2=4, side_chain=5)

    def kernel_timing(self, enable=True):
        """Clear and enable (or disable) the in-kernel launch timer (hmsc_kernel_timing)."""
        L.check(self.lib.hmsc_kernel_timing(self.h, 1 if enable else 0))

    def kernel_timing_get(self, name):
        """(total microseconds, launches) of one timed kernel since kernel_timing(True)."""
        t = np.zeros(1)
        n = np.zeros(1, dtype=np.int32)
        L.check(self.lib.hmsc_kernel_timing_get(self.h, self.KT_IDS[name], L.fptr(t), L.iptr(n)))
        return float(t[0]), int(n[0])

    def debug_get(self, name, n):
        out = np.zeros(int(n))
        L.check(self.lib.hmsc_debug_get(self.h, name.encode(), L.fptr(out), int(n)))
        return out

    def debug_poison(self, what):
        """Test hook (hmsc_debug_poison): corrupt one in-launch handshake ("trsv_ticket",
        "chol_publish") so the next launch using it must time out and report."""
        L.check(self.lib.hmsc_debug_poison(self.h, what.encode()))

    def run(self, transient, samples, thin=1, adaptNf=None, iter0=0, verbose=0, chain=1, record=True, fields=None):
        """hmsc_run: the device sweep loop with recording; returns the raw record arrays.
        fields: record only these (e.g. ("Beta",)); None records everything."""
        hM = self.hM
        lm = self.lm
        nr = hM.nr
        nd = lm.ndev
        ns = self.nsl
        nfMax = self.nf_cap_dev   # record slots are strided by the device's per-level factor capacity
        if adaptNf is not None and nr:
            a = list(adaptNf)
            a = a + [a[-1]] * (nr - len(a))
            adapt = L.i32(lm.expand(a))
        else:
            adapt = L.i32([transient] * max(1, nd))
        rec = None
        arrays = None
        if record and samples > 0:
            S = samples
            want = (lambda k: True) if fields is None else (lambda k: k in fields)  # noqa: E731
            # the library writes every element of a recorded field (and first touches its pages
            # in its unpack threads), so recorded fields need no zero fill: np.zeros of a large
            # array reused from the heap is a full memset on this thread (~2 ms per 16 MB)
            new = lambda k, shape, dt=np.float64: (np.empty if want(k) else np.zeros)(shape, dtype=dt)  # noqa: E731
            arrays = dict(Beta=new("Beta", (S, ns, hM.nc)), Gamma=new("Gamma", (S, hM.nt, hM.nc)),
                          iV=new("iV", (S, hM.nc, hM.nc)), iSigma=new("iSigma", (S, ns)),
                          rho=new("rho", S, np.int32), rec_nf=np.zeros((max(1, nd), S), dtype=np.int32))
            rec = L.hmsc_record()
            # (the arrays are held in `arrays` across the call: pointers that do not hold them)
            for k, fp in (("Beta", L.fptr_held), ("Gamma", L.fptr_held), ("iV", L.fptr_held), ("iSigma", L.fptr_held),
                          ("rho", L.iptr_held)):
                if want(k):
                    setattr(rec, k, fp(arrays[k]))
            rec.rec_nf = L.iptr_held(arrays["rec_nf"])
            for d in range(nd):
                nfm, r = nfMax[d], lm.owner[d]
                for k, shape, dt in (("Eta", (S, nfm, int(hM.np[r])), np.float64), ("Lambda", (S, ns, nfm), np.float64),
                                     ("Psi", (S, ns, nfm), np.float64), ("Delta", (S, nfm), np.float64),
                                     ("Alpha", (S, nfm), np.int32)):
                    if k in ("Eta", "Alpha") and d != lm.groups[r][0]:
                        continue  # (shared by a covariate-dependent level's device levels)
                    if want(k):
                        arrays[f"{k}{d}"] = np.empty(shape, dtype=dt)
                        getattr(rec, k)[d] = (L.iptr_held if dt == np.int32 else L.fptr_held)(arrays[f"{k}{d}"])
        L.check(self.lib.hmsc_run_verbose(self.h, int(transient), int(samples), int(thin), L.iptr(adapt),
                                          int(iter0), int(verbose), int(chain),
                                          C.byref(rec) if rec is not None else None))
        if arrays is None:
            return None
        # C buffers were written column-major per sample: view them in R orientation
        out = dict(Beta=arrays["Beta"].transpose(0, 2, 1), Gamma=arrays["Gamma"].transpose(0, 2, 1),
                   iV=arrays["iV"].transpose(0, 2, 1), iSigma=arrays["iSigma"], rho=arrays["rho"],
                   nf=arrays["rec_nf"][[g[0] for g in lm.groups]] if nr else arrays["rec_nf"][:0])
        for r in range(nr):
            g = lm.groups[r]
            # a covariate-dependent level: Lambda / Psi as (S, nf, ns, ncr), Delta as (S, nf, ncr)
            for k in ("Lambda", "Psi"):
                if f"{k}{g[0]}" in arrays:
                    parts = [arrays[f"{k}{d}"].transpose(0, 2, 1) for d in g]
                    out[f"{k}{r}"] = np.stack(parts, axis=-1) if lm.xdim[r] else parts[0]
            if f"Delta{g[0]}" in arrays:
                parts = [arrays[f"Delta{d}"] for d in g]
                out[f"Delta{r}"] = np.stack(parts, axis=-1) if lm.xdim[r] else parts[0]
            if f"Eta{g[0]}" in arrays:
                out[f"Eta{r}"] = arrays[f"Eta{g[0]}"].transpose(0, 2, 1)
            if f"Alpha{g[0]}" in arrays:
                out[f"Alpha{r}"] = arrays[f"Alpha{g[0]}"].astype(np.int64)
        return out


# ---------------------------------------------------------------------------
# combineParameters — R/combineParameters.R:1-58, vectorised over samples
# ---------------------------------------------------------------------------
def combine_parameters(rec, hM):
    Beta = rec["Beta"].copy()
    Gamma = rec["Gamma"].copy()
    iV = rec["iV"].copy()
    TrI = None if hM.TrInterceptInd is None else hM.TrInterceptInd - 1
    XI = None if hM.XInterceptInd is None else hM.XInterceptInd - 1
    for p in range(hM.nt):                                           # :2-10
        m, s = hM.TrScalePar[0, p], hM.TrScalePar[1, p]
        if m != 0 or s != 1:
            Gamma[:, :, p] = Gamma[:, :, p] / s
            if TrI is not None:
                Gamma[:, :, TrI] = Gamma[:, :, TrI] - m * Gamma[:, :, p]
    for k in range(hM.ncNRRR):                                       # :12-26
        m, s = hM.XScalePar[0, k], hM.XScalePar[1, k]
        if m != 0 or s != 1:
            Beta[:, k, :] = Beta[:, k, :] / s
            Gamma[:, k, :] = Gamma[:, k, :] / s
            if XI is not None:
                Beta[:, XI, :] = Beta[:, XI, :] - m * Beta[:, k, :]
                Gamma[:, XI, :] = Gamma[:, XI, :] - m * Gamma[:, k, :]
            iV[:, k, :] = iV[:, k, :] * s
            iV[:, :, k] = iV[:, :, k] * s
    V = np.linalg.inv(iV)                                            # :53 chol2inv(chol(iV))
    V = 0.5 * (V + V.transpose(0, 2, 1))
    sigma = 1.0 / rec["iSigma"]
    rho = hM.rhopw[rec["rho"] - 1, 0]
    S = Beta.shape[0]
    post = []
    for k in range(S):
        Eta, Lambda, Psi, Delta, Alpha = [], [], [], [], []
        for r in range(hM.nr):
            nf = int(rec["nf"][r][k])
            Eta.append(rec[f"Eta{r}"][k, :, :nf])
            Lambda.append(rec[f"Lambda{r}"][k, :nf, :])
            Psi.append(rec[f"Psi{r}"][k, :nf, :])
            Delta.append(rec[f"Delta{r}"][k, :nf].reshape(nf, -1))   # nf x 1, or nf x ncr
            Alpha.append(rec[f"Alpha{r}"][k, :nf])
        post.append(dict(Beta=Beta[k], wRRR=None, Gamma=Gamma[k], V=V[k], rho=float(rho[k]), sigma=sigma[k],
                         Eta=Eta, Lambda=Lambda, Alpha=Alpha, Psi=Psi, Delta=Delta, PsiRRR=None, DeltaRRR=None))
    return post


# ---------------------------------------------------------------------------
# alignPosterior — R/alignPosterior.R:18-100 (sign alignment + nfMax padding)
# ---------------------------------------------------------------------------
def alignPosterior(hM):
    """(For a covariate-dependent level, Lambda nf x ns x ncr, R's Lambda[k,] indexing fails on
    the array; factor k's values over all species and columns, a[k,,], are what its
    ns > 1 || xDim > 1 branch evidently compares and flips.)"""
    for r in range(hM.nr):
        nfVec = [pc[0]["Lambda"][r].shape[0] for pc in hM.postList]
        nfMax = max(nfVec)
        tmpl = hM.postList[int(np.argmax(nfVec))]
        LamMean = np.mean(np.stack([s["Lambda"][r] for s in tmpl]), axis=0)          # :31-33
        xd = int(hM.rL[r].xDim or 0)
        LamMean = LamMean.reshape(LamMean.shape[0], -1)
        for cInd, cpL in enumerate(hM.postList):
            lam = np.stack([s["Lambda"][r] for s in cpL])                           # (S, nf, ns[, ncr])
            lam = lam.reshape(lam.shape[0], lam.shape[1], -1)
            nf = lam.shape[1]
            if hM.ns > 1 or xd > 1:
                a = lam - lam.mean(axis=2, keepdims=True)
                b = LamMean[:nf] - LamMean[:nf].mean(axis=1, keepdims=True)
                num = np.einsum("skj,kj->sk", a, b)
                den = np.sqrt((a ** 2).sum(axis=2) * (b ** 2).sum(axis=1)[None, :])
                sd_ok = (lam.std(axis=2) > 0) & (LamMean[:nf].std(axis=1) > 0)[None, :]
                with np.errstate(invalid="ignore", divide="ignore"):
                    sgn = np.where(sd_ok, np.sign(num / den), 0.0)                # :41-46
            else:
                sgn = np.sign(LamMean[:nf, 0])[None, :] * np.sign(lam[:, :, 0])   # :48
            for j, s in enumerate(cpL):
                flip = sgn[j] < 0
                if flip.any():                                                      # :50-56
                    fl = flip.reshape((-1,) + (1,) * (s["Lambda"][r].ndim - 1))
                    s["Lambda"][r] = np.where(fl, -s["Lambda"][r], s["Lambda"][r])
                    s["Eta"][r] = np.where(flip[None, :], -s["Eta"][r], s["Eta"][r])
                if nf < nfMax:                                                      # :57-68
                    pad = nfMax - nf
                    lsh = (pad,) + s["Lambda"][r].shape[1:]
                    s["Lambda"][r] = np.concatenate([s["Lambda"][r], np.zeros(lsh)], axis=0)
                    s["Psi"][r] = np.concatenate([s["Psi"][r], np.zeros(lsh)], axis=0)
                    s["Delta"][r] = np.vstack([s["Delta"][r], np.ones((pad, s["Delta"][r].shape[1]))])
                    s["Eta"][r] = np.hstack([s["Eta"][r], np.zeros((s["Eta"][r].shape[0], pad))])
                    if hM.rL[r].sDim:
                        s["Alpha"][r] = np.r_[s["Alpha"][r], np.ones(pad, dtype=np.int64)]
    return hM


# ---------------------------------------------------------------------------
# sampleMcmc — R/sampleMcmc.R:68-372
# ---------------------------------------------------------------------------
def sampleMcmc(hM, samples, transient=0, thin=1, initPar=None, verbose=None, adaptNf=None, nChains=1,
               nParallel=1, dataParList=None, updater=None, fromPrior=False, alignPost=True, seed=None,
               devices=None, nf_capacity="warn"):
    if not isinstance(hM, Hmsc):
        raise TypeError("sampleMcmc: hM must be an Hmsc object")
    if verbose is None:
        verbose = samples * thin / 100                                     # :69
    if adaptNf is None:
        adaptNf = [transient] * hM.nr
    if fromPrior:
        raise NotImplementedError("fromPrior=TRUE (samplePrior) is out of scope (SURVEY.md §2 row 10)")
    if nParallel > nChains:                                                # :75-78
        warnings.warn("Number of cores cannot be greater than the number of chains")
        nParallel = nChains
    if any(a > transient for a in adaptNf):                                # :79-80
        raise ValueError("transient parameter should be no less than any element of adaptNf parameter")
    updater = dict(updater or {})
    rng = np.random.default_rng(seed)
    initSeed = rng.integers(1, 2 ** 31 - 1, size=nChains)                 # :121 sample.int(.Machine$integer.max)
    EPS = 1e-6                                                            # :123-152
    nc, nt = hM.nc, hM.nt
    iUGamma = np.linalg.inv(hM.UGamma)
    if _r_bool_on(updater, "Gamma2") and np.any(np.abs(hM.mGamma) > EPS):
        updater["Gamma2"] = False
        print("Setting updater$Gamma2=FALSE due to non-zero mGamma")
    if _r_bool_on(updater, "Gamma2") and np.any(np.abs(iUGamma - np.kron(iUGamma[:nc, :nc], np.eye(nt))) > EPS):
        updater["Gamma2"] = False
        print("Setting updater$Gamma2=FALSE due to non-kronecker structure of UGamma matrix")
    if _r_bool_on(updater, "Gamma2") and hM.C is not None:
        updater["Gamma2"] = False
        print("Setting updater$Gamma2=FALSE due to specified phylogeny matrix")
    if _r_bool_on(updater, "GammaEta") and np.any(np.abs(hM.mGamma) > EPS):
        updater["GammaEta"] = False
        print("Setting updater$GammaEta=FALSE due to non-zero mGamma")
    if _r_bool_on(updater, "GammaEta") and hM.nr == 0:
        updater["GammaEta"] = False
        print("Setting updater$GammaEta=FALSE due to absence of random effects included to the model")
    ndev = np.zeros(1, dtype=np.int32)
    L.check(L.lib().hmsc_device_count(L.iptr(ndev)))
    if ndev[0] < 1:
        raise L.HmscNativeError("no MI355X device visible")
    devices = list(range(int(ndev[0]))) if devices is None else list(devices)
    nf0 = [int(rl.nfMin) for rl in hM.rL] if hM.nr else None
    if initPar is not None and initPar != "fixed effects":
        for r in range(hM.nr):
            for key in ("Delta", "Psi", "Lambda", "Eta"):
                v = initPar.get(key)
                if v is not None and v[r] is not None:
                    a = np.asarray(v[r])
                    nf0[r] = a.shape[1] if key == "Eta" else a.shape[0]
    elif initPar == "fixed effects":                                  # R/computeInitialParameters.R:52-79
        print("Hmsc::computeInitialParameter - initializing fixed effects with SSDM estimates")
        from .initpar import fixed_effects_init
        initPar = fixed_effects_init(hM)

    results = [None] * nChains
    errors = []

    def make_chain(c):
        if nChains > 1:
            print(f'[1] "Computing chain {c + 1}"')
        ch = Chain(hM, int(initSeed[c]), device=devices[c % len(devices)], updater=updater,
                   nf_capacity=nf_capacity if c == 0 else "ignore")
        try:
            ch.init(nf0)
            if initPar is not None:
                ch.set_state(initPar)
                ch.init_z()        # the reference draws Z last, from the initPar state (:229-254)
        except BaseException:
            ch.close()
            raise
        return ch

    def run_chain(c, ch):                                                  # :155-327
        try:
            rec = ch.run(transient, samples, thin, adaptNf, verbose=int(verbose) if verbose else 0, chain=c + 1)
            results[c] = combine_parameters(rec, hM)
        except Exception as e:  # surface in the caller thread
            errors.append(e)

    # Chains are created, initialised and destroyed on this thread (device allocation and
    # synchronisation), and only their sweep loops run concurrently, nParallel at a time.
    for start in range(0, nChains, max(1, nParallel)):
        idx = list(range(start, min(nChains, start + max(1, nParallel))))
        chains = []
        try:
            for c in idx:   # built one at a time: a failure still closes the ones already made
                chains.append(make_chain(c))
            if len(idx) > 1:
                th = [threading.Thread(target=run_chain, args=(c, ch)) for c, ch in zip(idx, chains)]
                for t in th:
                    t.start()
                for t in th:
                    t.join()
            else:
                run_chain(idx[0], chains[0])
        finally:
            for ch in chains:
                ch.close()
        if errors:
            break
    if errors:
        raise errors[0]
    hM.postList = results
    hM.repList = [None] * nChains
    hM.samples, hM.transient, hM.thin, hM.verbose = samples, transient, thin, verbose   # :360-364
    hM.adaptNf = list(adaptNf)
    if alignPost:
        for _ in range(5):                                                 # :365-369
            hM = alignPosterior(hM)
    return hM
