"""ctypes binding of the C ABI in ``include/hmsc_amd.h`` (``hmsc_amd/libhmsc_amd.so``).

This is the binding a maintainer would write on the R side as a ``.Call`` shim
(INTEGRATION.md); here Python plays the role of the R wrapper.  There is no CPU
fallback: if the HIP library is missing, importing the sampler raises.
"""
import ctypes as C
import os

import numpy as np

MAX_LEVELS = 8
HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("HMSC_AMD_LIB", os.path.join(HERE, "libhmsc_amd.so"))

UP = dict(Gamma2=1 << 0, GammaEta=1 << 1, BetaLambda=1 << 2, wRRR=1 << 3, BetaSel=1 << 4, GammaV=1 << 5,
          Rho=1 << 6, LambdaPriors=1 << 7, wRRRPriors=1 << 8, Eta=1 << 9, Alpha=1 << 10, InvSigma=1 << 11,
          Z=1 << 12)
UP_ALL = 0x1FFF

dp = C.POINTER(C.c_double)
ip = C.POINTER(C.c_int32)


class hmsc_model(C.Structure):
    _fields_ = [("struct_size", C.c_int32),
                ("ny", C.c_int32), ("ns", C.c_int32), ("nc", C.c_int32), ("nt", C.c_int32), ("nr", C.c_int32),
                ("Y", dp), ("Yraw", dp), ("X", dp), ("Tr", dp), ("Pi", ip), ("np", ip), ("distr", ip),
                ("V0", dp), ("f0", C.c_double), ("mGamma", dp), ("UGamma", dp), ("aSigma", dp), ("bSigma", dp),
                ("nu", dp), ("a1", dp), ("b1", dp), ("a2", dp), ("b2", dp), ("nfMin", ip), ("nfMax", ip),
                ("sDim", ip), ("xDim", ip), ("C", dp), ("nrho", C.c_int32), ("rhopw", dp),
                ("C_vectors", dp), ("C_values", dp),
                ("spatialMethod", ip), ("nalpha", ip), ("alphapw", dp * MAX_LEVELS), ("iWg", dp * MAX_LEVELS),
                ("RiWg", dp * MAX_LEVELS), ("detWg", dp * MAX_LEVELS),
                ("sCoord", dp * MAX_LEVELS), ("distMat", dp * MAX_LEVELS),
                ("nKnots", ip), ("idDg", dp * MAX_LEVELS), ("idDW12g", dp * MAX_LEVELS), ("Fg", dp * MAX_LEVELS),
                ("iFg", dp * MAX_LEVELS), ("detDg", dp * MAX_LEVELS), ("nNeighbours", ip),
                ("etaShare", ip), ("xScale", dp * MAX_LEVELS)]

    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        self.struct_size = C.sizeof(hmsc_model)   # hmsc_create checks it (include/hmsc_amd.h)


class hmsc_params(C.Structure):
    _fields_ = [("Gamma", dp), ("iV", dp), ("Beta", dp), ("iSigma", dp), ("Z", dp), ("rho", C.c_int32),
                ("nf", C.c_int32 * MAX_LEVELS), ("Eta", dp * MAX_LEVELS), ("Lambda", dp * MAX_LEVELS),
                ("Psi", dp * MAX_LEVELS), ("Delta", dp * MAX_LEVELS), ("Alpha", ip * MAX_LEVELS)]


class hmsc_record(C.Structure):
    _fields_ = [("Beta", dp), ("Gamma", dp), ("iV", dp), ("iSigma", dp), ("rho", ip),
                ("Eta", dp * MAX_LEVELS), ("Lambda", dp * MAX_LEVELS), ("Psi", dp * MAX_LEVELS),
                ("Delta", dp * MAX_LEVELS), ("Alpha", ip * MAX_LEVELS), ("rec_nf", ip)]


class hmsc_predict_args(C.Structure):
    _fields_ = [("ny", C.c_int32), ("ns", C.c_int32), ("nc", C.c_int32), ("nr", C.c_int32),
                ("nsamples", C.c_int32), ("expected", C.c_int32), ("seed", C.c_uint64), ("device", C.c_int32),
                ("X", dp), ("Beta", dp), ("sigma", dp), ("family", ip), ("YScalePar", dp), ("Pi", ip),
                ("np", ip), ("nf", ip), ("Eta", dp * MAX_LEVELS), ("Lambda", dp * MAX_LEVELS)]


class hmsc_vp_args(C.Structure):
    _fields_ = [("device", C.c_int32), ("ny", C.c_int32), ("ns", C.c_int32), ("nc", C.c_int32), ("nt", C.c_int32),
                ("S", C.c_int32), ("ngroups", C.c_int32), ("nr", C.c_int32), ("group", ip), ("X", dp), ("Tr", dp),
                ("cM", dp), ("Beta", dp), ("Gamma", dp), ("nf", ip), ("nfmax", C.c_int32 * MAX_LEVELS),
                ("Lambda", dp * MAX_LEVELS)]


class HmscNativeError(RuntimeError):
    pass


_lib = None

# every symbol declared in include/hmsc_amd.h
# hmsc_allreduce_fn: int (*)(double* buf, int64_t n, void* ctx)
ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, C.POINTER(C.c_double), C.c_int64, C.c_void_p)

EXPORTS = ["hmsc_last_error", "hmsc_device_count", "hmsc_create", "hmsc_create_sharded", "hmsc_comm_unique_id",
           "hmsc_shard_range", "hmsc_create_sharded_host", "hmsc_dense_chol_solve", "hmsc_spatial_full_grid",
           "hmsc_destroy", "hmsc_init_state", "hmsc_init_z", "hmsc_set_state", "hmsc_get_state", "hmsc_get_nf", "hmsc_get_nf_cap",
           "hmsc_sweep",
           "hmsc_update", "hmsc_set_noise_mode", "hmsc_run", "hmsc_run_verbose", "hmsc_sync", "hmsc_debug_get",
           "hmsc_debug_poison",
           "hmsc_profile", "hmsc_profile_get", "hmsc_kernel_timing", "hmsc_kernel_timing_get", "hmsc_predict",
           "hmsc_prepare_graphs", "hmsc_post_omega", "hmsc_variance_partitioning", "hmsc_effective_size"]


def _check_fresh():
    """Refuse a library built from other sources than the ones beside it: build.py stamps the
    source digest next to the library (``libhmsc_amd.so.src``).  Only the in-tree library is
    checked; ``HMSC_AMD_LIB`` selects another build (A/B timing) without the check, and
    ``HMSC_AMD_ALLOW_STALE=1`` skips it."""
    if "HMSC_AMD_LIB" in os.environ or os.environ.get("HMSC_AMD_ALLOW_STALE") == "1":
        return
    from . import build as B
    stamp = LIB_PATH + ".src"
    have = open(stamp).read().strip() if os.path.exists(stamp) else None
    want = B.source_digest()
    if have != want:
        raise HmscNativeError(
            f"{LIB_PATH} is stale: " + ("no source stamp " + stamp if have is None else
                                        "built from other sources than hmsc_amd/csrc") +
            " -- rebuild it (python -m hmsc_amd.build)")


def lib():
    """Load the HIP library (raises if it has not been built: no CPU fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise HmscNativeError(
            f"{LIB_PATH} not found: build the gfx950 HIP library first (python -m hmsc_amd.build)")
    _check_fresh()
    L = C.CDLL(LIB_PATH)
    L.hmsc_last_error.restype = C.c_char_p
    L.hmsc_device_count.argtypes = [ip]
    L.hmsc_create.argtypes = [C.POINTER(hmsc_model), C.c_uint64, C.c_int32, C.c_uint32, C.POINTER(C.c_void_p)]
    L.hmsc_create_sharded.argtypes = [C.POINTER(hmsc_model), C.c_uint64, C.c_int32, C.c_uint32, C.c_int32,
                                      C.c_int32, C.c_void_p, C.POINTER(C.c_void_p)]
    L.hmsc_comm_unique_id.argtypes = [C.c_void_p]
    L.hmsc_destroy.argtypes = [C.c_void_p]
    L.hmsc_destroy.restype = None
    L.hmsc_init_state.argtypes = [C.c_void_p, ip]
    L.hmsc_init_z.argtypes = [C.c_void_p]
    L.hmsc_dense_chol_solve.argtypes = [C.c_int32, dp, C.c_int32, dp, ip]
    L.hmsc_spatial_full_grid.argtypes = [C.c_int32, C.c_int32, C.c_int32, dp, dp, C.c_int32, dp, dp, dp, dp]
    L.hmsc_shard_range.argtypes = [C.c_int32, C.c_int32, C.c_int32, ip, ip]
    L.hmsc_create_sharded_host.argtypes = [C.POINTER(hmsc_model), C.c_uint64, C.c_int32, C.c_uint32, C.c_int32,
                                           C.c_int32, ALLREDUCE_FN, C.c_void_p, C.POINTER(C.c_void_p)]
    L.hmsc_set_state.argtypes = [C.c_void_p, C.POINTER(hmsc_params)]
    L.hmsc_get_state.argtypes = [C.c_void_p, C.POINTER(hmsc_params)]
    L.hmsc_get_nf.argtypes = [C.c_void_p, ip]
    if hasattr(L, "hmsc_get_nf_cap"):  # (absent from a pre-round-4 library loaded for A/B timing)
        L.hmsc_get_nf_cap.argtypes = [C.c_void_p, ip]
    L.hmsc_sweep.argtypes = [C.c_void_p, C.c_int32, C.c_int32]
    L.hmsc_update.argtypes = [C.c_void_p, C.c_uint32, C.c_int32]
    L.hmsc_set_noise_mode.argtypes = [C.c_void_p, C.c_int32]
    L.hmsc_run.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_int32, ip, C.c_int32, C.POINTER(hmsc_record)]
    L.hmsc_run_verbose.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_int32, ip, C.c_int32, C.c_int32,
                                   C.c_int32, C.POINTER(hmsc_record)]
    L.hmsc_sync.argtypes = [C.c_void_p]
    L.hmsc_debug_get.argtypes = [C.c_void_p, C.c_char_p, dp, C.c_int64]
    if hasattr(L, "hmsc_debug_poison"):
        L.hmsc_debug_poison.argtypes = [C.c_void_p, C.c_char_p]
    L.hmsc_profile.argtypes = [C.c_void_p, C.c_int32]
    L.hmsc_profile_get.argtypes = [C.c_void_p, C.c_int32, dp, ip]
    L.hmsc_kernel_timing.argtypes = [C.c_void_p, C.c_int32]
    L.hmsc_kernel_timing_get.argtypes = [C.c_void_p, C.c_int32, dp, ip]
    L.hmsc_predict.argtypes = [C.POINTER(hmsc_predict_args), dp]
    L.hmsc_prepare_graphs.argtypes = [C.c_void_p, C.c_int32, ip]
    L.hmsc_post_omega.argtypes = [C.c_int32, C.c_int32, C.c_int32, C.c_int32, ip, dp, dp, dp, dp, dp]
    L.hmsc_variance_partitioning.argtypes = [C.POINTER(hmsc_vp_args), dp]
    L.hmsc_effective_size.argtypes = [C.c_int32, C.c_int32, C.c_int32, dp, dp, ip]
    _lib = L
    return L


def check(rc):
    if rc != 0:
        raise HmscNativeError(f"hmsc_amd error {rc}: {lib().hmsc_last_error().decode()}")


def f64(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.float64))


def i32(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.int32))


def fptr(a):
    return None if a is None else a.ctypes.data_as(dp)


def iptr(a):
    return None if a is None else a.ctypes.data_as(ip)


def fptr_held(a):
    """fptr for an array the caller keeps alive across the C call (the pointer does not hold
    it): half data_as's cost, for the record buffers of every run."""
    return C.cast(a.__array_interface__["data"][0], dp)


def iptr_held(a):
    return C.cast(a.__array_interface__["data"][0], ip)


def fortran(a, dtype=np.float64):
    """Column-major contiguous copy (R storage order)."""
    return np.asfortranarray(np.asarray(a, dtype=dtype))


def colmajor_ptr(a, keep, dtype=np.float64):
    arr = np.asarray(a, dtype=dtype)
    flat = np.ascontiguousarray(arr.reshape(-1, order="F")) if arr.ndim > 1 else np.ascontiguousarray(arr)
    keep.append(flat)
    return fptr(flat) if dtype == np.float64 else iptr(flat)
