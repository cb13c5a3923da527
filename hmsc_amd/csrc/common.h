// Shared helpers for the hmsc_amd HIP kernels (gfx950, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <stdexcept>
#include <string>

namespace hmsc {

// largest alphapw grid (nrow(rL$alphapw); R's default has 101 points) the device takes
// a debugging / A-B switch from the environment: set, non-empty and not "0"
inline bool getenv_flag(const char* name) {
  const char* v = getenv(name);
  return v && v[0] && v[0] != '0';
}

constexpr int HMSC_MAX_ALPHA = 2048;
// K = nc + sum(nf): the latent dimensions a chain may hold (z kernel NKB <= 8, LDS factors)
constexpr int HMSC_KCAP = 128;

struct HmscError : std::runtime_error {
  int code;
  HmscError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

#define HIP_OK(expr)                                                                         \
  do {                                                                                       \
    hipError_t _e = (expr);                                                                  \
    if (_e != hipSuccess)                                                                    \
      throw ::hmsc::HmscError(-2, std::string(#expr) + ": " + hipGetErrorString(_e) + " (" + \
                                      __FILE__ + ":" + std::to_string(__LINE__) + ")");      \
  } while (0)

#define HMSC_REQUIRE(cond, msg)                                \
  do {                                                         \
    if (!(cond)) throw ::hmsc::HmscError(-1, std::string(msg)); \
  } while (0)

constexpr int WAVE = 64;

// Philox sweep counter of a kernel-argument struct: the value passed at launch, or -- for
// launches captured into the per-sweep hipGraph -- the device word the graph advances.
#define SWEEP_ITER(a) ((a).iter_dev ? *(a).iter_dev : (a).iter)

// Live launch timing (hmsc_kernel_timing): each workgroup reads the constant-rate wall
// clock (s_memrealtime) when it starts and when it finishes, and the launch's first start /
// last finish are kept per sweep slot by device-scope atomic min / max -- the duration of
// every launch of the timed region, graph replays included, with no event in the stream.
// Layout per timed kernel: KT_SLOTS starts, then KT_SLOTS ends.
constexpr int KT_SLOTS = 8192;
// KT_TAIL: the fused Gamma2 + BetaLambda launch's last reducer; KT_G2: its Gamma2 workgroup
// KT_SIDE: the side chain launch (GammaV algebra + delta chains), on the side stream
// KT_IT: a graph replay's sweep-counter launch (set_iters_kernel), slot of the replay's first sweep
enum KtId { KT_Z = 0, KT_ETA = 1, KT_BL = 2, KT_TAIL = 3, KT_G2 = 4, KT_SIDE = 5, KT_IT = 6, KT_N = 7 };
__device__ inline unsigned long long kt_now() { return __builtin_amdgcn_s_memrealtime(); }
__device__ inline void kt_record(unsigned long long* kt, uint32_t iter, unsigned long long t0) {
  const unsigned long long t1 = kt_now();
  const uint32_t slot = iter & (KT_SLOTS - 1);
  __hip_atomic_fetch_min(kt + slot, t0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_fetch_max(kt + KT_SLOTS + slot, t1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Every bounded in-launch / cross-stream wait is bounded in wall-clock time: a wait that
// outlasts HS_TIMEOUT_TICKS of the 100 MHz wall clock (1 s; a legitimate wait is microseconds)
// gives up, the caller raises its error bit and carries on so the launch drains, and the host
// fails the call after the sweep (capi.cpp check_device_flags).  A bound by spin count would
// vary with load latency and clocks.
constexpr unsigned long long HS_TIMEOUT_TICKS = 100000000ull;

// Kernel arguments are read through the scalar cache, and the compiler waits for each argument
// load before the value's first use, so a large argument block read field by field as the code
// reaches them pays one cache round trip per 64-byte line, in sequence, at the start of every
// workgroup (the fused Gamma2 + BetaLambda launch's 0.8 KB block: ~a dozen dependent misses in
// its prologue).  kernarg_warm<bytes>() issues one scalar load per line first, all in flight
// together, so the later reads hit the scalar cache.  (Loads only.)
template <int BYTES>
__device__ __forceinline__ void kernarg_warm() {
  typedef const __attribute__((address_space(4))) uint32_t* kptr;
  const kptr p = (kptr)__builtin_amdgcn_kernarg_segment_ptr();
  uint32_t acc = 0;
#pragma unroll
  for (int o = 0; o < (BYTES + 3) / 4; o += 16) acc ^= p[o];
  asm volatile("" ::"s"(acc));
}

// poll done() with s_sleep(SLEEP) between tries until it holds (true) or the bound passes (false)
template <int SLEEP, class F>
__device__ __forceinline__ bool spin_until(F done) {
  if (done()) return true;
  const unsigned long long t0 = kt_now();
  for (int spin = 1;; ++spin) {
    __builtin_amdgcn_s_sleep(SLEEP);
    if (done()) return true;
    if ((spin & 63) == 0 && kt_now() - t0 > HS_TIMEOUT_TICKS) return false;
  }
}

// A device-scope (L2-bypassing) load of a value another workgroup of the same launch, on
// any XCD, published behind a flag: the reader polls the flag relaxed and then loads with
// these, instead of an acquire fence that would invalidate its XCD's whole L2.
__device__ __forceinline__ double load_coherent(const double* p) {
  return __longlong_as_double(
      (long long)__hip_atomic_load((const unsigned long long*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
// ... and its producer side: a device-scope (write-through) store.  A workgroup publishes a
// tile of these with vm_stores_done() + __syncthreads() + a relaxed ticket, without the
// release fence's write-back of the whole L2 (buffer_wbl2, ~0.1-1 us each under load, once
// per wave) that __threadfence() would cost.
__device__ __forceinline__ void store_coherent(double* p, double v) {
  __hip_atomic_store((unsigned long long*)p, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
// this wave's vector memory operations (the coherent stores above) have completed
__device__ __forceinline__ void vm_stores_done() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// Diagnostic build only (python -m hmsc_amd.build --stamps -> libhmsc_amd_stamps.so):
// HMSC_STAMP(i) records the shader clock (s_memtime) of lane 0 of the calling workgroup
// into slot i of a device table read back with hmsc_debug_get(s, "stamps", ...).  The
// product build compiles it away.
#ifdef HMSC_STAMPS
extern __device__ unsigned long long g_stamps[1024];  // [0, 256): named slots; [256, 1024): per-workgroup
#define HMSC_STAMP(i)                                                              \
  do {                                                                             \
    unsigned long long t_;                                                         \
    __builtin_amdgcn_sched_barrier(0);                                             \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");    \
    __builtin_amdgcn_sched_barrier(0);                                             \
    if (threadIdx.x == 0) g_stamps[(i)] = t_;                                      \
  } while (0)
// the same from lane 0 of whichever wave executes it
#define HMSC_STAMP_W(i)                                                            \
  do {                                                                             \
    unsigned long long t_;                                                         \
    __builtin_amdgcn_sched_barrier(0);                                             \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");    \
    __builtin_amdgcn_sched_barrier(0);                                             \
    if ((threadIdx.x & 63) == 0) g_stamps[(i)] = t_;                               \
  } while (0)
// wall clock (s_memrealtime, 100 MHz: comparable across workgroups and XCDs)
#define HMSC_STAMP_RT(i)                                                           \
  do {                                                                             \
    unsigned long long t_;                                                         \
    __builtin_amdgcn_sched_barrier(0);                                             \
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory"); \
    __builtin_amdgcn_sched_barrier(0);                                             \
    if ((threadIdx.x & 63) == 0) g_stamps[(i)] = t_;                               \
  } while (0)
#else
#define HMSC_STAMP_RT(i) \
  do {                   \
  } while (0)
#define HMSC_STAMP(i) \
  do {                \
  } while (0)
#define HMSC_STAMP_W(i) \
  do {                  \
  } while (0)
#endif

// ---------------------------------------------------------------------------
// Single-workgroup dense linear algebra on small column-major matrices
// (n <= 64).  All threads of the workgroup call these together; the matrices
// may live in LDS or in (L2-resident) global scratch owned by this workgroup.
// They carry the small blocks of updateGammaV / updateGamma2 / the per-species
// and per-unit solves (chol / chol2inv / backsolve of the R code).
// ---------------------------------------------------------------------------

// In-place lower Cholesky A = L L^T (lower triangle overwritten, upper untouched).
// Right-looking, two barriers per column; the trailing update is distributed over a
// 32 (rows) x (blockDim/32) (columns) thread grid so no integer division is needed.
// Returns false (uniformly) if A is not positive definite.
__device__ inline bool wg_chol(double* A, int n, int lda, int* flag) {
  const int t = threadIdx.x, nt = blockDim.x;
  const int tr = t & 31, tc = t >> 5, ntc = nt >> 5;
  if (t == 0) *flag = 0;
  __syncthreads();
  for (int c = 0; c < n; ++c) {
    const double d = A[c + c * lda];
    const double sd = sqrt(d > 0.0 ? d : 1.0);
    const double inv = 1.0 / sd;
    for (int i = c + 1 + t; i < n; i += nt) A[i + c * lda] *= inv;
    __syncthreads();
    if (t == 0) {
      if (!(d > 0.0)) *flag = 1;
      A[c + c * lda] = sd;
    }
    for (int i = c + 1 + tr; i < n; i += 32) {
      const double lic = A[i + c * lda];
      for (int j = c + 1 + tc; j <= i; j += ntc) A[i + j * lda] -= lic * A[j + c * lda];
    }
    __syncthreads();
  }
  const bool bad = *flag != 0;
  __syncthreads();
  return !bad;
}

// x <- L^{-1} x (forward substitution), x shared; executed by thread 0.
__device__ inline void t0_forward(const double* L, int n, int lda, double* x) {
  if (threadIdx.x == 0) {
    for (int i = 0; i < n; ++i) {
      double s = x[i];
      for (int k = 0; k < i; ++k) s -= L[i + k * lda] * x[k];
      x[i] = s / L[i + i * lda];
    }
  }
  __syncthreads();
}

// x <- L^{-T} x (back substitution with the transpose of lower L); thread 0.
__device__ inline void t0_backward_t(const double* L, int n, int lda, double* x) {
  if (threadIdx.x == 0) {
    for (int i = n - 1; i >= 0; --i) {
      double s = x[i];
      for (int k = i + 1; k < n; ++k) s -= L[k + i * lda] * x[k];
      x[i] = s / L[i + i * lda];
    }
  }
  __syncthreads();
}

// Triangular solves for one right-hand side, column-oriented, one barrier per column:
// the pivot x_c is final once column c-1 has been applied; every thread reads it.
__device__ inline void wg_forward(const double* L, int n, int lda, double* x) {
  const int t = threadIdx.x, nt = blockDim.x;
  for (int c = 0; c < n; ++c) {
    const double xc = x[c] / L[c + c * lda];
    for (int i = c + 1 + t; i < n; i += nt) x[i] -= L[i + c * lda] * xc;
    __syncthreads();
    if (t == 0) x[c] = xc;
  }
  __syncthreads();
}

__device__ inline void wg_backward_t(const double* L, int n, int lda, double* x) {
  const int t = threadIdx.x, nt = blockDim.x;
  for (int c = n - 1; c >= 0; --c) {
    const double xc = x[c] / L[c + c * lda];
    for (int i = t; i < c; i += nt) x[i] -= L[c + i * lda] * xc;
    __syncthreads();
    if (t == 0) x[c] = xc;
  }
  __syncthreads();
}

// Inv <- (L L^T)^{-1} (R's chol2inv), Inv n x n with leading dim ldi; W scratch n*n.
// W = L^{-1} by column-oriented forward elimination of all n right-hand sides at once
// (one barrier per pivot), then Inv = W^T W.
__device__ inline void wg_chol2inv(const double* L, int n, int lda, double* Inv, int ldi, double* W) {
  const int t = threadIdx.x, nt = blockDim.x;
  const int tr = t & 31, tc = t >> 5, ntc = nt >> 5;
  for (int i = tr; i < n; i += 32)
    for (int j = tc; j < n; j += ntc) W[i + j * n] = (i == j) ? 1.0 : 0.0;
  __syncthreads();
  for (int c = 0; c < n; ++c) {
    const double inv = 1.0 / L[c + c * lda];
    // row c of W is final (columns j <= c); rows i > c get -L_ic * W_cj
    for (int i = c + 1 + tr; i < n; i += 32) {
      const double lic = L[i + c * lda] * inv;
      for (int j = tc; j <= c; j += ntc) W[i + j * n] -= lic * W[c + j * n];
    }
    __syncthreads();
    for (int j = t; j <= c; j += nt) W[c + j * n] *= inv;
    __syncthreads();
  }
  // Inv = W^T W (W lower triangular)
  for (int i = tr; i < n; i += 32)
    for (int j = tc; j < n; j += ntc) {
      double s = 0.0;
      for (int k = (i > j ? i : j); k < n; ++k) s += W[k + i * n] * W[k + j * n];
      Inv[i + j * ldi] = s;
    }
  __syncthreads();
}

// C = alpha * op(A) * op(B) + beta * C, all column-major, op = transpose if flag set.
__device__ inline void wg_gemm(int m, int n, int k, double alpha, const double* A, int lda, bool ta,
                               const double* B, int ldb, bool tb, double beta, double* C, int ldc) {
  const int t = threadIdx.x, nt = blockDim.x;
  const int tr = t & 31, tc = t >> 5, ntc = nt >> 5;
  const int sa_i = ta ? lda : 1, sa_q = ta ? 1 : lda;
  const int sb_q = tb ? ldb : 1, sb_j = tb ? 1 : ldb;
  for (int i = tr; i < m; i += 32)
    for (int j = tc; j < n; j += ntc) {
      double s = 0.0;
      const double* a = A + i * sa_i;
      const double* b = B + j * sb_j;
      for (int q = 0; q < k; ++q) s = fma(a[q * sa_q], b[q * sb_q], s);
      C[i + j * ldc] = alpha * s + (beta == 0.0 ? 0.0 : beta * C[i + j * ldc]);
    }
  __syncthreads();
}

// serial lower Cholesky of an n x n (ld n) block and the inverse of its factor, one thread
__device__ inline bool t_chol_inv(double* A, double* Li, int n) {
  bool ok = true;
  for (int c = 0; c < n; ++c) {
    double d = A[c + n * c];
    for (int k = 0; k < c; ++k) d -= A[c + n * k] * A[c + n * k];
    if (!(d > 0.0)) ok = false;
    d = sqrt(d > 0.0 ? d : 1.0);
    A[c + n * c] = d;
    for (int i = c + 1; i < n; ++i) {
      double s = A[i + n * c];
      for (int k = 0; k < c; ++k) s -= A[i + n * k] * A[c + n * k];
      A[i + n * c] = s / d;
    }
  }
  for (int j = 0; j < n; ++j)  // Li = L^-1 (lower), column by column
    for (int i = 0; i < n; ++i) {
      if (i < j) {
        Li[i + n * j] = 0.0;
        continue;
      }
      double s = (i == j) ? 1.0 : 0.0;
      for (int k = j; k < i; ++k) s -= A[i + n * k] * Li[k + n * j];
      Li[i + n * j] = s / A[i + n * i];
    }
  return ok;
}

// zero the strict upper triangle (turn an in-place wg_chol result into a clean L)
__device__ inline void wg_lower_only(double* A, int n, int lda) {
  const int t = threadIdx.x, tr = t & 31, tc = t >> 5, ntc = blockDim.x >> 5;
  for (int i = tr; i < n; i += 32)
    for (int j = tc; j < n; j += ntc)
      if (i < j) A[i + j * lda] = 0.0;
  __syncthreads();
}

__device__ inline void wg_copy(double* dst, const double* src, int n) {
  for (int p = threadIdx.x; p < n; p += blockDim.x) dst[p] = src[p];
  __syncthreads();
}

// XZ = XEta^T (Yx o Z) as stored (part == null), or still as updateZ's per-chunk partials
// (XZ_part[c], stride apart), summed where it is read in slab_sum_body's order -- the four
// waves' strided sums, paired -- so the value is the reduced buffer's, bit for bit.
struct XZSrc {
  const double* XZ;
  const double* part;
  int nparts;
  int64_t stride;
};
__device__ __forceinline__ double xz_get(const XZSrc& x, size_t g) {
  if (!x.part) return x.XZ[g];
  double s[4] = {0.0, 0.0, 0.0, 0.0};
  for (int cb = 0; cb < x.nparts; cb += 64) {  // 64 partials' loads in flight (one round up to
    double v[64];                                // the z launch's 64 chunks), then their sums
#pragma unroll
    for (int u = 0; u < 64; ++u) v[u] = x.part[(int64_t)min(cb + u, x.nparts - 1) * x.stride + g];  // (clamped)
#pragma unroll
    for (int u = 0; u < 64; ++u)
      if (cb + u < x.nparts) s[u & 3] += v[u];  // stripe u mod 4 in chunk order
  }
  return (s[0] + s[1]) + (s[2] + s[3]);
}

}  // namespace hmsc
