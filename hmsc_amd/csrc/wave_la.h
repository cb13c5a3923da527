// Register-resident dense algebra for one wave64 on small matrices (dimension <= NM <= 32).
//
// Layout: lane i holds ROW i of an NM x NM matrix in a register array `double a[NM]`.
// A problem of size n < NM is embedded as blockdiag(A, I) (wv_load pads with the identity),
// which every routine below maps to blockdiag(f(A), I), so all loops run at the compile-time
// size NM with no lane masking and no branches.  An element owned by another lane is fetched
// with v_readlane (wave-uniform lane index in fully unrolled loops): a factorisation is a chain
// of scalar broadcasts + FMAs with no LDS round trips and no barriers.  These carry the small
// Cholesky solves of updateBetaLambda, updateGammaV and updateGamma2 (chol / chol2inv /
// backsolve in the R code) when the dimension fits; common.h's LDS workgroup primitives cover
// larger ones.  Upper-triangle registers of a factor hold don't-care values (never read).
#pragma once
#include <hip/hip_runtime.h>

namespace hmsc {

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

// value of v in lane l (l wave-uniform)
__device__ __forceinline__ double bcast(double v, int l) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)b, l);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// dimension bucket for a runtime size (callers dispatch on it)
__host__ __device__ constexpr int wv_bucket(int n) { return n <= 8 ? 8 : n <= 16 ? 16 : n <= 24 ? 24 : 32; }
// the GammaV / Gamma2-prep chain (nc nt): also a 20 bucket -- its factorisations and
// inverses run every step to NM, so 20 x 20 systems (nc = 20, nt = 1) padded to 24 did
// (24/20)^3 = 1.7x the work of the cubic steps
__host__ __device__ constexpr int wv_bucket_gv(int n) { return n <= 8 ? 8 : n <= 16 ? 16 : n <= 20 ? 20 : n <= 24 ? 24 : 32; }

// rows/cols >= n (and lanes >= n) set to d * I
template <int NM>
__device__ inline void wv_pad(double (&a)[NM], int n, double d) {
  const int i = lane_id();
#pragma unroll
  for (int k = 0; k < NM; ++k)
    if (k >= n || i >= n) a[k] = (i == k) ? d : 0.0;
}

// lane i <- row i of a column-major n x n matrix (padded with the identity)
template <int NM>
__device__ inline void wv_load(const double* A, int lda, int n, double (&a)[NM]) {
  const int i = lane_id();
  const int ic = i < n ? i : 0;
#pragma unroll
  for (int k = 0; k < NM; ++k) {
    const double v = A[ic + (size_t)lda * (k < n ? k : 0)];
    a[k] = (i < n && k < n) ? v : (i == k ? 1.0 : 0.0);
  }
}

// lane i <- row i of J A J (J the exchange matrix of order n), padded with the identity
template <int NM>
__device__ inline void wv_load_rev(const double* A, int lda, int n, double (&a)[NM]) {
  const int i = lane_id();
  const int ic = i < n ? n - 1 - i : 0;
#pragma unroll
  for (int k = 0; k < NM; ++k) {
    const double v = A[ic + (size_t)lda * (k < n ? n - 1 - k : 0)];
    a[k] = (i < n && k < n) ? v : (i == k ? 1.0 : 0.0);
  }
}

template <int NM>
__device__ inline void wv_store(double* A, int lda, int n, const double (&a)[NM]) {
  const int i = lane_id();
  if (i < n)
#pragma unroll
    for (int k = 0; k < NM; ++k)
      if (k < n) A[i + (size_t)lda * k] = a[k];
}

// store the lower triangle of a factor (zeros above the diagonal)
template <int NM>
__device__ inline void wv_store_lower(double* A, int lda, int n, const double (&a)[NM]) {
  const int i = lane_id();
  if (i < n)
#pragma unroll
    for (int k = 0; k < NM; ++k)
      if (k < n) A[i + (size_t)lda * k] = (k <= i) ? a[k] : 0.0;
}

// 1 / sqrt(d) for d > 0 to full double precision: the hardware estimate refined by one
// Newton step (shorter dependency chain than sqrt followed by a division)
__device__ __forceinline__ double rsqrt_nr(double d) {
  const double y = __builtin_amdgcn_rsq(d);
  const double h = 0.5 * d * y;
  const double r = fma(-h, y, 0.5);  // 0.5 (1 - d y^2)
  return fma(y, r, y);
}

// In-place lower Cholesky: lane i ends with L[i][0..i] in a[0..i] and dinv = 1/L[i][i].
// Returns false (wave-uniformly) when a pivot is not positive.  The pivot chain is kept
// short: the column's entries are broadcast before the pivot's square root is known (the
// trailing update uses A[i][c] A[j][c] / d), and 1 / L[c][c] comes from a refined
// reciprocal square root (scripts/ubench_wave.hip: 5.7k vs 10.5k cycles at NM = 24 for the
// sqrt-then-divide form).
template <int NM>
__device__ inline bool wv_chol(double (&a)[NM], double& dinv) {
  const int i = lane_id();
  bool ok = true;
  dinv = 1.0;
#pragma unroll
  for (int c = 0; c < NM; ++c) {
    double col[NM];
#pragma unroll
    for (int j = c; j < NM; ++j) col[j] = bcast(a[c], j);
    const double d = col[c];
    ok = ok && d > 0.0;
    const double inv = rsqrt_nr(d > 0.0 ? d : 1.0);
    const double sc = a[c] * inv * inv;
#pragma unroll
    for (int j = c + 1; j < NM; ++j) a[j] = fma(-sc, col[j], a[j]);
    if (i == c) dinv = inv;
    a[c] = (i == c) ? d * inv : a[c] * inv;
  }
  return ok;
}

// L^{-1} by rows with the L entries broadcast by v_readlane (independent of the unknowns, so
// they issue ahead of the substitution chain): lane i, X_ij = -(sum_{k > j} X_ik L_kj) / L_jj
template <int NM>
__device__ inline void wv_inv_lower_rl(const double (&l)[NM], double dinv, double (&w)[NM]) {
  const int i = lane_id();
#pragma unroll
  for (int k = 0; k < NM; ++k) w[k] = (k == i) ? dinv : 0.0;
#pragma unroll
  for (int j = NM - 2; j >= 0; --j) {
    double s0 = 0.0, s1 = 0.0;
#pragma unroll
    for (int k = j + 1; k < NM; k += 2) {
      s0 = fma(w[k], bcast(l[j], k), s0);
      if (k + 1 < NM) s1 = fma(w[k + 1], bcast(l[j], k + 1), s1);
    }
    const double v = -(s0 + s1) * bcast(dinv, j);
    w[j] = (j < i) ? v : w[j];
  }
}

// The same factorisation with LDS broadcasts instead of v_readlane: per column every lane
// stores its A[i][c] once and then reads the column back at uniform addresses (LDS
// broadcast), so the NM - c - 1 trailing updates cost one ds_read each instead of two
// readlanes plus the SGPR->VALU wait states.  col: wave-private LDS scratch of 128 doubles
// (double-buffered by column parity; LDS executes one wave's instructions in order).
template <int NM>
__device__ inline bool wv_chol_s(double (&a)[NM], double& dinv, double* col) {
  const int i = lane_id();
  bool ok = true;
  dinv = 1.0;
#pragma unroll
  for (int c = 0; c < NM; ++c) {
    double* cb = col + 64 * (c & 1);
    cb[i] = a[c];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const double d = cb[c];
    ok = ok && d > 0.0;
    const double l = sqrt(d > 0.0 ? d : 1.0);
    const double inv = 1.0 / l;
    const double sc = a[c] * inv * inv;  // L[i][c] L[j][c] = sc * A[j][c]
#pragma unroll
    for (int j = c + 1; j < NM; ++j) a[j] = fma(-sc, cb[j], a[j]);
    if (i == c) dinv = inv;
    a[c] = (i == c) ? l : a[c] * inv;
  }
  return ok;
}

// x <- L^{-1} x, x lane-distributed (lane i holds x_i)
template <int NM>
__device__ inline void wv_forward(const double (&l)[NM], double dinv, double& x) {
  const int i = lane_id();
#pragma unroll
  for (int c = 0; c < NM; ++c) {
    const double xc = bcast(x * dinv, c);
    x = (i == c) ? xc : (i > c ? fma(-l[c], xc, x) : x);
  }
}

// x <- L^{-T} x given lt = L^T by rows (lane i holds column i of L: lt[k] = L[k][i], k >= i)
template <int NM>
__device__ inline void wv_backward_t(const double (&lt)[NM], double dinv, double& x) {
  const int i = lane_id();
#pragma unroll
  for (int c = NM - 1; c >= 0; --c) {
    const double xc = bcast(x * dinv, c);
    x = (i == c) ? xc : (i < c ? fma(-lt[c], xc, x) : x);
  }
}

// at <- a^T through an LDS scratch of NM*(NM+1) doubles private to this wave.
// LOWER: a is a factor whose entries above the diagonal are don't-care; they read as zero.
template <int NM, bool LOWER = false>
__device__ inline void wv_transpose(const double (&a)[NM], double (&at)[NM], double* lds) {
  constexpr int LD = NM + 1;
  const int i = lane_id();
  if (i < NM)
#pragma unroll
    for (int k = 0; k < NM; ++k) lds[i + LD * k] = (LOWER && k > i) ? 0.0 : a[k];  // element (i, k)
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
  for (int k = 0; k < NM; ++k) at[k] = (i < NM) ? lds[k + LD * i] : 0.0;  // element (k, i)
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// w <- L^{-1} (lower triangular, by rows) from the factor l of wv_chol
template <int NM>
__device__ inline void wv_inv_lower(const double (&l)[NM], double dinv, double (&w)[NM]) {
  const int i = lane_id();
#pragma unroll
  for (int k = 0; k < NM; ++k) w[k] = (i == k) ? 1.0 : 0.0;
#pragma unroll
  for (int m = 0; m < NM; ++m) {
    // row m is final up to the 1/L[m][m] scale
#pragma unroll
    for (int k = 0; k <= m; ++k) {
      const double wmk = bcast(w[k], m) * bcast(dinv, m);
      w[k] = (i == m) ? wmk : (i > m ? fma(-l[m], wmk, w[k]) : w[k]);
    }
  }
}

// w <- L^{-1} by rows (lane i: row i), L staged once in wave-private LDS (column-major,
// ld NM + 1, the diagonal slot holding 1 / L[i][i]); row i by substitution along the row,
// X_ij = -(sum_{k > j} X_ik L_kj) / L_jj, every L entry read at a uniform address (an LDS
// broadcast, no cross-lane register traffic), two partial sums per dot product.
// lds: NM * (NM + 1) doubles.
template <int NM>
__device__ inline void wv_inv_lower_rows(const double (&l)[NM], double dinv, double (&w)[NM], double* lds) {
  constexpr int LD = NM + 1;
  const int i = lane_id();
  if (i < NM) {
#pragma unroll
    for (int k = 0; k < NM; ++k) lds[i + LD * k] = (k < i) ? l[k] : (k == i ? dinv : 0.0);  // L[i][k]
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
  for (int k = 0; k < NM; ++k) w[k] = (k == i) ? dinv : 0.0;
#pragma unroll
  for (int j = NM - 2; j >= 0; --j) {
    double s0 = 0.0, s1 = 0.0;
#pragma unroll
    for (int k = j + 1; k < NM; k += 2) {
      s0 = fma(w[k], lds[k + LD * j], s0);
      if (k + 1 < NM) s1 = fma(w[k + 1], lds[k + 1 + LD * j], s1);
    }
    const double v = -(s0 + s1) * lds[j + LD * j];
    w[j] = (j < i) ? v : w[j];
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Columns of L^{-1}: lane i ends with column i of L^{-1} (w[r] = Linv[r][i]; zero for r < i).
// L is staged once in LDS; every lane then forward-substitutes its own unit vector reading
// L at uniform addresses (broadcasts) -- no cross-lane register traffic.  lds: scratch of
// NM * (NM + 1) doubles (the staged diagonal holds 1 / L[i][i]).
template <int NM>
__device__ inline void wv_inv_lower_cols(const double (&l)[NM], double dinv, double (&w)[NM], double* lds) {
  constexpr int LD = NM + 1;
  const int i = lane_id();
  if (i < NM) {
#pragma unroll
    for (int k = 0; k < NM; ++k) lds[i + LD * k] = (k < i) ? l[k] : (k == i ? dinv : 0.0);  // L[i][k]
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
  for (int r = 0; r < NM; ++r) w[r] = (r == i) ? 1.0 : 0.0;
#pragma unroll
  for (int c = 0; c < NM; ++c) {
    w[c] *= lds[c + LD * c];
#pragma unroll
    for (int r = c + 1; r < NM; ++r) w[r] = fma(-lds[r + LD * c], w[c], w[r]);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ---- products on the matrix cores -------------------------------------------------
// Operands are staged in LDS as zero-padded 32 x 32 column-major tiles (leading dim 33),
// multiplied with v_mfma_f64_16x16x4_f64 (lane l supplies A[l&15][k] / B[k][l&15] for
// k = k0 + (l>>4); D[(l>>4)+4r][l&15]) and read back by rows.  A wave needs 3 tiles of
// LDS (3 * 32 * 33 doubles).
constexpr int WV_LD = 33;
constexpr int WV_TILE = 32 * WV_LD;

typedef double wv_d4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void wv_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// lds <- a (TRANS: a^T), zero-padded to 32 x 32
template <int NM, bool TRANS = false, bool LOWER = false>
__device__ inline void wv_to_lds(const double (&a)[NM], double* lds) {
  const int i = lane_id();
  if (i < 32)
#pragma unroll
    for (int k = 0; k < 32; ++k) {
      double v = 0.0;
      if (k < NM && i < NM) v = (LOWER && k > i) ? 0.0 : a[k < NM ? k : 0];
      if (TRANS)
        lds[k + WV_LD * i] = v;  // element (k, i) of a^T
      else
        lds[i + WV_LD * k] = v;  // element (i, k)
    }
}

// lds <- blockdiag(J w_n J, I) zero-padded to 32 x 32, w an embedded blockdiag(w_n, I)
// by rows (J the exchange matrix of order n)
template <int NM>
__device__ inline void wv_to_lds_rev(const double (&w)[NM], int n, double* lds) {
  const int i = lane_id();
  if (i < 32)
#pragma unroll
    for (int k = 0; k < 32; ++k) {
      if (i < n && k < n)
        lds[(n - 1 - i) + WV_LD * (n - 1 - k)] = w[k < NM ? k : 0];
      else
        lds[i + WV_LD * k] = (i == k && i < NM) ? 1.0 : 0.0;
    }
}

template <int NM>
__device__ inline void wv_from_lds(const double* lds, double (&c)[NM]) {
  const int i = lane_id() < 32 ? lane_id() : 0;
#pragma unroll
  for (int k = 0; k < NM; ++k) c[k] = lds[i + WV_LD * k];
}

// lds C <- lds A * lds B  (T = 1 or 2 tiles of 16 per dimension)
template <int T>
__device__ inline void wv_mfma_lds(const double* A, const double* B, double* C) {
  const int l = lane_id(), lm = l & 15, lk = l >> 4;
#pragma unroll
  for (int mt = 0; mt < T; ++mt)
#pragma unroll
    for (int nt = 0; nt < T; ++nt) {
      wv_d4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int k0 = 0; k0 < 16 * T; k0 += 4)
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(A[16 * mt + lm + WV_LD * (k0 + lk)],
                                                   B[(k0 + lk) + WV_LD * (16 * nt + lm)], acc, 0, 0, 0);
#pragma unroll
      for (int r = 0; r < 4; ++r) C[(16 * mt + lk + 4 * r) + WV_LD * (16 * nt + lm)] = acc[r];
    }
}

// c <- op(a) op(b) with op = transpose when TA / TB; lds = 3 tiles
template <int NM, bool TA = false, bool TB = false, bool LA = false, bool LB = false>
__device__ inline void wv_gemm(const double (&a)[NM], const double (&b)[NM], double (&c)[NM], double* lds) {
  constexpr int T = NM <= 16 ? 1 : 2;
  wv_to_lds<NM, TA, LA>(a, lds);
  wv_to_lds<NM, TB, LB>(b, lds + WV_TILE);
  wv_sync();
  wv_mfma_lds<T>(lds, lds + WV_TILE, lds + 2 * WV_TILE);
  wv_sync();
  wv_from_lds<NM>(lds + 2 * WV_TILE, c);
  wv_sync();
}

// c <- A B with A, B already staged as padded LDS tiles; S = one scratch tile
template <int NM>
__device__ inline void wv_mm_lds(const double* A, const double* B, double (&c)[NM], double* S) {
  constexpr int T = NM <= 16 ? 1 : 2;
  wv_sync();
  wv_mfma_lds<T>(A, B, S);
  wv_sync();
  wv_from_lds<NM>(S, c);
  wv_sync();
}

// c <- a B with a in registers and B a staged tile; S = two scratch tiles
template <int NM>
__device__ inline void wv_mm_rt(const double (&a)[NM], const double* B, double (&c)[NM], double* S) {
  wv_to_lds<NM>(a, S);
  wv_mm_lds<NM>(S, B, c, S + WV_TILE);
}

// c <- w^T w for lower-triangular w by rows (chol2inv: (L L^T)^{-1} = L^{-T} L^{-1})
template <int NM>
__device__ inline void wv_syrk_tn_lower(const double (&w)[NM], double (&c)[NM], double* lds) {
  wv_gemm<NM, true, false, true, true>(w, w, c, lds);
}

// chol2inv: c <- (L L^T)^{-1} = L^{-T} L^{-1} from the factor of wv_chol; lds = 3 tiles.
template <int NM>
__device__ inline void wv_chol2inv(const double (&l)[NM], double dinv, double (&c)[NM], double* lds) {
  double w[NM];
  wv_inv_lower<NM>(l, dinv, w);
  wv_syrk_tn_lower<NM>(w, c, lds);
}

template <int NM>
__device__ inline void wv_chol2inv_rl(const double (&l)[NM], double dinv, double (&c)[NM], double* lds) {
  double w[NM];
  wv_inv_lower_rl<NM>(l, dinv, w);
  wv_syrk_tn_lower<NM>(w, c, lds);
}

// chol2inv through wv_inv_lower_rows (L staged in the third scratch tile)
template <int NM>
__device__ inline void wv_chol2inv_rows(const double (&l)[NM], double dinv, double (&c)[NM], double* lds) {
  double w[NM];
  wv_inv_lower_rows<NM>(l, dinv, w, lds + 2 * WV_TILE);
  wv_syrk_tn_lower<NM>(w, c, lds);
}

// the same through wv_inv_lower_cols (LDS broadcasts; measured slower on gfx950 at NM >= 24,
// kept for scripts/ubench_wave.hip)
template <int NM>
__device__ inline void wv_chol2inv_cols(const double (&l)[NM], double dinv, double (&c)[NM], double* lds) {
  double w[NM];
  wv_inv_lower_cols<NM>(l, dinv, w, lds + 2 * WV_TILE);
  wv_gemm<NM, false, true>(w, w, c, lds);
}

}  // namespace hmsc
