// Multi-workgroup blocked dense fp64 linear algebra on the matrix cores (gfx950), for the
// dense systems of the sweep that outgrow one workgroup: the spatial updateEta precision
// (R/updateEta.R:115-147, (np nf)^2), the spatial data-parameter grid
// (R/computeDataParameters.R:53-81: chol / inverse of every W_g) and the phylogeny
// BetaLambda system (R/updateBetaLambda.R:124-147, (ns K)^2).
//
// Cholesky A = L L^T, right-looking in 64-column panels, three launches per panel:
//   1. chol_diag_kernel    one workgroup factors the 64 x 64 diagonal block in LDS and
//                          writes L_kk and its inverse L_kk^-1 (a 64 x 64 workspace).  (Fusing
//                          it into workgroup 0 of the previous trailing update was measured: its
//                          register demand halves the update's occupancy, no net gain.)
//   2. chol_panel_kernel   every 64-row block below: A_ik <- A_ik L_kk^-T, a 64x64x64 GEMM
//                          on v_mfma_f64_16x16x4 (L_kk^-1 from the workspace, in LDS)
//   3. chol_update_kernel  every lower tile (i >= j) of the trailing matrix:
//                          A_ij <- A_ij - A_ik A_jk^T, one 64 x 64 tile per workgroup, both
//                          panels staged in LDS, 4 waves x (2 x 2) MFMA tiles; the product is
//                          formed transposed so a lane's accumulator entries are 16
//                          consecutive rows of one column (128-B coalesced read-modify-write)
// This is where the n^3 / 3 flops are (SYRK / GEMM of the trailing matrix): MFMA-bound.
// Triangular solves with one right-hand side (L y = b, L^T x = y) are blocked the same way:
// a one-workgroup solve of the diagonal block, then a multi-workgroup GEMV of the panel.
// Only the lower triangle of A is read; its upper triangle is left untouched except inside
// diagonal tiles (scratch).
#include <cstdlib>

#include "common.h"
#include "state.h"
#include "z_kernel.h"  // d4, mfma_f64
#include "wave_la.h"

namespace hmsc {

// phase clock stamps of chol_diag_kernel for scripts/tmp-style microbenchmarks that define
// g_stamps in their own translation unit (-DHMSC_STAMPS -DHMSC_DENSE_STAMPS)
#ifdef HMSC_DENSE_STAMPS
#define DENSE_STAMP(i) HMSC_STAMP(i)
#else
#define DENSE_STAMP(i) \
  do {                 \
  } while (0)
#endif

constexpr int DB = 64;       // panel / tile size
constexpr int DLD = DB + 1;  // padded LDS leading dimension

// Element (r, c) of a matrix argument.  ld > 0: column-major with leading dimension ld.  ld < 0:
// the tile-band layout of a band matrix (dense_band_ld, state.h): each 64-column panel J is a
// (-ld) x 64 column-major block holding rows 64 J .. 64 J - ld - 1, i.e. element (r, c) at
// (r - 64 J) + (-ld) c -- N (bw + 128) doubles instead of N^2.  The factorization and the
// solves touch only tiles inside the band (their bw restriction), which that block holds whole.
__device__ __forceinline__ size_t aix(int ld, int r, int c) {
  return ld > 0 ? (size_t)r + (size_t)ld * c : (size_t)(r - (c & ~(DB - 1))) + (size_t)(-ld) * c;
}

// Every in-launch handshake of this file (the sync-free solve's block flags, the fused
// panel's diagonal-inverse flag) is bounded in time: a wait that outlasts HS_TIMEOUT_TICKS of
// the 100 MHz wall clock (common.h) raises its bit in the sync block's error word
// (DENSE_SYNC_ERR, state.h) and the workgroup carries on, so the launch drains; the host reads
// that word after the sweep (capi.cpp check_device_flags) and fails the call instead of
// returning a half-solved system.

__device__ __forceinline__ void hs_raise(int* sync, int bit) {
  __hip_atomic_fetch_or(sync + DENSE_SYNC_ERR, bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// poll *f (relaxed, device scope) until pred(value); false (and bit raised) on timeout
template <class P>
__device__ __forceinline__ bool hs_wait(const int* f, P pred, int* sync, int bit) {
  if (pred(__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) return true;
  const unsigned long long t0 = kt_now();
  for (int spin = 1;; ++spin) {
    __builtin_amdgcn_s_sleep(1);
    if (pred(__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) return true;
    if ((spin & 255) == 0 && kt_now() - t0 > HS_TIMEOUT_TICKS) {
      hs_raise(sync, bit);
      return false;
    }
  }
}

// ---------------------------------------------------------------------------------------
// 1. diagonal block: L_kk (in place) and Linv_k = L_kk^-1 (64 x 64, ld 64, zero above)
// ---------------------------------------------------------------------------------------
// The block sits in LDS and is factored in four 16-column steps (the serial pivot chain is
// only ever 16 long inside one wave):
//   a. wave 0 factors the 16 x 16 diagonal sub-block with one row per lane in registers,
//      pivots and column entries broadcast by v_readlane (no LDS round trip per pivot); the
//      rows of its inverse then follow by substitution along each row with the factor read
//      back from LDS at wave-uniform addresses (broadcast reads, no cross-lane traffic);
//   b. the panel below, P = A L16^-T, as 16 x 16 MFMA tiles (one wave per 16-row tile);
//   c. the trailing lower 16 x 16 tiles, A_IJ -= P_I P_J^T, on the matrix cores, the tiles
//      spread over the four waves.
// L^-1's off-diagonal 16-blocks then follow by diagonal distance (one wave per block, MFMA),
//   I_ib,jb = -I_ib,ib sum_{k = jb}^{ib - 1} L_ib,k I_k,jb.
// Rows / columns past n are identity padding.
// Panel staging and the output read-modify-write are latency-bound, not bandwidth-bound (a
// 64 x 64 tile is 96 KB of traffic): every global load of a thread is issued before the first
// LDS store or use, at clamped (always valid) addresses, and the output tile is read into
// registers before the MFMA loop, so one memory latency covers the whole tile.
template <int ROWS>
__device__ __forceinline__ void panel_load(const double* A, int lda, int R0, int rows, int k0, int nb,
                                           double (&v)[ROWS * DB / 256]) {
#pragma unroll
  for (int u = 0; u < ROWS * DB / 256; ++u) {
    const int p = threadIdx.x + 256 * u, r = p % ROWS, c = p / ROWS;
    v[u] = A[aix(lda, R0 + min(r, rows - 1), k0 + min(c, nb - 1))];
  }
}

template <int ROWS, int LD>
__device__ __forceinline__ void panel_store(double* P, int rows, int nb, const double (&v)[ROWS * DB / 256]) {
#pragma unroll
  for (int u = 0; u < ROWS * DB / 256; ++u) {
    const int p = threadIdx.x + 256 * u, r = p % ROWS, c = p / ROWS;
    P[r + LD * c] = (r < rows && c < nb) ? v[u] : 0.0;
  }
}

__device__ __forceinline__ double readlane_d(double v, int l) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)b, l), hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// D[i][j] (+)= sum_{k < 16} X[xr + i][xc + k] Y[yr + j][yc + k] for LDS tiles (ld DLD); lane
// holds D[lk + 4 r][lm]
__device__ __forceinline__ d4 mma16_nt(const double* X, int xr, int xc, const double* Y, int yr, int yc, d4 acc) {
  const int lane = threadIdx.x & 63, lm = lane & 15, lk = lane >> 4;
#pragma unroll
  for (int s4 = 0; s4 < 4; ++s4)
    acc = mfma_f64(X[(xr + lm) + DLD * (xc + 4 * s4 + lk)], Y[(yr + lm) + DLD * (yc + 4 * s4 + lk)], acc);
  return acc;
}

// 16 x 16 lower Cholesky L and L^-1 by one wave, in 4-column steps on the matrix cores.
// The block is held in the MFMA accumulator layout, d[r] = A[lk + 4 r][lm] (the full
// symmetric matrix, read from the lower triangle at Tb, ld DLD).  Step s:
//   - the 4 x 4 pivot block (register s, lanes (4 s + j) + 16 i) is gathered by v_readlane
//     and factored uniformly: L4 and Li4 = L4^-1 (refined rsqrt pivots, no divisions);
//   - the column panel P = A[:, 4s:4s+4] L4^-T = (Li4 A[4s:4s+4, :])^T is one MFMA whose B
//     operand is register s itself (by symmetry), and lands in the A-operand layout
//     (lane (lm = i, lk = j) holds P[i][j]); rows above the block are masked to zero;
//   - the Schur complement update A -= P P^T is one MFMA with P as both operands.
// L^-1 then follows by block forward substitution on R = I - L X: X_t = Li4_t R_t and
// R -= P_t X_t, two MFMAs per block row.  Writes L (zeros above) to Tb and L^-1 to Ib.
// 8 MFMAs and 80 readlanes in place of ~500 readlanes of the row-per-lane form.
__device__ inline bool chol16_mfma(double* Tb, double* Ib) {
  const int lane = threadIdx.x & 63, lm = lane & 15, lk = lane >> 4;
  d4 d;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = lk + 4 * r;
    d[r] = row >= lm ? Tb[row + DLD * lm] : Tb[lm + DLD * row];
  }
  const d4 zero = {0.0, 0.0, 0.0, 0.0};
  double pc[4], li_op[4];
  bool ok = true;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    double a[4][4], l[4][4], li[4][4], rinv[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j <= i; ++j) a[i][j] = readlane_d(d[s], (4 * s + j) + 16 * i);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      double piv = a[j][j];
#pragma unroll
      for (int m = 0; m < j; ++m) piv = fma(-l[j][m], l[j][m], piv);
      ok = ok && piv > 0.0;
      rinv[j] = rsqrt_nr(piv > 0.0 ? piv : 1.0);
      l[j][j] = piv * rinv[j];
#pragma unroll
      for (int i = j + 1; i < 4; ++i) {
        double v = a[i][j];
#pragma unroll
        for (int m = 0; m < j; ++m) v = fma(-l[i][m], l[j][m], v);
        l[i][j] = v * rinv[j];
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      li[i][i] = rinv[i];
#pragma unroll
      for (int j = i - 1; j >= 0; --j) {
        double v = 0.0;
#pragma unroll
        for (int m = j; m < i; ++m) v = fma(l[i][m], li[m][j], v);
        li[i][j] = -rinv[i] * v;
      }
    }
    // Li4 as an A operand: lane (lm = k, lk = m) -> Li4[k][m]
    double op = 0.0;
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int m = 0; m <= k; ++m) op = (lm == k && lk == m) ? li[k][m] : op;
    li_op[s] = op;
    double p = mfma_f64(op, d[s], zero)[0];  // P[lm][lk]
    const int rel = lm - 4 * s;
    p = (rel < 0 || (rel < 4 && lk > rel)) ? 0.0 : p;
    pc[s] = p;
    d = mfma_f64(-p, p, d);
  }
  // L: column block s at lane (lm = i, lk = j) = L[i][4 s + j]
#pragma unroll
  for (int s = 0; s < 4; ++s) Tb[lm + DLD * (4 * s + lk)] = pc[s];
  d4 R;
#pragma unroll
  for (int r = 0; r < 4; ++r) R[r] = (lk + 4 * r == lm) ? 1.0 : 0.0;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const double x = mfma_f64(li_op[t], R[t], zero)[0];  // X_t[lk][lm] = Linv[4 t + lk][lm]
    Ib[(4 * t + lk) + DLD * lm] = x;
    R = mfma_f64(-pc[t], x, R);
  }
  return ok;
}

// Off-diagonal 16-block (ib, jb) of L^-1 by one wave: I_ib,jb = -I_ib,ib sum_{k = jb}^{ib - 1}
// L_ib,k I_k,jb -- needs L's block row ib and the inverse blocks (k, jb), k < ib, and
// (ib, ib).  Sw: this wave's 16 x 17 scratch.
__device__ __forceinline__ void inv_block(const double* T, double* I, double* Sw, int ib, int jb) {
  const int lane = threadIdx.x & 63, lm = lane & 15, lk = lane >> 4;
  // S = sum_{k = jb}^{ib - 1} L_ib,k I_k,jb   (B operand B[k][j] = I[16 k' + k][16 jb + j])
  d4 acc = {0.0, 0.0, 0.0, 0.0};
  for (int kk = 16 * jb; kk < 16 * ib; kk += 4)
    acc = mfma_f64(T[(16 * ib + lm) + DLD * (kk + lk)], I[(kk + lk) + DLD * (16 * jb + lm)], acc);
#pragma unroll
  for (int r = 0; r < 4; ++r) Sw[(lk + 4 * r) + 17 * lm] = acc[r];
  wave_lds_sync();
  // I_ib,jb = -I_ib,ib S
  d4 acc2 = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int s4 = 0; s4 < 4; ++s4)
    acc2 = mfma_f64(I[(16 * ib + lm) + DLD * (16 * ib + 4 * s4 + lk)], Sw[(4 * s4 + lk) + 17 * lm], acc2);
#pragma unroll
  for (int r = 0; r < 4; ++r) I[(16 * ib + lk + 4 * r) + DLD * (16 * jb + lm)] = -acc2[r];
}

// The factorization of the block staged in T (lower triangle, zeros above, identity past nb);
// I zeroed; S: 4 x 16 x 17 doubles.  All 256 threads.  L^-1's off-diagonal blocks are formed
// by the waves that would idle while wave 0 factors the next 16 x 16 pivot block (row kb - 1
// of the inverse during step kb's pivot), the last block row after the loop.  Linv goes out
// first (device-coherent stores); with pflag (the fused update's next panel waits on it) the
// flag is raised before L itself is written back to A (no launch reads the block's L).
__device__ inline void diag_body(double* T, double* I, double (*S)[16 * 17], double* A, int lda, int n, int k0,
                          double* Linv, int* info, int* pflag = nullptr, int pflag_value = 0, int* sync = nullptr) {
  __shared__ int bad;
  const int nb = min(DB, n - k0), t = threadIdx.x, lane = t & 63, w = t >> 6, lm = lane & 15, lk = lane >> 4;
  if (t == 0) bad = 0;
  __syncthreads();
  // a. 16 x 16 Cholesky and inverse of pivot block 0 on the matrix cores (chol16_mfma)
  if (w == 0 && !chol16_mfma(T, I) && lane == 0) bad = 1;
  __syncthreads();
  DENSE_STAMP(102);
  for (int kb = 0; kb < 3; ++kb) {
    const int K0 = 16 * kb;
    const int nrt = 3 - kb;  // 16-row tiles below this diagonal block
    // b. P_I = A_I,kb L16^-T for tiles I = kb + 1 + w (w < nrt)
    if (w < nrt) {
      const int R = K0 + 16 + 16 * w;
      d4 acc = {0.0, 0.0, 0.0, 0.0};
      acc = mma16_nt(T, R, K0, I, K0, K0, acc);
#pragma unroll
      for (int r = 0; r < 4; ++r) T[(R + lk + 4 * r) + DLD * (K0 + lm)] = acc[r];
    }
    __syncthreads();
    DENSE_STAMP(103 + 2 * kb);
    // c. A_IJ -= P_I P_J^T for kb < J <= I.  Wave 0 takes the next pivot block (kb+1, kb+1)
    // and goes straight on to factor it (a. of step kb + 1); waves 1-3 take the other tiles
    // and then block row kb of L^-1 (its blocks are independent of each other): the pivot
    // chain no longer waits for the whole trailing update, nor for the inverse.
    const int ntile = nrt * (nrt + 1) / 2;
    if (w == 0) {
      const int R = K0 + 16;
      d4 acc = {0.0, 0.0, 0.0, 0.0};
      acc = mma16_nt(T, R, K0, T, R, K0, acc);
#pragma unroll
      for (int r = 0; r < 4; ++r) T[(R + lk + 4 * r) + DLD * (R + lm)] -= acc[r];
      wave_lds_sync();
      if (!chol16_mfma(T + R + DLD * R, I + R + DLD * R) && lane == 0) bad = 1;
    } else {
      for (int q = w; q < ntile; q += 3) {  // tiles 1 .. ntile - 1 over waves 1-3
        int ti = 0;
        while ((ti + 1) * (ti + 2) / 2 <= q) ++ti;
        const int tj = q - ti * (ti + 1) / 2;
        const int R = K0 + 16 + 16 * ti, C = K0 + 16 + 16 * tj;
        d4 acc = {0.0, 0.0, 0.0, 0.0};
        acc = mma16_nt(T, R, K0, T, C, K0, acc);
#pragma unroll
        for (int r = 0; r < 4; ++r) T[(R + lk + 4 * r) + DLD * (C + lm)] -= acc[r];
      }
      if (w <= kb) inv_block(T, I, S[w], kb, w - 1);  // block row kb: jb = 0 .. kb - 1
    }
    __syncthreads();
    DENSE_STAMP(104 + 2 * kb);
  }
  DENSE_STAMP(109);
  // the last block row of L^-1 (its three blocks are independent), one wave per block
  if (w < 3) inv_block(T, I, S[w], 3, w);
  __syncthreads();
  DENSE_STAMP(110);
  {
    double iv[DB * DB / 256];  // every LDS read before the first store
#pragma unroll
    for (int u = 0; u < DB * DB / 256; ++u) {
      const int p = t + 256 * u, r = p & 63, c = p >> 6;
      iv[u] = I[r + DLD * c];
    }
#pragma unroll
    for (int u = 0; u < DB * DB / 256; ++u) store_coherent(Linv + t + 256 * u, iv[u]);
  }
  if (pflag) {
    // Linv out at device scope (write-through stores, each wave waits for its own), then the
    // publish.  A test (hmsc_debug_poison "chol_publish") can withhold one publish: the waiting
    // tiles must then time out and report.
    vm_stores_done();
    __syncthreads();
    if (t == 0) {
      const bool skip = __hip_atomic_exchange(sync + DENSE_SYNC_TEST, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                        HS_TEST_SKIP_PUBLISH;
      if (!skip) __hip_atomic_store(pflag, pflag_value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  {
    double tv[DB * DB / 256];
#pragma unroll
    for (int u = 0; u < DB * DB / 256; ++u) {
      const int p = t + 256 * u, r = p & 63, c = p >> 6;
      tv[u] = T[r + DLD * c];
    }
#pragma unroll
    for (int u = 0; u < DB * DB / 256; ++u) {
      const int p = t + 256 * u, r = p & 63, c = p >> 6;
      if (r < nb && c < nb && r >= c) A[aix(lda, k0 + r, k0 + c)] = tv[u];
    }
  }
  if (t == 0 && bad) atomicExch(info, 1);
  DENSE_STAMP(111);
}

__global__ __launch_bounds__(256) void chol_diag_kernel(double* A, int lda, int n, int k0, double* Linv, int* info,
                                                        int* pflag_reset = nullptr) {
  if (pflag_reset && threadIdx.x == 0) *pflag_reset = 0;  // a factorization's first launch: its steps start at 1
  __shared__ double T[DB * DLD];  // the block; its lower triangle becomes L
  __shared__ double I[DB * DLD];  // L^-1 (lower)
  __shared__ double S[4][16 * 17];  // per-wave 16 x 16 scratch (ld 17)
  DENSE_STAMP(100);
  const int nb = min(DB, n - k0), t = threadIdx.x;
  double v[DB * DB / 256];
  panel_load<DB>(A, lda, k0, nb, k0, nb, v);  // all 16 loads in flight (see panel_load)
#pragma unroll
  for (int u = 0; u < DB * DB / 256; ++u) {
    const int p = t + 256 * u, r = p & 63, c = p >> 6;
    T[r + DLD * c] = (r < nb && c < nb) ? (r >= c ? v[u] : 0.0) : (r == c ? 1.0 : 0.0);
    I[r + DLD * c] = 0.0;
  }
  __syncthreads();
  DENSE_STAMP(101);
  diag_body(T, I, S, A, lda, n, k0, Linv, info);
}

// ---------------------------------------------------------------------------------------
// 2. panel: A[i0:i0+64, k0:k0+64] <- A[..] Linv^T for every 64-row block below the diagonal
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void chol_panel_kernel(double* A, int lda, int n, int k0, const double* Linv) {
  __shared__ double P[DB * DLD];   // P[r][k] at r + DLD k
  __shared__ double Li[DB * DLD];  // Linv[c][k] at c + DLD k
  const int nb = min(DB, n - k0), i0 = k0 + nb + blockIdx.x * DB, rows = min(DB, n - i0);
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, lm = lane & 15, lk = lane >> 4;
  {
    double v[DB * DB / 256], li[DB * DB / 256];
    panel_load<DB>(A, lda, i0, rows, k0, nb, v);
#pragma unroll
    for (int u = 0; u < DB * DB / 256; ++u) li[u] = Linv[t + 256 * u];
    panel_store<DB, DLD>(P, rows, nb, v);
#pragma unroll
    for (int u = 0; u < DB * DB / 256; ++u) Li[((t + 256 * u) & 63) + DLD * ((t + 256 * u) >> 6)] = li[u];
  }
  __syncthreads();
  // out^T[c][r] = sum_k Linv[c][k] P[r][k]: A operand rows = c (column of the output),
  // B operand columns = r (row of the output) -> lane holds rows lm of columns lk + 4q
  d4 acc[4];
#pragma unroll
  for (int ct = 0; ct < 4; ++ct) acc[ct] = d4{0.0, 0.0, 0.0, 0.0};
  const int r = 16 * w + lm;
#pragma unroll 4
  for (int s = 0; s < DB / 4; ++s) {
    const int k = 4 * s + lk;
    const double b = P[r + DLD * k];
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) acc[ct] = mfma_f64(Li[16 * ct + lm + DLD * k], b, acc[ct]);
  }
  // acc[ct][q] = out^T[16 ct + lk + 4 q][16 w + lm] = out[row 16w + lm][col 16ct + lk + 4q]
  // (MFMA D[(l>>4) + 4q][l & 15] with the A-operand index as D's row)
#pragma unroll
  for (int ct = 0; ct < 4; ++ct)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int c = 16 * ct + lk + 4 * q;
      if (r < rows && c < nb) A[aix(lda, i0 + r, k0 + c)] = acc[ct][q];
    }
}

// ---------------------------------------------------------------------------------------
// 3. trailing update of the lower tiles: A_IJ -= P_I P_J^T  (P = the just-finished panel)
// ---------------------------------------------------------------------------------------
// DIAG: workgroup 0 -- the next diagonal block's tile, (0, 0) -- then factors that block
// (diag_body on its LDS, the panels' buffers reused) while the other workgroups finish the
// trailing update, instead of a separate one-workgroup launch on the critical path per
// panel.  Two workgroups per CU either way (LDS), so the diagonal code may take 256 VGPRs.
// With pflag (dense, unbanded: the next panel is exactly the tiles (i, 0), i >= 1, of this
// update) those workgroups also apply the next panel step to their tile -- tile Linv_next^T,
// once workgroup 0 has raised pflag = step + 1 with Linv_next written -- so the next step
// needs no panel launch either.
template <bool DIAG>
__global__ __launch_bounds__(256, 2) void chol_update_kernel(double* A, int lda, int n, int k0, double* Linv_next,
                                                             int* info, int* pflag, int* sync) {
  __shared__ double PI[DB * DLD];
  __shared__ double PJ[DB * DLD];
  const int nb = min(DB, n - k0), base = k0 + nb;
  int ti = (int)((sqrt(8.0 * blockIdx.x + 1.0) - 1.0) * 0.5);
  int tj = (int)blockIdx.x - ti * (ti + 1) / 2;
  if (tj > ti) ++ti, tj = (int)blockIdx.x - ti * (ti + 1) / 2;  // guard sqrt rounding
  if (tj < 0) --ti, tj = (int)blockIdx.x - ti * (ti + 1) / 2;
  const int I0 = base + DB * ti, J0 = base + DB * tj;
  const int rowsI = min(DB, n - I0), rowsJ = min(DB, n - J0);
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, lm = lane & 15, lk = lane >> 4;
  // wave w: output quadrant rows 32 (w & 1) + [0, 32), columns 32 (w >> 1) + [0, 32); computed
  // transposed (A operand = PJ rows = output columns, B operand = PI rows = output rows);
  // acc[a][b][q] is column qc + 16 a + lk + 4 q, row qr + 16 b + lm
  const int qr = 32 * (w & 1), qc = 32 * (w >> 1);
  const bool live = !(ti == tj && qc > qr);  // strictly upper quadrant of a diagonal tile: idle
  {
    double vI[DB * DB / 256], vJ[DB * DB / 256];
    panel_load<DB>(A, lda, I0, rowsI, k0, nb, vI);
    panel_load<DB>(A, lda, J0, rowsJ, k0, nb, vJ);
    panel_store<DB, DLD>(PI, rowsI, nb, vI);
    panel_store<DB, DLD>(PJ, rowsJ, nb, vJ);
  }
  double cv[2][2][4];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int c = min(qc + 16 * a + lk + 4 * q, rowsJ - 1), r = min(qr + 16 * b + lm, rowsI - 1);
        cv[a][b][q] = live ? A[aix(lda, I0 + r, J0 + c)] : 0.0;
      }
  __syncthreads();
  const bool diag_next = DIAG && blockIdx.x == 0;  // tile (0, 0): the next diagonal block
  const bool panel_next = DIAG && pflag && tj == 0 && ti >= 1;  // a tile of the next panel
  if (!live && !diag_next) return;
  d4 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = d4{0.0, 0.0, 0.0, 0.0};
  if (live) {
#pragma unroll 4
    for (int s = 0; s < DB / 4; ++s) {
      const int k = 4 * s + lk;
      const double bI0 = PI[qr + lm + DLD * k], bI1 = PI[qr + 16 + lm + DLD * k];
      const double aJ0 = PJ[qc + lm + DLD * k], aJ1 = PJ[qc + 16 + lm + DLD * k];
      acc[0][0] = mfma_f64(aJ0, bI0, acc[0][0]);
      acc[0][1] = mfma_f64(aJ0, bI1, acc[0][1]);
      acc[1][0] = mfma_f64(aJ1, bI0, acc[1][0]);
      acc[1][1] = mfma_f64(aJ1, bI1, acc[1][1]);
    }
  }
  if (!diag_next && !panel_next) {
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int c = qc + 16 * a + lk + 4 * q, r = qr + 16 * b + lm;
          if (r < rowsI && c < rowsJ) A[aix(lda, I0 + r, J0 + c)] = cv[a][b][q] - acc[a][b][q];
        }
    return;
  }
  if constexpr (DIAG) {
    if (panel_next) {
      // the updated tile into P (= PI, P[r][k] at r + DLD k), then -- once the next diagonal
      // block's inverse is published -- Linv_next (coherent loads: written by workgroup 0,
      // possibly on another XCD) into Li (= PJ) and out = P Linv_next^T as in chol_panel_kernel
      __syncthreads();  // every wave's reads of the staged panels done
      double* P = PI;
      double* Li = PJ;
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int c = qc + 16 * a + lk + 4 * q, r = qr + 16 * b + lm;
            P[r + DLD * c] = (r < rowsI && c < rowsJ) ? cv[a][b][q] - acc[a][b][q] : 0.0;
          }
      const int step = k0 / DB + 1;
      if (t == 0) hs_wait(pflag, [&](int v) { return v == step; }, sync, HS_ERR_CHOL_PANEL);
      __syncthreads();
      {
        double li[DB * DB / 256];
#pragma unroll
        for (int u = 0; u < DB * DB / 256; ++u)
          li[u] = __longlong_as_double((long long)__hip_atomic_load(
              (const unsigned long long*)(Linv_next + t + 256 * u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
#pragma unroll
        for (int u = 0; u < DB * DB / 256; ++u) Li[((t + 256 * u) & 63) + DLD * ((t + 256 * u) >> 6)] = li[u];
      }
      __syncthreads();
      d4 pacc[4];
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) pacc[ct] = d4{0.0, 0.0, 0.0, 0.0};
      const int r = 16 * w + lm;
#pragma unroll 4
      for (int s = 0; s < DB / 4; ++s) {
        const int k = 4 * s + lk;
        const double bv = P[r + DLD * k];
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) pacc[ct] = mfma_f64(Li[16 * ct + lm + DLD * k], bv, pacc[ct]);
      }
#pragma unroll
      for (int ct = 0; ct < 4; ++ct)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int c = 16 * ct + lk + 4 * q;
          if (r < rowsI && c < rowsJ) A[aix(lda, I0 + r, base + c)] = pacc[ct][q];
        }
      return;
    }
    // the updated block into T (= PI: lower triangle, zeros above, identity past nb), I (= PJ)
    // zeroed, then the diagonal factorization of block base (writes L into A, Linv_next)
    __shared__ double S[4][16 * 17];
    __syncthreads();  // every wave's panel reads done
    double* T = PI;
    double* I = PJ;
#pragma unroll
    for (int u = 0; u < DB * DB / 256; ++u) {
      const int p = t + 256 * u, r = p & 63, c = p >> 6;
      T[r + DLD * c] = (r == c && r >= rowsI) ? 1.0 : 0.0;
      I[r + DLD * c] = 0.0;
    }
    __syncthreads();
    if (live)
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int c = qc + 16 * a + lk + 4 * q, r = qr + 16 * b + lm;
            if (r < rowsI && c < rowsJ && r >= c) T[r + DLD * c] = cv[a][b][q] - acc[a][b][q];
          }
    __syncthreads();
    // (Linv_next out with device-coherent stores and pflag raised inside, before L's write-back)
    diag_body(T, I, S, A, lda, n, base, Linv_next, info, pflag, k0 / DB + 1, sync);
  }
}

// ---------------------------------------------------------------------------------------
// triangular solves with one right-hand side, from the factorization's diagonal-block
// inverses: one launch per 64-block, every workgroup forming z = Linv_k x_k (or Linv_k^T x_k)
// -- a 64 x 64 matrix-vector product, no serial substitution -- and then applying its share
// of the block's update.  The solved block goes to y; the updates go to x -- a block of x is
// only written by launches of earlier blocks, so no workgroup reads a value another
// workgroup of its launch writes.
// ---------------------------------------------------------------------------------------
template <bool TR>
__device__ inline void stage(double* S, const double* M, int ld, int R0, int C0, int rows, int cols) {
  double v[DB * DB / 256];  // all loads in flight before the first LDS store (see panel_load)
#pragma unroll
  for (int u = 0; u < DB * DB / 256; ++u) {
    const int p = threadIdx.x + 256 * u, a = p & 63, b = p >> 6;
    v[u] = M[aix(ld, R0 + min(a, rows - 1), C0 + min(b, cols - 1))];
  }
#pragma unroll
  for (int u = 0; u < DB * DB / 256; ++u) {
    const int p = threadIdx.x + 256 * u, a = p & 63, b = p >> 6;
    S[TR ? b + DLD * a : a + DLD * b] = (a < rows && b < cols) ? v[u] : 0.0;
  }
}
__device__ inline void stage_n(double* S, const double* M, int ld, int R0, int C0, int rows, int cols) {
  stage<false>(S, M, ld, R0, C0, rows, cols);
}
__device__ inline void stage_t(double* S, const double* M, int ld, int R0, int C0, int rows, int cols) {
  stage<true>(S, M, ld, R0, C0, rows, cols);
}

__device__ inline void block_solve(const double* Linv, const double* x, int k0, int nb, int trans, double* T,
                                   double* z, double* part) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  {
    double v[DB * DB / 256];
#pragma unroll
    for (int u = 0; u < DB * DB / 256; ++u) v[u] = Linv[t + 256 * u];
    const double xv = x[k0 + min(t & 63, nb - 1)];
#pragma unroll
    for (int u = 0; u < DB * DB / 256; ++u) T[((t + 256 * u) & 63) + DLD * ((t + 256 * u) >> 6)] = v[u];
    if (t < DB) z[t] = t < nb ? xv : 0.0;
  }
  __syncthreads();
  double s = 0.0;
  for (int c = 16 * w; c < 16 * w + 16; ++c) s = fma(trans ? T[c + DLD * lane] : T[lane + DLD * c], z[c], s);
  part[w * DB + lane] = s;
  __syncthreads();
  if (t < DB) z[t] = (part[t] + part[DB + t]) + (part[2 * DB + t] + part[3 * DB + t]);
  __syncthreads();
}

// forward, block k: z = Linv_k x_k -> y_k; x[i] -= sum_c L[i, k0 + c] z_c for the rows
// below, 64 rows per workgroup (4 waves x 16 columns, reduced in LDS)
__global__ __launch_bounds__(256) void trsv_fwd_kernel(const double* L, int lda, int n, int k0, const double* Linv,
                                                       double* x, double* y) {
  __shared__ double T[DB * DLD];
  __shared__ double z[DB];
  __shared__ double part[4 * DB];
  const int nb = min(DB, n - k0), t = threadIdx.x, lane = t & 63, w = t >> 6;
  block_solve(Linv + (size_t)(k0 / DB) * DB * DB, x, k0, nb, 0, T, z, part);
  if (blockIdx.x == 0 && t < nb) y[k0 + t] = z[t];
  const int i = k0 + nb + blockIdx.x * DB + lane;
  double lv[16];
#pragma unroll
  for (int u = 0; u < 16; ++u) lv[u] = L[aix(lda, min(i, n - 1), k0 + min(16 * w + u, nb - 1))];
  double s = 0.0;
#pragma unroll
  for (int u = 0; u < 16; ++u) s = fma(16 * w + u < nb ? lv[u] : 0.0, z[16 * w + u], s);
  part[w * DB + lane] = s;
  __syncthreads();
  if (w == 0 && i < n) x[i] -= (part[lane] + part[DB + lane]) + (part[2 * DB + lane] + part[3 * DB + lane]);
}

// backward, block k: z = Linv_k^T x_k -> y_k; x[j] -= sum_c L[k0 + c, j] z_c for the
// columns j < k0, 64 columns per workgroup read as a coalesced 64 x 64 tile
__global__ __launch_bounds__(256) void trsv_bwd_kernel(const double* L, int lda, int n, int k0, const double* Linv,
                                                       double* x, double* y, int jb0) {
  __shared__ double T[DB * DLD];
  __shared__ double z[DB];
  __shared__ double part[4 * DB];
  const int nb = min(DB, n - k0), t = threadIdx.x, lane = t & 63, w = t >> 6;
  block_solve(Linv + (size_t)(k0 / DB) * DB * DB, x, k0, nb, 1, T, z, part);
  if (blockIdx.x == 0 && t < nb) y[k0 + t] = z[t];
  const int j0 = (jb0 + (int)blockIdx.x) * DB, cols = min(DB, k0 - j0);
  if (cols <= 0) return;
  stage_n(T, L, lda, k0, j0, nb, cols);
  __syncthreads();
  double s = 0.0;
  for (int r = w; r < DB; r += 4) s = fma(T[r + DLD * lane], z[r], s);
  part[w * DB + lane] = s;
  __syncthreads();
  if (w == 0 && lane < cols) x[j0 + lane] -= (part[lane] + part[DB + lane]) + (part[2 * DB + lane] + part[3 * DB + lane]);
}

// ---------------------------------------------------------------------------------------
// Sync-free triangular solve (dense, unbanded): one launch, one workgroup per 64-row block,
// blocks taken in dependency order through a ticket (so every block a workgroup waits on
// belongs to a workgroup that is already running: no residency assumption).  Block k
// accumulates its update from each finished block j as soon as that block's flag is up
// (forward: sum_j L_kj y_j, j < k; transposed: sum_j L_jk^T x_j, j > k), with the next
// block's L tile already in flight, then solves its diagonal block with the factorization's
// Linv_k (a 64 x 64 matrix-vector product) in place in x and raises its flag.  The chain of
// blocks costs one flag round trip + one block solve per block instead of one kernel launch
// per block.  Flags are read with relaxed polling and the solved values with device-coherent
// loads (an acquire per poll would invalidate the XCD's L2); the last workgroup to finish
// resets the ticket, the done count and the flags for the next call.
// sync (the DENSE_SYNC_INTS block of state.h, zeroed once): [0] ticket, [1] done count, [2 + b]
// flag of block b, [DENSE_SYNC_ERR] the handshake error word.

__device__ __forceinline__ void wait_flag(const int* f, int* sync) {
  hs_wait(f, [](int v) { return v != 0; }, sync, HS_ERR_TRSV_FLAG);
}

// a workgroup done with the call: the last one through resets the ticket, the done count and
// the flags (every other one has finished its reads: it counted itself done after them)
__device__ __forceinline__ void trsv_sf_done(int* sync, int nbk) {
  if (__hip_atomic_fetch_add(&sync[1], 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == nbk - 1) {
    for (int b = 0; b < nbk; ++b) __hip_atomic_store(sync + 2 + b, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&sync[0], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&sync[1], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

template <bool TR>
__global__ __launch_bounds__(256) void trsv_sf_kernel(const double* L, int lda, int n, const double* Linv, double* x,
                                                      int* sync) {
  __shared__ int s_ord;
  __shared__ double red[DB * (DB + 1)];  // [row][part] partial sums (ld DB + 1)
  __shared__ double z[DB];
  const int nbk = (n + DB - 1) / DB, t = threadIdx.x, lane = t & 63, g = t >> 6;
  if (t == 0) s_ord = __hip_atomic_fetch_add(&sync[0], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const int ord = s_ord;
  if (ord >= nbk) {  // a corrupt ticket (the call's handshake was not reset): report, drain
    if (t == 0) {
      hs_raise(sync, HS_ERR_TRSV_TICKET);
      trsv_sf_done(sync, nbk);
    }
    return;
  }
  const int k = TR ? nbk - 1 - ord : ord, R0 = k * DB, nb = min(DB, n - R0);
  int* flag = sync + 2;
  // this block's own operands -- Linv_k (lane = output row, wave g = terms 16 g ..) and x_k --
  // loaded before the dependency chain, so the solve after the last flag waits on no memory
  const double* Li = Linv + (size_t)k * DB * DB;
  double li[16];
#pragma unroll
  for (int u = 0; u < 16; ++u) {
    const int c = 16 * g + u;
    li[u] = TR ? Li[c + DB * lane] : Li[lane + DB * c];
  }
  const double xk = t < nb ? x[R0 + t] : 0.0;
  double acc[16];
#pragma unroll
  for (int u = 0; u < 16; ++u) acc[u] = 0.0;
  if (!TR) {
    // lane = row r of block k, wave g = columns 16 g .. 16 g + 15 of each block j < k (full blocks)
    const size_t row = (size_t)(R0 + min(lane, nb - 1));
    double lc[16], ln[16];
    if (k > 0)
#pragma unroll
      for (int u = 0; u < 16; ++u) lc[u] = L[row + (size_t)lda * (16 * g + u)];
    for (int j = 0; j < k; ++j) {
      if (j + 1 < k)
#pragma unroll
        for (int u = 0; u < 16; ++u) ln[u] = L[row + (size_t)lda * (DB * (j + 1) + 16 * g + u)];
      if (t == 0) wait_flag(flag + j, sync);
      __syncthreads();
#pragma unroll
      for (int u = 0; u < 16; ++u) acc[u] = fma(lc[u], load_coherent(x + DB * j + 16 * g + u), acc[u]);
#pragma unroll
      for (int u = 0; u < 16; ++u) lc[u] = ln[u];
    }
    double s = 0.0;
#pragma unroll
    for (int u = 0; u < 16; ++u) s += acc[u];
    red[lane * (DB + 1) + g] = s;
  } else {
    // lane = row c of block j > k (coalesced column runs), wave g = outputs r = 16 g .. 16 g + 15
    double lc[16], ln[16];
    auto ldt = [&](double (&v)[16], int j) {
      const int rows = min(DB, n - DB * j);
      const size_t row = (size_t)(DB * j + min(lane, rows - 1));
#pragma unroll
      for (int u = 0; u < 16; ++u) v[u] = lane < rows ? L[row + (size_t)lda * (R0 + min(16 * g + u, nb - 1))] : 0.0;
    };
    if (k < nbk - 1) ldt(lc, nbk - 1);
    for (int j = nbk - 1; j > k; --j) {
      if (j - 1 > k) ldt(ln, j - 1);
      if (t == 0) wait_flag(flag + j, sync);
      __syncthreads();
      const int rows = min(DB, n - DB * j);
      const double xv = lane < rows ? load_coherent(x + DB * j + lane) : 0.0;
#pragma unroll
      for (int u = 0; u < 16; ++u) acc[u] = fma(lc[u], xv, acc[u]);
#pragma unroll
      for (int u = 0; u < 16; ++u) lc[u] = ln[u];
    }
    // acc[u]: partial over this lane's row c for output 16 g + u -> red[output][c]
#pragma unroll
    for (int u = 0; u < 16; ++u) red[(16 * g + u) * (DB + 1) + lane] = acc[u];
  }
  __syncthreads();
  // b = x_k - update
  if (t < DB) {
    double s = 0.0;
    if (!TR) {
      s = (red[t * (DB + 1)] + red[t * (DB + 1) + 1]) + (red[t * (DB + 1) + 2] + red[t * (DB + 1) + 3]);
    } else {
      for (int c = 0; c < DB; ++c) s += red[t * (DB + 1) + c];
    }
    z[t] = t < nb ? xk - s : 0.0;
  }
  __syncthreads();
  // x_k = Linv_k b (or Linv_k^T b): lane = output row, wave g = 16 of the 64 terms
  double s = 0.0;
#pragma unroll
  for (int u = 0; u < 16; ++u) s = fma(li[u], z[16 * g + u], s);
  red[lane * (DB + 1) + g] = s;
  __syncthreads();
  if (t < nb) x[R0 + t] = (red[t * (DB + 1)] + red[t * (DB + 1) + 1]) + (red[t * (DB + 1) + 2] + red[t * (DB + 1) + 3]);
  __threadfence();  // each wave's stores of the block complete at device scope ...
  __syncthreads();  // ... before the flag
  if (t == 0) {
    __hip_atomic_store(flag + k, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    trsv_sf_done(sync, nbk);
  }
}

// ---------------------------------------------------------------------------------------
// inverse of a lower factor (trtri) and M^T M (lauum): the spatial grid precompute
// (R/computeDataParameters.R:53-81 evaluates iW = chol2inv(chol(W)) for every grid point)
// ---------------------------------------------------------------------------------------
// LDS staging of a 64 x 64 tile, zero padded: S[r][k] at r + DLD k
//   stage_n: S[r][k] = M[R0 + r, C0 + k]         (r < rows, k < cols)
//   stage_t: S[c][k] = M[R0 + k, C0 + c]         (k < rows, c < cols)
// out[r][c] += sum_k SA[r][k] SB[c][k] over the wave's 32 x 32 quadrant (as chol_update_kernel):
// acc[a][b][q] holds out[qr + 16 b + lm][qc + 16 a + lk + 4 q]
__device__ inline void tile_mma(d4 (&acc)[2][2], const double* SA, const double* SB) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, lm = lane & 15, lk = lane >> 4;
  const int qr = 32 * (w & 1), qc = 32 * (w >> 1);
#pragma unroll 4
  for (int s = 0; s < DB / 4; ++s) {
    const int k = 4 * s + lk;
    const double b0 = SA[qr + lm + DLD * k], b1 = SA[qr + 16 + lm + DLD * k];
    const double a0 = SB[qc + lm + DLD * k], a1 = SB[qc + 16 + lm + DLD * k];
    acc[0][0] = mfma_f64(a0, b0, acc[0][0]);
    acc[0][1] = mfma_f64(a0, b1, acc[0][1]);
    acc[1][0] = mfma_f64(a1, b0, acc[1][0]);
    acc[1][1] = mfma_f64(a1, b1, acc[1][1]);
  }
}

__device__ inline void zero_acc(d4 (&acc)[2][2]) {
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = d4{0.0, 0.0, 0.0, 0.0};
}

// visit the quadrant's entries: f(r, c, value)
template <class F>
__device__ inline void acc_each(const d4 (&acc)[2][2], F f) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, lm = lane & 15, lk = lane >> 4;
  const int qr = 32 * (w & 1), qc = 32 * (w >> 1);
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int q = 0; q < 4; ++q) f(qr + 16 * b + lm, qc + 16 * a + lk + 4 * q, acc[a][b][q]);
}

// the same visit order without values: f(r, c)
template <class F>
__device__ inline void acc_each_index(F f) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, lm = lane & 15, lk = lane >> 4;
  const int qr = 32 * (w & 1), qc = 32 * (w >> 1);
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int q = 0; q < 4; ++q) f(qr + 16 * b + lm, qc + 16 * a + lk + 4 * q);
}

// every diagonal block inverse of a lower-triangular L: Dinv[b] = L_bb^-1 (64 x 64, ld 64,
// zero above, identity-padded past n); one workgroup per block
__global__ __launch_bounds__(64) void trtri_diag_kernel(const double* L, int ld, int n, double* Dinv) {
  __shared__ double T[DB * DLD];
  __shared__ double I[DB * DLD];
  const int k0 = DB * blockIdx.x, nb = min(DB, n - k0), t = threadIdx.x;
  for (int c = 0; c < DB; ++c)
    T[t + DLD * c] = (t < nb && c < nb && t >= c) ? L[(size_t)(k0 + t) + (size_t)ld * (k0 + c)] : (t == c ? 1.0 : 0.0);
  __syncthreads();
  for (int i = 0; i < DB; ++i) {  // column t of T X = I by forward substitution
    double x = (i == t) ? 1.0 : 0.0;
    if (i >= t)
      for (int k = t; k < i; ++k) x -= T[i + DLD * k] * I[k + DLD * t];
    I[i + DLD * t] = i >= t ? x / T[i + DLD * i] : 0.0;
  }
  __syncthreads();
  double* D = Dinv + (size_t)DB * DB * blockIdx.x;
  for (int c = 0; c < DB; ++c) D[t + DB * c] = I[t + DLD * c];
}

// right-looking block forward substitution for X = L^-1, in M (zeroed beforehand):
//   row step k:    X_kj = Dinv_k B_kj (j < k), X_kk = Dinv_k       -- grid k + 1
//   update step k: B_ij -= L_ik X_kj   (i > k, j <= k)             -- grid (nbk-k-1)(k+1)
__global__ __launch_bounds__(256) void trtri_row_kernel(double* M, int ldm, int n, int k, const double* Dinv) {
  __shared__ double SA[DB * DLD];
  __shared__ double SB[DB * DLD];
  const int j = blockIdx.x, K0 = DB * k, J0 = DB * j, rowsK = min(DB, n - K0), colsJ = min(DB, n - J0);
  const double* D = Dinv + (size_t)DB * DB * k;
  if (j == k) {
    for (int p = threadIdx.x; p < DB * DB; p += 256) {
      const int r = p & 63, c = p >> 6;
      if (r < rowsK && c < rowsK) M[(size_t)(K0 + r) + (size_t)ldm * (K0 + c)] = D[r + DB * c];
    }
    return;
  }
  stage_n(SA, D, DB, 0, 0, DB, DB);
  stage_t(SB, M, ldm, K0, J0, rowsK, colsJ);
  __syncthreads();
  d4 acc[2][2];
  zero_acc(acc);
  tile_mma(acc, SA, SB);
  acc_each(acc, [&](int r, int c, double v) {
    if (r < rowsK && c < colsJ) M[(size_t)(K0 + r) + (size_t)ldm * (J0 + c)] = v;
  });
}

__global__ __launch_bounds__(256) void trtri_update_kernel(double* M, int ldm, const double* L, int ldl, int n, int k) {
  __shared__ double SA[DB * DLD];
  __shared__ double SB[DB * DLD];
  const int nbk = (n + DB - 1) / DB, ni = nbk - k - 1;
  const int i = k + 1 + (int)blockIdx.x % ni, j = (int)blockIdx.x / ni;
  const int I0 = DB * i, J0 = DB * j, K0 = DB * k;
  const int rowsI = min(DB, n - I0), rowsK = min(DB, n - K0), colsJ = min(DB, n - J0);
  stage_n(SA, L, ldl, I0, K0, rowsI, rowsK);
  stage_t(SB, M, ldm, K0, J0, rowsK, colsJ);
  double cv[16];  // the output tile, read before the MFMA loop
  int e = 0;
  acc_each_index([&](int r, int c) { cv[e++] = M[(size_t)(I0 + min(r, rowsI - 1)) + (size_t)ldm * (J0 + min(c, colsJ - 1))]; });
  __syncthreads();
  d4 acc[2][2];
  zero_acc(acc);
  tile_mma(acc, SA, SB);
  e = 0;
  acc_each(acc, [&](int r, int c, double v) {
    const double o = cv[e++];
    if (r < rowsI && c < colsJ) M[(size_t)(I0 + r) + (size_t)ldm * (J0 + c)] = o - v;
  });
}

// out = M^T M for lower-triangular M (full symmetric result): lower tile (i, j), i >= j, is
// sum_{k >= i} M_ki^T M_kj, mirrored into the upper triangle (diagonal tiles mirror their
// lower half, so the result is exactly symmetric)
__global__ __launch_bounds__(256) void lauum_kernel(const double* M, int ldm, int n, double* out, int ldo) {
  __shared__ double SA[DB * DLD];
  __shared__ double SB[DB * DLD];
  int ti = (int)((sqrt(8.0 * blockIdx.x + 1.0) - 1.0) * 0.5);
  int tj = (int)blockIdx.x - ti * (ti + 1) / 2;
  if (tj > ti) ++ti, tj = (int)blockIdx.x - ti * (ti + 1) / 2;
  if (tj < 0) --ti, tj = (int)blockIdx.x - ti * (ti + 1) / 2;
  const int nbk = (n + DB - 1) / DB, I0 = DB * ti, J0 = DB * tj;
  const int rowsI = min(DB, n - I0), rowsJ = min(DB, n - J0);
  d4 acc[2][2];
  zero_acc(acc);
  // chunk k's loads are issued during chunk k - 1's MFMAs (registers), stored after its barrier
  double va[DB * DB / 256], vb[DB * DB / 256];
  auto load = [&](int k) {
    const int K0 = DB * k, rowsK = min(DB, n - K0);
#pragma unroll
    for (int u = 0; u < DB * DB / 256; ++u) {
      const int p = threadIdx.x + 256 * u, kk = p & 63, c = p >> 6;
      va[u] = M[(size_t)(K0 + min(kk, rowsK - 1)) + (size_t)ldm * (I0 + min(c, rowsI - 1))];
      vb[u] = M[(size_t)(K0 + min(kk, rowsK - 1)) + (size_t)ldm * (J0 + min(c, rowsJ - 1))];
    }
  };
  load(ti);
  for (int k = ti; k < nbk; ++k) {
    const int rowsK = min(DB, n - DB * k);
#pragma unroll
    for (int u = 0; u < DB * DB / 256; ++u) {  // stage_t layout: S[c][k] = M[K0 + k, C0 + c]
      const int p = threadIdx.x + 256 * u, kk = p & 63, c = p >> 6;
      SA[c + DLD * kk] = (kk < rowsK && c < rowsI) ? va[u] : 0.0;
      SB[c + DLD * kk] = (kk < rowsK && c < rowsJ) ? vb[u] : 0.0;
    }
    __syncthreads();
    if (k + 1 < nbk) load(k + 1);
    tile_mma(acc, SA, SB);
    __syncthreads();
  }
  acc_each(acc, [&](int r, int c, double v) {
    if (r < rowsI && c < rowsJ && (ti != tj || r >= c)) {
      out[(size_t)(I0 + r) + (size_t)ldo * (J0 + c)] = v;
      out[(size_t)(J0 + c) + (size_t)ldo * (I0 + r)] = v;
    }
  });
}

// out = U diag(d) U^T (n x n, full symmetric, ld ldo) for U n x n (ld ldu) with
// d = dbase + n * (*rho - 1) (the phylogeny's spectral grid at the current rho index), or its
// reciprocal when `recip`: iQ = U diag(1/w) U^T and Q = U diag(w) U^T.  One lower 64 x 64
// tile per workgroup, MFMA tile products over 64-column chunks of U.
__global__ __launch_bounds__(256) void gram_diag_kernel(const double* U, int ldu, int n, const double* dbase,
                                                        const double* rho, int recip, double* out, int ldo) {
  __shared__ double SA[DB * DLD];
  __shared__ double SB[DB * DLD];
  int ti = (int)((sqrt(8.0 * blockIdx.x + 1.0) - 1.0) * 0.5);
  int tj = (int)blockIdx.x - ti * (ti + 1) / 2;
  if (tj > ti) ++ti, tj = (int)blockIdx.x - ti * (ti + 1) / 2;
  if (tj < 0) --ti, tj = (int)blockIdx.x - ti * (ti + 1) / 2;
  const int I0 = DB * ti, J0 = DB * tj, rowsI = min(DB, n - I0), rowsJ = min(DB, n - J0);
  const double* d = dbase + (size_t)n * ((int)(*rho) - 1);
  const int t = threadIdx.x;
  d4 acc[2][2];
  zero_acc(acc);
  double va[DB * DB / 256], vb[DB * DB / 256], dv[DB * DB / 256];
  auto load = [&](int K0) {  // chunk K0's loads, issued during the previous chunk's MFMAs
    const int cols = min(DB, n - K0);
#pragma unroll
    for (int u = 0; u < DB * DB / 256; ++u) {
      const int p = t + 256 * u, r = p & 63, k = p >> 6, kc = min(k, cols - 1);
      va[u] = U[(size_t)(I0 + min(r, rowsI - 1)) + (size_t)ldu * (K0 + kc)];
      vb[u] = U[(size_t)(J0 + min(r, rowsJ - 1)) + (size_t)ldu * (K0 + kc)];
      dv[u] = d[K0 + kc];
    }
  };
  load(0);
  for (int K0 = 0; K0 < n; K0 += DB) {
    const int cols = min(DB, n - K0);
    if (K0 > 0) __syncthreads();  // the previous chunk's products are done with SA / SB
#pragma unroll
    for (int u = 0; u < DB * DB / 256; ++u) {
      const int p = t + 256 * u, r = p & 63, k = p >> 6;
      const double dk = recip ? 1.0 / dv[u] : dv[u];
      SA[r + DLD * k] = (r < rowsI && k < cols) ? va[u] * dk : 0.0;
      SB[r + DLD * k] = (r < rowsJ && k < cols) ? vb[u] : 0.0;
    }
    __syncthreads();
    if (K0 + DB < n) load(K0 + DB);
    tile_mma(acc, SA, SB);
  }
  acc_each(acc, [&](int r, int c, double v) {
    if (r < rowsI && c < rowsJ && (ti != tj || r >= c)) {
      out[(size_t)(I0 + r) + (size_t)ldo * (J0 + c)] = v;
      out[(size_t)(J0 + c) + (size_t)ldo * (I0 + r)] = v;
    }
  });
}

void dense_gram_diag(hipStream_t st, const double* U, int ldu, int n, const double* dbase, const double* rho,
                     bool recip, double* out, int ldo) {
  const int nbk = (n + DB - 1) / DB;
  gram_diag_kernel<<<nbk * (nbk + 1) / 2, 256, 0, st>>>(U, ldu, n, dbase, rho, recip ? 1 : 0, out, ldo);
  HIP_OK(hipGetLastError());
}

// ---------------------------------------------------------------------------------------
// host launchers
// ---------------------------------------------------------------------------------------
// (kernels instead of hipMemset2DAsync / hipMemcpyAsync: one more kernel node in a captured
// sweep graph rather than a runtime blit)
__global__ __launch_bounds__(256) void zero_cols_kernel(double* M, int ldm, int n) {
  const int i = blockIdx.x * 256 + threadIdx.x, c = blockIdx.y;
  if (i < n) M[(size_t)i + (size_t)ldm * c] = 0.0;
}
__global__ __launch_bounds__(256) void copy_vec_kernel(double* x, const double* y, int n) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) x[i] = y[i];
}

// M <- L^-1 (lower, zero above; n x n, ld ldm) of the lower-triangular L; `dinv` holds
// ceil(n / 64) * 64 * 64 doubles: the diagonal-block inverses, computed here unless
// have_dinv (dense_potrf_lower's workspace already holds them)
void dense_trtri_lower(hipStream_t st, const double* L, int ldl, int n, double* M, int ldm, double* dinv,
                       bool have_dinv) {
  const int nbk = (n + DB - 1) / DB;
  zero_cols_kernel<<<dim3((n + 255) / 256, n), 256, 0, st>>>(M, ldm, n);
  if (!have_dinv) trtri_diag_kernel<<<nbk, 64, 0, st>>>(L, ldl, n, dinv);
  for (int k = 0; k < nbk; ++k) {
    trtri_row_kernel<<<k + 1, 256, 0, st>>>(M, ldm, n, k, dinv);
    const int ni = nbk - k - 1;
    if (ni > 0) trtri_update_kernel<<<ni * (k + 1), 256, 0, st>>>(M, ldm, L, ldl, n, k);
  }
  HIP_OK(hipGetLastError());
}

// out <- M^T M (full symmetric, n x n, ld ldo) of the lower-triangular M
void dense_lauum_lower(hipStream_t st, const double* M, int ldm, int n, double* out, int ldo) {
  const int nbk = (n + DB - 1) / DB;
  lauum_kernel<<<nbk * (nbk + 1) / 2, 256, 0, st>>>(M, ldm, n, out, ldo);
  HIP_OK(hipGetLastError());
}

// In-place lower Cholesky of the n x n matrix at A (column-major, ld lda; lower triangle
// read); `ws` holds dense_ws_doubles(n) doubles and keeps the diagonal-block inverses for
// dense_trsv_lower; *info (device) is set to 1 if A is not positive definite.  (A one-panel
// look-ahead on a second stream was measured slower: the co-running trailing update more
// than doubles the one-workgroup diagonal factorization, and the cross-stream joins add
// ~10 us per panel.)

// Banded (bw > 0): block column k0 has nonzeros in rows < k0 + DB + bw only, and the trailing
// update of its panel adds exact zeros outside the band, so the panel and update launches stop
// at the tiles covering rows k0 + DB .. k0 + DB + bw (the update's tile map depends on the
// launch size only: a smaller grid is the band's triangle of tiles).
void dense_potrf_lower(hipStream_t st, double* A, int n, int lda, double* ws, int* info, int bw, int* sync) {
  static const bool fuse_diag = [] {  // HMSC_NO_CHOL_DIAG_FUSION=1: the diagonal block as its own launch
    const char* e = std::getenv("HMSC_NO_CHOL_DIAG_FUSION");
    return !(e && e[0] && e[0] != '0');
  }();
  static const bool fuse_panel = [] {  // HMSC_NO_CHOL_PANEL_FUSION=1: the panel as its own launch
    const char* e = std::getenv("HMSC_NO_CHOL_PANEL_FUSION");
    return !(e && e[0] && e[0] != '0');
  }();
  // the panel handshake flag: past the workspace's diagonal-block inverses and solve vector
  // (dense_ws_doubles' slack), reset by the factorization's first launch
  const int nbk = (n + DB - 1) / DB;
  // (the fused panel needs the sync block for its timeout report)
  int* pflag = (fuse_diag && fuse_panel && bw <= 0 && lda > 0 && sync) ? (int*)(ws + (size_t)nbk * DB * DB + n + 8)
                                                                      : nullptr;
  HMSC_REQUIRE(lda > 0 || (bw > 0 && -lda >= dense_band_ld(bw)), "dense_potrf_lower: band layout narrower than the band");
  bool diag_done = false, panel_done = false;  // block k0 / panel k0 done by the previous trailing update
  for (int k0 = 0; k0 < n; k0 += DB) {
    double* Linv = ws + (size_t)(k0 / DB) * DB * DB;
    if (!diag_done) chol_diag_kernel<<<1, 256, 0, st>>>(A, lda, n, k0, Linv, info, k0 == 0 ? pflag : nullptr);
    const int rem = bw > 0 ? std::min(n - (k0 + DB), bw) : n - (k0 + DB);
    if (rem > 0) {
      const int nt = (rem + DB - 1) / DB;
      if (!panel_done) chol_panel_kernel<<<nt, 256, 0, st>>>(A, lda, n, k0, Linv);
      if (fuse_diag) {
        chol_update_kernel<true><<<nt * (nt + 1) / 2, 256, 0, st>>>(A, lda, n, k0, Linv + DB * DB, info, pflag,
                                                                      sync);
        diag_done = true;
        panel_done = pflag != nullptr;
      } else {
        chol_update_kernel<false><<<nt * (nt + 1) / 2, 256, 0, st>>>(A, lda, n, k0, nullptr, nullptr, nullptr,
                                                                       nullptr);
        diag_done = panel_done = false;
      }
    } else {
      diag_done = panel_done = false;
    }
  }
  HIP_OK(hipGetLastError());
}

// x <- L^-1 x  (trans = 0)  or  x <- L^-T x  (trans = 1), L lower (n x n, ld lda) as left by
// dense_potrf_lower together with its workspace `ws` (diagonal-block inverses, then n doubles
// in which the solution is assembled before it is copied back to x)
void dense_trsv_lower(hipStream_t st, const double* L, int n, int lda, double* x, int trans, double* ws, int bw,
                      int* sync) {
  const int nbk = (n + DB - 1) / DB;
  static const bool sf_off = [] {  // HMSC_NO_TRSV_SF=1: one launch per block (A/B diagnostics)
    const char* e = std::getenv("HMSC_NO_TRSV_SF");
    return e && e[0] && e[0] != '0';
  }();
  if (sync && bw <= 0 && lda > 0 && nbk >= 2 && nbk <= TRSV_SF_MAXB && !sf_off) {
    if (trans)
      trsv_sf_kernel<true><<<nbk, 256, 0, st>>>(L, lda, n, ws, x, sync);
    else
      trsv_sf_kernel<false><<<nbk, 256, 0, st>>>(L, lda, n, ws, x, sync);
    HIP_OK(hipGetLastError());
    return;
  }
  double* y = ws + (size_t)nbk * DB * DB;
  if (!trans) {
    for (int b = 0; b < nbk; ++b) {
      const int k0 = b * DB;
      const int rem = bw > 0 ? std::min(n - (k0 + DB), bw) : n - (k0 + DB);  // band: rows < k0 + DB + bw
      trsv_fwd_kernel<<<rem > 0 ? (rem + DB - 1) / DB : 1, 256, 0, st>>>(L, lda, n, k0, ws, x, y);
    }
  } else {
    for (int b = nbk - 1; b >= 0; --b) {
      const int k0 = b * DB;
      // band: block k's rows reach back to column k0 - bw only
      const int jb0 = bw > 0 ? std::max(0, (k0 - bw) / DB) : 0;
      const int nblk = k0 > 0 ? (k0 + DB - 1) / DB - jb0 : 1;
      trsv_bwd_kernel<<<std::max(1, nblk), 256, 0, st>>>(L, lda, n, k0, ws, x, y, jb0);
    }
  }
  copy_vec_kernel<<<(n + 255) / 256, 256, 0, st>>>(x, y, n);
  HIP_OK(hipGetLastError());
}

}  // namespace hmsc
