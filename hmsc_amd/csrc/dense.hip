// Multi-workgroup blocked dense fp64 linear algebra on the matrix cores (gfx950), for the
// dense systems of the sweep that outgrow one workgroup: the spatial updateEta precision
// (R/updateEta.R:115-147, (np nf)^2), the spatial data-parameter grid
// (R/computeDataParameters.R:53-81: chol / inverse of every W_g) and the phylogeny
// BetaLambda system (R/updateBetaLambda.R:124-147, (ns K)^2).
//
// Cholesky A = L L^T, right-looking in 64-column panels, three launches per panel:
//   1. chol_diag_kernel    one workgroup factors the 64 x 64 diagonal block in LDS and
//                          writes L_kk and its inverse L_kk^-1 (a 64 x 64 workspace)
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
#include "common.h"
#include "state.h"
#include "z_kernel.h"  // d4, mfma_f64

namespace hmsc {

constexpr int DB = 64;       // panel / tile size
constexpr int DLD = DB + 1;  // padded LDS leading dimension

// ---------------------------------------------------------------------------------------
// 1. diagonal block: L_kk (in place) and Linv = L_kk^-1 (64 x 64, ld 64, zero above)
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void chol_diag_kernel(double* A, int lda, int n, int k0, double* Linv, int* info) {
  __shared__ double T[DB * DLD];
  __shared__ double I[DB * DLD];
  __shared__ int bad;
  const int nb = min(DB, n - k0), t = threadIdx.x;
  if (t == 0) bad = 0;
  for (int p = t; p < DB * DB; p += 256) {
    const int r = p & 63, c = p >> 6;
    T[r + DLD * c] = (r < nb && c < nb && r >= c) ? A[(size_t)(k0 + r) + (size_t)lda * (k0 + c)] : (r == c ? 1.0 : 0.0);
  }
  __syncthreads();
  for (int c = 0; c < nb; ++c) {  // unblocked right-looking Cholesky in LDS
    const double d = T[c + DLD * c];
    if (t == 0 && !(d > 0.0)) bad = 1;
    const double s = sqrt(d > 0.0 ? d : 1.0), inv = 1.0 / s;
    __syncthreads();
    if (t == 0) T[c + DLD * c] = s;
    for (int r = c + 1 + t; r < nb; r += 256) T[r + DLD * c] *= inv;
    __syncthreads();
    const int m = nb - c - 1;  // trailing lower update, (m x m) lower triangle
    for (int p = t; p < m * m; p += 256) {
      const int r = c + 1 + p % m, cc = c + 1 + p / m;
      if (r >= cc) T[r + DLD * cc] -= T[r + DLD * c] * T[cc + DLD * c];
    }
    __syncthreads();
  }
  // Linv: thread t < 64 solves column t of L X = I by forward substitution
  if (t < DB) {
    for (int i = 0; i < DB; ++i) {
      double x = (i == t) ? 1.0 : 0.0;
      if (i >= t)
        for (int k = t; k < i; ++k) x -= T[i + DLD * k] * I[k + DLD * t];
      I[i + DLD * t] = i >= t ? x / T[i + DLD * i] : 0.0;
    }
  }
  __syncthreads();
  for (int p = t; p < DB * DB; p += 256) {
    const int r = p & 63, c = p >> 6;
    if (r < nb && c < nb && r >= c) A[(size_t)(k0 + r) + (size_t)lda * (k0 + c)] = T[r + DLD * c];
    Linv[r + DB * c] = I[r + DLD * c];
  }
  if (t == 0 && bad) atomicExch(info, 1);
}

// ---------------------------------------------------------------------------------------
// 2. panel: A[i0:i0+64, k0:k0+64] <- A[..] Linv^T for every 64-row block below the diagonal
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void chol_panel_kernel(double* A, int lda, int n, int k0, const double* Linv) {
  __shared__ double P[DB * DLD];   // P[r][k] at r + DLD k
  __shared__ double Li[DB * DLD];  // Linv[c][k] at c + DLD k
  const int nb = min(DB, n - k0), i0 = k0 + nb + blockIdx.x * DB, rows = min(DB, n - i0);
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, lm = lane & 15, lk = lane >> 4;
  for (int p = t; p < DB * DB; p += 256) {
    const int r = p & 63, c = p >> 6;
    P[r + DLD * c] = (r < rows && c < nb) ? A[(size_t)(i0 + r) + (size_t)lda * (k0 + c)] : 0.0;
    Li[r + DLD * c] = Linv[r + DB * c];
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
      if (r < rows && c < nb) A[(size_t)(i0 + r) + (size_t)lda * (k0 + c)] = acc[ct][q];
    }
}

// ---------------------------------------------------------------------------------------
// 3. trailing update of the lower tiles: A_IJ -= P_I P_J^T  (P = the just-finished panel)
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void chol_update_kernel(double* A, int lda, int n, int k0) {
  __shared__ double PI[DB * DLD];
  __shared__ double PJ[DB * DLD];
  const int nb = min(DB, n - k0), base = k0 + nb;
  const int tI = (int)((sqrt(8.0 * blockIdx.x + 1.0) - 1.0) * 0.5);
  int ti = tI, tj = (int)blockIdx.x - ti * (ti + 1) / 2;
  if (tj > ti) ++ti, tj = (int)blockIdx.x - ti * (ti + 1) / 2;  // guard sqrt rounding
  if (tj < 0) --ti, tj = (int)blockIdx.x - ti * (ti + 1) / 2;
  const int I0 = base + DB * ti, J0 = base + DB * tj;
  const int rowsI = min(DB, n - I0), rowsJ = min(DB, n - J0);
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, lm = lane & 15, lk = lane >> 4;
  for (int p = t; p < DB * DB; p += 256) {
    const int r = p & 63, c = p >> 6;
    PI[r + DLD * c] = (r < rowsI && c < nb) ? A[(size_t)(I0 + r) + (size_t)lda * (k0 + c)] : 0.0;
    PJ[r + DLD * c] = (r < rowsJ && c < nb) ? A[(size_t)(J0 + r) + (size_t)lda * (k0 + c)] : 0.0;
  }
  __syncthreads();
  // wave w: output quadrant rows 32 (w & 1) + [0, 32), columns 32 (w >> 1) + [0, 32); computed
  // transposed (A operand = PJ rows = output columns, B operand = PI rows = output rows)
  const int qr = 32 * (w & 1), qc = 32 * (w >> 1);
  d4 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = d4{0.0, 0.0, 0.0, 0.0};
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
  // acc[a][b][q]: column qc + 16 a + lk + 4 q, row qr + 16 b + lm
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int c = qc + 16 * a + lk + 4 * q, r = qr + 16 * b + lm;
        if (r < rowsI && c < rowsJ) {
          double* dst = A + (size_t)(I0 + r) + (size_t)lda * (J0 + c);
          *dst -= acc[a][b][q];
        }
      }
}

// ---------------------------------------------------------------------------------------
// triangular solves with one right-hand side, in place on x (length n)
// ---------------------------------------------------------------------------------------
// diagonal block: forward L_kk y = x_k, or backward L_kk^T y = x_k (one workgroup)
__global__ __launch_bounds__(64) void trsv_diag_kernel(const double* L, int lda, int n, int k0, double* x, int trans) {
  __shared__ double T[DB * DLD];
  __shared__ double v[DB];
  const int nb = min(DB, n - k0), t = threadIdx.x;
  for (int c = 0; c < nb; ++c) T[t + DLD * c] = t < nb ? L[(size_t)(k0 + t) + (size_t)lda * (k0 + c)] : 0.0;
  v[t] = t < nb ? x[k0 + t] : 0.0;
  __syncthreads();
  if (!trans) {
    for (int c = 0; c < nb; ++c) {
      const double xc = v[c] / T[c + DLD * c];
      __syncthreads();
      if (t > c && t < nb) v[t] -= T[t + DLD * c] * xc;
      if (t == c) v[c] = xc;
      __syncthreads();
    }
  } else {
    for (int c = nb - 1; c >= 0; --c) {
      const double xc = v[c] / T[c + DLD * c];
      __syncthreads();
      if (t < c) v[t] -= T[c + DLD * t] * xc;
      if (t == c) v[c] = xc;
      __syncthreads();
    }
  }
  if (t < nb) x[k0 + t] = v[t];
}

// forward update: x[i] -= sum_{c in block k} L[i, c] x_c for rows i below the block
__global__ __launch_bounds__(256) void trsv_fwd_update_kernel(const double* L, int lda, int n, int k0, double* x) {
  __shared__ double xc[DB];
  const int nb = min(DB, n - k0), t = threadIdx.x;
  if (t < DB) xc[t] = t < nb ? x[k0 + t] : 0.0;
  __syncthreads();
  const int i = k0 + nb + blockIdx.x * 256 + t;
  if (i >= n) return;
  double s = 0.0;
  for (int c = 0; c < nb; ++c) s = fma(L[(size_t)i + (size_t)lda * (k0 + c)], xc[c], s);
  x[i] -= s;
}

// backward update: x[j] -= sum_{c in block k} L[c, j] x_c for columns j above the block;
// a workgroup takes 64 columns and reads the 64 x 64 tile L[block k, its columns] coalesced
__global__ __launch_bounds__(256) void trsv_bwd_update_kernel(const double* L, int lda, int n, int k0, double* x) {
  __shared__ double T[DB * DLD];
  __shared__ double xc[DB];
  __shared__ double part[4][DB];
  const int nb = min(DB, n - k0), t = threadIdx.x, j0 = blockIdx.x * DB, cols = min(DB, k0 - j0);
  if (t < DB) xc[t] = t < nb ? x[k0 + t] : 0.0;
  for (int p = t; p < DB * DB; p += 256) {
    const int r = p & 63, c = p >> 6;
    T[r + DLD * c] = (r < nb && c < cols) ? L[(size_t)(k0 + r) + (size_t)lda * (j0 + c)] : 0.0;
  }
  __syncthreads();
  const int c = t & 63, g = t >> 6;
  double s = 0.0;
  for (int r = g; r < DB; r += 4) s = fma(T[r + DLD * c], xc[r], s);
  part[g][c] = s;
  __syncthreads();
  if (t < cols) x[j0 + t] -= (part[0][t] + part[1][t]) + (part[2][t] + part[3][t]);
}

// ---------------------------------------------------------------------------------------
// host launchers
// ---------------------------------------------------------------------------------------
// In-place lower Cholesky of the n x n matrix at A (column-major, ld lda; lower triangle
// read); `ws` >= 64 * 64 doubles; *info (device) is set to 1 if A is not positive definite.
void dense_potrf_lower(hipStream_t st, double* A, int n, int lda, double* ws, int* info) {
  for (int k0 = 0; k0 < n; k0 += DB) {
    chol_diag_kernel<<<1, 256, 0, st>>>(A, lda, n, k0, ws, info);
    const int rem = n - (k0 + DB);
    if (rem > 0) {
      const int nt = (rem + DB - 1) / DB;
      chol_panel_kernel<<<nt, 256, 0, st>>>(A, lda, n, k0, ws);
      chol_update_kernel<<<nt * (nt + 1) / 2, 256, 0, st>>>(A, lda, n, k0);
    }
  }
  HIP_OK(hipGetLastError());
}

// x <- L^-1 x  (trans = 0)  or  x <- L^-T x  (trans = 1), L lower (n x n, ld lda)
void dense_trsv_lower(hipStream_t st, const double* L, int n, int lda, double* x, int trans) {
  const int nbk = (n + DB - 1) / DB;
  if (!trans) {
    for (int b = 0; b < nbk; ++b) {
      const int k0 = b * DB;
      trsv_diag_kernel<<<1, 64, 0, st>>>(L, lda, n, k0, x, 0);
      const int rem = n - (k0 + DB);
      if (rem > 0) trsv_fwd_update_kernel<<<(rem + 255) / 256, 256, 0, st>>>(L, lda, n, k0, x);
    }
  } else {
    for (int b = nbk - 1; b >= 0; --b) {
      const int k0 = b * DB;
      trsv_diag_kernel<<<1, 64, 0, st>>>(L, lda, n, k0, x, 1);
      if (k0 > 0) trsv_bwd_update_kernel<<<(k0 + DB - 1) / DB, 256, 0, st>>>(L, lda, n, k0, x);
    }
  }
  HIP_OK(hipGetLastError());
}

}  // namespace hmsc
