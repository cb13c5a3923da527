// Shared helpers for the hmsc_amd HIP kernels (gfx950, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <stdexcept>
#include <string>

namespace hmsc {

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

// ---------------------------------------------------------------------------
// Single-workgroup dense linear algebra on small column-major matrices
// (n <= 64).  All threads of the workgroup call these together; the matrices
// may live in LDS or in (L2-resident) global scratch owned by this workgroup.
// They carry the small blocks of updateGammaV / updateGamma2 / the per-species
// and per-unit solves (chol / chol2inv / backsolve of the R code).
// ---------------------------------------------------------------------------

// In-place lower Cholesky A = L L^T (lower triangle overwritten, upper untouched).
// Returns false (uniformly) if A is not positive definite.
__device__ inline bool wg_chol(double* A, int n, int lda, int* flag) {
  const int t = threadIdx.x, nt = blockDim.x;
  if (t == 0) *flag = 0;
  __syncthreads();
  for (int c = 0; c < n; ++c) {
    if (t == 0) {
      const double d = A[c + c * lda];
      if (!(d > 0.0)) *flag = 1;
      A[c + c * lda] = sqrt(d > 0.0 ? d : 1.0);
    }
    __syncthreads();
    const double inv = 1.0 / A[c + c * lda];
    for (int i = c + 1 + t; i < n; i += nt) A[i + c * lda] *= inv;
    __syncthreads();
    const int m = n - c - 1;
    for (int p = t; p < m * m; p += nt) {
      const int i = c + 1 + p % m, j = c + 1 + p / m;
      if (i >= j) A[i + j * lda] -= A[i + c * lda] * A[j + c * lda];
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

// Wave-parallel triangular solves for one right-hand side (blockDim == 64 users):
// column-oriented, one barrier per column.
__device__ inline void wg_forward(const double* L, int n, int lda, double* x) {
  const int t = threadIdx.x, nt = blockDim.x;
  for (int c = 0; c < n; ++c) {
    if (t == 0) x[c] /= L[c + c * lda];
    __syncthreads();
    const double xc = x[c];
    for (int i = c + 1 + t; i < n; i += nt) x[i] -= L[i + c * lda] * xc;
    __syncthreads();
  }
}

__device__ inline void wg_backward_t(const double* L, int n, int lda, double* x) {
  const int t = threadIdx.x, nt = blockDim.x;
  for (int c = n - 1; c >= 0; --c) {
    if (t == 0) x[c] /= L[c + c * lda];
    __syncthreads();
    const double xc = x[c];
    for (int i = t; i < c; i += nt) x[i] -= L[c + i * lda] * xc;
    __syncthreads();
  }
}

// Inv <- (L L^T)^{-1} (R's chol2inv), Inv n x n with leading dim ldi; W scratch n*n.
__device__ inline void wg_chol2inv(const double* L, int n, int lda, double* Inv, int ldi, double* W) {
  const int t = threadIdx.x, nt = blockDim.x;
  // W = L^{-1}, column by column (each thread one column of the identity)
  for (int c = t; c < n; c += nt) {
    for (int i = 0; i < n; ++i) {
      double s = (i == c) ? 1.0 : 0.0;
      for (int k = c; k < i; ++k) s -= L[i + k * lda] * W[k + c * n];
      W[i + c * n] = (i < c) ? 0.0 : s / L[i + i * lda];
    }
  }
  __syncthreads();
  // Inv = W^T W
  for (int p = t; p < n * n; p += nt) {
    const int i = p % n, j = p / n;
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
  for (int p = t; p < m * n; p += nt) {
    const int i = p % m, j = p / m;
    double s = 0.0;
    for (int q = 0; q < k; ++q) {
      const double a = ta ? A[q + i * lda] : A[i + q * lda];
      const double b = tb ? B[j + q * ldb] : B[q + j * ldb];
      s += a * b;
    }
    C[i + j * ldc] = alpha * s + (beta == 0.0 ? 0.0 : beta * C[i + j * ldc]);
  }
  __syncthreads();
}

// zero the strict upper triangle (turn an in-place wg_chol result into a clean L)
__device__ inline void wg_lower_only(double* A, int n, int lda) {
  for (int p = threadIdx.x; p < n * n; p += blockDim.x) {
    const int i = p % n, j = p / n;
    if (i < j) A[i + j * lda] = 0.0;
  }
  __syncthreads();
}

__device__ inline void wg_copy(double* dst, const double* src, int n) {
  for (int p = threadIdx.x; p < n; p += blockDim.x) dst[p] = src[p];
  __syncthreads();
}

}  // namespace hmsc
