// Microbenchmark + cross-check of the register-resident wave primitives (wave_la.h):
// cycles per call (clock64 inside one wave) and errors against a host double-precision
// Cholesky / inverse, n = 10 / 20 / 30.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>
#include "../hmsc_amd/csrc/wave_la.h"
using namespace hmsc;

#define CK(x) (void)(x)

template <int NM>
__global__ __launch_bounds__(64) void k_chol(const double* A, int n, int reps, double* out, long long* cyc) {
  double l[NM], dinv;
  const long long t0 = clock64();
  for (int r = 0; r < reps; ++r) {
    wv_load<NM>(A, n, n, l);
    wv_chol<NM>(l, dinv);
  }
  const long long t1 = clock64();
  wv_store_lower<NM>(out, n, n, l);
  if (threadIdx.x == 0) *cyc = (t1 - t0) / reps;
}

template <int NM>
__global__ __launch_bounds__(64) void k_chol_s(const double* A, int n, int reps, double* out, long long* cyc) {
  __shared__ double col[128];
  double l[NM], dinv;
  const long long t0 = clock64();
  for (int r = 0; r < reps; ++r) {
    wv_load<NM>(A, n, n, l);
    wv_chol_s<NM>(l, dinv, col);
  }
  const long long t1 = clock64();
  wv_store_lower<NM>(out, n, n, l);
  if (threadIdx.x == 0) *cyc = (t1 - t0) / reps;
}

template <int NM>
__global__ __launch_bounds__(64) void k_inv(const double* A, int n, int reps, double* out, long long* cyc) {
  __shared__ double lds[3 * WV_TILE];
  double l[NM], c[NM], dinv;
  wv_load<NM>(A, n, n, l);
  wv_chol<NM>(l, dinv);
  const long long t0 = clock64();
  for (int r = 0; r < reps; ++r) wv_chol2inv<NM>(l, dinv, c, lds);
  const long long t1 = clock64();
  wv_store<NM>(out, n, n, c);
  if (threadIdx.x == 0) *cyc = (t1 - t0) / reps;
}

template <int NM>
__global__ __launch_bounds__(64) void k_inv2(const double* A, int n, int reps, double* out, long long* cyc) {
  __shared__ double lds[3 * WV_TILE];
  double l[NM], c[NM], dinv;
  wv_load<NM>(A, n, n, l);
  wv_chol<NM>(l, dinv);
  const long long t0 = clock64();
  for (int r = 0; r < reps; ++r) wv_chol2inv_rows<NM>(l, dinv, c, lds);
  const long long t1 = clock64();
  wv_store<NM>(out, n, n, c);
  if (threadIdx.x == 0) *cyc = (t1 - t0) / reps;
}

template <int NM>
__global__ __launch_bounds__(64) void k_inv3(const double* A, int n, int reps, double* out, long long* cyc) {
  __shared__ double lds[3 * WV_TILE];
  double l[NM], c[NM], dinv;
  wv_load<NM>(A, n, n, l);
  wv_chol<NM>(l, dinv);
  const long long t0 = clock64();
  for (int r = 0; r < reps; ++r) wv_chol2inv_rl<NM>(l, dinv, c, lds);
  const long long t1 = clock64();
  wv_store<NM>(out, n, n, c);
  if (threadIdx.x == 0) *cyc = (t1 - t0) / reps;
}

template <int NM>
__global__ __launch_bounds__(64) void k_chol_f(const double* A, int n, int reps, double* out, long long* cyc) {
  double l[NM], dinv;
  const long long t0 = clock64();
  for (int r = 0; r < reps; ++r) {
    wv_load<NM>(A, n, n, l);
    wv_chol<NM>(l, dinv);
  }
  const long long t1 = clock64();
  wv_store_lower<NM>(out, n, n, l);
  if (threadIdx.x == 0) *cyc = (t1 - t0) / reps;
}

template <int NM>
__global__ __launch_bounds__(64) void k_gemm(const double* A, const double* B, int n, int reps, double* out,
                                             long long* cyc) {
  __shared__ double lds[3 * WV_TILE];
  double a[NM], b[NM], c[NM];
  wv_load<NM>(A, n, n, a);
  wv_load<NM>(B, n, n, b);
  const long long t0 = clock64();
  for (int r = 0; r < reps; ++r) {
    wv_gemm<NM>(a, b, c, lds);
    a[0] += c[1] * 1e-300;
  }
  const long long t1 = clock64();
  wv_store<NM>(out, n, n, c);
  if (threadIdx.x == 0) *cyc = (t1 - t0) / reps;
}

template <int NM>
__global__ __launch_bounds__(64) void k_solve(const double* A, const double* b, int n, int reps, double* out,
                                              long long* cyc) {
  __shared__ double lds[3 * WV_TILE];
  double l[NM], lt[NM], dinv;
  wv_load<NM>(A, n, n, l);
  wv_chol<NM>(l, dinv);
  wv_transpose<NM, true>(l, lt, lds);
  double x = 0.0;
  const long long t0 = clock64();
  for (int r = 0; r < reps; ++r) {
    x = threadIdx.x < n ? b[threadIdx.x] : 0.0;
    wv_forward<NM>(l, dinv, x);
    wv_backward_t<NM>(lt, dinv, x);
  }
  const long long t1 = clock64();
  if (threadIdx.x < n) out[threadIdx.x] = x;
  if (threadIdx.x == 0) *cyc = (t1 - t0) / reps;
}

static void host_chol(std::vector<double>& a, int n) {
  for (int c = 0; c < n; ++c) {
    double d = a[c + n * c];
    for (int k = 0; k < c; ++k) d -= a[c + n * k] * a[c + n * k];
    d = std::sqrt(d);
    a[c + n * c] = d;
    for (int i = c + 1; i < n; ++i) {
      double s = a[i + n * c];
      for (int k = 0; k < c; ++k) s -= a[i + n * k] * a[c + n * k];
      a[i + n * c] = s / d;
    }
  }
}

template <int NM>
static void run(int n, double* dA, double* dB, double* dO, double* db, long long* dc) {
  const int reps = 50;
  std::vector<double> A(n * n), B(n * n), b(n);
  for (int j = 0; j < n; ++j)
    for (int i = 0; i < n; ++i) {
      A[i + n * j] = (i == j ? n : 0.0) + 1.0 / (1 + i + j);
      B[i + n * j] = std::sin(1.0 + i + 3.0 * j);
    }
  for (int i = 0; i < n; ++i) b[i] = 1.0 + i;
  CK(hipMemcpy(dA, A.data(), n * n * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(dB, B.data(), n * n * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(db, b.data(), n * 8, hipMemcpyHostToDevice));
  long long cy[5];
  std::vector<double> O(n * n);
  hipLaunchKernelGGL(k_chol<NM>, dim3(1), dim3(64), 0, 0, dA, n, reps, dO, dc);
  CK(hipMemcpy(&cy[0], dc, 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(O.data(), dO, n * n * 8, hipMemcpyDeviceToHost));
  std::vector<double> L = A;
  host_chol(L, n);
  double e_chol = 0;
  for (int j = 0; j < n; ++j)
    for (int i = j; i < n; ++i) e_chol = std::fmax(e_chol, std::fabs(O[i + n * j] - L[i + n * j]));
  hipLaunchKernelGGL(k_chol_s<NM>, dim3(1), dim3(64), 0, 0, dA, n, reps, dO, dc);
  CK(hipMemcpy(&cy[4], dc, 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(O.data(), dO, n * n * 8, hipMemcpyDeviceToHost));
  double e_chol_s = 0;
  for (int j = 0; j < n; ++j)
    for (int i = j; i < n; ++i) e_chol_s = std::fmax(e_chol_s, std::fabs(O[i + n * j] - L[i + n * j]));
  hipLaunchKernelGGL(k_inv<NM>, dim3(1), dim3(64), 0, 0, dA, n, reps, dO, dc);
  CK(hipMemcpy(&cy[1], dc, 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(O.data(), dO, n * n * 8, hipMemcpyDeviceToHost));
  double e_inv = 0;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) {
      double s = 0;
      for (int k = 0; k < n; ++k) s += A[i + n * k] * O[k + n * j];
      e_inv = std::fmax(e_inv, std::fabs(s - (i == j)));
    }
  long long cy_inv2 = 0;
  hipLaunchKernelGGL(k_inv2<NM>, dim3(1), dim3(64), 0, 0, dA, n, reps, dO, dc);
  CK(hipMemcpy(&cy_inv2, dc, 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(O.data(), dO, n * n * 8, hipMemcpyDeviceToHost));
  double e_inv2 = 0;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) {
      double s = 0;
      for (int k = 0; k < n; ++k) s += A[i + n * k] * O[k + n * j];
      e_inv2 = std::fmax(e_inv2, std::fabs(s - (i == j)));
    }
  printf("  chol2inv_rows=%lld cycles err=%.1e\n", cy_inv2, e_inv2);
  hipLaunchKernelGGL(k_inv3<NM>, dim3(1), dim3(64), 0, 0, dA, n, reps, dO, dc);
  CK(hipMemcpy(&cy_inv2, dc, 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(O.data(), dO, n * n * 8, hipMemcpyDeviceToHost));
  e_inv2 = 0;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) {
      double s = 0;
      for (int k = 0; k < n; ++k) s += A[i + n * k] * O[k + n * j];
      e_inv2 = std::fmax(e_inv2, std::fabs(s - (i == j)));
    }
  printf("  chol2inv_rl=%lld cycles err=%.1e\n", cy_inv2, e_inv2);
  hipLaunchKernelGGL(k_chol_f<NM>, dim3(1), dim3(64), 0, 0, dA, n, reps, dO, dc);
  CK(hipMemcpy(&cy_inv2, dc, 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(O.data(), dO, n * n * 8, hipMemcpyDeviceToHost));
  e_inv2 = 0;
  for (int j = 0; j < n; ++j)
    for (int i = j; i < n; ++i) e_inv2 = std::fmax(e_inv2, std::fabs(O[i + n * j] - L[i + n * j]));
  printf("  chol_fast=%lld cycles err=%.1e\n", cy_inv2, e_inv2);
  hipLaunchKernelGGL(k_gemm<NM>, dim3(1), dim3(64), 0, 0, dA, dB, n, reps, dO, dc);
  CK(hipMemcpy(&cy[2], dc, 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(O.data(), dO, n * n * 8, hipMemcpyDeviceToHost));
  double e_gemm = 0;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) {
      double s = 0;
      for (int k = 0; k < n; ++k) s += A[i + n * k] * B[k + n * j];
      e_gemm = std::fmax(e_gemm, std::fabs(s - O[i + n * j]));
    }
  hipLaunchKernelGGL(k_solve<NM>, dim3(1), dim3(64), 0, 0, dA, db, n, reps, dO, dc);
  CK(hipMemcpy(&cy[3], dc, 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(O.data(), dO, n * 8, hipMemcpyDeviceToHost));
  double e_solve = 0;
  for (int i = 0; i < n; ++i) {
    double s = 0;
    for (int k = 0; k < n; ++k) s += A[i + n * k] * O[k];
    e_solve = std::fmax(e_solve, std::fabs(s - b[i]));
  }
  printf("wave NM=%d n=%d  chol=%lld chol_s=%lld  chol2inv=%lld  gemm=%lld  fwd+bwd=%lld cycles | err chol=%.1e "
         "chol_s=%.1e inv=%.1e gemm=%.1e solve=%.1e\n",
         NM, n, cy[0], cy[4], cy[1], cy[2], cy[3], e_chol, e_chol_s, e_inv, e_gemm, e_solve);
}

int main() {
  double *dA, *dB, *dO, *db;
  long long* dc;
  CK(hipMalloc(&dA, 32 * 32 * 8));
  CK(hipMalloc(&dB, 32 * 32 * 8));
  CK(hipMalloc(&dO, 32 * 32 * 8));
  CK(hipMalloc(&db, 32 * 8));
  CK(hipMalloc(&dc, 8));
  run<16>(10, dA, dB, dO, db, dc);
  run<24>(20, dA, dB, dO, db, dc);
  run<32>(20, dA, dB, dO, db, dc);
  run<32>(30, dA, dB, dO, db, dc);
  return 0;
}
