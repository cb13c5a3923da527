// Microbenchmark: cycles per single-workgroup dense primitive (n = 20) on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../hmsc_amd/csrc/common.h"
using namespace hmsc;

__global__ void bench(int n, int reps, long long* out, double* gsink) {
  extern __shared__ double lds[];
  __shared__ int flag;
  double* A = lds;
  double* B = A + n * n;
  double* C = B + n * n;
  double* W = C + n * n;
  const int t = threadIdx.x;
  for (int p = t; p < n * n; p += blockDim.x) {
    const int i = p % n, j = p / n;
    B[p] = (i == j ? n : 0.0) + 1.0 / (1 + i + j);
  }
  __syncthreads();
  long long t0, t1;
  // chol
  t0 = clock64();
  for (int r = 0; r < reps; ++r) {
    wg_copy(A, B, n * n);
    wg_chol(A, n, n, &flag);
  }
  t1 = clock64();
  if (t == 0) out[0] = (t1 - t0) / reps;
  // chol2inv
  t0 = clock64();
  for (int r = 0; r < reps; ++r) wg_chol2inv(A, n, n, C, n, W);
  t1 = clock64();
  if (t == 0) out[1] = (t1 - t0) / reps;
  // gemm
  t0 = clock64();
  for (int r = 0; r < reps; ++r) wg_gemm(n, n, n, 1.0, B, n, false, C, n, false, 0.0, W, n);
  t1 = clock64();
  if (t == 0) out[2] = (t1 - t0) / reps;
  // barrier
  t0 = clock64();
  for (int r = 0; r < reps; ++r) __syncthreads();
  t1 = clock64();
  if (t == 0) out[3] = (t1 - t0) / reps;
  // forward solve
  t0 = clock64();
  for (int r = 0; r < reps; ++r) wg_forward(A, n, n, W);
  t1 = clock64();
  if (t == 0) out[4] = (t1 - t0) / reps;
  if (t == 0) gsink[0] = C[5] + W[3];
}

int main() {
  long long* d;
  double* g;
  hipMalloc(&d, 8 * sizeof(long long));
  hipMalloc(&g, 8);
  for (int threads : {64, 256}) {
    for (int n : {10, 20, 30}) {
      hipLaunchKernelGGL(bench, dim3(1), dim3(threads), 4 * n * n * 8, 0, n, 20, d, g);
      long long h[8];
      hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
      printf("threads=%d n=%d  chol=%lld  chol2inv=%lld  gemm=%lld  barrier=%lld  forward=%lld cycles\n", threads, n,
             h[0], h[1], h[2], h[3], h[4]);
    }
  }
  int clk = 0;
  hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
  printf("clock64 rate attr (kHz): %d\n", clk);
  return 0;
}
