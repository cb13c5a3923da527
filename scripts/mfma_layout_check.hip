#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));
// D[16x16] = A[16x4] * B[4x16]; A[m][k]: lane l -> m = l&15, k = l>>4 ; B[k][n]: k = l>>4, n = l&15
__global__ void k(const double* A, const double* B, double* D) {
  int l = threadIdx.x;
  double a = A[(l & 15) * 4 + (l >> 4)];   // A row-major 16x4
  double b = B[(l >> 4) * 16 + (l & 15)];  // B row-major 4x16
  d4 acc = {0, 0, 0, 0};
  acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
  for (int r = 0; r < 4; ++r) D[((l >> 4) + 4 * r) * 16 + (l & 15)] = acc[r];  // row = (l>>4)+4r, col = l&15
}
int main() {
  double hA[64], hB[64], hD[256], ref[256];
  for (int i = 0; i < 64; ++i) { hA[i] = (i * 7) % 11 - 5; hB[i] = (i * 5) % 13 - 6; }
  for (int m = 0; m < 16; ++m) for (int n = 0; n < 16; ++n) { double s = 0; for (int q = 0; q < 4; ++q) s += hA[m*4+q]*hB[q*16+n]; ref[m*16+n] = s; }
  double *A, *B, *D; hipMalloc(&A, 512); hipMalloc(&B, 512); hipMalloc(&D, 2048);
  hipMemcpy(A, hA, 512, hipMemcpyHostToDevice); hipMemcpy(B, hB, 512, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, 1, 64, 0, 0, A, B, D);
  hipMemcpy(hD, D, 2048, hipMemcpyDeviceToHost);
  int bad = 0; for (int i = 0; i < 256; ++i) bad += hD[i] != ref[i];
  printf("mfma f64 16x16x4 layout check: %d mismatches\n", bad);
  return bad != 0;
}
