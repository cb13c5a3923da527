// Microbenchmark: cost of each part of updateZ's paired truncated-normal draw (z_kernel.h
// z_probit_pair) at the synthetic shape (1e7 cells = 5e6 Philox pairs), in the product's
// occupancy (256 threads, <= 128 VGPRs).  The linear predictor comes from a 1024-entry LDS
// table shaped like the fitted probit chain (E ~ 3 N(0,1), Y = 1[E + N(0,1) > 0]).
//   V0 Philox + u53 only      V1 the whole pair draw      V2 pair draw, uniforms by a hash
//   V3 erfc part (both cells)  V4 log part                V5 central quantile polynomial
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <cmath>
#include <algorithm>
#include "../hmsc_amd/csrc/z_kernel.h"
using namespace hmsc;

constexpr int NTAB = 1024;

template <int V>
__global__ __launch_bounds__(256, 4) void parts_kernel(const double* Etab, const int* Ctab, int npairs, Key key,
                                                       double* out, const double* LT) {
  __shared__ double sE[NTAB];
  __shared__ int sC[NTAB];
  __shared__ double sLog[ZLOG_W * ZLOG_N];
  for (int p = threadIdx.x; p < NTAB; p += 256) sE[p] = Etab[p], sC[p] = Ctab[p];
  for (int p = threadIdx.x; p < ZLOG_W * ZLOG_N; p += 256) sLog[p] = LT[p];
  __syncthreads();
  double acc = 0.0;
  const int stride = gridDim.x * blockDim.x;
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < npairs; q += stride) {
    const int i0 = (2 * q) & (NTAB - 1), i1 = (2 * q + 1) & (NTAB - 1);
    const double e0 = sE[i0], e1 = sE[i1];
    const int c0 = sC[i0], c1 = sC[i1];
    Uniform2 u;
    if (V == 2 || V >= 3) {
      const uint32_t h = (uint32_t)q * 2654435761u;
      u.a = ((double)(h >> 8) + 0.5) * (1.0 / 16777216.0);
      u.b = ((double)((h * 747796405u) >> 8) + 0.5) * (1.0 / 16777216.0);
    } else {
      u = uniforms_wave_key(key, (uint32_t)q, 0, S_Z, 3u);
    }
    if (V == 0) {
      acc += u.a + u.b;
    } else if (V == 1 || V == 2) {
      const ZPair z = z_probit_pair(e0, e1, 1.0, 1.0, 1.0, 1.0, c0, c1, u.a, u.b, 0, sLog);
      acc += z.z0 + z.z1;
    } else if (V == 3) {
      const double h0 = e0 * 0.7071067811865476, h1 = e1 * 0.7071067811865476;
      const double a0 = fmin(fabs(h0), 40.0), a1 = fmin(fabs(h1), 40.0);
      const double t0 = 2.0 * rcp_pos(2.0 + a0), t1 = 2.0 * rcp_pos(2.0 + a1);
      const double x0 = 2.0 * t0 - 1.0, x1 = 2.0 * t1 - 1.0;
      double g0 = kErfcPoly[0], g1 = kErfcPoly[0];
#pragma unroll
      for (int k = 1; k < ERFC_NC; ++k) {
        g0 = fma_sc(g0, x0, kErfcPoly[k]);
        g1 = fma_sc(g1, x1, kErfcPoly[k]);
      }
      const double r0 = t0 * exp_small(fma(-a0, a0, g0)), r1 = t1 * exp_small(fma(-a1, a1, g1));
      acc += u.a * r0 + u.b * r1;
    } else if (V == 4) {
      acc += log_tab(u.a * e0 * e0 + 1e-3, sLog) + log_tab(u.b * e1 * e1 + 1e-3, sLog);
    } else if (V == 5) {
      const double y0 = u.a * 6.0 - 3.125, y1 = u.b * 6.0 - 3.125;
      double F0 = kQnormA[0], F1 = kQnormA[0];
#pragma unroll
      for (int k = 1; k < QNA_NC; ++k) {
        F0 = fma_sc(F0, y0, kQnormA[k]);
        F1 = fma_sc(F1, y1, kQnormA[k]);
      }
      acc += F0 + F1;
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

// accuracy of log_tab against the device libm log over x = 2^(-k / 64) (k < 64 * 1000) and
// x = 1 - j 2^-20 (j < 4096): max absolute and relative error
__global__ void logacc_kernel(const double* LT, double* out) {
  __shared__ double sLog[ZLOG_W * ZLOG_N];
  for (int p = threadIdx.x; p < ZLOG_W * ZLOG_N; p += blockDim.x) sLog[p] = LT[p];
  __syncthreads();
  double ea = 0.0, er = 0.0;
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < 64 * 1000 + 4096; k += gridDim.x * blockDim.x) {
    const double x = k < 64000 ? exp2(-k / 64.0 - 1e-7 * (k % 7)) : 1.0 - (k - 64000) * 0x1p-20;
    const double a = log_tab(x, sLog), b = log(x);
    ea = fmax(ea, fabs(a - b));
    if (b != 0.0) er = fmax(er, fabs(a - b) / fabs(b));
  }
  out[2 * (blockIdx.x * blockDim.x + threadIdx.x)] = ea;
  out[2 * (blockIdx.x * blockDim.x + threadIdx.x) + 1] = er;
}

static double* g_lt = nullptr;
template <int V>
float run(const double* E, const int* C, int npairs, double* out, int grid, int reps) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  parts_kernel<V><<<grid, 256>>>(E, C, npairs, Key{7u, 9u}, out, g_lt);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(a);
  for (int r = 0; r < reps; ++r) parts_kernel<V><<<grid, 256>>>(E, C, npairs, Key{7u, 9u}, out, g_lt);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms;
  (void)hipEventElapsedTime(&ms, a, b);
  return 1e3f * ms / reps;
}

int main() {
  std::vector<double> hE(NTAB);
  std::vector<int> hC(NTAB);
  unsigned s = 1;
  auto rnd = [&] { s = s * 1664525u + 1013904223u; return ((s >> 8) * (1.0 / 16777216.0)) - 0.5; };
  auto nrm = [&] { double t = 0; for (int q = 0; q < 12; ++q) t += rnd(); return t; };
  for (int p = 0; p < NTAB; ++p) {
    hE[p] = 3.0 * nrm();
    hC[p] = (hE[p] + nrm() > 0) ? 1 : 0;
  }
  double *E, *out;
  int* C;
  int ncu = 0;
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  const int grid = ncu * 4 * 3;  // three rounds of resident workgroups at 4 per CU
  (void)hipMalloc(&E, NTAB * 8);
  (void)hipMalloc(&C, NTAB * 4);
  (void)hipMalloc(&out, (size_t)grid * 256 * 8);
  (void)hipMemcpy(E, hE.data(), NTAB * 8, hipMemcpyHostToDevice);
  (void)hipMemcpy(C, hC.data(), NTAB * 4, hipMemcpyHostToDevice);
  {
    std::vector<double> lt(ZLOG_W * ZLOG_N);
    z_log_table(lt.data());
    (void)hipMalloc(&g_lt, lt.size() * 8);
    (void)hipMemcpy(g_lt, lt.data(), lt.size() * 8, hipMemcpyHostToDevice);
  }
  {
    double* acc;
    (void)hipMalloc(&acc, 2 * 64 * 256 * 8);
    logacc_kernel<<<64, 256>>>(g_lt, acc);
    std::vector<double> h(2 * 64 * 256);
    (void)hipMemcpy(h.data(), acc, h.size() * 8, hipMemcpyDeviceToHost);
    double ea = 0, er = 0;
    for (size_t q = 0; q < h.size(); q += 2) ea = std::max(ea, h[q]), er = std::max(er, h[q + 1]);
    printf("log_tab vs libm log: max abs err %.3e, max rel err %.3e\n", ea, er);
  }
  const int npairs = 5000000;
  printf("V0 philox+u53         %7.1f us\n", run<0>(E, C, npairs, out, grid, 20));
  printf("V1 pair draw          %7.1f us\n", run<1>(E, C, npairs, out, grid, 20));
  printf("V2 pair draw, hash u  %7.1f us\n", run<2>(E, C, npairs, out, grid, 20));
  printf("V3 erfc part          %7.1f us\n", run<3>(E, C, npairs, out, grid, 20));
  printf("V4 log part           %7.1f us\n", run<4>(E, C, npairs, out, grid, 20));
  printf("V5 central quantile   %7.1f us\n", run<5>(E, C, npairs, out, grid, 20));
  return 0;
}
