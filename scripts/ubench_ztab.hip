// Microbenchmark: the z draw with the round-5 LDS tables (z_kernel.h z_probit_pair_tab) against
// the global-polynomial draw (z_probit_pair) at the synthetic shape (1e7 cells = 5e6 Philox
// pairs), in the product's occupancy (256 threads, 4 workgroups per CU, <= 128 VGPRs).  The
// linear predictor comes from a 1024-entry LDS table shaped like the fitted probit chain
// (E ~ 3 N(0,1), Y = 1[E + N(0,1) > 0]).
//   V0 Philox + u53      V1 old pair draw     V2 table pair draw
//   V3 table erfc part   V4 table quantile    V5 log part
// build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -mllvm -disable-machine-licm scripts/ubench_ztab.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <vector>
#include "../hmsc_amd/csrc/z_kernel.h"
using namespace hmsc;

constexpr int NTAB = 1024;

template <int V>
__global__ __launch_bounds__(256, 4) void zt_kernel(const double* Etab, const int* Ctab, int npairs, Key key,
                                                    double* out, const double* LT) {
  __shared__ double sE[NTAB];
  __shared__ int sC[NTAB];
  __shared__ __attribute__((aligned(16))) double sLog[ZLOG_W * ZLOG_N + ZT_DOUBLES];
  __shared__ double pad[2048];  // (the product kernel's other LDS: 4 workgroups per CU)
  for (int p = threadIdx.x; p < NTAB; p += 256) sE[p] = Etab[p], sC[p] = Ctab[p];
  for (int p = threadIdx.x; p < ZLOG_W * ZLOG_N + ZT_DOUBLES; p += 256) sLog[p] = LT[p];
  if (threadIdx.x == 0) pad[0] = 0.0;
  __syncthreads();
  const double* sZT = sLog + ZLOG_W * ZLOG_N;
  double acc = pad[threadIdx.x & 1];
  const int stride = gridDim.x * blockDim.x;
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < npairs; q += stride) {
    const int i0 = (2 * q) & (NTAB - 1), i1 = (2 * q + 1) & (NTAB - 1);
    const double e0 = sE[i0], e1 = sE[i1];
    const int c0 = sC[i0], c1 = sC[i1];
    const Uniform2 u = uniforms_wave_key(key, (uint32_t)q, 0, S_Z, 3u);
    if (V == 0) {
      acc += u.a + u.b;
    } else if (V == 1) {
      const ZPair z = z_probit_pair(e0, e1, 1.0, 1.0, 1.0, 1.0, c0, c1, u.a, u.b, 0, sLog);
      acc += z.z0 + z.z1;
    } else if (V == 2) {
      const ZPair z = z_probit_pair_tab(e0, e1, 1.0, 1.0, 1.0, 1.0, c0, c1, u.a, u.b, 0, sLog, sZT);
      acc += z.z0 + z.z1;
    } else if (V == 3) {
      const double a0 = fmin(fabs(e0) * 0.7071067811865476 * u.a, 17.99), a1 = fmin(fabs(e1) * 0.7071067811865476 * u.b, 17.99);
      acc += zt_erfc(a0, sZT) + zt_erfc(a1, sZT);
    } else if (V == 4) {
      const double w0 = 6.0 * u.a * fabs(e0), w1 = 6.0 * u.b * fabs(e1);
      acc += zt_qnorm_w(u.a, fmin(w0, 15.9), sZT) + zt_qnorm_w(u.b, fmin(w1, 15.9), sZT);
    } else if (V == 5) {
      acc += log_tab(u.a * e0 * e0 + 1e-3, sLog) + log_tab(u.b * e1 * e1 + 1e-3, sLog);
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

// accuracy of the table draw against the global-polynomial draw over the same (E, code, u)
__global__ void zt_acc_kernel(const double* Etab, const int* Ctab, int npairs, Key key, double* out, const double* LT) {
  __shared__ __attribute__((aligned(16))) double sLog[ZLOG_W * ZLOG_N + ZT_DOUBLES];
  for (int p = threadIdx.x; p < ZLOG_W * ZLOG_N + ZT_DOUBLES; p += blockDim.x) sLog[p] = LT[p];
  __syncthreads();
  double er = 0.0;
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < npairs; q += gridDim.x * blockDim.x) {
    const int i0 = (2 * q) & (NTAB - 1), i1 = (2 * q + 1) & (NTAB - 1);
    const Uniform2 u = uniforms_wave_key(key, (uint32_t)q, 0, S_Z, 3u);
    const double e0 = Etab[i0] * (1.0 + 0.37 * u.b), e1 = Etab[i1] * (1.0 - 0.29 * u.a);
    const ZPair a = z_probit_pair(e0, e1, 1.0, 1.0, 1.0, 1.0, Ctab[i0], Ctab[i1], u.a, u.b, 0, sLog);
    const ZPair b = z_probit_pair_tab(e0, e1, 1.0, 1.0, 1.0, 1.0, Ctab[i0], Ctab[i1], u.a, u.b, 0, sLog,
                                      sLog + ZLOG_W * ZLOG_N);
    er = fmax(er, fabs(a.z0 - b.z0) / fmax(1.0, fabs(a.z0)));
    er = fmax(er, fabs(a.z1 - b.z1) / fmax(1.0, fabs(a.z1)));
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = er;
}

static double* g_lt = nullptr;
template <int V>
float run(const double* E, const int* C, int npairs, double* out, int grid, int reps) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  zt_kernel<V><<<grid, 256>>>(E, C, npairs, Key{7u, 9u}, out, g_lt);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(a);
  for (int r = 0; r < reps; ++r) zt_kernel<V><<<grid, 256>>>(E, C, npairs, Key{7u, 9u}, out, g_lt);
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
  const int grid = ncu * 4 * 3;
  (void)hipMalloc(&E, NTAB * 8);
  (void)hipMalloc(&C, NTAB * 4);
  (void)hipMalloc(&out, (size_t)grid * 256 * 8);
  (void)hipMemcpy(E, hE.data(), NTAB * 8, hipMemcpyHostToDevice);
  (void)hipMemcpy(C, hC.data(), NTAB * 4, hipMemcpyHostToDevice);
  {
    std::vector<double> lt(ZLOG_W * ZLOG_N + ZT_DOUBLES);
    z_log_table(lt.data());
    z_draw_tables(lt.data() + ZLOG_W * ZLOG_N);
    (void)hipMalloc(&g_lt, lt.size() * 8);
    (void)hipMemcpy(g_lt, lt.data(), lt.size() * 8, hipMemcpyHostToDevice);
  }
  const int npairs = 5000000;
  {
    zt_acc_kernel<<<grid, 256>>>(E, C, npairs, Key{7u, 9u}, out, g_lt);
    std::vector<double> h((size_t)grid * 256);
    (void)hipMemcpy(h.data(), out, h.size() * 8, hipMemcpyDeviceToHost);
    printf("table draw vs global-polynomial draw: max rel diff %.3e over %d pairs\n",
           *std::max_element(h.begin(), h.end()), npairs);
  }
  printf("V0 philox+u53          %7.1f us\n", run<0>(E, C, npairs, out, grid, 20));
  printf("V1 old pair draw       %7.1f us\n", run<1>(E, C, npairs, out, grid, 20));
  printf("V2 table pair draw     %7.1f us\n", run<2>(E, C, npairs, out, grid, 20));
  printf("V3 table erfc          %7.1f us\n", run<3>(E, C, npairs, out, grid, 20));
  printf("V4 table quantile      %7.1f us\n", run<4>(E, C, npairs, out, grid, 20));
  printf("V5 log part            %7.1f us\n", run<5>(E, C, npairs, out, grid, 20));
  return 0;
}
