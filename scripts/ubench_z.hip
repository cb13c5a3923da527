// Microbenchmark of the fused updateZ kernel (hmsc_amd/csrc/z_kernel.h) at the synthetic
// shape ny=10000, ns=1000, K=30, with parts switched off (MODE bits) to cost each of them.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
#include <cmath>
#include "../hmsc_amd/csrc/z_kernel.h"
using namespace hmsc;

template <int MODE>
float run(const ZArgs& a, dim3 grid, size_t smem, int reps) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  auto k = z_wave_kernel<true, false, 2, MODE, false, false>;
  k<<<grid, 256, smem>>>(a);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0);
  for (int i = 0; i < reps; ++i) k<<<grid, 256, smem>>>(a);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  return 1e3f * ms / reps;
}

int main(int argc, char** argv) {
  const bool prof_only = argc > 1 && argv[1][0] == 'p';
  const int ny = 10000, ns = 1000, K = 30, nt = 1;
  std::vector<double> hX((size_t)ny * K), hBL((size_t)K * ns), hTr(ns, 1.0), hIs(ns, 1.0);
  std::vector<int8_t> hY((size_t)ny * ns);
  std::vector<int> hF(ns, 2);
  unsigned s = 1;
  auto rnd = [&] { s = s * 1664525u + 1013904223u; return ((s >> 8) * (1.0 / 16777216.0)) - 0.5; };
  // like the synthetic probit chain: E = XEta BL with sd ~3, Y = 1[E + N(0,1) > 0]
  auto nrm = [&] { double t = 0; for (int q = 0; q < 12; ++q) t += rnd(); return t; };
  for (auto& v : hX) v = nrm();
  for (auto& v : hBL) v = 0.55 * nrm();
  for (int j = 0; j < ns; ++j)
    for (int i = 0; i < ny; ++i) {
      double e = 0;
      for (int k = 0; k < K; ++k) e += hX[i + (size_t)ny * k] * hBL[k + (size_t)K * j];
      hY[i + (size_t)ny * j] = (e + nrm() > 0) ? 1 : 0;
    }
  double *X, *BL, *Tr, *Is, *Z, *XZp, *ZTrp;
  int8_t* Y;
  int* F;
  const int ntile_j = (ns + 31) / 32, n_tiles = (ny + 63) / 64;
  // XEta padded as the product's (z_kernel.h ZArgs: 16 ceil(K / 16) columns + 64)
  (void)hipMalloc(&X, ((size_t)ny * 16 * ((K + 15) / 16) + 64) * 8);
  (void)hipMemset(X, 0, ((size_t)ny * 16 * ((K + 15) / 16) + 64) * 8);
  std::vector<uint64_t> hYb((size_t)ntile_j * ny + 64, 0x5555555555555555ull);
  for (int j = 0; j < ns; ++j)
    for (int i = 0; i < ny; ++i) {
      uint64_t& w = hYb[(size_t)(j / 32) * ny + i];
      const int sh = 2 * (j % 32);
      w = (w & ~(3ull << sh)) | ((uint64_t)(hY[i + (size_t)ny * j] + 1) << sh);
    }
  uint64_t* Yb;
  (void)hipMalloc(&Yb, hYb.size() * 8);
  (void)hipMemcpy(Yb, hYb.data(), hYb.size() * 8, hipMemcpyHostToDevice);
  (void)hipMalloc(&BL, hBL.size() * 8);
  (void)hipMalloc(&Tr, ns * 8);
  (void)hipMalloc(&Is, ns * 8);
  (void)hipMalloc(&Z, (size_t)ny * ns * 8);
  (void)hipMalloc(&Y, (size_t)ny * (ns + 32) + 64);
  (void)hipMalloc(&F, ns * 4);
  (void)hipMalloc(&XZp, (size_t)n_tiles * K * ns * 8);
  (void)hipMalloc(&ZTrp, (size_t)ntile_j * ny * 8);
  (void)hipMemcpy(X, hX.data(), hX.size() * 8, hipMemcpyHostToDevice);
  (void)hipMemcpy(BL, hBL.data(), hBL.size() * 8, hipMemcpyHostToDevice);
  (void)hipMemcpy(Tr, hTr.data(), ns * 8, hipMemcpyHostToDevice);
  (void)hipMemcpy(Is, hIs.data(), ns * 8, hipMemcpyHostToDevice);
  (void)hipMemcpy(Y, hY.data(), hY.size(), hipMemcpyHostToDevice);
  (void)hipMemcpy(F, hF.data(), ns * 4, hipMemcpyHostToDevice);
  double* LT;
  {
    std::vector<double> lt(4 * ZLOG_N);
    z_log_table(lt.data());
    (void)hipMalloc(&LT, lt.size() * 8);
    (void)hipMemcpy(LT, lt.data(), lt.size() * 8, hipMemcpyHostToDevice);
  }
  uint32_t* dIter;
  (void)hipMalloc(&dIter, 4);
  { const uint32_t three = 3; (void)hipMemcpy(dIter, &three, 4, hipMemcpyHostToDevice); }
  const size_t smem = z_smem_bytes(K, nt);
  int nb = 0, ncu = 0;
  (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, z_wave_kernel<true, false, 2, Z_ALL, false, false>, 256, smem);
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  printf("occupancy %d blocks/CU, %d CUs, smem %zu B\n", nb, ncu, smem);
  for (int nchunk_req : {nb * ncu / ntile_j, 3 * nb * ncu / ntile_j}) {
    ZArgs a{};
    a.XEta = X; a.ny = ny; a.K = K; a.ns_loc = ns; a.sp0 = 0; a.nt = nt;
    a.tiles_per_chunk = (n_tiles + nchunk_req - 1) / nchunk_req;
    const int nchunk = (n_tiles + a.tiles_per_chunk - 1) / a.tiles_per_chunk;
    a.BL = BL; a.iSigma = Is; a.Ycode = Y; a.Ybits = Yb; a.Yval = nullptr; a.fam = F; a.Tr = Tr; a.Z = Z;
    a.XZ_part = XZp; a.ZTr_part = ZTrp; a.key = Key{7u, 9u}; a.iter = 3; a.noise_zero = 0;
    a.iter_dev = dIter;  // as in the product's graph replays
    a.logtab = LT;
    dim3 grid(ntile_j, nchunk);
    printf("grid %d x %d (tiles/chunk %d)\n", nchunk, ntile_j, a.tiles_per_chunk);
    if (prof_only) {
      printf("  product (MODE 7)    %7.1f us\n", run<7>(a, grid, smem, 20));
      return 0;
    }
    printf("  product (MODE 7)    %7.1f us\n", run<7>(a, grid, smem, 20));
    printf("  product, no stores  %7.1f us\n", run<7 | 16>(a, grid, smem, 20));
    printf("  no XZ               %7.1f us\n", run<3>(a, grid, smem, 20));
    printf("  no draw             %7.1f us\n", run<5>(a, grid, smem, 20));
    printf("  draw only (E VALU)  %7.1f us\n", run<2>(a, grid, smem, 20));
    printf("  nothing             %7.1f us\n", run<0>(a, grid, smem, 20));
    printf("  nothing, no stores  %7.1f us\n", run<16>(a, grid, smem, 20));
    run<7>(a, grid, smem, 1);
    std::vector<double> hz((size_t)ny * ns);
    (void)hipMemcpy(hz.data(), Z, hz.size() * 8, hipMemcpyDeviceToHost);
    double cs = 0, ca = 0;
    for (size_t q = 0; q < hz.size(); ++q) cs += hz[q], ca += std::fabs(hz[q]) * (1 + (q % 7));
    printf("  checksum Z %.15e %.15e  z[12345] %.17g\n", cs, ca, hz[12345]);
    std::vector<double> hp((size_t)nchunk * K * ns);
    (void)hipMemcpy(hp.data(), XZp, hp.size() * 8, hipMemcpyDeviceToHost);
    double px = 0;
    for (size_t q = 0; q < hp.size(); ++q) px += hp[q] * (1 + (q % 5));
    printf("  checksum XZ partials %.15e\n", px);
  }
  return 0;
}
