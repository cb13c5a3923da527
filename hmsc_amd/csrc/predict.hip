// predict.Hmsc on the device (R/predict.R:143-229): for every posterior
// sample s,
//   L_s = X Beta_s + sum_r Eta_r,s[Pi_r,] Lambda_r,s                               (:154-189)
//   expected:  probit pnorm(L), Poisson exp(L + sigma/2), normal L                  (:203-218)
//   draws:     Z = L + sqrt(sigma) N(0,1); probit 1[Z > 0], Poisson rpois(exp(Z))   (:198-218)
//   then the YScalePar back-transform Z s + m                                       (:222-227)
// out[s] is ny x ns column-major, as R's pred[[s]].
//
// One launch covers all samples: grid (site tiles, species tiles, samples); a workgroup
// stages the 64-site rows of [X | Eta_1[Pi_1,] | ...] and the K x 32 coefficient block
// [Beta_s; Lambda_1,s; ...] in LDS and writes a 64 x 32 output tile with coalesced
// 512-B site runs.  K = nc + sum nf is small (<= 64), so the kernel streams its output:
// the HBM bound is nsamples * ny * ns * 8 B of writes.
// Randomness: normal = inversion of the first uniform of (cell, 0, S_PREDICT, s), Poisson
// PTRS trial t uses (cell, 1 + t, S_PREDICT, s); cell = i + ny j (oracle predict_oracle).
#include <vector>

#include "../../include/hmsc_amd.h"
#include "common.h"
#include "rng.h"

namespace hmsc {

constexpr uint32_t S_PREDICT = 30;
constexpr int PT_I = 64, PT_J = 32, PK_MAX = HMSC_KCAP;

struct PredArgs {
  int ny, ns, nc, nr, nsamples, K, expected;
  int np[HMSC_MAX_LEVELS], nf[HMSC_MAX_LEVELS];
  const double* X;
  const double* Beta;    // nsamples x nc x ns
  const double* sigma;   // nsamples x ns
  const int* family;     // ns
  const double* yscale;  // 2 x ns
  const int* Pi;         // ny x nr, 0-based
  const double* Eta[HMSC_MAX_LEVELS];     // nsamples x np x nf
  const double* Lambda[HMSC_MAX_LEVELS];  // nsamples x nf x ns
  double* out;           // nsamples x ny x ns
  Key key;
};

// Poisson(lam) by PTRS (Hormann 1993, the transformed rejection numpy uses) for lam >= 10,
// sequential inversion below; uniforms from the cell's own counters
__device__ double rpois_dev(double lam, Key key, uint32_t cell, uint32_t s) {
  if (!(lam > 0.0)) return 0.0;
  if (lam < 10.0) {
    const double u = uniforms(key, cell, 1, S_PREDICT, s).a;
    double p = exp(-lam), c = p;
    int k = 0;
    while (u > c && k < 1000) {
      ++k;
      p *= lam / k;
      c += p;
    }
    return (double)k;
  }
  const double slam = sqrt(lam), loglam = log(lam);
  const double b = 0.931 + 2.53 * slam, a = -0.059 + 0.02483 * b;
  const double invalpha = 1.1239 + 1.1328 / (b - 3.4), vr = 0.9277 - 3.6224 / (b - 2.0);
  for (uint32_t t = 0; t < 256; ++t) {
    const Uniform2 uv = uniforms(key, cell, 1 + t, S_PREDICT, s);
    const double U = uv.a - 0.5, V = uv.b;
    const double us = 0.5 - fabs(U);
    const double k = floor((2.0 * a / us + b) * U + lam + 0.43);
    if (us >= 0.07 && V <= vr) return k;
    if (k < 0.0 || (us < 0.013 && V > us)) continue;
    if (log(V) + log(invalpha) - log(a / (us * us) + b) <= -lam + k * loglam - lgamma(k + 1.0)) return k;
  }
  return floor(lam);  // not reached in practice (acceptance ~0.9 per trial)
}

__global__ __launch_bounds__(256) void predict_kernel(PredArgs a) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int t = threadIdx.x, i0 = blockIdx.x * PT_I, j0 = blockIdx.y * PT_J, s = blockIdx.z;
  const int ny = a.ny, ns = a.ns, nc = a.nc, K = a.K;
  const int LD = K | 1;                 // odd: conflict-free column reads
  double* sA = smem;                    // [site][k], padded
  double* sB = smem + PT_I * LD;        // [k][species]
  for (int p = t; p < PT_I * K; p += 256) {
    const int ii = p % PT_I, k = p / PT_I, i = i0 + ii;
    double v = 0.0;
    if (i < ny) {
      if (k < nc) {
        v = a.X[i + (size_t)ny * k];
      } else {
        int kk = k - nc, r = 0;
        while (kk >= a.nf[r]) kk -= a.nf[r++];
        const int u = a.Pi[i + (size_t)ny * r];
        v = a.Eta[r][(size_t)s * a.np[r] * a.nf[r] + u + (size_t)a.np[r] * kk];
      }
    }
    sA[ii * LD + k] = v;
  }
  for (int p = t; p < K * PT_J; p += 256) {
    const int k = p / PT_J, jj = p % PT_J, j = j0 + jj;
    double v = 0.0;
    if (j < ns) {
      if (k < nc) {
        v = a.Beta[(size_t)s * nc * ns + k + (size_t)nc * j];
      } else {
        int kk = k - nc, r = 0;
        while (kk >= a.nf[r]) kk -= a.nf[r++];
        v = a.Lambda[r][(size_t)s * a.nf[r] * ns + kk + (size_t)a.nf[r] * j];
      }
    }
    sB[k * PT_J + jj] = v;
  }
  __syncthreads();
  const int ii = t & 63, jb = t >> 6;  // thread: site ii, species jb, jb+4, ..., jb+28
  const int i = i0 + ii;
  if (i >= ny) return;
  double acc[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) acc[q] = 0.0;
  for (int k = 0; k < K; ++k) {
    const double x = sA[ii * LD + k];
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[q] = fma(x, sB[k * PT_J + jb + 4 * q], acc[q]);
  }
  double* out = a.out + (size_t)s * ny * ns;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int j = j0 + jb + 4 * q;
    if (j >= ns) continue;
    const double L = acc[q];
    const double sg = a.sigma[(size_t)s * ns + j];
    const int fam = a.family[j];
    const uint32_t cell = (uint32_t)((size_t)i + (size_t)ny * j);
    double z;
    if (a.expected) {
      z = fam == 2 ? 0.5 * erfc_fast(-L * 0.7071067811865476) : fam == 3 ? exp(L + 0.5 * sg) : L;
    } else {
      z = fma(sqrt(sg), normal(a.key, cell, 0, S_PREDICT, (uint32_t)s), L);
      if (fam == 2) z = z > 0.0 ? 1.0 : 0.0;
      if (fam == 3) z = rpois_dev(exp(z), a.key, cell, (uint32_t)s);
    }
    const double m = a.yscale[2 * j], sd = a.yscale[2 * j + 1];
    if (m != 0.0 || sd != 1.0) z = fma(z, sd, m);
    out[i + (size_t)ny * j] = z;
  }
}

// host side: upload, one launch, download (called by hmsc_predict in capi.cpp)
void run_predict(const hmsc_predict_args* p, double* out) {
  HMSC_REQUIRE(p->nr >= 0 && p->nr <= HMSC_MAX_LEVELS, "predict: bad nr");
  int K = p->nc;
  for (int r = 0; r < p->nr; ++r) K += p->nf[r];
  HMSC_REQUIRE(K <= PK_MAX, "predict: nc + sum(nf) must be <= 128");
  HMSC_REQUIRE((size_t)p->ny * p->ns < ((size_t)1 << 32), "predict: ny * ns must fit 32-bit cell counters");
  HIP_OK(hipSetDevice(p->device));
  const size_t S = p->nsamples, ny = p->ny, ns = p->ns, nc = p->nc;
  std::vector<void*> bufs;
  auto up = [&](const void* src, size_t bytes) {
    void* d = nullptr;
    HIP_OK(hipMalloc(&d, std::max<size_t>(bytes, 8)));
    bufs.push_back(d);
    if (src && bytes) HIP_OK(hipMemcpy(d, src, bytes, hipMemcpyHostToDevice));
    return d;
  };
  PredArgs a{};
  a.ny = p->ny;
  a.ns = p->ns;
  a.nc = p->nc;
  a.nr = p->nr;
  a.nsamples = p->nsamples;
  a.K = K;
  a.expected = p->expected;
  a.X = (const double*)up(p->X, ny * nc * 8);
  a.Beta = (const double*)up(p->Beta, S * nc * ns * 8);
  a.sigma = (const double*)up(p->sigma, S * ns * 8);
  a.family = (const int*)up(p->family, ns * 4);
  a.yscale = (const double*)up(p->YScalePar, 2 * ns * 8);
  std::vector<int> pi0((size_t)ny * std::max(1, p->nr));
  for (int r = 0; r < p->nr; ++r) {
    a.np[r] = p->np[r];
    a.nf[r] = p->nf[r];
    for (size_t i = 0; i < ny; ++i) {
      const int u = p->Pi[i + ny * r] - 1;
      HMSC_REQUIRE(u >= 0 && u < p->np[r], "predict: Pi out of range");
      pi0[i + ny * r] = u;
    }
    a.Eta[r] = (const double*)up(p->Eta[r], S * p->np[r] * p->nf[r] * 8);
    a.Lambda[r] = (const double*)up(p->Lambda[r], S * p->nf[r] * ns * 8);
  }
  a.Pi = (const int*)up(pi0.data(), pi0.size() * 4);
  a.out = (double*)up(nullptr, S * ny * ns * 8);
  a.key = Key{(uint32_t)p->seed, (uint32_t)(p->seed >> 32)};
  if (S > 0) {
    dim3 grid((p->ny + PT_I - 1) / PT_I, (p->ns + PT_J - 1) / PT_J, p->nsamples);
    const size_t smem = ((size_t)PT_I * (K | 1) + (size_t)K * PT_J) * sizeof(double);
    predict_kernel<<<grid, 256, smem>>>(a);
    HIP_OK(hipGetLastError());
    HIP_OK(hipMemcpy(out, a.out, S * ny * ns * 8, hipMemcpyDeviceToHost));
  }
  for (void* d : bufs) (void)hipFree(d);
}

}  // namespace hmsc
