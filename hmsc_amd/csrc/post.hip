// Post-sampling statistics on the device: the per-sample loops of
// computeAssociations (R/computeAssociations.R), computeVariancePartitioning
// (R/computeVariancePartitioning.R:37-204) and coda::effectiveSize (spectrum0.ar, the ESS
// behind BASELINE's "Beta ESS/sec").  At ns = 1000 one posterior sample of Omega is 8 MB and
// X Beta 80 MB: these loops are reductions over samples of ns^2 / ny ns work each, so they run
// where the samples are small (Lambda, Beta, Gamma) and only the summaries come back.
// Every reduction is in a fixed order (samples in order, fixed lane trees): results repeat
// bit for bit.  The numpy restatements in oracle/post_oracle.py are the checkers.
#include <algorithm>
#include <cmath>
#include <vector>

#include "../../include/hmsc_amd.h"
#include "common.h"

namespace hmsc {

// ---------------------------------------------------------------------------------------
// computeAssociations: OmegaCor_s = cov2cor(Lambda_s' Lambda_s); mean over samples and
// support = mean(OmegaCor_s > 0); plus the posterior mean of Omega_s itself (getPostEstimate
// "Omega").  A 64 x 64 output tile per workgroup (16 x 16 threads, 4 x 4 outputs each); per
// sample the tile's two 64-species blocks of Lambda_s are staged in LDS.
// ---------------------------------------------------------------------------------------
constexpr int OT = 64, OF_MAX = HMSC_KCAP;

__global__ __launch_bounds__(256) void omega_assoc_kernel(int S, int ns, int nfmax, const int* nf, const double* Lam,
                                                           double* mean_cor, double* support, double* support_neg,
                                                           double* mean_omega) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  double* LI = smem;                // [h][species in block], h < nfmax
  double* LJ = smem + nfmax * OT;
  const int ntile = (ns + OT - 1) / OT;
  const int bi = blockIdx.x % ntile, bj = blockIdx.x / ntile;
  const int i0 = bi * OT, j0 = bj * OT, t = threadIdx.x, ti = t & 15, tj = t >> 4;
  double sc[4][4], sp[4][4], sn[4][4], so[4][4];
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int v = 0; v < 4; ++v) sc[u][v] = sp[u][v] = sn[u][v] = so[u][v] = 0.0;
  for (int s = 0; s < S; ++s) {
    const int f = nf[s];
    const double* L = Lam + (size_t)s * nfmax * ns;
    __syncthreads();
    for (int q = t; q < f * OT; q += 256) {
      const int h = q / OT, c = q - h * OT;
      LI[q] = i0 + c < ns ? L[h + (size_t)nfmax * (i0 + c)] : 0.0;
      LJ[q] = j0 + c < ns ? L[h + (size_t)nfmax * (j0 + c)] : 0.0;
    }
    __syncthreads();
    double o[4][4], di[4], dj[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      di[u] = dj[u] = 0.0;
#pragma unroll
      for (int v = 0; v < 4; ++v) o[u][v] = 0.0;
    }
    for (int h = 0; h < f; ++h) {
      double a[4], b[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        a[u] = LI[h * OT + ti + 16 * u];
        b[u] = LJ[h * OT + tj + 16 * u];
        di[u] = fma(a[u], a[u], di[u]);
        dj[u] = fma(b[u], b[u], dj[u]);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int v = 0; v < 4; ++v) o[u][v] = fma(a[u], b[v], o[u][v]);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        // cov2cor (its diagonal set to exactly 1, as R's)
        const double c = i0 + ti + 16 * u == j0 + tj + 16 * v ? 1.0 : o[u][v] / sqrt(di[u] * dj[v]);
        sc[u][v] += c;
        sp[u][v] += c > 0.0 ? 1.0 : 0.0;
        sn[u][v] += o[u][v] < 0.0 ? 1.0 : 0.0;
        so[u][v] += o[u][v];
      }
  }
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int i = i0 + ti + 16 * u, j = j0 + tj + 16 * v;
      if (i < ns && j < ns) {
        const size_t o = i + (size_t)ns * j;
        mean_cor[o] = sc[u][v] / S;
        support[o] = sp[u][v] / S;
        support_neg[o] = sn[u][v] / S;
        mean_omega[o] = so[u][v] / S;
      }
    }
}

// ---------------------------------------------------------------------------------------
// computeVariancePartitioning, one workgroup per posterior sample s:
//   mu = Gamma Tr' (nc x ns), R2T.Beta[k] += cor(Beta[k,], mu[k,])^2            (:126-128)
//   a = X mu, f = X Beta, rows centred over species; res1 = sum_i (a_i . f_i / (ns-1))^2,
//   res2 = sum_i |a_i|^2 |f_i|^2 / (ns-1)^2, R2T.Y += res1 / res2                (:133-141)
// With Mc, Bc the rows of mu, Beta centred over species, a_i - mean = x_i Mc and
// f_i - mean = x_i Bc exactly, so a_i . f_i = x_i (Mc Bc') x_i': three nc x nc Gram matrices
// replace the two ny x ns products (ny nc^2 instead of ny ns nc work; their diagonals are
// the sums of R2T.Beta's correlations).
//   fixed1[j] = Beta_j' cM Beta_j, fixedsplit1[j, g] over the group's rows / columns,
//   random1[j, r] = sum_h Lambda_r[h, j]^2, then the per-sample normalisations   (:142-173)
// The sample's terms go to a per-sample slot; vp_reduce_kernel adds them in sample order.
// ---------------------------------------------------------------------------------------
constexpr int VP_NC = HMSC_KCAP;
constexpr size_t VP_LDS_MAX = 150 * 1024;  // the three Gram matrices in LDS up to here, else global

struct VpArgs {
  int ny, ns, nc, nt, S, ngroups, nr;
  const int* group;      // nc, 1-based
  const double* X;       // ny x nc
  const double* Tr;      // ns x nt
  const double* cM;      // nc x nc
  const double* Beta;    // S x nc x ns
  const double* Gamma;   // S x nc x nt
  const int* nf;         // nr x S
  int nfmax[HMSC_MAX_LEVELS];
  const double* Lambda[HMSC_MAX_LEVELS];  // S x nfmax_r x ns
  double* work;          // S x slot
  size_t slot;           // doubles per sample: nc + 1 + ns (1 + nr + ngroups)
  double* gram;          // S x 3 nc^2 when they do not fit LDS (nc > 80), else null
};

__global__ __launch_bounds__(256) void vp_sample_kernel(VpArgs a) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  __shared__ double mB[VP_NC], mM[VP_NC], red[8];
  const int s = blockIdx.x, t = threadIdx.x, nc = a.nc, ns = a.ns, nt = a.nt;
  double* Cb = a.gram ? a.gram + (size_t)s * 3 * nc * nc : smem;
  double* C[3] = {Cb, Cb + (size_t)nc * nc, Cb + (size_t)2 * nc * nc};  // Mc Bc', Mc Mc', Bc Bc'

  const double* B = a.Beta + (size_t)s * nc * ns;
  const double* G = a.Gamma + (size_t)s * nc * nt;
  double* out = a.work + (size_t)s * a.slot;
  auto mu = [&](int k, int j) {
    double v = 0.0;
    for (int q = 0; q < nt; ++q) v = fma(G[k + (size_t)nc * q], a.Tr[j + (size_t)ns * q], v);
    return v;
  };
  // row means over species
  for (int k = t; k < nc; k += 256) {
    double sb = 0.0, sm = 0.0;
    for (int j = 0; j < ns; ++j) sb += B[k + (size_t)nc * j], sm += mu(k, j);
    mB[k] = sb / ns;
    mM[k] = sm / ns;
  }
  __syncthreads();
  for (int p = t; p < nc * nc; p += 256) {
    const int k = p % nc, l = p / nc;
    double caf = 0.0, caa = 0.0, cff = 0.0;
    for (int j = 0; j < ns; ++j) {
      const double mk = mu(k, j) - mM[k], ml = mu(l, j) - mM[l];
      const double bk = B[k + (size_t)nc * j] - mB[k], bl = B[l + (size_t)nc * j] - mB[l];
      caf = fma(mk, bl, caf);
      caa = fma(mk, ml, caa);
      cff = fma(bk, bl, cff);
    }
    C[0][p] = caf;
    C[1][p] = caa;
    C[2][p] = cff;
  }
  __syncthreads();
  for (int k = t; k < nc; k += 256)  // cor(Beta[k,], mu[k,])^2
    out[k] = C[0][k + nc * k] * C[0][k + nc * k] / (C[2][k + nc * k] * C[1][k + nc * k]);
  // per-site quadratic forms (sites strided over the threads, fixed order per thread)
  const double dn = 1.0 / (ns - 1);
  double r1 = 0.0, r2 = 0.0;
  for (int i = t; i < a.ny; i += 256) {
    double qaf = 0.0, qaa = 0.0, qff = 0.0;
    for (int l = 0; l < nc; ++l) {
      const double xl = a.X[i + (size_t)a.ny * l];
      double uaf = 0.0, uaa = 0.0, uff = 0.0;
      for (int k = 0; k < nc; ++k) {
        const double xk = a.X[i + (size_t)a.ny * k];
        uaf = fma(xk, C[0][k + nc * l], uaf);
        uaa = fma(xk, C[1][k + nc * l], uaa);
        uff = fma(xk, C[2][k + nc * l], uff);
      }
      qaf = fma(uaf, xl, qaf);
      qaa = fma(uaa, xl, qaa);
      qff = fma(uff, xl, qff);
    }
    qaf *= dn, qaa *= dn, qff *= dn;
    r1 = fma(qaf, qaf, r1);
    r2 = fma(qaa, qff, r2);
  }
  for (int o = 32; o > 0; o >>= 1) r1 += __shfl_xor(r1, o), r2 += __shfl_xor(r2, o);
  if ((t & 63) == 0) red[t >> 6] = r1, red[4 + (t >> 6)] = r2;
  __syncthreads();
  if (t == 0) out[nc] = ((red[0] + red[1]) + (red[2] + red[3])) / ((red[4] + red[5]) + (red[6] + red[7]));
  // species terms
  double* fx = out + nc + 1;            // ns
  double* rnd = fx + ns;                // nr x ns
  double* fsp = rnd + (size_t)a.nr * ns;  // ngroups x ns
  for (int j = t; j < ns; j += 256) {
    const double* b = B + (size_t)nc * j;
    double f1 = 0.0;
    for (int l = 0; l < nc; ++l) {
      double u = 0.0;
      for (int k = 0; k < nc; ++k) u = fma(a.cM[k + (size_t)nc * l], b[k], u);
      f1 = fma(u, b[l], f1);
    }
    double fsum = 0.0;
    for (int g = 1; g <= a.ngroups; ++g) {  // Beta[sel, j]' cM[sel, sel] Beta[sel, j]
      double fg = 0.0;
      for (int l = 0; l < nc; ++l) {
        if (a.group[l] != g) continue;
        double u = 0.0;
        for (int k = 0; k < nc; ++k)
          if (a.group[k] == g) u = fma(a.cM[k + (size_t)nc * l], b[k], u);
        fg = fma(u, b[l], fg);
      }
      fsp[(size_t)(g - 1) * ns + j] = fg;
      fsum += fg;
    }
    for (int g = 0; g < a.ngroups; ++g) fsp[(size_t)g * ns + j] /= fsum;
    double tot = f1;
    for (int r = 0; r < a.nr; ++r) {
      const int f = a.nf[r * a.S + s];
      const double* lam = a.Lambda[r] + (size_t)s * a.nfmax[r] * ns + (size_t)a.nfmax[r] * j;
      double v = 0.0;
      for (int h = 0; h < f; ++h) v = fma(lam[h], lam[h], v);
      rnd[(size_t)r * ns + j] = v;
      tot += v;
    }
    fx[j] = a.nr > 0 ? f1 / tot : 1.0;
    for (int r = 0; r < a.nr; ++r) rnd[(size_t)r * ns + j] /= tot;
  }
}

// sum over samples in order, divided by S; out: [R2T.Beta (nc) | R2T.Y | fixed (ns) |
// random (nr x ns) | fixedsplit (ngroups x ns)]
__global__ __launch_bounds__(256) void vp_reduce_kernel(const double* work, size_t slot, int S, double* out) {
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= slot) return;
  double v = 0.0;
  for (int s = 0; s < S; ++s) v += work[(size_t)s * slot + e];
  out[e] = v / S;
}

// ---------------------------------------------------------------------------------------
// coda::effectiveSize = n var(x) / spectrum0.ar(x)$spec per column (one wave per column):
// linear-trend residual check, autocovariances to order.max = min(n - 1, 10 log10 n),
// Levinson-Durbin (R's eureka), AIC order choice, var.pred / (1 - sum ar)^2.
// ---------------------------------------------------------------------------------------
constexpr int ESS_OMAX = 64;

__device__ __forceinline__ double wave_sum(double v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

__global__ __launch_bounds__(256) void ess_kernel(int n, int p, const double* x, double* ess, int* order_out) {
  __shared__ double rr[4][ESS_OMAX + 1];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int col = blockIdx.x * 4 + w;
  if (col >= p) return;  // whole waves exit together: no workgroup barrier below
  const double* c = x + (size_t)n * col;
  double s = 0.0, amax = 0.0;
  for (int i = lane; i < n; i += 64) s += c[i], amax = fmax(amax, fabs(c[i]));
  const double mean = wave_sum(s) / n;
  for (int o = 32; o > 0; o >>= 1) amax = fmax(amax, __shfl_xor(amax, o));
  const double zm = 0.5 * (n + 1);
  double szx = 0.0, szz = 0.0, sxx = 0.0;
  for (int i = lane; i < n; i += 64) {
    const double zc = (i + 1) - zm, xc = c[i] - mean;
    szx = fma(zc, xc, szx);
    szz = fma(zc, zc, szz);
    sxx = fma(xc, xc, sxx);
  }
  szx = wave_sum(szx), szz = wave_sum(szz), sxx = wave_sum(sxx);
  const double beta = szx / szz;
  double srr = 0.0, srm = 0.0;
  for (int i = lane; i < n; i += 64) srm += (c[i] - mean) - ((i + 1) - zm) * beta;
  srm = wave_sum(srm) / n;
  for (int i = lane; i < n; i += 64) {
    const double rsd = (c[i] - mean) - ((i + 1) - zm) * beta - srm;
    srr = fma(rsd, rsd, srr);
  }
  srr = wave_sum(srr);
  const bool constant = sqrt(srr / (n - 1)) <= 1.5e-8 * fmax(amax, 1e-300);
  const int omax = min(min(n - 1, (int)floor(10.0 * log10((double)n))), ESS_OMAX);
  for (int k = 0; k <= omax; ++k) {
    double v = 0.0;
    for (int i = lane; i + k < n; i += 64) v = fma(c[i] - mean, c[i + k] - mean, v);
    v = wave_sum(v);
    if (lane == 0) rr[w][k] = v / n;
  }
  __builtin_amdgcn_wave_barrier();
  if (lane != 0) return;
  const double* r = rr[w];
  const double r0 = r[0] > 0.0 ? r[0] : 1.0;
  double a[ESS_OMAX + 1], an[ESS_OMAX + 1], asum[ESS_OMAX + 1], vars[ESS_OMAX + 1];
  for (int m = 0; m <= omax; ++m) a[m] = 0.0;
  double v = r0;
  vars[0] = r0;
  asum[0] = 0.0;
  for (int m = 1; m <= omax; ++m) {
    double acc = r[m];
    for (int j = 1; j < m; ++j) acc -= a[j] * r[m - j];
    const double k = acc / v;
    for (int j = 1; j < m; ++j) an[j] = a[j] - k * a[m - j];
    for (int j = 1; j < m; ++j) a[j] = an[j];
    a[m] = k;
    v = v * (1.0 - k * k);
    vars[m] = v;
    double sm = 0.0;
    for (int j = 1; j <= m; ++j) sm += a[j];
    asum[m] = sm;
  }
  // order = which.min(xaic) as numpy's argmin: the first NaN if any, else the first minimum
  int order = 0;
  double best = INFINITY;
  bool seen_val = false;
  for (int m = 0; m <= omax; ++m) {
    const double xa = n * log(vars[m]) + 2.0 * m + 2.0;
    if (xa != xa) {
      order = m;
      break;
    }
    if (!seen_val || xa < best) best = xa, order = m, seen_val = true;
  }
  const double var_pred = vars[order] * n / (n - (order + 1));
  const double spec = constant ? 0.0 : var_pred / ((1.0 - asum[order]) * (1.0 - asum[order]));
  const double var = sxx / (n - 1);
  ess[col] = spec == 0.0 ? 0.0 : n * var / spec;
  if (order_out) order_out[col] = order;
}

struct PostBufs {
  std::vector<void*> p;
  template <class T>
  T* alloc(size_t n) {
    void* q = nullptr;
    HIP_OK(hipMalloc(&q, std::max<size_t>(1, n) * sizeof(T)));
    p.push_back(q);
    return static_cast<T*>(q);
  }
  template <class T>
  T* up(const T* h, size_t n, hipStream_t st) {
    T* d = alloc<T>(n);
    if (n) HIP_OK(hipMemcpyAsync(d, h, n * sizeof(T), hipMemcpyHostToDevice, st));
    return d;
  }
  ~PostBufs() {
    for (void* q : p) (void)hipFree(q);
  }
};
struct PostStream {
  hipStream_t s = nullptr;
  PostStream() { HIP_OK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking)); }
  ~PostStream() {
    (void)hipStreamSynchronize(s);
    (void)hipStreamDestroy(s);
  }
};

void post_omega(int device, int S, int ns, int nfmax, const int* nf, const double* Lambda, double* mean_cor,
                double* support, double* support_neg, double* mean_omega) {
  HMSC_REQUIRE(S > 0 && ns > 0 && nfmax > 0 && nfmax <= OF_MAX && nf && Lambda && mean_cor && support && support_neg &&
                   mean_omega,
               "hmsc_post_omega: bad arguments (nfmax <= 128)");
  for (int s = 0; s < S; ++s) HMSC_REQUIRE(nf[s] >= 1 && nf[s] <= nfmax, "hmsc_post_omega: nf out of range");
  HIP_OK(hipSetDevice(device));
  PostBufs b;  // before the stream: the stream drains before the buffers are freed
  PostStream ps;
  const size_t n2 = (size_t)ns * ns;
  const int* dnf = b.up(nf, S, ps.s);
  const double* dL = b.up(Lambda, (size_t)S * nfmax * ns, ps.s);
  double *mc = b.alloc<double>(n2), *sp = b.alloc<double>(n2), *sn = b.alloc<double>(n2), *mo = b.alloc<double>(n2);
  const int nt = (ns + OT - 1) / OT;
  omega_assoc_kernel<<<nt * nt, 256, (size_t)2 * nfmax * OT * sizeof(double), ps.s>>>(S, ns, nfmax, dnf, dL, mc, sp, sn,
                                                                                     mo);
  HIP_OK(hipGetLastError());
  HIP_OK(hipMemcpyAsync(mean_cor, mc, n2 * sizeof(double), hipMemcpyDeviceToHost, ps.s));
  HIP_OK(hipMemcpyAsync(support, sp, n2 * sizeof(double), hipMemcpyDeviceToHost, ps.s));
  HIP_OK(hipMemcpyAsync(support_neg, sn, n2 * sizeof(double), hipMemcpyDeviceToHost, ps.s));
  HIP_OK(hipMemcpyAsync(mean_omega, mo, n2 * sizeof(double), hipMemcpyDeviceToHost, ps.s));
  HIP_OK(hipStreamSynchronize(ps.s));
}

void post_vp(const hmsc_vp_args* v, double* out) {
  HMSC_REQUIRE(v && out && v->ny > 1 && v->ns > 1 && v->nc >= 1 && v->nc <= VP_NC && v->nt >= 1 && v->S >= 1 &&
                   v->ngroups >= 1 && v->ngroups <= VP_NC && v->nr >= 0 && v->nr <= HMSC_MAX_LEVELS,
               "hmsc_variance_partitioning: bad dimensions (nc, ngroups <= 128)");
  for (int k = 0; k < v->nc; ++k)
    HMSC_REQUIRE(v->group[k] >= 1 && v->group[k] <= v->ngroups, "hmsc_variance_partitioning: group out of range");
  HIP_OK(hipSetDevice(v->device));
  PostBufs b;
  PostStream ps;
  VpArgs a{};
  a.ny = v->ny, a.ns = v->ns, a.nc = v->nc, a.nt = v->nt, a.S = v->S, a.ngroups = v->ngroups, a.nr = v->nr;
  a.group = b.up(v->group, a.nc, ps.s);
  a.X = b.up(v->X, (size_t)a.ny * a.nc, ps.s);
  a.Tr = b.up(v->Tr, (size_t)a.ns * a.nt, ps.s);
  a.cM = b.up(v->cM, (size_t)a.nc * a.nc, ps.s);
  a.Beta = b.up(v->Beta, (size_t)a.S * a.nc * a.ns, ps.s);
  a.Gamma = b.up(v->Gamma, (size_t)a.S * a.nc * a.nt, ps.s);
  a.nf = b.up(v->nf, (size_t)std::max(1, a.nr) * a.S, ps.s);
  for (int r = 0; r < a.nr; ++r) {
    a.nfmax[r] = v->nfmax[r];
    a.Lambda[r] = b.up(v->Lambda[r], (size_t)a.S * v->nfmax[r] * a.ns, ps.s);
  }
  a.slot = (size_t)a.nc + 1 + (size_t)a.ns * (1 + a.nr + a.ngroups);
  a.work = b.alloc<double>(a.slot * a.S);
  const size_t gram_bytes = (size_t)3 * a.nc * a.nc * sizeof(double);
  a.gram = gram_bytes > VP_LDS_MAX ? b.alloc<double>((size_t)a.S * 3 * a.nc * a.nc) : nullptr;
  vp_sample_kernel<<<a.S, 256, a.gram ? 0 : gram_bytes, ps.s>>>(a);
  double* dout = b.alloc<double>(a.slot);
  vp_reduce_kernel<<<(unsigned)((a.slot + 255) / 256), 256, 0, ps.s>>>(a.work, a.slot, a.S, dout);
  HIP_OK(hipGetLastError());
  HIP_OK(hipMemcpyAsync(out, dout, a.slot * sizeof(double), hipMemcpyDeviceToHost, ps.s));
  HIP_OK(hipStreamSynchronize(ps.s));
}

void post_ess(int device, int n, int p, const double* x, double* ess, int* order) {
  HMSC_REQUIRE(n >= 3 && p >= 1 && x && ess, "hmsc_effective_size: bad arguments (n >= 3)");
  HIP_OK(hipSetDevice(device));
  PostBufs b;
  PostStream ps;
  const double* dx = b.up(x, (size_t)n * p, ps.s);
  double* de = b.alloc<double>(p);
  int* dord = b.alloc<int>(p);
  ess_kernel<<<(p + 3) / 4, 256, 0, ps.s>>>(n, p, dx, de, dord);
  HIP_OK(hipGetLastError());
  HIP_OK(hipMemcpyAsync(ess, de, (size_t)p * sizeof(double), hipMemcpyDeviceToHost, ps.s));
  if (order) HIP_OK(hipMemcpyAsync(order, dord, (size_t)p * sizeof(int), hipMemcpyDeviceToHost, ps.s));
  HIP_OK(hipStreamSynchronize(ps.s));
}

}  // namespace hmsc
