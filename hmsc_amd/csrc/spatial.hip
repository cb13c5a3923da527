// Spatial latent factors, method "Full" (SURVEY.md §8 f2), on the device.
//
// updateEta, spatial branch (R/updateEta.R:111-140): for a level with np units and nf
// factors, one dense system in the vec(np x nf) ordering (unit fastest)
//   iUEta = bdiag(iWg[,,alpha_1], ..., iWg[,,alpha_nf]) + kron(Lam D Lam', diag(n_p))
//   fS    = P'S (Lam diag(iSigma))',  S = Z - X Beta - other levels' Eta Lambda
//   eta   = R^-1 (R^-T vec(fS) + xi),  R = chol(iUEta)
// np = ny (observation-level, P a permutation) and np < ny are the same formula.
// updateAlpha (R/updateAlpha.R:20-79, 'Full'): v_gh = |RiWg[,,g] eta_h|^2 for every grid
// point g, log-likelihood log(alphapw[g,2]) - detWg[g]/2 - v_gh/2, categorical draw.
//
// Layout in HBM: the alphapw grid arrays iWg / RiWg (np^2 x nalpha each, column-major as R
// holds them) stay resident for the whole chain -- at np = 5000 and 101 grid points that is
// 20 GB per array, which 288 GB of HBM holds -- so no sweep ever recomputes a grid matrix.
// The grid is either uploaded (computeDataParameters' arrays) or, for 'Full' levels given
// by coordinates / distances, built in place by spatial_full_grid (chol, trtri, lauum on
// the matrix cores, dense.hip).  The Eta system is one workgroup with the shared wg_*
// Cholesky up to np nf = 1024 and the blocked multi-workgroup Cholesky above;
// updateAlpha's nalpha x nf quadratic forms stream each grid matrix once over
// nalpha x ceil(np / 256) workgroups (the HBM-bound step at large np).
// Randomness (oracle/hmsc_oracle.py _eta_spatial_full / update_alpha): Eta normal(p, h,
// S_ETA + LEVEL_STRIDE r) -- the same counters as the non-spatial branch --, Alpha the first
// uniform of (h, 0, S_ALPHA + LEVEL_STRIDE r).
#include <algorithm>
#include <cmath>
#include <thread>
#include <utility>
#include <vector>

#include "common.h"
#include "state.h"

namespace hmsc {

// factor capacity of a spatial level's workspace layout (sp_ensure_capacity)
static inline int sp_nfc(const Level& L) { return L.nf_alloc > 1 ? L.nf_alloc : 1; }


struct SpArgs {
  int ny, ns, K, nf, np, loff, nalpha, r;
  const double* Z;        // ny x ns
  const double* XEta;     // ny x Kmax (ld ny): [X, Eta_1[Pi_1,], ...]
  const double* BL;       // K x ns
  const double* iSigma;
  const int* unit_ptr;
  const int* unit_rows;
  const double* iWg;      // np x np x nalpha
  const double* RiWg;
  int riw_lower;          // RiWg lower triangular (NNGP's Vecchia factor), else upper (chol)
  const double* detWg;
  const double* alphapw;  // nalpha x 2
  // GPP in R's low-rank form (Level::gpp)
  int nK;
  const double* idDg;     // np x nalpha
  const double* idDW12g;  // np x nK x nalpha
  const double* Fg;       // nK x nK x nalpha
  const double* iFg;      // nK x nK x nalpha
  double* AlphaD;         // nf (1-based grid index as double)
  double* Eta;            // np x nf (ld np)
  double* work;
  int* fail;
  Key key;
  uint32_t iter;
  const uint32_t* iter_dev;
  int noise_zero;
};

__global__ __launch_bounds__(1024) void eta_spatial_full_kernel(SpArgs a) {
  __shared__ int flag;
  const int t = threadIdx.x, nthr = blockDim.x;
  const int np = a.np, nf = a.nf, ns = a.ns, ny = a.ny, K = a.K, N = np * nf;
  double* U = a.work;                       // N x N
  double* rhs = U + (size_t)N * N;          // N
  double* LDL = rhs + N;                    // nf x nf
  const double* lam = a.BL + a.loff;        // Lambda_r[h, j] = lam[h + K j]
  for (int p = t; p < nf * nf; p += nthr) {
    const int h1 = p % nf, h2 = p / nf;
    double s = 0.0;
    for (int j = 0; j < ns; ++j) s = fma(lam[h1 + (size_t)K * j] * a.iSigma[j], lam[h2 + (size_t)K * j], s);
    LDL[p] = s;
  }
  // fS[p, h] = sum_{rows i of unit p} sum_j S[i, j] Lam[h, j] iSigma[j], where S excludes this
  // level's own columns of XEta (R/updateEta.R:31-37, :119-127)
  for (int e = t; e < N; e += nthr) {
    const int q = e % np, h = e / np;
    double acc = 0.0;
    for (int k = a.unit_ptr[q]; k < a.unit_ptr[q + 1]; ++k) {
      const int i = a.unit_rows[k];
      for (int j = 0; j < ns; ++j) {
        double sv = a.Z[i + (size_t)ny * j];
        for (int c = 0; c < K; ++c) {
          if (c >= a.loff && c < a.loff + nf) continue;
          sv = fma(-a.XEta[i + (size_t)ny * c], a.BL[c + (size_t)K * j], sv);
        }
        acc = fma(sv, lam[h + (size_t)K * j] * a.iSigma[j], acc);
      }
    }
    rhs[e] = acc;
  }
  __syncthreads();
  // iUEta (upper triangle is all wg_chol reads; fill the whole matrix for simplicity)
  for (size_t e = t; e < (size_t)N * N; e += nthr) {
    const int r1 = (int)(e % N), r2 = (int)(e / N);
    const int q1 = r1 % np, h1 = r1 / np, q2 = r2 % np, h2 = r2 / np;
    double v = 0.0;
    if (h1 == h2) {
      const int g = (int)a.AlphaD[h1] - 1;
      v = a.iWg[q1 + (size_t)np * q2 + (size_t)np * np * g];
    }
    if (q1 == q2) v = fma(LDL[h1 + nf * h2], (double)(a.unit_ptr[q1 + 1] - a.unit_ptr[q1]), v);
    U[e] = v;
  }
  __syncthreads();
  if (!wg_chol(U, N, N, &flag) && t == 0) a.fail[0] = 1;
  wg_forward(U, N, N, rhs);  // backsolve(R, fS, transpose=TRUE)
  for (int e = t; e < N; e += nthr)
    if (!a.noise_zero) rhs[e] += normal(a.key, (uint32_t)(e % np), (uint32_t)(e / np), S_ETA + LEVEL_STRIDE * a.r, SWEEP_ITER(a));
  __syncthreads();
  wg_backward_t(U, N, N, rhs);  // backsolve(R, tmp2)
  for (int e = t; e < N; e += nthr) a.Eta[e] = rhs[e];
}

// ---- blocked path for large np * nf (dense.hip): the same system, assembled and factorised
// by many workgroups (one-workgroup wg_chol above is the latency-optimal shape only while
// the (np nf)^2 matrix is small)
// LDL = Lam diag(iSigma) Lam' (block 0) and rhs = vec(fS) (every thread one (p, h))
__global__ __launch_bounds__(256) void sp_rhs_kernel(SpArgs a, double* rhs, double* LDL) {
  const int np = a.np, nf = a.nf, ns = a.ns, ny = a.ny, K = a.K, N = np * nf;
  const double* lam = a.BL + a.loff;
  if (blockIdx.x == 0)
    for (int p = threadIdx.x; p < nf * nf; p += blockDim.x) {
      const int h1 = p % nf, h2 = p / nf;
      double s = 0.0;
      for (int j = 0; j < ns; ++j) s = fma(lam[h1 + (size_t)K * j] * a.iSigma[j], lam[h2 + (size_t)K * j], s);
      LDL[p] = s;
    }
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= N) return;
  const int q = e % np, h = e / np;
  double acc = 0.0;
  for (int k = a.unit_ptr[q]; k < a.unit_ptr[q + 1]; ++k) {
    const int i = a.unit_rows[k];
    for (int j = 0; j < ns; ++j) {
      double sv = a.Z[i + (size_t)ny * j];
      for (int c = 0; c < K; ++c) {
        if (c >= a.loff && c < a.loff + nf) continue;
        sv = fma(-a.XEta[i + (size_t)ny * c], a.BL[c + (size_t)K * j], sv);
      }
      acc = fma(sv, lam[h + (size_t)K * j] * a.iSigma[j], acc);
    }
  }
  rhs[e] = acc;
}

// lower triangle of iUEta = bdiag(iWg[,,alpha_h]) + kron(LDL, diag(n_p)); grid (N / 256, N)
__global__ __launch_bounds__(256) void sp_assemble_kernel(SpArgs a, double* U, const double* LDL) {
  const int np = a.np, nf = a.nf, N = np * nf;
  const int r2 = blockIdx.y, r1 = blockIdx.x * blockDim.x + threadIdx.x;
  if (r1 >= N || r1 < r2) return;
  const int q1 = r1 % np, h1 = r1 / np, q2 = r2 % np, h2 = r2 / np;
  double v = 0.0;
  if (h1 == h2) {
    const int g = (int)a.AlphaD[h1] - 1;
    v = a.iWg[q1 + (size_t)np * q2 + (size_t)np * np * g];
  }
  if (q1 == q2) v = fma(LDL[h1 + nf * h2], (double)(a.unit_ptr[q1 + 1] - a.unit_ptr[q1]), v);
  U[r1 + (size_t)N * r2] = v;
}

__global__ __launch_bounds__(256) void sp_noise_kernel(SpArgs a, double* rhs) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x, np = a.np;
  if (e >= np * a.nf || a.noise_zero) return;
  rhs[e] += normal(a.key, (uint32_t)(e % np), (uint32_t)(e / np), S_ETA + LEVEL_STRIDE * a.r, SWEEP_ITER(a));
}

__global__ __launch_bounds__(256) void sp_store_kernel(SpArgs a, const double* rhs) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e < a.np * a.nf) a.Eta[e] = rhs[e];
}

// v[g, h] = |RiWg[,,g] eta_h|^2 ; RiWg upper triangular (chol(iW), Full from the host) or lower
// triangular (NNGP's D^-1/2 (I - A), R/computeDataParameters.R:127; GPP's and the device-built
// Full grid's chol(W)^-1).  Grid (nalpha, ceil(np / 256)): a workgroup takes 256 rows p of one
// grid matrix (coalesced down the columns), four factors per pass, and leaves its partial
// sums at work[(g * nch + chunk) * nf + h]; alpha_draw_kernel adds the chunks in order.
constexpr int AQ_LDS = 6144;  // Eta values (np x 4-factor block) staged per workgroup: 48 KB

__global__ __launch_bounds__(256) void alpha_quad_kernel(SpArgs a) {
  const int g = blockIdx.x, chunk = blockIdx.y, nch = gridDim.y, np = a.np, nf = a.nf;
  const double* Rg = a.RiWg + (size_t)np * np * g;
  const int p = chunk * 256 + threadIdx.x, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __shared__ double red[4][4];
  __shared__ double sE[AQ_LDS];
  // The column range is the workgroup's (uniform): the Eta block is staged in LDS and read
  // back at uniform addresses (broadcast), so the vector memory path carries only the R
  // stream; the triangle's edge inside the workgroup's 256 x 256 diagonal block is an exec
  // mask on the loads (masked columns add exact zeros: the per-row sums are unchanged).
  const int p0 = chunk * 256, lower = a.riw_lower;
  const int c_lo = lower ? 0 : p0, c_hi = lower ? min(np, p0 + 256) : np;
  const int pr = min(p, np - 1);
  for (int h0 = 0; h0 < nf; h0 += 4) {
    const int nh = min(4, nf - h0);
    const int ncol = c_hi - c_lo;
    const bool staged = ncol * nh <= AQ_LDS;
    const double* e = a.Eta + (size_t)np * h0;
    if (staged) {  // sE[(c - c_lo) nh + hh] = Eta[c, h0 + hh]
      const int n = ncol * nh;
      for (int q0 = threadIdx.x; q0 < n; q0 += 8 * 256) {
        double v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int q = min(q0 + 256 * u, n - 1), c = q / nh, hh = q - c * nh;
          v[u] = e[c_lo + c + (size_t)np * hh];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (q0 + 256 * u < n) sE[q0 + 256 * u] = v[u];
      }
      __syncthreads();
    }
    double x[4] = {0.0, 0.0, 0.0, 0.0};
    auto rows = [&](auto ev) {  // ev(c, hh) = Eta[c, h0 + hh]
      int p2 = c_lo;
      for (; p2 + 16 <= c_hi; p2 += 16) {  // sixteen column loads in flight per lane
        double rv[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          const int c = p2 + u;
          rv[u] = (p < np && (lower ? c <= p : c >= p)) ? Rg[pr + (size_t)np * c] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < 16; ++u)
#pragma unroll
          for (int hh = 0; hh < 4; ++hh)
            if (hh < nh) x[hh] = fma(rv[u], ev(p2 + u, hh), x[hh]);
      }
      for (; p2 < c_hi; ++p2) {
        const double rv = (p < np && (lower ? p2 <= p : p2 >= p)) ? Rg[pr + (size_t)np * p2] : 0.0;
#pragma unroll
        for (int hh = 0; hh < 4; ++hh)
          if (hh < nh) x[hh] = fma(rv, ev(p2, hh), x[hh]);
      }
    };
    if (staged)
      rows([&](int c, int hh) { return sE[(c - c_lo) * nh + hh]; });
    else
      rows([&](int c, int hh) { return e[c + (size_t)np * hh]; });
#pragma unroll
    for (int hh = 0; hh < 4; ++hh) {
      double s = x[hh] * x[hh];
      for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
      if (lane == 0) red[w][hh] = s;
    }
    __syncthreads();
    if (threadIdx.x < nh)
      a.work[((size_t)g * nch + chunk) * nf + h0 + threadIdx.x] =
          (red[0][threadIdx.x] + red[1][threadIdx.x]) + (red[2][threadIdx.x] + red[3][threadIdx.x]);
    __syncthreads();
  }
}

__device__ inline double alpha_quad_sum(const SpArgs& a, int g, int h) {
  const int nch = (a.np + 255) / 256;
  double v = 0.0;
  for (int c = 0; c < nch; ++c) v += a.work[((size_t)g * nch + c) * a.nf + h];
  return v;
}

// likelihood over the grid and inverse-CDF categorical draw (R's sample.int(gN, 1,
// prob=like), R/updateAlpha.R:76-78), one workgroup: the grid points' log-likelihoods (their
// chunk sums) in parallel, then one thread per factor runs the max / total / cumulative sum
// over them in grid order (sequential sums, as the oracle's)
__global__ __launch_bounds__(256) void alpha_draw_kernel(SpArgs a) {
  __shared__ double like[HMSC_MAX_ALPHA];
  __shared__ double mx_s;
  const int G = a.nalpha, t = threadIdx.x;
  for (int h = 0; h < a.nf; ++h) {
    for (int g = t; g < G; g += blockDim.x)
      like[g] = log(a.alphapw[G + g]) - 0.5 * a.detWg[g] - 0.5 * alpha_quad_sum(a, g, h);
    __syncthreads();
    if (t == 0) {
      double mx = -INFINITY;
      for (int g = 0; g < G; ++g) mx = fmax(mx, like[g]);
      mx_s = mx;
    }
    __syncthreads();
    for (int g = t; g < G; g += blockDim.x) like[g] = exp(like[g] - mx_s);
    __syncthreads();
    if (t == 0) {
      double tot = 0.0;
      for (int g = 0; g < G; ++g) tot += like[g];
      const double u = uniforms(a.key, (uint32_t)h, 0, S_ALPHA + LEVEL_STRIDE * a.r, SWEEP_ITER(a)).a * tot;
      double c = 0.0;
      int pick = G;
      for (int g = 0; g < G; ++g) {
        c += like[g];
        if (c > u) {
          pick = g + 1;
          break;
        }
      }
      a.AlphaD[h] = (double)(pick > G ? G : pick);
    }
    __syncthreads();
  }
}

static SpArgs sp_args(State& s, int r, uint32_t iter) {
  const Level& L = s.lev[r];
  SpArgs a{};
  a.ny = s.ny;
  a.ns = s.nsl;
  a.K = s.K;
  a.nf = L.nf;
  a.np = L.np;
  a.loff = s.loff(r);
  a.nalpha = L.nalpha;
  a.r = r;
  a.Z = s.Z;
  a.XEta = s.XEta;
  a.BL = s.BL;
  a.iSigma = s.iSigma;
  a.unit_ptr = L.unit_ptr;
  a.unit_rows = L.unit_rows;
  a.iWg = L.iWg;
  a.RiWg = L.RiWg;
  a.riw_lower = L.riw_lower;
  a.detWg = L.detWg;
  a.alphapw = L.alphapw;
  a.nK = L.nK;
  a.idDg = L.idDg;
  a.idDW12g = L.idDW12g;
  a.Fg = L.Fg;
  a.iFg = L.iFg;
  a.AlphaD = L.AlphaD;
  a.Eta = L.Eta;
  a.work = L.spWork;
  a.fail = s.dev_flags;
  a.key = s.key;
  a.iter = iter;
  a.iter_dev = s.capturing ? s.d_iter : nullptr;
  a.noise_zero = s.noise_mode;
  return a;
}

// ---------------------------------------------------------------------------------------
// 'GPP' levels in R's low-rank form (R/updateEta.R:148-196; np == ny, units in unit order).
// With B0_i = Lam iSigma Lam' + diag(idD[i, alpha_h]) (nf x nf per unit), iA = bdiag(B0_i^-1),
// W = bdiag_h(idDW12g[,,alpha_h]) ((np nf) x (nK nf)), H = bdiag_h(Fg[,,alpha_h]) - W' iA W:
//   eta = iA fS + T (T' fS + xi2) + LiA xi1,   T = iA W RH^-1,  RH = chol(H),
// LiA = bdiag(chol(B0_i^-1)) (lower) -- O(np (nK nf)^2) work, nothing np^2.  Normals: xi1 of
// unit i, factor h = normal(i, h, S_ETA + LEVEL_STRIDE r) (the counters of the other
// branches), xi2 of knot k, factor h = normal(k, GPP_XI2_SUB + h, same stream).
// updateAlpha (R/updateAlpha.R:35-75): v_gh = eta_h' diag(idDg[,g]) eta_h - t_h iFg[,,g] t_h'
// with t_h = eta_h' idDW12g[,,g] (eta_h' eta_h at alpha_g = 0), likelihood with detDg.
// ---------------------------------------------------------------------------------------
constexpr uint32_t GPP_XI2_SUB = 1024;

struct GppLayout {
  size_t rhs, LDL, B1, LB1, iAW, H, M, ws, T, v, alpha, tot;
};

// nfc: factor capacity (nfmax), nch: updateAlpha's partial-sum chunks
inline GppLayout gpp_layout(int np, int nfc, int nK, int nalpha) {
  GppLayout o{};
  const size_t NP = (size_t)np * nfc, KF = (size_t)nK * nfc;
  size_t p = 0;
  auto take = [&](size_t n) {
    const size_t at = p;
    p += (n + 7) & ~(size_t)7;
    return at;
  };
  o.rhs = take(NP);
  o.LDL = take((size_t)nfc * nfc);
  o.B1 = take((size_t)np * nfc * nfc);
  o.LB1 = take((size_t)np * nfc * nfc);
  o.iAW = take(NP * KF);
  o.H = take(KF * KF);
  o.M = take(KF * KF);
  o.ws = take(dense_ws_doubles((int)KF));
  o.T = take(NP * KF);
  o.v = take(KF);
  o.alpha = take((size_t)nalpha * ((np + 255) / 256) * nfc);
  o.tot = p;
  return o;
}

// per unit i: B1_i = B0_i^-1 and LB1_i = chol(B1_i) (lower), nf x nf column-major at i nf^2
__global__ __launch_bounds__(256) void gpp_unit_kernel(SpArgs a, const double* LDL, double* B1, double* LB1) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x, nf = a.nf, np = a.np;
  if (i >= np) return;
  double A[16 * 16], Li[16 * 16];
  for (int c = 0; c < nf; ++c)
    for (int r = 0; r < nf; ++r)
      A[r + nf * c] = LDL[r + nf * c] + (r == c ? a.idDg[i + (size_t)np * ((int)a.AlphaD[r] - 1)] : 0.0);
  bool ok = t_chol_inv(A, Li, nf);  // A <- L0 (lower), Li = L0^-1
  double* b1 = B1 + (size_t)i * nf * nf;
  double* lb = LB1 + (size_t)i * nf * nf;
  for (int c = 0; c < nf; ++c)
    for (int r = 0; r < nf; ++r) {  // B1 = L0^-T L0^-1
      double s = 0.0;
      for (int k = (r > c ? r : c); k < nf; ++k) s += Li[k + nf * r] * Li[k + nf * c];
      b1[r + nf * c] = s;
      A[r + nf * c] = s;
    }
  ok = t_chol_inv(A, Li, nf) && ok;  // A <- chol(B1)
  for (int c = 0; c < nf; ++c)
    for (int r = 0; r < nf; ++r) lb[r + nf * c] = r >= c ? A[r + nf * c] : 0.0;
  if (!ok) a.fail[0] = 1;
}

// iAW[e, c] = B1_i[h, h'] idDW12g[i, k, alpha_h'],  e = i + np h, c = k + nK h'
__global__ __launch_bounds__(256) void gpp_iaw_kernel(SpArgs a, const double* B1, double* iAW) {
  const int np = a.np, nf = a.nf, nK = a.nK, NP = np * nf;
  const int e = blockIdx.x * blockDim.x + threadIdx.x, c = blockIdx.y;
  if (e >= NP) return;
  const int i = e % np, h = e / np, k = c % nK, h2 = c / nK;
  const double w = a.idDW12g[i + (size_t)np * k + (size_t)np * nK * ((int)a.AlphaD[h2] - 1)];
  iAW[e + (size_t)NP * c] = B1[(size_t)i * nf * nf + h + nf * h2] * w;
}

// H = bdiag_h(Fg[,,alpha_h]) - W' iAW, one workgroup per entry (reduction over the np units)
__global__ __launch_bounds__(256) void gpp_h_kernel(SpArgs a, const double* iAW, double* H) {
  const int np = a.np, nf = a.nf, nK = a.nK, NP = np * nf, KF = nK * nf;
  const int c1 = blockIdx.x, c2 = blockIdx.y, k = c1 % nK, h = c1 / nK;
  const double* w = a.idDW12g + (size_t)np * k + (size_t)np * nK * ((int)a.AlphaD[h] - 1);
  const double* x = iAW + (size_t)np * h + (size_t)NP * c2;
  double s = 0.0;
  for (int i = threadIdx.x; i < np; i += 256) s = fma(w[i], x[i], s);
  __shared__ double red[4];
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const int k2 = c2 % nK, h2 = c2 / nK;
    const double f = h == h2 ? a.Fg[k + (size_t)nK * k2 + (size_t)nK * nK * ((int)a.AlphaD[h] - 1)] : 0.0;
    H[c1 + (size_t)KF * c2] = f - ((red[0] + red[1]) + (red[2] + red[3]));
  }
}

// T = iAW RH^-1 = iAW M^T with M = L_H^-1 (lower): T[e, c] = sum_{c' <= c} iAW[e, c'] M[c, c']
__global__ __launch_bounds__(256) void gpp_t_kernel(SpArgs a, const double* iAW, const double* M, double* T) {
  const int NP = a.np * a.nf, KF = a.nK * a.nf;
  const int e = blockIdx.x * blockDim.x + threadIdx.x, c = blockIdx.y;
  if (e >= NP) return;
  double s = 0.0;
  for (int c2 = 0; c2 <= c; ++c2) s = fma(iAW[e + (size_t)NP * c2], M[c + (size_t)KF * c2], s);
  T[e + (size_t)NP * c] = s;
}

// v[c] = T[, c]' fS + xi2[c], one workgroup per c
__global__ __launch_bounds__(256) void gpp_v_kernel(SpArgs a, const double* T, const double* rhs, double* v) {
  const int NP = a.np * a.nf, c = blockIdx.x;
  double s = 0.0;
  for (int e = threadIdx.x; e < NP; e += 256) s = fma(T[e + (size_t)NP * c], rhs[e], s);
  __shared__ double red[4];
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const int k = c % a.nK, h = c / a.nK;
    const double xi2 = a.noise_zero ? 0.0 : normal(a.key, (uint32_t)k, GPP_XI2_SUB + (uint32_t)h, S_ETA + LEVEL_STRIDE * a.r,
                                                    SWEEP_ITER(a));
    v[c] = (red[0] + red[1]) + (red[2] + red[3]) + xi2;
  }
}

// eta[e] = (B1_i fS_i)_h + (LB1_i xi1_i)_h + T[e, ] v
__global__ __launch_bounds__(256) void gpp_eta_kernel(SpArgs a, const double* B1, const double* LB1, const double* T,
                                                      const double* rhs, const double* v) {
  const int np = a.np, nf = a.nf, NP = np * nf, KF = a.nK * nf;
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= NP) return;
  const int i = e % np, h = e / np;
  const double* b1 = B1 + (size_t)i * nf * nf;
  const double* lb = LB1 + (size_t)i * nf * nf;
  double s = 0.0;
  for (int h2 = 0; h2 < nf; ++h2) s = fma(b1[h + nf * h2], rhs[i + (size_t)np * h2], s);
  if (!a.noise_zero)
    for (int h2 = 0; h2 <= h; ++h2)
      s = fma(lb[h + nf * h2], normal(a.key, (uint32_t)i, (uint32_t)h2, S_ETA + LEVEL_STRIDE * a.r, SWEEP_ITER(a)), s);
  for (int c = 0; c < KF; ++c) s = fma(T[e + (size_t)NP * c], v[c], s);
  a.Eta[e] = s;
}

// updateAlpha's GPP statistic, one workgroup per grid point; v_gh goes to chunk 0 of the
// partial-sum slots alpha_draw_kernel adds (the other chunks zero).  t_h = eta_h' idDW12g[,,g]:
// wave w takes the knots k = w, w + 4, ..., its 64 lanes stride down the units (coalesced
// column reads of idDW12g, the HBM stream of this updater) and reduce by shuffles -- no
// workgroup barrier per knot.
__global__ __launch_bounds__(256) void gpp_alpha_kernel(SpArgs a, double* out) {
  const int g = blockIdx.x, np = a.np, nf = a.nf, nK = a.nK, nch = (np + 255) / 256;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  __shared__ double red[4], t2[1024];
  const bool zero = a.alphapw[g] == 0.0;
  const double* idD = a.idDg + (size_t)np * g;
  const double* W = a.idDW12g + (size_t)np * nK * g;
  const double* iF = a.iFg + (size_t)nK * nK * g;
  auto wave_sum = [&](double s) {
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    return s;
  };
  for (int h = 0; h < nf; ++h) {
    const double* eta = a.Eta + (size_t)np * h;
    double s = 0.0;
    for (int i = t; i < np; i += 256) s = fma(eta[i] * (zero ? 1.0 : idD[i]), eta[i], s);
    s = wave_sum(s);
    if (lane == 0) red[w] = s;
    if (!zero)
      for (int k = w; k < nK; k += 4) {  // t_h = eta_h' idDW12g[,,g]
        const double* col = W + (size_t)np * k;
        double q0 = 0.0, q1 = 0.0;
        int i = lane;
        for (; i + 64 < np; i += 128) {
          q0 = fma(eta[i], col[i], q0);
          q1 = fma(eta[i + 64], col[i + 64], q1);
        }
        if (i < np) q0 = fma(eta[i], col[i], q0);
        const double tk = wave_sum(q0 + q1);
        if (lane == 0) t2[k] = tk;
      }
    __syncthreads();
    double v = (red[0] + red[1]) + (red[2] + red[3]);
    if (!zero) {
      double q = 0.0;  // t_h iF t_h'
      for (int p = t; p < nK * nK; p += 256) q = fma(t2[p % nK] * iF[p], t2[p / nK], q);
      q = wave_sum(q);
      __syncthreads();
      if (lane == 0) red[w] = q;
      __syncthreads();
      v -= (red[0] + red[1]) + (red[2] + red[3]);
    }
    if (t == 0) {
      double* o = out + (size_t)g * nch * nf;
      for (int c = 0; c < nch; ++c) o[(size_t)c * nf + h] = c == 0 ? v : 0.0;
    }
    __syncthreads();
  }
}

static void launch_eta_gpp(State& s, int r, uint32_t iter) {
  const Level& L = s.lev[r];
  HMSC_REQUIRE(L.nK <= 1024, "GPP level: at most 1024 knots in this build");
  const SpArgs a = sp_args(s, r, iter);
  const int np = L.np, nf = L.nf, NP = np * nf, KF = L.nK * nf;
  const GppLayout o = gpp_layout(np, sp_nfc(L), L.nK, L.nalpha);
  double* w = L.spWork;
  double *rhs = w + o.rhs, *LDL = w + o.LDL, *B1 = w + o.B1, *LB1 = w + o.LB1, *iAW = w + o.iAW, *H = w + o.H;
  double *M = w + o.M, *ws = w + o.ws, *T = w + o.T, *v = w + o.v;
  const int g1 = (NP + 255) / 256;
  sp_rhs_kernel<<<g1, 256, 0, s.stream>>>(a, rhs, LDL);
  gpp_unit_kernel<<<(np + 255) / 256, 256, 0, s.stream>>>(a, LDL, B1, LB1);
  gpp_iaw_kernel<<<dim3(g1, KF), 256, 0, s.stream>>>(a, B1, iAW);
  gpp_h_kernel<<<dim3(KF, KF), 256, 0, s.stream>>>(a, iAW, H);
  HIP_OK(hipGetLastError());
  {
    ProfScope pc(s, PROF_CHOL);
    dense_potrf_lower(s.stream, H, KF, KF, ws, s.dev_flags, 0, s.trsv_sync);  // RH = chol(H) = L_H^T
  }
  dense_trtri_lower(s.stream, H, KF, KF, M, KF, ws, true);     // M = L_H^-1, RH^-1 = M^T
  gpp_t_kernel<<<dim3(g1, KF), 256, 0, s.stream>>>(a, iAW, M, T);
  gpp_v_kernel<<<KF, 256, 0, s.stream>>>(a, T, rhs, v);
  gpp_eta_kernel<<<g1, 256, 0, s.stream>>>(a, B1, LB1, T, rhs, v);
  HIP_OK(hipGetLastError());
}

static int* dupload_i32(const int* h, size_t n) {
  int* p = nullptr;
  HIP_OK(hipMalloc(&p, std::max<size_t>(1, n) * sizeof(int)));
  if (n) HIP_OK(hipMemcpy(p, h, n * sizeof(int), hipMemcpyHostToDevice));
  return p;
}
static double* dupload_f64(const double* h, size_t n) {
  double* p = nullptr;
  HIP_OK(hipMalloc(&p, std::max<size_t>(1, n) * sizeof(double)));
  if (n) HIP_OK(hipMemcpy(p, h, n * sizeof(double), hipMemcpyHostToDevice));
  return p;
}

// ---------------------------------------------------------------------------------------
// 'NNGP' levels in the sparse Vecchia form (R/computeDataParameters.R:82-136, R/updateEta.R:
// 137-147, R/updateAlpha.R:21-34).  Per grid point g the prior precision is
// iW_g = B_g' D_g^-1 B_g, B_g = I - A_g unit lower triangular with A_g[i, nb(i, k)] on the nnK
// nearest EARLIER units of unit i: nnK + 1 numbers per unit, no np^2 array anywhere.
//  * updateAlpha: v_gh = sum_i (eta_ih - sum_k A_g[i, nb(i,k)] eta_nb(i,k),h)^2 / D_g[i], one
//    thread per unit (nalpha x ceil(np / 256) workgroups, the same chunk-partial layout as the
//    'Full' kernel, so alpha_draw_kernel draws the grid index).
//  * updateEta: iUEta = bdiag_h(iW_alpha_h) + kron(Lam iSigma Lam', I) is sparse; in the reverse
//    Cuthill-McKee order of the units (setup_nngp_level), factors interleaved per unit (index
//    pos(q) nf + h), it is a band matrix of bandwidth bw = (bwUnits + 1) nf - 1 (bwUnits 301 at
//    np = 5000, 10 neighbours, against 4968 in the data order).  It is assembled straight into
//    that band (one wave per column: each entry is the sum over the rows i whose support holds
//    both units, in ascending i), factored by the blocked Cholesky restricted to the band's
//    tiles (dense.hip, n bw^2 instead of n^3 / 3 flops) and solved: eta = P' L^-T (L^-1 P vec(fS)
//    + P xi) with L L' = P iUEta P' -- the conditional of R's code, the noise of (unit q,
//    factor h) the normal of R's order (S_ETA counters); the oracle restates this order
//    (oracle/hmsc_oracle.py nngp_rcm, _eta_spatial_full).
// ---------------------------------------------------------------------------------------
struct NnArgs {
  int np, nf, N, K, bw, ldq;  // ldq: rows per panel of the tile-band layout of the band matrix
  const int* idx;      // K x np
  const double* A;     // nalpha x K x np
  const double* D;     // nalpha x np
  const int* perm;
  const int* pos;
  const int* chptr;
  const int* ch;
  const int* unit_ptr;
  const double* AlphaD;
};

static NnArgs nn_args(const State& s, int r) {
  const Level& L = s.lev[r];
  NnArgs n{};
  n.np = L.np;
  n.nf = L.nf;
  n.N = L.np * L.nf;
  n.K = L.nnK;
  n.bw = (L.nnBwUnits + 1) * L.nf - 1;
  n.ldq = dense_band_ld(n.bw);
  n.idx = L.nnIdx;
  n.A = L.nnA;
  n.D = L.nnD;
  n.perm = L.nnPerm;
  n.pos = L.nnPos;
  n.chptr = L.nnChPtr;
  n.ch = L.nnCh;
  n.unit_ptr = L.unit_ptr;
  n.AlphaD = L.AlphaD;
  return n;
}

__global__ __launch_bounds__(256) void nngp_alpha_kernel(SpArgs a, NnArgs n) {
  const int g = blockIdx.x, chunk = blockIdx.y, nch = gridDim.y, np = n.np, K = n.K;
  const int i = chunk * 256 + threadIdx.x, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __shared__ double red[4];
  for (int h = 0; h < n.nf; ++h) {
    const double* eta = a.Eta + (size_t)np * h;
    double v = 0.0;
    if (i < np) {
      double r = eta[i];
      for (int k = 0; k < K; ++k) {
        const int j = n.idx[(size_t)k * np + i];
        if (j >= 0) r = fma(-n.A[((size_t)g * K + k) * np + i], eta[j], r);
      }
      v = r * r / n.D[(size_t)g * np + i];
    }
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if (lane == 0) red[w] = v;
    __syncthreads();
    if (threadIdx.x == 0) a.work[((size_t)g * nch + chunk) * n.nf + h] = (red[0] + red[1]) + (red[2] + red[3]);
    __syncthreads();
  }
}

// B_g[i, u] for the support entry e = i (K + 1) + slot of unit u in row i
__device__ __forceinline__ double nn_b(const NnArgs& n, int g, int e) {
  const int i = e / (n.K + 1), slot = e - i * (n.K + 1);
  return slot == 0 ? 1.0 : -n.A[((size_t)g * n.K + slot - 1) * n.np + i];
}

// column c of the band (rows c .. c + bw) of P iUEta P', one wave per column
__global__ __launch_bounds__(64) void nngp_assemble_kernel(NnArgs n, const double* LDL, double* Q) {
  constexpr int SB = 256;
  __shared__ int sb[SB];
  const int c = blockIdx.x, lane = threadIdx.x, nf = n.nf, N = n.N, K1 = n.K + 1;
  const int pb = c / nf, h = c - pb * nf, b = n.perm[pb];
  const int g = (int)n.AlphaD[h] - 1;
  const int b0 = n.chptr[b], nb = n.chptr[b + 1] - b0;
  for (int q = lane; q < min(nb, SB); q += 64) sb[q] = n.ch[b0 + q];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  auto sb_at = [&](int q) { return q < SB ? sb[q] : n.ch[b0 + q]; };
  for (int t = lane; t <= n.bw && c + t < N; t += 64) {
    const int row = c + t, pa = row / nf, h2 = row - pa * nf, a = n.perm[pa];
    double v = 0.0;
    if (h2 == h) {  // iW_g[a, b] = sum over rows i holding both: B[i, a] B[i, b] / D[i]
      const int a0 = n.chptr[a], na = n.chptr[a + 1] - a0;
      int p = 0, q = 0;
      while (p < na && q < nb) {
        const int ea = n.ch[a0 + p], eb = sb_at(q);
        const int ia = ea / K1, ib = eb / K1;
        if (ia < ib) {
          ++p;
        } else if (ib < ia) {
          ++q;
        } else {
          v = fma(nn_b(n, g, ea) * nn_b(n, g, eb), 1.0 / n.D[(size_t)g * n.np + ia], v);
          ++p, ++q;
        }
      }
    }
    if (a == b) v = fma(LDL[h2 + nf * h], (double)(n.unit_ptr[a + 1] - n.unit_ptr[a]), v);
    Q[(size_t)(row - (c & ~63)) + (size_t)n.ldq * c] = v;  // tile-band layout (dense.hip aix)
  }
}

// x[pos(q) nf + h] = rhs[q + np h]  (mode 0);  Eta[q + np h] = x[pos(q) nf + h]  (mode 2);
// x[pos(q) nf + h] += normal(q, h, S_ETA + LEVEL_STRIDE r)  (mode 1, the noise of R's order)
__global__ __launch_bounds__(256) void nngp_perm_kernel(SpArgs a, NnArgs n, const double* rhs, double* x, int mode) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n.N) return;
  const int q = e % n.np, h = e / n.np, k = n.pos[q] * n.nf + h;
  if (mode == 0)
    x[k] = rhs[e];
  else if (mode == 1) {
    if (!a.noise_zero) x[k] += normal(a.key, (uint32_t)q, (uint32_t)h, S_ETA + LEVEL_STRIDE * a.r, SWEEP_ITER(a));
  } else
    a.Eta[e] = x[k];
}

struct NnLayout {
  size_t Q, x, rhs, ws, LDL, tot;
};
// the band matrix in the tile-band layout (N x dense_band_ld(bw) doubles, O(N bw)), at the
// level's factor capacity nfc
static NnLayout nn_layout(int np, int nfc, int bw_units) {
  NnLayout o{};
  const size_t N = (size_t)np * nfc;
  o.Q = 0;
  o.x = o.Q + N * (size_t)dense_band_ld((bw_units + 1) * nfc - 1);
  o.rhs = o.x + N + 8;
  o.ws = o.rhs + N + 8;
  o.LDL = o.ws + dense_ws_doubles((int)N);
  o.tot = o.LDL + (size_t)nfc * nfc + 64;
  return o;
}

static void launch_eta_nngp(State& s, int r, uint32_t iter) {
  Level& L = s.lev[r];
  const SpArgs a = sp_args(s, r, iter);
  const NnArgs n = nn_args(s, r);
  const NnLayout o = nn_layout(L.np, sp_nfc(L), L.nnBwUnits);
  double* w = L.spWork;
  double *Q = w + o.Q, *x = w + o.x, *rhs = w + o.rhs, *ws = w + o.ws, *LDL = w + o.LDL;
  const int N = n.N, g1 = (N + 255) / 256;
  if (L.nnAssembledN != N) {  // a new system size (updateNf): entries outside its band must be 0
    HIP_OK(hipMemsetAsync(Q, 0, (size_t)N * n.ldq * sizeof(double), s.stream));
    L.nnAssembledN = N;
  }
  sp_rhs_kernel<<<g1, 256, 0, s.stream>>>(a, rhs, LDL);
  nngp_assemble_kernel<<<N, 64, 0, s.stream>>>(n, LDL, Q);
  nngp_perm_kernel<<<g1, 256, 0, s.stream>>>(a, n, rhs, x, 0);
  HIP_OK(hipGetLastError());
  {
    ProfScope pc(s, PROF_CHOL);
    dense_potrf_lower(s.stream, Q, N, -n.ldq, ws, s.dev_flags, n.bw, s.trsv_sync);
  }
  dense_trsv_lower(s.stream, Q, N, -n.ldq, x, 0, ws, n.bw, s.trsv_sync);   // backsolve(R, fS, transpose = TRUE)
  nngp_perm_kernel<<<g1, 256, 0, s.stream>>>(a, n, rhs, x, 1);
  dense_trsv_lower(s.stream, Q, N, -n.ldq, x, 1, ws, n.bw, s.trsv_sync);   // backsolve(R, tmp2)
  nngp_perm_kernel<<<g1, 256, 0, s.stream>>>(a, n, rhs, x, 2);
  HIP_OK(hipGetLastError());
}

// ---- host setup (chain creation) ----
void setup_nngp_level(State& s, int r, const double* crd, int sdim, int k, const double* alphapw, int G) {
  Level& L = s.lev[r];
  const int n = L.np;
  HMSC_REQUIRE(crd != nullptr && sdim > 0, "NNGP level: pass the unit coordinates (sCoord); nearest neighbours are "
                                           "not available for distance matrices (R/computeDataParameters.R:86-88)");
  HMSC_REQUIRE(k >= 1 && k < n, "NNGP level: nNeighbours must be in [1, np - 1]");
  auto d2 = [&](int i, int j) {
    double t = 0.0;
    for (int c = 0; c < sdim; ++c) {
      const double u = crd[i + (size_t)n * c] - crd[j + (size_t)n * c];
      t += u * u;
    }
    return t;
  };
  const int nth = std::max(1, std::min(16, (int)std::thread::hardware_concurrency()));
  auto par_for = [&](int count, auto&& body) {
    std::vector<std::thread> th;
    for (int t = 0; t < nth; ++t)
      th.emplace_back([&, t] {
        for (int i = t; i < count; i += nth) body(i);
      });
    for (auto& x : th) x.join();
  };
  // FNN::get.knn(s, k): the k nearest other units (exact Euclidean; ties to the lower index),
  // sorted ascending, only earlier units kept (:93-104)
  std::vector<int> nb((size_t)k * n, -1), cnt(n, 0);
  par_for(n, [&](int i) {
    std::vector<std::pair<double, int>> dj;
    dj.reserve(n - 1);
    for (int j = 0; j < n; ++j)
      if (j != i) dj.emplace_back(d2(i, j), j);
    std::partial_sort(dj.begin(), dj.begin() + k, dj.end());
    std::vector<int> near;
    for (int q = 0; q < k; ++q)
      if (dj[q].second < i) near.push_back(dj[q].second);
    std::sort(near.begin(), near.end());
    cnt[i] = (int)near.size();
    for (int q = 0; q < (int)near.size(); ++q) nb[(size_t)q * n + i] = near[q];
  });
  // Vecchia factor per grid point: A[i, nb] = K11^-1 k12, D[i] = 1 - k21 K11^-1 k12 (:105-126)
  std::vector<double> A((size_t)G * k * n, 0.0), D((size_t)G * n, 1.0), det(G, 0.0);
  par_for(G, [&](int g) {
    const double al = alphapw[g];
    if (al == 0.0) return;  // iW = RiW = I, detW = 0
    std::vector<double> Km((size_t)k * k), v(k);
    double ld = 0.0;
    for (int i = 0; i < n; ++i) {
      const int m = cnt[i];
      if (m == 0) continue;  // D[i] = 1
      for (int p = 0; p < m; ++p) {
        const int jp = nb[(size_t)p * n + i];
        v[p] = std::exp(-std::sqrt(d2(jp, i)) / al);
        for (int q = 0; q <= p; ++q) Km[p + (size_t)k * q] = std::exp(-std::sqrt(d2(jp, nb[(size_t)q * n + i])) / al);
      }
      for (int c = 0; c < m; ++c) {  // Cholesky of K11 (lower, in place)
        double dd = Km[c + (size_t)k * c];
        for (int q = 0; q < c; ++q) dd -= Km[c + (size_t)k * q] * Km[c + (size_t)k * q];
        HMSC_REQUIRE(dd > 0.0, "NNGP level: a neighbour covariance is not positive definite (duplicated coordinates?)");
        dd = std::sqrt(dd);
        Km[c + (size_t)k * c] = dd;
        for (int p = c + 1; p < m; ++p) {
          double t = Km[p + (size_t)k * c];
          for (int q = 0; q < c; ++q) t -= Km[p + (size_t)k * q] * Km[c + (size_t)k * q];
          Km[p + (size_t)k * c] = t / dd;
        }
      }
      std::vector<double> y(v.begin(), v.begin() + m);
      for (int p = 0; p < m; ++p) {  // L y = k12
        for (int q = 0; q < p; ++q) y[p] -= Km[p + (size_t)k * q] * y[q];
        y[p] /= Km[p + (size_t)k * p];
      }
      double Di = 1.0;
      for (int p = 0; p < m; ++p) Di -= y[p] * y[p];
      for (int p = m - 1; p >= 0; --p) {  // L' a = y
        for (int q = p + 1; q < m; ++q) y[p] -= Km[q + (size_t)k * p] * y[q];
        y[p] /= Km[p + (size_t)k * p];
      }
      HMSC_REQUIRE(Di > 0.0, "NNGP level: a conditional variance is not positive");
      for (int p = 0; p < m; ++p) A[((size_t)g * k + p) * n + i] = y[p];
      D[(size_t)g * n + i] = Di;
      ld += std::log(Di);
    }
    det[g] = ld;  // detW = sum(log(D))
  });
  // reverse Cuthill-McKee over the units that share a row support (oracle nngp_rcm)
  std::vector<std::vector<int>> adj(n);
  for (int i = 0; i < n; ++i) {
    std::vector<int> sup{i};
    for (int p = 0; p < cnt[i]; ++p) sup.push_back(nb[(size_t)p * n + i]);
    for (int u : sup)
      for (int w : sup)
        if (u != w) adj[u].push_back(w);
  }
  std::vector<int> deg(n);
  for (int u = 0; u < n; ++u) {
    std::sort(adj[u].begin(), adj[u].end());
    adj[u].erase(std::unique(adj[u].begin(), adj[u].end()), adj[u].end());
    deg[u] = (int)adj[u].size();
  }
  std::vector<char> seen(n, 0);
  std::vector<int> order;
  order.reserve(n);
  while ((int)order.size() < n) {
    int start = -1;
    for (int u = 0; u < n; ++u)
      if (!seen[u] && (start < 0 || deg[u] < deg[start])) start = u;
    seen[start] = 1;
    size_t head = order.size();
    order.push_back(start);
    while (head < order.size()) {
      const int v = order[head++];
      std::vector<int> nx;
      for (int u : adj[v])
        if (!seen[u]) nx.push_back(u);
      std::sort(nx.begin(), nx.end(), [&](int x, int y) { return deg[x] != deg[y] ? deg[x] < deg[y] : x < y; });
      for (int u : nx) {
        seen[u] = 1;
        order.push_back(u);
      }
    }
  }
  std::reverse(order.begin(), order.end());
  std::vector<int> pos(n);
  for (int p = 0; p < n; ++p) pos[order[p]] = p;
  int bwu = 0;
  for (int u = 0; u < n; ++u)
    for (int w : adj[u]) bwu = std::max(bwu, std::abs(pos[u] - pos[w]));
  // rows whose support holds each unit, ascending row (children CSR)
  std::vector<int> chptr(n + 1, 0), ch;
  {
    std::vector<std::vector<int>> lists(n);
    for (int i = 0; i < n; ++i) {
      lists[i].push_back(i * (k + 1));
      for (int p = 0; p < cnt[i]; ++p) lists[nb[(size_t)p * n + i]].push_back(i * (k + 1) + p + 1);
    }
    for (int u = 0; u < n; ++u) {
      std::sort(lists[u].begin(), lists[u].end());
      chptr[u + 1] = chptr[u] + (int)lists[u].size();
      ch.insert(ch.end(), lists[u].begin(), lists[u].end());
    }
  }
  L.nngp = true;
  L.nnK = k;
  L.nnIdx = dupload_i32(nb.data(), nb.size());
  L.nnA = dupload_f64(A.data(), A.size());
  L.nnD = dupload_f64(D.data(), D.size());
  L.detWg = dupload_f64(det.data(), det.size());
  L.nnPerm = dupload_i32(order.data(), order.size());
  L.nnPos = dupload_i32(pos.data(), pos.size());
  L.nnChPtr = dupload_i32(chptr.data(), chptr.size());
  L.nnCh = dupload_i32(ch.data(), ch.size());
  L.nnBwUnits = bwu;
}

// np * nf above which updateEta's dense system goes to the multi-workgroup blocked path
constexpr int SP_BLOCKED_N = 1024;

size_t spatial_work_doubles(const State& s, int r) {
  const Level& L = s.lev[r];
  const size_t nfc = sp_nfc(L);
  if (L.gpp) return gpp_layout(L.np, (int)nfc, L.nK, L.nalpha).tot + 64;
  if (L.nngp)  // updateAlpha's partial sums after the band matrix: its zeros outside the band persist
    return nn_layout(L.np, (int)nfc, L.nnBwUnits).tot + (size_t)L.nalpha * ((L.np + 255) / 256) * nfc + 64;
  const size_t N = (size_t)L.np * nfc;
  const size_t eta = N * N + N + dense_ws_doubles((int)N) + nfc * nfc + 64;
  const size_t alpha = (size_t)L.nalpha * ((L.np + 255) / 256) * sp_nfc(L);
  return std::max(eta, alpha) + 64;
}

// The level's workspace follows the factors in use: laid out for L.nf_alloc factors at chain
// creation (nfMin), re-laid out for more when updateNf has added factors -- always outside a
// graph capture (nf changes only in eager adaptive sweeps, or by set_state / init) -- so a
// level with R's default nfMax = ns never holds an (np nfMax)^2 system it does not use.
static void sp_ensure_capacity(State& s, int r) {
  Level& L = s.lev[r];
  if (L.nf <= L.nf_alloc) return;
  HMSC_REQUIRE(!s.capturing, "internal: spatial workspace growth inside a graph capture");
  L.nf_alloc = L.nf;
  L.spWork = device_realloc_doubles(s, L.spWork, spatial_work_doubles(s, r));
  L.nnAssembledN = 0;  // the band layout's zeros are gone with the old buffer
}

void launch_eta_spatial(State& s, int r, uint32_t iter) {
  sp_ensure_capacity(s, r);
  const Level& L = s.lev[r];
  HMSC_REQUIRE(!s.sharded, "spatial levels: species-sharded chains are not supported");
  if (!s.xeta_valid) launch_xeta(s);
  ProfScope ps(s, PROF_ETA_SP);
  if (L.gpp) {
    launch_eta_gpp(s, r, iter);
    return;
  }
  if (L.nngp) {
    launch_eta_nngp(s, r, iter);
    return;
  }
  const SpArgs a = sp_args(s, r, iter);
  const int N = L.np * L.nf;
  if (N <= SP_BLOCKED_N) {
    eta_spatial_full_kernel<<<1, 1024, 0, s.stream>>>(a);
    HIP_OK(hipGetLastError());
    return;
  }
  // blocked: R = chol(iUEta) as the lower factor L = R^T; eta = L^-T (L^-1 fS + xi)
  double* U = L.spWork;
  double* rhs = U + (size_t)N * N;
  double* ws = rhs + N;
  double* LDL = ws + dense_ws_doubles(N);
  const int g1 = (N + 255) / 256;
  sp_rhs_kernel<<<g1, 256, 0, s.stream>>>(a, rhs, LDL);
  sp_assemble_kernel<<<dim3(g1, N), 256, 0, s.stream>>>(a, U, LDL);
  HIP_OK(hipGetLastError());
  {
    ProfScope pc(s, PROF_CHOL);
    dense_potrf_lower(s.stream, U, N, N, ws, s.dev_flags, 0, s.trsv_sync);
  }
  dense_trsv_lower(s.stream, U, N, N, rhs, 0, ws, 0, s.trsv_sync);   // backsolve(R, fS, transpose = TRUE)
  sp_noise_kernel<<<g1, 256, 0, s.stream>>>(a, rhs);
  dense_trsv_lower(s.stream, U, N, N, rhs, 1, ws, 0, s.trsv_sync);   // backsolve(R, tmp2)
  sp_store_kernel<<<g1, 256, 0, s.stream>>>(a, rhs);
  HIP_OK(hipGetLastError());
}

void launch_alpha(State& s, uint32_t iter) {
  for (int r = 0; r < s.nr; ++r) {
    if (!s.lev[r].spatial || s.lev[r].nf == 0) continue;  // rep(1, nf) otherwise (R/updateAlpha.R:81-82)
    sp_ensure_capacity(s, r);
    const Level& L = s.lev[r];
    const SpArgs a = sp_args(s, r, iter);
    ProfScope ps(s, PROF_ALPHA);
    if (L.gpp) {
      HMSC_REQUIRE(L.nK <= 1024, "GPP level: at most 1024 knots in this build");  // t2[1024] in LDS
      const GppLayout o = gpp_layout(L.np, sp_nfc(L), L.nK, L.nalpha);
      SpArgs b = a;
      b.work = L.spWork + o.alpha;
      gpp_alpha_kernel<<<L.nalpha, 256, 0, s.stream>>>(b, b.work);
      HIP_OK(hipGetLastError());
      alpha_draw_kernel<<<1, 256, 0, s.stream>>>(b);
      HIP_OK(hipGetLastError());
      continue;
    }
    if (L.nngp) {  // the band matrix at the start of spWork stays untouched (zeros outside the band)
      SpArgs b = a;
      b.work = L.spWork + nn_layout(L.np, sp_nfc(L), L.nnBwUnits).tot;
      nngp_alpha_kernel<<<dim3(L.nalpha, (L.np + 255) / 256), 256, 0, s.stream>>>(b, nn_args(s, r));
      HIP_OK(hipGetLastError());
      alpha_draw_kernel<<<1, 256, 0, s.stream>>>(b);
      HIP_OK(hipGetLastError());
      continue;
    }
    alpha_quad_kernel<<<dim3(L.nalpha, (L.np + 255) / 256), 256, 0, s.stream>>>(a);
    HIP_OK(hipGetLastError());
    alpha_draw_kernel<<<1, 256, 0, s.stream>>>(a);
    HIP_OK(hipGetLastError());
  }
}

// ---------------------------------------------------------------------------------------
// the 'Full' alphapw grid on the device (R/computeDataParameters.R:53-81): for every grid
// point W = exp(-d / alpha) (W = I for alpha = 0), RW = chol(W), detW = 2 sum log diag(RW),
// iW = chol2inv(RW).  R keeps RiW = chol(iW) (upper); here RiW = RW^-1 with RW the lower
// factor, which has the same RiW' RiW = iW and quadratic forms, so updateAlpha reads it
// through riw_lower.  Costs per grid point: chol + trtri + lauum = np^3 flops on MFMA.
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void sp_w_kernel(double* W, int np, int sdim, const double* crd, const double* dist,
                                                   double alpha) {
  const int q = blockIdx.y, p = blockIdx.x * 256 + threadIdx.x;
  if (p >= np || p < q) return;
  double d;
  if (dist) {
    d = dist[p + (size_t)np * q];
  } else {  // dist(s): sqrt of the summed squared coordinate differences
    double s = 0.0;
    for (int k = 0; k < sdim; ++k) {
      const double e = crd[p + (size_t)np * k] - crd[q + (size_t)np * k];
      s += e * e;
    }
    d = sqrt(s);
  }
  W[p + (size_t)np * q] = exp(-d / alpha);
}

__global__ __launch_bounds__(256) void sp_logdet_kernel(const double* L, int n, double* out) {
  __shared__ double red[256];
  double s = 0.0;
  for (int i = threadIdx.x; i < n; i += 256) s += log(L[i + (size_t)n * i]);
  red[threadIdx.x] = s;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) *out = 2.0 * red[0];
}

__global__ __launch_bounds__(256) void sp_identity_kernel(double* A, double* B, int n) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) A[i + (size_t)n * i] = B[i + (size_t)n * i] = 1.0;
}

void spatial_full_grid(hipStream_t st, int np, int sdim, const double* coords, const double* dist,
                       const double* alphas, int G, double* iWg, double* RiWg, double* detWg, int* info) {
  const size_t n2 = (size_t)np * np;
  double *W = nullptr, *dinv = nullptr;
  int* sync = nullptr;  // the dense handshake block (the fused panel step's flag timeout)
  HIP_OK(hipMalloc(&W, n2 * sizeof(double)));
  HIP_OK(hipMalloc(&dinv, dense_ws_doubles(np) * sizeof(double)));
  HIP_OK(hipMalloc(&sync, DENSE_SYNC_INTS * sizeof(int)));
  HIP_OK(hipMemsetAsync(sync, 0, DENSE_SYNC_INTS * sizeof(int), st));
  for (int g = 0; g < G; ++g) {
    double* iW = iWg + n2 * g;
    double* RiW = RiWg + n2 * g;
    if (alphas[g] == 0.0) {
      HIP_OK(hipMemsetAsync(iW, 0, n2 * sizeof(double), st));
      HIP_OK(hipMemsetAsync(RiW, 0, n2 * sizeof(double), st));
      HIP_OK(hipMemsetAsync(detWg + g, 0, sizeof(double), st));
      sp_identity_kernel<<<(np + 255) / 256, 256, 0, st>>>(iW, RiW, np);
      continue;
    }
    sp_w_kernel<<<dim3((np + 255) / 256, np), 256, 0, st>>>(W, np, sdim, coords, dist, alphas[g]);
    dense_potrf_lower(st, W, np, np, dinv, info, 0, sync);
    sp_logdet_kernel<<<1, 256, 0, st>>>(W, np, detWg + g);
    dense_trtri_lower(st, W, np, np, RiW, np, dinv, true);
    dense_lauum_lower(st, RiW, np, np, iW, np);
  }
  HIP_OK(hipGetLastError());
  int err = 0;
  HIP_OK(hipMemcpyAsync(&err, sync + DENSE_SYNC_ERR, sizeof(int), hipMemcpyDeviceToHost, st));
  HIP_OK(hipStreamSynchronize(st));
  HIP_OK(hipFree(W));
  HIP_OK(hipFree(dinv));
  HIP_OK(hipFree(sync));
  HMSC_REQUIRE(err == 0, "spatial grid: an in-launch handshake of the blocked Cholesky timed out (error bits " +
                             std::to_string(err) + ")");
}

}  // namespace hmsc
