// updateGammaEta on the device (R/updateGammaEta.R:7-206), levels with xDim = 0: non-spatial
// levels below, spatial 'Full' levels in gamma_eta_spatial_kernel further down.
//
// Per random level r (sequentially, each level sees the new Eta of the levels before it):
//   S    = Z - sum_{q != r} Eta_q[Pi_q,] Lambda_q                                  (:37-42)
//   A    = (Tr x I) U (Tr x I)^T + Q x V,  iA = A^-1                               (:32-33)
//   Beta ~ N(A (mb10 - mb20 - mb30), M^-1),  M = iA + T1                            (:57-66 / :101-126)
//          with T1 = kron(diag(id) - LamiD' iW0 LamiD, X'X)       (np = ny, one W0 = I + Lam D Lam')
//          or   T1 = kron(diag(id), X'X) - sum_p (P'X)_p (P'X)_p' x LamiD' iW_p LamiD  (np < ny)
//   Gamma ~ N(Pg^-1 vec(iV Beta iQ Tr), Pg^-1),  Pg = iU + (Tr' iQ Tr) x iV          (:66-69)
//   Eta_r | Beta, S: per row (np = ny) or per unit (np < ny) nf x nf solves          (:71-74 / :136-146)
// Beta is an auxiliary draw and is discarded, as in the reference.
//
// The whole update is one workgroup (1024 threads) per level on an L2-resident workspace:
// the dense systems are (nc ns)^2 -- tiny at the configs that run this updater (TD: 12,
// vignette_3: a few hundred) -- and every step is a chain of dependent factorizations,
// so a single workgroup with barrier-separated stages is the latency-optimal shape.
// Randomness (oracle/hmsc_oracle.py update_gamma_eta): Beta normal(c + nc j, 0, S_GE_BETA),
// Gamma normal(c + nc t, 0, S_GE_GAMMA), Eta normal(row i | unit p, h, S_GE_ETA), each
// + LEVEL_STRIDE r.
#include "common.h"
#include "state.h"
#include "wave_la.h"

namespace hmsc {

// Per-thread arrays over the level's factors (tv, x1) are sized by a compile-time capacity:
// the launcher picks the 16-factor instantiation while nf <= 16 (registers), the 64-factor one
// up to 64 and the 128-factor one above it (K = nc + sum nf <= 128 bounds nf; its arrays live
// in scratch memory, slower but with no factor limit below the chain's), so the updater follows
// the nf in use -- R's default nfMax = ns (R/Hmsc.R:554, truncated to the allocation) adapts
// upward from nfMin = 2 (R/updateNf.R) -- instead of refusing a large nfMax at chain creation.
constexpr int GE_NF_SMALL = 16;
constexpr int GE_NF_LARGE = 64;
constexpr int GE_NF_XL = HMSC_KCAP;

struct GEArgs {
  int ny, ns, nc, nt, K, r, nr, nf, np, loff;
  int lev_np[HMSC_MAX_LEVELS], lev_nf[HMSC_MAX_LEVELS], lev_loff[HMSC_MAX_LEVELS];
  const double* lev_eta[HMSC_MAX_LEVELS];
  const int* lev_pi[HMSC_MAX_LEVELS];
  double* Eta;            // level r, np x nf (ld np), written
  const int* unit_ptr;    // level r CSR over rows
  const int* unit_rows;
  const double* Z;        // ny x ns
  const double* X;        // ny x nc
  const double* Tr;       // ns x nt
  const double* BL;       // K x ns   [Beta; Lambda_1; ...]
  const double* iSigma;   // ns
  const double* UGamma;   // (nc nt)^2
  const double* iUGamma;  // (nc nt)^2
  const double* iV;       // nc x nc
  double* Gamma;          // nc x nt, written
  // phylogeny: iQ = U diag(w) U^T, Q = U diag(1/w) U^T (w = Winv row rho); null: identity
  const double* phU;
  const double* phWinv;
  const double* rho;
  double* work;
  int* fail;
  Key key;
  uint32_t iter;
  const uint32_t* iter_dev;
  int noise_zero;
};

// workspace carve-up (doubles), shared by the launcher's size computation
struct GELayout {
  size_t A, L, M, T, S, XtX, V, Wv, XtS, LamiD, LDL, W0, iW0, L0i, tmp1, Qm, iQm, iQTr, vec, Beta, Pg, rg, PtX, PtS,
      iWp, Lip, Ltp, m21, tot;
};

__host__ __device__ inline GELayout ge_layout(int ny, int ns, int nc, int nt, int nf, int np) {
  GELayout o{};
  const size_t N = (size_t)nc * ns, G = (size_t)nc * nt;
  size_t p = 0;
  auto take = [&](size_t n) {
    const size_t at = p;
    p += (n + 7) & ~(size_t)7;
    return at;
  };
  o.A = take(N * N);
  o.L = take(N * N);
  o.M = take(N * N);
  o.T = take(N * N);
  o.S = take((size_t)ny * ns);
  o.XtX = take((size_t)nc * nc);
  o.V = take((size_t)nc * nc);
  o.Wv = take((size_t)nc * nc);
  o.XtS = take(N);
  o.LamiD = take((size_t)nf * ns);
  o.LDL = take((size_t)nf * nf);
  o.W0 = take((size_t)nf * nf);
  o.iW0 = take((size_t)nf * nf);
  o.L0i = take((size_t)nf * nf);
  o.tmp1 = take((size_t)ns * ns);
  o.Qm = take((size_t)ns * ns);
  o.iQm = take((size_t)ns * ns);
  o.iQTr = take((size_t)ns * nt);
  o.vec = take(6 * N);
  o.Beta = take(N);
  o.Pg = take(G * G);
  o.rg = take(G);
  o.PtX = take((size_t)np * nc);
  o.PtS = take((size_t)np * ns);
  o.iWp = take((size_t)np * nf * nf);
  o.Lip = take((size_t)np * nf * nf);
  o.Ltp = take((size_t)np * nf * ns);
  o.m21 = take((size_t)np * nf);
  o.tot = p;
  return o;
}

// Workspace pointers of one level's update (ge_layout)
struct GEPtrs {
  double *A, *L, *M, *T, *S, *XtX, *V, *Wv, *XtS, *LamiD, *LDL, *W0, *iW0, *L0i, *tmp1, *Qm, *iQm, *iQTr;
  double *mb10, *mb20, *v, *wv, *mb, *xi, *Beta, *Pg, *rg, *PtX, *PtS, *iWp, *Lip, *Ltp, *m21;
  bool obs;
  int N, G;
};

__host__ __device__ inline GEPtrs ge_ptrs(const GEArgs& a) {
  GEPtrs P;
  P.obs = (a.np == a.ny);
  P.N = a.nc * a.ns;
  P.G = a.nc * a.nt;
  const GELayout o = ge_layout(a.ny, a.ns, a.nc, a.nt, a.nf, P.obs ? 0 : a.np);
  double* w = a.work;
  P.A = w + o.A, P.L = w + o.L, P.M = w + o.M, P.T = w + o.T, P.S = w + o.S, P.XtX = w + o.XtX, P.V = w + o.V;
  P.Wv = w + o.Wv, P.XtS = w + o.XtS, P.LamiD = w + o.LamiD, P.LDL = w + o.LDL, P.W0 = w + o.W0, P.iW0 = w + o.iW0;
  P.L0i = w + o.L0i, P.tmp1 = w + o.tmp1, P.Qm = w + o.Qm, P.iQm = w + o.iQm, P.iQTr = w + o.iQTr;
  P.mb10 = w + o.vec, P.mb20 = P.mb10 + P.N, P.v = P.mb20 + P.N, P.wv = P.v + P.N, P.mb = P.wv + P.N,
  P.xi = P.mb + P.N;
  P.Beta = w + o.Beta, P.Pg = w + o.Pg, P.rg = w + o.rg, P.PtX = w + o.PtX, P.PtS = w + o.PtS, P.iWp = w + o.iWp;
  P.Lip = w + o.Lip, P.Ltp = w + o.Ltp, P.m21 = w + o.m21;
  return P;
}

// The update's element-parallel segments.  Each loops p = g0, g0 + gs, ...: the one-workgroup
// kernel calls them with (threadIdx.x, blockDim.x) between its barriers, the blocked path
// (large nc ns) with the global thread index and grid size from one launch per segment.

// S, X'X (+ a copy of iV), LamiD, Lam D Lam', Q / iQ   (:37-42, :27-31)
__device__ inline void ge_seg_prep(const GEArgs& a, const GEPtrs& P, int g0, int gs, bool with_q = true,
                                   bool with_sums = true) {
  const int ny = a.ny, ns = a.ns, nc = a.nc, nf = a.nf, K = a.K;
  const double* lam = a.BL + a.loff;  // Lambda_r[h, j] = lam[h + K j]
  for (size_t p = g0; p < (size_t)ny * ns; p += gs) {
    const int i = (int)(p % ny), j = (int)(p / ny);
    double sv = a.Z[p];
    for (int q = 0; q < a.nr; ++q) {
      if (q == a.r) continue;
      const double* eq = a.lev_eta[q];
      const int u = a.lev_pi[q][i], npq = a.lev_np[q];
      const double* lq = a.BL + a.lev_loff[q] + (size_t)K * j;
      for (int h = 0; h < a.lev_nf[q]; ++h) sv -= eq[u + (size_t)npq * h] * lq[h];
    }
    P.S[p] = sv;
  }
  for (int p = g0; p < nc * nc; p += gs) {
    const int c1 = p % nc, c2 = p / nc;
    if (with_sums) {
      double s = 0.0;
      for (int i = 0; i < ny; ++i) s = fma(a.X[i + (size_t)ny * c1], a.X[i + (size_t)ny * c2], s);
      P.XtX[p] = s;
    }
    P.Wv[p] = a.iV[p];
  }
  for (int p = g0; p < nf * ns; p += gs) {
    const int h = p % nf, j = p / nf;
    P.LamiD[p] = lam[h + (size_t)K * j] * a.iSigma[j];
  }
  if (with_sums)
    for (int p = g0; p < nf * nf; p += gs) {
      const int h1 = p % nf, h2 = p / nf;
      double s = 0.0;
      for (int j = 0; j < ns; ++j) s = fma(lam[h1 + (size_t)K * j] * a.iSigma[j], lam[h2 + (size_t)K * j], s);
      P.LDL[p] = s;
    }
  if (!with_q) return;  // (blocked path: Q / iQ by dense_gram_diag)
  if (a.phU) {
    const double* wq = a.phWinv + (size_t)ns * ((int)(*a.rho) - 1);
    for (int p = g0; p < ns * ns; p += gs) {
      const int j1 = p % ns, j2 = p / ns;
      double s = 0.0, si = 0.0;
      for (int i = 0; i < ns; ++i) {
        const double uu = a.phU[j1 + (size_t)ns * i] * a.phU[j2 + (size_t)ns * i];
        si = fma(uu, wq[i], si);
        s = fma(uu, 1.0 / wq[i], s);
      }
      P.iQm[p] = si;
      P.Qm[p] = s;
    }
  } else {
    for (int p = g0; p < ns * ns; p += gs) P.iQm[p] = P.Qm[p] = (p % ns == p / ns) ? 1.0 : 0.0;
  }
}

// X'S, iQ Tr
__device__ inline void ge_seg_xts(const GEArgs& a, const GEPtrs& P, int g0, int gs) {
  const int ny = a.ny, ns = a.ns, nc = a.nc, nt = a.nt;
  for (int p = g0; p < P.N; p += gs) {
    const int c = p % nc, j = p / nc;
    double s = 0.0;
    for (int i = 0; i < ny; ++i) s = fma(a.X[i + (size_t)ny * c], P.S[i + (size_t)ny * j], s);
    P.XtS[p] = s;
  }
  for (int p = g0; p < ns * nt; p += gs) {
    const int j = p % ns, q = p / ns;
    double s = 0.0;
    for (int j2 = 0; j2 < ns; ++j2) s = fma(P.iQm[j + (size_t)ns * j2], a.Tr[j2 + (size_t)ns * q], s);
    P.iQTr[p] = s;
  }
}

// A = (Tr x I) U (Tr x I)^T + Q x V   (:32), and its copy L to be factorised
__device__ inline void ge_seg_a(const GEArgs& a, const GEPtrs& P, int g0, int gs) {
  const int ns = a.ns, nc = a.nc, nt = a.nt, N = P.N, G = P.G;
  for (size_t p = g0; p < (size_t)N * N; p += gs) {
    const int r1 = (int)(p % N), r2 = (int)(p / N);
    const int c1 = r1 % nc, j1 = r1 / nc, c2 = r2 % nc, j2 = r2 / nc;
    double s = P.Qm[j1 + (size_t)ns * j2] * P.V[c1 + nc * c2];
    for (int t1 = 0; t1 < nt; ++t1) {
      const double a1 = a.Tr[j1 + (size_t)ns * t1];
      for (int t2 = 0; t2 < nt; ++t2)
        s = fma(a1 * a.UGamma[(c1 + nc * t1) + (size_t)G * (c2 + nc * t2)], a.Tr[j2 + (size_t)ns * t2], s);
    }
    P.A[p] = s;
    P.L[p] = s;
  }
}

// np = ny: W0 = Lam D Lam' + I, RW0 = chol(W0), iW0 = chol2inv(RW0)  (:53-55); one thread
__device__ inline bool ge_w0(const GEArgs& a, const GEPtrs& P) {
  const int nf = a.nf;
  for (int p = 0; p < nf * nf; ++p) P.W0[p] = P.LDL[p] + ((p % nf == p / nf) ? 1.0 : 0.0);
  const bool ok = t_chol_inv(P.W0, P.L0i, nf);
  for (int h1 = 0; h1 < nf; ++h1)
    for (int h2 = 0; h2 < nf; ++h2) {
      double s = 0.0;
      for (int k = 0; k < nf; ++k) s += P.L0i[k + nf * h1] * P.L0i[k + nf * h2];
      P.iW0[h1 + nf * h2] = s;
    }
  return ok;
}

// np = ny: tmp1 = diag(id) - LamiD' iW0 LamiD   (:57)
__device__ inline void ge_seg_tmp1(const GEArgs& a, const GEPtrs& P, int g0, int gs) {
  const int ns = a.ns, nf = a.nf;
  for (int p = g0; p < ns * ns; p += gs) {
    const int j1 = p % ns, j2 = p / ns;
    double s = 0.0;
    for (int h1 = 0; h1 < nf; ++h1) {
      double u = 0.0;
      for (int h2 = 0; h2 < nf; ++h2) u = fma(P.iW0[h1 + nf * h2], P.LamiD[h2 + nf * j2], u);
      s = fma(P.LamiD[h1 + nf * j1], u, s);
    }
    P.tmp1[p] = (j1 == j2 ? a.iSigma[j1] : 0.0) - s;
  }
}

// np = ny: M = iA + kron(tmp1, X'X) (:58), mb20 = vec((X'S LamiD') iW0 LamiD) (:62)
template <int NFC>
__device__ inline void ge_seg_m_obs(const GEArgs& a, const GEPtrs& P, int g0, int gs) {
  const int ns = a.ns, nc = a.nc, nf = a.nf, N = P.N;
  for (size_t p = g0; p < (size_t)N * N; p += gs) {
    const int r1 = (int)(p % N), r2 = (int)(p / N);
    P.M[p] += P.tmp1[(r1 / nc) + (size_t)ns * (r2 / nc)] * P.XtX[(r1 % nc) + nc * (r2 % nc)];
  }
  for (int p = g0; p < N; p += gs) {
    const int c = p % nc, j = p / nc;
    double x1[NFC];  // (X'S LamiD')[c, h1]: the same for every j, formed once
    for (int h1 = 0; h1 < nf; ++h1) {
      double x = 0.0;
      for (int j2 = 0; j2 < ns; ++j2) x = fma(P.XtS[c + nc * j2], P.LamiD[h1 + nf * j2], x);
      x1[h1] = x;
    }
    double s = 0.0;
    for (int h2 = 0; h2 < nf; ++h2) {
      double u = 0.0;
      for (int h1 = 0; h1 < nf; ++h1) u = fma(x1[h1], P.iW0[h1 + nf * h2], u);
      s = fma(u, P.LamiD[h2 + nf * j], s);
    }
    P.mb20[p] = s;
  }
}

// np < ny, per unit q: P'X, P'S, W_p = I + n_p Lam D Lam', iW_p, LiW_p^T LamiD, mb22_p (:78-117)
__device__ inline bool ge_seg_units(const GEArgs& a, const GEPtrs& P, int g0, int gs) {
  const int ny = a.ny, ns = a.ns, nc = a.nc, nf = a.nf, np = a.np;
  bool ok = true;
  for (int q = g0; q < np; q += gs) {
    const int b = a.unit_ptr[q], e = a.unit_ptr[q + 1];
    for (int c = 0; c < nc; ++c) {
      double s = 0.0;
      for (int k = b; k < e; ++k) s += a.X[a.unit_rows[k] + (size_t)ny * c];
      P.PtX[q + (size_t)np * c] = s;
    }
    for (int j = 0; j < ns; ++j) {
      double s = 0.0;
      for (int k = b; k < e; ++k) s += P.S[a.unit_rows[k] + (size_t)ny * j];
      P.PtS[q + (size_t)np * j] = s;
    }
    double* Wq = P.iWp + (size_t)q * nf * nf;  // W_p factorised in place, then replaced by iW_p
    double* Li = P.Lip + (size_t)q * nf * nf;
    const double cnt = (double)(e - b);
    for (int p = 0; p < nf * nf; ++p) Wq[p] = ((p % nf == p / nf) ? 1.0 : 0.0) + cnt * P.LDL[p];
    if (!t_chol_inv(Wq, Li, nf)) ok = false;
    for (int h1 = 0; h1 < nf; ++h1)
      for (int h2 = 0; h2 < nf; ++h2) {
        double s = 0.0;
        for (int k = 0; k < nf; ++k) s += Li[k + nf * h1] * Li[k + nf * h2];
        Wq[h1 + nf * h2] = s;
      }
    // Lt_p = L_p^-1 LamiD  (nf x ns): rows of LiW_p^T LamiD  (:104)
    double* Lt = P.Ltp + (size_t)q * nf * ns;
    for (int j = 0; j < ns; ++j)
      for (int h = 0; h < nf; ++h) {
        double s = 0.0;
        for (int k = 0; k <= h; ++k) s += Li[h + nf * k] * P.LamiD[k + nf * j];
        Lt[h + (size_t)nf * j] = s;
      }
    // mb22_p = iW_p (P'S LamiD')_p    (:115-117)
    for (int h = 0; h < nf; ++h) {
      double s = 0.0;
      for (int h2 = 0; h2 < nf; ++h2) {
        double u = 0.0;
        for (int j = 0; j < ns; ++j) u = fma(P.PtS[q + (size_t)np * j], P.LamiD[h2 + nf * j], u);
        s = fma(Wq[h + nf * h2], u, s);
      }
      P.m21[q + (size_t)np * h] = s;
    }
  }
  return ok;
}

// np < ny: T = kron(diag(id), X'X) - sum_p (P'X)_p (P'X)_p' x Lt_p' Lt_p ; M = iA + T (:105-108),
// mb20 = vec(P'X' mb22 LamiD) (:118)
__device__ inline void ge_seg_m_units(const GEArgs& a, const GEPtrs& P, int g0, int gs) {
  const int ns = a.ns, nc = a.nc, nf = a.nf, np = a.np, N = P.N;
  for (size_t p = g0; p < (size_t)N * N; p += gs) {
    const int r1 = (int)(p % N), r2 = (int)(p / N);
    const int c1 = r1 % nc, j1 = r1 / nc, c2 = r2 % nc, j2 = r2 / nc;
    double s = 0.0;
    for (int q = 0; q < np; ++q) {
      const double* Lt = P.Ltp + (size_t)q * nf * ns;
      double u = 0.0;
      for (int h = 0; h < nf; ++h) u = fma(Lt[h + (size_t)nf * j1], Lt[h + (size_t)nf * j2], u);
      s = fma(P.PtX[q + (size_t)np * c1] * P.PtX[q + (size_t)np * c2], u, s);
    }
    const double tv = (j1 == j2 ? a.iSigma[j1] * P.XtX[c1 + nc * c2] : 0.0) - s;
    P.T[p] = tv;
    P.M[p] += tv;
  }
  for (int p = g0; p < N; p += gs) {
    const int c = p % nc, j = p / nc;
    double s = 0.0;
    for (int h = 0; h < nf; ++h) {
      double u = 0.0;
      for (int q = 0; q < np; ++q) u = fma(P.PtX[q + (size_t)np * c], P.m21[q + (size_t)np * h], u);
      s = fma(u, P.LamiD[h + nf * j], s);
    }
    P.mb20[p] = s;
  }
}

// mb10 = vec(X'S o id) (:61 / :113), v = mb10 - mb20 (same index set as mb20's loop)
__device__ inline void ge_seg_mb10(const GEArgs& a, const GEPtrs& P, int g0, int gs) {
  for (int p = g0; p < P.N; p += gs) {
    P.mb10[p] = P.XtS[p] * a.iSigma[p / a.nc];
    P.v[p] = P.mb10[p] - P.mb20[p];
  }
}

// with v = M^-1 (mb10 - mb20): wv = mb10 - mb20 - T1 v (mb30, :63-64), xi ~ N(0, I)
__device__ inline void ge_seg_wv(const GEArgs& a, const GEPtrs& P, int g0, int gs, uint32_t it) {
  const int ns = a.ns, nc = a.nc, N = P.N;
  const uint32_t str = LEVEL_STRIDE * (uint32_t)a.r;
  for (int p = g0; p < N; p += gs) {
    const int c = p % nc, j = p / nc;
    double s = 0.0;
    if (P.obs) {
      for (int j2 = 0; j2 < ns; ++j2) {
        const double tj = P.tmp1[j + (size_t)ns * j2];
        if (tj == 0.0) continue;
        double u = 0.0;
        for (int c2 = 0; c2 < nc; ++c2) u = fma(P.XtX[c + nc * c2], P.v[c2 + nc * j2], u);
        s = fma(tj, u, s);
      }
    } else {
      for (int p2 = 0; p2 < N; ++p2) s = fma(P.T[p + (size_t)N * p2], P.v[p2], s);
    }
    P.wv[p] = P.mb10[p] - P.mb20[p] - s;
    P.xi[p] = a.noise_zero ? 0.0 : normal(a.key, (uint32_t)p, 0, S_GE_BETA + str, it);
  }
}

// mb = A wv   (:65)
__device__ inline void ge_seg_mb(const GEPtrs& P, int g0, int gs) {
  const int N = P.N;
  for (int p = g0; p < N; p += gs) {
    double s = 0.0;
    for (int p2 = 0; p2 < N; ++p2) s = fma(P.A[p + (size_t)N * p2], P.wv[p2], s);
    P.mb[p] = s;
  }
}

// Beta = mb + RM^-1 xi (xi already back-solved); then Gamma | Beta (:66-71) -- one workgroup
__device__ inline void ge_wg_gamma(const GEArgs& a, const GEPtrs& P, int* flag, uint32_t it) {
  const int t = threadIdx.x, nthr = blockDim.x;
  const int ns = a.ns, nc = a.nc, G = P.G, N = P.N;
  const uint32_t str = LEVEL_STRIDE * (uint32_t)a.r;
  for (int p = t; p < N; p += nthr) P.Beta[p] = P.mb[p] + P.xi[p];
  __syncthreads();
  for (size_t p = t; p < (size_t)G * G; p += nthr) {
    const int r1 = (int)(p % G), r2 = (int)(p / G);
    const int c1 = r1 % nc, t1 = r1 / nc, c2 = r2 % nc, t2 = r2 / nc;
    double tq = 0.0;
    for (int j = 0; j < ns; ++j) tq = fma(a.Tr[j + (size_t)ns * t1], P.iQTr[j + (size_t)ns * t2], tq);
    P.Pg[p] = a.iUGamma[p] + tq * a.iV[c1 + nc * c2];
  }
  for (int p = t; p < G; p += nthr) {
    const int c = p % nc, q = p / nc;
    double s = 0.0;
    for (int j = 0; j < ns; ++j) {
      double ib = 0.0;
      for (int c2 = 0; c2 < nc; ++c2) ib = fma(a.iV[c + nc * c2], P.Beta[c2 + nc * j], ib);
      s = fma(ib, P.iQTr[j + (size_t)ns * q], s);
    }
    P.rg[p] = s;
  }
  __syncthreads();
  if (!wg_chol(P.Pg, G, G, flag) && t == 0) a.fail[0] = 1;
  wg_forward(P.Pg, G, G, P.rg);
  for (int p = t; p < G; p += nthr)
    if (!a.noise_zero) P.rg[p] += normal(a.key, (uint32_t)p, 0, S_GE_GAMMA + str, it);
  __syncthreads();
  wg_backward_t(P.Pg, G, G, P.rg);
  for (int p = t; p < G; p += nthr) a.Gamma[p] = P.rg[p];
}

// Eta | Beta, S   (:71-74 / :136-146); S1 = S - X Beta, per row (np = ny) or per unit
template <int NFC>
__device__ inline void ge_seg_eta(const GEArgs& a, const GEPtrs& P, int g0, int gs, uint32_t it) {
  const int ny = a.ny, ns = a.ns, nc = a.nc, nf = a.nf, np = a.np;
  const uint32_t str = LEVEL_STRIDE * (uint32_t)a.r;
  if (P.obs) {
    for (int i = g0; i < ny; i += gs) {
      double tv[NFC];
      for (int h = 0; h < nf; ++h) tv[h] = 0.0;
      for (int j = 0; j < ns; ++j) {
        double s1 = P.S[i + (size_t)ny * j];
        for (int c = 0; c < nc; ++c) s1 -= a.X[i + (size_t)ny * c] * P.Beta[c + nc * j];
        for (int h = 0; h < nf; ++h) tv[h] = fma(s1, P.LamiD[h + nf * j], tv[h]);
      }
      const int u = a.lev_pi[a.r][i];
      for (int h = 0; h < nf; ++h) {
        double me = 0.0, nz = 0.0;
        for (int h2 = 0; h2 < nf; ++h2) me = fma(tv[h2], P.iW0[h2 + nf * h], me);
        if (!a.noise_zero)
          for (int h2 = h; h2 < nf; ++h2)  // (RW0^-1 xi)_h = sum_h2 L0i[h2, h] xi_h2
            nz = fma(P.L0i[h2 + nf * h], normal(a.key, (uint32_t)i, (uint32_t)h2, S_GE_ETA + str, it), nz);
        a.Eta[u + (size_t)np * h] = me + nz;
      }
    }
  } else {
    for (int q = g0; q < np; q += gs) {
      double tv[NFC];
      for (int h = 0; h < nf; ++h) tv[h] = 0.0;
      for (int j = 0; j < ns; ++j) {
        double s1 = P.PtS[q + (size_t)np * j];
        for (int c = 0; c < nc; ++c) s1 -= P.PtX[q + (size_t)np * c] * P.Beta[c + nc * j];
        for (int h = 0; h < nf; ++h) tv[h] = fma(s1, P.LamiD[h + nf * j], tv[h]);
      }
      const double* iW = P.iWp + (size_t)q * nf * nf;
      const double* Li = P.Lip + (size_t)q * nf * nf;
      for (int h = 0; h < nf; ++h) {
        double me = 0.0, nz = 0.0;
        for (int h2 = 0; h2 < nf; ++h2) me = fma(iW[h + nf * h2], tv[h2], me);
        if (!a.noise_zero)
          for (int h2 = h; h2 < nf; ++h2)  // (LiW_p xi)_h = sum_h2 Li[h2, h] xi_h2
            nz = fma(Li[h2 + nf * h], normal(a.key, (uint32_t)q, (uint32_t)h2, S_GE_ETA + str, it), nz);
        a.Eta[q + (size_t)np * h] = me + nz;
      }
    }
  }
}

// One workgroup per level (small nc ns): the segments between barriers, the factorizations
// by wg_chol / wg_chol2inv on the L2-resident workspace.
template <int NFC>
__global__ __launch_bounds__(1024) void gamma_eta_kernel(GEArgs a) {
  __shared__ int flag;
  const int t = threadIdx.x, nthr = blockDim.x;
  const GEPtrs P = ge_ptrs(a);
  const int N = P.N, nc = a.nc;
  const uint32_t it = SWEEP_ITER(a);
  ge_seg_prep(a, P, t, nthr);
  __syncthreads();
  // V = chol2inv(chol(iV))
  if (!wg_chol(P.Wv, nc, nc, &flag) && t == 0) a.fail[0] = 1;
  wg_chol2inv(P.Wv, nc, nc, P.V, nc, P.T /* scratch: nc^2 <= N^2 */);
  ge_seg_xts(a, P, t, nthr);
  ge_seg_a(a, P, t, nthr);
  __syncthreads();
  // iA = chol2inv(chol(A)) into M (scratch T)
  if (!wg_chol(P.L, N, N, &flag) && t == 0) a.fail[0] = 1;
  wg_chol2inv(P.L, N, N, P.M, N, P.T);
  if (P.obs) {
    if (t == 0 && !ge_w0(a, P)) a.fail[0] = 1;
    __syncthreads();
    ge_seg_tmp1(a, P, t, nthr);
    __syncthreads();
    ge_seg_m_obs<NFC>(a, P, t, nthr);
  } else {
    if (!ge_seg_units(a, P, t, nthr)) a.fail[0] = 1;
    __syncthreads();
    ge_seg_m_units(a, P, t, nthr);
  }
  ge_seg_mb10(a, P, t, nthr);
  __syncthreads();
  // RM = chol(M); v = M^-1 (mb10 - mb20)
  if (!wg_chol(P.M, N, N, &flag) && t == 0) a.fail[0] = 1;
  wg_forward(P.M, N, N, P.v);
  wg_backward_t(P.M, N, N, P.v);
  ge_seg_wv(a, P, t, nthr, it);
  __syncthreads();
  ge_seg_mb(P, t, nthr);
  __syncthreads();
  wg_backward_t(P.M, N, N, P.xi);  // backsolve(RM, rnorm(nc ns))  (:66)
  ge_wg_gamma(a, P, &flag, it);
  __syncthreads();
  ge_seg_eta<NFC>(a, P, t, nthr, it);
}

// ---- the blocked path (nc ns > GE_WG_MAX): one launch per segment, the three (nc ns)^2
// factorizations (chol(A) and its inverse, chol(M)) and the solves on dense.hip's
// multi-workgroup MFMA kernels
constexpr int GE_WG_MAX = 512;

#define GE_GRID_IDX                                        \
  const GEPtrs P = ge_ptrs(a);                             \
  const int g0 = blockIdx.x * blockDim.x + threadIdx.x;    \
  const int gs = gridDim.x * blockDim.x;                   \
  (void)P, (void)g0, (void)gs;

// The blocked path's reductions: one wave per output, lanes over the summation index
// (coalesced where the operand is a column), U terms' loads in flight per lane, a
// cross-lane sum at the end.  (A thread per output with a serial loop over ns or nc ns
// terms waited out one L2 round trip per few terms: 0.1-0.3 ms per segment at nc ns = 1200.)
template <int U, class F>
__device__ inline double wave_sum(int n, F f) {
  const int lane = threadIdx.x & 63;
  double s = 0.0;
  for (int k0 = lane; k0 < n; k0 += 64 * U) {
    double v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = k0 + 64 * u < n ? f(k0 + 64 * u) : 0.0;
#pragma unroll
    for (int u = 0; u < U; ++u) s += v[u];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  return s;
}

#define GE_WAVE_IDX                                                      \
  const GEPtrs P = ge_ptrs(a);                                           \
  const int lane = threadIdx.x & 63;                                     \
  const int w0 = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);    \
  const int ws = (int)((gridDim.x * blockDim.x) >> 6);                   \
  (void)P, (void)lane;

__global__ __launch_bounds__(256) void ge_b_prep_kernel(GEArgs a) {
  GE_GRID_IDX
  ge_seg_prep(a, P, g0, gs, a.phU == nullptr, false);
  // X'X and Lam D Lam', one wave per entry
  const int lane = threadIdx.x & 63, w0 = g0 >> 6, ws = gs >> 6;
  const int ny = a.ny, ns = a.ns, nc = a.nc, nf = a.nf, K = a.K;
  const double* lam = a.BL + a.loff;
  for (int p = w0; p < nc * nc + nf * nf; p += ws) {
    if (p < nc * nc) {
      const int c1 = p % nc, c2 = p / nc;
      const double s = wave_sum<8>(ny, [&](int i) { return a.X[i + (size_t)ny * c1] * a.X[i + (size_t)ny * c2]; });
      if (lane == 0) P.XtX[p] = s;
    } else {
      const int q = p - nc * nc, h1 = q % nf, h2 = q / nf;
      const double s = wave_sum<8>(ns, [&](int j) { return lam[h1 + (size_t)K * j] * a.iSigma[j] * lam[h2 + (size_t)K * j]; });
      if (lane == 0) P.LDL[q] = s;
    }
  }
}
// X'S, iQ Tr; V = iV^-1 and (np = ny) W0 by single threads; (np < ny) the per-unit blocks
__global__ __launch_bounds__(256) void ge_b_xts_kernel(GEArgs a) {
  GE_GRID_IDX
  {  // X'S and iQ Tr, one wave per output (iQ symmetric: read by columns)
    const int lane = threadIdx.x & 63, w0 = g0 >> 6, ws = gs >> 6;
    const int ny = a.ny, ns = a.ns, nc = a.nc, N = P.N;
    for (int p = w0; p < N + ns * a.nt; p += ws) {
      if (p < N) {
        const int c = p % nc, j = p / nc;
        const double s = wave_sum<8>(ny, [&](int i) { return a.X[i + (size_t)ny * c] * P.S[i + (size_t)ny * j]; });
        if (lane == 0) P.XtS[p] = s;
      } else {
        const int q0 = p - N, j = q0 % ns, q = q0 / ns;
        const double s = wave_sum<8>(ns, [&](int j2) { return P.iQm[j2 + (size_t)ns * j] * a.Tr[j2 + (size_t)ns * q]; });
        if (lane == 0) P.iQTr[q0] = s;
      }
    }
  }
  const int nc = a.nc;
  if (g0 == 0) {  // V = chol2inv(chol(iV)) = L^-T L^-1, L^-1 in the (not yet used) T block
    if (!t_chol_inv(P.Wv, P.T, nc)) a.fail[0] = 1;
    for (int c1 = 0; c1 < nc; ++c1)
      for (int c2 = 0; c2 < nc; ++c2) {
        double s = 0.0;
        for (int k = 0; k < nc; ++k) s += P.T[k + nc * c1] * P.T[k + nc * c2];
        P.V[c1 + nc * c2] = s;
      }
  }
  if (P.obs) {
    if (g0 == 64 && !ge_w0(a, P)) a.fail[0] = 1;
  } else if (!ge_seg_units(a, P, g0, gs)) {
    a.fail[0] = 1;
  }
}
__global__ __launch_bounds__(256) void ge_b_a_kernel(GEArgs a) {
  GE_GRID_IDX
  ge_seg_a(a, P, g0, gs);
  if (P.obs) ge_seg_tmp1(a, P, g0, gs);
}
template <int NFC>
__global__ __launch_bounds__(256) void ge_b_m_kernel(GEArgs a) {
  GE_GRID_IDX
  if (!P.obs) {
    ge_seg_m_units(a, P, g0, gs);
    ge_seg_mb10(a, P, g0, gs);
    return;
  }
  // np = ny: M += kron(tmp1, X'X) elementwise; mb20, mb10 and v one wave per entry   (:58-62)
  const int ns = a.ns, nc = a.nc, nf = a.nf, N = P.N;
  for (size_t p = g0; p < (size_t)N * N; p += gs) {
    const int r1 = (int)(p % N), r2 = (int)(p / N);
    P.M[p] += P.tmp1[(r1 / nc) + (size_t)ns * (r2 / nc)] * P.XtX[(r1 % nc) + nc * (r2 % nc)];
  }
  const int lane = threadIdx.x & 63, w0 = g0 >> 6, ws = gs >> 6;
  for (int p = w0; p < N; p += ws) {
    const int c = p % nc, j = p / nc;
    double x1[NFC];
    for (int h1 = 0; h1 < nf; ++h1)
      x1[h1] = wave_sum<8>(ns, [&](int j2) { return P.XtS[c + nc * j2] * P.LamiD[h1 + nf * j2]; });
    if (lane == 0) {
      double s = 0.0;
      for (int h2 = 0; h2 < nf; ++h2) {
        double u = 0.0;
        for (int h1 = 0; h1 < nf; ++h1) u = fma(x1[h1], P.iW0[h1 + nf * h2], u);
        s = fma(u, P.LamiD[h2 + nf * j], s);
      }
      P.mb20[p] = s;
      P.mb10[p] = P.XtS[p] * a.iSigma[j];
      P.v[p] = P.mb10[p] - s;
    }
  }
}
// with v = M^-1 (mb10 - mb20): wv = mb10 - mb20 - T1 v (mb30, :63-64), xi ~ N(0, I); T1 is
// symmetric (kron(tmp1, X'X) for np = ny, T otherwise), read by columns
__global__ __launch_bounds__(256) void ge_b_wv_kernel(GEArgs a) {
  GE_WAVE_IDX
  const int ns = a.ns, nc = a.nc, N = P.N;
  const uint32_t str = LEVEL_STRIDE * (uint32_t)a.r, it = SWEEP_ITER(a);
  for (int p = w0; p < N; p += ws) {
    const int c = p % nc, j = p / nc;
    double s;
    if (P.obs)
      s = wave_sum<8>(ns, [&](int j2) {
        double u = 0.0;
        for (int c2 = 0; c2 < nc; ++c2) u = fma(P.XtX[c + nc * c2], P.v[c2 + nc * j2], u);
        return P.tmp1[j2 + (size_t)ns * j] * u;
      });
    else
      s = wave_sum<8>(N, [&](int p2) { return P.T[p2 + (size_t)N * p] * P.v[p2]; });
    if (lane == 0) {
      P.wv[p] = P.mb10[p] - P.mb20[p] - s;
      P.xi[p] = a.noise_zero ? 0.0 : normal(a.key, (uint32_t)p, 0, S_GE_BETA + str, it);
    }
  }
}
// mb = A wv   (:65); A symmetric, read by columns
__global__ __launch_bounds__(256) void ge_b_mb_kernel(GEArgs a) {
  GE_WAVE_IDX
  const int N = P.N;
  for (int p = w0; p < N; p += ws) {
    const double s = wave_sum<8>(N, [&](int p2) { return P.A[p2 + (size_t)N * p] * P.wv[p2]; });
    if (lane == 0) P.mb[p] = s;
  }
}
// Beta = mb + RM^-1 xi; Gamma | Beta (:66-71): one 1024-thread workgroup, the Pg entries and
// the right-hand side one wave each
__global__ __launch_bounds__(1024) void ge_b_gamma_kernel(GEArgs a) {
  __shared__ int flag;
  const GEPtrs P = ge_ptrs(a);
  const int t = threadIdx.x, nthr = blockDim.x, lane = t & 63, w = t >> 6, nw = nthr >> 6;
  const int ns = a.ns, nc = a.nc, G = P.G, N = P.N;
  const uint32_t str = LEVEL_STRIDE * (uint32_t)a.r, it = SWEEP_ITER(a);
  for (int p = t; p < N; p += nthr) P.Beta[p] = P.mb[p] + P.xi[p];
  __syncthreads();
  for (int p = w; p < G * G + G; p += nw) {
    if (p < G * G) {
      const int r1 = p % G, r2 = p / G;
      const int c1 = r1 % nc, t1 = r1 / nc, c2 = r2 % nc, t2 = r2 / nc;
      const double tq = wave_sum<8>(ns, [&](int j) { return a.Tr[j + (size_t)ns * t1] * P.iQTr[j + (size_t)ns * t2]; });
      if (lane == 0) P.Pg[p] = a.iUGamma[p] + tq * a.iV[c1 + nc * c2];
    } else {
      const int q0 = p - G * G, c = q0 % nc, q = q0 / nc;
      const double sv = wave_sum<8>(ns, [&](int j) {
        double ib = 0.0;
        for (int c2 = 0; c2 < nc; ++c2) ib = fma(a.iV[c + nc * c2], P.Beta[c2 + nc * j], ib);
        return ib * P.iQTr[j + (size_t)ns * q];
      });
      if (lane == 0) P.rg[q0] = sv;
    }
  }
  __syncthreads();
  if (G <= 16) {  // the G x G solve in one wave's registers (wave_la.h) instead of wg_chol's
    __shared__ __attribute__((aligned(16))) double tile[WV_TILE];  // per-column barriers
    if (w == 0) {
      double x[16], y[16], dinv;
      wv_load<16>(P.Pg, G, G, x);
      double r = lane < G ? P.rg[lane] : 0.0;
      const bool ok = wv_chol<16>(x, dinv);
      wv_forward<16>(x, dinv, r);
      if (lane < G && !a.noise_zero) r += normal(a.key, (uint32_t)lane, 0, S_GE_GAMMA + str, it);
      wv_transpose<16, true>(x, y, tile);
      wv_backward_t<16>(y, dinv, r);
      if (lane < G) a.Gamma[lane] = r;
      if (!ok && lane == 0) a.fail[0] = 1;
    }
    return;
  }
  if (!wg_chol(P.Pg, G, G, &flag) && t == 0) a.fail[0] = 1;
  wg_forward(P.Pg, G, G, P.rg);
  for (int p = t; p < G; p += nthr)
    if (!a.noise_zero) P.rg[p] += normal(a.key, (uint32_t)p, 0, S_GE_GAMMA + str, it);
  __syncthreads();
  wg_backward_t(P.Pg, G, G, P.rg);
  for (int p = t; p < G; p += nthr) a.Gamma[p] = P.rg[p];
}
// Eta | Beta, S (:71-74 / :136-146): one wave per row (np = ny) or unit, lanes over species
template <int NFC>
__global__ __launch_bounds__(256) void ge_b_eta_kernel(GEArgs a) {
  GE_WAVE_IDX
  const int ny = a.ny, ns = a.ns, nc = a.nc, nf = a.nf, np = a.np;
  const uint32_t str = LEVEL_STRIDE * (uint32_t)a.r, it = SWEEP_ITER(a);
  const int nrow = P.obs ? ny : np;
  for (int i = w0; i < nrow; i += ws) {
    double tv[NFC];
    for (int h = 0; h < nf; ++h) tv[h] = 0.0;
    for (int j = lane; j < ns; j += 64) {
      double s1;
      if (P.obs) {
        s1 = P.S[i + (size_t)ny * j];
        for (int c = 0; c < nc; ++c) s1 -= a.X[i + (size_t)ny * c] * P.Beta[c + nc * j];
      } else {
        s1 = P.PtS[i + (size_t)np * j];
        for (int c = 0; c < nc; ++c) s1 -= P.PtX[i + (size_t)np * c] * P.Beta[c + nc * j];
      }
      for (int h = 0; h < nf; ++h) tv[h] = fma(s1, P.LamiD[h + nf * j], tv[h]);
    }
    for (int h = 0; h < nf; ++h)
      for (int o = 32; o > 0; o >>= 1) tv[h] += __shfl_xor(tv[h], o);
    for (int h = lane; h < nf; h += 64) {  // (nf > 64: two factors a lane)
      double me = 0.0, nz = 0.0;
      if (P.obs) {
        for (int h2 = 0; h2 < nf; ++h2) me = fma(tv[h2], P.iW0[h2 + nf * h], me);
        if (!a.noise_zero)
          for (int h2 = h; h2 < nf; ++h2)  // (RW0^-1 xi)_h = sum_h2 L0i[h2, h] xi_h2
            nz = fma(P.L0i[h2 + nf * h], normal(a.key, (uint32_t)i, (uint32_t)h2, S_GE_ETA + str, it), nz);
        a.Eta[a.lev_pi[a.r][i] + (size_t)np * h] = me + nz;
      } else {
        const double* iW = P.iWp + (size_t)i * nf * nf;
        const double* Li = P.Lip + (size_t)i * nf * nf;
        for (int h2 = 0; h2 < nf; ++h2) me = fma(iW[h + nf * h2], tv[h2], me);
        if (!a.noise_zero)
          for (int h2 = h; h2 < nf; ++h2)  // (LiW_p xi)_h = sum_h2 Li[h2, h] xi_h2
            nz = fma(Li[h2 + nf * h], normal(a.key, (uint32_t)i, (uint32_t)h2, S_GE_ETA + str, it), nz);
        a.Eta[i + (size_t)np * h] = me + nz;
      }
    }
  }
}
#undef GE_WAVE_IDX
#undef GE_GRID_IDX

static int ge_blocks(size_t elems) { return (int)std::max<size_t>(1, std::min<size_t>(4096, (elems + 255) / 256)); }

// workspace of the blocked path past ge_layout: the two dense_potrf_lower workspaces
static size_t ge_blocked_extra(int N) { return N > GE_WG_MAX ? 2 * dense_ws_doubles(N) + 16 : 0; }

static void launch_gamma_eta_blocked(State& s, const GEArgs& a, hipStream_t st) {
  const bool obs = a.np == a.ny;
  const int N = a.nc * a.ns;
  const GELayout o = ge_layout(a.ny, a.ns, a.nc, a.nt, a.nf, obs ? 0 : a.np);
  double* w = a.work;
  double *L = w + o.L, *M = w + o.M, *T = w + o.T;
  double *v = w + o.vec + 2 * (size_t)N, *xi = w + o.vec + 5 * (size_t)N;
  double* ws1 = w + o.tot;
  double* ws2 = ws1 + dense_ws_doubles(N);
  const size_t NN = (size_t)N * N;
  const size_t big = std::max<size_t>((size_t)a.ny * a.ns, (size_t)a.ns * a.ns);
  ge_b_prep_kernel<<<ge_blocks(big), 256, 0, st>>>(a);
  if (a.phU) {  // Q = U diag(w) U^T, iQ = U diag(1/w) U^T on the matrix cores
    const GEPtrs hp = ge_ptrs(a);
    dense_gram_diag(st, a.phU, a.ns, a.ns, a.phWinv, a.rho, true, hp.Qm, a.ns);
    dense_gram_diag(st, a.phU, a.ns, a.ns, a.phWinv, a.rho, false, hp.iQm, a.ns);
  }
  ge_b_xts_kernel<<<ge_blocks(std::max<size_t>(64 * ((size_t)N + a.ns * a.nt), obs ? 128 : a.np)), 256, 0, st>>>(a);
  ge_b_a_kernel<<<ge_blocks(NN), 256, 0, st>>>(a);
  // iA = chol2inv(chol(A)) = L^-T L^-1   (:33)
  dense_potrf_lower(st, L, N, N, ws1, a.fail, 0, s.trsv_sync);
  dense_trtri_lower(st, L, N, N, T, N, ws1, true);
  dense_lauum_lower(st, T, N, N, M, N);
  if (a.nf <= GE_NF_SMALL)
    ge_b_m_kernel<GE_NF_SMALL><<<ge_blocks(NN), 256, 0, st>>>(a);
  else if (a.nf <= GE_NF_LARGE)
    ge_b_m_kernel<GE_NF_LARGE><<<ge_blocks(NN), 256, 0, st>>>(a);
  else
    ge_b_m_kernel<GE_NF_XL><<<ge_blocks(NN), 256, 0, st>>>(a);
  // RM = chol(M); v = M^-1 (mb10 - mb20)
  dense_potrf_lower(st, M, N, N, ws2, a.fail, 0, s.trsv_sync);
  dense_trsv_lower(st, M, N, N, v, 0, ws2, 0, s.trsv_sync);
  dense_trsv_lower(st, M, N, N, v, 1, ws2, 0, s.trsv_sync);
  ge_b_wv_kernel<<<ge_blocks(64 * (size_t)N), 256, 0, st>>>(a);  // one wave per output
  ge_b_mb_kernel<<<ge_blocks(64 * (size_t)N), 256, 0, st>>>(a);
  dense_trsv_lower(st, M, N, N, xi, 1, ws2, 0, s.trsv_sync);  // backsolve(RM, rnorm(nc ns))  (:66)
  ge_b_gamma_kernel<<<1, 1024, 0, st>>>(a);
  const int eta_grid = ge_blocks(64 * (size_t)(obs ? a.ny : a.np));
  if (a.nf <= GE_NF_SMALL)
    ge_b_eta_kernel<GE_NF_SMALL><<<eta_grid, 256, 0, st>>>(a);
  else if (a.nf <= GE_NF_LARGE)
    ge_b_eta_kernel<GE_NF_LARGE><<<eta_grid, 256, 0, st>>>(a);
  else
    ge_b_eta_kernel<GE_NF_XL><<<eta_grid, 256, 0, st>>>(a);
  HIP_OK(hipGetLastError());
}

// ---------------------------------------------------------------------------------------
// Spatial 'Full' level (R/updateGammaEta.R:139-198): (vec Gamma, vec Eta_r) drawn jointly
// with Beta integrated out, from the precision
//   iG = bdiag(iU, iK) + Gm'Gm - tmp'tmp,  Gm = [kron(iD^.5 Tr, X), kron(iD^.5 Lam', P)],
//   tmp = L_H^-1 C,  H = kron(iQ, iV) + kron(iD, X'X) = L_H L_H',
//   C = [kron(iD Tr, X'X), t(kron(Lam iD, P'X))],  iK = bdiag(iWg[,,alpha_h]),
// and mean iG^-1 (c0 - tmp' L_H^-1 vec(X'S iD)), c0 = [vec(X'S iD Tr); vec(P'S iD Lam')]:
// the natural form of R's mg / me chain (the oracle pins the two equal,
// tests/test_oracle_spatial.py).  Draw: m + chol(iG)^-1 xi, xi = normal(p, 0, S_GE_GAMMA).
// One workgroup: every step is a dependent dense factorization of (nc ns)^2 or
// (nc nt + np nf)^2, small at the configs that run this updater (TD's plot level).
struct GESLayout {
  size_t S, XtX, XtS, LamiD, LDL, iQm, PtX, PtS, cnt, TdT, TdL, H, C, y, iG, b, tot;
};

__host__ __device__ inline GESLayout ges_layout(int ny, int ns, int nc, int nt, int nf, int np) {
  GESLayout o{};
  const size_t N = (size_t)nc * ns, D2 = (size_t)nc * nt + (size_t)np * nf;
  size_t p = 0;
  auto take = [&](size_t n) {
    const size_t at = p;
    p += (n + 7) & ~(size_t)7;
    return at;
  };
  o.S = take((size_t)ny * ns);
  o.XtX = take((size_t)nc * nc);
  o.XtS = take(N);
  o.LamiD = take((size_t)nf * ns);
  o.LDL = take((size_t)nf * nf);
  o.iQm = take((size_t)ns * ns);
  o.PtX = take((size_t)np * nc);
  o.PtS = take((size_t)np * ns);
  o.cnt = take(np);
  o.TdT = take((size_t)nt * nt);
  o.TdL = take((size_t)nt * nf);
  o.H = take(N * N);
  o.C = take(N * D2);
  o.y = take(N);
  o.iG = take(D2 * D2);
  o.b = take(D2);
  o.tot = p;
  return o;
}

struct GESArgs {
  GEArgs g;
  const double* iWg;      // np x np x nalpha
  const double* AlphaD;   // nf, 1-based grid index
};

// The stages below are written over a flat index range [t0, n) with stride nthr, so the
// same code runs inside one workgroup (gamma_eta_spatial_kernel: threads of the block,
// __syncthreads between stages) and over a grid (the blocked path above GES_WG_MAX: one
// launch per stage, the two factorizations on dense.hip's MFMA Cholesky).
struct GESView {
  int ny, ns, nc, nt, nf, np, K, N, G, D2;
  double *S, *XtX, *XtS, *LamiD, *LDL, *iQm, *PtX, *PtS, *cnt, *TdT, *TdL, *H, *C, *y, *iG, *b;
  const double *lam, *id;
  const int* pi;
};

__device__ inline GESView ges_view(const GESArgs& sa) {
  const GEArgs& a = sa.g;
  GESView v;
  v.ny = a.ny, v.ns = a.ns, v.nc = a.nc, v.nt = a.nt, v.nf = a.nf, v.np = a.np, v.K = a.K;
  v.N = v.nc * v.ns, v.G = v.nc * v.nt, v.D2 = v.G + v.np * v.nf;
  const GESLayout o = ges_layout(v.ny, v.ns, v.nc, v.nt, v.nf, v.np);
  double* w = a.work;
  v.S = w + o.S, v.XtX = w + o.XtX, v.XtS = w + o.XtS, v.LamiD = w + o.LamiD, v.LDL = w + o.LDL;
  v.iQm = w + o.iQm, v.PtX = w + o.PtX, v.PtS = w + o.PtS, v.cnt = w + o.cnt, v.TdT = w + o.TdT;
  v.TdL = w + o.TdL, v.H = w + o.H, v.C = w + o.C, v.y = w + o.y, v.iG = w + o.iG, v.b = w + o.b;
  v.lam = a.BL + a.loff;  // Lambda_r[h, j] = lam[h + K j]
  v.id = a.iSigma;
  v.pi = a.lev_pi[a.r];
  return v;
}

// stage 1: S (:37-42), X'X, Lam iD, Lam iD Lam', iQ, P'X, unit counts, Tr'iD Tr, Tr'iD Lam'
__device__ void ges_stage1(const GESArgs& sa, const GESView& v, size_t t, size_t nthr) {
  const GEArgs& a = sa.g;
  const int ny = v.ny, ns = v.ns, nc = v.nc, nt = v.nt, nf = v.nf, np = v.np, K = v.K;
  const double *lam = v.lam, *id = v.id;
  for (size_t p = t; p < (size_t)ny * ns; p += nthr) {
    const int i = (int)(p % ny), j = (int)(p / ny);
    double sv = a.Z[p];
    for (int q = 0; q < a.nr; ++q) {
      if (q == a.r) continue;
      const double* eq = a.lev_eta[q];
      const int u = a.lev_pi[q][i], npq = a.lev_np[q];
      const double* lq = a.BL + a.lev_loff[q] + (size_t)K * j;
      for (int h = 0; h < a.lev_nf[q]; ++h) sv -= eq[u + (size_t)npq * h] * lq[h];
    }
    v.S[p] = sv;
  }
  for (size_t p = t; p < (size_t)nc * nc; p += nthr) {
    const int c1 = (int)(p % nc), c2 = (int)(p / nc);
    double s = 0.0;
    for (int i = 0; i < ny; ++i) s = fma(a.X[i + (size_t)ny * c1], a.X[i + (size_t)ny * c2], s);
    v.XtX[p] = s;
  }
  for (size_t p = t; p < (size_t)nf * ns; p += nthr) {
    const int h = (int)(p % nf), j = (int)(p / nf);
    v.LamiD[p] = lam[h + (size_t)K * j] * id[j];
  }
  for (size_t p = t; p < (size_t)nf * nf; p += nthr) {
    const int h1 = (int)(p % nf), h2 = (int)(p / nf);
    double s = 0.0;
    for (int j = 0; j < ns; ++j) s = fma(lam[h1 + (size_t)K * j] * id[j], lam[h2 + (size_t)K * j], s);
    v.LDL[p] = s;
  }
  if (a.phU) {
    const double* wq = a.phWinv + (size_t)ns * ((int)(*a.rho) - 1);
    for (size_t p = t; p < (size_t)ns * ns; p += nthr) {
      const int j1 = (int)(p % ns), j2 = (int)(p / ns);
      double si = 0.0;
      for (int i = 0; i < ns; ++i) si = fma(a.phU[j1 + (size_t)ns * i] * a.phU[j2 + (size_t)ns * i], wq[i], si);
      v.iQm[p] = si;
    }
  } else {
    for (size_t p = t; p < (size_t)ns * ns; p += nthr) v.iQm[p] = (p % ns == p / ns) ? 1.0 : 0.0;
  }
  // P'X and the unit counts from the level's unit -> rows lists
  for (size_t p = t; p < (size_t)np * (nc + 1); p += nthr) {
    const int u = (int)(p % np), c = (int)(p / np);
    double s = 0.0;
    for (int q = a.unit_ptr[u]; q < a.unit_ptr[u + 1]; ++q) s += (c < nc) ? a.X[a.unit_rows[q] + (size_t)ny * c] : 1.0;
    if (c < nc) v.PtX[p] = s; else v.cnt[u] = s;
  }
  for (size_t p = t; p < (size_t)nt * (nt + nf); p += nthr) {
    const int t1 = (int)(p % nt), k = (int)(p / nt);
    double s = 0.0;
    for (int j = 0; j < ns; ++j)
      s = fma(id[j] * a.Tr[j + (size_t)ns * t1], k < nt ? a.Tr[j + (size_t)ns * k] : lam[(k - nt) + (size_t)K * j], s);
    if (k < nt) v.TdT[t1 + nt * k] = s; else v.TdL[t1 + nt * (k - nt)] = s;
  }
}

// stage 2: X'S, P'S, H = kron(iQ, iV) + kron(iD, X'X)  (:183)
__device__ void ges_stage2(const GESArgs& sa, const GESView& v, size_t t, size_t nthr) {
  const GEArgs& a = sa.g;
  const int ny = v.ny, ns = v.ns, nc = v.nc, np = v.np, N = v.N;
  for (size_t p = t; p < (size_t)N; p += nthr) {
    const int c = (int)(p % nc), j = (int)(p / nc);
    double s = 0.0;
    for (int i = 0; i < ny; ++i) s = fma(a.X[i + (size_t)ny * c], v.S[i + (size_t)ny * j], s);
    v.XtS[p] = s;
  }
  for (size_t p = t; p < (size_t)np * ns; p += nthr) {
    const int u = (int)(p % np), j = (int)(p / np);
    double s = 0.0;
    for (int q = a.unit_ptr[u]; q < a.unit_ptr[u + 1]; ++q) s += v.S[a.unit_rows[q] + (size_t)ny * j];
    v.PtS[p] = s;
  }
  for (size_t p = t; p < (size_t)N * N; p += nthr) {
    const int r1 = (int)(p % N), r2 = (int)(p / N);
    const int c1 = r1 % nc, j1 = r1 / nc, c2 = r2 % nc, j2 = r2 / nc;
    v.H[p] = v.iQm[j1 + (size_t)ns * j2] * a.iV[c1 + nc * c2] + (j1 == j2 ? v.id[j1] * v.XtX[c1 + nc * c2] : 0.0);
  }
}

// stage 3: C = [kron(iD Tr, X'X), t(kron(Lam iD, P'X))] and y = vec(X'S iD)
__device__ void ges_stage3(const GESArgs& sa, const GESView& v, size_t t, size_t nthr) {
  const GEArgs& a = sa.g;
  const int ns = v.ns, nc = v.nc, nf = v.nf, np = v.np, N = v.N, G = v.G;
  for (size_t p = t; p < (size_t)N * v.D2; p += nthr) {
    const int r1 = (int)(p % N), col = (int)(p / N);
    const int c1 = r1 % nc, j = r1 / nc;
    double val;
    if (col < G) {
      const int c2 = col % nc, q = col / nc;
      val = v.id[j] * a.Tr[j + (size_t)ns * q] * v.XtX[c1 + nc * c2];
    } else {
      const int e = col - G, u = e % np, h = e / np;
      val = v.LamiD[h + nf * j] * v.PtX[u + (size_t)np * c1];
    }
    v.C[p] = val;
  }
  for (size_t p = t; p < (size_t)N; p += nthr) v.y[p] = v.XtS[p] * v.id[p / nc];
}

// tmp = L_H^-1 [C | y], one column per index (L_H lower, in H)
__device__ void ges_forward_cols(const GESView& v, size_t t, size_t nthr) {
  const int N = v.N;
  for (size_t col = t; col < (size_t)v.D2 + 1; col += nthr) {
    double* x = col < (size_t)v.D2 ? v.C + (size_t)N * col : v.y;
    for (int i = 0; i < N; ++i) {
      double s = x[i];
      for (int k = 0; k < i; ++k) s -= v.H[i + (size_t)N * k] * x[k];
      x[i] = s / v.H[i + (size_t)N * i];
    }
  }
}

// stage 4: iG = bdiag(iU, iK) + Gm'Gm - tmp'tmp (:184-191), b = c0 - tmp'y; lower_only:
// entries p1 >= p2 of iG (all the blocked Cholesky reads)
__device__ void ges_stage4(const GESArgs& sa, const GESView& v, size_t t, size_t nthr, bool lower_only) {
  const GEArgs& a = sa.g;
  const int ns = v.ns, nc = v.nc, nt = v.nt, nf = v.nf, np = v.np, N = v.N, G = v.G, D2 = v.D2;
  for (size_t p = t; p < (size_t)D2 * D2; p += nthr) {
    const int p1 = (int)(p % D2), p2 = (int)(p / D2);
    if (lower_only && p1 < p2) continue;
    double val;
    if (p1 < G && p2 < G) {
      const int c1 = p1 % nc, t1 = p1 / nc, c2 = p2 % nc, t2 = p2 / nc;
      val = v.TdT[t1 + nt * t2] * v.XtX[c1 + nc * c2] + a.iUGamma[p1 + (size_t)G * p2];
    } else if (p1 >= G && p2 >= G) {
      const int e1 = p1 - G, e2 = p2 - G, u1 = e1 % np, h1 = e1 / np, u2 = e2 % np, h2 = e2 / np;
      val = (u1 == u2) ? v.cnt[u1] * v.LDL[h1 + nf * h2] : 0.0;
      if (h1 == h2) {
        const int g = (int)sa.AlphaD[h1] - 1;
        val += sa.iWg[(size_t)np * np * g + u1 + (size_t)np * u2];
      }
    } else {
      const int pg = p1 < G ? p1 : p2, pe = (p1 < G ? p2 : p1) - G;
      const int c = pg % nc, q = pg / nc, u = pe % np, h = pe / np;
      val = v.TdL[q + nt * h] * v.PtX[u + (size_t)np * c];
    }
    const double* c1 = v.C + (size_t)N * p1;
    const double* c2 = v.C + (size_t)N * p2;
    double s = 0.0;
    for (int k = 0; k < N; ++k) s = fma(c1[k], c2[k], s);
    v.iG[p] = val - s;
  }
  for (size_t p = t; p < (size_t)D2; p += nthr) {
    double c0 = 0.0;
    if ((int)p < G) {
      const int c = (int)p % nc, q = (int)p / nc;
      for (int j = 0; j < ns; ++j) c0 = fma(v.XtS[c + nc * j] * v.id[j], a.Tr[j + (size_t)ns * q], c0);
    } else {
      const int e = (int)p - G, u = e % np, h = e / np;
      for (int j = 0; j < ns; ++j) c0 = fma(v.PtS[u + (size_t)np * j], v.LamiD[h + nf * j], c0);
    }
    const double* cp = v.C + (size_t)N * p;
    double s = 0.0;
    for (int k = 0; k < N; ++k) s = fma(cp[k], v.y[k], s);
    v.b[p] = c0 - s;
  }
}

__device__ inline void ges_add_noise(const GESArgs& sa, const GESView& v, size_t t, size_t nthr) {
  const GEArgs& a = sa.g;
  const uint32_t it = SWEEP_ITER(a);
  const uint32_t str = LEVEL_STRIDE * (uint32_t)a.r;
  for (size_t p = t; p < (size_t)v.D2; p += nthr)
    if (!a.noise_zero) v.b[p] += normal(a.key, (uint32_t)p, 0, S_GE_GAMMA + str, it);
}

__device__ inline void ges_store(const GESArgs& sa, const GESView& v, size_t t, size_t nthr) {
  const GEArgs& a = sa.g;
  for (size_t p = t; p < (size_t)v.G; p += nthr) a.Gamma[p] = v.b[p];
  for (size_t p = t; p < (size_t)v.np * v.nf; p += nthr) a.Eta[p] = v.b[v.G + p];
}

__global__ __launch_bounds__(1024) void gamma_eta_spatial_kernel(GESArgs sa) {
  __shared__ int flag;
  const GESView v = ges_view(sa);
  const size_t t = threadIdx.x, nthr = blockDim.x;
  ges_stage1(sa, v, t, nthr);
  __syncthreads();
  ges_stage2(sa, v, t, nthr);
  __syncthreads();
  ges_stage3(sa, v, t, nthr);
  __syncthreads();
  if (!wg_chol(v.H, v.N, v.N, &flag) && t == 0) sa.g.fail[0] = 1;
  ges_forward_cols(v, t, nthr);
  __syncthreads();
  ges_stage4(sa, v, t, nthr, false);
  __syncthreads();
  // stage 5: m + chol(iG)^-1 xi = L^-T (L^-1 b + xi)   (:193-194)
  if (!wg_chol(v.iG, v.D2, v.D2, &flag) && t == 0) sa.g.fail[0] = 1;
  wg_forward(v.iG, v.D2, v.D2, v.b);
  ges_add_noise(sa, v, t, nthr);
  __syncthreads();
  wg_backward_t(v.iG, v.D2, v.D2, v.b);
  ges_store(sa, v, t, nthr);
}

// blocked path: each stage one grid launch
template <int STAGE>
__global__ __launch_bounds__(256) void ges_grid_kernel(GESArgs sa) {
  const GESView v = ges_view(sa);
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x, nthr = (size_t)gridDim.x * blockDim.x;
  if (STAGE == 1) ges_stage1(sa, v, t, nthr);
  if (STAGE == 2) ges_stage2(sa, v, t, nthr);
  if (STAGE == 3) ges_stage3(sa, v, t, nthr);
  if (STAGE == 4) ges_forward_cols(v, t, nthr);
  if (STAGE == 5) ges_stage4(sa, v, t, nthr, true);
  if (STAGE == 6) ges_add_noise(sa, v, t, nthr);
  if (STAGE == 7) ges_store(sa, v, t, nthr);
}

// one workgroup up to this joint size; above it the blocked path
constexpr int GES_WG_MAX = 1024;

static bool ges_blocked(int N, int D2) {
  const char* env = getenv("HMSC_GES_BLOCKED");  // 1 / 0: force the blocked / one-workgroup path
  const int force = env ? atoi(env) : -1;
  if (force >= 0) return force > 0;
  return D2 > GES_WG_MAX || N > GES_WG_MAX;
}

// the blocked path's workspace past ges_layout: dense_potrf_lower workspaces for H and iG
static size_t ges_blocked_extra(int N, int D2) { return dense_ws_doubles(N) + dense_ws_doubles(D2) + 16; }

static void launch_gamma_eta_spatial(State& s, const GESArgs& sa, hipStream_t st) {
  const GEArgs& a = sa.g;
  const int N = a.nc * a.ns, D2 = a.nc * a.nt + a.np * a.nf;
  if (!ges_blocked(N, D2)) {
    gamma_eta_spatial_kernel<<<1, 1024, 0, st>>>(sa);
    HIP_OK(hipGetLastError());
    return;
  }
  const GESLayout o = ges_layout(a.ny, a.ns, a.nc, a.nt, a.nf, a.np);
  double* w = a.work;
  double* ws1 = w + o.tot;
  double* ws2 = ws1 + dense_ws_doubles(N);
  auto grid = [](size_t n) { return (int)std::max<size_t>(1, std::min<size_t>(8192, (n + 255) / 256)); };
  const size_t big1 = std::max({(size_t)a.ny * a.ns, (size_t)a.np * (a.nc + 1), (size_t)a.ns * a.ns});
  ges_grid_kernel<1><<<grid(big1), 256, 0, st>>>(sa);
  ges_grid_kernel<2><<<grid(std::max((size_t)N * N, (size_t)a.np * a.ns)), 256, 0, st>>>(sa);
  ges_grid_kernel<3><<<grid((size_t)N * D2), 256, 0, st>>>(sa);
  dense_potrf_lower(st, w + o.H, N, N, ws1, a.fail, 0, s.trsv_sync);
  ges_grid_kernel<4><<<grid((size_t)D2 + 1), 256, 0, st>>>(sa);
  ges_grid_kernel<5><<<grid((size_t)D2 * D2), 256, 0, st>>>(sa);
  dense_potrf_lower(st, w + o.iG, D2, D2, ws2, a.fail, 0, s.trsv_sync);
  dense_trsv_lower(st, w + o.iG, D2, D2, w + o.b, 0, ws2, 0, s.trsv_sync);
  ges_grid_kernel<6><<<grid(D2), 256, 0, st>>>(sa);
  dense_trsv_lower(st, w + o.iG, D2, D2, w + o.b, 1, ws2, 0, s.trsv_sync);
  ges_grid_kernel<7><<<grid(D2), 256, 0, st>>>(sa);
  HIP_OK(hipGetLastError());
}

// sized by the factors each level has now: a level's nf grows only in updateNf's adaptive
// sweeps (eager, never inside a graph capture), and launch_gamma_eta grows the workspace then
size_t gamma_eta_work_doubles(const State& s) {
  size_t m = 0;
  for (int r = 0; r < s.nr; ++r) {
    const int nf = std::max(1, s.lev[r].nf);
    const int np = s.lev[r].np == s.ny ? 0 : s.lev[r].np;
    m = std::max(m, ge_layout(s.ny, s.ns, s.nc, s.nt, nf, np).tot + ge_blocked_extra(s.nc * s.ns));
    if (s.lev[r].spatial) {
      const int N = s.nc * s.ns, D2 = s.nc * s.nt + s.lev[r].np * nf;
      m = std::max(m, ges_layout(s.ny, s.ns, s.nc, s.nt, nf, s.lev[r].np).tot +
                          (ges_blocked(N, D2) ? ges_blocked_extra(N, D2) : 0));
    }
  }
  return m + 64;
}

void launch_gamma_eta(State& s, uint32_t iter) {
  HMSC_REQUIRE(!s.sharded, "updateGammaEta: species-sharded chains are not supported (dense (nc ns)^2 system)");
  HMSC_REQUIRE(s.geWork != nullptr, "updateGammaEta: workspace not allocated");
  for (int r = 0; r < s.nr; ++r)
    HMSC_REQUIRE(!s.lev[r].spatial || (size_t)s.nc * s.nt + (size_t)s.lev[r].np * s.lev[r].nf <= 32768,
                 "updateGammaEta, spatial level: nc nt + np nf must be <= 32768 (dense joint system, 8.6 GB)");
  {
    const size_t need = gamma_eta_work_doubles(s);
    if (need > s.geWork_doubles) {  // nf grew (updateNf): a larger workspace, outside any capture
      HMSC_REQUIRE(!s.capturing, "internal: updateGammaEta workspace growth inside a graph capture");
      s.geWork = device_realloc_doubles(s, s.geWork, need);
      s.geWork_doubles = need;
    }
  }
  ProfScope ps(s, PROF_GE);
  for (int r = 0; r < s.nr; ++r) {
    GEArgs a{};
    a.ny = s.ny;
    a.ns = s.ns;
    a.nc = s.nc;
    a.nt = s.nt;
    a.K = s.K;
    a.r = r;
    a.nr = s.nr;
    a.nf = s.lev[r].nf;
    a.np = s.lev[r].np;
    a.loff = s.loff(r);
    HMSC_REQUIRE(a.nf <= GE_NF_XL, "updateGammaEta: a level's nf must be <= 128 in this build");
    for (int q = 0; q < s.nr; ++q) {
      a.lev_np[q] = s.lev[q].np;
      a.lev_nf[q] = s.lev[q].nf;
      a.lev_loff[q] = s.loff(q);
      a.lev_eta[q] = s.lev[q].Eta;
      a.lev_pi[q] = s.lev[q].Pi;
    }
    a.Eta = s.lev[r].Eta;
    a.unit_ptr = s.lev[r].unit_ptr;
    a.unit_rows = s.lev[r].unit_rows;
    a.Z = s.Z;
    a.X = s.X;
    a.Tr = s.Tr;
    a.BL = s.BL;
    a.iSigma = s.iSigma;
    a.UGamma = s.UGamma;
    a.iUGamma = s.iUGamma;
    a.iV = s.iV;
    a.Gamma = s.Gamma;
    a.phU = s.phylo ? s.phU : nullptr;
    a.phWinv = s.phWinv;
    a.rho = s.rho;
    a.work = s.geWork;
    a.fail = s.dev_flags;
    a.key = s.key;
    a.iter = iter;
    a.iter_dev = s.capturing ? s.d_iter : nullptr;
    a.noise_zero = s.noise_mode;
    if (s.lev[r].spatial) {
      GESArgs sa{};
      sa.g = a;
      sa.iWg = s.lev[r].iWg;
      sa.AlphaD = s.lev[r].AlphaD;
      launch_gamma_eta_spatial(s, sa, s.stream);
    } else if (a.nc * a.ns > GE_WG_MAX) {
      launch_gamma_eta_blocked(s, a, s.stream);
    } else {
      if (a.nf <= GE_NF_SMALL)
        gamma_eta_kernel<GE_NF_SMALL><<<1, 1024, 0, s.stream>>>(a);
      else if (a.nf <= GE_NF_LARGE)
        gamma_eta_kernel<GE_NF_LARGE><<<1, 1024, 0, s.stream>>>(a);
      else
        gamma_eta_kernel<GE_NF_XL><<<1, 1024, 0, s.stream>>>(a);
    }
    HIP_OK(hipGetLastError());
  }
  // Eta changed: XEta, its Gram and X'Eta Z of the next BetaLambda are stale
  s.xeta_valid = false;
  s.zt_valid = false;
}

}  // namespace hmsc
