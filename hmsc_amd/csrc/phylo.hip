// Phylogeny branch (hM$C != NULL) on the device.
//
// The reference precomputes, for every grid value rho_g of hM$rhopw, the dense
// Q_g = rho_g C + (1 - rho_g) I, its inverse iQg, Cholesky factor RQg and log-determinant
// (R/computeDataParameters.R:19-39), and then per sweep takes iQg[,,rho] in updateGammaV
// (R/updateGammaV.R:14-32), runs 101 triangular solves in updateRho (R/updateRho.R:14-17) and
// builds a dense (ns K)^2 precision in updateBetaLambda (R/updateBetaLambda.R:124-147).
//
// Here every Q_g shares the eigenvectors of C:  C = U diag(d) U^T  gives
//   Q_g = U diag(q_g) U^T,   q_g,i = rho_g d_i + 1 - rho_g   (rho_g >= 0)
//                                    -rho_g / d_i + 1 + rho_g  (rho_g < 0, iC branch)
// so the whole grid is one ns x nrho table of 1 / q_g,i plus log det Q_g = sum_i log q_g,i
// (host, hmsc_create).  Per sweep the only ns^2 work is Bt = Beta U; then
//   E iQ E^T         = Et diag(w) Et^T          Et = Bt - Gamma Tt^T, Tt = U^T Tr
//   Tr^T iQ Tr       = Tt^T diag(w) Tt
//   (iV B)(iQ Tr)    = iV Bt diag(w) Tt
//   |RQ_g^-T E RiV^T|^2 = sum_i w_g,i Et_i^T iV Et_i          (updateRho's v_g)
// with w = 1 / q_rho: the 101 backsolves become one weighted sum per grid point.  Only the
// dense BetaLambda system needs iQ itself, assembled from U and w inside that kernel.
#include <algorithm>

#include "common.h"
#include "state.h"

namespace hmsc {

struct PhyloArgs {
  int ns, nc, nt, K, Kmax, NF, nr, nrho;
  int lev_nf[HMSC_MAX_LEVELS];
  const double* U;       // ns x ns eigenvectors of C
  const double* Winv;    // nrho x ns: 1 / q_g,i  (row g contiguous)
  const double* rbase;   // nrho: log(rhopw[g,2]) - 0.5 nc logdet Q_g
  const double* Tt;      // ns x nt  U^T Tr
  const double* Tr;      // ns x nt
  const double* BL;      // K x ns
  double* BLout;         // K x ns (dense BetaLambda draw)
  const double* Gamma;   // nc x nt
  const double* iV;      // nc x nc
  const double* G;       // Kmax x Kmax  XEta^T XEta
  const double* XZ;      // K x ns       XEta^T Z
  const double* iSigma;  // ns
  const double* Psi;     // NF x ns
  const double* Delta;   // NF
  double* rho;           // 1-based grid index (double)
  double* Bt;            // nc x ns
  double* Et;            // nc x ns
  double* part;          // [E iQ E^T (nc^2) | B iQ Tr (nc nt)]
  double* TTw;           // nt x nt
  double* work;          // dense BetaLambda: M (N^2) | iQ (ns^2) | rhs (N) | Y (nc ns) | tau (NF)
  int* fail;
  Key key;
  uint32_t iter;
  const uint32_t* iter_dev;
  int noise_zero;
};

__device__ inline int rho_index(const double* rho) { return (int)(*rho) - 1; }

// Bt = Beta U  (nc x ns): one thread per output, U columns read contiguously
__global__ __launch_bounds__(256) void phylo_bt_kernel(PhyloArgs a) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= a.nc * a.ns) return;
  const int c = idx % a.nc, i = idx / a.nc;
  const double* u = a.U + (size_t)a.ns * i;
  double s = 0.0;
  for (int j = 0; j < a.ns; ++j) s = fma(a.BL[c + (size_t)a.K * j], u[j], s);
  a.Bt[idx] = s;
}

// Et = Bt - Gamma Tt^T for the current Gamma (workgroup-wide, ends with a barrier)
__device__ inline void phylo_et(const PhyloArgs& a) {
  for (int p = threadIdx.x; p < a.nc * a.ns; p += blockDim.x) {
    const int c = p % a.nc, i = p / a.nc;
    double m = 0.0;
    for (int q = 0; q < a.nt; ++q) m = fma(a.Gamma[c + a.nc * q], a.Tt[i + (size_t)a.ns * q], m);
    a.Et[p] = a.Bt[p] - m;
  }
  __syncthreads();
}

// updateGammaV's iQ-weighted sums (R/updateGammaV.R:16-18,29-30) in the eigenbasis; the
// Wishart / Gamma algebra that follows is the shared gammav kernel with nparts = 1, TT = TTw.
__global__ __launch_bounds__(1024) void phylo_gv_kernel(PhyloArgs a) {
  phylo_et(a);
  const double* w = a.Winv + (size_t)a.ns * rho_index(a.rho);
  const int nc = a.nc, nt = a.nt, ns = a.ns, nA = nc * nc, nB = nc * nt;
  const int lane = threadIdx.x & 63, nw = blockDim.x >> 6;
  // one wave per output, lanes over species (a thread per output waited out ns dependent
  // L2 round trips)
  for (int p = threadIdx.x >> 6; p < nA + nB + nt * nt; p += nw) {
    double s = 0.0;
    if (p < nA) {  // A = E iQ E^T
      const int c1 = p % nc, c2 = p / nc;
      for (int i = lane; i < ns; i += 64) s = fma(w[i] * a.Et[c1 + nc * i], a.Et[c2 + nc * i], s);
    } else if (p < nA + nB) {  // B iQ Tr
      const int q = p - nA, c = q % nc, t = q / nc;
      for (int i = lane; i < ns; i += 64) s = fma(w[i] * a.Bt[c + nc * i], a.Tt[i + (size_t)ns * t], s);
    } else {  // Tr^T iQ Tr = crossprod(backsolve(RQ, Tr, transpose=TRUE))
      const int q = p - nA - nB, t1 = q % nt, t2 = q / nt;
      for (int i = lane; i < ns; i += 64) s = fma(w[i] * a.Tt[i + (size_t)ns * t1], a.Tt[i + (size_t)ns * t2], s);
    }
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if (lane == 0) {
      if (p < nA + nB)
        a.part[p] = s;
      else
        a.TTw[p - nA - nB] = s;
    }
  }
}

// updateRho (R/updateRho.R:1-25) given the new Gamma and iV: v_g = sum_i w_g,i Et_i^T iV Et_i,
// logLike_g = log(rhopw[g,2]) - nc/2 logdet Q_g - v_g/2, one categorical draw by inversion.
__global__ __launch_bounds__(1024) void phylo_rho_kernel(PhyloArgs a) {
  phylo_et(a);
  const int nc = a.nc, ns = a.ns;
  double* sq = a.work;  // ns quadratic forms
  for (int i = threadIdx.x; i < ns; i += blockDim.x) {
    const double* e = a.Et + (size_t)nc * i;
    double s = 0.0;
    for (int c2 = 0; c2 < nc; ++c2) {
      double r = 0.0;
      for (int c1 = 0; c1 < nc; ++c1) r = fma(a.iV[c1 + nc * c2], e[c1], r);
      s = fma(r, e[c2], s);
    }
    sq[i] = s;
  }
  __syncthreads();
  double* ll = a.work + ns;  // nrho log-likelihoods: one wave per grid point, lanes over species
  {
    const int lane = threadIdx.x & 63, nw = blockDim.x >> 6;
    for (int g = threadIdx.x >> 6; g < a.nrho; g += nw) {
      const double* w = a.Winv + (size_t)ns * g;
      double v = 0.0;
      for (int i = lane; i < ns; i += 64) v = fma(w[i], sq[i], v);
      for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
      if (lane == 0) ll[g] = a.rbase[g] - 0.5 * v;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double mx = -INFINITY;
    for (int g = 0; g < a.nrho; ++g) mx = fmax(mx, ll[g]);
    double tot = 0.0;
    for (int g = 0; g < a.nrho; ++g) {
      ll[g] = exp(ll[g] - mx);  // like
      tot += ll[g];
    }
    // sample.int(rhoN, 1, prob = like): first g whose cumulative weight exceeds u * total
    const double u = uniforms(a.key, 0, 0, S_RHO, SWEEP_ITER(a)).a;
    const double target = u * tot;
    double cum = 0.0;
    int pick = 0;
    for (int g = 0; g < a.nrho; ++g) {
      cum += ll[g];
      if (cum <= target) pick = g + 1;
    }
    if (pick >= a.nrho) pick = a.nrho - 1;
    *a.rho = (double)(pick + 1);
  }
}

// Dense updateBetaLambda with phylogeny (R/updateBetaLambda.R:124-147), one workgroup.
// Unknowns in R's species-fastest order u = k ns + j (vec(t(BetaLambda)), byrow=TRUE at :146):
//   iU = kron(XEtaTXEta, diag(iSigma)) + bdiag(kron(iV, iQ), diag(vec(t(priorLambda))))
//   RiU = chol(iU); m1 = RiU^-T (P vec(t(Mu)) + vec(t(isXTS))); BL = RiU^-1 (m1 + xi)
__global__ __launch_bounds__(1024) void phylo_beta_lambda_kernel(PhyloArgs a) {
  __shared__ int flag;
  const int ns = a.ns, nc = a.nc, K = a.K, N = K * ns, t = threadIdx.x, nt = blockDim.x;
  double* M = a.work;
  double* iQ = M + (size_t)N * N;
  double* rhs = iQ + (size_t)ns * ns;
  double* Y = rhs + N;
  double* tau = Y + (size_t)nc * ns;
  const double* w = a.Winv + (size_t)ns * rho_index(a.rho);
  if (t == 0) {  // tau = cumprod(Delta) per level (:42-53)
    int f = 0;
    for (int r = 0; r < a.nr; ++r) {
      double c = 1.0;
      for (int h = 0; h < a.lev_nf[r]; ++h, ++f) {
        c *= a.Delta[f];
        tau[f] = c;
      }
    }
  }
  // iQ = U diag(w) U^T (= iQg[,,rho])
  for (int p = t; p < ns * ns; p += nt) {
    const int j1 = p % ns, j2 = p / ns;
    double s = 0.0;
    for (int i = 0; i < ns; ++i) s = fma(a.U[j1 + (size_t)ns * i] * w[i], a.U[j2 + (size_t)ns * i], s);
    iQ[p] = s;
  }
  // Y = iV Mu, Mu = Gamma Tr^T (:62)
  for (int p = t; p < nc * ns; p += nt) {
    const int c = p % nc, j = p / nc;
    double s = 0.0;
    for (int c2 = 0; c2 < nc; ++c2) {
      double mu = 0.0;
      for (int q = 0; q < a.nt; ++q) mu = fma(a.Gamma[c2 + nc * q], a.Tr[j + (size_t)ns * q], mu);
      s = fma(a.iV[c + nc * c2], mu, s);
    }
    Y[p] = s;
  }
  __syncthreads();
  for (size_t p = t; p < (size_t)N * N; p += nt) {
    const int r = (int)(p % N), c = (int)(p / N);
    const int k1 = r / ns, j1 = r % ns, k2 = c / ns, j2 = c % ns;
    double v = (j1 == j2) ? a.G[k1 + a.Kmax * k2] * a.iSigma[j1] : 0.0;
    if (k1 < nc && k2 < nc)
      v = fma(a.iV[k1 + nc * k2], iQ[j1 + (size_t)ns * j2], v);
    else if (k1 == k2 && j1 == j2)
      v += a.Psi[(k1 - nc) + (size_t)a.NF * j1] * tau[k1 - nc];
    M[p] = v;
  }
  for (int r = t; r < N; r += nt) {  // P vec(t(Mu)) + vec(t(isXTS))
    const int k = r / ns, j = r % ns;
    double v = a.iSigma[j] * a.XZ[k + (size_t)K * j];
    if (k < nc)
      for (int j2 = 0; j2 < ns; ++j2) v = fma(Y[k + nc * j2], iQ[j2 + (size_t)ns * j], v);
    rhs[r] = v;
  }
  __syncthreads();
  if (!wg_chol(M, N, N, &flag) && t == 0) a.fail[2] = 1;  // RiU = chol(.)  (:129)
  wg_forward(M, N, N, rhs);                                // m1 = backsolve(RiU, ., transpose=TRUE)  (:145)
  for (int r = t; r < N; r += nt) {
    const int k = r / ns, j = r % ns;
    if (!a.noise_zero) rhs[r] += normal(a.key, (uint32_t)j, (uint32_t)k, S_BETALAMBDA, SWEEP_ITER(a));
  }
  __syncthreads();
  wg_backward_t(M, N, N, rhs);                             // backsolve(RiU, m1 + rnorm)  (:146)
  for (int r = t; r < N; r += nt) {
    const int k = r / ns, j = r % ns;
    a.BLout[k + (size_t)K * j] = rhs[r];
  }
}

// ---- the same system above one workgroup's reach: multi-workgroup assembly, the blocked
// ---- Cholesky / triangular solves of dense.hip (MFMA trailing updates), elementwise noise
// iQ = U diag(w) U^T  (ns^2 outputs), Y = iV Mu and tau (thread 0 of workgroup 0)
__global__ __launch_bounds__(256) void ph_prep_kernel(PhyloArgs a) {
  const int ns = a.ns, nc = a.nc;
  double* iQ = a.work + (size_t)a.K * ns * (size_t)a.K * ns;
  double* rhs = iQ + (size_t)ns * ns;
  double* Y = rhs + (size_t)a.K * ns;
  double* tau = Y + (size_t)nc * ns;
  const double* w = a.Winv + (size_t)ns * rho_index(a.rho);
  (void)iQ, (void)w;  // iQ = U diag(w) U^T: dense_gram_diag (MFMA tiles)
  const size_t p = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (p < (size_t)nc * ns) {
    const int q = (int)p, c = q % nc, j = q / nc;
    double s = 0.0;
    for (int c2 = 0; c2 < nc; ++c2) {
      double mu = 0.0;
      for (int t = 0; t < a.nt; ++t) mu = fma(a.Gamma[c2 + nc * t], a.Tr[j + (size_t)ns * t], mu);
      s = fma(a.iV[c + nc * c2], mu, s);
    }
    Y[q] = s;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    int f = 0;
    for (int r = 0; r < a.nr; ++r) {
      double c = 1.0;
      for (int h = 0; h < a.lev_nf[r]; ++h, ++f) {
        c *= a.Delta[f];
        tau[f] = c;
      }
    }
  }
}

// lower triangle of iU (grid (N / 256, N)) and the right-hand side (column 0 row of blocks)
__global__ __launch_bounds__(256) void ph_assemble_kernel(PhyloArgs a) {
  const int ns = a.ns, nc = a.nc, N = a.K * ns;
  double* M = a.work;
  const double* iQ = M + (size_t)N * N;
  const double* tau = iQ + (size_t)ns * ns + N + (size_t)nc * ns;
  const int c = blockIdx.y, r = blockIdx.x * 256 + threadIdx.x;
  if (r >= N || r < c) return;
  const int k1 = r / ns, j1 = r % ns, k2 = c / ns, j2 = c % ns;
  double v = (j1 == j2) ? a.G[k1 + a.Kmax * k2] * a.iSigma[j1] : 0.0;
  if (k1 < nc && k2 < nc)
    v = fma(a.iV[k1 + nc * k2], iQ[j1 + (size_t)ns * j2], v);
  else if (k1 == k2 && j1 == j2)
    v += a.Psi[(k1 - nc) + (size_t)a.NF * j1] * tau[k1 - nc];
  M[r + (size_t)N * c] = v;
}

// rhs = vec(iSigma XZ) + (P Mu) rows: one wave per output (the nc ns P Mu entries are
// ns-term sums over iQ's column j, lanes over j2)
__global__ __launch_bounds__(256) void ph_rhs_kernel(PhyloArgs a) {
  const int ns = a.ns, nc = a.nc, K = a.K, N = K * ns;
  const double* iQ = a.work + (size_t)N * N;
  double* rhs = (double*)iQ + (size_t)ns * ns;
  const double* Y = rhs + N;
  const int lane = threadIdx.x & 63;
  const int w0 = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6), ws = (int)((gridDim.x * blockDim.x) >> 6);
  for (int r = w0; r < N; r += ws) {
    const int k = r / ns, j = r % ns;
    double pm = 0.0;
    if (k < nc) {
      for (int j2 = lane; j2 < ns; j2 += 64) pm = fma(Y[k + nc * j2], iQ[j2 + (size_t)ns * j], pm);
      for (int o = 32; o > 0; o >>= 1) pm += __shfl_xor(pm, o);
    }
    if (lane == 0) rhs[r] = a.iSigma[j] * a.XZ[k + (size_t)K * j] + pm;
  }
}

__global__ __launch_bounds__(256) void ph_noise_kernel(PhyloArgs a) {
  const int ns = a.ns, N = a.K * ns;
  double* rhs = a.work + (size_t)N * N + (size_t)ns * ns;
  const int r = blockIdx.x * 256 + threadIdx.x;
  if (r >= N || a.noise_zero) return;
  rhs[r] += normal(a.key, (uint32_t)(r % ns), (uint32_t)(r / ns), S_BETALAMBDA, SWEEP_ITER(a));
}

__global__ __launch_bounds__(256) void ph_store_kernel(PhyloArgs a) {
  const int ns = a.ns, N = a.K * ns;
  const double* rhs = a.work + (size_t)N * N + (size_t)ns * ns;
  const int r = blockIdx.x * 256 + threadIdx.x;
  if (r >= N) return;
  a.BLout[r / ns + (size_t)a.K * (r % ns)] = rhs[r];
}

// K * ns above which the dense BetaLambda system goes to the multi-workgroup blocked path
constexpr int PH_BLOCKED_N = 1024;

static PhyloArgs phylo_args(State& s, uint32_t iter) {
  PhyloArgs a{};
  a.ns = s.ns;
  a.nc = s.nc;
  a.nt = s.nt;
  a.K = s.K;
  a.Kmax = s.Kmax;
  a.NF = s.NF;
  a.nr = s.nr;
  a.nrho = s.nrho;
  for (int r = 0; r < s.nr; ++r) a.lev_nf[r] = s.lev[r].nf;
  a.U = s.phU;
  a.Winv = s.phWinv;
  a.rbase = s.phRbase;
  a.Tt = s.phTt;
  a.Tr = s.Tr;
  a.BL = s.BL;
  a.BLout = s.BL;
  a.Gamma = s.Gamma;
  a.iV = s.iV;
  a.G = s.G;
  flush_xz(s);
  a.XZ = s.XZ;
  a.iSigma = s.iSigma;
  a.Psi = s.Psi;
  a.Delta = s.Delta;
  a.rho = s.rho;
  a.Bt = s.phBt;
  a.Et = s.phEt;
  a.part = s.ABpart;
  a.TTw = s.phTTw;
  a.work = s.phWork;
  a.fail = s.dev_flags;
  a.key = s.key;
  a.iter = iter;
  a.iter_dev = s.capturing ? s.d_iter : nullptr;
  a.noise_zero = s.noise_mode;
  return a;
}

size_t phylo_work_doubles(int ns, int Kmax, int nc, int nrho) {
  const size_t N = (size_t)Kmax * ns;
  const size_t bl = N * N + (size_t)ns * ns + N + (size_t)nc * ns + (size_t)Kmax + dense_ws_doubles((int)N) + 64;
  const size_t rho = (size_t)ns + nrho + 64;
  return bl > rho ? bl : rho;
}

void launch_phylo_gv_sums(State& s, uint32_t iter, hipStream_t st) {
  PhyloArgs a = phylo_args(s, iter);
  phylo_bt_kernel<<<(s.nc * s.ns + 255) / 256, 256, 0, st>>>(a);
  HIP_OK(hipGetLastError());
  phylo_gv_kernel<<<1, 1024, 0, st>>>(a);
  HIP_OK(hipGetLastError());
}

void launch_rho(State& s, uint32_t iter, hipStream_t st) {
  ProfScope ps(s, PROF_RHO);
  PhyloArgs a = phylo_args(s, iter);
  phylo_bt_kernel<<<(s.nc * s.ns + 255) / 256, 256, 0, st>>>(a);  // Beta may have changed since GammaV
  HIP_OK(hipGetLastError());
  phylo_rho_kernel<<<1, 1024, 0, st>>>(a);
  HIP_OK(hipGetLastError());
}

void launch_beta_lambda_phylo(State& s, uint32_t iter) {
  HMSC_REQUIRE((size_t)s.K * s.ns <= (size_t)s.phNmax, "phylogeny BetaLambda: K * ns exceeds the allocation");
  PhyloArgs a = phylo_args(s, iter);
  const int N = s.K * s.ns;
  if (N <= PH_BLOCKED_N) {
    phylo_beta_lambda_kernel<<<1, 1024, 0, s.stream>>>(a);
    HIP_OK(hipGetLastError());
    return;
  }
  // blocked: RiU = chol(iU) as the lower factor L = RiU^T; BL = L^-T (L^-1 rhs + xi)
  const size_t ns2 = (size_t)s.ns * s.ns;
  double* M = s.phWork;
  double* rhs = M + (size_t)N * N + ns2;
  double* ws = rhs + N + (size_t)s.nc * s.ns + s.Kmax;
  const int g1 = (N + 255) / 256;
  dense_gram_diag(s.stream, s.phU, s.ns, s.ns, s.phWinv, s.rho, false, M + (size_t)N * N, s.ns);  // iQ
  ph_prep_kernel<<<(unsigned)(((size_t)s.nc * s.ns + 255) / 256), 256, 0, s.stream>>>(a);
  ph_assemble_kernel<<<dim3(g1, N), 256, 0, s.stream>>>(a);
  ph_rhs_kernel<<<(unsigned)std::min<size_t>(4096, ((size_t)N * 64 + 255) / 256), 256, 0, s.stream>>>(a);
  HIP_OK(hipGetLastError());
  dense_potrf_lower(s.stream, M, N, N, ws, s.dev_flags + 2, 0, s.trsv_sync);
  dense_trsv_lower(s.stream, M, N, N, rhs, 0, ws, 0, s.trsv_sync);   // m1 = backsolve(RiU, ., transpose=TRUE)  (:145)
  ph_noise_kernel<<<g1, 256, 0, s.stream>>>(a);
  dense_trsv_lower(s.stream, M, N, N, rhs, 1, ws, 0, s.trsv_sync);   // backsolve(RiU, m1 + rnorm)  (:146)
  ph_store_kernel<<<g1, 256, 0, s.stream>>>(a);
  HIP_OK(hipGetLastError());
}

}  // namespace hmsc
