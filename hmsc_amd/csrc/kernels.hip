// HIP kernels for one Gibbs sweep of Hmsc's sampleMcmc (R/sampleMcmc.R:219-306) on gfx950.
//
// Dataflow (per sweep, synthetic config ny=10k ns=1k nc=20 nf=10):
//   updateZ      z_wave_kernel    (z_kernel.h) E = XEta*BL on the matrix cores, truncated-
//                                 normal draw, stores Z, and, while the Z tile is still on
//                                 chip, the contractions of Z the next sweep needs:
//                                   XZ  = XEta^T (Yx o Z)   (updateBetaLambda, R/updateBetaLambda.R:66)
//                                   ZTr = Z Tr              (updateGamma2, R/updateGamma2.R:46)
//                                 so updateBetaLambda never re-reads Z from HBM
//                xeta_gram_kernel G = XEta^T XEta (R/updateBetaLambda.R:65), once per Eta update.
//   updateBetaLambda  beta_lambda_kernel  one wave per species: K x K precision in LDS,
//                                 Cholesky, two triangular solves, draw.
//   updateGammaV / updateGamma2 / updateLambdaPriors: species-parallel partial reductions
//                                 + one single-workgroup kernel for the tiny dense algebra.
//   updateEta    zl_kernel        the one HBM pass over Z: ZL = Z (Lambda diag(iSigma))^T
//                eta_unit_kernel  one wave per unit: nf x nf precision, Cholesky, draw.
//   updateInvSigma  inv_sigma_kernel (normal species only).
// All randomness: counter-based Philox (rng.h), keyed by chain seed, counted by
// (element, sub, stream, sweep), so draws do not depend on grid shape or sharding.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <vector>
#include <map>
#include <mutex>

#include "common.h"
#include "rng.h"
#include "state.h"
#include "wave_la.h"
#include "z_kernel.h"

namespace hmsc {

#ifdef HMSC_STAMPS
__device__ unsigned long long g_stamps[1024];
#endif

void read_stamps(double* out, int n) {
#ifdef HMSC_STAMPS
  unsigned long long h[1024];
  HMSC_REQUIRE(n <= 1024, "stamps: at most 1024 slots");
  HIP_OK(hipMemcpyFromSymbol(h, HIP_SYMBOL(g_stamps), sizeof(h)));
  for (int i = 0; i < n; ++i) out[i] = (double)h[i];
#else
  (void)out;
  (void)n;
  throw HmscError(-1, "stamps: this library was built without --stamps");
#endif
}

// ---------------------------------------------------------------------------
// XEta row gather: XEta[i, k] = X[i, k] (k < nc) or Eta_r[Pi_r[i], h]
// ---------------------------------------------------------------------------
struct EtaView {
  const double* X;
  int ny, nc, nr;
  const double* Eta[HMSC_MAX_LEVELS];
  const int* Pi[HMSC_MAX_LEVELS];
  int np[HMSC_MAX_LEVELS];
  int nf[HMSC_MAX_LEVELS];
  // covariate-dependent level r: its columns are Eta[Pi, h] * x[Pi, k] (R/updateBetaLambda.R:25-27)
  const double* xs[HMSC_MAX_LEVELS];
};

__device__ __forceinline__ double xeta_at(const EtaView& v, int i, int k) {
  if (k < v.nc) return v.X[i + (size_t)v.ny * k];
  int h = k - v.nc;
  for (int r = 0; r < v.nr; ++r) {
    if (h < v.nf[r]) {
      const int q = v.Pi[r][i];
      const double e = v.Eta[r][q + (size_t)v.np[r] * h];
      return v.xs[r] ? e * v.xs[r][q] : e;
    }
    h -= v.nf[r];
  }
  return 0.0;
}

static void launch_gamma2_prep(State& s, hipStream_t st);

static EtaView make_view(const State& s) {
  EtaView v{};
  v.X = s.X;
  v.ny = s.ny;
  v.nc = s.nc;
  v.nr = s.nr;
  for (int r = 0; r < s.nr; ++r) {
    v.Eta[r] = s.lev[r].Eta;
    v.Pi[r] = s.lev[r].Pi;
    v.np[r] = s.lev[r].np;
    v.nf[r] = s.lev[r].nf;
    v.xs[r] = s.lev[r].xs;
  }
  return v;
}

// Materialise XEta = [X, Eta_1[Pi_1,], ...] (R/updateBetaLambda.R:21-41) for one 64-site
// tile and accumulate its Gram XEta^T XEta (:65) -> slab part[tile].
__global__ __launch_bounds__(256) void xeta_gram_kernel(EtaView ev, int K, int Kmax, double* XEta, double* G_part) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  double* sXE = smem;  // [k][ZT_LD]
  const int t = threadIdx.x, ny = ev.ny, i0 = blockIdx.x * 64;
  for (int p = t; p < K * 64; p += 256) {
    const int k = p >> 6, ii = p & 63, i = i0 + ii;
    double v = 0.0;
    if (i < ny) {
      v = xeta_at(ev, i, k);
      XEta[i + (size_t)ny * k] = v;
    }
    sXE[k * ZT_LD + ii] = v;
  }
  __syncthreads();
  double* dst = G_part + (size_t)blockIdx.x * Kmax * Kmax;
  for (int p = t; p < K * K; p += 256) {
    const int k1 = p % K, k2 = p / K;
    const double* x1 = sXE + k1 * ZT_LD;
    const double* x2 = sXE + k2 * ZT_LD;
    double acc = 0.0;
#pragma unroll 8
    for (int ii = 0; ii < 64; ++ii) acc = fma(x1[ii], x2[ii], acc);
    dst[k1 + Kmax * k2] = acc;
  }
}

// deterministic slab reduction: out[e] = sum_c part[c*stride + e]; 64 outputs per block,
// the four waves take every fourth partial (coalesced 512-B rows), fixed summation order.
// (bid, nb): this block's index among the nb blocks of the reduction (co-launched kernels
// hand a slab reduction a sub-range of their grid).
__device__ __forceinline__ void slab_sum_body(const double* __restrict__ part, double* __restrict__ out, int64_t n,
                                              int nparts, int64_t stride, int bid, int nb) {
  __shared__ double red[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int64_t base = (int64_t)bid * 64; base < n; base += (int64_t)nb * 64) {
    const int64_t e = base + lane;
    double s = 0.0;
    if (e < n) {  // up to 16 partials of a wave's loads in flight, summed in the same order
      for (int c0 = w; c0 < nparts; c0 += 64) {
        double x[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) x[u] = part[(int64_t)min(c0 + 4 * u, nparts - 1) * stride + e];
#pragma unroll
        for (int u = 0; u < 16; ++u)
          if (c0 + 4 * u < nparts) s += x[u];
      }
    }
    red[w][lane] = s;
    __syncthreads();
    if (w == 0 && e < n) out[e] = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void slab_sum_kernel(const double* __restrict__ part, double* __restrict__ out,
                                                       int64_t n, int nparts, int64_t stride) {
  slab_sum_body(part, out, n, nparts, stride, blockIdx.x, gridDim.x);
}

struct SlabJob {
  const double* part;
  double* out;
  int64_t n, stride;
  int nparts, nb;
};

// all-reduce A's species sums of a sharded chain (g2_stats_body, below)
struct G2SArgs {
  const double* XZ;
  const double* XZpart;  // updateZ's chunk partials (the slab launch's co-launched stats), else null
  int64_t xz_stride;
  int xz_nparts;
  const double* BL;
  const double* Tr;
  const double* iSigma;
  const double* xtztr;
  double* part;
  int* ticket;
  double* out;
  int K, nc, NF, nt, nsl, nparts;
};
__device__ void g2_stats_body(const G2SArgs& a, int bid, double* smem);
struct G2SJob {
  G2SArgs a;
  size_t smem;
};
G2SJob shard_g2_job(State& s, const double* xz_part, int xz_nparts);

__device__ void side_gate_body(const SideGate& g);

// two independent slab reductions in one launch: blocks [0, j0.nb) reduce j0, the next j1.nb
// j1, then (a sharded chain's sweep) ng2 blocks of all-reduce A's species sums from updateZ's
// chunk partials, and a last block the side gate when there is one
__global__ __launch_bounds__(256) void slab_sum2_kernel(SlabJob j0, SlabJob j1, SideGate g, G2SArgs g2, int ng2) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int b = blockIdx.x;
  if (b < j0.nb)
    slab_sum_body(j0.part, j0.out, j0.n, j0.nparts, j0.stride, b, j0.nb);
  else if (b < j0.nb + j1.nb)
    slab_sum_body(j1.part, j1.out, j1.n, j1.nparts, j1.stride, b - j0.nb, j1.nb);
  else if (b < j0.nb + j1.nb + ng2)
    g2_stats_body(g2, b - j0.nb - j1.nb, smem);
  else
    side_gate_body(g);
}

static int grid_for(int64_t n, int block = 64, int cap = 2048) {
  int64_t g = (n + block - 1) / block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

void launch_xeta(State& s) {
  s.g_pending = false;  // G rebuilt below
  const int n_tiles = (s.ny + 63) / 64;
  xeta_gram_kernel<<<n_tiles, 256, (size_t)s.K * ZT_LD * sizeof(double), s.stream>>>(make_view(s), s.K, s.Kmax,
                                                                                       s.XEta, s.G_part);
  HIP_OK(hipGetLastError());
  const int64_t nG = (int64_t)s.Kmax * s.Kmax;
  slab_sum_kernel<<<grid_for(nG), 256, 0, s.stream>>>(s.G_part, s.G, nG, n_tiles, nG);
  HIP_OK(hipGetLastError());
  s.xeta_valid = true;
}

// masked Gram XEta^T diag(Yx_j) XEta for species with NA (R/updateBetaLambda.R:103-112)
__global__ __launch_bounds__(256) void gram_na_kernel(EtaView ev, const double* XEta, int K, int Kmax, const int* na_cols,
                                                      const int8_t* Ycode, double* Gna) {
  const int c = blockIdx.x;
  const int j = na_cols[c];
  const int ny = ev.ny;
  double* out = Gna + (size_t)c * Kmax * Kmax;
  for (int p = threadIdx.x; p < K * K; p += blockDim.x) {
    const int k1 = p % K, k2 = p / K;
    if (k1 > k2) continue;
    double s = 0.0;
    for (int i = 0; i < ny; ++i)
      if (Ycode[(size_t)i + (size_t)ny * j] >= 0) s += XEta[i + (size_t)ny * k1] * XEta[i + (size_t)ny * k2];
    out[k1 + Kmax * k2] = s;
    out[k2 + Kmax * k1] = s;
  }
}

// the two slab reductions that follow the z kernel (XZ, ZTr), one launch (zdraw.hip)
void launch_slab_sum2(const double* p0, double* o0, int64_t n0, int np0, const double* p1, double* o1, int64_t n1,
                      int np1, hipStream_t st, SideGate gate, State* g2s) {
  const SlabJob j0{p0, o0, n0, n0, np0, grid_for(n0)};
  const SlabJob j1{p1, o1, n1, n1, np1, grid_for(n1)};
  G2SJob job{};
  if (g2s) job = shard_g2_job(*g2s, p0, np0);  // (p0: updateZ's XZ chunk partials)
  const G2SJob* g2 = g2s ? &job : nullptr;
  const int ng2 = g2 ? g2->a.nparts : 0;
  slab_sum2_kernel<<<j0.nb + j1.nb + ng2 + (gate.n > 0 ? 1 : 0), 256, g2 ? g2->smem : 0, st>>>(
      j0, j1, gate, g2 ? g2->a : G2SArgs{}, ng2);
  HIP_OK(hipGetLastError());
}

// XZ as its consumers read it: the reduced buffer, or updateZ's chunk partials when the z
// launch left the reduction to them (State::xz_parts)
XZSrc xz_src(const State& s) {
  return s.xz_parts > 0 ? XZSrc{s.XZ, s.XZ_part, s.xz_parts, (int64_t)s.K * s.nsl} : XZSrc{s.XZ, nullptr, 0, 0};
}

// the reduction itself, for consumers that read s.XZ directly
void flush_xz(State& s) {
  if (s.xz_parts == 0) return;
  launch_slab_sum2(s.XZ_part, s.XZ, (int64_t)s.K * s.nsl, s.xz_parts, nullptr, nullptr, 0, 1, s.stream);
  s.xz_parts = 0;
}

// ---------------------------------------------------------------------------
// updateBetaLambda, C = NULL branch (R/updateBetaLambda.R:76-123): one wave per
// species, K x K precision iU = P + iSigma_j G in LDS, Cholesky, m = iU^-1 rhs,
// draw m + R^-1 xi  computed as  L^-T (L^-1 rhs + xi).
// ---------------------------------------------------------------------------
struct BLArgs {
  int K, Kmax, nc, nt, nr, NF, ns_loc, ns_glob, sp0;
  const double* G;
  const double* Gna;
  const int* na_index;  // per local species: row in Gna or -1
  XZSrc xz;
  const double* iV;
  const double* Gamma;
  const double* Tr;
  const double* Psi;
  const double* Delta;
  const double* iSigma;
  int lev_nf[HMSC_MAX_LEVELS];
  double* BL;
  double* dbg_prec;
  Key key;
  uint32_t iter;
  const uint32_t* iter_dev;  // graph replay: the sweep counter is read from the device
  unsigned long long* kt;    // live launch timing (KT_BL block) or null
  int kt_defer;              // the fused launch's tail records the BetaLambda timing (BLCol kt0 / kt1)
  int noise_zero;
  // the draws of this sweep made ahead by the previous sweep's Eta launch (bl_predraw_body),
  // used when pre_tag holds (this sweep, K); else drawn here -- the same bits either way
  const double* pre_buf;
  const int* pre_tag;
};

__global__ __launch_bounds__(64) void beta_lambda_kernel(BLArgs a) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int K = a.K, nc = a.nc;
  double* A = smem;               // K x K
  double* rhs = A + K * K;        // K
  double* tau = rhs + K;          // NF
  double* mu = tau + a.NF + 1;    // nc
  int* flag = (int*)(mu + nc + 1);
  const int j = blockIdx.x, t = threadIdx.x;
  if (t == 0) {  // tau = cumprod(delta) per level (R/updateBetaLambda.R:51)
    int f = 0;
    for (int r = 0; r < a.nr; ++r) {
      double c = 1.0;
      for (int h = 0; h < a.lev_nf[r]; ++h, ++f) {
        c *= a.Delta[f];
        tau[f] = c;
      }
    }
  }
  for (int c = t; c < nc; c += 64) {  // Mu_j = Gamma Tr_j^T   (:62)
    double m = 0.0;
    for (int q = 0; q < a.nt; ++q) m += a.Gamma[c + nc * q] * a.Tr[j + (size_t)a.ns_loc * q];
    mu[c] = m;
  }
  __syncthreads();
  const double isig = a.iSigma[j];
  const int nai = a.na_index ? a.na_index[j] : -1;
  const double* Gj = nai >= 0 ? a.Gna + (size_t)nai * a.Kmax * a.Kmax : a.G;
  for (int p = t; p < K * K; p += 64) {  // iU = P + XEtaTXEta * iSigma[j]   (:83-92)
    const int r = p % K, c = p / K;
    double v = isig * Gj[r + a.Kmax * c];
    if (r < nc && c < nc)
      v += a.iV[r + nc * c];
    else if (r == c)
      v += a.Psi[(r - nc) + (size_t)a.NF * j] * tau[r - nc];
    A[p] = v;
  }
  for (int r = t; r < K; r += 64) {  // rhs = P Mu + isXTS   (:66, :100)
    double v = isig * xz_get(a.xz, r + (size_t)K * j);
    if (r < nc) {
      double pm = 0.0;
      for (int c = 0; c < nc; ++c) pm += a.iV[r + nc * c] * mu[c];
      v += pm;
    }
    rhs[r] = v;
  }
  __syncthreads();
  if (a.dbg_prec)
    for (int p = t; p < K * K; p += 64) a.dbg_prec[(size_t)j * K * K + p] = A[p];
  wg_chol(A, K, K, flag);                 // RiU = chol(iU)  (:98)
  wg_forward(A, K, K, rhs);               // y = L^-1 rhs
  for (int r = t; r < K; r += 64) {
    const double xi = a.noise_zero ? 0.0 : normal(a.key, (uint32_t)(a.sp0 + j), (uint32_t)r, S_BETALAMBDA, SWEEP_ITER(a));
    rhs[r] += xi;
  }
  __syncthreads();
  wg_backward_t(A, K, K, rhs);            // L^-T (y + xi) = m + backsolve(RiU, xi)  (:101)
  for (int r = t; r < K; r += 64) a.BL[r + (size_t)K * j] = rhs[r];
}

// Wave-resident variant for K <= 32: one species per wave, four per workgroup; the K x K
// precision lives in registers (row r in lane r), Cholesky / solves via wave_la.h.  The
// inputs every species shares (G = XEta^T XEta, iV, Gamma, tau = cumprod(Delta)) are staged
// into LDS once per workgroup by all 256 threads, so each wave's prologue is LDS reads plus
// its own species' column loads, all issued before the first use.
// LDS of the body (doubles): the four waves' tiles, G, iV, Gamma, tau
constexpr int BLW_LDS = 4 * WV_TILE + 32 * 33 + 32 * 32 + 32 * 8 + 64;
// (gamma2_partial_body from XZ's chunk partials in the fused launch: K x SB, SB x nt, 4 nc SB)
// species per block of updateGamma2's species sums (gamma2_partial_body): small blocks, so that
// a block's partial is quick when it sums XZ from updateZ's chunk partials itself (the fused
// launch with xz_parts > 0)
constexpr int G2SB = 8;
static_assert(32 * G2SB + G2SB * 8 + 4 * 32 * G2SB <= BLW_LDS, "fused Gamma2 partial: LDS");

// the fused Gamma2 + BetaLambda launch's publish value for sweep `iter`: never 0 (the reset
// value hmsc_run / the eager launcher write), distinct for distinct sweeps of a run
__device__ __host__ inline int g2bl_epoch(uint32_t iter) { return (int)(iter | 0x80000000u); }

// WAIT_GAMMA (the fused Gamma2 + BetaLambda launch, gamma2_bl_kernel): the new Gamma is
// published by another workgroup of the same launch (gsync[1]); everything that does not
// depend on it -- the prologue, iU and its Cholesky factor -- runs first.
// Bounded wait (every thread) until flags[0 .. n-1] all hold `epoch`; a wait that outlasts the
// bound raises the launch's handshake error word (err[3], reported as error -5 by the host)
// and goes on.  Relaxed polls: the data behind the flags is read with load_coherent.
__device__ __forceinline__ void side_wait(const int* flags, int n, int epoch, int* err) {
  for (int q = 0; q < n; ++q)
    if (!spin_until<8>([&] { return __hip_atomic_load(&flags[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == epoch; }))
      __hip_atomic_store(&err[3], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// side_wait over n <= 64 flags by a whole wave, lane q polling flag q: the flags' round trips
// overlap instead of following one another (two flags in sequence were ~3 us of the BetaLambda
// prologue); every lane of the wave must be active
__device__ __forceinline__ void side_wait_lanes(const int* flags, int n, int epoch, int* err) {
  const int q = threadIdx.x & 63;
  auto seen = [&] {
    return q >= n || __hip_atomic_load(&flags[q < n ? q : 0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == epoch;
  };
  if (!spin_until<8>([&] { return __all(seen()) != 0; }) && q == 0)
    __hip_atomic_store(&err[3], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The gate: wave 0 of the slab launch's extra workgroup polls the side chain's flags of sweep
// `iter` (GammaV, the delta chains, Gamma2's prep), so that launch ends only once they are up and
// the next fused launch -- after a launch boundary -- reads iV, Delta, Psi and the prep with plain
// loads and no poll at its start (on its critical path the polls and the device-coherent loads
// behind them were ~4 us of the BetaLambda prologue).  Bounded like every in-launch wait.
__device__ void side_gate_body(const SideGate& g) {
  if (g.n > 0 && threadIdx.x < 64) side_wait_lanes(g.flags, g.n, g2bl_epoch(SWEEP_ITER(g)), g.err);
}

SideGate side_gate_next(State& s, uint32_t iter) {
  SideGate g{};
  s.side_gated = false;
  if (s.sharded || !s.capturing || !s.edge_free_now || !s.side_tail || !gamma2_bl_fusion_ok(s) ||
      getenv_flag("HMSC_NO_SIDE_GATE"))
    return g;
  g.flags = s.side_sync;
  g.n = 1 + s.nr + ((s.mask & HMSC_UP_GAMMA2) ? 1 : 0);
  g.iter = iter;
  g.iter_dev = s.d_iter;
  g.err = s.gbl_sync;
  s.side_gated = true;
  return g;
}

// What the fused launch's tail (bl_tail) needs of a species' update, lane k holding row k:
// the new column BL[:, j], Mu_j = Gamma Tr_j^T (rows < nc) and tau = cumprod(Delta) (rows >= nc)
struct BLCol {
  double r, mu, tau, isig;
  unsigned long long kt0, kt1;  // the wave's body start / end (wall clock) when the tail records them
  double gpre;                  // the tail's psi draw before its rate (BLPre), when pre-drawn
};

// Work the body runs for the tail while its prologue's loads fly: none by default
struct BLNoPre {
  __device__ double operator()(int, int) const { return 0.0; }
  __device__ double from(const double*, int) const { return 0.0; }
};

// side_wait (the fused launch inside a sweep graph, sweeps after the first): iV and Delta come
// from the previous sweep's side chain, which publishes them through side_sync instead of a
// cross-queue graph edge; they are read with device-coherent loads after its flags.
template <int NM, bool WAIT_GAMMA, class Pre = BLNoPre>
__device__ __forceinline__ BLCol beta_lambda_wave_body(const BLArgs& a, double* lds0, int blk, int* gsync,
                                                       const int* side_sync = nullptr, int side_epoch = 0,
                                                       int side_n = 0, Pre pre = Pre{}) {
  double* tiles = lds0;
  double* sG = tiles + 4 * WV_TILE;
  double* sIV = sG + 32 * 33;
  double* sGam = sIV + 32 * 32;
  double* sTau = sGam + 32 * 8;
  const unsigned long long kt0 = a.kt ? kt_now() : 0ull;
  const int K = a.K, nc = a.nc, nt = a.nt, i = lane_id(), w = threadIdx.x >> 6, t = threadIdx.x;
  const int j = blk * 4 + w;
  if (blk == 0) HMSC_STAMP(60);
  if (WAIT_GAMMA && blk == 40 && w == 0) HMSC_STAMP_RT(91);
  // every global load of the prologue is issued before the first LDS store (a staging loop
  // with a store per iteration waits out one memory latency per iteration); the loads no side
  // flag guards go out first, so their latency overlaps the flags' polls
  double gv[4], ivv[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int p = t + 256 * u, pc = p < K * K ? p : 0;
    gv[u] = a.G[pc % K + (size_t)a.Kmax * (pc / K)];
  }
  const double gam = WAIT_GAMMA ? 0.0 : a.Gamma[t < nc * nt ? t : 0];
  // this species' own inputs, loaded before the barrier so their latency overlaps it
  const int jj = j < a.ns_loc ? j : a.ns_loc - 1;
  const double isig = a.iSigma[jj];
  const double xz = i < K ? xz_get(a.xz, (i < K ? i : 0) + (size_t)K * jj) : 0.0;
  double trj[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) trj[q] = q < nt ? a.Tr[jj + (size_t)a.ns_loc * q] : 0.0;
  const int nai = a.na_index ? a.na_index[jj] : -1;
  // the draw's noise (R/updateBetaLambda.R:101) needs none of it: drawn while the loads fly
  const bool have_pre = a.pre_buf && a.pre_tag[0] == (int)SWEEP_ITER(a) && a.pre_tag[1] == K;
  const double* prow = have_pre ? a.pre_buf + (size_t)jj * 64 : nullptr;
  const double xi_bl = (i < K && !a.noise_zero && j < a.ns_loc)
                           ? (have_pre ? prow[i] : normal(a.key, (uint32_t)(a.sp0 + j), (uint32_t)i, S_BETALAMBDA, SWEEP_ITER(a)))
                           : 0.0;
  const double gpre = j < a.ns_loc ? (have_pre ? pre.from(prow, i) : pre(j, i)) : 0.0;
  if (side_n > 0) side_wait_lanes(side_sync, side_n, side_epoch, gsync);
  if (WAIT_GAMMA && blk == 0 && w == 0) HMSC_STAMP_RT(84);
  // what the previous sweep's side chain published (device-coherent after its flags)
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int p = t + 256 * u;
    ivv[u] = side_n > 0 ? load_coherent(a.iV + (p < nc * nc ? p : 0)) : a.iV[p < nc * nc ? p : 0];
  }
  const double* dp = a.Delta + (t < a.NF ? t : 0);
  const double del = a.NF > 0 ? (side_n > 0 ? load_coherent(dp) : *dp) : 1.0;
  const double* pp = a.Psi + ((i >= nc && i < K) ? (i - nc) + (size_t)a.NF * jj : 0);
  const double psi = (i >= nc && i < K) ? (side_n > 0 ? load_coherent(pp) : *pp) : 0.0;  // (post_bl_kernel's, side)
  if (WAIT_GAMMA && blk == 40 && w == 0) HMSC_STAMP_RT(92);
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int p = t + 256 * u;
    if (p < K * K) sG[p % K + 33 * (p / K)] = gv[u];
    if (p < nc * nc) sIV[p] = ivv[u];
  }
  if (!WAIT_GAMMA && t < nc * nt && t < 32 * 8) sGam[t] = gam;
  if (t < a.NF) sTau[t] = del;  // Delta here; each lane forms its own cumprod below
  __syncthreads();
  if (WAIT_GAMMA && blk == 40 && w == 0) HMSC_STAMP_RT(93);
  if (j >= a.ns_loc) return BLCol{0.0, 0.0, 1.0, 0.0, ~0ull, 0ull, 0.0};
  double* lds = tiles + w * WV_TILE;
  // tau = cumprod(Delta) within the level of factor i - nc   (:51)
  double tau = 1.0;
  if (i >= nc && i < K) {
    int f0 = 0, r = 0;
    while (r < a.nr && f0 + a.lev_nf[r] <= i - nc) f0 += a.lev_nf[r++];
    for (int h = f0; h <= i - nc; ++h) tau *= sTau[h];
  }
  if (WAIT_GAMMA && blk == 40 && w == 0) HMSC_STAMP_RT(100);
  // prior precision diagonal of Lambda rows: Psi_hj * tau_h
  const double pd = (i >= nc && i < K) ? psi * tau : 0.0;
  // iU = P + XEtaTXEta * iSigma[j]   (:83-92)
  double x[NM];
  const int ir = i < K ? i : 0;
  if (nai >= 0) {  // species with NA: its own masked Gram
    const double* Gj = a.Gna + (size_t)nai * a.Kmax * a.Kmax;
#pragma unroll
    for (int k = 0; k < NM; ++k) {
      const int kc = k < K ? k : 0;
      double v = isig * Gj[ir + a.Kmax * kc];
      if (i < nc && k < nc) v += sIV[ir + nc * kc];
      if (i == k) v += pd;
      x[k] = (i < K && k < K) ? v : (i == k ? 1.0 : 0.0);
    }
  } else {
    // every LDS read of the row first, at clamped addresses, then the sums (a read per column
    // with its use right behind it waited out two LDS round trips per column: ~8 k cycles at K =
    // 32); the same operations as one column at a time, uncontracted
    double gk[NM], vk[NM];
    const int ivr = i < nc ? ir : 0;
#pragma unroll
    for (int k = 0; k < NM; ++k) {
      const int kc = k < K ? k : 0;
      gk[k] = sG[ir + 33 * kc];
      vk[k] = sIV[ivr + nc * (k < nc ? k : 0)];
    }
    {
#pragma clang fp contract(off)
#pragma unroll
      for (int k = 0; k < NM; ++k) {
        double v = isig * gk[k];
        if (i < nc && k < nc) v += vk[k];
        if (i == k) v += pd;
        x[k] = (i < K && k < K) ? v : (i == k ? 1.0 : 0.0);
      }
    }
  }
  if (a.dbg_prec && i < K)
#pragma unroll
    for (int k = 0; k < NM; ++k)
      if (k < K) a.dbg_prec[(size_t)j * K * K + i + (size_t)K * k] = x[k];
  double dinv;
  if (blk == 0) HMSC_STAMP(61);
  if (WAIT_GAMMA && blk == 40 && w == 0) HMSC_STAMP_RT(101);
  // the Gamma flag's first poll goes out ahead of the factorization, its latency under it
  const int g_epoch = WAIT_GAMMA ? g2bl_epoch(SWEEP_ITER(a)) : 0;
  const int g_seen = WAIT_GAMMA ? __hip_atomic_load(&gsync[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
  wv_chol<NM>(x, dinv);                    // RiU = chol(iU)  (:98)
  if (blk == 0) HMSC_STAMP(62);
  if (WAIT_GAMMA && blk == 0 && w == 0) HMSC_STAMP_RT(74);
  if (WAIT_GAMMA && blk == 40 && w == 0) HMSC_STAMP_RT(94);
  double mu = 0.0;  // Mu_j = Gamma Tr_j^T   (:62)
  if (WAIT_GAMMA) {
    // the new Gamma of this sweep (updateGamma2, published by the launch's Gamma2 workgroup
    // as this sweep's epoch, so nothing has to reset the flag: a per-wave "done" count for
    // that reset was 1000 same-address device-scope atomics, ~10 us of serialised tail)
    // relaxed polling, and Gamma (the only datum published inside the launch) read with
    // device-coherent loads below: an acquire -- per poll, or one fence per wave after it --
    // invalidates the XCD's L2, and a thousand of them under every other wave of the device
    // took the solves after the wait from 5 to 16 us; bounded: a broken handshake raises the
    // error flag (hmsc_run reports it) instead of hanging
    if (g_seen != g_epoch &&
        !spin_until<8>([&] { return __hip_atomic_load(&gsync[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == g_epoch; }) &&
        i == 0)
      __hip_atomic_store(&gsync[3], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (blk == 0 && w == 0) HMSC_STAMP_RT(75);
    if (blk == 40 && w == 0) HMSC_STAMP_RT(95);
    if (i < nc)
#pragma unroll
      for (int q = 0; q < 8; ++q)
        if (q < nt) {
          const unsigned long long gb = __hip_atomic_load((const unsigned long long*)(a.Gamma + i + nc * q),
                                                          __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          mu += __longlong_as_double((long long)gb) * trj[q];
        }
  } else if (i < nc) {
#pragma unroll
    for (int q = 0; q < 8; ++q)
      if (q < nt) mu += sGam[i + nc * q] * trj[q];
  }
  // rhs = P Mu + isXTS   (:66, :100)
  double r = isig * xz;
  {
    double ivc[NM];  // (the row's LDS reads together, then the chain)
    const int ivr = i < nc ? i : 0;
#pragma unroll
    for (int c = 0; c < NM; ++c) ivc[c] = sIV[ivr + nc * (c < nc ? c : 0)];
    if (i < nc) {
      double pm = 0.0;
#pragma unroll
      for (int c = 0; c < NM; ++c)
        if (c < nc) pm += ivc[c] * bcast(mu, c);
      r += pm;
    }
  }
  if (WAIT_GAMMA && blk == 40 && w == 0) HMSC_STAMP_RT(102);
  wv_forward<NM>(x, dinv, r);              // y = L^-1 rhs
  if (WAIT_GAMMA && blk == 40 && w == 0) HMSC_STAMP_RT(103);
  if (i < K && !a.noise_zero) r += xi_bl;
  if (blk == 0) HMSC_STAMP(63);
  double lt[NM];
  wv_transpose<NM, true>(x, lt, lds);
  if (WAIT_GAMMA && blk == 40 && w == 0) HMSC_STAMP_RT(104);
  wv_backward_t<NM>(lt, dinv, r);          // m + backsolve(RiU, xi)  (:101)
  if (WAIT_GAMMA && blk == 40 && w == 0) HMSC_STAMP_RT(105);
  // the fused launch: write-through, so the side work forked on the device at the tails flag
  // (post_bl_kernel, still inside this launch's lifetime) reads the new column coherently
  if (i < K) {
    if (WAIT_GAMMA)
      store_coherent(a.BL + i + (size_t)K * j, r);
    else
      a.BL[i + (size_t)K * j] = r;
  }
  if (blk == 0) HMSC_STAMP(64);
  if (WAIT_GAMMA && blk == 0 && w == 0) HMSC_STAMP_RT(76);
  if (WAIT_GAMMA && blk == 40 && w == 0) HMSC_STAMP_RT(96);
  // (the fused launch's tail folds the waves' start / end into its reduction tree and records
  // once: a thousand same-address device atomics at the end of the bodies cost ~10 us)
  const unsigned long long kt1 = (a.kt && a.kt_defer) ? kt_now() : 0ull;
  if (a.kt && !a.kt_defer && i == 0) kt_record(a.kt, SWEEP_ITER(a), kt0);
#ifdef HMSC_STAMPS
  if (WAIT_GAMMA && w == 0 && blk < 384) {  // per-workgroup body start / end (wall clock)
    unsigned long long t1;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
    if (i == 0) g_stamps[256 + blk] = t1;
  }
#endif
  return BLCol{r, mu, tau, isig, kt0, kt1, gpre};
}

template <int NM>
__global__ __launch_bounds__(256) void beta_lambda_wave_kernel(BLArgs a) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  beta_lambda_wave_body<NM, false>(a, smem, blockIdx.x, nullptr);
}

static BLArgs make_bl_args(State& s, uint32_t iter);

void launch_beta_lambda(State& s, uint32_t iter) {
  if (!s.xeta_valid) launch_xeta(s);
  flush_g(s);
  if (!s.zt_valid) launch_zt_refresh(s);
  if (s.phylo) {  // dense branch with phylogeny (R/updateBetaLambda.R:124-147), phylo.hip
    ProfScope ps(s, PROF_BL);
    launch_beta_lambda_phylo(s, iter);
    return;
  }
  if (s.n_na_cols > 0) {
    EtaView ev = make_view(s);
    gram_na_kernel<<<s.n_na_cols, 256, 0, s.stream>>>(ev, s.XEta, s.K, s.Kmax, s.na_cols, s.Ycode, s.Gna);
  }
  const BLArgs a = make_bl_args(s, iter);
  ProfScope ps(s, PROF_BL);
  if (s.K <= 32 && s.nt <= 8 && s.nc * s.nt <= 256 && s.NF <= 64) {
    const int nb = (s.nsl + 3) / 4;
    switch (wv_bucket(s.K)) {
      case 8: beta_lambda_wave_kernel<8><<<nb, 256, BLW_LDS * sizeof(double), s.stream>>>(a); break;
      case 16: beta_lambda_wave_kernel<16><<<nb, 256, BLW_LDS * sizeof(double), s.stream>>>(a); break;
      case 24: beta_lambda_wave_kernel<24><<<nb, 256, BLW_LDS * sizeof(double), s.stream>>>(a); break;
      default: beta_lambda_wave_kernel<32><<<nb, 256, BLW_LDS * sizeof(double), s.stream>>>(a); break;
    }
    HIP_OK(hipGetLastError());
    return;
  }
  const size_t smem = ((size_t)s.K * s.K + s.K + s.NF + 1 + s.nc + 1) * sizeof(double) + 16;
  beta_lambda_kernel<<<s.nsl, 64, smem, s.stream>>>(a);
  HIP_OK(hipGetLastError());
}

static BLArgs make_bl_args(State& s, uint32_t iter) {
  BLArgs a{};
  a.K = s.K;
  a.Kmax = s.Kmax;
  a.nc = s.nc;
  a.nt = s.nt;
  a.nr = s.nr;
  a.NF = s.NF;
  a.ns_loc = s.nsl;
  a.ns_glob = s.ns;
  a.sp0 = s.sp0;
  a.G = s.G;
  a.Gna = s.Gna;
  a.na_index = s.n_na_cols > 0 ? s.na_index : nullptr;
  a.xz = xz_src(s);
  a.iV = s.iV;
  a.Gamma = s.Gamma;
  a.Tr = s.Tr;
  a.Psi = s.Psi;
  a.Delta = s.Delta;
  a.iSigma = s.iSigma;
  for (int r = 0; r < s.nr; ++r) a.lev_nf[r] = s.lev[r].nf;
  a.BL = s.BL;
  a.dbg_prec = s.dbg_prec;
  a.key = s.key;
  a.iter = iter;
  a.iter_dev = s.capturing ? s.d_iter : nullptr;
  a.noise_zero = s.noise_mode;
  a.kt = s.kt_on ? s.d_kt + (size_t)KT_BL * 2 * KT_SLOTS : nullptr;
  return a;
}

// ---------------------------------------------------------------------------
// Species-parallel partial sums for updateGammaV (R/updateGammaV.R:16-18,30):
//   A = E E^T (E = Beta - Gamma Tr^T) and BTr = Beta Tr.
// ---------------------------------------------------------------------------
constexpr int SB = 32;  // species per block of the species-sum reductions

// Species-block partial sums for updateGammaV (R/updateGammaV.R:16-18,30):
//   A = E E^T (E = Beta - Gamma Tr^T) and BTr = Beta Tr, staged through LDS.
// coh: BL and Gamma read with device-coherent loads (post_bl_kernel forked on the device while
// the fused Gamma2 + BetaLambda launch that wrote them is still running, post_bl_kernel)
__device__ __forceinline__ void gammav_partial_body(const double* BL, int K, int nc, int nt, int ns_loc,
                                                    const double* Gamma, const double* Tr, double* part,
                                                    double* smem, int bid, bool coh = false) {
  double* sB = smem;             // nc x SB
  double* sE = sB + nc * SB;     // nc x SB
  double* sTr = sE + nc * SB;    // SB x nt
  const int t = threadIdx.x, j0 = bid * SB, nj = min(SB, ns_loc - j0);
  for (int p = t; p < nc * nj; p += 256) {
    const int c = p % nc, jj = p / nc;
    const double* q = BL + c + (size_t)K * (j0 + jj);
    sB[p] = coh ? load_coherent(q) : *q;
  }
  for (int p = t; p < SB * nt; p += 256) {
    const int jj = p % SB, q = p / SB;
    sTr[p] = jj < nj ? Tr[j0 + jj + (size_t)ns_loc * q] : 0.0;
  }
  __syncthreads();
  for (int p = t; p < nc * nj; p += 256) {
    const int c = p % nc, jj = p / nc;
    double e = sB[p];
    for (int q = 0; q < nt; ++q) e -= (coh ? load_coherent(Gamma + c + nc * q) : Gamma[c + nc * q]) * sTr[jj + SB * q];
    sE[p] = e;
  }
  __syncthreads();
  const int nA = nc * nc, nB = nc * nt;
  double* out = part + (size_t)bid * (nA + nB);
  for (int p = t; p < nA + nB; p += 256) {
    double acc = 0.0;
    if (p < nA) {
      const int c1 = p % nc, c2 = p / nc;
      for (int jj = 0; jj < nj; ++jj) acc = fma(sE[c1 + nc * jj], sE[c2 + nc * jj], acc);
    } else {
      const int pp = p - nA, c = pp % nc, q = pp / nc;
      for (int jj = 0; jj < nj; ++jj) acc = fma(sB[c + nc * jj], sTr[jj + SB * q], acc);
    }
    out[p] = acc;
  }
}

__global__ __launch_bounds__(256) void gammav_partial_kernel(const double* BL, int K, int nc, int nt, int ns_loc,
                                                             const double* Gamma, const double* Tr,
                                                             double* part) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  gammav_partial_body(BL, K, nc, nt, ns_loc, Gamma, Tr, part, smem, blockIdx.x);
}

// Bartlett draw of MCMCpack::rwish(v, S): W = (Zb CC)^T (Zb CC), CC = chol(S) upper,
// Zb upper-triangular, diag sqrt(chisq(v - i)), off-diagonal N(0,1).
// Sl holds lower L = CC^T (n x n, ld n); result into W; T, Zb scratch n*n each.
__device__ void wg_rwish(const double* Sl, int n, double v, double* W, double* T, double* Zb, Key key,
                         uint32_t s_diag, uint32_t s_off, uint32_t iter, int noise_zero) {
  for (int p = threadIdx.x; p < n * n; p += blockDim.x) {
    const int i = p % n, k = p / n;
    double z = 0.0;
    if (k == i)
      z = sqrt(2.0 * gamma_std(key, (uint32_t)i, s_diag, iter, 0.5 * (v - i)));
    else if (k > i)
      z = noise_zero ? 0.0 : normal(key, (uint32_t)(i + n * k), 0, s_off, iter);
    Zb[p] = z;
  }
  __syncthreads();
  // T = Zb * L^T
  wg_gemm(n, n, n, 1.0, Zb, n, false, Sl, n, true, 0.0, T, n);
  wg_gemm(n, n, n, 1.0, T, n, true, T, n, false, 0.0, W, n);
}

struct GVArgs {
  int nc, nt, ns_glob, nparts;
  const double* iUmG;  // iUGamma %*% mGamma (constant, host precomputed)
  const double* part;  // summed partials (already all-reduced in sharded mode)
  const double* V0;
  double f0;
  const double* iUGamma;
  const double* mGamma;
  const double* TT;
  double* iV;
  double* Gamma;
  double* scratch;
  Key key;
  uint32_t iter;
  const uint32_t* iter_dev;  // graph replay: the sweep counter is read from the device
  int noise_zero;
  int* fail;
  int use_lds;
};

__global__ __launch_bounds__(256) void gammav_final_kernel(GVArgs a) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int nc = a.nc, nt = a.nt, N = nc * nt, t = threadIdx.x;
  __shared__ int flag;
  double* A = a.use_lds ? lds : a.scratch;  // nc*nc
  double* Vn = A + nc * nc;         // nc*nc
  double* W = Vn + nc * nc;         // nc*nc scratch
  double* T = W + nc * nc;          // nc*nc scratch
  double* BTr = T + nc * nc;        // nc*nt
  double* Pm = BTr + nc * nt;       // N*N
  double* rhs = Pm + N * N;         // N
  double* Zb = rhs + N;             // nc*nc
  double* iVl = Zb + nc * nc;       // nc*nc (the new iV, kept on chip)
  const int nA = nc * nc, nB = nc * nt;
  for (int p = t; p < nA + nB; p += blockDim.x) {
    double s = 0.0;
#pragma unroll 8
    for (int b = 0; b < a.nparts; ++b) s += a.part[(size_t)b * (nA + nB) + p];
    if (p < nA)
      A[p] = s + a.V0[p];                        // A + V0   (:19)
    else
      BTr[p - nA] = s;
  }
  __syncthreads();
  if (!wg_chol(A, nc, nc, &flag)) {
    if (t == 0) *a.fail = 1;
  }
  wg_chol2inv(A, nc, nc, Vn, nc, W);             // Vn = chol2inv(chol(A+V0))  (:19)
  wg_copy(A, Vn, nc * nc);
  wg_chol(A, nc, nc, &flag);                      // CC = chol(Vn)
  wg_lower_only(A, nc, nc);
  wg_rwish(A, nc, a.f0 + a.ns_glob, iVl, T, Zb, a.key, S_WISHART_DIAG, S_WISHART_OFF, SWEEP_ITER(a), a.noise_zero);  // (:20)
  for (int p = t; p < nc * nc; p += blockDim.x) a.iV[p] = iVl[p];
  // Gamma | iV: prec = iUGamma + kron(Tr'Tr, iV); rhs = iUGamma mGamma + vec(iV B Tr)   (:29-31)
  for (int p = t; p < N * N; p += blockDim.x) {
    const int r = p % N, c = p / N;
    const int c1 = r % nc, t1 = r / nc, c2 = c % nc, t2 = c / nc;
    Pm[p] = a.iUGamma[p] + a.TT[t1 + nt * t2] * iVl[c1 + nc * c2];
  }
  for (int r = t; r < N; r += blockDim.x) {
    const int c1 = r % nc, t1 = r / nc;
    double v = a.iUmG[r];
    for (int c2 = 0; c2 < nc; ++c2) v += iVl[c1 + nc * c2] * BTr[c2 + nc * t1];
    rhs[r] = v;
  }
  __syncthreads();
  wg_chol(Pm, N, N, &flag);
  wg_forward(Pm, N, N, rhs);
  for (int r = t; r < N; r += blockDim.x)
    rhs[r] += a.noise_zero ? 0.0 : normal(a.key, (uint32_t)r, 0, S_GAMMAV, SWEEP_ITER(a));
  __syncthreads();
  wg_backward_t(Pm, N, N, rhs);
  for (int r = t; r < N; r += blockDim.x) a.Gamma[r] = rhs[r];
}


// ---------------------------------------------------------------------------
// Wave-resident GammaV + Gamma2-prep for N = nc*nt <= 32 (the common case): one workgroup,
// all four waves reduce the species partials into LDS, then wave 0 runs the whole chain
// of small factorisations in registers (wave_la.h), products on the matrix cores.
// Same algebra and the same Philox counters as gammav_final_kernel + gamma2_prep_kernel.
// ---------------------------------------------------------------------------
struct GVWArgs {
  int nc, nt, ns_glob, nparts, do_prep;
  const double* part;  // nparts species partials [A nc^2 | BTr nc nt], ld part_ld (device-coherent loads)
  int part_ld;
  double* Gamma_side;  // copy of the new Gamma for the side stream's record pack, or null
  int* flags;          // side_sync or null: wave 0 raises flags[0] (Gamma, iV), wave 1 flags[prep_flag]
  int prep_flag;
  const double* V0;
  double f0;
  const double* iUGamma;
  const double* iUmG;
  const double* TT;
  double* iV;
  double* Gamma;
  // Gamma2 prep constants / output
  const double* XX;
  const double* iV0;
  double* prep;      // Gamma2 prep [B1 nc^2 | LS N^2]
  Key key;
  uint32_t iter;
  const uint32_t* iter_dev;  // graph replay: the sweep counter is read from the device
  int noise_zero;
  int* fail;
};

// out(r, c) = alpha * (I_nt (x) Ablk)(r, c) + (TT (x) Bblk)(r, c) + C(r, c), padded with I.
// Ablk / Bblk: nc x nc column-major with leading dims lda / ldb, C: N x N or null.
template <int NM>
__device__ inline void wv_kron(double (&o)[NM], int nc, int nt, const double* TT, double alpha, const double* Ablk,
                               int lda, const double* Bblk, int ldb, const double* C) {
  const int i = lane_id(), N = nc * nt;
  const int ir = i < N ? i : 0;
  const int c1 = ir % nc, t1 = ir / nc;
  int c2 = 0, t2 = 0;
#pragma unroll
  for (int c = 0; c < NM; ++c) {
    double v = (i == c) ? 1.0 : 0.0;
    if (c < N) {
      double e = TT[t1 + nt * t2] * Bblk[c1 + ldb * c2];
      if (Ablk && t1 == t2) e += alpha * Ablk[c1 + lda * c2];
      if (C) e += C[ir + (size_t)N * c];
      if (i < N) v = e;
      if (++c2 == nc) {
        c2 = 0;
        ++t2;
      }
    }
    o[c] = v;
  }
}

// Phases (one workgroup of 4 waves; block-wide barriers only between phases):
//   A  all waves: reduce the species partials, draw the Bartlett factor;
//   B  wave 0: Vn and iV.  R_S = chol(Vn) (upper) comes from one factorization: with J the
//      exchange matrix, chol(J (A + V0) J) = M M^T gives A + V0 = (J M J)(J M J)^T and hence
//      R_S = J M^-1 J -- the same matrix R's chol(chol2inv(chol(A + V0))) forms, up to
//      rounding, with one factorization and one triangular inverse instead of two and a
//      product;
//   C  wave 0: Gamma | iV;  wave 1 (concurrently): Gamma2's iV-only prep.
template <int NM>
__device__ __forceinline__ void gammav_body(const GVWArgs& a) {
  // S: 3 scratch tiles for products (wave 1 in phase C); SG: wave 0's scratch in phase C;
  // T0..T3: named tiles (sA aliases T0 during the reduction)
  __shared__ __attribute__((aligned(16))) double S[3 * WV_TILE];
  __shared__ __attribute__((aligned(16))) double SG[WV_TILE];
  __shared__ __attribute__((aligned(16))) double T0[WV_TILE], T1[WV_TILE], T2[WV_TILE], T3[WV_TILE];
  __shared__ __attribute__((aligned(16))) double sXX[WV_TILE];  // X'X for wave 1 (ld WV_LD)
  __shared__ double sBTr[32];
  // the constants the serial phases read (kron factors, prior terms), staged by all waves in
  // phase A so that no global-memory latency sits inside the factorisation chains
  __shared__ double sTT[NM * NM], sIV0[NM * NM], sIUG[NM * NM], sIUmG[NM];  // nt, nc <= N <= NM
  __shared__ int sok;
  double* sA = T0;
  const int nc = a.nc, nt = a.nt, N = nc * nt, t = threadIdx.x, w = t >> 6;
  const int nA = nc * nc, nB = nc * nt;
  HMSC_STAMP(0);
  if (t == 0) sok = 1;
  // the constants' loads all issued first and stored after the partial sums' loads below (a
  // staging loop with a store per iteration waits out one memory latency per iteration:
  // five arrays were ~8 round trips before the first partial load).  nc^2, N^2 <= 1024.
  double cXX[4], cIUG[4], cIV0[4], cTT, cIUmG;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int p = t + 256 * u;
    cXX[u] = p < nA ? a.XX[p] : 0.0;
    cIUG[u] = p < N * N ? a.iUGamma[p] : 0.0;
    cIV0[u] = (a.do_prep && p < nA) ? a.iV0[p] : 0.0;
  }
  cTT = t < nt * nt ? a.TT[t] : 0.0;
  cIUmG = t < N ? a.iUmG[t] : 0.0;
  for (int p = t; p < nA + nB; p += blockDim.x) {
    // species-block partials in block order, 32 loads in flight (one L2 round trip per 32)
    const double v0 = p < nA ? a.V0[p] : 0.0;
    const double* src = a.part + p;
    const size_t st = (size_t)a.part_ld;
    double sum = 0.0;
    int b = 0;
    // (device-coherent loads: the partials may come from another launch still running on
    // another XCD -- the fused BetaLambda tail -- published by a flag, not a kernel boundary)
    for (; b + 32 <= a.nparts; b += 32) {
      double x[32];
#pragma unroll
      for (int u = 0; u < 32; ++u) x[u] = load_coherent(src + st * (b + u));
#pragma unroll
      for (int u = 0; u < 32; ++u) sum += x[u];
    }
    for (; b + 8 <= a.nparts; b += 8) {
      double x[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) x[u] = load_coherent(src + st * (b + u));
#pragma unroll
      for (int u = 0; u < 8; ++u) sum += x[u];
    }
    for (; b < a.nparts; ++b) sum += load_coherent(src + st * b);
    if (p < nA)
      sA[p] = sum + v0;       // E E^T + V0   (R/updateGammaV.R:18-19)
    else
      sBTr[p - nA] = sum;     // B Tr
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int p = t + 256 * u;
    if (p < nA) sXX[p % nc + WV_LD * (p / nc)] = cXX[u];
    if (p < N * N) sIUG[p] = cIUG[u];
    if (a.do_prep && p < nA) sIV0[p] = cIV0[u];
  }
  if (t < nt * nt) sTT[t] = cTT;
  if (t < N) sIUmG[t] = cIUmG;
  // Bartlett factor Zb of rwish (MCMCpack: diag sqrt(chisq(v - i)), upper N(0,1)), drawn by
  // all 256 threads at once: T3 = Zb padded with I to 32 x 32
  {
    const double v = a.f0 + a.ns_glob;
    for (int p = t; p < 32 * 32; p += blockDim.x) {
      const int ii = p & 31, k = p >> 5;
      double zz = (ii == k && ii < NM) ? 1.0 : 0.0;
      if (ii < nc && k < nc) {
        if (k == ii)
          zz = sqrt(2.0 * gamma_std(a.key, (uint32_t)ii, S_WISHART_DIAG, SWEEP_ITER(a), 0.5 * (v - ii)));
        else if (k > ii)
          zz = a.noise_zero ? 0.0 : normal(a.key, (uint32_t)(ii + nc * k), 0, S_WISHART_OFF, SWEEP_ITER(a));
        else
          zz = 0.0;
      }
      T3[ii + WV_LD * k] = zz;
    }
  }
  __syncthreads();
  HMSC_STAMP(1);
  if (w >= 2 || (w == 1 && !a.do_prep)) return;
  const int i = lane_id();
  double x[NM], y[NM], z[NM], dinv;
  if (w == 0) {
    bool ok = true;
    wv_load_rev<NM>(sA, nc, nc, x);                     // J (A + V0) J
    ok &= wv_chol<NM>(x, dinv);                         // = M M^T
    wv_inv_lower<NM>(x, dinv, y);                       // M^-1
    HMSC_STAMP(2);
    wv_to_lds_rev<NM>(y, nc, S);                        // R_S = J M^-1 J = chol(Vn)
    // iV = rwish(f0 + ns, Vn) by Bartlett: iV = (Zb R_S)^T (Zb R_S)
    wv_mm_lds<NM>(T3, S, x, S + WV_TILE);               // x = T = Zb R_S
    wv_gemm<NM, true, false>(x, x, z, S);               // z = iV = T^T T
    wv_store<NM>(a.iV, nc, nc, z);
    wv_to_lds<NM>(z, T1);                               // T1 = iV
    if (!ok && i == 0) sok = 0;
    HMSC_STAMP(3);
  }
  __syncthreads();
  if (w == 0) {
    // Gamma | iV: prec = iUGamma + kron(TT, iV), rhs = iUGamma mGamma + vec(iV B Tr)   (:29-31)
    bool ok = sok != 0;
    wv_kron<NM>(x, nc, nt, sTT, 0.0, nullptr, 0, T1, WV_LD, sIUG);
    double r = 0.0;
    if (i < N) {
      const int c1 = i % nc, t1 = i / nc;
      r = sIUmG[i];
      for (int c2 = 0; c2 < nc; ++c2) r += T1[c1 + WV_LD * c2] * sBTr[c2 + nc * t1];
    }
    ok &= wv_chol<NM>(x, dinv);
    wv_forward<NM>(x, dinv, r);
    if (i < N && !a.noise_zero) r += normal(a.key, (uint32_t)i, 0, S_GAMMAV, SWEEP_ITER(a));
    wv_transpose<NM, true>(x, y, SG);
    wv_backward_t<NM>(y, dinv, r);
    if (i < N) a.Gamma[i] = r;
    if (i < N && a.Gamma_side) a.Gamma_side[i] = r;
    HMSC_STAMP(4);
    if (!ok && i == 0) a.fail[0] = 1;
    if (a.flags) {  // Gamma and iV are out (the next sweep's fused launch waits on this)
      HMSC_STAMP_RT(83);
      __threadfence();
      if (i == 0) __hip_atomic_store(&a.flags[0], g2bl_epoch(SWEEP_ITER(a)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return;
  }

  // ---- wave 1: Gamma2 prep (algebra as in gamma2_prep_kernel) ----
  HMSC_STAMP_W(10);
  wv_from_lds<NM>(T1, z);                               // z = iV
  bool ok2 = true;
  // iP = inv(iV + XX)
  wv_load<NM>(sXX, WV_LD, nc, x);
#pragma unroll
  for (int k = 0; k < NM; ++k) x[k] = (i < nc && k < nc) ? x[k] + z[k] : x[k];
  ok2 &= wv_chol<NM>(x, dinv);
  wv_chol2inv<NM>(x, dinv, y, S);                       // y = iP
  wv_to_lds<NM>(y, T2);                                 // T2 = iP
  HMSC_STAMP_W(11);
  wv_mm_rt<NM>(z, T2, x, S);                            // x = B1 = iV iP
  wv_store<NM>(a.prep, nc, nc, x);
  wv_load<NM>(sXX, WV_LD, nc, y);
  wv_gemm<NM, false, true>(y, x, z, S);                 // z = M = XX iP iV = XX B1^T
  wv_to_lds<NM>(z, T3);                                 // T3 = M
  wv_sync();
  wv_kron<NM>(x, nc, nt, sTT, 1.0, sIV0, nc, T3, WV_LD, nullptr);  // Pg = I (x) iV0 + TT (x) M
  wv_pad<NM>(x, N, 1.0);
  wv_to_lds<NM>(x, T0);
  wv_sync();
  HMSC_STAMP_W(12);
  wv_load_rev<NM>(T0, WV_LD, N, x);                     // J Pg J
  ok2 &= wv_chol<NM>(x, dinv);                          // = Mc Mc^T
  wv_inv_lower<NM>(x, dinv, y);                         // Mc^-1 by rows
  HMSC_STAMP_W(13);
  // LS = J Mc^-T J: element (i, k) of Mc^-1 (lane i, k <= i) is LS[N-1-k][N-1-i]
  double* LS = a.prep + nA;
  if (i < N)
#pragma unroll
    for (int k = 0; k < NM; ++k)
      if (k < N) LS[(N - 1 - k) + (size_t)N * (N - 1 - i)] = (k <= i) ? y[k] : 0.0;
  if (!ok2 && i == 0) a.fail[1] = 1;
  HMSC_STAMP_W(14);
  if (a.flags) {  // Gamma2's prep is out
    __threadfence();
    if (i == 0) __hip_atomic_store(&a.flags[a.prep_flag], g2bl_epoch(SWEEP_ITER(a)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

template <int NM>
__global__ __launch_bounds__(256) void gammav_wave_kernel(GVWArgs a) {
  gammav_body<NM>(a);
}

static GVWArgs make_gvw_args(State& s, uint32_t iter, const double* part, int np, const uint32_t* iter_dev) {
  GVWArgs w{};
  w.nc = s.nc;
  w.nt = s.nt;
  w.ns_glob = s.ns;
  w.nparts = np;
  w.do_prep = (s.mask & HMSC_UP_GAMMA2) ? 1 : 0;
  w.part = part;
  w.part_ld = s.nc * s.nc + s.nc * s.nt;
  w.Gamma_side = s.Gamma_side;
  w.flags = nullptr;
  w.prep_flag = 1 + s.nr;
  w.V0 = s.V0;
  w.f0 = s.f0;
  w.iUGamma = s.iUGamma;
  w.iUmG = s.iUmG;
  w.TT = s.phylo ? s.phTTw : s.TT;  // Tr^T iQ Tr with phylogeny (R/updateGammaV.R:29)
  w.iV = s.iV;
  w.Gamma = s.Gamma;
  w.XX = s.XX;
  w.iV0 = s.iV0;
  w.prep = s.g2prep;
  w.key = s.key;
  w.iter = iter;
  w.iter_dev = iter_dev;
  w.noise_zero = s.noise_mode;
  w.fail = s.dev_flags;
  return w;
}

static void launch_gammav_wave(State& s, uint32_t iter, hipStream_t st, const double* part, int np,
                               const uint32_t* iter_dev) {
  const GVWArgs w = make_gvw_args(s, iter, part, np, iter_dev);
  switch (wv_bucket_gv(s.nc * s.nt)) {
    case 8: gammav_wave_kernel<8><<<1, 256, 0, st>>>(w); break;
    case 16: gammav_wave_kernel<16><<<1, 256, 0, st>>>(w); break;
    case 20: gammav_wave_kernel<20><<<1, 256, 0, st>>>(w); break;
    case 24: gammav_wave_kernel<24><<<1, 256, 0, st>>>(w); break;
    default: gammav_wave_kernel<32><<<1, 256, 0, st>>>(w); break;
  }
  HIP_OK(hipGetLastError());
  if (w.do_prep) s.g2prep_valid = true;
}


void launch_gamma_v(State& s, uint32_t iter, hipStream_t st) {
  const int nparts = (s.nsl + SB - 1) / SB;
  double* part = s.ABpart;
  int np = nparts;
  if (s.phylo) {  // E iQ E^T, B iQ Tr, Tr^T iQ Tr in the eigenbasis of C (phylo.hip)
    launch_phylo_gv_sums(s, iter, st);
    np = 1;
  } else {
    gammav_partial_kernel<<<nparts, 256, (size_t)(2 * s.nc * SB + SB * s.nt) * sizeof(double), st>>>(
        s.BL, s.K, s.nc, s.nt, s.nsl, s.Gamma, s.Tr, part);
    HIP_OK(hipGetLastError());
  }
  const int Ng = s.nc * s.nt;
  if (Ng <= 32) {
    launch_gammav_wave(s, iter, st, part, np, s.capturing ? s.d_iter : nullptr);
    return;
  }
  GVArgs a{};
  a.nc = s.nc;
  a.nt = s.nt;
  a.ns_glob = s.ns;
  a.nparts = np;
  a.part = part;
  a.V0 = s.V0;
  a.f0 = s.f0;
  a.iUGamma = s.iUGamma;
  a.mGamma = s.mGamma;
  a.iUmG = s.iUmG;
  a.TT = s.phylo ? s.phTTw : s.TT;
  a.iV = s.iV;
  a.Gamma = s.Gamma;
  a.scratch = s.scratch;
  a.key = s.key;
  a.iter = iter;
  a.iter_dev = s.capturing ? s.d_iter : nullptr;
  a.noise_zero = s.noise_mode;
  a.fail = s.dev_flags;
  const size_t need = (6 * (size_t)s.nc * s.nc + (size_t)s.nc * s.nt + (size_t)s.nc * s.nt * s.nc * s.nt +
                       (size_t)s.nc * s.nt) * sizeof(double);
  a.use_lds = need <= 64 * 1024;
  HMSC_REQUIRE(a.use_lds || need <= s.scratch_doubles * sizeof(double), "internal: GammaV scratch too small");
  gammav_final_kernel<<<1, 64, a.use_lds ? need : 0, st>>>(a);
  HIP_OK(hipGetLastError());
  if (s.mask & HMSC_UP_GAMMA2) launch_gamma2_prep(s, st);  // Gamma2's iV-only algebra for the next sweep
}

// ---------------------------------------------------------------------------
// updateGamma2 (R/updateGamma2.R:6-60): Gamma with Beta integrated out.
// Stage 1 (species-parallel): XZT = X^T S Tr with S = Z - sum_r LRan_r, via
//   X^T Z Tr = XZ[0:nc,:] Tr (no NA)  and  X^T Eta_r[Pi] (Lambda_r Tr)  from G.
// Stage 2: single-workgroup dense algebra.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void gamma2_partial_body(const XZSrc& XZ, const double* BL, int K, int nc, int NF, int nt,
                                                    int ns_loc, const double* Tr, double* part, double* smem, int bid,
                                                    bool coherent = false) {
  // part[b] = [ XZ[0:nc, block] Tr (nc*nt) | Lambda_all[:, block] Tr (NF*nt) ]
  double* sX = smem;             // K x G2SB: rows < nc from XZ, rows >= nc from BL (Lambda)
  double* sTr = sX + K * G2SB;     // G2SB x nt
  const int t = threadIdx.x, j0 = bid * G2SB, nj = min(G2SB, ns_loc - j0);
  if (XZ.part) {
    // rows < nc from updateZ's chunk partials (the fused launch; LDS for the stripe sums):
    // task (element e of the nc x nj block, stripe w) sums partials w, w + 4, ... in order
    // (slab_sum_body's), four tasks' loads in flight per thread; the stripes then meet as
    // (s0 + s1) + (s2 + s3), the reduced buffer's bits
    double* sS = sTr + G2SB * nt;  // [stripe][e] (task w ne + e: neighbouring threads, neighbouring rows)
    const int ne = nc * nj, ntask = 4 * ne, n = XZ.nparts;
    for (int q0 = 0; q0 < ntask; q0 += 256 * 4) {
      double acc[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) acc[u] = 0.0;
      for (int cb = 0; cb < n; cb += 48) {  // (one round at the z launch's 48 chunks)
        double x[4][12];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int task = q0 + t + 256 * u, e = task % ne, w = task / ne, k = e % nc, jj = e / nc;
          const double* src = XZ.part + k + (size_t)K * (j0 + jj);
#pragma unroll
          for (int v = 0; v < 12; ++v) {
            const int c = cb + w + 4 * v;
            x[u][v] = task < ntask ? src[(int64_t)min(c, n - 1) * XZ.stride] : 0.0;
          }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int w = (q0 + t + 256 * u) / ne;
#pragma unroll
          for (int v = 0; v < 12; ++v)
            if (cb + w + 4 * v < n) acc[u] += x[u][v];
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int task = q0 + t + 256 * u;
        if (task < ntask) sS[task] = acc[u];
      }
    }
    __syncthreads();
    for (int e = t; e < ne; e += 256) {
      const int k = e % nc, jj = e / nc;
      sX[k + K * jj] = (sS[e] + sS[ne + e]) + (sS[2 * ne + e] + sS[3 * ne + e]);
    }
    for (int p = t; p < K * nj; p += 256) {
      const int k = p % K, jj = p / K;
      if (k >= nc) sX[p] = BL[k + (size_t)K * (j0 + jj)];
    }
  } else {
    for (int p = t; p < K * nj; p += 256) {
      const int k = p % K, jj = p / K;
      const size_t g = k + (size_t)K * (j0 + jj);
      sX[p] = k < nc ? XZ.XZ[g] : BL[g];
    }
  }
  for (int p = t; p < G2SB * nt; p += 256) {
    const int jj = p % G2SB, q = p / G2SB;
    sTr[p] = jj < nj ? Tr[j0 + jj + (size_t)ns_loc * q] : 0.0;
  }
  __syncthreads();
  const int n1 = nc * nt, n2 = NF * nt;
  double* out = part + (size_t)bid * (n1 + n2);
  for (int p = t; p < n1 + n2; p += 256) {
    int k, q;
    if (p < n1) {
      k = p % nc;
      q = p / nc;
    } else {
      k = nc + (p - n1) % NF;
      q = (p - n1) / NF;
    }
    double acc = 0.0;
#pragma unroll 8
    for (int jj = 0; jj < nj; ++jj) acc = fma(sX[k + K * jj], sTr[jj + G2SB * q], acc);
    if (coherent)
      store_coherent(out + p, acc);
    else
      out[p] = acc;
  }
}

__global__ __launch_bounds__(256) void gamma2_partial_kernel(XZSrc XZ, const double* BL, int K, int nc,
                                                             int NF, int nt, int ns_loc, const double* Tr,
                                                             double* part) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  gamma2_partial_body(XZ, BL, K, nc, NF, nt, ns_loc, Tr, part, smem, blockIdx.x);
}

// X^T ZTr (nc x nt) for models with NA (where XZ is masked): reduction over sites
__global__ __launch_bounds__(256) void xt_ztr_kernel(const double* X, const double* ZTr, int ny, int nc, int nt,
                                                     double* out) {
  __shared__ double red[256];
  const int p = blockIdx.x, c = p % nc, q = p / nc;
  double s = 0.0;
  for (int i = threadIdx.x; i < ny; i += 256) s += X[i + (size_t)ny * c] * ZTr[i + (size_t)ny * q];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[p] = red[0];
}

// Gamma2 splits into the part that depends only on iV (prep; runs on the side stream right
// after updateGammaV of the previous sweep, overlapped with updateEta / updateZ) and the part
// that needs the new Z (final).  R (R/updateGamma2.R:40-54) forms the posterior covariance
// SigmaG of Gamma (B integrated out) and its mean muG through Rm = (I (x) iV0 + TT (x) (iV -
// iV iP iV))^-1, iP = (iV + X'X)^-1.  With M = X'X iP iV (= iV - iV iP iV, symmetric) and
// B1 = iV iP the same two quantities are
//   SigmaG = Pg^-1,  Pg = I (x) iV0 + TT (x) M   (Woodbury on R's expression),
//   muG    = Pg^-1 vec(B1 XZT)                    (XZT - X'X iP XZT = B1 XZT),
// so the prep keeps B1 and LS = chol(SigmaG) (lower; unique, hence R's LSigmaG), and the final
// stage draws Gamma = muG + LS xi = LS (LS^T vec(B1 XZT) + xi) -- two triangular products.
// LS without forming SigmaG: chol(J Pg J) = Mc Mc^T (J the exchange matrix) gives
// Pg = (J Mc J)(J Mc J)^T and LS = J Mc^-T J.
struct G2PrepArgs {
  int nc, nt;
  const double* iV;
  const double* XX;
  const double* TT;
  const double* iV0;
  double* prep;      // [B1 nc^2 | LS N^2]
  double* scratch;
  int use_lds;
  int* fail;
};

__global__ __launch_bounds__(256) void gamma2_prep_kernel(G2PrepArgs a) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int nc = a.nc, nt = a.nt, N = nc * nt, t = threadIdx.x, n2 = nc * nc;
  __shared__ int flag;
  double* iV = a.use_lds ? lds : a.scratch;  // nc^2
  double* XX = iV + n2;
  double* W = XX + n2;
  double* iP = W + n2;
  double* B1 = iP + n2;
  double* M = B1 + n2;
  double* T1 = M + n2;
  double* Pg = T1 + n2;      // N^2
  double* Sg = Pg + N * N;   // N^2
  double* Tn = Sg + N * N;   // N^2 scratch
  for (int p = t; p < n2; p += blockDim.x) {
    iV[p] = a.iV[p];
    XX[p] = a.XX[p];
    W[p] = a.iV[p] + a.XX[p];
  }
  __syncthreads();
  if (!wg_chol(W, nc, nc, &flag) && t == 0) *a.fail = 1;
  wg_chol2inv(W, nc, nc, iP, nc, T1);                                      // iP = inv(iV + XX)
  wg_gemm(nc, nc, nc, 1.0, iV, nc, false, iP, nc, false, 0.0, B1, nc);     // B1 = iV iP
  wg_gemm(nc, nc, nc, 1.0, XX, nc, false, B1, nc, true, 0.0, M, nc);       // M = XX iP iV
  for (int p = t; p < N * N; p += blockDim.x) {
    const int r = p % N, c = p / N, c1 = r % nc, q1 = r / nc, c2 = c % nc, q2 = c / nc;
    Pg[p] = (q1 == q2 ? a.iV0[c1 + nc * c2] : 0.0) + a.TT[q1 + nt * q2] * M[c1 + nc * c2];
  }
  __syncthreads();
  if (!wg_chol(Pg, N, N, &flag) && t == 0) *a.fail = 1;
  wg_chol2inv(Pg, N, N, Sg, N, Tn);                                        // SigmaG = Pg^-1
  if (!wg_chol(Sg, N, N, &flag) && t == 0) *a.fail = 1;                    // LSigmaG   (:52)
  double* out = a.prep;
  for (int p = t; p < n2; p += blockDim.x) out[p] = B1[p];
  for (int p = t; p < N * N; p += blockDim.x) out[n2 + p] = (p % N >= p / N) ? Sg[p] : 0.0;
}

struct G2Args {
  int nc, nt, Kmax, NF, nparts, ns_loc, use_xtztr, check_isigma, stage;
  int coherent;       // partials written by other workgroups of the same launch
  int prep_coherent;  // the prep written by another queue's launch, behind a flag polled in this one
  const double* isig_count;  // sharded chain: all-reduced count of species with iSigma != 1
  const double* part;
  const double* xtztr;
  const double* G;
  const double* prep;
  const double* iSigma;
  double* Gamma;
  Key key;
  uint32_t iter;
  const uint32_t* iter_dev;  // graph replay: the sweep counter is read from the device
  int noise_zero;
  // the final stage's working arrays (G2FLds): lay_dyn == 0 is the fixed layout below (the fused
  // launches, N + NF nt <= 64); otherwise offsets sized for this nc, nt, NF (g2f_layout), in LDS
  // or, when they do not fit a workgroup's LDS, at gbase in global memory
  int lay_ltr, lay_v1, lay_v2, lay_xi, lay_red, lay_sgl, lay_dyn;
  double* gbase;
};

// for (p = threadIdx.x; p < n; p += blockDim.x) store(p, load(p)) with U loads of a thread in
// flight before its stores (a loop with a store per iteration waits one latency per iteration)
template <int U, class Load, class Store>
__device__ __forceinline__ void batched_for(int n, Load load, Store store) {
  const int nt = blockDim.x;
  for (int p0 = threadIdx.x; p0 < n; p0 += U * nt) {
    double v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = load(min(p0 + u * nt, n - 1));  // (clamped, unconditional)
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (p0 + u * nt < n) store(p0 + u * nt, v[u]);
  }
}

// LDS of the final stage (doubles) in the fixed layout, before the staged B1 | LS (n2 + N^2 more
// when a.stage)
constexpr int G2F_LDS = 512 + 512 + 3 * 256 + 8 * 64 + 2048;

struct G2FLds {
  double *S0, *LTr, *v1, *v2, *xi, *sGL, *dyn;
  double (*red)[64];
  __device__ G2FLds(double* lds, const G2Args& a) {
    if (a.gbase) lds = a.gbase;
    const bool fixed = a.lay_dyn == 0;
    S0 = lds;
    LTr = lds + (fixed ? 512 : a.lay_ltr);
    v1 = lds + (fixed ? 1024 : a.lay_v1);
    v2 = lds + (fixed ? 1280 : a.lay_v2);
    xi = lds + (fixed ? 1536 : a.lay_xi);
    red = (double (*)[64])(lds + (fixed ? 1792 : a.lay_red));
    sGL = lds + (fixed ? 1792 + 8 * 64 : a.lay_sgl);
    dyn = lds + (fixed ? 1792 + 8 * 64 + 2048 : a.lay_dyn);
  }
};

// The final stage in two phases.  gamma2_final_pre: what no flag guards -- iSigma's all-ones
// test (:36), G's X^T Eta block, the noise -- so that the fused launch's workgroup 0 issues it
// while it waits for the partials and the side chain's flags; returns this thread's vote of the
// all-ones test (the caller's barrier ANDs them).  Everything is staged into LDS by all 256
// threads (coalesced, every load of a thread issued before its first use).
__device__ __forceinline__ int gamma2_final_pre(const G2Args& a, double* lds) {
  const G2FLds L(lds, a);
  const int nc = a.nc, N = nc * a.nt, t = threadIdx.x;
  int ok = 1;
  if (a.check_isigma)
    batched_for<8>(a.ns_loc, [&](int j) { return a.iSigma[j]; }, [&](int, double v) {
      if (v != 1.0) ok = 0;
    });
  if (t == 0 && a.isig_count && *a.isig_count != 0.0) ok = 0;  // ... over every rank's species
  if (nc * a.NF <= 2048)  // X^T Eta block of G, read by the XZT products
    batched_for<8>(nc * a.NF, [&](int p) { return a.G[p % nc + (size_t)a.Kmax * (nc + p / nc)]; },
                   [&](int p, double v) { L.sGL[p] = v; });
  for (int r = t; r < N; r += blockDim.x) L.xi[r] = a.noise_zero ? 0.0 : normal(a.key, (uint32_t)r, 0, S_GAMMA2, SWEEP_ITER(a));
  return ok;
}

// gamma2_final_main: after the barrier that follows the pre phase (and the flags): the prep
// matrices and the species-block partials (their loads issued together), then the products.
__device__ __forceinline__ void gamma2_final_main(const G2Args& a, double* lds) {
  const G2FLds L(lds, a);
  HMSC_STAMP(30);
  const int nc = a.nc, nt = a.nt, N = nc * nt, t = threadIdx.x, n2 = nc * nc;
  const int n1 = nc * nt, nL = a.NF * nt, P = n1 + nL;
  const double *B1 = a.prep, *LS = a.prep + n2;
  const bool grouped = P <= 64 && a.nparts > 1;
  // species-block partials: 8 groups of 32 threads, each summing every 8th part in order; up to
  // 64 parts every load of a thread is issued before the prep staging's (one latency for both)
  const int g = t >> 5, l = t & 31;
  double x[2][16];
  const bool direct = grouped && a.nparts <= 128;
  if (direct)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int p = min(32 * h + l, P - 1);
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const double* q = a.part + (size_t)min(g + 8 * u, a.nparts - 1) * P + p;
        x[h][u] = a.coherent ? load_coherent(q) : *q;  // (clamped address, unconditional)
      }
    }
  if (a.stage) {
    double* d = L.dyn;
    batched_for<8>(n2 + N * N, [&](int p) { return a.prep_coherent ? load_coherent(a.prep + p) : a.prep[p]; },
                   [&](int p, double v) { d[p] = v; });
    B1 = d;
    LS = d + n2;
  }
  if (grouped) {
    for (int p0 = 0; p0 < P; p0 += 32) {
      const int p = p0 + l;
      double s = 0.0;
      if (p < P) {
        if (direct) {
#pragma unroll
          for (int u = 0; u < 16; ++u)
            if (g + 8 * u < a.nparts) s += x[p0 ? 1 : 0][u];
        } else {
          for (int b = g; b < a.nparts; b += 64) {  // eight loads in flight per step, summed in order
            double y[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
              const double* q = a.part + (size_t)min(b + 8 * u, a.nparts - 1) * P + p;
              y[u] = a.coherent ? load_coherent(q) : *q;
            }
#pragma unroll
            for (int u = 0; u < 8; ++u)
              if (b + 8 * u < a.nparts) s += y[u];
          }
        }
      }
      L.red[g][l + (p0 ? 32 : 0)] = s;
    }
    __syncthreads();
    for (int p = t; p < P; p += blockDim.x) {
      double s = 0.0;
#pragma unroll
      for (int g2 = 0; g2 < 8; ++g2) s += L.red[g2][p];
      if (p < n1)
        L.S0[p] = a.use_xtztr ? a.xtztr[p] : s;
      else
        L.LTr[p - n1] = s;
    }
  } else {
    for (int p = t; p < P; p += blockDim.x) {
      double s = 0.0;
#pragma unroll 8
      for (int b = 0; b < a.nparts; ++b) s += a.coherent ? load_coherent(a.part + (size_t)b * P + p) : a.part[(size_t)b * P + p];
      if (p < n1)
        L.S0[p] = a.use_xtztr ? a.xtztr[p] : s;
      else
        L.LTr[p - n1] = s;
    }
  }
  const bool stage_g = nc * a.NF <= 2048;
  __syncthreads();
  HMSC_STAMP(31);
  // (the products' LDS operands unrolled eight deep, so their loads issue ahead of the
  // accumulation chain; the accumulation order is unchanged)
  // XZT = X^T Z Tr - sum_r (X^T Eta_r[Pi]) (Lambda_r Tr)   (:46 with S = Z - sum LRan)
  for (int p = t; p < n1; p += blockDim.x) {
    const int c = p % nc, q = p / nc;
    double s = 0.0;
    if (stage_g) {
#pragma unroll 8
      for (int f = 0; f < a.NF; ++f) s += L.sGL[c + nc * f] * L.LTr[f + a.NF * q];
    } else {
      for (int f = 0; f < a.NF; ++f) s += a.G[c + a.Kmax * (nc + f)] * L.LTr[f + a.NF * q];
    }
    L.S0[p] -= s;
  }
  __syncthreads();
  // r = vec(B1 XZT); u = LS^T r + xi; Gamma = LS u = muG + LS xi   (:49, :53-54)
  for (int p = t; p < N; p += blockDim.x) {
    const int c = p % nc, q = p / nc;
    double s2 = 0.0;
#pragma unroll 8
    for (int k = 0; k < nc; ++k) s2 += B1[c + nc * k] * L.S0[k + nc * q];
    L.v2[p] = s2;
  }
  __syncthreads();
  for (int r = t; r < N; r += blockDim.x) {
    double u = L.xi[r];
#pragma unroll 8
    for (int c = r; c < N; ++c) u = fma(LS[c + N * r], L.v2[c], u);
    L.v1[r] = u;
  }
  __syncthreads();
  for (int r = t; r < N; r += blockDim.x) {
    double gm = 0.0;
#pragma unroll 8
    for (int c = 0; c <= r; ++c) gm = fma(LS[r + N * c], L.v1[c], gm);
    a.Gamma[r] = gm;
  }
  HMSC_STAMP(32);
}

__global__ __launch_bounds__(256) void gamma2_final_kernel(G2Args a) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int ok = gamma2_final_pre(a, smem);
  if (!__syncthreads_and(ok)) return;  // acts only if all(iSigma == 1)  (:36)
  gamma2_final_main(a, smem);
}

// ---------------------------------------------------------------------------
// updateGamma2 + updateBetaLambda in one launch (R/sampleMcmc.R:221-229 runs them back to
// back; BetaLambda's precision iU and its Cholesky factor do not depend on the Gamma that
// Gamma2 draws, only its mean does).  Workgroups 1 .. nbl run the wave BetaLambda body (four
// species each, one per wave), which factors iU while Gamma2 runs and waits for Gamma only
// for the mean and the solves; nparts further workgroups after them (G2SB species each) form
// Gamma2's species-block partials (device-coherent stores, a relaxed count in sync[0]).
// Workgroup 0 waits for the count, reduces the partials in block order, runs the final stage
// and publishes Gamma (sync[1]).  (Round 4 put the partials ahead of the first BetaLambda
// bodies to keep the launch at one workgroup per CU; those bodies then ended ~3 us after the
// rest, and the trailing partial workgroups measured faster, HMSC_G2_PART_INLINE restores
// it.)  Every workgroup of the launch is resident at once (two per CU: 52 KB of LDS and
// __launch_bounds__(256, 2)), and workgroup 0 is dispatched before the ones it waits for.
// Workgroup 0 resets the count; the flag holds the sweep's epoch (g2bl_epoch), reset to 0 by
// the host at the start of every run and before every eager launch, so it never needs a reset
// inside the launch.
// ---------------------------------------------------------------------------
// ---------------------------------------------------------------------------
// The fused Eta kernel's per-sweep constants (kernels.hip eta_fused_kernel, R/updateEta.R
// :53-56 for one unstructured level):
//   CR = BL diag(iSigma) Lambda^T   (K x nf; rows nc.. are Q - I, Q = I + Lambda diag(iSigma) Lambda^T)
//   W  = L^-1, L L^T = Q            (16 x 16, row m at 16 m, zero padded)
//   LS = Lambda diag(iSigma)        ([species][16], the Eta stream's MFMA B operand)
// formed either in the tail of the fused Gamma2 + BetaLambda launch (crw_tail, where each
// species' new column is still in registers) or, on the other paths, by crw_kernel.
// ---------------------------------------------------------------------------
constexpr int CRW_PARTS = 4;    // crw_kernel's workgroups
constexpr int CRW_GROUP = 16;   // crw_tail: BetaLambda workgroups summed by one group reducer
constexpr int CRW_TILE = 520;   // bl_tail partial tile: [h < 16][k < 32], then 2 timing words
struct CRWArgs {
  const double* BL;
  const double* iSigma;
  int K, nc, nf, ns, ldcr;
  double* CR;
  double* W;
  double* LS;
  double* part;  // crw_kernel: CRW_PARTS x (4 x 256); crw_tail: (nbl + ngroups) x CRW_TILE
  int* ticket;   // [crw_kernel, crw_tail's groups, crw_tail's group tickets ...]; zero between
                 // launches, each reset by the workgroup that takes its last value
};

// Q = I + (rows nc.. of CR) -> its Cholesky factor and W = L^-1 by rows, on one wave;
// sCR is CR in LDS as [row][16], scratch >= 16 x 17 doubles.
// qm[r * ld + c] = (Q - I)[r][c] (r, c < nf): W[m * wld + c] = row m of L^-1, L L^T = Q, for
// m, c < wn (zero past nf and above the diagonal); one wave, scratch >= NFB (NFB + 1) doubles
template <int NFB>
__device__ __forceinline__ void q_inv_factor(const double* qm, int ld, int nf, double* W, int wld, int wn,
                                             double* scratch) {
  const int lane = lane_id();
  double qv[NFB], dinv;
  const int r = lane < nf ? lane : 0;
#pragma unroll
  for (int c = 0; c < NFB; ++c) {
    const double v = (r == c ? 1.0 : 0.0) + qm[r * ld + (c < nf ? c : 0)];
    qv[c] = (lane < nf && c < nf) ? v : (lane == c ? 1.0 : 0.0);
  }
  wv_chol<NFB>(qv, dinv);
  double wr[NFB];
  wv_inv_lower_rows<NFB>(qv, dinv, wr, scratch);  // lane m: row m of L^-1
  if (lane < wn)
#pragma unroll
    for (int c = 0; c < 16; ++c)  // (compile-time trip: wr stays in registers)
      if (c < wn) W[lane * wld + c] = (lane < nf && c < NFB && c < nf && c <= lane) ? wr[c < NFB ? c : 0] : 0.0;
}

// the same factorization bucketed by nf exactly as the BetaLambda tail does it (8 / 10 / 12 / 16),
// so a sharded chain's Eta solve forms the unsharded chain's W bit for bit
__device__ __forceinline__ void q_inv_factor_nf(const double* qm, int ld, int nf, double* W, int wld, int wn,
                                                double* scratch) {
  if (nf <= 8)
    q_inv_factor<8>(qm, ld, nf, W, wld, wn, scratch);
  else if (nf <= 10)
    q_inv_factor<10>(qm, ld, nf, W, wld, wn, scratch);
  else if (nf <= 12)
    q_inv_factor<12>(qm, ld, nf, W, wld, wn, scratch);
  else
    q_inv_factor<16>(qm, ld, nf, W, wld, wn, scratch);
}

template <int NFB>
__device__ __forceinline__ void crw_finish(const CRWArgs& a, const double* sCR, double* W, double* scratch) {
  q_inv_factor<NFB>(sCR + a.nc * 16, 16, a.nf, W, 16, 16, scratch);
}

// The tail of a BetaLambda workgroup of the fused launch (K <= 32, nf <= 16), with the
// species' new column still in registers:
//   * the fused Eta kernel's constants: BL[k, j] iSigma_j Lambda[h, j] and LS (above);
//   * gv_on: updateGammaV's species sums (R/updateGammaV.R:17-19) -- E E^T, E = Beta - Gamma
//     Tr^T (Mu_j from the body) and Beta Tr -- and updateLambdaPriors' psi draws (:22-24),
//     written to Psi, with their per-factor sums psi Lambda^2, as a second partial tile
//     [A nc^2 | BTr nc nt | rs NF] (ld gvt_ld).  The side chain (GammaV algebra, delta chains)
//     reads the group tiles of these.
// The workgroups' four species are summed in LDS; the last workgroup of each group of
// CRW_GROUP (a ticket) sums the group's tiles in workgroup order, the last group through sums
// the CR group tiles in group order (deterministic), raises tails_flag (the side chain's
// start, when it is not behind a graph edge) and factors Q.  No workgroup waits for another:
// each level's work is done by whichever arrives last.  The tiles cross XCDs as device-scope
// (write-through) stores and loads, published by relaxed tickets once every wave's stores
// have completed: no release / acquire fence, whose whole-L2 write-back / invalidate per wave
// of ~250 workgroups cost ~45 us here.
struct BLTailArgs {
  CRWArgs crw;
  int gv_on;
  int psi_pre;      // the body pre-drew the psi gamma variates (BLPsiPre, BLCol::gpre)
  int nt, NF, nr, sp0, gvt_ld;
  int lev_nf[HMSC_MAX_LEVELS];
  double nu[HMSC_MAX_LEVELS];
  const double* Tr;
  double* Psi;
  double* gvt;      // (nbl + ngroups) x gvt_ld
  int* tails_flag;  // epoch of the sweep whose tails are all in
  int* crw_flag;    // deferred: epoch of the sweep whose CR and W are out (the Eta tiles wait on it)
  Key key;
  unsigned long long* kt;     // live timing of the last reducer (KT_TAIL block) or null
  unsigned long long* kt_bl;  // live timing of the BetaLambda bodies (KT_BL block), via the tiles
  // sharded chain: the last reducer also sums the GammaV / psi group tiles in group order into
  // ar_gv (ar_b's [GV | RS] sections, the all-reduce's input) and leaves W to the Eta solve
  // (Q = I + Lambda diag(iSigma) Lambda^T is a sum over every rank's species)
  double* ar_gv;
  // sweep graphs after the first, edge-free: the fused Eta launch runs the last reduction level
  // (defer 1: this launch ends after the group reducers) or both (defer 2: it ends after the
  // workgroups' tiles) in its leading workgroups
  int defer;
};

// Level 1 of the tail's reduction: group g's tiles (workgroups g0 .. g0 + gn - 1) summed in
// workgroup order into group tile nbl + g (write-through), with the bodies' timing words.
// src_coh / dst_coh: the workgroup tiles / the group tile cross workgroups of one launch
// (device-scope loads / write-through stores), else a launch boundary (plain).
__device__ __forceinline__ void tail_group_sum(const BLTailArgs& ta, int g, int nbl, bool src_coh, bool dst_coh) {
  const CRWArgs& a = ta.crw;
  const int t = threadIdx.x, nc = a.nc, nf = a.nf;
  const int g0 = g * CRW_GROUP, gn = min(CRW_GROUP, nbl - g0);
  const int ngv = nc * nc + nc * ta.nt + ta.NF, ne = nf * 32;
  double* P = a.part;
  double* V = ta.gvt;
  const int ld = ta.gvt_ld;
  auto put = [&](double* p, double v) {
    if (dst_coh)
      store_coherent(p, v);
    else
      *p = v;
  };
  auto get = [&](const double* p) { return src_coh ? load_coherent(p) : *p; };
  if (g == 0 && t < 64) HMSC_STAMP_RT(78);
  // group reducer: the group's tiles in workgroup order.  Every load of a thread (TG_E elements
  // x the group's tiles, and the timing words on threads 254 / 255) is issued before the first
  // sum, so a pass costs one memory latency (a load-use loop pays one per tile)
  const int ntot = ne + (ta.gv_on ? ngv : 0);
  const bool kt_thr = ta.kt_bl && t >= 254;  // timing words 512 (min) / 513 (max)
  double ktx[CRW_GROUP];
  if (kt_thr)
#pragma unroll
    for (int u = 0; u < CRW_GROUP; ++u)
      ktx[u] = u < gn ? get(P + (size_t)(g0 + u) * CRW_TILE + 512 + (t - 254)) : (t == 254 ? 1e300 : 0.0);
  // (TG_E elements per thread and pass: config 4's 750 elements (CR 320, GammaV 430) in one
  // pass instead of two, one memory latency less on the way to the Eta launch)
#ifndef HMSC_TG_E
#define HMSC_TG_E 3
#endif
  constexpr int TG_E = HMSC_TG_E;
  for (int q0 = 0; q0 < ntot; q0 += 256 * TG_E) {
    double x[TG_E][CRW_GROUP];
#pragma unroll
    for (int e = 0; e < TG_E; ++e) {
      const int q = q0 + t + 256 * e;
      const bool cr = q < ne;
      const double* src = cr ? P + q : V + (q - ne);
      const size_t st = cr ? CRW_TILE : ld;
#pragma unroll
      for (int u = 0; u < CRW_GROUP; ++u)
        x[e][u] = (q < ntot && u < gn) ? get(src + (size_t)(g0 + u) * st) : 0.0;
    }
#pragma unroll
    for (int e = 0; e < TG_E; ++e) {
      const int q = q0 + t + 256 * e;
      if (q >= ntot) continue;
      const bool cr = q < ne;
      double v = 0.0;
#pragma unroll
      for (int u = 0; u < CRW_GROUP; ++u) v += x[e][u];
      put((cr ? P + q : V + (q - ne)) + (size_t)(nbl + g) * (cr ? CRW_TILE : ld), v);
    }
  }
  if (kt_thr) {
    double m = ktx[0];
#pragma unroll
    for (int u = 1; u < CRW_GROUP; ++u) m = t == 254 ? fmin(m, ktx[u]) : fmax(m, ktx[u]);
    put(P + (size_t)(nbl + g) * CRW_TILE + 512 + (t - 254), m);
  }
}

// Level 2 (the last group through): CR = the group tiles in group order, W = L^-1 of Q, the
// sharded chain's GammaV / psi sums.  tails_flag (every group tile is in: the side chain's
// start) is raised here unless the group level already did (raise_tails); deferred, in the
// Eta launch, crw_flag is raised once CR and W are out (the tile workgroups read them behind it).
// grp_coh: the group tiles were written in this launch (device-scope loads), else in the
// previous one.
__device__ __forceinline__ void tail_final(const BLTailArgs& ta, int nbl, uint32_t iter, double* smem, bool defer,
                                           bool grp_coh, bool raise_tails) {
  const CRWArgs& a = ta.crw;
  const int t = threadIdx.x, w = t >> 6, K = a.K, nc = a.nc, nf = a.nf;
  const int ng = (nbl + CRW_GROUP - 1) / CRW_GROUP;
  const int ngv = nc * nc + nc * ta.nt + ta.NF;
  double* P = a.part;
  double* V = ta.gvt;
  const int ld = ta.gvt_ld;
  auto get = [&](const double* p) { return grp_coh ? load_coherent(p) : *p; };
  const unsigned long long kt0 = ta.kt ? kt_now() : 0ull;
  // every group tile is in: the side chain may start (it sums the GammaV / psi group tiles)
  if (t < 64) HMSC_STAMP_RT(79);
  if (t == 0) {
    __hip_atomic_store(&a.ticket[1], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // every BetaLambda column and tile is out: the side work (post_bl_kernel, or the side
    // chain reading the tail's GammaV / psi group tiles) may start
    if (ta.tails_flag && raise_tails)
      __hip_atomic_store(ta.tails_flag, g2bl_epoch(iter), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  double* sCR = smem + 4 * CRW_TILE;  // [row k][16]
  {
    // CR = the group tiles summed in group order; each thread's two elements' loads of a
    // chunk of groups issued together
    double v[2] = {0.0, 0.0};
    for (int q0 = 0; q0 < ng; q0 += CRW_GROUP) {
      double x[2][CRW_GROUP];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int q = t + 256 * e, h = q >> 5;
#pragma unroll
        for (int u = 0; u < CRW_GROUP; ++u)
          x[e][u] = (h < nf && q0 + u < ng) ? get(P + (size_t)(nbl + q0 + u) * CRW_TILE + q) : 0.0;
      }
#pragma unroll
      for (int e = 0; e < 2; ++e)
#pragma unroll
        for (int u = 0; u < CRW_GROUP; ++u) v[e] += x[e][u];
    }
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int q = t + 256 * e, h = q >> 5, k = q & 31;
      sCR[k * 16 + h] = v[e];
      if (h < nf && k < K) {
        double* d = a.CR + k + (size_t)a.ldcr * h;
        if (defer)
          store_coherent(d, v[e]);
        else
          *d = v[e];
      }
    }
  }
  if (ta.ar_gv && ta.gv_on)  // (sharded) the GammaV / psi sums of this rank's species, group order
    for (int q = t; q < ngv; q += 256) {
      double v = 0.0;
      for (int q0 = 0; q0 < ng; q0 += CRW_GROUP) {
        double x[CRW_GROUP];
#pragma unroll
        for (int u = 0; u < CRW_GROUP; ++u) x[u] = q0 + u < ng ? get(V + (size_t)(nbl + q0 + u) * ld + q) : 0.0;
#pragma unroll
        for (int u = 0; u < CRW_GROUP; ++u) v += x[u];
      }
      ta.ar_gv[q] = v;
    }
  __syncthreads();
  if (t < 64) HMSC_STAMP_RT(88);
  // (deferred: W is formed in LDS and published write-through with CR behind tails_flag, which
  // the Eta launch's tile workgroups wait on before their solves)
  double* wdst = defer ? sCR + 32 * 16 : a.W;
  if (w == 0 && !ta.ar_gv) {
    if (nf <= 8)
      crw_finish<8>(a, sCR, wdst, smem);
    else if (nf <= 10)
      crw_finish<10>(a, sCR, wdst, smem);
    else if (nf <= 12)
      crw_finish<12>(a, sCR, wdst, smem);
    else
      crw_finish<16>(a, sCR, wdst, smem);
  }
  if (defer) {
    __syncthreads();
    store_coherent(a.W + t, wdst[t]);  // 16 x 16, one element per thread
    vm_stores_done();
    __syncthreads();
    if (t == 0) __hip_atomic_store(ta.crw_flag, g2bl_epoch(iter), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (w == 0) HMSC_STAMP_RT(80);
  if (ta.kt && t == 0) kt_record(ta.kt, iter, kt0);
  if (ta.kt_bl && t == 64) {  // the BetaLambda bodies' first start / last end, once (wave 1, beside wave 0's factor)
    double m0 = 1e300, m1 = 0.0;
    for (int q0 = 0; q0 < ng; q0 += CRW_GROUP) {
      double x0[CRW_GROUP], x1[CRW_GROUP];
#pragma unroll
      for (int u = 0; u < CRW_GROUP; ++u) {
        const double* p = P + (size_t)(nbl + (q0 + u < ng ? q0 + u : q0)) * CRW_TILE + 512;
        x0[u] = get(p);
        x1[u] = get(p + 1);
      }
#pragma unroll
      for (int u = 0; u < CRW_GROUP; ++u) {
        m0 = fmin(m0, x0[u]);
        m1 = fmax(m1, x1[u]);
      }
    }
    const uint32_t slot = iter & (KT_SLOTS - 1);
    __hip_atomic_fetch_min(ta.kt_bl + slot, (unsigned long long)m0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_max(ta.kt_bl + KT_SLOTS + slot, (unsigned long long)m1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

__device__ __forceinline__ void bl_tail(const BLTailArgs& ta, const BLCol& col, int b, int nbl, uint32_t iter,
                                        double* smem) {
  __shared__ int s_last;
  const CRWArgs& a = ta.crw;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, K = a.K, nc = a.nc, nf = a.nf;
  const int j = 4 * b + w;
  const bool act = j < a.ns;
  const double r = col.r;
  if (b == 0 && w == 0) HMSC_STAMP_RT(77);
  double trq[8];  // Tr[j, q] (loaded first: its latency overlaps the draws below)
#pragma unroll
  for (int q = 0; q < 8; ++q) trq[q] = (ta.gv_on && act && q < ta.nt) ? ta.Tr[j + (size_t)a.ns * q] : 0.0;
  const double isig = act ? col.isig : 0.0;
  const double lam = __shfl(r, nc + (lane & 15));  // lane h: Lambda[h, j]
  if (act && lane < 16) a.LS[(size_t)16 * j + lane] = lane < nf ? isig * lam : 0.0;
  const double rk = (act && lane < K) ? r * isig : 0.0;
  double c[16];
#pragma unroll
  for (int h = 0; h < 16; ++h) {
    const double l = __shfl(r, nc + h < 64 ? nc + h : 0);
    c[h] = (h < nf) ? rk * l : 0.0;
  }
  // GammaV's E = Beta - Gamma Tr^T (lanes < nc) and the psi draw of factor lane - nc
  const int nt = ta.nt, NF = ta.NF, nA = nc * nc, nB = nc * nt, ngv = nA + nB + NF;
  const double e = (act && lane < nc) ? r - col.mu : 0.0;
  double m2 = 0.0;
  if (ta.gv_on && act && lane >= nc && lane < K) {  // (R/updateLambdaPriors.R:22-24)
    const int f = lane - nc;
    int f0 = 0, lv = 0;
    while (lv < ta.nr - 1 && f >= f0 + ta.lev_nf[lv]) f0 += ta.lev_nf[lv++];
    const int h = f - f0;
    const double lam2 = r * r;
    const double shape = ta.nu[lv] / 2 + 0.5;
    const double rate = ta.nu[lv] / 2 + 0.5 * lam2 * col.tau;
    const uint32_t idx = (uint32_t)(h + ta.lev_nf[lv] * (ta.sp0 + j));
    // (the standard gamma draw needs only the shape: drawn ahead by the body, BLPsiPre; drawn
    // by Gamma2's partial workgroups instead it delayed Gamma: 6,549-6,577 vs 6,676-6,704)
    const double gs = ta.psi_pre ? col.gpre : gamma_std(ta.key, idx, S_PSI + LEVEL_STRIDE * lv, iter, shape);
    const double psi = gs / rate;
    ta.Psi[f + (size_t)NF * j] = psi;
    m2 = psi * lam2;
  }
  if (b == 0 && w == 0) HMSC_STAMP_RT(85);
  __syncthreads();  // every wave is past the body's LDS tiles
  double* sC = smem;                  // [w][h][k]
  double* sV = smem + 4 * CRW_TILE;   // [w][ngv]
  if (lane < 32)
#pragma unroll
    for (int h = 0; h < 16; ++h)
      if (h < nf) sC[w * CRW_TILE + h * 32 + lane] = c[h];
  if (ta.kt_bl && lane == 0) {
    sC[w * CRW_TILE + 512] = (double)col.kt0;
    sC[w * CRW_TILE + 513] = (double)col.kt1;
  }
  if (ta.gv_on) {
    double* v = sV + w * ngv;
#pragma unroll
    for (int c2 = 0; c2 < 32; ++c2) {
      const double e2 = __shfl(e, c2);
      if (c2 < nc && lane < nc) v[lane + nc * c2] = e * e2;  // E E^T
    }
    if (lane < nc)
#pragma unroll
      for (int q = 0; q < 8; ++q)
        if (q < nt) v[nA + lane + nc * q] = r * trq[q];  // Beta Tr
    if (lane >= nc && lane < K) v[nA + nB + lane - nc] = m2;
    else if (lane >= K && lane < nc + NF) v[nA + nB + lane - nc] = 0.0;
  }
  __syncthreads();
  const int ne = nf * 32;
  double* P = a.part;
  double* V = ta.gvt;
  const int ld = ta.gvt_ld;
  // (plain stores + one L2 write-back per workgroup before the ticket measured 3 % slower per
  // sweep than these write-through stores; defer 2: the tiles are read in the next launch)
  const int defer = ta.defer;
  auto put = [&](double* p, double v) {
    if (defer == 2)
      *p = v;
    else
      store_coherent(p, v);
  };
  for (int q = t; q < ne; q += 256)
    put(P + (size_t)b * CRW_TILE + q, (sC[q] + sC[CRW_TILE + q]) + (sC[2 * CRW_TILE + q] + sC[3 * CRW_TILE + q]));
  if (ta.kt_bl && t < 2) {  // the workgroup's first body start / last body end
    const int q = 512 + t;
    const double x0 = sC[q], x1 = sC[CRW_TILE + q], x2 = sC[2 * CRW_TILE + q], x3 = sC[3 * CRW_TILE + q];
    put(P + (size_t)b * CRW_TILE + q, t == 0 ? fmin(fmin(x0, x1), fmin(x2, x3)) : fmax(fmax(x0, x1), fmax(x2, x3)));
  }
  if (ta.gv_on)
    for (int q = t; q < ngv; q += 256)
      put(V + (size_t)b * ld + q, (sV[q] + sV[ngv + q]) + (sV[2 * ngv + q] + sV[3 * ngv + q]));
  if (defer == 2) return;  // both reduction levels run in the Eta launch's leading workgroups
  vm_stores_done();
  __syncthreads();
  if (b == 0 && t < 64) HMSC_STAMP_RT(86);
  const int g = b / CRW_GROUP, gn = min(CRW_GROUP, nbl - g * CRW_GROUP);
  const int ng = (nbl + CRW_GROUP - 1) / CRW_GROUP;
  if (t == 0) s_last = __hip_atomic_fetch_add(&a.ticket[2 + g], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gn - 1;
  __syncthreads();
  if (!s_last) return;
  tail_group_sum(ta, g, nbl, true, true);
  if (t == 0) __hip_atomic_store(&a.ticket[2 + g], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  vm_stores_done();
  __syncthreads();
  if (g == 0 && t < 64) HMSC_STAMP_RT(87);
  if (t == 0) s_last = __hip_atomic_fetch_add(&a.ticket[1], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ng - 1;
  __syncthreads();
  if (!s_last) return;
  if (defer == 1) {  // every group tile is in: the side chain may start; the last level runs in the Eta launch
    if (t == 0) {
      __hip_atomic_store(&a.ticket[1], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (ta.tails_flag) __hip_atomic_store(ta.tails_flag, g2bl_epoch(iter), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return;
  }
  tail_final(ta, nbl, iter, smem, false, true, true);
}

struct G2BLArgs {
  G2Args g2;
  BLArgs bl;
  XZSrc xz;
  const double* BLold;  // Lambda rows of the partials (read before any BetaLambda write: the
                        // writes follow the Gamma flag, which follows every partial's ticket)
  const double* Tr;
  double* part;
  int K, nc, NF, nt, nsl;
  // BetaLambda workgroups that first form one of Gamma2's species-block partials (and the count
  // workgroup 0 waits for): g2.nparts on one rank; 0 on a sharded chain, whose Gamma2 sums
  // arrive all-reduced (g2.part = ar_a, g2.nparts = 1)
  int part_wg;
  int part_tail;        // the partial workgroups follow the BetaLambda ones (else: the first of them)
  int* sync;            // [ticket, epoch of the published Gamma, -, handshake timed out]
  BLTailArgs tail;      // the BetaLambda workgroups' tail (crw_on): Eta constants [+ side partials]
  int crw_on;
  const int* side_sync; // side_wait: [GammaV, delta chain per level ..., Gamma2 prep] flags of
  int side_wait;        // the previous sweep's side chain (graph sweeps after the first)
  int side_prep;        // ... and its Gamma2 prep flag
  unsigned long long* kt_g2;  // live timing of workgroup 0 (KT_G2 block) or null
};

// (two workgroups per CU: with Gamma2's partial workgroups after the BetaLambda ones the launch
// exceeds one per CU, and its workgroups wait on each other, so all must be resident together)
// The tail's psi draw (R/updateLambdaPriors.R:22-24) is psi = g / rate with g a standard
// gamma variate of shape nu / 2 + 1 / 2 -- independent of the new Lambda, so the body draws g
// while its prologue's loads fly and the tail only divides (the rejection sampler was ~2.5 us
// of the tail's chain); the same (key, index, stream, sweep), so the same bits
__device__ __forceinline__ double psi_gamma_std(const BLTailArgs& ta, uint32_t iter, int j, int fct) {
  int f0 = 0, lv = 0;
  while (lv < ta.nr - 1 && fct >= f0 + ta.lev_nf[lv]) f0 += ta.lev_nf[lv++];
  const int h = fct - f0;
  const double shape = ta.nu[lv] / 2 + 0.5;
  const uint32_t idx = (uint32_t)(h + ta.lev_nf[lv] * (ta.sp0 + j));
  return gamma_std(ta.key, idx, S_PSI + LEVEL_STRIDE * lv, iter, shape);
}
struct BLPsiPre {
  const BLTailArgs& ta;
  uint32_t iter;
  bool on;
  int nc, K;
  __device__ double operator()(int j, int lane) const {
    if (!on || !ta.gv_on || lane < nc || lane >= K) return 0.0;
    return psi_gamma_std(ta, iter, j, lane - nc);
  }
  // the same variate from the species' pre-drawn row (bl_predraw_body)
  __device__ double from(const double* row, int lane) const {
    if (!on || !ta.gv_on || lane < nc || lane >= K) return 0.0;
    return row[32 + lane - nc];
  }
};

template <int NM>
__global__ __launch_bounds__(256, 2) void gamma2_bl_kernel(G2BLArgs f) {
  kernarg_warm<sizeof(G2BLArgs)>();
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int nparts = f.part_wg, nbl = (int)gridDim.x - 1 - (f.part_tail ? nparts : 0);
  if (blockIdx.x == 0) {
    const unsigned long long kt0 = f.kt_g2 ? kt_now() : 0ull;
    if (threadIdx.x < 64) HMSC_STAMP_RT(70);
    // wave 0's lanes poll together: lane 0 the partials' count (relaxed; the partials are
    // device-coherent stores, read with device-coherent loads), lanes 1 and 2 the previous
    // sweep's GammaV (Gamma, iV) and Gamma2 prep flags.  Their first loads are issued before
    // the pre phase's, whose latency they share; every wait bounded like every in-launch wait.
    const int lane = threadIdx.x & 63;
    const int ep = g2bl_epoch(SWEEP_ITER(f.g2) - 1);
    const int* pf = nullptr;
    if (threadIdx.x < 64) {
      if (lane == 0) pf = &f.sync[0];
      else if (lane == 1 && f.side_wait) pf = f.side_sync;
      else if (lane == 2 && f.side_wait && f.side_prep) pf = f.side_sync + 1 + f.bl.nr;
    }
    auto seen = [&](int v) { return !pf || (lane == 0 ? v >= nparts : v == ep); };
    auto poll = [&] { return pf ? __hip_atomic_load(pf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0; };
    const int v0 = poll();
    const int ok = gamma2_final_pre(f.g2, smem);
    if (threadIdx.x < 64 && !__all(seen(v0)) && !spin_until<2>([&] { return __all(seen(poll())) != 0; }) && lane == 0)
      __hip_atomic_store(&f.sync[3], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int all_one = __syncthreads_and(ok);
    if (threadIdx.x < 64) HMSC_STAMP_RT(72);
    if (all_one) gamma2_final_main(f.g2, smem);
    __syncthreads();
    if (threadIdx.x < 64) HMSC_STAMP_RT(73);
    if (threadIdx.x == 0) {
      __hip_atomic_store(&f.sync[0], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // every partial is in
      __hip_atomic_store(&f.sync[1], g2bl_epoch(SWEEP_ITER(f.g2)), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      if (f.kt_g2) kt_record(f.kt_g2, SWEEP_ITER(f.g2), kt0);
    }
    return;
  }
  const int b = blockIdx.x - 1;
  if (b == 40 && threadIdx.x < 64) HMSC_STAMP_RT(97);
  // Gamma2's partials: part_tail, on workgroups of their own after the BetaLambda ones (default);
  // else on the first nparts BetaLambda workgroups ahead of their bodies
  const int pb = f.part_tail ? b - nbl : b;
  if (pb >= 0 && pb < nparts) {
    if (pb == 0 && threadIdx.x < 64) HMSC_STAMP_RT(71);
#ifdef HMSC_STAMPS
    if (pb < 160 && threadIdx.x == 0) g_stamps[700 + pb] = __builtin_amdgcn_s_memrealtime();
#endif
    gamma2_partial_body(f.xz, f.BLold, f.K, f.nc, f.NF, f.nt, f.nsl, f.Tr, f.part, smem, pb, true);
    vm_stores_done();
    __syncthreads();  // every wave's partial stores have completed (and the LDS is free again)
    if (threadIdx.x == 0) __hip_atomic_fetch_add(&f.sync[0], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#ifdef HMSC_STAMPS
    if (pb < 160 && threadIdx.x == 0) g_stamps[860 + pb] = __builtin_amdgcn_s_memrealtime();
#endif
    if (f.part_tail) return;
  }
  const uint32_t iter = SWEEP_ITER(f.g2);
  const BLCol col = beta_lambda_wave_body<NM, true>(f.bl, smem, b, f.sync, f.side_sync, g2bl_epoch(iter - 1),
                                                    f.side_wait ? 1 + f.bl.nr : 0,
                                                    BLPsiPre{f.tail, iter, f.crw_on && f.tail.psi_pre, f.nc, f.K});
  if (f.crw_on) bl_tail(f.tail, col, b, nbl, iter, smem);
}

// doubles of gamma2_prep_kernel's working set (in s.scratch2 when past 64 KB)
static size_t g2_prep_doubles(const State& s) {
  const size_t N = (size_t)s.nc * s.nt;
  return 7 * (size_t)s.nc * s.nc + 3 * N * N;
}

static void launch_gamma2_prep(State& s, hipStream_t st) {
  G2PrepArgs a{};
  a.nc = s.nc;
  a.nt = s.nt;
  a.iV = s.iV;
  a.XX = s.XX;
  a.TT = s.TT;
  a.iV0 = s.iV0;
  a.prep = s.g2prep;
  a.scratch = s.scratch2;
  a.fail = s.dev_flags + 1;
  const size_t need = g2_prep_doubles(s) * sizeof(double);
  a.use_lds = need <= 64 * 1024;
  HMSC_REQUIRE(a.use_lds || g2_prep_doubles(s) <= s.scratch2_doubles, "internal: Gamma2 prep scratch too small");
  gamma2_prep_kernel<<<1, 256, a.use_lds ? need : 0, st>>>(a);
  HIP_OK(hipGetLastError());
  s.g2prep_valid = true;
}

constexpr size_t G2F_LDS_CAP = 64 * 1024;  // bytes of LDS the unfused final stage takes at most

// the unfused final stage's layout for this chain's nc, nt, NF (G2FLds): S0 | LTr | v1 | v2 | xi |
// red | sGL | B1 LS; staged B1 | LS when everything fits 64 KB, in LDS without them when the rest
// does, else every array in global memory after the prep's working set (s.scratch2).  Returns
// the launch's dynamic LDS bytes.
static size_t g2f_layout(const State& s, G2Args& a) {
  const int N = s.nc * s.nt, nL = s.NF * s.nt, ngl = s.nc * s.NF <= 2048 ? s.nc * s.NF : 0;
  auto up2 = [](int v) { return (v + 1) & ~1; };  // 16-byte aligned arrays
  int o = up2(N);
  a.lay_ltr = o;
  o += up2(nL);
  a.lay_v1 = o;
  o += up2(N);
  a.lay_v2 = o;
  o += up2(N);
  a.lay_xi = o;
  o += up2(N);
  a.lay_red = o;
  o += 8 * 64;
  a.lay_sgl = o;
  o += up2(ngl);
  a.lay_dyn = o;
  const size_t core = (size_t)o * sizeof(double);
  const size_t stage_bytes = ((size_t)s.nc * s.nc + (size_t)N * N) * sizeof(double);
  a.gbase = nullptr;
  const bool force_global = getenv_flag("HMSC_G2F_GLOBAL");  // (tests: the global-memory layout at small N)
  a.stage = !force_global && core + stage_bytes <= G2F_LDS_CAP;
  if (a.stage) return core + stage_bytes;
  if (!force_global && core <= G2F_LDS_CAP) return core;
  a.gbase = s.scratch2 + ((g2_prep_doubles(s) + 15) & ~(size_t)15);
  HMSC_REQUIRE((size_t)(a.gbase - s.scratch2) + o <= s.scratch2_doubles, "internal: Gamma2 scratch too small");
  return 0;
}

void launch_gamma2(State& s, uint32_t iter) {
  if (!s.xeta_valid) launch_xeta(s);
  flush_g(s);
  if (!s.zt_valid) launch_zt_refresh(s);
  if (!s.g2prep_valid) {
    join_side(s);
    launch_gamma2_prep(s, s.stream);
  }
  const int nparts = (s.nsl + G2SB - 1) / G2SB;
  flush_xz(s);  // (the stripe sums of a partial-reading gamma2_partial_body need the fused launch's LDS)
  gamma2_partial_kernel<<<nparts, 256, (size_t)(s.K * G2SB + G2SB * s.nt) * sizeof(double), s.stream>>>(
      xz_src(s), s.BL, s.K, s.nc, s.NF, s.nt, s.nsl, s.Tr, s.ABpart);
  HIP_OK(hipGetLastError());
  const int n1 = s.nc * s.nt, n2 = s.NF * s.nt;
  double* part = s.ABpart;
  int np = nparts;
  double* xtztr = s.allreduce_buf + (n1 + n2);
  if (s.has_na) xt_ztr_kernel<<<n1, 256, 0, s.stream>>>(s.X, s.ZTr, s.ny, s.nc, s.nt, xtztr);
  double* isig_count = nullptr;
  G2Args a{};
  a.nc = s.nc;
  a.nt = s.nt;
  a.Kmax = s.Kmax;
  a.NF = s.NF;
  a.nparts = np;
  a.ns_loc = s.nsl;
  a.use_xtztr = s.has_na ? 1 : 0;
  a.check_isigma = 1;
  a.isig_count = isig_count;
  a.part = part;
  a.xtztr = xtztr;
  a.G = s.G;
  a.prep = s.g2prep;
  a.iSigma = s.iSigma;
  a.Gamma = s.Gamma;
  a.key = s.key;
  a.iter = iter;
  a.iter_dev = s.capturing ? s.d_iter : nullptr;
  a.noise_zero = s.noise_mode;
  const size_t lds = g2f_layout(s, a);
  join_side(s);  // iV and the prep matrices come from the previous sweep's GammaV (side stream)
  gamma2_final_kernel<<<1, 256, lds, s.stream>>>(a);
  HIP_OK(hipGetLastError());
}

// workgroup slots the side stream may hold while the fused launch runs (side chain, record pack)
constexpr int G2BL_SLOT_MARGIN = 64;

// workgroups of the fused Gamma2 + BetaLambda launch resident on the whole device at once
static int g2bl_resident_slots(const State& s, size_t smem) {
  static std::mutex mu;
  static std::map<std::pair<int, int>, int> cache;  // (device, K bucket) -> slots
  const int kb = wv_bucket(s.K);
  std::lock_guard<std::mutex> lk(mu);
  auto it = cache.find({s.device, kb});
  if (it != cache.end()) return it->second;
  int nb = 0, ncu = 0;
  switch (kb) {
    case 8: HIP_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, gamma2_bl_kernel<8>, 256, smem)); break;
    case 16: HIP_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, gamma2_bl_kernel<16>, 256, smem)); break;
    case 24: HIP_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, gamma2_bl_kernel<24>, 256, smem)); break;
    default: HIP_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, gamma2_bl_kernel<32>, 256, smem)); break;
  }
  HIP_OK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, s.device));
  const int slots = std::max(0, nb) * std::max(0, ncu);
  cache[{s.device, kb}] = slots;
  return slots;
}

bool gamma2_bl_fusion_ok(const State& s) {
  const uint32_t need = HMSC_UP_GAMMA2 | HMSC_UP_BETALAMBDA;
  const size_t N = (size_t)s.nc * s.nt;
  return (s.mask & need) == need && !(s.mask & HMSC_UP_GAMMAETA) && !s.sharded && !s.has_na && !s.phylo && !s.any_xs &&
         s.K <= 32 && s.nt <= 8 && N <= 256 && s.NF <= 64 && s.NF * s.nt + N <= 64 && s.gbl_sync != nullptr &&
         (G2F_LDS + (size_t)s.nc * s.nc + N * N) <= (size_t)BLW_LDS && !getenv_flag("HMSC_NO_G2BL_FUSION") &&
         // workgroup 0 waits for the partials' workgroups, so they (dispatched first when not
         // trailing) and workgroup 0 must be resident together, beside the side stream's kernels
         1 + (s.nsl + G2SB - 1) / G2SB + G2BL_SLOT_MARGIN <= g2bl_resident_slots(s, BLW_LDS * sizeof(double));
}

// updateGamma2 then updateBetaLambda as one launch (gamma2_bl_kernel)
static CRWArgs make_crw_args(const State& s);
static void shard_g2_stats(State& s);
bool side_fusion_ok(const State& s);


// The Eta launch of a captured one-rank sweep draws the next sweep's BetaLambda noise and psi
// variates ahead (bl_predraw_body; the wave body's K <= 32).  With both tail levels in the Eta
// launch: 1000-step 6,842 -> 6,947 sweeps/s, 3 of 3 same-box rounds; either alone within noise
// (profiles/r06_predraw_ab.txt).  HMSC_NO_BL_PREDRAW=1: drawn in the BetaLambda prologue.
static bool bl_predraw_on(const State& s) {
  return !getenv_flag("HMSC_NO_BL_PREDRAW") && !s.sharded && s.capturing && s.K <= 32 && s.bl_pre != nullptr;
}

// how many of the tail's reduction levels a deferred tail leaves to the Eta launch: both
// (default since the BetaLambda draws are made ahead: the fused launch then ends with its
// bodies and the Eta launch starts ~8 us sooner), or the last (HMSC_TAIL_DEFER_LEVELS=1;
// round 5's default, when the bodies were draw-bound and two levels measured 0.5 % slower)
static int tail_defer_levels() {
  const char* e = getenv("HMSC_TAIL_DEFER_LEVELS");
  return (e && atoi(e) == 1) ? 1 : 2;
}

// the BetaLambda workgroups' tail (crw_on), also the Eta launch's reducers under EF_DEFER
static BLTailArgs make_tail_args(State& s, bool tail_gv, bool sh) {
  BLTailArgs t{};
  t.crw = make_crw_args(s);
  t.gv_on = tail_gv;
  t.nt = s.nt;
  t.NF = s.NF;
  t.nr = s.nr;
  t.sp0 = s.sp0;
  t.gvt_ld = s.gvt_ld;
  for (int r = 0; r < s.nr; ++r) {
    t.lev_nf[r] = s.lev[r].nf;
    t.nu[r] = s.lev[r].nu;
  }
  t.Tr = s.Tr;
  t.Psi = s.Psi;
  t.gvt = s.gvt;
  t.tails_flag = s.gbl_sync + 2;
  t.crw_flag = s.crw_flag;
  t.key = s.key;
  t.kt = s.kt_on ? s.d_kt + (size_t)KT_TAIL * 2 * KT_SLOTS : nullptr;
  t.kt_bl = s.kt_on ? s.d_kt + (size_t)KT_BL * 2 * KT_SLOTS : nullptr;
  t.ar_gv = nullptr;
  t.defer = 0;
  if (sh) {
    const ArbLayout L = arb_layout(s);
    t.crw.CR = s.ar_b + L.cr;
    t.crw.ldcr = L.ldcr;
    t.ar_gv = s.ar_b + L.gv;  // [GV | RS], the tile layout
  }
  return t;
}
void launch_gamma2_bl(State& s, uint32_t iter) {
  if (!s.xeta_valid) launch_xeta(s);
  flush_g(s);
  if (!s.zt_valid) launch_zt_refresh(s);
  // the co-launched sweep (launch_side_fused) runs the fused Eta kernel next: its constants
  // are formed in the BetaLambda workgroups' tail (K <= 32 on this path, nf <= 16), with
  // GammaV's and LambdaPriors' species partials when their tile fits the tail's LDS
  // a sharded chain (sharded_fused_ok): Gamma2's sums arrive all-reduced in ar_a, and the tail
  // leaves this rank's CR and GammaV / psi sums in ar_b for the all-reduce B
  const bool sh = s.sharded;
  const bool crw_on = sh || (side_fusion_ok(s) && s.lev[0].nf <= 16 && s.K <= 32);
  const bool tail_gv = sh || (!s.side_partials && crw_on && (s.mask & HMSC_UP_GAMMA2) && s.nt <= 8 &&
                              s.nc * s.nc + s.nc * s.nt + s.NF <= 1024 && s.gvt != nullptr);
  // graph sweeps after the first: the previous sweep's side chain is joined on the device
  const bool dev_join = (!sh || s.shard_dev) && crw_on && s.edge_free_now && s.capturing && s.cap_sweep > 0 && s.side_tail;
  // iV, Gamma2's prep, Psi and Delta come from the previous sweep's side updaters
  if (!dev_join) join_side(s);
  // ... and when the slab launch after the last updateZ has waited for them (SideGate), this
  // launch reads them with plain loads
  const bool gated = dev_join && s.side_gated;
  s.side_gated = false;
  if (sh && !s.g2s_valid) shard_g2_stats(s);
  if (!s.g2prep_valid) launch_gamma2_prep(s, s.stream);
  G2BLArgs f{};
  const int nparts = (s.nsl + G2SB - 1) / G2SB;
  const int n12 = s.nc * s.nt + s.NF * s.nt;
  G2Args& a = f.g2;
  a.nc = s.nc;
  a.nt = s.nt;
  a.Kmax = s.Kmax;
  a.NF = s.NF;
  a.nparts = sh ? 1 : nparts;
  a.ns_loc = s.nsl;
  a.use_xtztr = 0;
  // probit iSigma is 1 by construction (updateInvSigma leaves it) unless set from outside; a
  // sharded chain counts iSigma != 1 over every rank's species (ar_a)
  a.check_isigma = (sh || (s.all_probit && s.isigma_fixed_one)) ? 0 : 1;
  a.isig_count = sh ? s.ar_a + n12 : nullptr;
  a.part = sh ? s.ar_a : s.ABpart;
  a.xtztr = nullptr;
  a.G = s.G;
  a.prep = s.g2prep;
  a.iSigma = s.iSigma;
  a.Gamma = s.Gamma;
  a.key = s.key;
  a.iter = iter;
  a.iter_dev = s.capturing ? s.d_iter : nullptr;
  a.noise_zero = s.noise_mode;
  a.stage = 1;
  a.coherent = 1;
  f.bl = make_bl_args(s, iter);
  f.xz = xz_src(s);
  f.BLold = s.BL;
  f.Tr = s.Tr;
  f.part = s.ABpart;
  f.K = s.K;
  f.nc = s.nc;
  f.NF = s.NF;
  f.nt = s.nt;
  f.nsl = s.nsl;
  f.part_wg = sh ? 0 : nparts;
  f.sync = s.gbl_sync;
  f.crw_on = crw_on;
  // sweep graphs after the first, edge-free (the side work forked on the device, see
  // launch_side_fused): the tail's reductions move into the Eta launch (EF_DEFER)
  const bool defer = crw_on && !sh && s.edge_free_now && s.capturing && (s.cap_sweep > 0 || s.side_root) &&
                     !getenv_flag("HMSC_NO_TAIL_DEFER");
  if (crw_on) {
    f.tail = make_tail_args(s, tail_gv, sh);
    f.tail.defer = defer ? tail_defer_levels() : 0;
    f.tail.psi_pre = getenv_flag("HMSC_NO_PSI_PRE") ? 0 : 1;
    f.bl.kt_defer = 1;
  }
  if (bl_predraw_on(s)) {  // (used only when the tag names this sweep)
    f.bl.pre_buf = s.bl_pre;
    f.bl.pre_tag = s.bl_pre_tag;
  }
  s.tail_defer = defer;
  s.crw_fresh = crw_on && !sh;
  s.tail_gv = tail_gv && !sh;
  s.side_tail = false;  // (both set again by this sweep's launch_side_fused)
  s.psi_side = !sh;     // (a sharded chain's tail draws psi: its record pack reads Psi on the main stream)
  f.side_sync = s.side_sync;
  f.side_wait = dev_join && !gated;
  a.prep_coherent = f.side_wait;
  f.side_prep = (s.mask & HMSC_UP_GAMMA2) ? 1 : 0;
  f.kt_g2 = s.kt_on ? s.d_kt + (size_t)KT_G2 * 2 * KT_SLOTS : nullptr;
  if (!s.capturing) {  // an eager sweep may repeat an iter
    HIP_OK(hipMemsetAsync(s.gbl_sync + 1, 0, 2 * sizeof(int), s.stream));
    HIP_OK(hipMemsetAsync(s.crw_flag, 0, sizeof(int), s.stream));
  }
  // the partials on workgroups of their own after the BetaLambda ones (the launch's 52 KB of
  // LDS and <= 256 VGPRs keep two workgroups per CU resident); HMSC_G2_PART_INLINE: ahead of
  // the first BetaLambda bodies instead
  // Trailing partial workgroups are waited on by workgroup 0, which every BetaLambda
  // workgroup waits on: they must all be resident at once, so the trailing layout is taken
  // only when the whole grid fits the device's resident slots with room to spare for the side
  // stream's kernels, and only with one chain on the device (two overlapping fused launches
  // share the slots).  Otherwise the partials run ahead of the first BetaLambda bodies, whose
  // workgroups are dispatched before any workgroup that waits.
  const size_t smem = BLW_LDS * sizeof(double);
  const int nb_tail = 1 + (s.nsl + 3) / 4 + f.part_wg;
  f.part_tail = !getenv_flag("HMSC_G2_PART_INLINE") && live_chains_on(s.device) == 1 &&
                nb_tail + G2BL_SLOT_MARGIN <= g2bl_resident_slots(s, smem);
  const int nb = 1 + (s.nsl + 3) / 4 + (f.part_tail ? f.part_wg : 0);
  HMSC_REQUIRE(f.part_tail || f.part_wg <= nb - 1, "fused Gamma2 + BetaLambda: more Gamma2 partials than BetaLambda workgroups");
  s.g2bl_last_tail = f.part_tail;
  s.g2bl_last_nb = nb;
  ProfScope ps(s, PROF_BL);
  switch (wv_bucket(s.K)) {
    case 8: gamma2_bl_kernel<8><<<nb, 256, smem, s.stream>>>(f); break;
    case 16: gamma2_bl_kernel<16><<<nb, 256, smem, s.stream>>>(f); break;
    case 24: gamma2_bl_kernel<24><<<nb, 256, smem, s.stream>>>(f); break;
    default: gamma2_bl_kernel<32><<<nb, 256, smem, s.stream>>>(f); break;
  }
  HIP_OK(hipGetLastError());
}

// ---------------------------------------------------------------------------
// updateLambdaPriors (R/updateLambdaPriors.R:3-53, matrix branch :21-33)
// ---------------------------------------------------------------------------
struct LPArgs {
  int NF, K, nc, nr, ns_loc, sp0;
  int lev_nf[HMSC_MAX_LEVELS];
  double nu[HMSC_MAX_LEVELS], a1[HMSC_MAX_LEVELS], b1[HMSC_MAX_LEVELS], a2[HMSC_MAX_LEVELS],
      b2[HMSC_MAX_LEVELS];
  const double* BL;
  double* Psi;
  double* Delta;
  double* rs_part;  // [block][NF]
  int ns_glob;
  Key key;
  uint32_t iter;
  const uint32_t* iter_dev;  // graph replay: the sweep counter is read from the device
};

__device__ __forceinline__ void psi_body(const LPArgs& a, int bid, int nb, bool coh = false) {
  // grid over species columns; each block handles a contiguous species range
  __shared__ double sM[256];
  __shared__ double sTau[HMSC_KCAP];
  __shared__ int sLev[HMSC_KCAP], sH[HMSC_KCAP];
  const int t = threadIdx.x;
  if (t == 0) {
    int f = 0;
    for (int r = 0; r < a.nr; ++r) {
      double c = 1.0;
      for (int h = 0; h < a.lev_nf[r]; ++h, ++f) {
        c *= a.Delta[f];
        sTau[f] = c;       // tau = cumprod(delta)  (:17)
        sLev[f] = r;
        sH[f] = h;
      }
    }
  }
  __syncthreads();
  const int NF = a.NF;
  const int per = (a.ns_loc + nb - 1) / nb;
  const int ja = bid * per, jb = min(a.ns_loc, ja + per);
  const int nelem = (jb > ja ? jb - ja : 0) * NF;
  double* rs = a.rs_part + (size_t)bid * NF;
  double acc = 0.0;  // thread t < NF accumulates row t in fixed order
  for (int base = 0; base < nelem; base += 256) {
    const int p = base + t;
    double m = 0.0;
    if (p < nelem) {
      const int f = p % NF, j = ja + p / NF;
      const int r = sLev[f], h = sH[f];
      const double* lp = a.BL + a.nc + f + (size_t)a.K * j;
      const double lam = coh ? load_coherent(lp) : *lp;
      const double lam2 = lam * lam;
      const double shape = a.nu[r] / 2 + 0.5;
      const double rate = a.nu[r] / 2 + 0.5 * lam2 * sTau[f];            // (:22)
      const uint32_t idx = (uint32_t)(h + a.lev_nf[r] * (a.sp0 + j));
      const double psi = gamma_std(a.key, idx, S_PSI + LEVEL_STRIDE * r, SWEEP_ITER(a), shape) / rate;  // (:23)
      a.Psi[f + (size_t)NF * j] = psi;
      m = psi * lam2;                                                     // M = psi*lambda^2 (:24)
    }
    sM[t] = m;
    __syncthreads();
    if (t < NF) {
      const int q0 = (t - base % NF + NF) % NF;  // first q with (base + q) % NF == t
      for (int q = q0; q < 256 && base + q < nelem; q += NF) acc += sM[q];
    }
    __syncthreads();
  }
  if (t < NF) rs[t] = acc;
}

__global__ __launch_bounds__(256) void psi_kernel(LPArgs a) { psi_body(a, blockIdx.x, gridDim.x); }

// Marsaglia-Tsang with its first 64 trials evaluated in parallel by one wave; the
// first accepted trial is taken, so the value equals the sequential gamma_std().
__device__ double wave_gamma_std(Key key, uint32_t idx, uint32_t stream, uint32_t iter, double shape) {
  const int lane = threadIdx.x & 63;
  const double a = shape < 1.0 ? shape + 1.0 : shape;
  const double d = a - 1.0 / 3.0;
  const double c = 1.0 / sqrt(9.0 * d);
  const double x = normal(key, idx, 2u * lane, stream, iter);
  double v = 1.0 + c * x;
  bool acc = false;
  double val = d;
  if (v > 0.0) {
    v = v * v * v;
    const double u = uniforms(key, idx, 2u * lane + 1u, stream, iter).a;
    acc = log_fast(u) < 0.5 * x * x + d - d * v + d * log_fast(v);
    val = d * v;
  }
  const unsigned long long m = __ballot(acc);
  double out = d;
  if (m) out = __shfl(val, __ffsll((long long)m) - 1);
  if (shape < 1.0) out *= pow(uniforms(key, idx, GAMMA_BOOST_SUB, stream, iter).a, 1.0 / shape);
  return out;
}

// any block size that is a multiple of 64.  The standard gamma draw of step h has shape
// a + ns (nf - h) / 2 (R/updateLambdaPriors.R:26-31), independent of the chain -- only its
// rate depends on the deltas drawn before it -- so the waves first draw all nf standard
// gammas in parallel (wave w takes h = w, w + nwaves, ...), and the sequential chain that
// remains is nf rate evaluations and divisions on one thread: the same values, in the same
// order, as drawing gamma(shape, rate) step by step.
__device__ __forceinline__ void delta_body(const LPArgs& a, const double* rs_part, int nparts, int r,
                                           int rs_ld = 0, int* flags = nullptr) {
  if (rs_ld == 0) rs_ld = a.NF;
  // one workgroup per level: the sequential delta chain (R/updateLambdaPriors.R:25-32)
  __shared__ double rs[HMSC_KCAP], delta[HMSC_KCAP], gstd[HMSC_KCAP];
  const int t = threadIdx.x, w = t >> 6, nw = blockDim.x >> 6;
  const int nf = a.lev_nf[r];
  int f0 = 0;
  for (int q = 0; q < r; ++q) f0 += a.lev_nf[q];
  for (int h = t; h < nf; h += blockDim.x) {
    double sum = 0.0;
    for (int b = 0; b < nparts; ++b) sum += load_coherent(rs_part + (size_t)b * rs_ld + f0 + h);
    rs[h] = sum;
    delta[h] = a.Delta[f0 + h];
  }
  if (r == 0) HMSC_STAMP(20);
  const uint32_t stream = S_DELTA + LEVEL_STRIDE * r;
  const double ns = (double)a.ns_glob;
  for (int h = w; h < nf; h += nw) {
    const double ad = (h == 0 ? a.a1[r] : a.a2[r]) + 0.5 * ns * (nf - h);
    const double g = wave_gamma_std(a.key, (uint32_t)h, stream, SWEEP_ITER(a), ad);
    if ((t & 63) == 0) gstd[h] = g;
  }
  __syncthreads();
  if (t == 0) {
    for (int h = 0; h < nf; ++h) {
      // sum_{h' >= h} tau_h' rs_h' / delta_h with tau = cumprod(current delta)
      double c = 1.0, sum = 0.0;
      for (int q = 0; q < nf; ++q) {
        c *= delta[q];
        if (q >= h) sum += c * rs[q];
      }
      const double bd = (h == 0 ? a.b1[r] : a.b2[r]) + 0.5 * sum / delta[h];
      delta[h] = gstd[h] / bd;
    }
  }
  __syncthreads();
  for (int h = t; h < nf; h += blockDim.x) a.Delta[f0 + h] = delta[h];
  if (r == 0) HMSC_STAMP(21);
  if (flags) {  // this level's Delta is out (the next sweep's fused launch waits on this)
    __threadfence();
    __syncthreads();
    if (t == 0) __hip_atomic_store(&flags[1 + r], g2bl_epoch(SWEEP_ITER(a)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

__global__ __launch_bounds__(64) void delta_kernel(LPArgs a, const double* rs_part, int nparts) {
  delta_body(a, rs_part, nparts, blockIdx.x);
}

// The side stream's whole chain in one launch: workgroup 0 runs updateGammaV (+ Gamma2's
// prep), workgroups 1..nr the delta chains of updateLambdaPriors -- independent updaters, so
// neither waits behind the other.
// tails_flag (graph sweeps after the first): the launch is not behind a graph edge from the
// fused Gamma2 + BetaLambda launch it reads; it waits for that launch's tails to be in.
template <int NM>
__global__ __launch_bounds__(256) void side_chain_kernel(GVWArgs g, LPArgs lp, const double* rs_part, int nparts,
                                                         int rs_ld, const int* tails_flag, int* err,
                                                         unsigned long long* kt) {
  kernarg_warm<sizeof(GVWArgs) + sizeof(LPArgs) + 64>();
  const unsigned long long kt0 = kt ? kt_now() : 0ull;
  // A latency-bound chain of small factorisations running beside the main stream's Eta and z
  // waves on the same SIMDs: raised issue priority, so its few waves are not starved by the
  // VALU-bound z waves (the arbiter picks the highest-priority ready wave).
  __builtin_amdgcn_s_setprio(3);
  if (blockIdx.x == 0 && threadIdx.x < 64) HMSC_STAMP_RT(81);
  if (tails_flag) side_wait(tails_flag, 1, g2bl_epoch(SWEEP_ITER(g)), err);
  if (blockIdx.x == 0 && threadIdx.x < 64) HMSC_STAMP_RT(82);
  if (blockIdx.x == 0)
    gammav_body<NM>(g);
  else
    delta_body(lp, rs_part, nparts, blockIdx.x - 1, rs_ld, g.flags);
  if (kt && threadIdx.x == 0) kt_record(kt, SWEEP_ITER(g), kt0);
}

constexpr int LP_PARTS = 64;

static LPArgs make_lp_args(State& s, uint32_t iter) {
  LPArgs a{};
  a.NF = s.NF;
  a.K = s.K;
  a.nc = s.nc;
  a.nr = s.nr;
  a.ns_loc = s.nsl;
  a.sp0 = s.sp0;
  a.ns_glob = s.ns;
  for (int r = 0; r < s.nr; ++r) {
    a.lev_nf[r] = s.lev[r].nf;
    a.nu[r] = s.lev[r].nu;
    a.a1[r] = s.lev[r].a1;
    a.b1[r] = s.lev[r].b1;
    a.a2[r] = s.lev[r].a2;
    a.b2[r] = s.lev[r].b2;
  }
  a.BL = s.BL;
  a.Psi = s.Psi;
  a.Delta = s.Delta;
  a.rs_part = s.psi_rs;
  a.key = s.key;
  a.iter = iter;
  a.iter_dev = s.capturing ? s.d_iter : nullptr;
  return a;
}

void launch_lambda_priors(State& s, uint32_t iter, hipStream_t st) {
  if (s.nr == 0) return;
  HMSC_REQUIRE(s.NF <= HMSC_KCAP, "updateLambdaPriors: sum(nf) must be <= 128 in this build");
  const LPArgs a = make_lp_args(s, iter);
  const int nparts = std::min(LP_PARTS, std::max(1, s.nsl));
  psi_kernel<<<nparts, 256, 0, st>>>(a);
  HIP_OK(hipGetLastError());
  delta_kernel<<<s.nr, 64, 0, st>>>(a, s.psi_rs, nparts);
  HIP_OK(hipGetLastError());
}

// ---------------------------------------------------------------------------
// updateEta, non-spatial levels (R/updateEta.R:42-92).
//   ZL  = Z (Lambda_all diag(iSigma))^T      (ny x NF; the one HBM pass over Z)
//   CR  = BL diag(iSigma) Lambda_all^T       (K x NF; small)
//   per level r, per unit q:
//     Q_q = I + n_q Lambda_r diag(iSigma) Lambda_r^T                         (:45,52,76)
//     b_q = sum_{i in q} [ ZL_i,r - sum_{k not in level r} XEta_ik CR_k,r ]  (= S_i Lambda~^T, :55,79)
//     eta_q = Q_q^-1 b_q + R_q^-1 xi                                          (:56,90)
// ---------------------------------------------------------------------------
template <int NFB>
__global__ __launch_bounds__(256) void zl_kernel(const double* __restrict__ Z, const double* __restrict__ BL,
                                                 const double* __restrict__ iSigma, const int8_t* __restrict__ mask,
                                                 int ny, int ns_loc, int K, int nc, int NFtot, int split,
                                                 double* __restrict__ ZL_part, int fo, int NF) {
  // factors fo .. fo + NF - 1 of the NFtot (NF <= NFB <= 64 per launch)
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int i = blockIdx.x * 64 + lane;
  const int per = (ns_loc + split - 1) / split;
  const int ja = blockIdx.y * per, jb = min(ns_loc, ja + per);
  const int nj = jb > ja ? jb - ja : 0;
  double* sL = smem;  // [jj][NF]
  for (int p = t; p < nj * NF; p += 256) {
    const int jj = p / NF, f = p % NF, j = ja + jj;
    sL[p] = BL[nc + fo + f + (size_t)K * j] * iSigma[j];
  }
  __syncthreads();
  double acc[NFB];
#pragma unroll
  for (int f = 0; f < NFB; ++f) acc[f] = 0.0;
  // mask (a sharded chain's NA cells, R/updateEta.R:59-70): Y codes; NA cells add nothing
  auto zv = [&](int j) {
    const double z = Z[i + (size_t)ny * j];
    return (mask && mask[i + (size_t)ny * j] < 0) ? 0.0 : z;
  };
  if (i < ny) {
    int jj = w;
    for (; jj + 12 < nj; jj += 16) {
      const double z0 = zv(ja + jj);
      const double z1 = zv(ja + jj + 4);
      const double z2 = zv(ja + jj + 8);
      const double z3 = zv(ja + jj + 12);
      const double* l0 = sL + jj * NF;
      const double* l1 = l0 + 4 * NF;
      const double* l2 = l0 + 8 * NF;
      const double* l3 = l0 + 12 * NF;
#pragma unroll
      for (int f = 0; f < NFB; ++f)
        if (f < NF) acc[f] = fma(z3, l3[f], fma(z2, l2[f], fma(z1, l1[f], fma(z0, l0[f], acc[f]))));
    }
    for (; jj < nj; jj += 4) {
      const double z0 = zv(ja + jj);
      const double* l0 = sL + jj * NF;
#pragma unroll
      for (int f = 0; f < NFB; ++f)
        if (f < NF) acc[f] = fma(z0, l0[f], acc[f]);
    }
  }
  __syncthreads();
  double* sR = smem;  // reuse: [w][f][lane]
#pragma unroll
  for (int f = 0; f < NFB; ++f)
    if (f < NF) sR[(w * NF + f) * 64 + lane] = acc[f];
  __syncthreads();
  for (int p = t; p < NF * 64; p += 256) {
    const int f = p / 64, l = p % 64, ii = blockIdx.x * 64 + l;
    const double v = sR[(0 * NF + f) * 64 + l] + sR[(1 * NF + f) * 64 + l] + sR[(2 * NF + f) * 64 + l] +
                     sR[(3 * NF + f) * 64 + l];
    if (ii < ny) ZL_part[(size_t)blockIdx.y * ny * NFtot + (size_t)ii * NFtot + fo + f] = v;
  }
}

// CR[k, f] = sum_j BL[k, j] iSigma[j] BL[nc + f, j] over a block of SB species -> slab
// (and LS = Lambda_all diag(iSigma), NF x ns_loc, for the fused Eta kernel when LS != null)
__device__ __forceinline__ void cr_body(const double* BL, const double* iSigma, int K, int nc, int NF, int ns_loc,
                                        double* CR_part, int ldcr, int slab, double* LS, double* smem, int bid) {
  double* sX = smem;   // K x SB
  const int t = threadIdx.x, j0 = bid * SB, nj = min(SB, ns_loc - j0);
  for (int p = t; p < K * nj; p += 256) {
    const int jj = p / K;
    sX[p] = BL[(size_t)K * j0 + p];
    (void)jj;
  }
  __syncthreads();
  if (LS)  // [species][16], zero past NF (<= 16): the fused Eta kernel's MFMA B operand
    for (int p = t; p < 16 * nj; p += 256) {
      const int f = p & 15, jj = p >> 4;
      LS[f + (size_t)16 * (j0 + jj)] = f < NF ? sX[nc + f + K * jj] * iSigma[j0 + jj] : 0.0;
    }
  double* out = CR_part + (size_t)bid * slab;
  for (int p = t; p < K * NF; p += 256) {
    const int k = p % K, f = p / K;
    double acc = 0.0;
    for (int jj = 0; jj < nj; ++jj) acc = fma(sX[k + K * jj] * iSigma[j0 + jj], sX[nc + f + K * jj], acc);
    out[k + (size_t)ldcr * f] = acc;
  }
}

// The fused Eta kernel's per-sweep constants, formed once per sweep on the matrix cores by
// CRW_PARTS workgroups (instead of in each of the Eta kernel's ~600 workgroups):
//   CR = BL diag(iSigma) Lambda^T   (K x nf; rows nc.. are Q - I, Q = I + Lambda diag(iSigma) Lambda^T)
//   W  = L^-1, L L^T = Q            (16 x 16, row m at 16 m, zero padded)
//   LS = Lambda diag(iSigma)        ([species][16], the Eta stream's MFMA B operand)
// v_mfma_f64_16x16x4 over groups of 4 species: A[i][k] = BL[16 q + i, j0 + k] (tile q of the K
// rows), B[k][h] = iSigma_j Lambda[h, j] (= LS, written as it is formed).  Workgroup p, wave w
// take every (4 CRW_PARTS)-th species group, eight groups' loads in flight per lane; the
// waves' accumulators meet in LDS in wave order, the workgroups' partial tiles in global
// memory; the last workgroup through (a ticket) adds them in part order (deterministic) and
// factors Q in one wave's registers (wave_la.h).

template <int NFB>
__device__ __forceinline__ void crw_body(const CRWArgs& a, int p, double* smem) {
  __shared__ int s_last;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, lm = lane & 15, lk = lane >> 4;
  const int K = a.K, nc = a.nc, nf = a.nf, ns = a.ns, nq = (K + 15) >> 4;  // nq <= 4
  d4 acc[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) acc[q] = d4{0.0, 0.0, 0.0, 0.0};
  const int ng = (ns + 3) >> 2, gstride = 4 * CRW_PARTS;
  constexpr int D = 8;  // species groups' loads in flight per lane
  for (int g0 = 4 * p + w; g0 < ng; g0 += gstride * D) {
    double av[D][4], bv[D];
#pragma unroll
    for (int u = 0; u < D; ++u) {
      const int g = g0 + gstride * u, j = 4 * g + lk;
      const bool in = g < ng && j < ns;
      const double* col = a.BL + (size_t)K * (in ? j : 0);
#pragma unroll
      for (int q = 0; q < 4; ++q) av[u][q] = (in && q < nq && 16 * q + lm < K) ? col[16 * q + lm] : 0.0;
      bv[u] = (in && lm < nf) ? col[nc + lm] * a.iSigma[j] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < D; ++u) {
      const int g = g0 + gstride * u, j = 4 * g + lk;
      if (g < ng && j < ns) a.LS[(size_t)16 * j + lm] = bv[u];
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (q < nq) acc[q] = mfma_f64(av[u][q], bv[u], acc[q]);
    }
  }
  // acc[q][r] = partial CR[16 q + lk + 4 r][lm]: the waves' sum in LDS, then to this part's slot
  double* sAcc = smem;  // [wave][q][16 rows][16 cols]
#pragma unroll
  for (int q = 0; q < 4; ++q)
    if (q < nq)
#pragma unroll
      for (int r = 0; r < 4; ++r) sAcc[((w * 4 + q) * 16 + lk + 4 * r) * 16 + lm] = acc[q][r];
  __syncthreads();
  double* mine = a.part + (size_t)p * 4 * 256;
  for (int e = t; e < nq * 256; e += 256) {
    const int q = e >> 8, rc = e & 255;
    mine[e] = (sAcc[(0 * 4 + q) * 256 + rc] + sAcc[(1 * 4 + q) * 256 + rc]) +
              (sAcc[(2 * 4 + q) * 256 + rc] + sAcc[(3 * 4 + q) * 256 + rc]);
  }
  __threadfence();  // every wave's partial stores complete at device scope before the ticket
  __syncthreads();
  if (t == 0) s_last = __hip_atomic_fetch_add(a.ticket, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == CRW_PARTS - 1;
  __syncthreads();
  if (!s_last) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // every part's tiles
  double* sCR = smem + 4 * 4 * 256;  // [row k][16]
  for (int e = t; e < nq * 256; e += 256) {
    double v = 0.0;
#pragma unroll
    for (int q2 = 0; q2 < CRW_PARTS; ++q2) v += a.part[(size_t)q2 * 4 * 256 + e];
    sCR[e] = v;
    const int row = e >> 4, h = e & 15;
    if (row < K && h < nf) a.CR[row + (size_t)a.ldcr * h] = v;
  }
  __syncthreads();
  if (w == 0) {
    crw_finish<NFB>(a, sCR, a.W, sAcc);  // the wave partials are consumed: their LDS is the scratch
    if (lane == 0) __hip_atomic_store(a.ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
// LDS of crw_body (doubles): the waves' partial tiles, the reduced CR
constexpr int CRW_LDS = 4 * 4 * 256 + 4 * 16 * 16;

template <int NFB>
__global__ __launch_bounds__(256) void crw_kernel(CRWArgs a) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  crw_body<NFB>(a, blockIdx.x, smem);
}

__global__ __launch_bounds__(256) void cr_kernel(const double* BL, const double* iSigma, int K, int nc, int NF,
                                                 int ns_loc, double* CR_part, int ldcr, int slab, double* LS) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  cr_body(BL, iSigma, K, nc, NF, ns_loc, CR_part, ldcr, slab, LS, smem, blockIdx.x);
}

struct EtaArgs {
  EtaView ev;
  const double* XEta;  // ny x K materialised [X, Eta_1[Pi_1,], ...] (before this update)
  int r, nf, np, K, nc, NF, foff, loff, ldcr, nzl;
  const double* ZL;  // ny x NF (row-major per site), or partials [nzl][ny*NF]
  const double* CR;  // K x NF (ld ldcr)
  const int* unit_ptr;
  const int* unit_rows;
  const int8_t* row_na;   // ny (1 if any NA in row) or null
  const double* Mrow;     // per-row masked precision (nf*nf) for NA rows, indexed by row_slot
  const double* brow;     // per-row masked numerator (nf) for NA rows
  const int* row_slot;    // ny -> slot or -1
  double* Eta;            // np x nf
  Key key;
  uint32_t iter;
  const uint32_t* iter_dev;  // graph replay: the sweep counter is read from the device
  int noise_zero;
};

__global__ __launch_bounds__(64) void eta_unit_kernel(EtaArgs a) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int nf = a.nf, t = threadIdx.x, q = blockIdx.x;
  double* Q = smem;        // nf x nf
  double* b = Q + nf * nf; // nf
  int* flag = (int*)(b + nf + 1);
  const int rb = a.unit_ptr[q], re = a.unit_ptr[q + 1];
  int n_full = 0;
  for (int p = rb; p < re; ++p) n_full += (a.row_na && a.row_na[a.unit_rows[p]]) ? 0 : 1;
  for (int p = t; p < nf * nf; p += 64) {
    const int r1 = p % nf, c1 = p / nf;
    double v = (r1 == c1 ? 1.0 : 0.0) + n_full * a.CR[a.loff + r1 + (size_t)a.ldcr * (a.foff + c1)];
    if (a.row_na)
      for (int pp = rb; pp < re; ++pp) {
        const int slot = a.row_slot[a.unit_rows[pp]];
        if (slot >= 0) v += a.Mrow[(size_t)slot * nf * nf + p];
      }
    Q[p] = v;
  }
  for (int h = t; h < nf; h += 64) {
    double v = 0.0;
    for (int pp = rb; pp < re; ++pp) {
      const int i = a.unit_rows[pp];
      const int slot = a.row_na ? a.row_slot[i] : -1;
      if (slot >= 0) {
        v += a.brow[(size_t)slot * nf + h];
        continue;
      }
      double zl = 0.0;
      for (int c = 0; c < a.nzl; ++c) zl += a.ZL[(size_t)c * a.ev.ny * a.NF + (size_t)i * a.NF + a.foff + h];
      double corr = 0.0;
      for (int k = 0; k < a.K; ++k) {
        if (k >= a.loff && k < a.loff + nf) continue;
        corr += xeta_at(a.ev, i, k) * a.CR[k + (size_t)a.ldcr * (a.foff + h)];
      }
      v += zl - corr;
    }
    b[h] = v;
  }
  __syncthreads();
  wg_chol(Q, nf, nf, flag);                         // RiV = chol(iV)
  wg_forward(Q, nf, nf, b);
  for (int h = t; h < nf; h += 64)
    b[h] += a.noise_zero ? 0.0 : normal(a.key, (uint32_t)q, (uint32_t)h, S_ETA + LEVEL_STRIDE * a.r, SWEEP_ITER(a));
  __syncthreads();
  wg_backward_t(Q, nf, nf, b);                      // mu + t(backsolve(RiV, xi))
  for (int h = t; h < nf; h += 64) a.Eta[q + (size_t)a.np * h] = b[h];
}

// Fast path (no NA, every unit of level r has the same number n of rows, e.g. np == ny):
// all units share Q = I + n Lambda_r diag(iSigma) Lambda_r^T, so each workgroup (one wave)
// factors Q once in LDS and every lane solves one unit with the shared factor
// (R/updateEta.R:52-56).  The residual correction reads the materialised XEta (valid: Eta
// has not changed since it was built), so a lane's loads are plain column reads.
template <int NFB>
__global__ __launch_bounds__(64) void eta_shared_kernel(EtaArgs a, int nrow) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int nf = a.nf, K = a.K, t = threadIdx.x, ny = a.ev.ny;
  double* Q = smem;               // nf x nf -> lower L
  double* sCR = Q + nf * nf;      // K x nf   (column h of level r)
  int* flag = (int*)(sCR + K * nf + 1);
  if (blockIdx.x == 0) HMSC_STAMP(40);
  for (int p = t; p < K * nf; p += 64) {
    const int k = p % K, h = p / K;
    sCR[p] = a.CR[k + (size_t)a.ldcr * (a.foff + h)];
  }
  __syncthreads();
  for (int p = t; p < nf * nf; p += 64) {
    const int r1 = p % nf, c1 = p / nf;
    Q[p] = (r1 == c1 ? 1.0 : 0.0) + nrow * sCR[a.loff + r1 + K * c1];
  }
  __syncthreads();
  wg_chol(Q, nf, nf, flag);
  if (blockIdx.x == 0) HMSC_STAMP(41);
  const int q = blockIdx.x * 64 + t;
  if (q >= a.np) return;
  double b[NFB];
#pragma unroll
  for (int h = 0; h < NFB; ++h) b[h] = 0.0;
  for (int pp = a.unit_ptr[q]; pp < a.unit_ptr[q + 1]; ++pp) {
    const int i = a.unit_rows[pp];
    for (int c = 0; c < a.nzl; ++c) {
      const double* zl = a.ZL + (size_t)c * ny * a.NF + (size_t)i * a.NF + a.foff;
#pragma unroll
      for (int h = 0; h < NFB; ++h)
        if (h < nf) b[h] += zl[h];
    }
#pragma unroll 4
    for (int k = 0; k < K; ++k) {
      if (k >= a.loff && k < a.loff + nf) continue;
      const double x = a.XEta[i + (size_t)ny * k];
#pragma unroll
      for (int h = 0; h < NFB; ++h)
        if (h < nf) b[h] -= x * sCR[k + K * h];
    }
  }
  if (blockIdx.x == 0) HMSC_STAMP(42);
  // y = L^-1 b ; y += xi ; eta = L^-T y
#pragma unroll
  for (int h = 0; h < NFB; ++h) {
    if (h < nf) {
      double v = b[h];
#pragma unroll
      for (int k = 0; k < NFB; ++k)
        if (k < h) v -= Q[h + nf * k] * b[k];
      b[h] = v / Q[h + nf * h];
    }
  }
#pragma unroll
  for (int h = 0; h < NFB; ++h)
    if (h < nf && !a.noise_zero) b[h] += normal(a.key, (uint32_t)q, (uint32_t)h, S_ETA + LEVEL_STRIDE * a.r, SWEEP_ITER(a));
  if (blockIdx.x == 0) HMSC_STAMP(43);
#pragma unroll
  for (int h = NFB - 1; h >= 0; --h) {
    if (h < nf) {
      double v = b[h];
#pragma unroll
      for (int k = 0; k < NFB; ++k)
        if (k > h && k < nf) v -= Q[k + nf * h] * b[k];
      b[h] = v / Q[h + nf * h];
    }
  }
#pragma unroll
  for (int h = 0; h < NFB; ++h)
    if (h < nf) a.Eta[q + (size_t)a.np * h] = b[h];
  if (blockIdx.x == 0) HMSC_STAMP(44);
}

// NA rows (R/updateEta.R:59-70, :80-87): masked per-row precision and numerator
// with the residual S computed on the fly.  One workgroup per NA row.
__global__ __launch_bounds__(64) void eta_na_row_kernel(EtaView ev, int r, int nf, int K, int nc, int loff,
                                                        const int* na_rows, const double* Z, const double* BL,
                                                        const double* iSigma, const int8_t* Ycode, int ns_loc,
                                                        double* Mrow, double* brow) {
  const int slot = blockIdx.x, i = na_rows[slot], t = threadIdx.x, ny = ev.ny;
  extern __shared__ __attribute__((aligned(16))) double sx[];  // XEta row (K)
  for (int k = t; k < K; k += 64) sx[k] = xeta_at(ev, i, k);
  __syncthreads();
  for (int p = t; p < nf * nf + nf; p += 64) {
    double s = 0.0;
    if (p < nf * nf) {
      const int h1 = p % nf, h2 = p / nf;
      for (int j = 0; j < ns_loc; ++j)
        if (Ycode[(size_t)i + (size_t)ny * j] >= 0)
          s += BL[loff + h1 + (size_t)K * j] * iSigma[j] * BL[loff + h2 + (size_t)K * j];
      Mrow[(size_t)slot * nf * nf + p] = s;
    } else {
      const int h = p - nf * nf;
      for (int j = 0; j < ns_loc; ++j) {
        if (Ycode[(size_t)i + (size_t)ny * j] < 0) continue;
        double l = 0.0;  // L^{(-r)}_ij = XEta_i BL_j excluding level r
        for (int k = 0; k < K; ++k)
          if (k < loff || k >= loff + nf) l += sx[k] * BL[k + (size_t)K * j];
        s += (Z[(size_t)i + (size_t)ny * j] - l) * iSigma[j] * BL[loff + h + (size_t)K * j];
      }
      brow[(size_t)slot * nf + h] = s;
    }
  }
}

// ---------------------------------------------------------------------------
// Covariate-dependent level (R/updateEta.R:93-108).  The m levels r0 .. r0+m-1 of a group share
// Eta (np x nf, owned by r0); level r0+k scales its XEta columns by x[:, k] (EtaView::xs), so
// its BL rows are R's Lambda[,,k].  Per unit q, with lambdaLocal = sum_k x_qk Lambda_k:
//   Q_q = I + sum_{rows i of q} lambdaLocal diag(iSigma Yx_i) lambdaLocal^T
//   b_q = sum_{rows i of q} S_i diag(iSigma Yx_i) lambdaLocal^T,   S = Z - XEta_(-group) BL
//   eta_q = Q_q^-1 b_q + chol(Q_q)^-1 xi    (xi: normal(q, h, S_ETA + LEVEL_STRIDE r0))
// A row with every cell observed adds the CR blocks (the group's K rows are loff0 + k nf + f,
// its factor columns foff0 + k nf + f):
//   Q += sum_{k,k'} x_qk x_qk' CR[loff0 + k nf + f1, foff0 + k' nf + f2]
//   b += sum_k x_qk (ZL_i[foff0 + k nf + f] - sum_{c outside the group} XEta_ic CR[c, foff0 + k nf + f])
// and an NA row its masked terms from eta_na_row_x_kernel.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(64) void eta_na_row_x_kernel(EtaView ev, int r0, int m, int nf, int K, int loff0,
                                                          const int* na_rows, const double* Z, const double* BL,
                                                          const double* iSigma, const int8_t* Ycode, int ns_loc,
                                                          double* Mrow, double* brow) {
  const int slot = blockIdx.x, i = na_rows[slot], t = threadIdx.x, ny = ev.ny;
  extern __shared__ __attribute__((aligned(16))) double sx[];  // XEta row (K), then x_q (m)
  double* xq = sx + K;
  const int q = ev.Pi[r0][i], gend = loff0 + m * nf;
  for (int k = t; k < K; k += 64) sx[k] = xeta_at(ev, i, k);
  for (int k = t; k < m; k += 64) xq[k] = ev.xs[r0 + k][q];
  __syncthreads();
  auto lam_local = [&](int h, int j) {
    double v = 0.0;
    for (int k = 0; k < m; ++k) v += xq[k] * BL[loff0 + k * nf + h + (size_t)K * j];
    return v;
  };
  for (int p = t; p < nf * nf + nf; p += 64) {
    double acc = 0.0;
    if (p < nf * nf) {
      const int h1 = p % nf, h2 = p / nf;
      for (int j = 0; j < ns_loc; ++j)
        if (Ycode[(size_t)i + (size_t)ny * j] >= 0) acc += lam_local(h1, j) * iSigma[j] * lam_local(h2, j);
      Mrow[(size_t)slot * nf * nf + p] = acc;
    } else {
      const int h = p - nf * nf;
      for (int j = 0; j < ns_loc; ++j) {
        if (Ycode[(size_t)i + (size_t)ny * j] < 0) continue;
        double l = 0.0;  // the linear predictor without the group's columns
        for (int c = 0; c < K; ++c)
          if (c < loff0 || c >= gend) l += sx[c] * BL[c + (size_t)K * j];
        acc += (Z[(size_t)i + (size_t)ny * j] - l) * iSigma[j] * lam_local(h, j);
      }
      brow[(size_t)slot * nf + h] = acc;
    }
  }
}

__global__ __launch_bounds__(64) void eta_unit_x_kernel(EtaArgs a, int m) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int nf = a.nf, t = threadIdx.x, q = blockIdx.x, gend = a.loff + m * nf;
  double* Q = smem;         // nf x nf
  double* b = Q + nf * nf;  // nf
  double* xq = b + nf;      // m
  int* flag = (int*)(xq + m + 1);
  for (int k = t; k < m; k += 64) xq[k] = a.ev.xs[a.r + k][q];
  __syncthreads();
  const int rb = a.unit_ptr[q], re = a.unit_ptr[q + 1];
  int n_full = 0;
  for (int p = rb; p < re; ++p) n_full += (a.row_na && a.row_na[a.unit_rows[p]]) ? 0 : 1;
  for (int p = t; p < nf * nf; p += 64) {
    const int r1 = p % nf, c1 = p / nf;
    double g = 0.0;
    for (int k = 0; k < m; ++k)
      for (int k2 = 0; k2 < m; ++k2)
        g += xq[k] * xq[k2] * a.CR[a.loff + k * nf + r1 + (size_t)a.ldcr * (a.foff + k2 * nf + c1)];
    double v = (r1 == c1 ? 1.0 : 0.0) + n_full * g;
    if (a.row_na)
      for (int pp = rb; pp < re; ++pp) {
        const int slot = a.row_slot[a.unit_rows[pp]];
        if (slot >= 0) v += a.Mrow[(size_t)slot * nf * nf + p];
      }
    Q[p] = v;
  }
  for (int h = t; h < nf; h += 64) {
    double v = 0.0;
    for (int pp = rb; pp < re; ++pp) {
      const int i = a.unit_rows[pp];
      const int slot = a.row_na ? a.row_slot[i] : -1;
      if (slot >= 0) {
        v += a.brow[(size_t)slot * nf + h];
        continue;
      }
      for (int k = 0; k < m; ++k) {
        const int col = a.foff + k * nf + h;
        double zl = 0.0;
        for (int c = 0; c < a.nzl; ++c) zl += a.ZL[(size_t)c * a.ev.ny * a.NF + (size_t)i * a.NF + col];
        double corr = 0.0;
        for (int kk = 0; kk < a.K; ++kk) {
          if (kk >= a.loff && kk < gend) continue;
          corr += xeta_at(a.ev, i, kk) * a.CR[kk + (size_t)a.ldcr * col];
        }
        v += xq[k] * (zl - corr);
      }
    }
    b[h] = v;
  }
  __syncthreads();
  wg_chol(Q, nf, nf, flag);                         // RiV = chol(iV)   (:103)
  wg_forward(Q, nf, nf, b);
  for (int h = t; h < nf; h += 64)
    b[h] += a.noise_zero ? 0.0 : normal(a.key, (uint32_t)q, (uint32_t)h, S_ETA + LEVEL_STRIDE * a.r, SWEEP_ITER(a));
  __syncthreads();
  wg_backward_t(Q, nf, nf, b);                      // mu + t(backsolve(RiV, rnorm))   (:106-107)
  for (int h = t; h < nf; h += 64) a.Eta[q + (size_t)a.np * h] = b[h];
}

// ---------------------------------------------------------------------------
// Fused updateEta for the common case -- one random level with np == ny (one row per
// unit), no NA, one rank (R/updateEta.R:42-57).  One 256-thread workgroup per 16-site tile:
//   1. ZL_i = sum_j Z_ij LS_j, LS = Lambda diag(iSigma)  (:55), on the matrix cores: wave w
//      takes every 4th group of 4 species, A = Z (16 sites x 4 species, loaded straight from
//      HBM as 128-B site runs), B = LS (4 species x 16 factors, from L2); the 4 waves'
//      partials meet in LDS
//   2. b_i = ZL_i - sum_{k < nc} XEta_ik CR_k  (the residual S of :31-37), and the noise
//      xi_q for q = Pi_i (:56), one (site, factor) pair per thread
//   3. eta_q = L^-T (L^-1 b_i + xi_q), L = chol(I + Lambda diag(iSigma) Lambda^T) (:45-56),
//      factored once per tile by wave 0
//   4. the tile's XEta rows get the new Eta (R/updateBetaLambda.R:21-41 of the next sweep)
//      and the tile's Gram partial Eta^T XEta (nf x K; X^T X is constant) goes to G_part[tile]
// This replaces zl_kernel + eta_shared_kernel + xeta_gram_kernel (and their Z / XEta
// re-reads) with one pass over Z.
// ---------------------------------------------------------------------------
struct EtaFArgs {
  const double* Z;
  const double* LS;   // ns_loc x 16: Lambda diag(iSigma), zero past nf (cr_body)
  const double* CR;   // Kmax x NF (ld ldcr): CR = BL diag(iSigma) Lambda^T (crw_body)
  const double* W;    // 16 x 16: L^-1 of Q = I + Lambda diag(iSigma) Lambda^T, row m at 16 m (crw_body)
  double* XEta;       // ny x K (ld ny)
  const int* Pi;      // ny: unit of each row (0-based)
  double* Eta;        // np x nf
  double* G_part;     // [tile][K x nf]  (Eta^T XEta partial, ld Kmax)
  double* ZL;         // sharded chain: ZL [site][nf] -- written by the stream (EF_STREAM), read by the solve (EF_SOLVE)
  int ny, ns_loc, K, Kmax, nc, nf, np, ldcr;
  Key key;
  uint32_t iter;
  const uint32_t* iter_dev;  // graph replay: the sweep counter is read from the device
  int noise_zero;
  unsigned long long* kt;    // live launch timing (KT_ETA block) or null
  // EF_DEFER: the BetaLambda tail's two reduction levels run in workgroups 0 .. nred - 1 (one
  // per group of CRW_GROUP BetaLambda workgroups, nbl of them); the tile workgroups after them
  // stream Z meanwhile and wait for tail.tails_flag before reading CR and W
  BLTailArgs tail;
  int nred, nbl;
  int* err;
  // EF_SOLVE of an edge-free sharded sweep graph: raised (this sweep's epoch) at the launch's
  // start, i.e. after all-reduce B, for the side chain that reads ar_b (sweep_sharded)
  int* arb_flag;
  // EF_DEFER: npre workgroups between the reducers and the tile workgroups draw the next
  // sweep's BetaLambda noise and psi gamma variates (bl_predraw_body) into pre_buf (last in
  // dispatch order they outlasted the tiles: Eta end -> z start 3.4 -> 6.8 us)
  double* pre_buf;
  int* pre_tag;
  int npre, ntile;
  int red_prio;
};

// The next sweep's BetaLambda draws, made while this launch streams Z, into [species][64]:
// slot k < K the noise xi_k of R/updateBetaLambda.R:101, slot 32 + f factor f's standard
// gamma variate of R/updateLambdaPriors.R:22-24 (psi = variate / rate, in the tail).  Same
// (key, index, stream, sweep) as the in-kernel draws, so the same bits; the BetaLambda
// prologue (on the sweep's critical path) then loads them instead of drawing (~2 us of its
// chain at config 4).  The ns K normals first, then the ns (K - nc) gamma variates, spread
// over every thread of the npre workgroups, so a wave draws one kind (no divergence between
// the two samplers).
__device__ void bl_predraw_body(const EtaFArgs& a, int bid) {
  const uint32_t it = SWEEP_ITER(a) + 1;
  const BLTailArgs& ta = a.tail;
  const int K = a.K, nc = a.nc, nl = K - nc;
  const int nN = a.ns_loc * K, nG = a.ns_loc * nl;
  for (int q = bid * 256 + (int)threadIdx.x; q < nN + nG; q += a.npre * 256) {
    double v;
    int j, slot;
    if (q < nN) {
      j = q / K;
      slot = q - j * K;
      v = a.noise_zero ? 0.0 : normal(a.key, (uint32_t)(ta.sp0 + j), (uint32_t)slot, S_BETALAMBDA, it);
    } else {
      j = (q - nN) / nl;
      const int f = q - nN - j * nl;
      slot = 32 + f;
      v = psi_gamma_std(ta, it, j, f);
    }
    a.pre_buf[(size_t)j * 64 + slot] = v;
  }
  if (bid == 0 && threadIdx.x == 0) {  // read after this launch's boundary
    a.pre_tag[0] = (int)it;
    a.pre_tag[1] = K;
  }
}

constexpr int EF_SITES = 16;
// EF_FUSED: the one-pass kernel above.  A species-sharded chain splits it at the all-reduce
// of ZL (a sum over every rank's species): EF_STREAM is stage 1 alone over this rank's species,
// its 4 waves' partials added in the fused kernel's order and stored as ZL [site][nf];
// EF_SOLVE is stages 2-4 on the all-reduced ZL and CR, each workgroup forming W = L^-1 itself
// (one wave, the BetaLambda tail's factorization) -- on one rank the pair reproduces the
// fused kernel bit for bit.
// EF_DEFER: EF_FUSED with the BetaLambda tail's reductions folded in (EtaFArgs::nred), so the
// Gamma2 + BetaLambda launch ends with its bodies and this launch's Z stream overlaps the
// reductions and Q's factorization instead of following them.
enum EtaMode { EF_FUSED = 0, EF_STREAM = 1, EF_SOLVE = 2, EF_DEFER = 3 };
template <int NFB>
constexpr int ef_lds_doubles() {
  return 4 * 16 * (EF_SITES + 1) + NFB * NFB + 3 * NFB * EF_SITES + 64 * (EF_SITES + 1) + 64 * NFB;
}
static_assert(ef_lds_doubles<8>() >= 4 * CRW_TILE + 32 * 16 + 256, "EF_DEFER reducers: LDS scratch");

// __launch_bounds__(256, 3): <= 168 VGPRs, three waves per SIMD, so the 625 workgroups of the
// synthetic config (2500 waves) are resident in one round (at 196 VGPRs they took two: 33 ->
// 29 us).  A fifth wave doing the Z-independent work during the stream measured slower (49 us).
// The stream's depth: EF_DEPTH 16-species steps' loads in flight per lane before their MFMAs
// (16, and a software-pipelined stream of two 6- or 8-step batches, measured the same within
// 1 %: the stream is not bound by the loads a wave has in flight, profiles/r05_eta_ab.txt).
#ifndef EF_DEPTH
#define EF_DEPTH 12
#endif
template <int NFB, int MODE>
__global__ __launch_bounds__(256, 3) void eta_fused_kernel(EtaFArgs a) {
  kernarg_warm<sizeof(EtaFArgs)>();
  // one block carved into the stages' arrays (EF_DEFER's reducer workgroups: their scratch)
  __shared__ __attribute__((aligned(16))) double sAll[ef_lds_doubles<NFB>()];
  double(*sPart)[16][EF_SITES + 1] = reinterpret_cast<double(*)[16][EF_SITES + 1]>(sAll);  // [wave][factor][site] ZL partials (EF_SOLVE: W's scratch)
  double* sW = sAll + 4 * 16 * (EF_SITES + 1);  // W = L^-1, L the lower factor of Q (row m at m NFB)
  double(*sB)[EF_SITES] = reinterpret_cast<double(*)[EF_SITES]>(sW + NFB * NFB);
  double(*sXi)[EF_SITES] = sB + NFB;
  double(*sU)[EF_SITES] = sXi + NFB;
  double(*sX)[EF_SITES + 1] = reinterpret_cast<double(*)[EF_SITES + 1]>(&sU[NFB][0]);  // XEta tile [k][site] (K <= 64)
  double* sCR = &sX[64][0];  // CR[k][h], k < K
  __shared__ int sPi[EF_SITES];  // the tile's units
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, lm = lane & 15, lk = lane >> 4;
  if (MODE == EF_DEFER && blockIdx.x < a.nred) {  // the BetaLambda tail's reductions
    if (a.red_prio) __builtin_amdgcn_s_setprio(3);  // (HMSC_RED_PRIO=1: issue ahead of the streams)
    const bool two = a.tail.defer == 2;
    if (two) {  // group blockIdx.x's tiles, then the last group through sums the group tiles
      __shared__ int s_last;
      tail_group_sum(a.tail, blockIdx.x, a.nbl, false, true);
      vm_stores_done();
      __syncthreads();
      if (t == 0)
        s_last = __hip_atomic_fetch_add(&a.tail.crw.ticket[1], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == a.nred - 1;
      __syncthreads();
      if (!s_last) return;
    }
    tail_final(a.tail, a.nbl, SWEEP_ITER(a), sAll, true, two, two);
    return;
  }
  if (MODE == EF_DEFER && (int)blockIdx.x < a.nred + a.npre) {  // (after the reducers, ahead of the tiles)
    bl_predraw_body(a, (int)blockIdx.x - a.nred);
    return;
  }
  const int tile = MODE == EF_DEFER ? blockIdx.x - a.nred - a.npre : blockIdx.x;
  const unsigned long long kt0 = a.kt ? kt_now() : 0ull;
  const int ny = a.ny, nf = a.nf, K = a.K, nc = a.nc, ns = a.ns_loc;
  const int i0 = tile * EF_SITES;
  if (tile == 0) HMSC_STAMP(50);
  const uint32_t iter = SWEEP_ITER(a);       // read once, ahead of the stream
  if (MODE == EF_SOLVE && a.arb_flag && tile == 0 && t == 0)  // all-reduce B is in (stream order)
    __hip_atomic_store(a.arb_flag, g2bl_epoch(iter), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  if (MODE != EF_STREAM && t < EF_SITES) sPi[t] = i0 + t < ny ? a.Pi[i0 + t] : 0;
  // ---- stage 1: ZL = Z (Lambda diag(iSigma))^T on the matrix cores, the HBM stream of the
  // launch, issued first: species j = 16 s + 4 w + lk, B = LS[j][lm] straight from L2 (128 KB,
  // shared by every workgroup); eight steps' loads in flight before their MFMAs
  d4 acc = {0.0, 0.0, 0.0, 0.0};
  // the tile's X columns (the residual's fixed part and the Gram tile), loaded before the
  // stream so they arrive during it: nc x 16 values, at most 4 per thread (nc < 64)
  double xr[4] = {0.0, 0.0, 0.0, 0.0};
  if (MODE != EF_STREAM)
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int p = t + 256 * u, s2 = p % EF_SITES, k = p / EF_SITES, ii = i0 + s2;
      xr[u] = (k < nc && ii < ny) ? a.XEta[ii + (size_t)ny * k] : 0.0;
    }
  // CR (K x nf) and W (nf x nf) of this sweep, formed once by crw_body: loads issued here,
  // ahead of the stream, stored to LDS after it
  double crv[4] = {0.0, 0.0, 0.0, 0.0}, wv[NFB * NFB / 256 + 1];
  if (MODE == EF_FUSED || MODE == EF_SOLVE)
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int p = t + 256 * u, k = p % K, h = p / K;
      crv[u] = p < K * nf ? a.CR[k + (size_t)a.ldcr * h] : 0.0;
    }
#pragma unroll
  for (int u = 0; u < NFB * NFB / 256 + 1; ++u) {
    const int p = t + 256 * u, m = p / NFB, c = p % NFB;
    wv[u] = (MODE == EF_FUSED && p < NFB * NFB) ? a.W[m * 16 + c] : 0.0;
  }
  // EF_SOLVE: the tile's all-reduced ZL (16 sites x nf, contiguous), one element per thread
  double zlv = 0.0;
  if (MODE == EF_SOLVE && t < EF_SITES * nf) {
    const int s2 = t % EF_SITES, h = t / EF_SITES;
    zlv = i0 + s2 < ny ? a.ZL[(size_t)(i0 + s2) * nf + h] : 0.0;
  }
  const double* zc = a.Z + min(i0 + lm, ny - 1);  // sites past ny: any finite row, unused
  const int nsteps = MODE == EF_SOLVE ? 0 : (ns + 15) >> 4;
  // the per-site noise of stage 2 (one (site, factor) pair per thread, t < EF_SITES nf <= 256):
  // drawn while the stream's first loads are in flight instead of after the stream
  double xi_pre = 0.0;
  const int xs2 = t % EF_SITES, xh = t / EF_SITES;
  const bool x_on = MODE != EF_STREAM && t < EF_SITES * nf && i0 + xs2 < ny && !a.noise_zero;
  const int x_unit = x_on ? a.Pi[i0 + xs2] : 0;
  int s = 0;
  for (; s + EF_DEPTH <= nsteps; s += EF_DEPTH) {
    double zv[EF_DEPTH], lv[EF_DEPTH];
#pragma unroll
    for (int u = 0; u < EF_DEPTH; ++u) {
      const int j = 16 * (s + u) + 4 * w + lk;
      zv[u] = j < ns ? zc[(size_t)ny * j] : 0.0;
      lv[u] = j < ns ? a.LS[(size_t)16 * j + lm] : 0.0;
    }
    if (s == 0 && x_on) xi_pre = normal(a.key, (uint32_t)x_unit, (uint32_t)xh, S_ETA, iter);
#pragma unroll
    for (int u = 0; u < EF_DEPTH; ++u) acc = mfma_f64(zv[u], lv[u], acc);
  }
  if (s == 0 && x_on) xi_pre = normal(a.key, (uint32_t)x_unit, (uint32_t)xh, S_ETA, iter);  // (a short stream)
  for (; s < nsteps; s += 8) {  // the tail: eight steps' loads at once
    double zv[8], lv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int j = 16 * (s + u) + 4 * w + lk;
      const bool in = s + u < nsteps && j < ns;
      zv[u] = in ? zc[(size_t)ny * j] : 0.0;
      lv[u] = in ? a.LS[(size_t)16 * j + lm] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) acc = mfma_f64(zv[u], lv[u], acc);
  }
  // acc[r] = partial ZL[site lk + 4 r][factor lm]
  if (MODE != EF_SOLVE)
#pragma unroll
    for (int r = 0; r < 4; ++r) sPart[w][lm][lk + 4 * r] = acc[r];
  if (MODE == EF_STREAM) {  // this rank's ZL, the 4 waves' partials added as stage 2 adds them
    __syncthreads();
    for (int p = t; p < EF_SITES * nf; p += 256) {
      const int s2 = p % EF_SITES, h = p / EF_SITES, ii = i0 + s2;
      const double zl = (sPart[0][h][s2] + sPart[1][h][s2]) + (sPart[2][h][s2] + sPart[3][h][s2]);
      if (ii < ny) a.ZL[(size_t)ii * nf + h] = zl;
    }
    if (a.kt) {
      __syncthreads();
      if (t == 0) kt_record(a.kt, iter, kt0);
    }
    return;
  }
  if (MODE == EF_DEFER) {  // CR and W of this sweep: out once the tail's last reducer raises the flag
    if (t == 0 && !spin_until<2>([&] {
          return __hip_atomic_load(a.tail.crw_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == g2bl_epoch(iter);
        }))
      __hip_atomic_store(&a.err[3], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int p = t + 256 * u, k = p % K, h = p / K;
      crv[u] = p < K * nf ? load_coherent(a.CR + k + (size_t)a.ldcr * h) : 0.0;
    }
#pragma unroll
    for (int u = 0; u < NFB * NFB / 256 + 1; ++u) {
      const int p = t + 256 * u, m = p / NFB, c = p % NFB;
      wv[u] = p < NFB * NFB ? load_coherent(a.W + m * 16 + c) : 0.0;
    }
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int p = t + 256 * u, s2 = p % EF_SITES, k = p / EF_SITES;
    if (k < nc) sX[k][s2] = xr[u];
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int p = t + 256 * u, k = p % K, h = p / K;
    if (p < K * nf) sCR[k * NFB + h] = crv[u];
  }
  if (MODE == EF_FUSED || MODE == EF_DEFER)
#pragma unroll
    for (int u = 0; u < NFB * NFB / 256 + 1; ++u) {
      const int p = t + 256 * u;
      if (p < NFB * NFB) sW[p] = wv[u];
    }
  __syncthreads();
  if (MODE == EF_SOLVE) {  // W = L^-1 of Q = I + (rows nc.. of CR), one wave, into sW (rows m < NFB)
    if (w == 0) q_inv_factor_nf(sCR + nc * NFB, NFB, nf, sW, NFB, NFB, sAll);
    __syncthreads();
  }
  if (tile == 0) HMSC_STAMP(51);
  // ---- stage 2: b = ZL - X CR_x, and the noise, one (site, factor) per thread
  for (int p = t; p < EF_SITES * nf; p += 256) {
    const int s2 = p % EF_SITES, h = p / EF_SITES, ii = i0 + s2;
    const double zl = MODE == EF_SOLVE ? zlv : (sPart[0][h][s2] + sPart[1][h][s2]) + (sPart[2][h][s2] + sPart[3][h][s2]);
    double corr = 0.0, xi = 0.0;
    if (ii < ny) {
      // X from the tile staged in LDS (a global load per term here waited out one L2
      // round trip per covariate: ~6 us of the kernel's serial tail); eight terms' LDS reads
      // issued before their FMAs (a read-FMA chain waited one LDS latency per covariate:
      // stage 2 took ~3.9 k cycles of tile 0's ~39 k, scripts/stamps_sweep.py), same order
      int k = 0;
      for (; k + 8 <= nc; k += 8) {
        double xv[8], cv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          xv[u] = sX[k + u][s2];
          cv[u] = sCR[(k + u) * NFB + h];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) corr = fma(xv[u], cv[u], corr);
      }
      for (; k < nc; ++k) corr = fma(sX[k][s2], sCR[k * NFB + h], corr);
      xi = p == t ? xi_pre : (a.noise_zero ? 0.0 : normal(a.key, (uint32_t)sPi[s2], (uint32_t)h, S_ETA, iter));
    }
    sB[h][s2] = zl - corr;
    sXi[h][s2] = xi;
  }
  __syncthreads();
  if (tile == 0) HMSC_STAMP(53);
  // ---- stage 3: eta = L^-T (L^-1 b + xi) = W^T (W b + xi), two matrix-vector phases over
  // the (factor, site) pairs (no serial substitution chain)
  // (every LDS operand of a thread's chain read before the chain, as in stage 2; same order)
  for (int p = t; p < EF_SITES * nf; p += 256) {
    const int s2 = p % EF_SITES, m = p / EF_SITES;
    double u = sXi[m][s2], wv[NFB], bv[NFB];
#pragma unroll
    for (int k = 0; k < NFB; ++k) {
      wv[k] = k <= m ? sW[m * NFB + k] : 0.0;
      bv[k] = k <= m ? sB[k][s2] : 0.0;
    }
#pragma unroll
    for (int k = 0; k < NFB; ++k)
      if (k <= m) u = fma(wv[k], bv[k], u);
    sU[m][s2] = u;
  }
  __syncthreads();
  for (int p = t; p < EF_SITES * nf; p += 256) {
    const int s2 = p % EF_SITES, h = p / EF_SITES, ii = i0 + s2;
    double e = 0.0, wv[NFB], uv[NFB];
#pragma unroll
    for (int m = 0; m < NFB; ++m) {
      wv[m] = (m >= h && m < nf) ? sW[m * NFB + h] : 0.0;
      uv[m] = (m >= h && m < nf) ? sU[m][s2] : 0.0;
    }
#pragma unroll
    for (int m = 0; m < NFB; ++m)
      if (m >= h && m < nf) e = fma(wv[m], uv[m], e);
    if (ii < ny) {
      a.Eta[sPi[s2] + (size_t)a.np * h] = e;
      a.XEta[ii + (size_t)ny * (nc + h)] = e;
    }
    sX[nc + h][s2] = ii < ny ? e : 0.0;
  }
  __syncthreads();
  if (tile == 0) HMSC_STAMP(54);
  // ---- stage 4: Gram partial of the tile's Eta rows, Eta^T XEta (nf x K, ld Kmax)
  double* dst = a.G_part + (size_t)tile * a.Kmax * nf;
  for (int p = t; p < K * nf; p += 256) {
    const int k = p % K, h = p / K;
    double g = 0.0;
#pragma unroll
    for (int s2 = 0; s2 < EF_SITES; ++s2) g = fma(sX[nc + h][s2], sX[k][s2], g);
    dst[k + a.Kmax * h] = g;
  }
  if (tile == 0) HMSC_STAMP(55);
  if (a.kt) {
    __syncthreads();
    if (t == 0) kt_record(a.kt, iter, kt0);
  }
}

// ---------------------------------------------------------------------------
// Co-launched side updaters.  After BetaLambda a sweep has the fused updateEta on the
// critical path (its constants CR, W, LS already formed in the BetaLambda launch's tail,
// crw_tail) and, off it, two species-parallel passes -- the GammaV partials
// (R/updateGammaV.R:17-19) and the psi draws of updateLambdaPriors (:22-24) -- followed by
// two small serial tails, the GammaV algebra and the delta chain (:25-32).  The passes share
// one launch (post_bl_kernel) and the tails another (side_chain_kernel, one workgroup each),
// both on the side stream.  Eager sweeps and a capture's first sweep fork them behind one
// event after BetaLambda and join the side stream before the next sweep's Gamma2 +
// BetaLambda launch; later graph sweeps do both on the device (post_bl_kernel waits for the
// fused launch's tails flag, the next fused launch for the side chain's side_sync flags).
// ---------------------------------------------------------------------------
struct PostBLArgs {
  const double* BL;
  const double* iSigma;
  int K, nc, NF, ns_loc;
  int nt, n_gv;
  const double* Gamma;
  const double* Tr;
  double* gv_part;
  LPArgs lp;
  int n_psi;
  const uint32_t* iter_src;  // graph replay: d_iter, snapshotted into iter_side for the side stream
  uint32_t* iter_side;
  // graph sweeps after the first (edge-free): not behind a graph edge from the fused Gamma2 +
  // BetaLambda launch; every workgroup waits for that launch's tails flag (its last reducer,
  // after every BetaLambda workgroup's write-through column stores) and reads BL and Gamma
  // with device-coherent loads
  const int* tails_flag;
  int* err;
};

// workgroup b < n_gv: GammaV partial block b; b < n_psi: psi part b
__global__ __launch_bounds__(256) void post_bl_kernel(PostBLArgs a) {
  kernarg_warm<sizeof(PostBLArgs)>();
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int b = blockIdx.x;
  const bool coh = a.tails_flag != nullptr;
  if (b == 0 && threadIdx.x < 64) HMSC_STAMP_RT(89);
  if (coh) {
    if (threadIdx.x == 0) side_wait(a.tails_flag, 1, g2bl_epoch(SWEEP_ITER(a.lp)), a.err);
    __syncthreads();
  }
  if (b == 0 && threadIdx.x < 64) HMSC_STAMP_RT(90);
  if (b == 0 && threadIdx.x == 0 && a.iter_src) *a.iter_side = *a.iter_src;
  // workgroup b: the GammaV partial of species block b, then the psi draws of its own species
  // range (one launch of ceil(ns / SB) workgroups beside Eta and z, not one per pass)
  if (b < a.n_gv) gammav_partial_body(a.BL, a.K, a.nc, a.nt, a.ns_loc, a.Gamma, a.Tr, a.gv_part, smem, b, coh);
  if (b < a.n_psi) {
    if (b < a.n_gv) __syncthreads();
    psi_body(a.lp, b, a.n_psi, coh);
  }
}

static bool eta_fused_ok(const State& s);
static void launch_eta_fused(State& s, uint32_t iter, bool cr_done, bool defer, bool tail_gv);

static CRWArgs make_crw_args(const State& s) {
  CRWArgs c{};
  c.BL = s.BL;
  c.iSigma = s.iSigma;
  c.K = s.K;
  c.nc = s.nc;
  c.nf = s.lev[0].nf;
  c.ns = s.nsl;
  c.ldcr = s.Kmax;
  c.CR = s.CR;
  c.W = s.etaW;
  c.LS = s.LS;
  c.part = s.crw_part;
  c.ticket = s.crw_ticket;
  return c;
}

bool side_fusion_ok(const State& s) {
  const uint32_t need = HMSC_UP_GAMMAV | HMSC_UP_LAMBDAPRIORS | HMSC_UP_ETA;
  return (s.mask & need) == need && !s.single_stream && !s.phylo && s.nc * s.nt <= 32 && s.NF <= 64 && eta_fused_ok(s) &&
         !getenv_flag("HMSC_NO_SIDE_FUSION");
}

// GammaV + LambdaPriors + Eta of one sweep (BetaLambda done), main stream + one side launch
template <int NM>
static void launch_side_chain(State& s, const GVWArgs& gw, const LPArgs& lp, const double* rs, int nparts, int rs_ld,
                              const int* tails_flag) {
  side_chain_kernel<NM><<<1 + s.nr, 256, 0, s.side>>>(gw, lp, rs, nparts, rs_ld, tails_flag, s.gbl_sync,
                                                      s.kt_on ? s.d_kt + (size_t)KT_SIDE * 2 * KT_SLOTS : nullptr);
}

// GammaV + LambdaPriors + Eta of one sweep (BetaLambda done), main stream + the side stream
void launch_side_fused(State& s, uint32_t iter) {
  if (!s.xeta_valid) launch_xeta(s);
  // the main continuation is captured before the side branch (the graph executor keeps the
  // first-created child of a node on its parent's queue, so the critical path stays on one
  // queue); CR, W and LS come from the fused Gamma2 + BetaLambda launch's tail when it formed
  // them, else from crw_kernel ahead of the Eta kernel
  const bool cr_done = s.crw_fresh, tail = s.tail_gv;
  s.crw_fresh = false;
  s.tail_gv = false;
  // graph sweeps after the first: the side work is not forked by a graph edge; its first
  // launch waits on the device for the fused launch's tails flag (raised by the last reducer
  // of the tail, after every BetaLambda workgroup's stores), see State::cap_sweep
  const bool dev_fork = cr_done && s.edge_free_now && s.capturing && (s.cap_sweep > 0 || s.side_root);
  const bool defer = cr_done && s.tail_defer;
  s.tail_defer = false;
  HMSC_REQUIRE(!defer || dev_fork, "fused Eta: the tail's reductions deferred to a launch the side work is not forked from");
  if (!dev_fork) HIP_OK(hipEventRecord(s.ev_bl, s.stream));
  launch_eta_fused(s, iter, cr_done, defer, tail);
  if (!dev_fork) HIP_OK(hipStreamWaitEvent(s.side, s.ev_bl, 0));
  LPArgs lp = make_lp_args(s, iter);
  const double* rs;
  int nparts, rs_ld;
  GVWArgs gw;
  if (tail) {
    // the BetaLambda tail's group tiles: [A nc^2 | BTr nc nt | rs NF], ld gvt_ld
    const int nbl = (s.nsl + 3) / 4, ngr = (nbl + CRW_GROUP - 1) / CRW_GROUP;
    const double* gt = s.gvt + (size_t)nbl * s.gvt_ld;
    gw = make_gvw_args(s, iter, gt, ngr, s.capturing ? s.d_iter : nullptr);
    gw.part_ld = s.gvt_ld;
    gw.flags = s.side_sync;
    rs = gt + s.nc * s.nc + s.nc * s.nt;
    nparts = ngr;
    rs_ld = s.gvt_ld;
  } else {
    // the species partials of GammaV and LambdaPriors first (post_bl_kernel), on the side stream
    const int ngv = (s.nsl + SB - 1) / SB;
    const int npsi = std::max(1, std::min({ngv, LP_PARTS, s.nsl}));  // psi_rs holds LP_PARTS rows
    PostBLArgs a{};
    a.BL = s.BL;
    a.iSigma = s.iSigma;
    a.K = s.K;
    a.nc = s.nc;
    a.NF = s.NF;
    a.ns_loc = s.nsl;
    a.nt = s.nt;
    a.n_gv = ngv;
    a.Gamma = s.Gamma;
    a.Tr = s.Tr;
    a.gv_part = s.gv_part;
    a.lp = lp;
    a.n_psi = npsi;
    a.iter_src = s.capturing ? s.d_iter : nullptr;
    a.iter_side = s.d_iter_side;
    a.tails_flag = dev_fork ? s.gbl_sync + 2 : nullptr;
    a.err = s.gbl_sync;
    const size_t smem = (size_t)(2 * s.nc * SB + SB * s.nt) * sizeof(double);
    post_bl_kernel<<<std::max(ngv, npsi), 256, smem, s.side>>>(a);
    HIP_OK(hipGetLastError());
    gw = make_gvw_args(s, iter, s.gv_part, ngv, s.capturing ? s.d_iter_side : nullptr);
    rs = s.psi_rs;
    nparts = npsi;
    rs_ld = s.NF;
  }
  // the side chain publishes Gamma / iV, its Gamma2 prep and each level's Delta through
  // side_sync, so the next graph sweep's fused launch can join it on the device
  if (cr_done) gw.flags = s.side_sync;
  s.side_tail = cr_done;
  s.psi_side = !tail;
  lp.iter_dev = gw.iter_dev;
  // the GammaV algebra (writes Gamma, iV and Gamma2's prep) with the delta chains as extra
  // workgroups of the same launch
  const int* tf = (dev_fork && tail) ? s.gbl_sync + 2 : nullptr;  // (else post_bl_kernel waited)
  auto launch = [&s](GVWArgs g, LPArgs l, const double* r, int np, int ld, const int* f) {
    switch (wv_bucket_gv(s.nc * s.nt)) {
      case 8: launch_side_chain<8>(s, g, l, r, np, ld, f); break;
      case 16: launch_side_chain<16>(s, g, l, r, np, ld, f); break;
      case 20: launch_side_chain<20>(s, g, l, r, np, ld, f); break;
      case 24: launch_side_chain<24>(s, g, l, r, np, ld, f); break;
      default: launch_side_chain<32>(s, g, l, r, np, ld, f); break;
    }
    HIP_OK(hipGetLastError());
  };
  if (gw.do_prep) s.g2prep_valid = true;
  // a capture's first sweep, side stream forked at the root: the side chain is left out of the
  // graph and launched ahead of each replay (State::ext_side), reading the sweep counter the
  // replay writes to d_ext_iter
  if (s.capturing && s.cap_sweep == 0 && s.side_root && dev_fork && tail && !getenv_flag("HMSC_NO_EXT_SIDE")) {
    GVWArgs g2 = gw;
    LPArgs l2 = lp;
    g2.iter_dev = s.d_ext_iter;
    l2.iter_dev = s.d_ext_iter;
    s.ext_pending = [launch, g2, l2, rs, nparts, rs_ld, tf] { launch(g2, l2, rs, nparts, rs_ld, tf); };
    return;
  }
  launch(gw, lp, rs, nparts, rs_ld, tf);
  s.side_pending |= 1;  // joined (ev_side recorded) by the next join_side
}

// G = XEta^T XEta after the fused Eta pass: the X^T X block is the constant s.XX, the Eta
// rows the sum of the tiles' partials G_part[tile][k + Kmax h] in a fixed order
// (deterministic).  Workgroup b: outputs 64 b .. 64 b + 63 of the K x nf slab (lane =
// output), its 16 waves taking every 16th tile, combined in LDS; written to both (k, nc + h)
// and (nc + h, k).
__global__ __launch_bounds__(1024) void g_eta_reduce_kernel(const double* part, int ntile, int K, int Kmax, int nc,
                                                            int nf, const double* XX, double* G) {
  __shared__ double red[16][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, o = blockIdx.x * 64 + lane;
  const int k = o % K, h = o / K;
  const size_t stride = (size_t)Kmax * nf;
  double s = 0.0;
  if (o < K * nf) {
    const double* p = part + k + (size_t)Kmax * h;
    // twenty tiles' loads in flight per lane before they are added (the partials were
    // written by workgroups on every XCD: each round trip goes past the local L2)
    int b = w;
    for (; b + 16 * 19 < ntile; b += 16 * 20) {
      double x[20];
#pragma unroll
      for (int u = 0; u < 20; ++u) x[u] = p[stride * (b + 16 * u)];
#pragma unroll
      for (int u = 0; u < 20; ++u) s += x[u];
    }
    for (; b < ntile; b += 16) s += p[stride * b];
  }
  red[w][lane] = s;
  __syncthreads();
  if (w == 0 && o < K * nf) {
    double v = 0.0;
#pragma unroll
    for (int q = 0; q < 16; ++q) v += red[q][lane];
    G[k + (size_t)Kmax * (nc + h)] = v;
    G[(nc + h) + (size_t)Kmax * k] = v;
  }
  if (blockIdx.x == 0)
    for (int p = threadIdx.x; p < nc * nc; p += 1024) G[p % nc + (size_t)Kmax * (p / nc)] = XX[p];
}

void flush_g(State& s) {
  if (!s.g_pending) return;
  g_eta_reduce_kernel<<<(s.K * s.g_nf + 63) / 64, 1024, 0, s.stream>>>(s.G_part, s.g_ntile, s.K, s.Kmax, s.nc, s.g_nf,
                                                                       s.XX, s.G);
  HIP_OK(hipGetLastError());
  s.g_pending = false;
}

static bool eta_fused_ok(const State& s) {
  return !s.sharded && !s.any_xs && s.nr == 1 && !s.lev[0].spatial && s.n_na_rows == 0 && s.lev[0].np == s.ny && s.lev[0].uniform_n == 1 &&
         s.lev[0].nf <= 16 && s.K <= 64 && s.LS != nullptr && !getenv_flag("HMSC_NO_ETA_FUSION");
}

static EtaFArgs make_etaf_args(State& s, uint32_t iter) {
  const Level& L = s.lev[0];
  EtaFArgs a{};
  a.Z = s.Z;
  a.LS = s.LS;
  a.CR = s.CR;
  a.W = s.etaW;
  a.XEta = s.XEta;
  a.Pi = L.Pi;
  a.Eta = L.Eta;
  a.G_part = s.G_part;
  a.ZL = nullptr;
  a.ny = s.ny;
  a.ns_loc = s.nsl;
  a.K = s.K;
  a.Kmax = s.Kmax;
  a.nc = s.nc;
  a.nf = L.nf;
  a.np = L.np;
  a.ldcr = s.Kmax;
  a.key = s.key;
  a.iter = iter;
  a.iter_dev = s.capturing ? s.d_iter : nullptr;
  a.noise_zero = s.noise_mode;
  a.kt = s.kt_on ? s.d_kt + (size_t)KT_ETA * 2 * KT_SLOTS : nullptr;
  a.err = s.gbl_sync;
  return a;
}

template <int MODE>
static void launch_eta_fused_mode(State& s, const EtaFArgs& a) {
  const int ntile = (s.ny + EF_SITES - 1) / EF_SITES;
  const int nf = s.lev[0].nf, nb = ntile + (MODE == EF_DEFER ? a.nred + a.npre : 0);
  if (nf <= 8)
    eta_fused_kernel<8, MODE><<<nb, 256, 0, s.stream>>>(a);
  else if (nf <= 12)
    eta_fused_kernel<12, MODE><<<nb, 256, 0, s.stream>>>(a);
  else
    eta_fused_kernel<16, MODE><<<nb, 256, 0, s.stream>>>(a);
  HIP_OK(hipGetLastError());
  if (MODE != EF_STREAM) {
    // G's Eta rows: reduced from G_part by the next updateZ launch (or flush_g)
    s.g_pending = true;
    s.g_ntile = ntile;
    s.g_nf = nf;
    s.zt_valid = false;   // Eta changed: XZ is stale until the next updateZ
    s.xeta_valid = true;  // XEta rows rewritten, G pending
  }
}

static void launch_eta_fused(State& s, uint32_t iter, bool cr_done = false, bool defer = false, bool tail_gv = false) {
  if (!cr_done) {  // CR, W and LS (post_bl_kernel's workgroup 0 forms them in the co-launched path)
    const size_t smem = (size_t)CRW_LDS * sizeof(double);
    const CRWArgs c = make_crw_args(s);
    if (c.nf <= 8)
      crw_kernel<8><<<CRW_PARTS, 256, smem, s.stream>>>(c);
    else if (c.nf <= 12)
      crw_kernel<12><<<CRW_PARTS, 256, smem, s.stream>>>(c);
    else
      crw_kernel<16><<<CRW_PARTS, 256, smem, s.stream>>>(c);
    HIP_OK(hipGetLastError());
  }
  EtaFArgs a = make_etaf_args(s, iter);
  ProfScope ps(s, PROF_ETA_UNIT);
  if (defer) {
    a.nbl = (s.nsl + 3) / 4;
    a.tail = make_tail_args(s, tail_gv, false);
    a.tail.defer = tail_defer_levels();
    a.nred = a.tail.defer == 2 ? (a.nbl + CRW_GROUP - 1) / CRW_GROUP : 1;
    a.red_prio = getenv_flag("HMSC_RED_PRIO") ? 1 : 0;
    if (bl_predraw_on(s)) {
      a.npre = 64;  // ~40 k draws at config 4: 2-3 per thread
      a.ntile = (s.ny + EF_SITES - 1) / EF_SITES;
      a.pre_buf = s.bl_pre;
      a.pre_tag = s.bl_pre_tag;
    }
    launch_eta_fused_mode<EF_DEFER>(s, a);
  } else {
    launch_eta_fused_mode<EF_FUSED>(s, a);
  }
}

// NA rows of a sharded chain, level r (R/updateEta.R:59-70): the masked per-row precision and
// numerator of eta_na_row_kernel from the all-reduced row-masked CR (na_crrow_kernel) and the
// masked ZL, so no per-row sum over species is left after the all-reduce:
//   Mrow = CRrow[loff + h1, foff + h2],  brow_h = ZL_i[foff + h] - sum_{k not in r} XEta_ik CRrow[k, foff + h]
__global__ __launch_bounds__(64) void na_row_finish_kernel(EtaView ev, int r, int nf, int K, int NF, int loff, int foff,
                                                           const int* na_rows, const double* ZL, const double* CRrow,
                                                           double* Mrow, double* brow) {
  extern __shared__ __attribute__((aligned(16))) double sx[];  // XEta row (K)
  const int slot = blockIdx.x, i = na_rows[slot], t = threadIdx.x;
  const double* C = CRrow + (size_t)slot * K * NF;  // [k + K f]
  for (int k = t; k < K; k += 64) sx[k] = xeta_at(ev, i, k);
  __syncthreads();
  for (int p = t; p < nf * nf + nf; p += 64) {
    if (p < nf * nf) {
      const int h1 = p % nf, h2 = p / nf;
      Mrow[(size_t)slot * nf * nf + p] = C[loff + h1 + (size_t)K * (foff + h2)];
    } else {
      const int h = p - nf * nf;
      double v = ZL[(size_t)i * NF + foff + h];
      for (int k = 0; k < K; ++k)
        if (k < loff || k >= loff + nf) v -= sx[k] * C[k + (size_t)K * (foff + h)];
      brow[(size_t)slot * nf + h] = v;
    }
  }
}

// The per-level Eta draws of the general path (R/updateEta.R:42-92, levels in order, each
// seeing the new Eta of the previous ones): ZL (nzl partials, [site][NF]) and CR (ld ldcr)
// are the sums over species -- this chain's own, or a sharded chain's all-reduced ones, whose
// NA rows then come from the all-reduced row-masked CR (na_crrow) instead of eta_na_row_kernel.
static void eta_levels(State& s, uint32_t iter, const double* zl, int nzl, const double* cr, int ldcr,
                       const double* na_crrow) {
  for (int r = 0; r < s.nr; ++r) {
    const Level& L = s.lev[r];
    if (L.eta_alias()) continue;  // a covariate-dependent level's Eta is drawn once, by its group's first level
    if (r > 0) launch_xeta(s);  // levels r' < r were just redrawn (R/updateEta.R:218-226 rebuilds LRan[[r']])
    if (L.spatial) {            // R/updateEta.R:111-140 (spatial.hip)
      launch_eta_spatial(s, r, iter);
      continue;
    }
    EtaArgs a{};
    a.ev = make_view(s);
    a.XEta = s.XEta;
    a.r = r;
    a.nf = L.nf;
    a.np = L.np;
    a.K = s.K;
    a.nc = s.nc;
    a.NF = s.NF;
    a.foff = s.foff(r);
    a.loff = s.loff(r);
    a.ldcr = ldcr;
    a.nzl = nzl;
    a.ZL = zl;
    a.CR = cr;
    a.unit_ptr = L.unit_ptr;
    a.unit_rows = L.unit_rows;
    a.Eta = L.Eta;
    a.key = s.key;
    a.iter = iter;
    a.iter_dev = s.capturing ? s.d_iter : nullptr;
    a.noise_zero = s.noise_mode;
    if (s.n_na_rows > 0) {
      double* Mrow = s.Msmall;
      double* brow = Mrow + (size_t)s.n_na_rows * L.nf * L.nf;
      if (L.xs) {
        HMSC_REQUIRE(!na_crrow, "covariate-dependent levels: not on a species-sharded chain");
        eta_na_row_x_kernel<<<s.n_na_rows, 64, (s.K + L.xgroup) * sizeof(double), s.stream>>>(
            a.ev, r, L.xgroup, L.nf, s.K, a.loff, s.na_rows, s.Z, s.BL, s.iSigma, s.Ycode, s.nsl, Mrow, brow);
      } else if (na_crrow) {
        na_row_finish_kernel<<<s.n_na_rows, 64, s.K * sizeof(double), s.stream>>>(
            a.ev, r, L.nf, s.K, s.NF, a.loff, a.foff, s.na_rows, zl, na_crrow, Mrow, brow);
      } else {
        eta_na_row_kernel<<<s.n_na_rows, 64, s.K * sizeof(double), s.stream>>>(
            a.ev, r, L.nf, s.K, s.nc, a.loff, s.na_rows, s.Z, s.BL, s.iSigma, s.Ycode, s.nsl, Mrow, brow);
      }
      HIP_OK(hipGetLastError());
      a.row_na = s.row_na;
      a.row_slot = s.row_slot;
      a.Mrow = Mrow;
      a.brow = brow;
    }
    ProfScope ps(s, PROF_ETA_UNIT);
    if (L.xs) {
      const size_t smem = ((size_t)L.nf * L.nf + L.nf + L.xgroup + 2) * sizeof(double);
      eta_unit_x_kernel<<<L.np, 64, smem, s.stream>>>(a, L.xgroup);
    } else if (s.n_na_rows == 0 && L.uniform_n > 0 && L.nf <= 32) {
      const size_t smem = ((size_t)L.nf * L.nf + (size_t)s.K * L.nf + 2) * sizeof(double);
      const int grid = (L.np + 63) / 64;
      if (L.nf <= 8)
        eta_shared_kernel<8><<<grid, 64, smem, s.stream>>>(a, L.uniform_n);
      else if (L.nf <= 16)
        eta_shared_kernel<16><<<grid, 64, smem, s.stream>>>(a, L.uniform_n);
      else
        eta_shared_kernel<32><<<grid, 64, smem, s.stream>>>(a, L.uniform_n);
    } else {
      const size_t smem = ((size_t)L.nf * L.nf + L.nf + 2) * sizeof(double);
      eta_unit_kernel<<<L.np, 64, smem, s.stream>>>(a);
    }
    HIP_OK(hipGetLastError());
  }
  s.zt_valid = false;  // Eta changed: XZ is stale until the next updateZ
  launch_xeta(s);      // XEta and G for the new Eta
}

static void launch_zl(State& s, const int8_t* mask) {
  dim3 grid((s.ny + 63) / 64, s.zl_split);
  const int per = (s.nsl + s.zl_split - 1) / s.zl_split;
  ProfScope ps(s, PROF_ZL);
  // at most 64 factors per pass over Z (NF > 64: two passes)
  for (int fo = 0; fo < s.NF; fo += 64) {
    const int nf = std::min(64, s.NF - fo);
    const size_t smem = std::max((size_t)per * nf, (size_t)4 * nf * 64) * sizeof(double);
#define ZL_ARGS s.Z, s.BL, s.iSigma, mask, s.ny, s.nsl, s.K, s.nc, s.NF, s.zl_split, s.ZL_part, fo, nf
    if (nf <= 8)
      zl_kernel<8><<<grid, 256, smem, s.stream>>>(ZL_ARGS);
    else if (nf <= 16)
      zl_kernel<16><<<grid, 256, smem, s.stream>>>(ZL_ARGS);
    else if (nf <= 32)
      zl_kernel<32><<<grid, 256, smem, s.stream>>>(ZL_ARGS);
    else
      zl_kernel<64><<<grid, 256, smem, s.stream>>>(ZL_ARGS);
#undef ZL_ARGS
    HIP_OK(hipGetLastError());
  }
}

void launch_eta(State& s, uint32_t iter) {
  s.crw_fresh = false;  // (the co-launched path consumes the tail's constants itself)
  if (s.nr == 0) return;
  if (!s.xeta_valid) launch_xeta(s);  // the Eta kernels read XEta of the current Eta
  if (eta_fused_ok(s)) {
    launch_eta_fused(s, iter);
    return;
  }
  HMSC_REQUIRE(s.NF <= HMSC_KCAP, "updateEta: sum(nf) must be <= 128 in this build");
  for (int r = 0; r < s.nr; ++r)
    HMSC_REQUIRE(s.lev[r].nf >= 1, "updateEta: a level has zero factors");
  launch_zl(s, nullptr);  // ZL over all levels in one pass over Z
  {
    const int ncr = (s.nsl + SB - 1) / SB;
    const int64_t slab = (int64_t)s.Kmax * s.NFmax;
    cr_kernel<<<ncr, 256, (size_t)s.K * SB * sizeof(double), s.stream>>>(s.BL, s.iSigma, s.K, s.nc, s.NF, s.nsl,
                                                                           s.CR_part, s.Kmax, (int)slab, nullptr);
    HIP_OK(hipGetLastError());
    slab_sum_kernel<<<grid_for(slab), 256, 0, s.stream>>>(s.CR_part, s.CR, slab, ncr, slab);
    HIP_OK(hipGetLastError());
  }
  eta_levels(s, iter, s.ZL_part, s.zl_split, s.CR, s.Kmax, nullptr);
}

// ---------------------------------------------------------------------------
// updateInvSigma (R/updateInvSigma.R:3-43): species with distr[,2] == 1 only.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void inv_sigma_kernel(EtaView ev, const double* XEta, int K, const double* BL, const double* Z,
                                                        const int8_t* Ycode, const int* varest,
                                                        const double* aSigma, const double* bSigma, int sp0,
                                                        double* iSigma, Key key, uint32_t iter_h,
                                                        const uint32_t* iter_dev) {
  const uint32_t iter = iter_dev ? *iter_dev : iter_h;
  __shared__ double red[256];
  __shared__ int cnt[256];
  const int j = blockIdx.x, t = threadIdx.x, ny = ev.ny;
  if (!varest[j]) return;
  double ss = 0.0;
  int n = 0;
  for (int i = t; i < ny; i += 256) {
    if (Ycode[(size_t)i + (size_t)ny * j] < 0) continue;
    double e = 0.0;
    for (int k = 0; k < K; ++k) e += XEta[i + (size_t)ny * k] * BL[k + (size_t)K * j];
    const double d = Z[(size_t)i + (size_t)ny * j] - e;
    ss += d * d;
    ++n;
  }
  red[t] = ss;
  cnt[t] = n;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (t < w) {
      red[t] += red[t + w];
      cnt[t] += cnt[t + w];
    }
    __syncthreads();
  }
  if (t == 0) {
    const double shape = aSigma[j] + cnt[0] / 2.0;   // (:37-38)
    const double rate = bSigma[j] + red[0] / 2.0;    // (:39)
    iSigma[j] = gamma_std(key, (uint32_t)(sp0 + j), S_INVSIGMA, iter, shape) / rate;  // (:40)
  }
}

void launch_inv_sigma(State& s, uint32_t iter) {
  if (!s.any_var) return;
  if (!s.xeta_valid) launch_xeta(s);
  inv_sigma_kernel<<<s.nsl, 256, 0, s.stream>>>(make_view(s), s.XEta, s.K, s.BL, s.Z, s.Ycode, s.varest, s.aSigma,
                                                 s.bSigma, s.sp0, s.iSigma, s.key, iter,
                                                 s.capturing ? s.d_iter : nullptr);
  HIP_OK(hipGetLastError());
}

// ---------------------------------------------------------------------------
// computeInitialParameters (R/computeInitialParameters.R:17-273), initPar = NULL.
// ---------------------------------------------------------------------------
struct InitArgs {
  int nc, nt, ns_loc, sp0, K, NF, nr;
  int lev_nf[HMSC_MAX_LEVELS], lev_np[HMSC_MAX_LEVELS];
  double nu[HMSC_MAX_LEVELS], a1[HMSC_MAX_LEVELS], b1[HMSC_MAX_LEVELS], a2[HMSC_MAX_LEVELS],
      b2[HMSC_MAX_LEVELS];
  double* Eta[HMSC_MAX_LEVELS];
  const double* UGammaL;  // lower chol of UGamma
  const double* mGamma;
  const double* V0inv;    // V0^{-1}  (riwish(f0, V0) = solve(rwish(f0, solve(V0))))
  double f0;
  const double* Tr;
  const int* fam;
  const int* varest;
  const double* aSigma;
  const double* bSigma;
  double* Gamma;
  double* iV;
  double* LV;             // lower chol of V (scratch)
  double* BL;
  double* Psi;
  double* Delta;
  double* iSigma;
  double* scratch;
  Key key;
};

__global__ __launch_bounds__(256) void init_small_kernel(InitArgs a) {
  const int nc = a.nc, N = nc * a.nt, t = threadIdx.x;
  __shared__ int flag;
  double* S = a.scratch;        // nc*nc
  double* T = S + nc * nc;      // nc*nc
  double* W = T + nc * nc;      // nc*nc
  double* Zb = W + nc * nc;     // nc*nc
  for (int r = t; r < N; r += blockDim.x) {  // Gamma ~ N(mGamma, UGamma)   (:85)
    double v = a.mGamma[r];
    for (int c = 0; c <= r; ++c) v += a.UGammaL[r + N * c] * normal(a.key, (uint32_t)c, 0, S_INIT_GAMMA, 0);
    a.Gamma[r] = v;
  }
  wg_copy(S, a.V0inv, nc * nc);
  wg_chol(S, nc, nc, &flag);
  wg_lower_only(S, nc, nc);
  wg_rwish(S, nc, a.f0, a.iV, T, Zb, a.key, S_INIT_V_DIAG, S_INIT_V_OFF, 0, 0);   // iV = rwish(f0, V0^-1)  (:91)
  wg_copy(S, a.iV, nc * nc);
  wg_chol(S, nc, nc, &flag);
  wg_chol2inv(S, nc, nc, T, nc, W);          // V = iV^-1
  wg_copy(a.LV, T, nc * nc);
  wg_chol(a.LV, nc, nc, &flag);
  wg_lower_only(a.LV, nc, nc);
  for (int j = t; j < a.ns_loc; j += blockDim.x) {  // sigma   (:111-126)
    double sig = 1.0;
    if (a.varest[j])
      sig = gamma_std(a.key, (uint32_t)(a.sp0 + j), S_INIT_SIGMA, 0, a.aSigma[j]) / a.bSigma[j];
    else if (a.fam[j] == 3)
      sig = 1e-2;
    a.iSigma[j] = 1.0 / sig;
  }
  if (t < a.nr) {  // Delta   (:175)
    const int r = t;
    int f0 = 0;
    for (int q = 0; q < r; ++q) f0 += a.lev_nf[q];
    const uint32_t st = S_INIT_DELTA + LEVEL_STRIDE * r;
    for (int h = 0; h < a.lev_nf[r]; ++h) {
      const double sh = h == 0 ? a.a1[r] : a.a2[r];
      const double rt = h == 0 ? a.b1[r] : a.b2[r];
      a.Delta[f0 + h] = gamma_std(a.key, (uint32_t)h, st, 0, sh) / rt;
    }
  }
}

__global__ __launch_bounds__(256) void init_big_kernel(InitArgs a) {
  const int nc = a.nc, K = a.K, NF = a.NF;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t t0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  // Beta_j ~ N(Gamma Tr_j^T, V)   (:97-101)
  for (int64_t p = t0; p < (int64_t)nc * a.ns_loc; p += stride) {
    const int c = (int)(p % nc), j = (int)(p / nc);
    double mu = 0.0;
    for (int q = 0; q < a.nt; ++q) mu += a.Gamma[c + nc * q] * a.Tr[j + (size_t)a.ns_loc * q];
    double v = mu;
    for (int c2 = 0; c2 <= c; ++c2)
      v += a.LV[c + nc * c2] * normal(a.key, (uint32_t)(a.sp0 + j), (uint32_t)c2, S_INIT_BETA, 0);
    a.BL[c + (size_t)K * j] = v;
  }
  // Psi, Lambda   (:183, :189-193)
  for (int64_t p = t0; p < (int64_t)NF * a.ns_loc; p += stride) {
    const int f = (int)(p % NF), j = (int)(p / NF);
    int r = 0, h = f, f0 = 0;
    while (h >= a.lev_nf[r]) {
      h -= a.lev_nf[r];
      f0 += a.lev_nf[r];
      ++r;
    }
    double tau = 1.0;
    for (int q = 0; q <= h; ++q) tau *= a.Delta[f0 + q];
    const uint32_t idx = (uint32_t)(h + a.lev_nf[r] * (a.sp0 + j));
    const double psi = gamma_std(a.key, idx, S_INIT_PSI + LEVEL_STRIDE * r, 0, a.nu[r] / 2) / (a.nu[r] / 2);
    a.Psi[f + (size_t)NF * j] = psi;
    a.BL[nc + f + (size_t)K * j] = normal(a.key, idx, 0, S_INIT_LAMBDA + LEVEL_STRIDE * r, 0) / sqrt(psi * tau);
  }
  // Eta ~ N(0,1)   (:207)
  for (int r = 0; r < a.nr; ++r) {
    if (!a.Eta[r]) continue;  // (a level sharing another level's Eta: drawn once, by its owner)
    const int64_t n = (int64_t)a.lev_np[r] * a.lev_nf[r];
    for (int64_t p = t0; p < n; p += stride) {
      const int q = (int)(p % a.lev_np[r]), h = (int)(p / a.lev_np[r]);
      a.Eta[r][p] = normal(a.key, (uint32_t)q, (uint32_t)h, S_INIT_ETA + LEVEL_STRIDE * r, 0);
    }
  }
}

void launch_init(State& s) {
  InitArgs a{};
  a.nc = s.nc;
  a.nt = s.nt;
  a.ns_loc = s.nsl;
  a.sp0 = s.sp0;
  a.K = s.K;
  a.NF = s.NF;
  a.nr = s.nr;
  for (int r = 0; r < s.nr; ++r) {
    a.lev_nf[r] = s.lev[r].nf;
    a.lev_np[r] = s.lev[r].np;
    a.nu[r] = s.lev[r].nu;
    a.a1[r] = s.lev[r].a1;
    a.b1[r] = s.lev[r].b1;
    a.a2[r] = s.lev[r].a2;
    a.b2[r] = s.lev[r].b2;
    a.Eta[r] = s.lev[r].eta_alias() ? nullptr : s.lev[r].Eta;
  }
  a.UGammaL = s.UGammaL;
  a.mGamma = s.mGamma;
  a.V0inv = s.V0inv;
  a.f0 = s.f0;
  a.Tr = s.Tr;
  a.fam = s.fam;
  a.varest = s.varest;
  a.aSigma = s.aSigma;
  a.bSigma = s.bSigma;
  a.Gamma = s.Gamma;
  a.iV = s.iV;
  a.LV = s.scratch + 4 * (size_t)s.nc * s.nc;
  a.BL = s.BL;
  a.Psi = s.Psi;
  a.Delta = s.Delta;
  a.iSigma = s.iSigma;
  a.scratch = s.scratch;
  a.key = s.key;
  init_small_kernel<<<1, 256, 0, s.stream>>>(a);
  HIP_OK(hipGetLastError());
  init_big_kernel<<<512, 256, 0, s.stream>>>(a);
  HIP_OK(hipGetLastError());
}

// ---------------------------------------------------------------------------
// record: pack the state into one contiguous ring slot (device), the D2H copy of
// the slot then runs on the copy stream overlapped with the next sweeps.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void pack_kernel(PackArgs a) { pack_body(a, blockIdx.x, gridDim.x); }

// updateZ's two slab reductions and the record pack of the sweep's main-stream outputs in one
// launch (graph replays of recorded sweeps): the pack reads none of what the slab sums or
// updateZ write (Z is not recorded), so it need not wait for them
__global__ __launch_bounds__(256) void slab_pack_kernel(SlabJob j0, SlabJob j1, PackArgs pk, int npack, SideGate g,
                                                        G2SArgs g2, int ng2) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int b = blockIdx.x;
  if (b < j0.nb)
    slab_sum_body(j0.part, j0.out, j0.n, j0.nparts, j0.stride, b, j0.nb);
  else if (b < j0.nb + j1.nb)
    slab_sum_body(j1.part, j1.out, j1.n, j1.nparts, j1.stride, b - j0.nb, j1.nb);
  else if (b < j0.nb + j1.nb + ng2)
    g2_stats_body(g2, b - j0.nb - j1.nb, smem);
  else if (b < j0.nb + j1.nb + ng2 + npack)
    pack_body(pk, b - j0.nb - j1.nb - ng2, npack);
  else
    side_gate_body(g);
}

// Publishes "samples < value have landed in the host ring" to the host with a system-scope
// release store into fine-grained pinned memory; enqueued on the copy stream after the
// sample's D2H copy, so the unpack threads poll memory instead of calling into HIP.
__global__ void copied_flag_kernel(uint64_t* flag, uint64_t value) {
  __hip_atomic_store(flag, value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

void launch_copied_flag(State& s, uint64_t value) {
  copied_flag_kernel<<<1, 1, 0, s.copy_stream>>>(s.copied_dev, value);
  HIP_OK(hipGetLastError());
}

// slot layout: BL(K*nsl) | Psi(NF*nsl) | Delta(NF) | Gamma(nc*nt) | iV(nc*nc) | iSigma(nsl) | Eta_r ... | rho(1)
size_t record_slot_doubles(const State& s) {
  size_t n = (size_t)s.Kmax * s.nsl + (size_t)s.NFmax * s.nsl + s.NFmax + (size_t)s.nc * s.nt +
             (size_t)s.nc * s.nc + s.nsl + 2;
  for (int r = 0; r < s.nr; ++r) n += (size_t)s.lev[r].np * s.lev[r].nfcap + (s.lev[r].spatial ? s.lev[r].nfcap : 0);
  return n;
}

static PackArgs make_pack_args(State& s, double* slot, int part) {
  PackArgs a{};
  int64_t off = 0;
  int k = 0;
  // side pieces (Gamma, iV, Delta; Psi unless the BetaLambda tail drew it) are written by the
  // GammaV algebra, the delta chain and the species partials, which may still run on the side
  // stream: part 2 packs them there, part 1 the rest
  auto add = [&](const double* src, int64_t n, bool side) {
    if (part == 0 || (part == 2) == side) a.p[k++] = PackPiece{src, n, off};
    off += n;
  };
  add(s.BL, (int64_t)s.K * s.nsl, false);
  add(s.Psi, (int64_t)s.NF * s.nsl, s.psi_side);  // post_bl_kernel (side) or the BetaLambda tail (main)
  add(s.Delta, s.NF, true);
  add(part == 2 ? s.Gamma_side : s.Gamma, (int64_t)s.nc * s.nt, true);  // (the next sweep's Gamma2 rewrites Gamma)
  add(s.iV, (int64_t)s.nc * s.nc, true);
  add(s.iSigma, s.nsl, false);
  for (int r = 0; r < s.nr; ++r) add(s.lev[r].Eta, (int64_t)s.lev[r].np * s.lev[r].nf, false);
  add(s.rho, 1, true);  // updateRho's grid index (written with GammaV's outputs)
  for (int r = 0; r < s.nr; ++r)
    if (s.lev[r].spatial) add(s.lev[r].AlphaD, s.lev[r].nf, false);  // updateAlpha's grid indices
  a.npieces = k;
  a.slot = slot;
  if (slot == nullptr) {  // captured into a graph replay: slot chosen on the device
    a.slot = s.ring;
    a.iter_dev = (part == 2 && s.psi_side) ? s.d_iter_side : s.d_iter;
    a.desc = s.d_rec_desc;
    a.slot_stride = (int64_t)s.slot_doubles;
    a.ring_slots = s.ring_slots;
    if (s.cap_kcopy) {  // this part's completion flag for the copy kernels
      a.flags = s.pack_flags + (size_t)part * s.ring_slots;
      a.ticket = s.pack_ticket + part;
      s.cap_pack_mask |= 1 << part;
    }
  }
  return a;
}

// ---------------------------------------------------------------------------
// Kernel record copies (State::kcopy): sample k's ring slot to the pinned host ring by a small
// kernel on the copy stream, launched with the replay that packs it and waiting on the device
// for the pack parts' flags -- each sample lands on the host as soon as it is packed, instead
// of every sample of a replay behind one copy after the replay (so a recorded run needs no
// single-sweep replays at its end to keep the copy tail short).  Write-through (system scope)
// stores, then the last workgroup publishes *copied = k + 1 for the unpack threads.
// ---------------------------------------------------------------------------
struct RecCopyArgs {
  const double* ring;
  double* host;
  int64_t slot_doubles;
  int ring_slots, k, parts;
  const uint64_t* flags;  // [3][ring_slots]
  uint64_t want;
  int* ticket;
  uint64_t* copied;
  int* err;
};

constexpr int REC_COPY_WG = 16;

__global__ __launch_bounds__(256) void rec_copy_kernel(RecCopyArgs a) {
  const int slot = a.k % a.ring_slots, t = threadIdx.x;
  if (t < 3 && ((a.parts >> t) & 1)) {
    const uint64_t* f = a.flags + (size_t)t * a.ring_slots + slot;
    if (!spin_until<8>([&] { return __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == a.want; }))
      __hip_atomic_store(&a.err[3], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  const double* src = a.ring + (int64_t)slot * a.slot_doubles;
  double* dst = a.host + (int64_t)slot * a.slot_doubles;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + t; e < a.slot_doubles; e += (int64_t)gridDim.x * blockDim.x)
    __hip_atomic_store((unsigned long long*)(dst + e), (unsigned long long)__double_as_longlong(load_coherent(src + e)),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t == 0 && __hip_atomic_fetch_add(a.ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (int)gridDim.x - 1) {
    __hip_atomic_store(a.ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(a.copied, (uint64_t)a.k + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

void launch_rec_copy(State& s, int k, int parts) {
  RecCopyArgs a{};
  a.ring = s.ring;
  a.host = s.host_rec_dev;
  a.slot_doubles = (int64_t)s.slot_doubles;
  a.ring_slots = s.ring_slots;
  a.k = k;
  a.parts = parts;
  a.flags = s.pack_flags;
  a.want = ((uint64_t)s.run_nonce << 32) | (uint32_t)(k + 1);
  a.ticket = s.pack_ticket + 3;
  a.copied = s.copied_dev;
  a.err = s.gbl_sync;
  rec_copy_kernel<<<REC_COPY_WG, 256, 0, s.copy_stream>>>(a);
  HIP_OK(hipGetLastError());
}

PackArgs record_pack_args(State& s, int part) { return make_pack_args(s, nullptr, part); }

// the external first-sweep side work (State::ext_side) also packs the record's side pieces
void ext_add_record(State& s) {
  PackArgs a = make_pack_args(s, nullptr, 2);
  a.iter_dev = s.d_ext_iter;
  auto prev = std::move(s.ext_pending);
  s.ext_pending = [prev, a, &s] {
    prev();
    pack_kernel<<<8, 256, 0, s.side>>>(a);
    HIP_OK(hipGetLastError());
  };
}

void launch_record(State& s, double* slot, int part) {
  const PackArgs a = make_pack_args(s, slot, part);
  if (part == 2)
    pack_kernel<<<8, 256, 0, s.side>>>(a);
  else
    pack_kernel<<<512, 256, 0, s.stream>>>(a);
  HIP_OK(hipGetLastError());
}

void launch_slab_sum2_pack(State& s, const double* p0, double* o0, int64_t n0, int np0, const double* p1, double* o1,
                           int64_t n1, int np1, SideGate gate, State* g2s) {
  const SlabJob j0{p0, o0, n0, n0, np0, grid_for(n0)};
  const SlabJob j1{p1, o1, n1, n1, np1, grid_for(n1)};
  const PackArgs pk = make_pack_args(s, nullptr, 1);
  constexpr int NPACK = 256;
  G2SJob job{};
  if (g2s) job = shard_g2_job(*g2s, p0, np0);
  const G2SJob* g2 = g2s ? &job : nullptr;
  const int ng2 = g2 ? g2->a.nparts : 0;
  slab_pack_kernel<<<j0.nb + j1.nb + ng2 + NPACK + (gate.n > 0 ? 1 : 0), 256, g2 ? g2->smem : 0, s.stream>>>(
      j0, j1, pk, NPACK, gate, g2 ? g2->a : G2SArgs{}, ng2);
  HIP_OK(hipGetLastError());
}

// ===========================================================================
// Species-sharded sweep (the data layout in state.h "species-sharded chain").
// Every rank owns a block of species; each updater's sums over species become one section of
// the all-reduce buffers, and the sweep issues exactly two all-reduces (ar_point, capi.cpp):
//   A  after updateZ:          ar_a, the next updateGamma2's species sums
//   B  after updateBetaLambda: ar_b, updateEta's ZL / CR (+ NA rows), updateGammaV's and
//                              updateLambdaPriors' species sums
// With every updater of the synthetic config on, the same fused launches as one rank run:
// the Gamma2 + BetaLambda launch (Gamma2 from ar_a; its tail leaves CR and the GammaV / psi
// sums in ar_b), the Eta stream (ZL into ar_b), the all-reduce, the side chain (GammaV algebra,
// delta chains) on the side stream, and the Eta solve.  On one rank that reproduces the
// unsharded chain bit for bit (tests/test_gpu_sharded.py).
// ===========================================================================
ArbLayout arb_layout(const State& s) {
  ArbLayout L;
  const bool eta = (s.mask & HMSC_UP_ETA) && s.nr > 0;
  const bool gv = (s.mask & HMSC_UP_GAMMAV) != 0;
  const bool lp = (s.mask & HMSC_UP_LAMBDAPRIORS) && s.nr > 0;
  size_t o = 0;
  L.zl = o;
  o += eta ? (size_t)s.ny * s.NF : 0;
  L.cr = o;
  o += eta ? (size_t)s.K * s.NF : 0;
  L.ldcr = s.K;
  L.gv = o;
  o += gv ? (size_t)s.nc * s.nc + (size_t)s.nc * s.nt : 0;
  L.rs = o;
  o += lp ? (size_t)s.NF : 0;
  L.na = o;
  o += (eta && s.n_na_rows > 0) ? (size_t)s.n_na_rows * s.K * s.NF : 0;
  L.n = o;
  return L;
}

size_t arb_capacity(const State& s) {
  const size_t NF = std::max(1, s.NFmax), K = s.Kmax;
  return (size_t)s.ny * NF + K * NF + (size_t)s.nc * s.nc + (size_t)s.nc * s.nt + NF + (size_t)s.n_na_rows * K * NF + 64;
}

bool sharded_fused_ok(const State& s) {
  const uint32_t need = HMSC_UP_GAMMA2 | HMSC_UP_BETALAMBDA | HMSC_UP_GAMMAV | HMSC_UP_LAMBDAPRIORS | HMSC_UP_ETA;
  const size_t N = (size_t)s.nc * s.nt;
  return s.sharded && (s.mask & need) == need && !(s.mask & HMSC_UP_GAMMAETA) && !s.any_na_global && !s.phylo &&
         s.nr == 1 && !s.lev[0].spatial && s.n_na_rows == 0 && s.lev[0].np == s.ny && s.lev[0].uniform_n == 1 &&
         s.lev[0].nf <= 16 && s.K <= 32 && s.nt <= 8 && N <= 32 && s.NF * s.nt + N <= 64 &&
         (G2F_LDS + (size_t)s.nc * s.nc + N * N) <= (size_t)BLW_LDS &&
         (size_t)s.nc * s.nc + N + s.NF <= 1024 && s.LS != nullptr && s.gvt != nullptr && s.gbl_sync != nullptr &&
         !getenv_flag("HMSC_NO_G2BL_FUSION") && !getenv_flag("HMSC_NO_ETA_FUSION") && !getenv_flag("HMSC_NO_SHARD_FUSION");
}

// out[p] = sum_b part[b * ld + p] in b order from 0 (the order gammav_body / delta_body sum
// a single rank's partials), eight partials' loads in flight per thread
__global__ __launch_bounds__(256) void seq_sum_kernel(const double* __restrict__ part, int nparts, int64_t ld,
                                                      int64_t n, double* __restrict__ out) {
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < n; p += (int64_t)gridDim.x * blockDim.x) {
    double v = 0.0;
    int b = 0;
    for (; b + 8 <= nparts; b += 8) {
      double x[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) x[u] = part[(int64_t)(b + u) * ld + p];
#pragma unroll
      for (int u = 0; u < 8; ++u) v += x[u];
    }
    for (; b < nparts; ++b) v += part[(int64_t)b * ld + p];
    out[p] = v;
  }
}

static void seq_sum(const double* part, int nparts, int64_t ld, int64_t n, double* out, hipStream_t st) {
  if (n <= 0) return;
  seq_sum_kernel<<<grid_for(n, 256, 1024), 256, 0, st>>>(part, nparts, ld, n, out);
  HIP_OK(hipGetLastError());
}

// ---- all-reduce A: updateGamma2's sums over this rank's species (R/updateGamma2.R:36,46)
//   ar_a = [X^T Z Tr (nc nt) | Lambda_all Tr (NF nt) | #(iSigma != 1)]
// Workgroup b forms the partial of species block b (gamma2_partial_body, as the BetaLambda
// workgroups of the fused launch do); the last one through (a ticket) adds them in the order
// gamma2_final_body adds a single rank's partials, so Gamma2 of a 1-rank sharded chain is the
// unsharded chain's bit for bit.  With NA in this rank's Y, XZ is masked and X^T Z Tr comes
// from ZTr (xtztr) instead.
// (G2SArgs: declared with the slab kernels.)  With XZpart the rows < nc come from updateZ's
// chunk partials, summed in the slab reduction's order (gamma2_partial_body): the same bits as
// from the reduced XZ, so the stats can ride in the slab launch instead of following it.
__device__ void g2_stats_body(const G2SArgs& a, int bid, double* smem) {
  __shared__ int s_last, s_cnt;
  const int t = threadIdx.x;
  gamma2_partial_body(XZSrc{a.XZ, a.XZpart, a.xz_nparts, a.xz_stride}, a.BL, a.K, a.nc, a.NF, a.nt, a.nsl, a.Tr,
                      a.part, smem, bid, true);
  vm_stores_done();
  __syncthreads();
  if (t == 0) s_last = __hip_atomic_fetch_add(a.ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == a.nparts - 1;
  __syncthreads();
  if (!s_last) return;
  if (t == 0) {
    s_cnt = 0;
    __hip_atomic_store(a.ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  const int n1 = a.nc * a.nt, P = n1 + a.NF * a.nt;
  if (P <= 64 && a.nparts > 1) {
    // gamma2_final_main's order: 8 groups of 32 threads, group g summing parts g, g + 8, ... (16
    // loads of a thread in flight), then the groups in order -- the 256 threads together
    // instead of one thread per output walking every part
    __shared__ double red[8][64];
    const int g = t >> 5, l = t & 31;
    for (int p0 = 0; p0 < P; p0 += 32) {
      const int p = min(p0 + l, P - 1);
      double sg = 0.0;
      for (int b0 = g; b0 < a.nparts; b0 += 128) {
        double x[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) x[u] = load_coherent(a.part + (size_t)min(b0 + 8 * u, a.nparts - 1) * P + p);
#pragma unroll
        for (int u = 0; u < 16; ++u)
          if (b0 + 8 * u < a.nparts) sg += x[u];
      }
      red[g][p0 + l] = sg;
    }
    __syncthreads();
    for (int p = t; p < P; p += 256) {
      double v = 0.0;
#pragma unroll
      for (int g2 = 0; g2 < 8; ++g2) v += red[g2][p];
      a.out[p] = (p < n1 && a.xtztr) ? a.xtztr[p] : v;
    }
  } else {
    for (int p = t; p < P; p += 256) {
      double v = 0.0;
      for (int b0 = 0; b0 < a.nparts; b0 += 32) {
        double x[32];
#pragma unroll
        for (int u = 0; u < 32; ++u) x[u] = load_coherent(a.part + (size_t)min(b0 + u, a.nparts - 1) * P + p);
#pragma unroll
        for (int u = 0; u < 32; ++u)
          if (b0 + u < a.nparts) v += x[u];
      }
      a.out[p] = (p < n1 && a.xtztr) ? a.xtztr[p] : v;
    }
  }
  __syncthreads();
  int c = 0;
  for (int j = t; j < a.nsl; j += 256) c += a.iSigma[j] != 1.0;
  if (c) atomicAdd(&s_cnt, c);
  __syncthreads();
  if (t == 0) a.out[P] = (double)s_cnt;
}

__global__ __launch_bounds__(256) void g2_stats_kernel(G2SArgs a) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  g2_stats_body(a, blockIdx.x, smem);
}

// all-reduce A's stats job for this chain (with parts: from updateZ's chunk partials)
G2SJob shard_g2_job(State& s, const double* xz_part, int xz_nparts) {
  G2SJob j{};
  G2SArgs& a = j.a;
  a.XZ = s.XZ;
  a.XZpart = xz_part;
  a.xz_nparts = xz_part ? xz_nparts : 0;
  a.xz_stride = xz_part ? (int64_t)s.K * s.nsl : 0;
  a.BL = s.BL;
  a.Tr = s.Tr;
  a.iSigma = s.iSigma;
  a.xtztr = nullptr;
  a.part = s.ABpart;
  a.ticket = s.shard_ticket;
  a.out = s.ar_a;
  a.K = s.K;
  a.nc = s.nc;
  a.NF = s.NF;
  a.nt = s.nt;
  a.nsl = s.nsl;
  a.nparts = (s.nsl + G2SB - 1) / G2SB;
  j.smem = (size_t)(s.K * G2SB + G2SB * s.nt + (xz_part ? 4 * s.nc * G2SB : 0)) * sizeof(double);
  return j;
}

static void shard_g2_stats(State& s) {
  if (!(s.mask & HMSC_UP_GAMMA2)) return;
  const int n1 = s.nc * s.nt, n12 = n1 + s.NF * s.nt;
  if (s.g2s_slab) {  // formed by updateZ's slab launch of this sweep (zdraw.hip)
    s.g2s_slab = false;
    ar_point(s, s.ar_a, (size_t)n12 + 1);  // all-reduce A
    s.g2s_valid = true;
    return;
  }
  if (!s.xeta_valid) launch_xeta(s);
  if (!s.zt_valid) launch_zt_refresh(s);  // XZ (and ZTr) of the current Z and Eta
  const double* xt = nullptr;
  if (s.has_na) {  // this rank's XZ is masked: X^T (Z Tr) from ZTr
    xt_ztr_kernel<<<n1, 256, 0, s.stream>>>(s.X, s.ZTr, s.ny, s.nc, s.nt, s.allreduce_buf);
    HIP_OK(hipGetLastError());
    xt = s.allreduce_buf;
  }
  G2SJob j = shard_g2_job(s, nullptr, 0);
  j.a.xtztr = xt;
  g2_stats_kernel<<<j.a.nparts, 256, j.smem, s.stream>>>(j.a);
  HIP_OK(hipGetLastError());
  ar_point(s, s.ar_a, (size_t)n12 + 1);  // all-reduce A
  s.g2s_valid = true;
}

// updateGamma2 of a sharded chain on the general path: the final stage on the all-reduced sums
static void launch_gamma2_sharded(State& s, uint32_t iter) {
  if (!s.g2s_valid) shard_g2_stats(s);
  if (!s.xeta_valid) launch_xeta(s);
  flush_g(s);  // the final stage reads G's X^T Eta block
  if (!s.g2prep_valid) {
    join_side(s);
    launch_gamma2_prep(s, s.stream);
  }
  const int n12 = s.nc * s.nt + s.NF * s.nt;
  G2Args a{};
  a.nc = s.nc;
  a.nt = s.nt;
  a.Kmax = s.Kmax;
  a.NF = s.NF;
  a.nparts = 1;
  a.ns_loc = s.nsl;
  a.use_xtztr = 0;
  a.check_isigma = 0;
  a.isig_count = s.ar_a + n12;
  a.part = s.ar_a;
  a.xtztr = nullptr;
  a.G = s.G;
  a.prep = s.g2prep;
  a.iSigma = s.iSigma;
  a.Gamma = s.Gamma;
  a.key = s.key;
  a.iter = iter;
  a.iter_dev = s.capturing ? s.d_iter : nullptr;
  a.noise_zero = s.noise_mode;
  const size_t lds = g2f_layout(s, a);
  join_side(s);  // iV and the prep matrices come from the previous sweep's GammaV (side stream)
  gamma2_final_kernel<<<1, 256, lds, s.stream>>>(a);
  HIP_OK(hipGetLastError());
}

// ---- all-reduce B producers of the general path (this rank's species -> ar_b sections)
// updateGammaV: E E^T and B Tr (R/updateGammaV.R:16-18)
static void shard_gv_stats(State& s, hipStream_t st) {
  const ArbLayout L = arb_layout(s);
  const int nparts = (s.nsl + SB - 1) / SB;
  gammav_partial_kernel<<<nparts, 256, (size_t)(2 * s.nc * SB + SB * s.nt) * sizeof(double), st>>>(
      s.BL, s.K, s.nc, s.nt, s.nsl, s.Gamma, s.Tr, s.gv_part);
  HIP_OK(hipGetLastError());
  const int64_t n = (int64_t)s.nc * s.nc + (int64_t)s.nc * s.nt;
  seq_sum(s.gv_part, nparts, n, n, s.ar_b + L.gv, st);
}

// updateLambdaPriors: the psi draws of this rank's species and sum_j psi lambda^2 (:22-24)
static void shard_psi(State& s, uint32_t iter, hipStream_t st) {
  const ArbLayout L = arb_layout(s);
  HMSC_REQUIRE(s.NF <= HMSC_KCAP, "updateLambdaPriors: sum(nf) must be <= 128 in this build");
  const LPArgs a = make_lp_args(s, iter);
  const int nparts = std::min(LP_PARTS, std::max(1, s.nsl));
  psi_kernel<<<nparts, 256, 0, st>>>(a);
  HIP_OK(hipGetLastError());
  seq_sum(s.psi_rs, nparts, s.NF, s.NF, s.ar_b + L.rs, st);
}

// the row-masked CR of every NA row (all ranks agree on the rows: any NA in the whole Y), this
// rank's part: CR - sum over its species NA in row i of BL_j iSigma_j Lambda_j^T, species in
// ascending order (deterministic); the codes of the row's species from the packed Ybits words
struct NACRArgs {
  const double* CR;  // this rank's CR (K x NF, ld K), before the all-reduce
  const int* na_rows;
  const uint64_t* Ybits;
  const double* BL;
  const double* iSigma;
  double* out;       // n_na_rows x (K x NF)
  int ny, nsl, K, NF, nc;
};

__global__ __launch_bounds__(256) void na_crrow_kernel(NACRArgs a) {
  extern __shared__ uint64_t sw[];  // the row's code words, one per 32-species block
  const int slot = blockIdx.x, i = a.na_rows[slot], t = threadIdx.x, nblk = (a.nsl + 31) / 32;
  for (int b = t; b < nblk; b += 256) sw[b] = a.Ybits[(size_t)b * a.ny + i];
  __syncthreads();
  double* dst = a.out + (size_t)slot * a.K * a.NF;
  for (int p = t; p < a.K * a.NF; p += 256) {
    const int k = p % a.K, f = p / a.K;
    double v = a.CR[p];
    for (int b = 0; b < nblk; ++b) {
      const uint64_t wd = sw[b];
      uint64_t na = ~(wd | (wd >> 1)) & 0x5555555555555555ull;  // 2-bit fields equal to 0: code -1 (NA)
      while (na) {
        const int q = __ffsll((long long)na) - 1;
        na &= na - 1;
        const int j = 32 * b + (q >> 1);
        if (j < a.nsl) v -= a.BL[k + (size_t)a.K * j] * a.iSigma[j] * a.BL[a.nc + f + (size_t)a.K * j];
      }
    }
    dst[p] = v;
  }
}

// updateEta: ZL = Z (Lambda diag(iSigma))^T over this rank's observed cells and CR (+ the NA rows)
static void shard_eta_stats(State& s) {
  const ArbLayout L = arb_layout(s);
  HMSC_REQUIRE(s.NF <= HMSC_KCAP, "updateEta: sum(nf) must be <= 128 in this build");
  launch_zl(s, s.has_na ? s.Ycode : nullptr);
  const int64_t nzl = (int64_t)s.ny * s.NF;
  slab_sum_kernel<<<grid_for(nzl), 256, 0, s.stream>>>(s.ZL_part, s.ar_b + L.zl, nzl, s.zl_split, nzl);
  HIP_OK(hipGetLastError());
  const int ncr = (s.nsl + SB - 1) / SB;
  const int64_t slab = (int64_t)s.K * s.NF;
  cr_kernel<<<ncr, 256, (size_t)s.K * SB * sizeof(double), s.stream>>>(s.BL, s.iSigma, s.K, s.nc, s.NF, s.nsl, s.CR_part,
                                                                         L.ldcr, (int)slab, nullptr);
  HIP_OK(hipGetLastError());
  slab_sum_kernel<<<grid_for(slab), 256, 0, s.stream>>>(s.CR_part, s.ar_b + L.cr, slab, ncr, slab);
  HIP_OK(hipGetLastError());
  if (s.n_na_rows > 0) {
    NACRArgs a{};
    a.CR = s.ar_b + L.cr;
    a.na_rows = s.na_rows;
    a.Ybits = s.Ybits;
    a.BL = s.BL;
    a.iSigma = s.iSigma;
    a.out = s.ar_b + L.na;
    a.ny = s.ny;
    a.nsl = s.nsl;
    a.K = s.K;
    a.NF = s.NF;
    a.nc = s.nc;
    na_crrow_kernel<<<s.n_na_rows, 256, (size_t)((s.nsl + 31) / 32) * sizeof(uint64_t), s.stream>>>(a);
    HIP_OK(hipGetLastError());
  }
}

// ---- consumers of all-reduce B
static void shard_gammav_final(State& s, uint32_t iter, hipStream_t st) {
  const ArbLayout L = arb_layout(s);
  const double* part = s.ar_b + L.gv;
  if (s.nc * s.nt <= 32) {
    launch_gammav_wave(s, iter, st, part, 1, s.capturing ? s.d_iter : nullptr);  // (+ Gamma2's prep)
    return;
  }
  GVArgs a{};
  a.nc = s.nc;
  a.nt = s.nt;
  a.ns_glob = s.ns;
  a.nparts = 1;
  a.part = part;
  a.V0 = s.V0;
  a.f0 = s.f0;
  a.iUGamma = s.iUGamma;
  a.mGamma = s.mGamma;
  a.iUmG = s.iUmG;
  a.TT = s.TT;
  a.iV = s.iV;
  a.Gamma = s.Gamma;
  a.scratch = s.scratch;
  a.key = s.key;
  a.iter = iter;
  a.iter_dev = s.capturing ? s.d_iter : nullptr;
  a.noise_zero = s.noise_mode;
  a.fail = s.dev_flags;
  const size_t need = (6 * (size_t)s.nc * s.nc + (size_t)s.nc * s.nt + (size_t)s.nc * s.nt * s.nc * s.nt +
                       (size_t)s.nc * s.nt) * sizeof(double);
  a.use_lds = need <= 64 * 1024;
  HMSC_REQUIRE(a.use_lds || need <= s.scratch_doubles * sizeof(double), "internal: GammaV scratch too small");
  gammav_final_kernel<<<1, 64, a.use_lds ? need : 0, st>>>(a);
  HIP_OK(hipGetLastError());
  if (s.mask & HMSC_UP_GAMMA2) launch_gamma2_prep(s, st);
}

static void shard_delta(State& s, uint32_t iter, hipStream_t st) {
  const ArbLayout L = arb_layout(s);
  LPArgs a = make_lp_args(s, iter);
  delta_kernel<<<s.nr, 64, 0, st>>>(a, s.ar_b + L.rs, 1);
  HIP_OK(hipGetLastError());
}

static void shard_eta_solve(State& s, uint32_t iter, bool fused) {
  const ArbLayout L = arb_layout(s);
  if (fused) {
    EtaFArgs a = make_etaf_args(s, iter);
    a.ZL = s.ar_b + L.zl;
    a.CR = s.ar_b + L.cr;
    a.ldcr = L.ldcr;
    a.kt = nullptr;  // (the live Eta timer times the stream)
    a.arb_flag = s.shard_dev ? arb_flag_ptr(s) : nullptr;
    launch_eta_fused_mode<EF_SOLVE>(s, a);
    return;
  }
  for (int r = 0; r < s.nr; ++r) HMSC_REQUIRE(s.lev[r].nf >= 1, "updateEta: a level has zero factors");
  eta_levels(s, iter, s.ar_b + L.zl, 1, s.ar_b + L.cr, L.ldcr, s.n_na_rows > 0 ? s.ar_b + L.na : nullptr);
}

// One sweep of a sharded chain in the reference order (R/sampleMcmc.R:219-306); see the
// section comment above.  GammaV's algebra and the delta chains (they feed only the next
// sweep) run on the side stream after all-reduce B, joined before the next sweep's Gamma2.
void sweep_sharded(State& s, uint32_t iter) {
  ProfScope ps(s, PROF_SWEEP);
  HMSC_REQUIRE(!(s.mask & HMSC_UP_GAMMAETA), "updateGammaEta cannot run on a species-sharded chain");
  const bool fused = sharded_fused_ok(s);
  s.side_fused = false;
  // edge-free graph sweeps (an RCCL chain alone on its device, the side stream forked at the
  // capture's root): as on one chain's unsharded sweep, the side chain is neither forked nor
  // joined by graph edges -- it waits on the device for arb_flag, raised by the Eta solve after
  // all-reduce B, and the next fused launch waits for its side_sync flags -- so the sweep's main
  // kernels stay on one queue (each cross-queue edge cost ~10 us per sweep)
  s.shard_dev = fused && s.comm != nullptr && s.capturing && s.edge_free_now && s.side_root;
  if (!(s.shard_dev && s.cap_sweep > 0 && s.side_tail)) join_side(s);
  if (s.nr > 0 && !s.xeta_valid) launch_xeta(s);
  if (fused) {
    launch_gamma2_bl(s, iter);  // Gamma2 from ar_a; BetaLambda; the tail's CR, LS, psi, GammaV / psi sums
    EtaFArgs a = make_etaf_args(s, iter);
    a.ZL = s.ar_b + arb_layout(s).zl;
    ProfScope pe(s, PROF_ETA_UNIT);
    launch_eta_fused_mode<EF_STREAM>(s, a);  // this rank's ZL
  } else {
    if (s.mask & HMSC_UP_GAMMA2) launch_gamma2_sharded(s, iter);
    if (s.mask & HMSC_UP_BETALAMBDA) launch_beta_lambda(s, iter);
    if (s.mask & HMSC_UP_GAMMAV) shard_gv_stats(s, s.stream);
    if ((s.mask & HMSC_UP_LAMBDAPRIORS) && s.nr > 0) shard_psi(s, iter, s.stream);
    if ((s.mask & HMSC_UP_ETA) && s.nr > 0) {
      if (!s.xeta_valid) launch_xeta(s);
      shard_eta_stats(s);
    }
  }
  const ArbLayout L = arb_layout(s);
  ar_point(s, s.ar_b, L.n);  // all-reduce B
  // GammaV (+ Gamma2's prep) and the delta chains, beside Eta and updateZ
  const bool side_gv = (s.mask & HMSC_UP_GAMMAV) != 0, side_lp = (s.mask & HMSC_UP_LAMBDAPRIORS) && s.nr > 0;
  s.side_tail = false;
  if (s.shard_dev && (s.mask & HMSC_UP_ETA) && s.nr > 0) {
    // the main continuation first (the Eta solve raises arb_flag), then the side chain on the
    // side stream, in the capture since the root fork, behind no edge
    shard_eta_solve(s, iter, fused);
    GVWArgs gw = make_gvw_args(s, iter, s.ar_b + L.gv, 1, s.d_iter);
    LPArgs lp = make_lp_args(s, iter);
    lp.iter_dev = gw.iter_dev;
    gw.flags = s.side_sync;  // published for the next fused launch (side_wait)
    const int* af = arb_flag_ptr(s);
    switch (wv_bucket_gv(s.nc * s.nt)) {
      case 8: launch_side_chain<8>(s, gw, lp, s.ar_b + L.rs, 1, s.NF, af); break;
      case 16: launch_side_chain<16>(s, gw, lp, s.ar_b + L.rs, 1, s.NF, af); break;
      case 20: launch_side_chain<20>(s, gw, lp, s.ar_b + L.rs, 1, s.NF, af); break;
      case 24: launch_side_chain<24>(s, gw, lp, s.ar_b + L.rs, 1, s.NF, af); break;
      default: launch_side_chain<32>(s, gw, lp, s.ar_b + L.rs, 1, s.NF, af); break;
    }
    HIP_OK(hipGetLastError());
    if (gw.do_prep) s.g2prep_valid = true;
    s.side_tail = true;
    s.side_pending |= 1;
  } else if (side_gv || side_lp) {
    HIP_OK(hipEventRecord(s.ev_bl, s.stream));
    HIP_OK(hipStreamWaitEvent(s.side, s.ev_bl, 0));
    if (fused) {
      GVWArgs gw = make_gvw_args(s, iter, s.ar_b + L.gv, 1, s.capturing ? s.d_iter : nullptr);
      LPArgs lp = make_lp_args(s, iter);
      lp.iter_dev = gw.iter_dev;
      switch (wv_bucket_gv(s.nc * s.nt)) {
        case 8: launch_side_chain<8>(s, gw, lp, s.ar_b + L.rs, 1, s.NF, nullptr); break;
        case 16: launch_side_chain<16>(s, gw, lp, s.ar_b + L.rs, 1, s.NF, nullptr); break;
        case 20: launch_side_chain<20>(s, gw, lp, s.ar_b + L.rs, 1, s.NF, nullptr); break;
        case 24: launch_side_chain<24>(s, gw, lp, s.ar_b + L.rs, 1, s.NF, nullptr); break;
        default: launch_side_chain<32>(s, gw, lp, s.ar_b + L.rs, 1, s.NF, nullptr); break;
      }
      HIP_OK(hipGetLastError());
      if (gw.do_prep) s.g2prep_valid = true;
    } else {
      if (side_gv) shard_gammav_final(s, iter, s.side);
      if (side_lp) shard_delta(s, iter, s.side);
    }
    s.side_pending |= 1;
  }
  if ((s.mask & HMSC_UP_ETA) && s.nr > 0 && !s.shard_dev) shard_eta_solve(s, iter, fused);
  if (s.mask & HMSC_UP_ALPHA) launch_alpha(s, iter);
  if (s.mask & HMSC_UP_INVSIGMA) launch_inv_sigma(s, iter);
  s.g2s_valid = false;
  // HMSC_G2S_SLAB: all-reduce A's sums formed in updateZ's slab launch from the chunk partials
  // instead of a launch after it -- measured slower (ns = 1000: Z end -> next Gamma2 16.3 ->
  // 18.7 us; ns = 125: 18.7 -> 25.4 us; the stats' 64-deep partial sums lengthen the slab
  // launch more than the launch they replace), so off by default
  s.g2s_slab_req = fused && !s.has_na && getenv_flag("HMSC_G2S_SLAB");  // (with NA: X^T Z Tr from ZTr)
  if (s.mask & HMSC_UP_Z) launch_update_z(s, iter, false);
  s.g2s_slab_req = false;
  shard_g2_stats(s);  // all-reduce A, for the next sweep's updateGamma2
  s.g2s_slab = false;
  s.shard_dev = false;
}

// hmsc_update(which) on a sharded chain: the updater with its own all-reduce (the sweep merges
// them into A and B)
void run_updater_sharded(State& s, uint32_t which, uint32_t iter) {
  const ArbLayout L = arb_layout(s);
  switch (which) {
    case HMSC_UP_GAMMA2:
      launch_gamma2_sharded(s, iter);
      break;
    case HMSC_UP_GAMMAETA:
      throw HmscError(-1, "updateGammaEta cannot run on a species-sharded chain");
    case HMSC_UP_BETALAMBDA:
      join_side(s);
      launch_beta_lambda(s, iter);
      s.g2s_valid = false;
      break;
    case HMSC_UP_GAMMAV:
      join_side(s);
      shard_gv_stats(s, s.stream);
      ar_point(s, s.ar_b + L.gv, (size_t)s.nc * s.nc + (size_t)s.nc * s.nt);
      shard_gammav_final(s, iter, s.stream);
      break;
    case HMSC_UP_RHO:
      break;  // no phylogeny on a sharded chain
    case HMSC_UP_LAMBDAPRIORS:
      if (s.nr == 0) break;
      join_side(s);
      shard_psi(s, iter, s.stream);
      ar_point(s, s.ar_b + L.rs, s.NF);
      shard_delta(s, iter, s.stream);
      break;
    case HMSC_UP_ETA:
      if (s.nr == 0) break;
      join_side(s);
      if (!s.xeta_valid) launch_xeta(s);
      shard_eta_stats(s);
      ar_point(s, s.ar_b + L.zl, L.gv - L.zl);  // ZL | CR
      if (s.n_na_rows > 0) ar_point(s, s.ar_b + L.na, L.n - L.na);
      shard_eta_solve(s, iter, false);
      s.g2s_valid = false;
      break;
    case HMSC_UP_ALPHA:
      launch_alpha(s, iter);
      break;
    case HMSC_UP_INVSIGMA:
      launch_inv_sigma(s, iter);
      s.g2s_valid = false;
      break;
    case HMSC_UP_Z:
      launch_update_z(s, iter, false);
      s.g2s_valid = false;
      break;
    default:
      throw HmscError(-1, "unknown or out-of-scope updater bit");
  }
}

}  // namespace hmsc
