// updateZ device kernel (R/updateZ.R:4-94), shared by kernels.hip and the microbenchmark
// scripts/ubench_z.hip.  See kernels.hip for the launcher (run_z_fused).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.h"
#include "rng.h"
#include "record.h"
#include "z_tables.h"

namespace hmsc {

// ---------------------------------------------------------------------------
// updateZ (R/updateZ.R:4-94) fused with the contractions of Z the next sweep needs.
//
// A workgroup (4 waves) owns 32 species (sBL in LDS) and a chunk of 64-site tiles;
// wave w takes the 16-site sub-tile w of every tile, and the waves never synchronise
// inside the site loop.  Per 16-site x 32-species wave tile, all in registers:
//   E    = XEta BL          v_mfma_f64_16x16x4 (A = XEta rows, B = BL columns); the
//                           accumulator leaves lane l holding sites lk+4r (r=0..3) of
//                           species pair m = l&15, i.e. species j0+2m and j0+2m+1
//   Z    truncated-normal draws (VALU); one Philox call feeds a species quad (two of the
//                           lane's pairs, one 32-bit uniform a cell)
//   XZ  += XEta^T (Yx o Z)  the drawn Z already sits in the B-operand layout of this
//                           MFMA (sites = reduction index), A = XEta^T from a wave-
//                           private LDS copy of the site tile
//   ZTr  = Z Tr             DPP row reductions over the 16 species pairs
// so Z is written once and never re-read by updateBetaLambda or updateGamma2.
// ---------------------------------------------------------------------------
// XEta and Ycode are allocated with padding (capi.cpp build_state) so the kernel loads them
// unguarded: XEta holds ny * 16 ceil(Kmax / 16) + 64 doubles (finite; columns >= K and the
// rows past ny of the last tile only ever meet zero BL rows / zeroed Z), Ycode ny (nsl + 32) + 64
// bytes (zero past the last species), Ybits ceil(nsl / 32) ny + 64 words (code 0 past the last
// species and site).
struct ZArgs {
  const double* XEta;  // ny x K (ld ny)
  int ny, K, ns_loc, sp0, nt, tiles_per_chunk;
  const double* BL;
  const double* iSigma;
  const int8_t* Ycode;
  const uint64_t* Ybits;  // [species block][site]: 2 bits per species (code + 1: 0 NA, 1 zero, 2 one)
  const double* Yval;
  const int* fam;
  const double* Tr;  // local species rows, ld ns_loc
  double* Z;
  double* XZ_part;   // [chunk][K x ns_loc]
  double* ZTr_part;  // [species block][ny x nt]
  Key key;
  uint32_t iter;
  const uint32_t* iter_dev;  // graph replay: the sweep counter is read from the device
  int noise_zero;
  int zprev_is_e;            // chain init: ZPrev = LFix + LRan (R/computeInitialParameters.R:250-254)
  // NA cells leave the XZ contraction (the C = NULL branch's per-species observed rows,
  // R/updateBetaLambda.R:103-117); 0 with a phylogeny, whose dense system takes the full
  // crossprod(XEta, S) over the imputed Z (:66, :124-146)
  int mask_na;
  unsigned long long* kt;    // live launch timing (KT_Z block) or null
  // G = XEta^T XEta's Eta rows from the fused Eta pass' tile partials, reduced by the first
  // grid row's workgroups while the others draw (gred_y0 = 1; see g_reduce_body)
  int gred_y0, gred_groups, gred_ntile, gred_nf, gred_Kmax;
  const double* gred_part;
  const double* gred_XX;
  double* gred_G;
  const double* logtab;  // z_log_table (ZLOG_N x ZLOG_W doubles), staged in LDS by every workgroup
  const double* ztab;    // z_draw_tables (ZT_DOUBLES: erfcx | F(w) | 2^(k/64)), staged in LDS likewise
  // pack_row: a grid row packs the sweep's main-stream record pieces (BL, Psi, iSigma, Eta:
  // final before this launch, not written by it) instead of a launch after it -- the last
  // row (1) or the first after the G row (2)
  int pack_row;
  PackArgs pack;
};

constexpr int ZT_I = 64;   // sites per workgroup tile (4 waves x 16)
constexpr int ZT_J = 32;   // species per workgroup (16 pairs)
constexpr int KMAX_Z = 128;
constexpr int ZT_LD = 65;  // padded LDS leading dimension of the 64-site XEta tile (xeta_gram_kernel)

typedef double d4 __attribute__((ext_vector_type(4)));

// v_mfma_f64_16x16x4_f64: D[16x16] += A[16x4] B[4x16]; lane l supplies A[l&15][l>>4] and
// B[l>>4][l&15] and holds D[(l>>4) + 4r][l&15], r = 0..3 (checked by scripts/mfma_layout_check.hip).
__device__ __forceinline__ d4 mfma_f64(double a, double b, d4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// LDS written by one lane of a wave and read by another lane of the same wave
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// v rotated right by N lanes inside each row of 16 lanes (DPP row_ror)
template <int N>
__device__ __forceinline__ double row_ror(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)b, 0x120 + N, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), 0x120 + N, 0xF, 0xF, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ double row_sum16(double v) {
  v += row_ror<8>(v);
  v += row_ror<4>(v);
  v += row_ror<2>(v);
  v += row_ror<1>(v);
  return v;
}

// one latent draw (rare paths: Poisson-chain kernels, the tails of the paired draw below)
//   code 1 / 0: probit TN(E, sd) on [0, inf) / (-inf, 0]     R/updateZ.R:43-63
//   code < 0 : NA cell, N(E, sd) = truncation at -inf           R/updateZ.R:92
__device__ __noinline__ double z_probit_draw(double e, double sd, double isd, int code, double u, int noise_zero) {
  const double sg = code == 0 ? -1.0 : 1.0;
  if (code < 0 && noise_zero) return e;
  const double alpha = code < 0 ? -INFINITY : -sg * e * isd;
  return e + sd * sg * trunc_normal_lower(alpha, u);
}

// Two truncated-normal draws of one Philox block (species 2m and 2m+1 of a site), out of
// line (the ~60 polynomial coefficients then live in SGPRs only inside the call, instead of
// being hoisted into the kernel's register file), with their Horner chains interleaved: the
// same arithmetic as trunc_normal_lower (rng.h) on each cell, two independent dependency
// chains per lane.  Tails (alpha > 25, or a quantile outside qnorm_fast's central branch,
// w >= 6.25) take the scalar path.
// log x for positive normal x by Tang's table method: x = m 2^e with m in [1, 2), c_j the
// midpoint of the 1/64-wide interval holding m (its top six mantissa bits), r = (m - c_j) / c_j
// with |r| <= 1/129, log x = e ln2 + log c_j + log1p(r), log1p by its degree-5 series (|r^6/6|
// < 4e-14 absolute).  The table row j = {1 / c_j, log c_j} (16 bytes: one ds_read_b128) lives
// in LDS (z_log_table fills it on the host in extended precision); ~14 VALU instructions.
constexpr int ZLOG_N = 64;
constexpr int ZLOG_W = 2;  // doubles per table row
inline void z_log_table(double* t) {
  for (int j = 0; j < ZLOG_N; ++j) {
    const long double c = 1.0L + (2 * j + 1) / 128.0L;
    t[ZLOG_W * j] = (double)(1.0L / c);
    t[ZLOG_W * j + 1] = (double)logl(c);
  }
}
HMSC_TABLE double kLog1pSeries[5] = {1.0 / 5.0, -1.0 / 4.0, 1.0 / 3.0, -1.0 / 2.0, 1.0};
__device__ __forceinline__ double log_tab(double x, const double* tab) {
  const int e = __builtin_amdgcn_frexp_exp(x) - 1;        // x = m2 2^e, m2 in [1, 2)
  const double m2 = 2.0 * __builtin_amdgcn_frexp_mant(x);
  uint64_t b;
  __builtin_memcpy(&b, &m2, 8);
  const uint32_t hi = (uint32_t)(b >> 32);
  const int j = (int)((hi >> 14) & 63u);
  const uint64_t cb = (uint64_t)((hi & 0xFFFFC000u) | 0x2000u) << 32;  // c_j = 1 + j / 64 + 1 / 128
  double c;
  __builtin_memcpy(&c, &cb, 8);
  const double* tj = tab + ZLOG_W * j;
  const double r = (m2 - c) * tj[0];                      // m2 - c_j exact
  double P = kLog1pSeries[0];
#pragma unroll
  for (int k = 1; k < 5; ++k) P = fma_sc(P, r, kLog1pSeries[k]);
  const double de = (double)e;
  return fma(de, 0.6931471803691238, tj[1]) + fma(r, P, de * 1.9082149292705877e-10);
}

struct ZPair {
  double z0, z1;
};

// ---------------------------------------------------------------------------------------------
// The LDS-table draw (round 5).  The same inversion, z = e - sd sg Phi^-1(u Phic(alpha)), with
// every special function a table lookup plus a low-degree polynomial (scripts/fit_tables.py,
// z_tables.h; coefficients staged in LDS, read as 16-byte pairs):
//   Phic(alpha)  = erfc(a) / 2 (alpha >= 0) or 1 - erfc(a) / 2, a = |alpha| / sqrt 2, with
//                  erfc(a) = exp(-a^2) erfcx(a): erfcx on 72 segments of width 1/4 (degree 9,
//                  1.1e-14 relative), exp(-a^2) with a^2 split exactly (hi + lo) and exp by the
//                  2^(k/64) table and a degree-5 polynomial (|r| <= ln2 / 128: 4e-17)
//   w            = -log(4 p (1 - p))  (log_tab, as before)
//   Phi^-1(p)    = (2p - 1) F(w), F on 64 segments of width 1/4 over w in [0, 16) (degree 7,
//                  3.3e-15) -- one branch for all p in (2.8e-8, 1 - 2.8e-8), where the previous
//                  global fits switched to a second polynomial (and a sqrt) at w = 6.25 in a
//                  third of the wave iterations; AS241's tail beyond, as before
// replacing the degree-20 erfc polynomial with its reciprocal and exp, and the degree-18 / 14
// quantile polynomials (~45 fewer VALU instructions per cell, no region-B divergence).
// Row strides (doubles): rows start 16-byte aligned and their LDS banks (4-dword quads,
// bank = dword mod 64) differ for rows j, j' unless j = j' (mod 16) -- a stride of 20 dwords; an
// 8-coefficient row at its natural 16 dwords put rows j, j + 4, j + 8, ... of the quantile
// table on the same quad, a 4-way conflict among the lanes of a 16-lane group
#ifndef ZT_Q_LD_DEF
#define ZT_Q_LD_DEF 10
#endif
constexpr int ZT_E_LD = 10, ZT_Q_LD = ZT_Q_LD_DEF;
constexpr int ZT_E_SEG = ZT_E_MAX * ZT_E_PER_UNIT, ZT_Q_SEG = ZT_Q_MAX * ZT_Q_PER_UNIT;
// The exp and log tables are read at data-dependent rows by every lane.  ZT_COMPACT (round 6):
// 32-entry tables of 8-byte words, each 64 dwords -- one LDS bank row, so a ds_read_b64 half-wave
// (banks (a/4) mod 64) never meets two rows on one bank -- instead of the 64-entry 2^(k/64)
// table (rows k and k + 32 shared banks: 2-way) and the 64 x 16-byte log rows read by
// ds_read_b128 (rows j, j + 16, j + 32, j + 48 on one bank quad: up to 4-way among 16 lanes).
// The exp polynomial goes one degree up (|r| <= ln2 / 64) and the log1p series two (|r| <= 1 / 65).
// Measured (profiles/r06_zab.txt): conflicts 34 -> 26 % of LDS-active cycles, but +0.5 M VALU per
// launch and z 79.2 -> 80.0 us in the full sweep, so off by default.
#ifndef ZT_COMPACT
#define ZT_COMPACT 0
#endif
constexpr int ZT_X_N = ZT_COMPACT ? 32 : 64;
constexpr int ZT_OFF_E = 0, ZT_OFF_Q = ZT_E_SEG * ZT_E_LD, ZT_OFF_X = ZT_OFF_Q + ZT_Q_SEG * ZT_Q_LD;
constexpr int ZT_OFF_LI = ZT_OFF_X + ZT_X_N, ZT_OFF_LL = ZT_OFF_LI + 32;  // (ZT_COMPACT) 1 / c_j, log c_j
constexpr int ZT_DOUBLES = ZT_OFF_LL + 32;
static_assert(ZT_E_NC % 2 == 0 && ZT_Q_NC % 2 == 0 && ZT_E_LD % 2 == 0 && ZT_Q_LD % 2 == 0 && ZT_E_LD >= ZT_E_NC &&
                  ZT_Q_LD >= ZT_Q_NC,
              "16-byte rows");
inline void z_draw_tables(double* t) {
  for (int i = 0; i < ZT_DOUBLES; ++i) t[i] = 0.0;
  for (int j = 0; j < ZT_E_SEG; ++j)
    for (int k = 0; k < ZT_E_NC; ++k) t[ZT_OFF_E + ZT_E_LD * j + k] = kZtErfcx[ZT_E_NC * j + k];
  for (int j = 0; j < ZT_Q_SEG; ++j)
    for (int k = 0; k < ZT_Q_NC; ++k) t[ZT_OFF_Q + ZT_Q_LD * j + k] = kZtQnormF[ZT_Q_NC * j + k];
  for (int i = 0; i < ZT_X_N; ++i) t[ZT_OFF_X + i] = kZtExp2[(64 / ZT_X_N) * i];  // 2^(i / ZT_X_N)
  for (int j = 0; j < 32; ++j) {  // log table on 32 intervals of [1, 2): c_j = 1 + j / 32 + 1 / 64
    const long double c = 1.0L + (2 * j + 1) / 64.0L;
    t[ZT_OFF_LI + j] = (double)(1.0L / c);
    t[ZT_OFF_LL + j] = (double)logl(c);
  }
}
typedef double zt_d2 __attribute__((ext_vector_type(2)));

// polynomial of table row `row` (NC coefficients, highest first, 16-byte aligned) at d
template <int NC>
__device__ __forceinline__ double zt_poly(const double* row, double d) {
  const zt_d2* r2 = (const zt_d2*)row;
  zt_d2 c[NC / 2];
#pragma unroll
  for (int k = 0; k < NC / 2; ++k) c[k] = r2[k];  // ds_read_b128, all issued before the chain
  double v = c[0][0];
  v = fma(v, d, c[0][1]);
#pragma unroll
  for (int k = 1; k < NC / 2; ++k) {
    v = fma(v, d, c[k][0]);
    v = fma(v, d, c[k][1]);
  }
  return v;
}

HMSC_TABLE double kZtExpPoly[6] = {1.0 / 120.0, 1.0 / 24.0, 1.0 / 6.0, 0.5, 1.0, 1.0};
HMSC_TABLE double kZtExpPoly7[7] = {1.0 / 720.0, 1.0 / 120.0, 1.0 / 24.0, 1.0 / 6.0, 0.5, 1.0, 1.0};
HMSC_TABLE double kLog1pSeries7[7] = {1.0 / 7.0, -1.0 / 6.0, 1.0 / 5.0, -1.0 / 4.0, 1.0 / 3.0, -1.0 / 2.0, 1.0};
// log x for positive normal x (log_tab on the compact tables): m2 in [1, 2) on 32 intervals,
// |r| <= 1 / 65, log1p(r) by its degree-7 series (|r^8 / 8| < 4e-16 absolute)
__device__ __forceinline__ double log_tab32(double x, const double* zt) {
  const int e = __builtin_amdgcn_frexp_exp(x) - 1;
  const double m2 = 2.0 * __builtin_amdgcn_frexp_mant(x);
  uint64_t b;
  __builtin_memcpy(&b, &m2, 8);
  const uint32_t hi = (uint32_t)(b >> 32);
  const int j = (int)((hi >> 15) & 31u);
  const uint64_t cb = (uint64_t)((hi & 0xFFFF8000u) | 0x4000u) << 32;  // c_j = 1 + j / 32 + 1 / 64
  double c;
  __builtin_memcpy(&c, &cb, 8);
  const double r = (m2 - c) * zt[ZT_OFF_LI + j];
  double P = kLog1pSeries7[0];
#pragma unroll
  for (int k = 1; k < 7; ++k) P = fma_sc(P, r, kLog1pSeries7[k]);
  const double de = (double)e;
  return fma(de, 0.6931471803691238, zt[ZT_OFF_LL + j]) + fma(r, P, de * 1.9082149292705877e-10);
}
// erfc(a) for 0 <= a < ZT_E_MAX (the caller clamps a)
__device__ __forceinline__ double zt_erfc(double a, const double* zt) {
  const int j = min((int)(a * (double)ZT_E_PER_UNIT), ZT_E_SEG - 1);
  const double d = a - ((double)j + 0.5) * (1.0 / ZT_E_PER_UNIT);
  const double cx = zt_poly<ZT_E_NC>(zt + ZT_OFF_E + ZT_E_LD * j, d);
  // exp(-(hi + lo)), a^2 = hi + lo exactly: k = rint(-hi N / ln2), r = -hi - k ln2 / N - lo
  const double hi = a * a, lo = fma(a, a, -hi);
#if ZT_COMPACT
  const double kf = __builtin_rint(hi * -46.16624130844683);  // 32 / ln2
  double r = fma(kf, -0.02166084938653512, -hi);              // ln2 / 32 = hi (fdlibm's ln2_hi / 32: k hi exact)
  r = fma(kf, -5.9631716539705866e-12, r) - lo;               //            + lo
  double p = kZtExpPoly7[0];
#pragma unroll
  for (int k = 1; k < 7; ++k) p = fma_sc(p, r, kZtExpPoly7[k]);
  const int ki = (int)kf;
  return __builtin_ldexp(p * zt[ZT_OFF_X + (ki & 31)], ki >> 5) * cx;
#else
  const double kf = __builtin_rint(hi * -92.33248261689366);  // 64 / ln2
  double r = fma(kf, -0.01083042469326756, -hi);              // ln2 / 64 = hi (fdlibm's ln2_hi / 64: k hi exact)
  r = fma(kf, -2.9815858269852933e-12, r) - lo;               //            + lo
  double p = kZtExpPoly[0];
#pragma unroll
  for (int k = 1; k < 6; ++k) p = fma_sc(p, r, kZtExpPoly[k]);
  const int ki = (int)kf;
  return __builtin_ldexp(p * zt[ZT_OFF_X + (ki & 63)], ki >> 6) * cx;
#endif
}

// (2p - 1) F(w) = Phi^-1(p) for w = -log(4 p (1 - p)) < ZT_Q_MAX
__device__ __forceinline__ double zt_qnorm_w(double p, double w, const double* zt) {
  const int j = max(0, min((int)(w * (double)ZT_Q_PER_UNIT), ZT_Q_SEG - 1));
  const double d = w - ((double)j + 0.5) * (1.0 / ZT_Q_PER_UNIT);
  return (2.0 * p - 1.0) * zt_poly<ZT_Q_NC>(zt + ZT_OFF_Q + ZT_Q_LD * j, d);
}

__device__ __forceinline__ ZPair z_probit_pair_tab(double e0, double e1, double sd0, double sd1, double isd0,
                                                double isd1, int c0, int c1, double u0, double u1, int noise_zero,
                                                const double* ltab, const double* zt) {
  const double sg0 = c0 == 0 ? -1.0 : 1.0, sg1 = c1 == 0 ? -1.0 : 1.0;
  const double al0 = c0 < 0 ? -INFINITY : -sg0 * e0 * isd0;
  const double al1 = c1 < 0 ? -INFINITY : -sg1 * e1 * isd1;
  double q0, q1;  // -Phic^-1 (u Phic(alpha)) = qnorm(p), z = e - sd sg q
  if (al0 > 25.0 || al1 > 25.0) {  // deep tail of either cell: each cell by the scalar inversion
    q0 = -trunc_normal_lower(al0, u0);
    q1 = -trunc_normal_lower(al1, u1);
  } else {
    // a >= 17.99 only for alpha < -25.4, where Phic(alpha) = 1 - erfc(a) / 2 rounds to 1
    const double a0 = fmin(fabs(al0) * 0.7071067811865476, 17.99);
    const double a1 = fmin(fabs(al1) * 0.7071067811865476, 17.99);
    const double r0 = 0.5 * zt_erfc(a0, zt), r1 = 0.5 * zt_erfc(a1, zt);
    const double p0 = u0 * (al0 < 0.0 ? 1.0 - r0 : r0);
    const double p1 = u1 * (al1 < 0.0 ? 1.0 - r1 : r1);
#if ZT_COMPACT
    const double w0 = -log_tab32(4.0 * p0 * (1.0 - p0), zt), w1 = -log_tab32(4.0 * p1 * (1.0 - p1), zt);
#else
    const double w0 = -log_tab(4.0 * p0 * (1.0 - p0), ltab), w1 = -log_tab(4.0 * p1 * (1.0 - p1), ltab);
#endif
    q0 = zt_qnorm_w(p0, w0, zt);
    q1 = zt_qnorm_w(p1, w1, zt);
    if (w0 >= (double)ZT_Q_MAX || w1 >= (double)ZT_Q_MAX) {  // p < 2.8e-8 or > 1 - 2.8e-8: AS241's tail
      if (w0 >= (double)ZT_Q_MAX) q0 = qnorm_as241_tail_t(p0, kLogSeries);
      if (w1 >= (double)ZT_Q_MAX) q1 = qnorm_as241_tail_t(p1, kLogSeries);
    }
  }
  ZPair z;
  z.z0 = (c0 < 0 && noise_zero) ? e0 : e0 - sd0 * sg0 * q0;
  z.z1 = (c1 < 0 && noise_zero) ? e1 : e1 - sd1 * sg1 * q1;
  return z;
}
__device__ __forceinline__ ZPair z_probit_pair(double e0, double e1, double sd0, double sd1, double isd0, double isd1,
                                            int c0, int c1, double u0, double u1, int noise_zero,
                                            const double* ltab) {
  const double sg0 = c0 == 0 ? -1.0 : 1.0, sg1 = c1 == 0 ? -1.0 : 1.0;
  const double al0 = c0 < 0 ? -INFINITY : -sg0 * e0 * isd0;
  const double al1 = c1 < 0 ? -INFINITY : -sg1 * e1 * isd1;
  double q0, q1;  // -Phic^-1 (u Phic(alpha)) = qnorm(p), z = e - sd sg q
  if (al0 > 25.0 || al1 > 25.0) {  // deep tail of either cell: each cell by the scalar inversion
    q0 = -trunc_normal_lower(al0, u0);
    q1 = -trunc_normal_lower(al1, u1);
  } else {
    // erfc_fast(alpha / sqrt 2) for both cells
    const double h0 = al0 * 0.7071067811865476, h1 = al1 * 0.7071067811865476;
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
    const double p0 = u0 * (0.5 * (h0 < 0.0 ? 2.0 - r0 : r0));
    const double p1 = u1 * (0.5 * (h1 < 0.0 ? 2.0 - r1 : r1));
    // w = -log(4 p (1 - p)) for both cells (table log, ltab in LDS)
    const double w0 = -log_tab(4.0 * p0 * (1.0 - p0), ltab), w1 = -log_tab(4.0 * p1 * (1.0 - p1), ltab);
    // qnorm_fast's central branch (w < 6.25) for both cells, on every lane
    const double y0 = w0 - 3.125, y1 = w1 - 3.125;
    double F0 = kQnormA[0], F1 = kQnormA[0];
#pragma unroll
    for (int k = 1; k < QNA_NC; ++k) {
      F0 = fma_sc(F0, y0, kQnormA[k]);
      F1 = fma_sc(F1, y1, kQnormA[k]);
    }
    q0 = (2.0 * p0 - 1.0) * F0;
    q1 = (2.0 * p1 - 1.0) * F1;
    if (w0 >= 6.25 || w1 >= 6.25) {
      // a lane with a cell in qnorm_fast's outer branches (p within 4.8e-4 of 0 or 1: about
      // a third of the wave iterations on a fitted probit model hold one): region B for both
      // cells, reusing w -- not the whole quantile again -- and AS241's tail below p < 2.8e-8
      const double sw0 = sqrt(fmax(w0, 6.25)) - 3.25, sw1 = sqrt(fmax(w1, 6.25)) - 3.25;
      double B0 = kQnormB[0], B1 = kQnormB[0];
#pragma unroll
      for (int k = 1; k < QNB_NC; ++k) {
        B0 = fma_sc(B0, sw0, kQnormB[k]);
        B1 = fma_sc(B1, sw1, kQnormB[k]);
      }
      if (w0 >= 6.25) q0 = w0 < 16.0 ? (2.0 * p0 - 1.0) * B0 : qnorm_as241_tail_t(p0, kLogSeries);
      if (w1 >= 6.25) q1 = w1 < 16.0 ? (2.0 * p1 - 1.0) * B1 : qnorm_as241_tail_t(p1, kLogSeries);
    }
  }
  ZPair z;
  z.z0 = (c0 < 0 && noise_zero) ? e0 : e0 - sd0 * sg0 * q0;
  z.z1 = (c1 < 0 && noise_zero) ? e1 : e1 - sd1 * sg1 * q1;
  return z;
}

// Poisson cell (R/updateZ.R:65-90): omega ~ PG(y + r, zPrev - log r) with r = 1000, then
// Z ~ N(sigmaZ ((y - r)/2 + prec (E - log r)) + log r, sigmaZ), sigmaZ = 1 / (prec + omega).
// BayesLogit's rpg takes its normal-approximation branch for h > 170 (always: h >= 1000), so
// omega = PG mean + PG sd * N(0,1); both normals invert the cell's own Philox block (S_ZPOIS).
__device__ __noinline__ double z_poisson_draw(double e, double sd, double y, double zprev, Uniform2 u,
                                              int noise_zero) {
  constexpr double R_NB = 1000.0, LOG_R = 6.907755278982137;
  double m, v;
  pg_moments(y + R_NB, zprev - LOG_R, &m, &v);
  const double omega = noise_zero ? m : fma(sqrt(v), qnorm_fast(u.a), m);
  const double prec = 1.0 / (sd * sd);
  const double sigz = 1.0 / (prec + omega);
  const double muz = fma(sigz, fma(prec, e - LOG_R, 0.5 * (y - R_NB)), LOG_R);
  return noise_zero ? muz : fma(sqrt(sigz), qnorm_fast(u.b), muz);
}

// G's Eta rows (R/updateBetaLambda.R:21-41 of the next sweep: XEta^T XEta), deterministic:
// output group g (64 outputs of the K x nf slab, lane = output), the 4 waves taking every 4th
// tile, combined in LDS in wave order; written to (k, nc + h) and (nc + h, k).  The X^T X block
// is the constant XX.  Runs on the z launch's first grid row, off updateZ's critical path.
__device__ inline void g_reduce_body(const ZArgs& a, double* red) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int K = a.K, Kmax = a.gred_Kmax, nf = a.gred_nf, nc = K - nf;
  const size_t stride = (size_t)Kmax * nf;
  for (int g = blockIdx.x; g < a.gred_groups; g += gridDim.x) {
    const int o = g * 64 + lane, k = o % K, h = o / K;
    double s = 0.0;
    if (o < K * nf) {
      const double* p = a.gred_part + k + (size_t)Kmax * h;
      int b = w;
      for (; b + 4 * 19 < a.gred_ntile; b += 4 * 20) {
        double x[20];
#pragma unroll
        for (int u = 0; u < 20; ++u) x[u] = p[stride * (b + 4 * u)];
#pragma unroll
        for (int u = 0; u < 20; ++u) s += x[u];
      }
      for (; b < a.gred_ntile; b += 4) s += p[stride * b];
    }
    __syncthreads();
    red[w * 64 + lane] = s;
    __syncthreads();
    if (w == 0 && o < K * nf) {
      const double v = (red[lane] + red[64 + lane]) + (red[128 + lane] + red[192 + lane]);
      a.gred_G[k + (size_t)Kmax * (nc + h)] = v;
      a.gred_G[(nc + h) + (size_t)Kmax * k] = v;
    }
    if (g == 0)
      for (int p = threadIdx.x; p < nc * nc; p += blockDim.x) a.gred_G[p % nc + (size_t)Kmax * (p / nc)] = a.gred_XX[p];
  }
}

// NKB = 16-row blocks of K (XZ output tiles per species block)
// MODE bits (all set in the product; the microbenchmark clears them to cost each part):
//   1 = E on the matrix cores, 2 = draws, 4 = XZ contraction, 8 = ZTr contraction
constexpr int Z_ALL = 15;
constexpr int Z_NOSTORE = 16;  // microbenchmark only: skip the Z stores
constexpr int ZT_TLD = 17;  // leading dimension of the wave's 16-site x 32-species tile T[jj][site]

// POIS: instantiated only for chains with Poisson species, so the probit kernel carries no
// Poisson call site (its call-saved registers and code size cost the probit path ~5 %)
// NORMAL: the chain has normal species (their cells copy Yval, R/updateZ.R:40-41); a probit-
// only chain's kernel then issues no load inside the draw loop (a load there would make each
// use wait, vmcnt being in order, behind every Z store still in flight).
// NKB > 4 (64 < K <= 128, one instantiation NKB = 8): the XZ accumulators (128 registers, the
// matrix cores' accumulation registers) at two waves per SIMD; the E and XZ operands are
// loaded 64 rows at a time and the waves' XZ combined 64 rows at a time (LDS).
#ifndef Z_MIN_BLOCKS
#define Z_MIN_BLOCKS 4  // workgroups per CU the K <= 64 instantiations are compiled for (128 registers)
#endif
template <bool DRAW, bool HAS_NA, int NKB, int MODE = Z_ALL, bool POIS = false, bool NORMAL = true>
__global__ __launch_bounds__(256, NKB > 4 ? 2 : Z_MIN_BLOCKS) void z_wave_kernel(ZArgs a) {
  kernarg_warm<sizeof(ZArgs)>();
  extern __shared__ __attribute__((aligned(16))) double smem[];
  if (a.gred_y0 && blockIdx.y == 0) {  // the co-launched G reduction row
    g_reduce_body(a, smem);
    return;
  }
  // the record pack row: last in dispatch order (pack_row 1), or first after the G row (2)
  const int pack_y = a.pack_row == 2 ? a.gred_y0 : (int)gridDim.y - 1;
  if (a.pack_row && (int)blockIdx.y == pack_y) {
    pack_body(a.pack, blockIdx.x, gridDim.x);
    return;
  }
  // grid (species blocks, site chunks): the workgroups of one site chunk are consecutive in
  // dispatch order, so its XEta rows are fetched once per XCD (round-robin placement) while
  // they are L2-resident, instead of once per species block
  const int by = (int)blockIdx.x;                   // species block
  const int chunk = (int)blockIdx.y - a.gred_y0 - (a.pack_row == 2 ? 1 : 0);  // site chunk
  const unsigned long long kt0 = a.kt ? kt_now() : 0ull;
  constexpr int K16 = 16 * NKB;
  const int K = a.K, K4 = (K + 3) & ~3;
  const int ny = a.ny;
  double* sBL = smem;                               // [K16][32], column jj = species j0 + jj
  double* sTr = sBL + K16 * ZT_J;                   // [t][32]
  double* sSd = sTr + ZT_J * a.nt;                  // [32] iSigma^-1/2
  double* sIsd = sSd + ZT_J;                        // [32] iSigma^1/2
  int* sFam = (int*)(sIsd + ZT_J);                  // [32]
  double* sLog = (double*)(sFam + ZT_J);            // [ZLOG_N][ZLOG_W] log table (log_tab)
  double* sZT = sLog + ZLOG_W * ZLOG_N;              // z_draw_tables (16-byte aligned rows)
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, lm = lane & 15, lk = lane >> 4;
  // the Philox sweep counter, read once (a load inside the site loop would wait, vmcnt(0),
  // behind every Z store in flight)
  const uint32_t iter = SWEEP_ITER(a);
  double* sT = sZT + ZT_DOUBLES + w * (ZT_J * ZT_TLD);  // this wave's tile: E, then Z
  const int j0 = by * ZT_J;
  for (int p = t; p < K16 * ZT_J; p += 256) {
    const int k = p >> 5, jj = p & 31, j = j0 + jj;
    sBL[p] = (k < K && j < a.ns_loc) ? a.BL[k + (size_t)K * j] : 0.0;
  }
  for (int p = t; p < ZT_J * a.nt; p += 256) {
    const int jj = p & 31, tt = p >> 5, j = j0 + jj;
    sTr[p] = (j < a.ns_loc) ? a.Tr[j + (size_t)a.ns_loc * tt] : 0.0;
  }
  if (t < ZT_J) {
    const int j = j0 + t;
    const double is = (j < a.ns_loc) ? a.iSigma[j] : 1.0;
    sSd[t] = 1.0 / sqrt(is);
    sIsd[t] = sqrt(is);
    sFam[t] = (j < a.ns_loc) ? a.fam[j] : 0;
  }
  if (DRAW && (MODE & 2)) {
    for (int p = t; p < ZLOG_W * ZLOG_N; p += 256) sLog[p] = a.logtab[p];
    for (int p = t; p < ZT_DOUBLES; p += 256) sZT[p] = a.ztab[p];
  }
  __syncthreads();

  d4 acc[NKB][2];
#pragma unroll
  for (int q = 0; q < NKB; ++q) acc[q][0] = acc[q][1] = d4{0.0, 0.0, 0.0, 0.0};

  const int n_tiles = (ny + ZT_I - 1) / ZT_I;
  const int tb = chunk * a.tiles_per_chunk;
  const int te = min(n_tiles, tb + a.tiles_per_chunk);
  for (int tile = tb; tile < te; ++tile) {
    const int i0 = tile * ZT_I + 16 * w;
    if (i0 >= ny) break;
    // ---- this lane's 8 Y codes (site i0 + lm, species j0 + 2(4c + lk) + b), loaded before
    //      the E contraction so their latency overlaps it; 4 bits each, code + 1
    //      (one 8-byte word per site and species block: 2 bits per species, code + 1)
    uint64_t yw = 0;
    if (DRAW) yw = a.Ybits[(size_t)by * ny + (i0 + lm)];  // padded buffer (ZArgs)
    // code of species jj = 2 m + b of this lane's site
    auto ycode_of = [&](int m, int b) { return (int)((yw >> (4 * m + 2 * b)) & 3u) - 1; };
    // ---- E = XEta BL for 16 sites x 32 species (R/updateZ.R:11-34); T[2m+b][lk+4r] <- E
    if (DRAW) {
      d4 e0 = {0.0, 0.0, 0.0, 0.0}, e1 = {0.0, 0.0, 0.0, 0.0};
      // all K16 operand rows, loaded before the first MFMA (padded buffer, ZArgs: rows k >= K
      // meet zero BL rows), so their latency is paid once per tile
      const double* xp = a.XEta + (i0 + lm) + (size_t)ny * lk;
      constexpr int EC = NKB > 4 ? 16 : K16 / 4;  // operand steps loaded at once
#pragma unroll
      for (int c0 = 0; c0 < K16 / 4; c0 += EC) {
        double xa[EC];
#pragma unroll
        for (int s4 = 0; s4 < EC; ++s4) xa[s4] = xp[(size_t)ny * 4 * (c0 + s4)];
#pragma unroll
        for (int s4 = 0; s4 < EC; ++s4) {
          const int k = 4 * (c0 + s4) + lk;
          if (MODE & 1) {
            e0 = mfma_f64(xa[s4], sBL[k * ZT_J + 2 * lm], e0);
            e1 = mfma_f64(xa[s4], sBL[k * ZT_J + 2 * lm + 1], e1);
          } else {
            e0[s4 & 3] += xa[s4];
          }
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        sT[(2 * lm) * ZT_TLD + lk + 4 * r] = e0[r];
        sT[(2 * lm + 1) * ZT_TLD + lk + 4 * r] = e1[r];
      }
      wave_lds_sync();
    }
    // ---- draws in coalesced order: lane = site s (16 consecutive) x species pair m; the lane's
    //      four pairs are two species quads, m = 8 (c >> 1) + 2 lk + (c & 1); one Philox call per
    //      (site, quad), its words x, y for pair m (c even) and z, w for pair m + 1 (c odd), one
    //      32-bit uniform a cell (rng.h u32o); Z stores are 128-B site runs
    {
      const int s = lm, i = i0 + s;
      U4 qw{0u, 0u, 0u, 0u};
#pragma unroll 1
      for (int c = 0; c < 4; ++c) {
        const int m = 8 * (c >> 1) + 2 * lk + (c & 1), ja = j0 + 2 * m;
        Uniform2 u{0.0, 0.0};
        if (DRAW) {
          if (!(c & 1))  // (the species block and the shard start are multiples of 4)
            qw = philox4x32_10_wave_key(U4{(uint32_t)((size_t)i + (size_t)ny * (uint32_t)((a.sp0 + ja) >> 2)), 0u, (uint32_t)S_Z, iter}, a.key);
          u = (c & 1) ? Uniform2{u32o(qw.z), u32o(qw.w)} : Uniform2{u32o(qw.x), u32o(qw.y)};
        }
        if (DRAW && !POIS && (MODE & 2)) {
          // probit / NA pair (the whole chain is probit, or the pair's species are):
          // both draws inline with interleaved chains; normal species keep Z = Y
          const int cd0 = ycode_of(m, 0), cd1 = ycode_of(m, 1);
          const int jj0 = 2 * m, jj1 = 2 * m + 1;
          const bool in0 = i < ny && ja < a.ns_loc, in1 = i < ny && ja + 1 < a.ns_loc;
          const double e0 = sT[jj0 * ZT_TLD + s], e1 = sT[jj1 * ZT_TLD + s];
          const ZPair zp = z_probit_pair_tab(e0, e1, sSd[jj0], sSd[jj1], sIsd[jj0], sIsd[jj1], cd0, cd1, u.a, u.b,
                                             a.noise_zero, sLog, sZT);
          double z0 = zp.z0, z1 = zp.z1;
          if (NORMAL) {  // R/updateZ.R:40-41
            if (sFam[jj0] == 1 && cd0 >= 0 && in0) z0 = a.Yval[(size_t)i + (size_t)ny * ja];
            if (sFam[jj1] == 1 && cd1 >= 0 && in1) z1 = a.Yval[(size_t)i + (size_t)ny * (ja + 1)];
          }
          if (!(MODE & Z_NOSTORE)) {
            if (in0) a.Z[(size_t)i + (size_t)ny * ja] = z0;
            if (in1) a.Z[(size_t)i + (size_t)ny * (ja + 1)] = z1;
          }
          sT[jj0 * ZT_TLD + s] = in0 ? z0 : 0.0;
          sT[jj1 * ZT_TLD + s] = in1 ? z1 : 0.0;
          continue;
        }
#pragma unroll
        for (int b = 0; b < 2; ++b) {
          const int jj = 2 * m + b, j = ja + b;
          double z = 0.0;
          if (i < ny && j < a.ns_loc) {
            const size_t cell = (size_t)i + (size_t)ny * j;
            if (DRAW) {
              const int code = ycode_of(m, b);
              const double e = sT[jj * ZT_TLD + s];
              if (sFam[jj] == 1 && code >= 0)
                z = a.Yval[cell];  // normal: Z = Y   R/updateZ.R:40-41
              else if (POIS && sFam[jj] == 3 && code >= 0)
                z = z_poisson_draw(e, sSd[jj], a.Yval[cell], a.zprev_is_e ? e : a.Z[cell],
                                   uniforms(a.key, (uint32_t)((size_t)i + (size_t)ny * (uint32_t)(a.sp0 + j)), 0,
                                            S_ZPOIS, iter),
                                   a.noise_zero);
              else if (MODE & 2)
                z = z_probit_draw(e, sSd[jj], sIsd[jj], code, b ? u.b : u.a, a.noise_zero);
              else
                z = e + (b ? u.b : u.a);
              if (!(MODE & Z_NOSTORE)) a.Z[cell] = z;
            } else {
              z = a.Z[cell];
            }
          }
          sT[jj * ZT_TLD + s] = z;
        }
      }
    }
    // ---- ZTr partial of this species block for the 16 sites   (R/updateGamma2.R:46)
    if (MODE & 8) {
      for (int tt = 0; tt < a.nt; ++tt) {
        const double* tr = sTr + tt * ZT_J;
        double v = 0.0;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int m = 4 * c + lk;
          v = fma(sT[(2 * m) * ZT_TLD + lm], tr[2 * m], v);
          v = fma(sT[(2 * m + 1) * ZT_TLD + lm], tr[2 * m + 1], v);
        }
        v += __shfl_xor(v, 16);
        v += __shfl_xor(v, 32);
        const int i = i0 + lm;
        if (lk == 0 && i < ny) a.ZTr_part[(size_t)by * ny * a.nt + i + (size_t)ny * tt] = v;
      }
    }
    wave_lds_sync();
    // ---- XZ += XEta^T (Yx o Z) over the 16 sites (R/updateBetaLambda.R:66 of the next sweep);
    //      B operand = Z[site lk+4r][species 2lm+b] from the tile
    if ((MODE & 4) && NKB > 4) {  // 64 rows of A operands at a time
      double zz[4][2];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ir = i0 + 4 * r + lk;
        zz[r][0] = sT[(2 * lm) * ZT_TLD + lk + 4 * r];
        zz[r][1] = sT[(2 * lm + 1) * ZT_TLD + lk + 4 * r];
        if (HAS_NA && a.mask_na) {
          const uint64_t w2 = a.Ybits[(size_t)by * ny + ir];
          if (((w2 >> (4 * lm)) & 3u) == 0) zz[r][0] = 0.0;
          if (((w2 >> (4 * lm + 2)) & 3u) == 0) zz[r][1] = 0.0;
        }
      }
      const double* xq = a.XEta + (i0 + lk) + (size_t)ny * lm;
#pragma unroll
      for (int q0 = 0; q0 < NKB; q0 += 4) {
        double xt[4][4];
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int q = 0; q < 4; ++q) xt[r][q] = xq[4 * r + (size_t)ny * 16 * (q0 + q)];
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            acc[q0 + q][0] = mfma_f64(xt[r][q], zz[r][0], acc[q0 + q][0]);
            acc[q0 + q][1] = mfma_f64(xt[r][q], zz[r][1], acc[q0 + q][1]);
          }
      }
    } else if (MODE & 4) {
      // A operands (XEta^T rows) of all 4 x NKB MFMAs loaded first: one latency per tile
      double xt[4][NKB];
      const double* xq = a.XEta + (i0 + lk) + (size_t)ny * lm;
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int q = 0; q < NKB; ++q) xt[r][q] = xq[4 * r + (size_t)ny * 16 * q];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ir = i0 + 4 * r + lk;
        double z0 = sT[(2 * lm) * ZT_TLD + lk + 4 * r];
        double z1 = sT[(2 * lm + 1) * ZT_TLD + lk + 4 * r];
        if (HAS_NA && a.mask_na) {  // NA cells (code + 1 == 0) out of the contraction
          const uint64_t w2 = a.Ybits[(size_t)by * ny + ir];  // padded buffer: ir < ny + 64
          if (((w2 >> (4 * lm)) & 3u) == 0) z0 = 0.0;
          if (((w2 >> (4 * lm + 2)) & 3u) == 0) z1 = 0.0;
        }
#pragma unroll
        for (int q = 0; q < NKB; ++q) {  // rows >= K are discarded, sites >= ny have Z = 0
          acc[q][0] = mfma_f64(xt[r][q], z0, acc[q][0]);
          acc[q][1] = mfma_f64(xt[r][q], z1, acc[q][1]);
        }
      }
    }
    wave_lds_sync();
  }
  // combine the 4 waves' XZ and write this chunk's partial, 64 rows (4 blocks) at a time
  constexpr int QC = NKB > 4 ? 4 : NKB, KC = 16 * QC;
  double* sR = smem;  // [w-1][KC][32] (reuses the whole workgroup's LDS)
#pragma unroll
  for (int q0 = 0; q0 < NKB; q0 += QC) {
    __syncthreads();
    if (w > 0) {
#pragma unroll
      for (int q = 0; q < QC; ++q)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
          for (int rr = 0; rr < 4; ++rr)
            sR[((w - 1) * KC + 16 * q + lk + 4 * rr) * ZT_J + 2 * lm + b] = acc[q0 + q][b][rr];
    }
    __syncthreads();
    if (w == 0) {
      double* dst = a.XZ_part + (size_t)chunk * K * a.ns_loc;
#pragma unroll
      for (int q = 0; q < QC; ++q)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
          for (int rr = 0; rr < 4; ++rr) {
            const int kl = 16 * q + lk + 4 * rr, k = 16 * q0 + kl, jj = 2 * lm + b, j = j0 + jj;
            const double v = acc[q0 + q][b][rr] + sR[(0 * KC + kl) * ZT_J + jj] + sR[(1 * KC + kl) * ZT_J + jj] +
                             sR[(2 * KC + kl) * ZT_J + jj];
            if (k < K && j < a.ns_loc) dst[k + (size_t)K * j] = v;
          }
    }
  }
  if (w == 0 && a.kt && t == 0) kt_record(a.kt, iter, kt0);
}

// launch geometry shared by the launcher and the microbenchmark
// 16-row blocks of the instantiation serving K: 1 .. 4, or 8 for 64 < K <= 128
inline int z_nkb(int K) {
  const int n = (K + 15) / 16;
  return n > 4 ? 8 : n;
}
// XEta columns the z kernel reads (rows past K meet zero BL rows / are discarded)
inline int z_xeta_cols(int Kmax) { return 16 * z_nkb(Kmax); }

inline size_t z_smem_bytes(int K, int nt) {
  const size_t K16 = 16 * (size_t)z_nkb(K);
  const size_t body = K16 * ZT_J + (size_t)ZT_J * nt + 2 * ZT_J + ZT_J / 2 + ZLOG_W * (size_t)ZLOG_N + ZT_DOUBLES +
                      4 * (size_t)ZT_J * ZT_TLD;  // doubles
  const size_t red = 3 * (K16 > 64 ? 64 : K16) * ZT_J;                                                   // wave combine
  return (body > red ? body : red) * sizeof(double);
}

}  // namespace hmsc
