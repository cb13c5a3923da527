// Counter-based randomness for the Hmsc Gibbs sweep on gfx950.
//
// Every random variate in a sweep is a pure function of
//     key     = (seed_lo, seed_hi)              -- one 64-bit seed per chain
//     counter = (idx, sub, stream, iter)        -- element, sub-draw, updater stream, sweep
// so a draw does not depend on launch geometry, on how species are sharded over
// GPUs, or on the order kernels run in.  This replaces R's global Mersenne-Twister
// stream (set.seed(initSeed[chain]), R/sampleMcmc.R:158) and the samplers of the
// unvendored dependencies: stats::rnorm/rgamma, truncnorm::rtruncnorm
// (R/updateZ.R:217 via :59 of the original file), MCMCpack::rwish (R/updateGammaV.R:21).
//
// The CPU oracle (oracle/rng.py) implements the identical contract in numpy, so
// a device updater and the oracle updater fed the same state and key produce the
// same draws up to floating-point rounding.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace hmsc {

// updater stream ids (counter word 2); per-random-level streams add LEVEL_STRIDE*r
enum Stream : uint32_t {
  S_GAMMA2 = 1,
  S_BETALAMBDA = 3,
  S_WISHART_DIAG = 4,
  S_WISHART_OFF = 5,
  S_GAMMAV = 6,
  S_RHO = 7,
  S_GE_BETA = 8,   // updateGammaEta (+ LEVEL_STRIDE * r)
  S_GE_GAMMA = 9,
  S_GE_ETA = 10,
  S_INVSIGMA = 11,
  S_Z = 12,
  S_ZPOIS = 13,
  S_PSI = 20,
  S_DELTA = 21,
  S_ETA = 22,
  S_ALPHA = 23,
  S_NF = 24,
  S_NF_ETA = 25,
  S_NF_PSI = 26,
  S_NF_DELTA = 27,
  // chain initialisation (computeInitialParameters), iter = 0
  S_INIT_GAMMA = 40,
  S_INIT_V_DIAG = 41,
  S_INIT_V_OFF = 42,
  S_INIT_BETA = 43,
  S_INIT_SIGMA = 44,
  S_INIT_DELTA = 50,
  S_INIT_PSI = 51,
  S_INIT_LAMBDA = 52,
  S_INIT_ETA = 53,
};
constexpr uint32_t LEVEL_STRIDE = 256;
constexpr uint32_t GAMMA_BOOST_SUB = 0xFFFF0000u;  // sub-counter of the shape<1 boost uniform
constexpr int GAMMA_MAX_TRIALS = 64;

struct Key {
  uint32_t k0, k1;
};

struct U4 {
  uint32_t x, y, z, w;
};

__host__ __device__ __forceinline__ U4 philox4x32_10(U4 c, Key key) {
  uint32_t k0 = key.k0, k1 = key.k1;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c.z;
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    c = U4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

// 53-bit uniform on the open interval (0,1) from two 32-bit words
__host__ __device__ __forceinline__ double u53(uint32_t hi, uint32_t lo) {
  return ((double)(hi >> 5) * 67108864.0 + (double)(lo >> 6) + 0.5) * (1.0 / 9007199254740992.0);
}

// open-interval uniform from one 32-bit word, (w + 1/2) 2^-32 (exact in double): updateZ's
// uniforms, one Philox block feeding four cells, at the resolution of R's unif_rand
__host__ __device__ __forceinline__ double u32o(uint32_t w) { return ((double)w + 0.5) * (1.0 / 4294967296.0); }

struct Uniform2 {
  double a, b;
};

__host__ __device__ __forceinline__ Uniform2 uniforms(Key key, uint32_t idx, uint32_t sub, uint32_t stream,
                                             uint32_t iter) {
  const U4 r = philox4x32_10(U4{idx, sub, stream, iter}, key);
  return Uniform2{u53(r.x, r.y), u53(r.z, r.w)};
}

// The same Philox4x32-10 for a wave-uniform key (a kernel argument: the key words stay in
// SGPRs and the round keys are scalar adds): each round's two three-way XORs are single
// gfx950 v_bitop3_b32 instructions (truth table 0x96 = a ^ b ^ c) taking the round key as
// their SGPR operand (the compiler emits two v_xor_b32 each).  Same values as philox4x32_10.
__device__ __forceinline__ U4 philox4x32_10_wave_key(U4 c, Key key) {
  uint32_t k0 = key.k0, k1 = key.k1;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c.z;
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    uint32_t x, z;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(x) : "v"(hi1), "v"(c.y), "s"(k0));
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(z) : "v"(hi0), "v"(c.w), "s"(k1));
    c = U4{x, lo1, z, lo0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

__device__ __forceinline__ Uniform2 uniforms_wave_key(Key key, uint32_t idx, uint32_t sub, uint32_t stream,
                                                      uint32_t iter) {
  const U4 r = philox4x32_10_wave_key(U4{idx, sub, stream, iter}, key);
  return Uniform2{u53(r.x, r.y), u53(r.z, r.w)};
}

// Phi^-1(p), Wichura (1988) AS241 PPND16 (the algorithm behind R's qnorm), |rel err| ~1e-16.
__host__ __device__ __forceinline__ double qnorm_as241(double p) {
  const double q = p - 0.5;
  if (fabs(q) <= 0.425) {
    const double r = 0.180625 - q * q;
    const double num =
        (((((((2.5090809287301226727e+3 * r + 3.3430575583588128105e+4) * r + 6.7265770927008700853e+4) * r +
             4.5921953931549871457e+4) * r + 1.3731693765509461125e+4) * r + 1.9715909503065514427e+3) * r +
          1.3314166789178437745e+2) * r + 3.3871328727963666080e0);
    const double den =
        (((((((5.2264952788528545610e+3 * r + 2.8729085735721942674e+4) * r + 3.9307895800092710610e+4) * r +
             2.1213794301586595867e+4) * r + 5.3941960214247511077e+3) * r + 6.8718700749205790830e+2) * r +
          4.2313330701600911252e+1) * r + 1.0);
    return q * num / den;
  }
  double r = q < 0.0 ? p : 1.0 - p;
  r = sqrt(-log(r));
  double val;
  if (r <= 5.0) {
    r -= 1.6;
    const double num =
        (((((((7.74545014278341407640e-4 * r + 2.27238449892691845833e-2) * r + 2.41780725177450611770e-1) * r +
             1.27045825245236838258e0) * r + 3.64784832476320460504e0) * r + 5.76949722146069140550e0) * r +
          4.63033784615654529590e0) * r + 1.42343711074968357734e0);
    const double den =
        (((((((1.05075007164441684324e-9 * r + 5.47593808499534494600e-4) * r + 1.51986665636164571966e-2) * r +
             1.48103976427480074590e-1) * r + 6.89767334985100004550e-1) * r + 1.67638483018380384940e0) * r +
          2.05319162663775882187e0) * r + 1.0);
    val = num / den;
  } else {
    r -= 5.0;
    const double num =
        (((((((2.01033439929228813265e-7 * r + 2.71155556874348757815e-5) * r + 1.24266094738807843860e-3) * r +
             2.65321895265761230930e-2) * r + 2.96560571828504891230e-1) * r + 1.78482653991729133580e0) * r +
          5.46378491116411436990e0) * r + 6.65790464350110377720e0);
    const double den =
        (((((((2.04426310338993978564e-15 * r + 1.42151175831644588870e-7) * r + 1.84631831751005468180e-5) * r +
             7.86869131145613259100e-4) * r + 1.48753612908506148525e-2) * r + 1.36929880922735805310e-1) * r +
          5.99832206555887937690e-1) * r + 1.0);
    val = num / den;
  }
  return q < 0.0 ? -val : val;
}

// ---------------------------------------------------------------------------
// Truncated-normal draw of updateZ (probit, R/updateZ.R:43-63; NA cells :92).
//
// The device evaluates the same inversion as the oracle (oracle/rng.py,
// trunc_normal_lower: x = -Phi^-1(u Phic(alpha)) with R's AS241 quantile and erfc)
// through cheaper, equally accurate approximations of the two special functions:
//   erfc_fast   t exp(-z^2 + g(t)), g a degree-24 polynomial (scripts/fit_erfc.py; 3.3e-15
//               rel. on [0,18] with exact -z^2, ~5e-14 from rounding -z^2 + g near z = 18)
//   qnorm_fast  Giles-form y F(w), w = -log(4p(1-p)) (degree-22 / 18 polynomials,
//               1.2e-15 rel., scripts/fit_qnorm.py); no division, and one branch for
//               p in (4.8e-4, 1 - 4.8e-4) so a wave rarely diverges; AS241's tail
//               branch below p < 2.8e-8
//   log_fast    2 atanh((m-1)/(m+1)) series; the libm f64 log is the single most
//               expensive operation of the draw on gfx950
// ---------------------------------------------------------------------------
// Polynomial tables of the draw (fit scripts above).  Device code reads them from the
// constant segment: scalar loads put each coefficient in an SGPR pair that v_fma_f64 takes
// directly, instead of two v_mov_b32 per coefficient for an inline 64-bit constant (which
// doubled the VALU cost of every Horner step).
#define HMSC_TABLE static constexpr
// Degrees chosen for ~1e-13 relative accuracy (erfc 1.3e-13, quantile 1.0e-13 against scipy's
// ndtri over p in [1e-170, 1 - 1e-16]; scripts/fit_erfc.py DEG = 20, scripts/fit_qnorm.py 18 14):
// four orders of magnitude inside the 1e-9 draw parity the tests hold, at 16 fewer Horner steps
// per probit cell than the 1e-15 fits of rounds 1-3.
constexpr int ERFC_NC = 21, QNA_NC = 19, QNB_NC = 15;
HMSC_TABLE double kErfcPoly[ERFC_NC] = {1.6376767839449274e-07, 2.3266618798645898e-07, -1.72119617257043e-06, -9.482593124897482e-07, 8.961696172849177e-06, -2.181669006322301e-06, -3.0426211782697305e-05, 3.344182221368426e-05, 7.14963433719764e-05, -0.00017509998617504471, -9.375992582024659e-05, 0.00067391609038368, -0.0001462428461891559, -0.0023458553006862107, 0.0017589331973563102, 0.008824942825902316, -0.009872689352028938, -0.04689561042741337, 0.04734330684178697, 0.6726432239803275, -0.6717940840566928};
HMSC_TABLE double kQnormA[QNA_NC] = {-1.0875518868761332e-16, 4.63142976573437e-16, 7.824871070301776e-15, -6.386039019553726e-14, -9.819509084205816e-14, 3.7835637374349886e-12, -1.846255754688949e-11, -7.692151430644685e-11, 1.4870983005321307e-09, -5.814956310949196e-09, -4.111283999042869e-08, 5.988869248815612e-07, -1.9310634920507984e-06, -1.9632849914852812e-05, 0.00026408204847481575, -0.0010475115710453554, -0.008532899176989971, 0.3396349587013827, 2.338620710026582};
HMSC_TABLE double kQnormB[QNB_NC] = {1.225719388224846e-06, -5.277698325167675e-06, 4.988842960857911e-06, 1.7210019190814766e-05, -6.734362203040504e-05, 9.677574208297108e-05, 3.410330419484804e-05, -0.0005021491321574642, 0.0013481368125180162, -0.002387576041668264, 0.00352343255417981, -0.005305010274193076, 0.007595620164819752, 1.421650865815266, 4.361272855165519};
HMSC_TABLE double kLogSeries[10] = {2.0 / 21.0, 2.0 / 19.0, 2.0 / 17.0, 2.0 / 15.0, 2.0 / 13.0,
                                    2.0 / 11.0, 2.0 / 9.0,  2.0 / 7.0,  2.0 / 5.0,  2.0 / 3.0};

// Horner step a*b + c with c wave-uniform: forced into the VOP3 form whose third operand is
// an SGPR pair (the compiler otherwise tends to copy c into VGPRs with two v_mov_b32 and use
// v_fmac_f64, doubling the issue cost of each step).
__host__ __device__ __forceinline__ double fma_sc(double a, double b, double c) {
#if defined(__HIP_DEVICE_COMPILE__)
  double r;
  asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(c));
  return r;
#else
  return fma(a, b, c);
#endif
}

// 1/d for d in [1, 1e3] (well conditioned): v_rcp_f64 + two Newton steps, ~1 ulp; the IEEE
// division sequence (div_scale / div_fmas / div_fixup) costs twice as much
__host__ __device__ __forceinline__ double rcp_pos(double d) {
#if defined(__HIP_DEVICE_COMPILE__)
  double r = __builtin_amdgcn_rcp(d);
  r = fma(r, fma(-d, r, 1.0), r);
  r = fma(r, fma(-d, r, 1.0), r);
  return r;
#else
  return 1.0 / d;
#endif
}

// The *_t forms take their coefficient tables as pointers (device kernels pass pointers the
// compiler cannot hoist, z_kernel.h opaque_table); the plain forms use the global tables.
__host__ __device__ __forceinline__ double log_fast_t(double x, const double* ls) {  // x positive, normal
  uint64_t b;
  __builtin_memcpy(&b, &x, 8);
  int e = (int)(b >> 52) - 1023;
  const uint64_t mb = (b & 0x000FFFFFFFFFFFFFull) | 0x3FF0000000000000ull;
  double m;
  __builtin_memcpy(&m, &mb, 8);
  if (m > 1.4142135623730951) {
    m *= 0.5;
    e += 1;
  }
  const double f = m - 1.0;
  const double s = f * rcp_pos(2.0 + f);
  const double z = s * s;
  // P(z) = sum_{k=1..10} 2 z^(k-1) / (2k+1); truncation < 3e-17 relative for |s| <= 0.1716
  double P = ls[0];
#pragma unroll
  for (int k = 1; k < 10; ++k) P = fma_sc(P, z, ls[k]);
  const double lm = fma(s * z, P, 2.0 * s);
  const double de = (double)e;
  return fma(de, 0.6931471803691238, fma(de, 1.9082149292705877e-10, lm));  // ln2 = hi + lo, hi*e exact
}

__host__ __device__ __forceinline__ double log_fast(double x) { return log_fast_t(x, kLogSeries); }

// exp(x) for x <= 700 without the libm range handling (the truncated-normal draw evaluates it
// on -a^2 + g(t) <= 0 only): x = n ln2 + r, |r| <= ln2 / 2, exp(r) by its degree-11 Taylor
// polynomial (truncation 6e-15 relative), 2^n by ldexp (underflows to 0 below -745).
constexpr int EXP_NC = 12;
HMSC_TABLE double kExpTaylor[EXP_NC] = {1.0 / 39916800.0, 1.0 / 3628800.0, 1.0 / 362880.0, 1.0 / 40320.0,
                                        1.0 / 5040.0,     1.0 / 720.0,     1.0 / 120.0,    1.0 / 24.0,
                                        1.0 / 6.0,        0.5,             1.0,            1.0};
__host__ __device__ __forceinline__ double exp_small(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
  const double n = __builtin_rint(x * 1.4426950408889634);
  double r = fma(-n, 6.93147180369123816490e-01, x);  // ln2 = hi + lo (fdlibm split: n hi exact)
  r = fma(-n, 1.90821492927058770002e-10, r);
  double p = kExpTaylor[0];
#pragma unroll
  for (int k = 1; k < EXP_NC; ++k) p = fma_sc(p, r, kExpTaylor[k]);
  return __builtin_ldexp(p, (int)n);
#else
  return exp(x);
#endif
}

__host__ __device__ __forceinline__ double erfc_fast_t(double z, const double* ep) {
  const double a = fmin(fabs(z), 40.0);
  const double t = 2.0 * rcp_pos(2.0 + a);
  const double x = 2.0 * t - 1.0;
  double g = ep[0];
#pragma unroll
  for (int k = 1; k < ERFC_NC; ++k) g = fma_sc(g, x, ep[k]);
  const double r = t * exp(fma(-a, a, g));
  return z < 0.0 ? 2.0 - r : r;
}

__host__ __device__ __forceinline__ double erfc_fast(double z) { return erfc_fast_t(z, kErfcPoly); }

// AS241's |q| > 0.425 branch (R's qnorm), with log_fast
__host__ __device__ __forceinline__ double qnorm_as241_tail_t(double p, const double* ls) {
  const double q = p - 0.5;
  double r = q < 0.0 ? p : 1.0 - p;
  r = sqrt(-log_fast_t(r, ls));
  double val;
  if (r <= 5.0) {
    r -= 1.6;
    const double num =
        (((((((7.74545014278341407640e-4 * r + 2.27238449892691845833e-2) * r + 2.41780725177450611770e-1) * r +
             1.27045825245236838258e0) * r + 3.64784832476320460504e0) * r + 5.76949722146069140550e0) * r +
          4.63033784615654529590e0) * r + 1.42343711074968357734e0);
    const double den =
        (((((((1.05075007164441684324e-9 * r + 5.47593808499534494600e-4) * r + 1.51986665636164571966e-2) * r +
             1.48103976427480074590e-1) * r + 6.89767334985100004550e-1) * r + 1.67638483018380384940e0) * r +
          2.05319162663775882187e0) * r + 1.0);
    val = num / den;
  } else {
    r -= 5.0;
    const double num =
        (((((((2.01033439929228813265e-7 * r + 2.71155556874348757815e-5) * r + 1.24266094738807843860e-3) * r +
             2.65321895265761230930e-2) * r + 2.96560571828504891230e-1) * r + 1.78482653991729133580e0) * r +
          5.46378491116411436990e0) * r + 6.65790464350110377720e0);
    const double den =
        (((((((2.04426310338993978564e-15 * r + 1.42151175831644588870e-7) * r + 1.84631831751005468180e-5) * r +
             7.86869131145613259100e-4) * r + 1.48753612908506148525e-2) * r + 1.36929880922735805310e-1) * r +
          5.99832206555887937690e-1) * r + 1.0);
    val = num / den;
  }
  return q < 0.0 ? -val : val;
}

__host__ __device__ __forceinline__ double qnorm_fast_t(double p, const double* qa, const double* qb,
                                                        const double* ls) {
  const double y = 2.0 * p - 1.0;
  const double w = -log_fast_t(4.0 * p * (1.0 - p), ls);
  if (w < 6.25) {
    const double t = w - 3.125;
    double f = qa[0];
#pragma unroll
    for (int k = 1; k < QNA_NC; ++k) f = fma_sc(f, t, qa[k]);
    return y * f;
  }
  if (w < 16.0) {
    const double t = sqrt(w) - 3.25;
    double f = qb[0];
#pragma unroll
    for (int k = 1; k < QNB_NC; ++k) f = fma_sc(f, t, qb[k]);
    return y * f;
  }
  return qnorm_as241_tail_t(p, ls);
}

__host__ __device__ __forceinline__ double qnorm_fast(double p) { return qnorm_fast_t(p, kQnormA, kQnormB, kLogSeries); }

// standard normal by inversion of the first uniform of the (idx, sub) block (R's default
// rnorm method, INVERSION; the oracle uses AS241 itself, the device qnorm_fast)
__host__ __device__ __forceinline__ double normal(Key key, uint32_t idx, uint32_t sub, uint32_t stream,
                                                  uint32_t iter) {
  return qnorm_fast(uniforms(key, idx, sub, stream, iter).a);
}

// Gamma(shape, rate=1): Marsaglia & Tsang (2000); trial t uses sub-blocks 2t (normal)
// and 2t+1 (acceptance uniform); shape<1 uses the boost x*U^(1/shape).
__host__ __device__ __forceinline__ double gamma_std(Key key, uint32_t idx, uint32_t stream, uint32_t iter,
                                                     double shape) {
  const double a = shape < 1.0 ? shape + 1.0 : shape;
  const double d = a - 1.0 / 3.0;
  const double c = 1.0 / sqrt(9.0 * d);
  double out = d;  // fallback after GAMMA_MAX_TRIALS (probability < 1e-60)
  for (int t = 0; t < GAMMA_MAX_TRIALS; ++t) {
    const double x = normal(key, idx, 2u * t, stream, iter);
    double v = 1.0 + c * x;
    if (v <= 0.0) continue;
    v = v * v * v;
    const double u = uniforms(key, idx, 2u * t + 1u, stream, iter).a;
    if (log_fast(u) < 0.5 * x * x + d - d * v + d * log_fast(v)) {
      out = d * v;
      break;
    }
  }
  if (shape < 1.0) {
    const double u = uniforms(key, idx, GAMMA_BOOST_SUB, stream, iter).a;
    out *= pow(u, 1.0 / shape);
  }
  return out;
}

// Mean and variance of the Polya-Gamma PG(b, c) (Polson, Scott & Windle 2013):
//   E = b tanh(c/2) / (2c),   Var = b (sinh c - c) sech^2(c/2) / (4 c^3)
// written as b (2 tanh(x/2) - x sech^2(x/2)) / (4 x^3) for x = |c| >= 1 (no overflow) and
// as the Taylor series (sinh x - x) / x^3 = sum_k x^2k / (2k+3)! below 1 (no cancellation).
// oracle/hmsc_oracle.py pg_moments is the same formula.
__host__ __device__ inline void pg_moments(double b, double c, double* mean, double* var) {
  const double x = fabs(c), x2 = x * x;
  const double th = tanh(0.5 * x);
  *mean = b * (x < 1e-4 ? 0.25 - x2 / 48.0 : th / (2.0 * x));
  const double ch = cosh(0.5 * x);
  const double sech2 = 1.0 / (ch * ch);
  if (x < 1.0) {
    double q = 1.0 + x2 / 272.0;
    q = 1.0 + x2 / 210.0 * q;
    q = 1.0 + x2 / 156.0 * q;
    q = 1.0 + x2 / 110.0 * q;
    q = 1.0 + x2 / 72.0 * q;
    q = 1.0 + x2 / 42.0 * q;
    q = 1.0 + x2 / 20.0 * q;
    *var = b * (q / 6.0) * sech2 / 4.0;
  } else {
    *var = b * (2.0 * th - x * sech2) / (4.0 * x2 * x);
  }
}

// Standard normal truncated to [alpha, +inf) by inversion of the upper tail:
//   x = Phic^-1(u Phic(alpha)) = -Phi^-1(u * 0.5 erfc(alpha / sqrt 2)),
// with the exponential tail expansion beyond alpha > 25 (u Phic(alpha) < 1e-138 there).
// alpha = -inf (NA cells, R/updateZ.R:92) gives p = u: an untruncated normal.
__host__ __device__ __forceinline__ double trunc_normal_lower_t(double alpha, double u, const double* ep,
                                                                const double* qa, const double* qb,
                                                                const double* ls) {
  if (alpha > 25.0) return alpha - log_fast_t(u, ls) / alpha;
  const double p = u * (0.5 * erfc_fast_t(alpha * 0.7071067811865476, ep));
  return -qnorm_fast_t(p, qa, qb, ls);
}

__host__ __device__ __forceinline__ double trunc_normal_lower(double alpha, double u) {
  return trunc_normal_lower_t(alpha, u, kErfcPoly, kQnormA, kQnormB, kLogSeries);
}

}  // namespace hmsc
