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
  S_INVSIGMA = 11,
  S_Z = 12,
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

struct Uniform2 {
  double a, b;
};

__host__ __device__ __forceinline__ Uniform2 uniforms(Key key, uint32_t idx, uint32_t sub, uint32_t stream,
                                             uint32_t iter) {
  const U4 r = philox4x32_10(U4{idx, sub, stream, iter}, key);
  return Uniform2{u53(r.x, r.y), u53(r.z, r.w)};
}

// standard normal: Box-Muller cosine branch of the (idx, sub) block
__host__ __device__ __forceinline__ double normal(Key key, uint32_t idx, uint32_t sub, uint32_t stream,
                                         uint32_t iter) {
  const Uniform2 u = uniforms(key, idx, sub, stream, iter);
#if defined(__HIP_DEVICE_COMPILE__)
  // cospi: exact argument reduction, no Payne-Hanek table (keeps kernels spill-free)
  return sqrt(-2.0 * log(u.a)) * cospi(2.0 * u.b);
#else
  return sqrt(-2.0 * log(u.a)) * cos(6.283185307179586 * u.b);
#endif
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
    if (log(u) < 0.5 * x * x + d - d * v + d * log(v)) {
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

// Standard normal truncated to [alpha, +inf) by inversion of the upper tail:
//   x = Phic^-1(u * Phic(alpha)) = -qnorm(u * 0.5 erfc(alpha / sqrt 2)),
// with the exponential tail expansion beyond alpha > 25 where erfc underflows.
// Branch-free erfc for the truncated-normal transform: for z >= 0,
// erfc(z) = t exp(-z^2 + g(t)), t = 2 / (2 + z), with g a degree-24 Chebyshev series in 2t - 1
// (coefficients fitted by scripts/fit_erfc.py; max relative error 3.1e-14 on [0, 18], from
// rounding of -z^2 at large z), and erfc(-z) = 2 - erfc(z).  One division, one exp and a
// Clenshaw recurrence, the same instruction stream in every lane (the libm erfc branches on
// five argument ranges, which diverges across a wave of cells).
__device__ __forceinline__ double erfc_cheb(double z) {
  constexpr double c[25] = {-0.6513268598908547, 0.6419697923564907, 0.019476473204185794, -0.009561514786808322,
                            -0.0009465953444817606, 0.0003668394978524299, 4.252332480676113e-05,
                            -2.0278578112090017e-05, -1.624290004616037e-06, 1.3036558354648522e-06,
                            1.5626441965479678e-08, -8.523809553318847e-08, 6.5290545049341035e-09,
                            5.059343126909536e-09, -9.913638910734626e-10, -2.2736555453727975e-10,
                            9.646798632720434e-11, 2.393915069408435e-12, -6.886047244122345e-12,
                            8.947117551256468e-13, 3.1297560583840907e-13, -1.1280057646648457e-13,
                            8.695131613182434e-16, 6.889526006643458e-15, -1.856021631896973e-15};
  const double a = fabs(z);
  const double t = 2.0 / (2.0 + a);
  const double x = 2.0 * t - 1.0, x2 = 2.0 * x;
  double b1 = 0.0, b2 = 0.0;
#pragma unroll
  for (int k = 24; k >= 1; --k) {
    const double tmp = b1;
    b1 = fma(x2, b1, -b2) + c[k];
    b2 = tmp;
  }
  const double g = fma(x, b1, -b2) + c[0];
  const double r = t * exp(fma(-a, a, g));
  return z < 0.0 ? 2.0 - r : r;
}

__device__ __forceinline__ double trunc_normal_lower(double alpha, double u) {
  if (alpha > 25.0) return alpha - log(u) / alpha;
  const double p = u * (0.5 * erfc_cheb(alpha * 0.7071067811865476));
  return -qnorm_as241(p);
}

}  // namespace hmsc
