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
  return sqrt(-2.0 * log(u.a)) * cos(6.283185307179586 * u.b);
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

// Standard normal truncated to [alpha, +inf) by inversion of the upper tail,
//   x = sqrt(2) * erfcinv(u * erfc(alpha/sqrt(2))),
// with the exponential tail expansion beyond alpha > 25 where erfc underflows.
__device__ __forceinline__ double trunc_normal_lower(double alpha, double u) {
  if (alpha > 25.0) return alpha - log(u) / alpha;
  const double t = u * erfc(alpha * 0.7071067811865476);
  return 1.4142135623730951 * erfcinv(t);
}

}  // namespace hmsc
