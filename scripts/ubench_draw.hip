// Microbenchmark: cost of the pieces of the probit truncated-normal draw (updateZ) on
// gfx950 -- Philox, erfc, the normal quantile -- as a streaming kernel over ny*ns cells
// that writes one double per cell.  Prints us per 1e7 cells for each variant.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include "../hmsc_amd/csrc/rng.h"
using namespace hmsc;

__device__ __forceinline__ double alpha_of(uint32_t c) {
  // a spread of standardised bounds like a fitted probit chain: mostly |alpha| < 3, some tails
  const uint32_t h = c * 2654435761u;
  const double v = (double)(h >> 8) * (1.0 / 16777216.0);
  return 8.0 * v - 5.0;
}

__device__ __noinline__ double tn_noinline(double a, double u) { return trunc_normal_lower(a, u); }

template <int V>
__global__ __launch_bounds__(256) void k(double* out, uint32_t n, Key key) {
  const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c < n) {  // one cell per thread: no loop for the compiler to hoist table loads out of
    double r;
    if (V == 0) {
      r = alpha_of(c);
    } else if (V == 1) {
      r = uniforms(key, c, 0, S_Z, 7).a;
        } else if (V == 3) {
      r = qnorm_fast(uniforms(key, c, 0, S_Z, 7).a);
    } else if (V == 4) {
      const double u = uniforms(key, c, 0, S_Z, 7).a;
      r = trunc_normal_lower(alpha_of(c), u);
    } else if (V == 9) {
      const double u = uniforms(key, c, 0, S_Z, 7).a;
      r = tn_noinline(alpha_of(c), u);
    } else if (V == 10) {
      r = erfc_fast(alpha_of(c) * 0.7071067811865476);
    } else if (V == 11) {
      r = log_fast(alpha_of(c) + 6.0);
    } else if (V == 5) {
      r = log(alpha_of(c) + 6.0);
    } else if (V == 6) {
      r = exp(alpha_of(c));
    } else if (V == 7) {
      r = 1.0 / (alpha_of(c) + 6.0);
    } else if (V == 8) {
      r = sqrt(alpha_of(c) + 6.0);
    }
    out[c] = r;
  }
}

// paired: one Philox call feeds two cells
__global__ __launch_bounds__(256) void k_pair(double* out, uint32_t n, Key key) {
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t c = blockIdx.x * blockDim.x + threadIdx.x; 2 * c < n; c += stride) {
    const Uniform2 u = uniforms(key, c, 0, S_Z, 7);
    out[2 * c] = trunc_normal_lower(alpha_of(2 * c), u.a);
    out[2 * c + 1] = trunc_normal_lower(alpha_of(2 * c + 1), u.b);
  }
}

template <typename F>
float timeit(F f, int reps) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  f();
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(a);
  for (int i = 0; i < reps; ++i) f();
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  return 1e3f * ms / reps;
}

int main() {
  const uint32_t n = 10000000;
  double* d;
  (void)hipMalloc(&d, sizeof(double) * n);
  Key key{12345u, 678u};
  const char* names[] = {"store only", "philox", "(unused)", "philox+qnorm_fast", "philox+truncnorm", "log", "exp",
                         "rcp(div)", "sqrt", "philox+tn noinline", "erfc_fast", "log_fast"};
  for (int blocks : {(int)(n / 256)}) {
    printf("grid %d x 256 (one cell per thread)\n", blocks);
#define RUN(V) printf("  %-20s %8.1f us\n", names[V], timeit([&] { k<V><<<blocks, 256>>>(d, n, key); }, 20));
    RUN(0) RUN(1) RUN(3) RUN(4) RUN(9) RUN(10) RUN(5) RUN(11) RUN(6) RUN(7) RUN(8)
    printf("  %-20s %8.1f us\n", "paired philox+tn", timeit([&] { k_pair<<<blocks, 256>>>(d, n, key); }, 20));
  }
  return 0;
}
