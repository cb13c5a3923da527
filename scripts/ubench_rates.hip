// Microbenchmark: issue rate of the instructions the z draw is made of, on gfx950, per wave64
// instruction (8 independent chains per lane, 256-thread workgroups, 4 per CU):
//   fma_f64  v_fma_f64          mad64    v_mad_u64_u32 (Philox's 32x32 -> 64 multiply)
//   mulhi    v_mul_hi_u32       pkfma    v_pk_fma_f32
//   bitop3   v_bitop3_b32       fma_f32  v_fma_f32
// Prints ns per wave-instruction per SIMD slot (clock cycles at the measured rate).
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int ITERS = 4096;

template <int OP>
__global__ __launch_bounds__(256, 4) void rate_kernel(unsigned* out, unsigned seed) {
  const unsigned t = threadIdx.x + blockIdx.x * 256 + seed;
  unsigned u[8];
  double d[8];
  float f[8];
  typedef float f2 __attribute__((ext_vector_type(2)));
  f2 p[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    u[k] = t * (2 * k + 1);
    d[k] = (double)u[k] * 1e-9;
    f[k] = (float)d[k];
    p[k] = f2{f[k], f[k] + 1.0f};
  }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (OP == 0) d[k] = __builtin_fma(d[k], 0.9999999, 1e-7);
      if (OP == 1) {
        const unsigned long long m = (unsigned long long)u[k] * 0xD2511F53u + (unsigned long long)it;
        u[k] = (unsigned)(m >> 32) ^ (unsigned)m;
      }
      if (OP == 2) u[k] = __umulhi(u[k], 0xCD9E8D57u) + (unsigned)k;
      if (OP == 3) p[k] = __builtin_elementwise_fma(p[k], f2{0.9999f, 0.9999f}, f2{1e-4f, 1e-4f});
      if (OP == 4) u[k] = (u[k] ^ (unsigned)it) ^ (u[k] >> 3);
      if (OP == 5) f[k] = __builtin_fmaf(f[k], 0.9999f, 1e-4f);
    }
  }
  unsigned r = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) r ^= u[k] ^ (unsigned)(d[k] * 1e3) ^ (unsigned)(f[k] * 1e3) ^ (unsigned)(p[k].x + p[k].y);
  out[t - seed] = r;
}

template <int OP>
void run(const char* name, unsigned* out, int grid, int ncu) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  rate_kernel<OP><<<grid, 256>>>(out, 1);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(a);
  rate_kernel<OP><<<grid, 256>>>(out, 2);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, a, b);
  // wave-instructions per SIMD: grid * 4 waves * ITERS * 8 / (4 SIMDs * ncu)
  const double per_simd = (double)grid * 4 * ITERS * 8 / (4.0 * ncu);
  printf("%-8s %8.3f ms  %6.2f ns per wave-instruction per SIMD\n", name, ms, 1e6 * ms / per_simd);
}

int main() {
  int ncu = 0;
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  const int grid = ncu * 4 * 4;
  unsigned* out;
  (void)hipMalloc(&out, (size_t)grid * 256 * sizeof(unsigned));
  run<0>("fma_f64", out, grid, ncu);
  run<1>("mad64", out, grid, ncu);
  run<2>("mulhi", out, grid, ncu);
  run<3>("pkfma", out, grid, ncu);
  run<4>("xor2", out, grid, ncu);
  run<5>("fma_f32", out, grid, ncu);
  return 0;
}
