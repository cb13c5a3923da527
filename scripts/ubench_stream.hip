// Read-bandwidth microbenchmark of Z (ny x ns fp64, column-major) access patterns for the
// fused Eta pass: A = the eta_fused_kernel pattern (16 sites x 4 species per wave load, 128-B
// runs), B = 64 sites of one species per wave load (512-B runs), C = 128 sites of one species
// per wave load with 16-B lanes (1-KB runs).  Each wave sums what it reads; time by events.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CK(x) (void)(x)

// A: workgroup = 16 sites, 4 waves split the species (j = 16 s + 4 w + lk), 16 loads in flight
__global__ __launch_bounds__(256) void kA(const double* Z, int ny, int ns, double* out) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, lm = lane & 15, lk = lane >> 4;
  const int i0 = blockIdx.x * 16;
  const double* zc = Z + min(i0 + lm, ny - 1);
  double acc = 0.0;
  const int nsteps = (ns + 15) >> 4;
  for (int s = 0; s < nsteps; s += 16) {
    double zv[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int j = 16 * (s + u) + 4 * w + lk;
      zv[u] = (s + u < nsteps && j < ns) ? zc[(size_t)ny * j] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) acc += zv[u];
  }
  out[blockIdx.x * 256 + t] = acc;
}

// B: workgroup = 64 sites, wave w takes species w, w + 4, ...; lane = site; 16 loads in flight
__global__ __launch_bounds__(256) void kB(const double* Z, int ny, int ns, double* out) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int i = min(blockIdx.x * 64 + lane, ny - 1);
  double acc = 0.0;
  for (int j0 = w; j0 < ns; j0 += 64) {
    double zv[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int j = j0 + 4 * u;
      zv[u] = j < ns ? Z[i + (size_t)ny * j] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) acc += zv[u];
  }
  out[blockIdx.x * 256 + t] = acc;
}

// C: workgroup = 128 sites, 16-B lanes (2 sites), wave w takes species w, w + 8, ... (8 waves)
__global__ __launch_bounds__(512) void kC(const double* Z, int ny, int ns, double* out) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int i = min(blockIdx.x * 128 + 2 * lane, ny - 2);
  double acc = 0.0;
  for (int j0 = w; j0 < ns; j0 += 128) {
    double2 zv[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int j = j0 + 8 * u;
      zv[u] = j < ns ? *(const double2*)(Z + i + (size_t)ny * j) : double2{0.0, 0.0};
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) acc += zv[u].x + zv[u].y;
  }
  out[blockIdx.x * 512 + t] = acc;
}

// D: A's layout but 8 waves per workgroup (species split 8 ways), 8 loads in flight
__global__ __launch_bounds__(512) void kD(const double* Z, int ny, int ns, double* out) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, lm = lane & 15, lk = lane >> 4;
  const int i0 = blockIdx.x * 16;
  const double* zc = Z + min(i0 + lm, ny - 1);
  double acc = 0.0;
  for (int j0 = 4 * w + lk; j0 < ns; j0 += 32 * 16) {
    double zv[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int j = j0 + 32 * u;
      zv[u] = j < ns ? zc[(size_t)ny * j] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) acc += zv[u];
  }
  out[blockIdx.x * 512 + t] = acc;
}

int main() {
  const int ny = 10000, ns = 1000;
  double *Z, *out;
  CK(hipMalloc(&Z, (size_t)ny * ns * 8));
  CK(hipMalloc(&out, (size_t)ny * 512 * 8));
  CK(hipMemset(Z, 0, (size_t)ny * ns * 8));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const double mb = (double)ny * ns * 8 / 1e6;
  for (int k = 0; k < 4; ++k) {
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipEventRecord(a));
      const int R = 50;
      for (int r = 0; r < R; ++r) {
        if (k == 0) kA<<<(ny + 15) / 16, 256>>>(Z, ny, ns, out);
        if (k == 1) kB<<<(ny + 63) / 64, 256>>>(Z, ny, ns, out);
        if (k == 2) kC<<<(ny + 127) / 128, 512>>>(Z, ny, ns, out);
        if (k == 3) kD<<<(ny + 15) / 16, 512>>>(Z, ny, ns, out);
      }
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms = 0.f;
      CK(hipEventElapsedTime(&ms, a, b));
      const double us = 1e3 * ms / R;
      printf("pattern %c: %.1f us per pass, %.0f GB/s\n", "ABCD"[k], us, mb / us * 1e3);
    }
  }
  return 0;
}
