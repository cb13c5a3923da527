// Microbenchmark: phases of the blocked Cholesky's 64 x 64 diagonal-block factorization
// (dense.hip chol_diag_kernel / diag_body) on one workgroup, s_memtime clock stamps.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -DHMSC_STAMPS -DHMSC_DENSE_STAMPS \
//         -I hmsc_amd/csrc scripts/ubench_diag.hip -o scripts/ubench_diag
#include "../hmsc_amd/csrc/dense.hip"

#include <cstdio>
#include <vector>

namespace hmsc {
__device__ unsigned long long g_stamps[1024];
}

int main() {
  using namespace hmsc;
  const int n = 64, lda = 64;
  std::vector<double> A(n * n);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) A[i + n * j] = (i == j ? n + 1.0 : 0.0) + 1.0 / (1.0 + i + j);
  double *dA, *dL;
  int* info;
  (void)hipMalloc(&dA, sizeof(double) * n * n);
  (void)hipMalloc(&dL, sizeof(double) * 64 * 64);
  (void)hipMalloc(&info, sizeof(int));
  const char* names[] = {"load+stage", "pivot 0", "kb0 panel", "kb0 update | pivot 1 | inverse row 0",
                         "kb1 panel", "kb1 update | pivot 2 | inverse row 1", "kb2 panel",
                         "kb2 update | pivot 3 | inverse row 2", "-", "inverse row 3", "store"};
  for (int rep = 0; rep < 5; ++rep) {
    (void)hipMemcpy(dA, A.data(), sizeof(double) * n * n, hipMemcpyHostToDevice);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    chol_diag_kernel<<<1, 256>>>(dA, lda, n, 0, dL, info, nullptr);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    unsigned long long st[1024];
    (void)hipMemcpyFromSymbol(st, HIP_SYMBOL(g_stamps), sizeof(st));
    if (rep == 4) {
      std::printf("chol_diag_kernel: %.2f us (events); phases in shader clocks:\n", 1e3 * ms);
      for (int p = 0; p < 11; ++p) std::printf("  %-18s %8llu\n", names[p], st[101 + p] - st[100 + p]);
      std::printf("  total              %8llu\n", st[111] - st[100]);
    }
  }
  return 0;
}
