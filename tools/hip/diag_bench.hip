// Ablation timing of the diagonal-block kernel (dev tool, not part of libgpemu).
// Build variants with -DDG_ABLATE=0 (full), 1 (leaves only: no node products),
// 2 (node products only: leaves skipped), 3 (load/store only).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include <vector>
#ifndef DG_ABLATE
#define DG_ABLATE 0
#endif
#include "../../gp_emu_uqsa_amd/csrc/gpemu_kernels.hpp"
using namespace gpe;
int main() {
  const int n = 128, ld = 128;
  std::vector<double> h(n * n);
  for (int j = 0; j < n; ++j)
    for (int i = 0; i < n; ++i) h[i + j * n] = std::exp(-0.001 * (i - j) * (i - j)) + (i == j ? 1.0 : 0.0);
  double *A, *B, *lg, *A0;
  int* info;
  hipMalloc(&A, n * n * 8); hipMalloc(&A0, n * n * 8); hipMalloc(&B, n * n * 8); hipMalloc(&lg, 8); hipMalloc(&info, 4);
  hipMemcpy(A0, h.data(), n * n * 8, hipMemcpyHostToDevice);
  hipMemset(info, 0, 4);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  float best = 1e9;
  for (int rep = 0; rep < 20; ++rep) {
    hipMemcpy(A, A0, n * n * 8, hipMemcpyDeviceToDevice);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_potrf_diag, dim3(1), dim3(DIAG_THREADS), 0, 0, A, (long long)ld, 0, B, (long long)ld, lg, info);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    if (ms < best) best = ms;
  }
  int inf; hipMemcpy(&inf, info, 4, hipMemcpyDeviceToHost);
  printf("ablate=%d  best %.1f us  info=%d\n", DG_ABLATE, best * 1e3, inf);
  return 0;
}
