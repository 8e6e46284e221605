// Phase timing + check of the in-LDS diagonal-block factorisation (dev tool).
// hipcc --offload-arch=gfx950 -O3 -w [-DDB_TIMING] [-DDB_LEAF_PERMUTE] tools/hip/db_bench.hip -o tools/hip/db_bench_bin
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>
#include "../../gp_emu_uqsa_amd/csrc/gpemu_kernels.hpp"
using namespace gpe;
#ifndef DB_TIMING
__device__ unsigned long long db_tsc[8];   // stays zero: untimed build
#endif

__device__ unsigned long long db_clk[2];   // shader cycles, wall ticks (100 MHz) of the factor

__global__ void __launch_bounds__(256) k_db(double* A, long long ld, double* X, double* lg, int* info) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const unsigned long long c0 = clock64(), w0 = wall_clock64();
  for (int e = threadIdx.x; e < 128 * 128; e += 256) {
    const int i = e & 127, k = e >> 7;
    if (i >= k) lds[db_off(i, k)] = A[i + k * ld];
  }
  __syncthreads();
  const int bad = db_factor_invert(lds, A, ld, X, ld, lg, [] {});
  if (bad && threadIdx.x == 0) *info = bad;
  if (threadIdx.x == 0) {
    atomicAdd(&db_clk[0], clock64() - c0);
    atomicAdd(&db_clk[1], wall_clock64() - w0);
  }
}

int main() {
  const int n = 128;
  std::vector<double> h(n * n);
  for (int j = 0; j < n; ++j)
    for (int i = 0; i < n; ++i)
#ifdef DB_NO_UPDATE   // no trailing update in the probe: a diagonally dominant tile keeps every pivot positive
      h[i + j * n] = 1e-3 * std::exp(-0.001 * (i - j) * (i - j)) + (i == j ? 1.0 : 0.0);
#else
      h[i + j * n] = std::exp(-0.001 * (i - j) * (i - j)) + (i == j ? 1.0 : 0.0);
#endif
  double *A, *A0, *X, *lg;
  int* info;
  hipMalloc(&A, n * n * 8); hipMalloc(&A0, n * n * 8); hipMalloc(&X, n * n * 8); hipMalloc(&lg, 8); hipMalloc(&info, 4);
  hipMemcpy(A0, h.data(), n * n * 8, hipMemcpyHostToDevice);
  hipMemset(info, 0, 4);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  const size_t lds = (DB_LDS_DOUBLES + DB_EXTRA_DOUBLES) * 8;
  float best = 1e9;
  const int reps = 20;
  unsigned long long zero[8] = {0};
  hipMemcpyToSymbol(HIP_SYMBOL(db_tsc), zero, sizeof(zero));
  for (int rep = 0; rep < reps; ++rep) {
    hipMemcpy(A, A0, n * n * 8, hipMemcpyDeviceToDevice);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_db, dim3(1), dim3(256), lds, 0, A, (long long)n, X, lg, info);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    if (ms < best) best = ms;
  }
  unsigned long long t[8];
  hipMemcpyFromSymbol(t, HIP_SYMBOL(db_tsc), sizeof(t));
  int inf; hipMemcpy(&inf, info, 4, hipMemcpyDeviceToHost);
  std::vector<double> L(n * n), Xh(n * n);
  hipMemcpy(L.data(), A, n * n * 8, hipMemcpyDeviceToHost);
  hipMemcpy(Xh.data(), X, n * n * 8, hipMemcpyDeviceToHost);
  double e1m = 0, e2m = 0;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j <= i; ++j) {
      double s = 0, s2 = 0;
      for (int k = 0; k <= j; ++k) s += L[i + k * n] * L[j + k * n];
      e1m = fmax(e1m, fabs(s - h[i + j * n]));
      for (int k = j; k <= i; ++k) s2 += Xh[i + k * n] * L[k + j * n];
      e2m = fmax(e2m, fabs(s2 - (i == j ? 1.0 : 0.0)));
    }
  for (int i = 0; i < n; ++i)
    for (int j = i + 1; j < n; ++j) e2m = fmax(e2m, fabs(Xh[i + j * n]));
  printf("best %.1f us info=%d |LL^T-A| %.2e |XL-I| %.2e\n", best * 1e3, inf, e1m, e2m);
  const char* nm[8] = {"total", "leaf+update", "panel", "X assembly", "L/X out", "leaf (w0)", "diag syrk (w0)",
                       "update (w1)"};
  for (int i = 0; i < 8; ++i) printf("  %-14s %.1f us (mean)\n", nm[i], t[i] * 0.01 / reps);
  unsigned long long ck[2];
  hipMemcpyFromSymbol(ck, HIP_SYMBOL(db_clk), sizeof(ck));
  printf("  kernel body %.1f us (mean), shader clock %.2f GHz\n", ck[1] * 0.01 / reps, (double)ck[0] / (ck[1] * 10.0));
  return 0;
}
