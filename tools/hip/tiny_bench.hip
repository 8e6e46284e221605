// Phase clocks of the n <= 128 kernel (gpemu_tiny.hpp) on synthetic inputs (dev tool).
// hipcc --offload-arch=gfx950 -O3 -w -DTINY_TIMING tools/hip/tiny_bench.hip -o tools/hip/tiny_bench_bin
// Prints the average wall-clock (100 MHz) per phase over 200 launches and the hipEvent
// time per launch, with and without the gradient.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>
#include "../../gp_emu_uqsa_amd/csrc/gpemu_kernels.hpp"
#include "../../gp_emu_uqsa_amd/csrc/gpemu_tiny.hpp"
using namespace gpe;
#ifndef DB_TIMING
__device__ unsigned long long db_tsc[8];
#endif

int main() {
  const int n = 128, d = 10, P = 11, reps = 200;
  std::vector<double> X(n * d), F(TILE * P, 0.0), T2(P * P, 0.0);
  for (int i = 0; i < n; ++i)
    for (int k = 0; k < d; ++k) X[i * d + k] = std::fmod(0.37 * i + 0.11 * k * k + 0.05 * i * k, 1.0);
  for (int i = 0; i < n; ++i) {
    F[i] = std::sin(0.1 * i);
    for (int p = 1; p < P; ++p) F[i + p * TILE] = X[i * d + p - 1];
  }
  for (int p = 0; p < P; ++p) T2[p + p * P] = 1e-3;
  double *dX, *dF, *dT2, *xw, *L, *Xo, *Z, *small, *sums;   // (dT2, sums unused)
  int* flag;   // abort flag + the helpers' sync (4 ints, zeroed per launch)
  double *Wg, *part, *Xp;
  hipMalloc(&dX, X.size() * 8); hipMalloc(&dF, F.size() * 8); hipMalloc(&dT2, T2.size() * 8);
  hipMalloc(&xw, TILE * d * 8); hipMalloc(&L, TILE * TILE * 8); hipMalloc(&Xo, TILE * TILE * 8);
  hipMalloc(&Z, TILE * 32 * 8); hipMalloc(&small, 4096 * 8); hipMalloc(&sums, 64 * 8); hipMalloc(&flag, 32);
  hipMalloc(&Xp, 36 * DB_BS * 8);
  hipMalloc(&Wg, TILE * 32 * 8); hipMalloc(&part, TINY_NH * 64 * 8);
  hipMemcpy(dX, X.data(), X.size() * 8, hipMemcpyHostToDevice);
  hipMemcpy(dF, F.data(), F.size() * 8, hipMemcpyHostToDevice);
  hipMemcpy(dT2, T2.data(), T2.size() * 8, hipMemcpyHostToDevice);
  hipMemset(flag, 0, 4);
  TinyArgs a{};
  a.X = dX; a.F = dF; a.r = nullptr; a.rdiag = nullptr; a.xw = xw; a.L = L; a.Xo = Xo; a.Z = Z; a.small = small;
  a.K = L; a.Xp = Xp; a.Wg = Wg; a.sync = flag + 1;
  a.abort_flag = flag; a.n = n; a.d = d; a.P = P; a.want_grad = 1; a.mucm = 0;
  a.s2 = 1.0; a.coff = 1.0; a.cdiag = 1.0 + 1e-2; a.rscale = 0.0;
  for (int k = 0; k < 32; ++k) a.invd[k] = k < d ? 1.0 / 0.6 : 0.0;
  const size_t lds = (G_LDS_LAUNCH_DOUBLES + 2 * TILE * TINY_ZP) * sizeof(double);
  hipFuncSetAttribute((const void*)k_tiny<12>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int want = 1; want >= 0; --want) {
    a.want_grad = want;
    double ph[12] = {}, clk_ticks = 0.0, wall_ticks = 0.0;
    float tf = 0.f;
    for (int r = 0; r < reps + 5; ++r) {
      float ms;
      hipMemset(flag, 0, 32);
      a.ek = a.eg = 1;
      hipEventRecord(e0);
      hipLaunchKernelGGL(k_tiny<12>, dim3(1 + TINY_NH), dim3(256), lds, 0, a);
      hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
      if (r >= 5) tf += ms;
      unsigned long long t[12];
      hipMemcpyFromSymbol(t, HIP_SYMBOL(tiny_tsc), sizeof(t));
      // order of the marks: 0 1 2 3 4 5 [8 9 10] 6 7
      const int ord[11] = {0, 1, 2, 3, 4, 5, 8, 9, 10, 6, 7};
      if (r >= 5) for (int s = 1; s < 11; ++s) ph[s] += (t[ord[s]] > t[ord[s - 1]]) ? (double)(t[ord[s]] - t[ord[s - 1]]) : 0.0;
      unsigned long long ck[12];
      hipMemcpyFromSymbol(ck, HIP_SYMBOL(tiny_clk), sizeof(ck));
      const int last = want ? 7 : 5;
      if (r >= 5) { clk_ticks += (double)(ck[last] - ck[0]); wall_ticks += (double)(t[last] - t[0]); }
    }
    int fl = 0;
    double sm[4096];
    hipMemcpy(&fl, flag, 4, hipMemcpyDeviceToHost);
    hipMemcpy(sm, small, sizeof(sm), hipMemcpyDeviceToHost);
    printf("want_grad %d  k_tiny %.1f us/launch (flag %d, Q flag %g, log|L| %.6f)", want, tf / reps * 1e3, fl,
           sm[P * P + 2 + d + 3], sm[P * P]);
    const char* fn[11] = {"", "xw", "K_wait_load", "factor_inv", "Z", "gram", "Y", "cholQ", "T2", "W_publish",
                          "helpers_contract"};
    for (int s = 1; s < 11; ++s) printf("  %s %.2f", fn[s], ph[s] / reps / 100.0);
    printf(" us; shader clock %.0f MHz\n", clk_ticks / wall_ticks * 100.0);
  }
  return 0;
}
