// Clocks of the 2-4-tile one-launch objective (gpemu_snb.hpp) on synthetic inputs (dev tool).
// hipcc --offload-arch=gfx950 -O3 -w -DTINY_TIMING tools/hip/snb_bench.hip -o tools/hip/snb_bench_bin
// usage: snb_bench_bin [n] -- prints the launch time and the per-phase clocks (mean of 100).
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../../gp_emu_uqsa_amd/csrc/gpemu_kernels.hpp"
#include "../../gp_emu_uqsa_amd/csrc/gpemu_tiny.hpp"
#include "../../gp_emu_uqsa_amd/csrc/gpemu_snb.hpp"
using namespace gpe;
#ifndef DB_TIMING
__device__ unsigned long long db_tsc[8];
#endif

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 300, d = 10, P = 11, reps = 100;
  const int NB = (n + 127) / 128, np = NB * 128;
  std::vector<double> X(np * d, 0.0), F(np * P, 0.0);
  for (int i = 0; i < n; ++i)
    for (int k = 0; k < d; ++k) X[i * d + k] = std::fmod(0.37 * i + 0.11 * k * k + 0.05 * i * k, 1.0);
  for (int i = 0; i < n; ++i) {
    F[i] = std::sin(0.1 * i);
    for (int p = 1; p < P; ++p) F[i + p * np] = X[i * d + p - 1];
  }
  double *dX, *dF, *xw, *A, *Lb, *buf, *small;
  int* sync;
  hipMalloc(&dX, X.size() * 8); hipMalloc(&dF, F.size() * 8); hipMalloc(&xw, np * d * 8);
  hipMalloc(&A, (size_t)np * np * 8); hipMalloc(&Lb, (size_t)np * np * 8);
  const size_t nb = (size_t)np * np + 3 * 32 * (size_t)np + 32 * 33 + 128 * 128 + SNB_NH * 64;
  hipMalloc(&buf, nb * 8); hipMalloc(&small, 4096 * 8); hipMalloc(&sync, 16);
  hipMemcpy(dX, X.data(), X.size() * 8, hipMemcpyHostToDevice);
  hipMemcpy(dF, F.data(), F.size() * 8, hipMemcpyHostToDevice);
  SnbArgs a{};
  a.X = dX; a.F = dF; a.xw = xw; a.A = A; a.Lb = Lb; a.Xt = buf; a.Zt = buf + (size_t)np * np;
  a.Zo = a.Zt + 32 * np; a.Wg = a.Zo + 32 * np; a.T2g = a.Wg + 32 * np; a.Xscr = a.T2g + 32 * 33;
  a.small = small; a.sync = sync; a.abort_flag = sync + 3;
  a.n = n; a.np = np; a.NB = NB; a.d = d; a.P = P; a.mucm = 0;
  a.s2 = 1.0; a.coff = 1.0; a.cdiag = 1.0 + 1e-2; a.rscale = 0.0;
  for (int k = 0; k < 32; ++k) a.invd[k] = k < d ? 1.0 / 0.6 : 0.0;
  const size_t lds = SNB_LDS_DOUBLES * sizeof(double);
  hipFuncSetAttribute((const void*)k_snb<12>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int want = 1; want >= 0; --want) {
    a.want_grad = want;
    double acc[48] = {};
    float tot = 0.f;
    for (int r = 0; r < reps + 5; ++r) {
      hipMemset(sync, 0, 16);
      unsigned long long z[48] = {};
      hipMemcpyToSymbol(HIP_SYMBOL(snb_tsc), z, sizeof(z));
      hipEventRecord(e0);
      hipLaunchKernelGGL(k_snb<12>, dim3(1 + SNB_NH), dim3(256), lds, 0, a);
      hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      unsigned long long t[48];
      hipMemcpyFromSymbol(t, HIP_SYMBOL(snb_tsc), sizeof(t));
      if (r < 5) continue;
      tot += ms;
      for (int s = 0; s < 48; ++s) acc[s] += t[s] ? (double)(t[s] - t[0]) : 0.0;
    }
    double fl[2]; hipMemcpy(fl, small + P * P + NB, 8, hipMemcpyDeviceToHost);
    printf("n %d NB %d want_grad %d: %.1f us/launch (failed col %g); clocks (us from step 0 start):\n", n, NB, want,
           tot / reps * 1e3, fl[0]);
    for (int k = 0; k < NB; ++k)
      printf("  step %d: waited %.1f  tile in %.1f  factor %.1f  X out %.1f\n", k, acc[4 * k] / reps / 100,
             acc[4 * k + 1] / reps / 100, acc[4 * k + 2] / reps / 100, acc[4 * k + 3] / reps / 100);
    printf("  gram wait %.1f  gram %.1f  T2 %.1f\n  helper phase ends:", acc[16] / reps / 100, acc[17] / reps / 100,
           acc[18] / reps / 100);
    for (int p = 0; p < 4 * NB; ++p) printf(" %.1f", acc[20 + p] / reps / 100);
    printf("\n");
  }
  return 0;
}
