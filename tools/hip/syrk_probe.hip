// Cycles per trailing-update block pair (db_syrk_pair) on 1 and 3 waves of one workgroup (dev tool).
// hipcc --offload-arch=gfx950 -O3 -w tools/hip/syrk_probe.hip -o tools/hip/syrk_probe_bin
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../gp_emu_uqsa_amd/csrc/gpemu_diag.hpp"
using namespace gpe;

template <int MODE>
__global__ void __launch_bounds__(256) k_syrk(double* out, unsigned long long* t, int n, int nw) {
  extern __shared__ __attribute__((aligned(16))) double lb[];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  for (int e = threadIdx.x; e < 36 * DB_BS; e += 256) lb[e] = 1e-3 * (e % 97);
  __syncthreads();
  const unsigned long long s0 = clock64();
  if (wave < nw) {
    // each wave its own blocks: a = 3w, b = 3w + 1, o = 3w + 2 (and +12 for the pair's second)
    const int a0 = db_blk(1 + wave, 0), b0 = db_blk(4, 0), o0 = db_blk(4 + wave, 1 + wave);
    const int a1 = db_blk(5, 1), b1 = db_blk(6, 1), o1 = db_blk(7, 2 + wave);
    if (MODE >= 2) {   // the factor's update loop (its block enumeration), n / 16 sweeps of the 7 steps
      for (int it = 0; it < n / 16; ++it)
        for (int jb = 0; jb < 7; ++jb) {
          const int m = 7 - jb, cnt = m * (m + 1) / 2;
          for (int b = wave + 1; b < cnt; b += 6) {
            int rr = 0;
            while ((rr + 1) * (rr + 2) / 2 <= b) ++rr;
            const int ib = jb + 1 + rr, kb = jb + 1 + (b - rr * (rr + 1) / 2);
            const int b1 = b + 3;
            const bool has1 = b1 < cnt;
            int r1 = rr;
            while ((r1 + 1) * (r1 + 2) / 2 <= b1) ++r1;
            const int ib1 = jb + 1 + r1, kb1 = jb + 1 + (b1 - r1 * (r1 + 1) / 2);
            if (MODE == 2)
              db_syrk_pair(lb, db_blk(ib, jb), db_blk(kb, jb), db_blk(ib, kb),
                           has1 ? db_blk(ib1, jb) : 0, has1 ? db_blk(kb1, jb) : 0, has1 ? db_blk(ib1, kb1) : 0, has1);
            else   // as gpemu_diag.hpp now: a lone block goes twice, branch-free
              db_syrk_pair(lb, db_blk(ib, jb), db_blk(kb, jb), db_blk(ib, kb), db_blk(has1 ? ib1 : ib, jb),
                           db_blk(has1 ? kb1 : kb, jb), has1 ? db_blk(ib1, kb1) : db_blk(ib, kb), true);
          }
        }
    } else {
      for (int i = 0; i < n; ++i) {
        if (MODE == 0) db_syrk_pair(lb, a0, b0, o0, a1, b1, o1, true);
        else db_syrk_block(lb, a0, b0, o0);
      }
    }
  }
  __syncthreads();
  const unsigned long long s1 = clock64();
  out[threadIdx.x] = lb[threadIdx.x];
  if (threadIdx.x == 0) t[0] = s1 - s0;
}

int main() {
  double* out;
  unsigned long long* t;
  hipMalloc(&out, 256 * 8);
  hipMalloc(&t, 8);
  const int n = 2000;
  const size_t lds = 37 * DB_BS * 8;
  for (int mode = 0; mode < 4; ++mode)
    for (int nw = 1; nw <= 4; nw += (nw == 1 ? 2 : 1)) {
      unsigned long long th = 0;
      for (int it = 0; it < 3; ++it) {
        if (mode == 0) hipLaunchKernelGGL(k_syrk<0>, dim3(1), dim3(256), lds, 0, out, t, n, nw);
        else if (mode == 1) hipLaunchKernelGGL(k_syrk<1>, dim3(1), dim3(256), lds, 0, out, t, n, nw);
        else if (mode == 2) hipLaunchKernelGGL(k_syrk<2>, dim3(1), dim3(256), lds, 0, out, t, n, nw);
        else hipLaunchKernelGGL(k_syrk<3>, dim3(1), dim3(256), lds, 0, out, t, n, nw);
        hipDeviceSynchronize();
        hipMemcpy(&th, t, 8, hipMemcpyDeviceToHost);
      }
      printf("%s, %d waves: %.0f cycles per call per wave\n", mode == 0 ? "syrk_pair " : (mode == 1 ? "syrk_block" : (mode == 2 ? "factor loop, flagged lone block (per sweep / 16)" : "factor loop, lone block twice (per sweep / 16)")), nw, (double)th / n);
    }
  return 0;
}
