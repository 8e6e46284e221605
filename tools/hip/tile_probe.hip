// Per-tile timeline of one grouped-GEMM launch (dev tool): where a 128x128 tile's time
// goes -- start -> C + first stage landed -> K loop -> stores drained -- and how long a
// CU's two slots sit idle between tiles.
// hipcc --offload-arch=gfx950 -O3 -DGEMM_TTRACE tools/hip/tile_probe.hip -o tools/hip/tile_probe_bin
// usage: tile_probe_bin mt nt K kind [beta]   kind: 0 plain NN, 1 fused NN, 2 plain TN, 3 plain TT;
//        kind + 4: the CDEF instance
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <vector>
#include "../../gp_emu_uqsa_amd/csrc/gpemu_kernels.hpp"
using namespace gpe;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

int main(int argc, char** argv) {
  const int mt = argc > 1 ? atoi(argv[1]) : 48, nt = argc > 2 ? atoi(argv[2]) : 48;
  const int K = argc > 3 ? atoi(argv[3]) : 512;
  int fused = argc > 4 ? atoi(argv[4]) : 0;
  const double beta = argc > 5 ? atof(argv[5]) : 1.0;
  if (mt * nt > 65536 || K % GK) { printf("bad shape\n"); return 1; }
  const long long M = (long long)mt * TILE, N = (long long)nt * TILE;
  double *A, *B, *C;
  CK(hipMalloc(&A, M * K * 8));
  CK(hipMalloc(&B, (long long)K * N * 8));
  CK(hipMalloc(&C, M * N * 8));
  {
    std::vector<double> h(std::max(M * K, std::max((long long)K * N, M * N)));
    for (size_t i = 0; i < h.size(); ++i) h[i] = std::sin(0.37 * (double)i) * 0.5;
    CK(hipMemcpy(A, h.data(), M * K * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(B, h.data(), (long long)K * N * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(C, h.data(), M * N * 8, hipMemcpyHostToDevice));
  }
  GemmProb p{};
  p.A = A; p.B = B; p.C = C; p.lda = (fused & 3) >= 2 ? K : M; p.ldb = (fused & 3) == 3 ? K : N; p.ldc = M;
  p.mt = mt; p.nt = nt; p.K = K; p.flags = 0; p.alpha = -1.0; p.beta = beta;
  p.tile_begin = 0; p.ntiles = mt * nt;
  GemmProb* dp;
  CK(hipMalloc(&dp, sizeof(GemmProb)));
  CK(hipMemcpy(dp, &p, sizeof(GemmProb), hipMemcpyHostToDevice));
  const size_t lds = (size_t)G_LDS_LAUNCH_DOUBLES * 8;
  const bool cdef = fused >= 4;   // kind + 4: the CDEF instance (C added inside the K loop)
  fused &= 3;
  auto kern = cdef ? (fused == 1 ? k_gemm<false, false, true, true>
                      : fused == 2 ? k_gemm<true, false, false, true>
                      : fused == 3 ? k_gemm<true, true, false, true> : k_gemm<false, false, false, true>)
                   : (fused == 1 ? k_gemm<false, false, true>
                      : fused == 2 ? k_gemm<true, false, false>
                      : fused == 3 ? k_gemm<true, true, false> : k_gemm<false, false, false>);
  CK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  const int tiles = mt * nt;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float ms = 0.f;
  for (int rep = 0; rep < 4; ++rep) {   // warm clocks; the last launch is the one traced
    if (rep == 3) {   // entries are numbered in start order from the reset count
      const unsigned z = 0;
      CK(hipMemcpyToSymbol(HIP_SYMBOL(gemm_ttrace_n), &z, sizeof(z)));
    }
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(kern, dim3(tiles), dim3(256), lds, 0, dp, 1, (const unsigned*)nullptr, (int*)nullptr, (int*)nullptr);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
  }
  std::vector<unsigned long long> t((size_t)8 * GEMM_TTRACE_MAX);
  CK(hipMemcpyFromSymbol(t.data(), HIP_SYMBOL(gemm_ttrace), t.size() * 8));
  unsigned long long t0 = ~0ull, t3 = 0;
  double d01 = 0, d12 = 0, d23 = 0;
  std::map<unsigned, std::vector<std::pair<unsigned long long, unsigned long long>>> cu;
  for (int b = 0; b < tiles; ++b) {
    const unsigned long long* r = &t[(size_t)b * 8];
    t0 = std::min(t0, r[0]);
    t3 = std::max(t3, r[3]);
    d01 += (double)(r[1] - r[0]);
    d12 += (double)(r[2] - r[1]);
    d23 += (double)(r[3] - r[2]);
    const unsigned hw = (unsigned)r[4], xcc = (unsigned)r[5] & 0xf;
    const unsigned key = (xcc << 16) | ((hw >> 8) & 0xff);   // XCC, SE/SH/CU
    cu[key].push_back({r[0], r[3]});
  }
  // per CU: busy slot time against 2 slots x the launch span; the gap between a tile's
  // start and the end of the tile it replaced (k-th start vs (k-2)-th end)
  double busy = 0, gap = 0;
  int ngap = 0;
  for (auto& kv : cu) {
    auto& v = kv.second;
    std::vector<unsigned long long> st, en;
    for (auto& x : v) { busy += (double)(x.second - x.first); st.push_back(x.first); en.push_back(x.second); }
    std::sort(st.begin(), st.end());
    std::sort(en.begin(), en.end());
    for (size_t k = 2; k < st.size(); ++k) { gap += (double)st[k] - (double)en[k - 2]; ++ngap; }
  }
  const double span = (double)(t3 - t0);
  const double flops = 2.0 * M * N * K;
  printf("mt=%d nt=%d K=%d %s%s beta=%g: %.3f ms %.2f TF/s  span %.1f us  CUs %zu\n", mt, nt, K,
         (const char*[]){"NN", "fused NN", "TN", "TT"}[fused], cdef ? " cdef" : "", beta, ms, flops / ms / 1e9, span * 0.01, cu.size());
  printf("  per tile (us): start->first stage %.2f  K loop %.2f  store drain %.2f  total %.2f\n",
         d01 / tiles * 0.01, d12 / tiles * 0.01, d23 / tiles * 0.01, (d01 + d12 + d23) / tiles * 0.01);
  printf("  slot occupancy %.3f (busy / (2 x CUs x span)); mean refill gap %.2f us over %d\n",
         busy / (2.0 * cu.size() * span), ngap ? gap / ngap * 0.01 : 0.0, ngap);
  return 0;
}
