// Ping-pong fp64 GEMM probe (dev tool): one 512-thread workgroup per CU, a 128 x 256
// output tile, 8 waves of 64 x 64 (wave w: rows 64 (w >> 2), columns 64 (w & 3)), so
// the two waves on each SIMD (w and w + 4) belong to the two row groups.  Group 1
// runs one barrier behind group 0: while one group issues its 16 MFMAs of a k-step,
// the other reads its next fragments and issues its share of the LDS-DMA prefetch
// (guide: the 8-phase template).  K staged 16 deep in a ring of three 48 KiB buffers,
// loads two stages ahead, counted vmcnt, raw s_barrier.  TT layout (both operands
// K-contiguous, as the LAUUM's A^-1 = X^T X); compared with k_gemm<true, true> on the
// same problem, warm, interleaved.
// hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/hip/pp_probe.hip -o tools/hip/pp_probe_bin
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>
#include "../../gp_emu_uqsa_amd/csrc/gpemu_kernels.hpp"
using namespace gpe;

namespace {

constexpr int PP_M = 128, PP_N = 256;
constexpr int PP_A = PP_M * GK;                 // doubles per A stage (2048)
constexpr int PP_B = PP_N * GK;                 // doubles per B stage (4096)
constexpr int PP_STAGE = PP_A + PP_B;           // 6144 doubles = 48 KiB
constexpr int PP_LDS = 3 * PP_STAGE;            // 144 KiB

__device__ __forceinline__ void pp_bar() { __builtin_amdgcn_s_barrier(); }

// this wave's share of one stage's LDS-DMA: A 16 and B 32 wave-instructions (8 rows x
// 16 doubles each, swizzled as k_gemm's K-contiguous image), 6 per wave, issued in
// three pairs (part 0..2) so they spread over the stage's phases
__device__ __forceinline__ void pp_glds(const double* Ab, const double* Bb, long long lda, long long ldb, int k0,
                                        double* st, int part) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int w = wave + 8 * (2 * part + u);   // instruction 0..47
    if (w < 16) {
      const int m = 8 * w + (lane >> 3), kp = (lane & 7) ^ ((m >> 1) & 7);
      glds16(Ab + (long long)m * lda + k0 + 2 * kp, st + 8 * w * GK);
    } else {
      const int wb = w - 16;
      const int n = 8 * wb + (lane >> 3), kp = (lane & 7) ^ ((n >> 1) & 7);
      glds16(Bb + (long long)n * ldb + k0 + 2 * kp, st + PP_A + 8 * wb * GK);
    }
  }
}

__device__ __forceinline__ void pp_frags(const double* st, int ks, int lane, int wm, int wn, double (&af)[4],
                                         double (&bf)[4]) {
  const int krow = ks * 4 + (lane >> 4);
#pragma unroll
  for (int i = 0; i < 4; ++i) af[i] = st[kc_idx(wm + i * 16 + (lane & 15), krow)];
#pragma unroll
  for (int j = 0; j < 4; ++j) bf[j] = st[PP_A + kc_idx(wn + j * 16 + (lane & 15), krow)];
}

template <int NKS>   // k-steps (of 4) per phase: 1 or 2
__global__ void __launch_bounds__(512, 1) k_pp_tt(const double* __restrict__ A, long long lda,
                                                 const double* __restrict__ B, long long ldb, double* C,
                                                 long long ldc, int mt, int K, double alpha, double beta) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  constexpr int NPH = 4 / NKS;   // phases per stage
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int grp = wave >> 2;
  const int wm = grp * 64, wn = (wave & 3) * 64;
  const int ti = blockIdx.x % mt, tj = blockIdx.x / mt;   // tj: 256-column tile
  const double* Ab = A + (long long)ti * PP_M * lda;
  const double* Bb = B + (long long)tj * PP_N * ldb;
  double* Cb = C + (long long)ti * PP_M + (long long)tj * PP_N * ldc;
  d4 acc[4][4];
  const double sc = beta / alpha;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        acc[i][j][r] = sc * gld1(Cb + wm + i * 16 + (lane & 15) + (long long)(wn + j * 16 + mfma64_row(lane, r)) * ldc);
  const int nk = K / GK;
  // prologue: stages 0 and 1 in flight
  for (int p = 0; p < 3; ++p) pp_glds(Ab, Bb, lda, ldb, 0, lds, p);
  if (nk > 1)
    for (int p = 0; p < 3; ++p) pp_glds(Ab, Bb, lda, ldb, GK, lds + PP_STAGE, p);
  if (nk > 1) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  pp_bar();
  if (grp == 1) pp_bar();   // group 1 runs one barrier behind
  double af[NKS][4], bf[NKS][4];
  for (int s = 0; s < nk; ++s) {
    const double* st = lds + (s % 3) * PP_STAGE;
    double* nst = lds + ((s + 2) % 3) * PP_STAGE;
#pragma unroll
    for (int ph = 0; ph < NPH; ++ph) {
      // read slot: this phase's fragments; in the stage's last phase this wave's part of
      // stage s + 2's prefetch (>= 2 phases after the last read of that buffer), then
      // the wait that retires stage s + 1 (read from the next phase on)
#pragma unroll
      for (int q = 0; q < NKS; ++q) pp_frags(st, ph * NKS + q, lane, wm, wn, af[q], bf[q]);
      if (NKS == 1) {
        if (ph >= 1 && s + 2 < nk) pp_glds(Ab, Bb, lda, ldb, (s + 2) * GK, nst, ph - 1);
      } else if (ph == NPH - 1 && s + 2 < nk) {
        for (int p = 0; p < 3; ++p) pp_glds(Ab, Bb, lda, ldb, (s + 2) * GK, nst, p);
      }
      if (ph == NPH - 1 && s + 1 < nk) {
        if (s + 2 < nk) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      pp_bar();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int q = 0; q < NKS; ++q)
#pragma unroll
        for (int u = 0; u < 16; ++u)
          acc[u >> 2][u & 3] = __builtin_amdgcn_mfma_f64_16x16x4f64(bf[q][u & 3], af[q][u >> 2], acc[u >> 2][u & 3], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      pp_bar();
    }
  }
  if (grp == 0) pp_bar();   // equal barrier counts before the workgroup ends
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        gst1(Cb + wm + i * 16 + (lane & 15) + (long long)(wn + j * 16 + mfma64_row(lane, r)) * ldc, alpha * acc[i][j][r]);
}

}  // namespace

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main() {
  const int mt = 64, N = mt * TILE;   // 8192 x 8192 output
  const int Kmax = 4096;
  std::vector<double> h((size_t)N * Kmax);
  for (size_t i = 0; i < h.size(); ++i) h[i] = std::sin(0.37 * (double)(i % 100003)) * 0.5;
  double *A, *B, *C0, *C1;
  CK(hipMalloc(&A, h.size() * 8));
  CK(hipMalloc(&B, h.size() * 8));
  CK(hipMalloc(&C0, (size_t)N * N * 8));
  CK(hipMalloc(&C1, (size_t)N * N * 8));
  CK(hipMemcpy(A, h.data(), h.size() * 8, hipMemcpyHostToDevice));
  for (size_t i = 0; i < h.size(); ++i) h[i] = std::cos(0.11 * (double)(i % 70001)) * 0.5;
  CK(hipMemcpy(B, h.data(), h.size() * 8, hipMemcpyHostToDevice));
  GemmProb* dp;
  CK(hipMalloc(&dp, sizeof(GemmProb)));
  CK(hipFuncSetAttribute((const void*)k_pp_tt<1>, hipFuncAttributeMaxDynamicSharedMemorySize, PP_LDS * 8));
  CK(hipFuncSetAttribute((const void*)k_pp_tt<2>, hipFuncAttributeMaxDynamicSharedMemorySize, PP_LDS * 8));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const size_t lds4 = G_LDS_LAUNCH_DOUBLES * sizeof(double);
  for (int K : {512, 1024, 2048, 4096}) {
    GemmProb p{};
    p.A = A; p.B = B; p.C = C0; p.lda = K; p.ldb = K; p.ldc = N;
    p.mt = mt; p.nt = mt; p.K = K; p.flags = 0; p.alpha = -1.0; p.beta = 1.0; p.ntiles = mt * mt;
    CK(hipMemcpy(dp, &p, sizeof(p), hipMemcpyHostToDevice));
    auto run = [&](int v, int reps) -> float {
      float ms = 0;
      CK(hipEventRecord(e0));
      for (int r = 0; r < reps; ++r) {
        if (v == 0) hipLaunchKernelGGL((k_gemm<true, true>), dim3(mt * mt), dim3(256), lds4, 0, dp, 1, nullptr, nullptr, nullptr);
        else if (v == 1) hipLaunchKernelGGL(k_pp_tt<1>, dim3(mt * (mt / 2)), dim3(512), PP_LDS * 8, 0, A, (long long)K, B,
                                            (long long)K, C1, (long long)N, mt, K, -1.0, 1.0);
        else hipLaunchKernelGGL(k_pp_tt<2>, dim3(mt * (mt / 2)), dim3(512), PP_LDS * 8, 0, A, (long long)K, B,
                                (long long)K, C1, (long long)N, mt, K, -1.0, 1.0);
      }
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
      return ms / reps;
    };
    const int reps = K >= 2048 ? 4 : 12;
    // correctness: one launch each from C = 0
    CK(hipMemset(C0, 0, (size_t)N * N * 8));
    CK(hipMemset(C1, 0, (size_t)N * N * 8));
    run(0, 1);
    run(2, 1);
    std::vector<double> r0((size_t)N * N), r1((size_t)N * N);
    CK(hipMemcpy(r0.data(), C0, r0.size() * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(r1.data(), C1, r1.size() * 8, hipMemcpyDeviceToHost));
    double dmax = 0, ref = 0;
    for (size_t i = 0; i < r0.size(); ++i) { dmax = std::fmax(dmax, std::fabs(r0[i] - r1[i])); ref = std::fmax(ref, std::fabs(r0[i])); }
    float t0 = 0, t1 = 0, t2 = 0;
    for (int rep = 0; rep < 3; ++rep) { t0 += run(0, reps); t1 += run(1, reps); t2 += run(2, reps); }   // interleaved, warm
    const double fl = 2.0 * N * (double)N * K;
    printf("K=%5d  k_gemm<T,T> %6.2f TF/s   ping-pong x1 %6.2f   x2 %6.2f TF/s   (x2 max |diff| %.2e of %.2e)\n", K,
           fl / (t0 / 3) / 1e9, fl / (t1 / 3) / 1e9, fl / (t2 / 3) / 1e9, dmax, ref);
  }
  return 0;
}
