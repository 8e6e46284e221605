// i8_probe.hip -- dev probe: the int8 MFMA GEMM rate on
// gfx950 for the Ozaki-style fp64 emulation of the long-K GEMMs (verdict r5 item 7).
// C (int32, column-major) = A B^T over K, A (M x K) and B (N x K) int8 with K contiguous
// (the layout of X's columns for X^T X): 128 x 128 tiles, 4 waves of 64 x 64, 16 x 16 x 64
// i8 MFMA, stages of 128 k through double-buffered LDS (direct global -> LDS loads, 16-byte
// granules XOR-swizzled as the fp64 kernel's K-contiguous image), 2 workgroups per CU.
// Checks a small case exactly against the host, then times M = N = K = 8192.
// build: hipcc --offload-arch=gfx950 -O3 -o tools/hip/i8_probe_bin tools/hip/i8_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>

typedef int v4i __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int T = 128;     // tile
constexpr int SKB = 128;   // k (bytes) per stage
constexpr int OPND = T * SKB;   // one operand's stage image, bytes

__device__ __forceinline__ void glds16(const int8_t* src, int8_t* dst) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
}

__global__ void __launch_bounds__(256, 2) k_i8gemm(const int8_t* __restrict__ A, long long lda,
                                                   const int8_t* __restrict__ B, long long ldb,
                                                   int* __restrict__ C, long long ldc, int K, int mt) {
  extern __shared__ __attribute__((aligned(16))) int8_t lds[];
  const int ti = blockIdx.x % mt, tj = blockIdx.x / mt;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;
  // stage-load sources: instruction w = wave + 4 s writes LDS rows 8 w .. 8 w + 7; lane L row
  // 8 w + (L >> 3), slot L & 7 holds granule (L & 7) ^ ((row >> 1) & 7)
  const int kp = (lane & 7) ^ ((4 * wave + (lane >> 4)) & 7);
  const int8_t* sa = A + (long long)ti * T * lda + (long long)(8 * wave + (lane >> 3)) * lda + 16 * kp;
  const int8_t* sb = B + (long long)tj * T * ldb + (long long)(8 * wave + (lane >> 3)) * ldb + 16 * kp;
  auto stage = [&](int s, int buf) {
    int8_t* As = lds + buf * 2 * OPND;
    int8_t* Bs = As + OPND;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int w = wave + 4 * p;
      glds16(sa + (long long)p * 32 * lda + (long long)s * SKB, As + 8 * w * SKB);
      glds16(sb + (long long)p * 32 * ldb + (long long)s * SKB, Bs + 8 * w * SKB);
    }
  };
  v4i acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = v4i{0, 0, 0, 0};
  const int ns = K / SKB;
  stage(0, 0);
  const int r16 = lane & 15, sw = (lane & 15) >> 1;
  for (int s = 0; s < ns; ++s) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (s + 1 < ns) stage(s + 1, (s + 1) & 1);
    const int8_t* As = lds + (s & 1) * 2 * OPND;
    const int8_t* Bs = As + OPND;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int slot = ((4 * ks + (lane >> 4)) ^ sw) * 16;
      v4i af[4], bf[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = *reinterpret_cast<const v4i*>(As + (wm + 16 * i + r16) * SKB + slot);
#pragma unroll
      for (int j = 0; j < 4; ++j) bf[j] = *reinterpret_cast<const v4i*>(Bs + (wn + 16 * j + r16) * SKB + slot);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(bf[j], af[i], acc[i][j], 0, 0, 0);
    }
  }
  // D = (A B^T)^T per block: lane holds m = wm + 16 i + (lane & 15), n = wn + 16 j + 4 (lane >> 4) + r
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const long long m = (long long)ti * T + wm + 16 * i + r16, n = (long long)tj * T + wn + 16 * j + 4 * (lane >> 4) + r;
        C[m + n * ldc] = acc[i][j][r];
      }
}


// Variant B: 256 x 256 tiles, 4 waves of 128 x 128 (8 x 8 blocks, 256 int32 accumulators per
// lane), stages of 64 k (one MFMA k-step), double-buffered (2 x 32 KB), one workgroup per CU.
// LDS per CU per k-step: 64 KB of fragment reads + 32 KB of stage writes against 1024 MFMA
// cycles per SIMD (the 64 x 64 wave tile of variant A needs 512 + 128 cycles of LDS per 512).
constexpr int TB = 256, SKB2 = 64, OPND2 = TB * SKB2;
__global__ void __launch_bounds__(256, 1) k_i8gemm_b(const int8_t* __restrict__ A, long long lda,
                                                     const int8_t* __restrict__ B, long long ldb,
                                                     int* __restrict__ C, long long ldc, int K, int mt) {
  extern __shared__ __attribute__((aligned(16))) int8_t lds[];
  const int ti = blockIdx.x % mt, tj = blockIdx.x / mt;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = (wave >> 1) * 128, wn = (wave & 1) * 128;
  // instruction w = wave + 4 p (p < 4) writes rows 16 w .. 16 w + 15 (64 B each); lane L row
  // 16 w + (L >> 2), slot L & 3 holds granule (L & 3) ^ ((L >> 4) & 3)
  const int kp = (lane & 3) ^ ((lane >> 4) & 3);
  const int8_t* sa = A + (long long)ti * TB * lda + (long long)(16 * wave + (lane >> 2)) * lda + 16 * kp;
  const int8_t* sb = B + (long long)tj * TB * ldb + (long long)(16 * wave + (lane >> 2)) * ldb + 16 * kp;
  auto stage = [&](int s, int buf) {
    int8_t* As = lds + buf * 2 * OPND2;
    int8_t* Bs = As + OPND2;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int w = wave + 4 * p;
      glds16(sa + (long long)p * 64 * lda + (long long)s * SKB2, As + 16 * w * SKB2);
      glds16(sb + (long long)p * 64 * ldb + (long long)s * SKB2, Bs + 16 * w * SKB2);
    }
  };
  v4i acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = v4i{0, 0, 0, 0};
  const int ns = K / SKB2;
  stage(0, 0);
  const int r16 = lane & 15;
  const int slot = ((lane >> 4) ^ ((lane >> 2) & 3)) * 16;   // granule lane >> 4 of row r16
  for (int s = 0; s < ns; ++s) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (s + 1 < ns) stage(s + 1, (s + 1) & 1);
    const int8_t* As = lds + (s & 1) * 2 * OPND2;
    const int8_t* Bs = As + OPND2;
    v4i af[8], bf[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) af[i] = *reinterpret_cast<const v4i*>(As + (wm + 16 * i + r16) * SKB2 + slot);
#pragma unroll
    for (int j = 0; j < 8; ++j) bf[j] = *reinterpret_cast<const v4i*>(Bs + (wn + 16 * j + r16) * SKB2 + slot);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(bf[j], af[i], acc[i][j], 0, 0, 0);
  }
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const long long m = (long long)ti * TB + wm + 16 * i + r16, n = (long long)tj * TB + wn + 16 * j + 4 * (lane >> 4) + r;
        C[m + n * ldc] = acc[i][j][r];
      }
}

// Variant 2 (MFMA only): 16 independent accumulators per wave, operands in registers, no memory
__global__ void __launch_bounds__(256) k_i8peak(int* out, int iters) {
  v4i a = {(int)threadIdx.x, 3, 5, 7}, b = {11, (int)blockIdx.x, 13, 17};
  v4i acc[16];
#pragma unroll
  for (int u = 0; u < 16; ++u) acc[u] = v4i{u, 0, 0, 0};
  for (int it = 0; it < iters; ++it)
#pragma unroll
    for (int u = 0; u < 16; ++u) acc[u] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, acc[u], 0, 0, 0);
  int s = 0;
#pragma unroll
  for (int u = 0; u < 16; ++u) s += acc[u][0] + acc[u][1] + acc[u][2] + acc[u][3];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

typedef int v16i __attribute__((ext_vector_type(16)));
__global__ void __launch_bounds__(256) k_i8peak32(int* out, int iters) {
  v4i a = {(int)threadIdx.x, 3, 5, 7}, b = {11, (int)blockIdx.x, 13, 17};
  v16i acc[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) { acc[u] = v16i{}; acc[u][0] = u; }
  for (int it = 0; it < iters; ++it)
#pragma unroll
    for (int u = 0; u < 8; ++u) acc[u] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, acc[u], 0, 0, 0);
  int s = 0;
#pragma unroll
  for (int u = 0; u < 8; ++u)
#pragma unroll
    for (int r = 0; r < 16; ++r) s += acc[u][r];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

// Variant 3: 256 x 256 tiles, 4 waves of 128 x 128 as 4 x 4 blocks of the 32 x 32 x 32 i8 MFMA
// (256 int32 accumulators per lane), stages of 64 k (two k-steps) in a ring of 4 (128 KB), loads
// issued 3 stages ahead, one workgroup per CU.  Fragment of row r at granule g stored at slot
// g ^ ((r >> 2) & 3) of its 64-byte row (conflict-free for ds_read_b128's lane groups).
constexpr int T3 = 256, SK3 = 64, OP3 = T3 * SK3, NBUF3 = 4;
template <int N> __device__ __forceinline__ void vmwait() { asm volatile("s_waitcnt vmcnt(%0)" :: "n"(N) : "memory"); }
__global__ void __launch_bounds__(256, 1) k_i8gemm_c(const int8_t* __restrict__ A, long long lda,
                                                     const int8_t* __restrict__ B, long long ldb,
                                                     int* __restrict__ C, long long ldc, int K, int mt) {
  extern __shared__ __attribute__((aligned(16))) int8_t lds[];
  const int ti = blockIdx.x % mt, tj = blockIdx.x / mt;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = (wave >> 1) * 128, wn = (wave & 1) * 128;
  const int kp = (lane & 3) ^ ((lane >> 4) & 3);
  const int8_t* sa = A + (long long)ti * T3 * lda + (long long)(16 * wave + (lane >> 2)) * lda + 16 * kp;
  const int8_t* sb = B + (long long)tj * T3 * ldb + (long long)(16 * wave + (lane >> 2)) * ldb + 16 * kp;
  auto stage = [&](int s) {
    int8_t* As = lds + (s & (NBUF3 - 1)) * 2 * OP3;
    int8_t* Bs = As + OP3;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int w = wave + 4 * p;
      glds16(sa + (long long)p * 64 * lda + (long long)s * SK3, As + 16 * w * SK3);
      glds16(sb + (long long)p * 64 * ldb + (long long)s * SK3, Bs + 16 * w * SK3);
    }
  };
  v16i acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = v16i{};
  const int ns = K / SK3;
  stage(0);
  if (ns > 1) stage(1);
  if (ns > 2) stage(2);
  const int r32 = lane & 31, h = lane >> 5, sw = (r32 >> 2) & 3;
  for (int s = 0; s < ns; ++s) {
    if (s + 2 < ns) vmwait<16>();
    else if (s + 1 < ns) vmwait<8>();
    else vmwait<0>();
    __syncthreads();
    if (s + 3 < ns) stage(s + 3);
    const int8_t* As = lds + (s & (NBUF3 - 1)) * 2 * OP3;
    const int8_t* Bs = As + OP3;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int slot = ((2 * ks + h) ^ sw) * 16;
      v4i af[4], bf[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = *reinterpret_cast<const v4i*>(As + (wm + 32 * i + r32) * SK3 + slot);
#pragma unroll
      for (int j = 0; j < 4; ++j) bf[j] = *reinterpret_cast<const v4i*>(Bs + (wn + 32 * j + r32) * SK3 + slot);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(bf[j], af[i], acc[i][j], 0, 0, 0);
    }
  }
  // D = (A B^T)^T per block: lane holds m = wm + 32 i + (lane & 31), n = wn + 32 j + (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const long long m = (long long)ti * T3 + wm + 32 * i + r32;
        const long long n = (long long)tj * T3 + wn + 32 * j + (r & 3) + 8 * (r >> 2) + 4 * h;
        C[m + n * ldc] = acc[i][j][r];
      }
}

// MFMA-only 32x32x32 on random operands (8 pairs cycled): the clock the chip holds on random data
__global__ void __launch_bounds__(256) k_i8peak32r(const v4i* __restrict__ rnd, int* out, int iters) {
  v4i a[8], b[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) { a[u] = rnd[(blockIdx.x * 16 + u) * 256 + threadIdx.x]; b[u] = rnd[(blockIdx.x * 16 + 8 + u) * 256 + threadIdx.x]; }
  v16i acc[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) acc[u] = v16i{};
  for (int it = 0; it < iters; ++it)
#pragma unroll
    for (int u = 0; u < 8; ++u) acc[u] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[(u + it) & 7], b[u], acc[u], 0, 0, 0);
  int s = 0;
#pragma unroll
  for (int u = 0; u < 8; ++u)
#pragma unroll
    for (int r = 0; r < 16; ++r) s += acc[u][r];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

// Variants 4-6: the production loop of k_oz_gemm (gpemu_ozaki.hpp: 256 x 256 tiles, one k-step's
// MFMAs with the next k-step's fragment reads interleaved, one barrier per 64-k stage) with
// MODE 0: direct global -> LDS loads (4-stage ring, production); 1: register staging
// (global_load_dwordx4 into VGPRs three stages ahead, ds_write_b128 into a 3-buffer ring);
// 2: no global loads at all (the MFMA + LDS-read pipeline alone, on stale LDS)
template <int MODE>
__global__ void __launch_bounds__(256, 1) k_i8gemm_p(const int8_t* __restrict__ A, long long lda,
                                                     const int8_t* __restrict__ B, long long ldb,
                                                     int* __restrict__ C, long long ldc, int K, int mt) {
  extern __shared__ __attribute__((aligned(16))) int8_t lds[];
  constexpr int NB = MODE == 1 ? 3 : 4;
  const int ti = blockIdx.x % mt, tj = blockIdx.x / mt;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = (wave >> 1) * 128, wn = (wave & 1) * 128;
  const int kp = (lane & 3) ^ ((lane >> 4) & 3);
  const int8_t* sa = A + (long long)ti * T3 * lda + (long long)(16 * wave + (lane >> 2)) * lda + 16 * kp;
  const int8_t* sb = B + (long long)tj * T3 * ldb + (long long)(16 * wave + (lane >> 2)) * ldb + 16 * kp;
  auto bufp = [&](int s) { return lds + (s % NB) * 2 * OP3; };
  auto stage = [&](int s) {   // MODE 0
    int8_t* As = bufp(s);
    int8_t* Bs = As + OP3;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int w = wave + 4 * p;
      glds16(sa + (long long)p * 64 * lda + (long long)s * SK3, As + 16 * w * SK3);
      glds16(sb + (long long)p * 64 * ldb + (long long)s * SK3, Bs + 16 * w * SK3);
    }
  };
  v4i rg[2][8];   // MODE 1: two stages of staging registers
  auto gload = [&](int s, v4i (&r)[8]) {
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      r[2 * p] = *reinterpret_cast<const v4i*>(sa + (long long)p * 64 * lda + (long long)s * SK3);
      r[2 * p + 1] = *reinterpret_cast<const v4i*>(sb + (long long)p * 64 * ldb + (long long)s * SK3);
    }
  };
  auto lwrite = [&](int s, const v4i (&r)[8]) {
    int8_t* As = bufp(s);
    int8_t* Bs = As + OP3;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int w = wave + 4 * p;
      *reinterpret_cast<v4i*>(As + 16 * w * SK3 + 16 * lane) = r[2 * p];
      *reinterpret_cast<v4i*>(Bs + 16 * w * SK3 + 16 * lane) = r[2 * p + 1];
    }
  };
  v16i acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = v16i{};
  const int ns = K / SK3;
  const int r32 = lane & 31, h = lane >> 5, sw = (r32 >> 2) & 3;
  auto frags = [&](int s, int ks, v4i (&af)[4], v4i (&bf)[4]) {
    const int8_t* As = bufp(s);
    const int8_t* Bs = As + OP3;
    const int slot = ((2 * ks + h) ^ sw) * 16;
#pragma unroll
    for (int i = 0; i < 4; ++i) af[i] = *reinterpret_cast<const v4i*>(As + (wm + 32 * i + r32) * SK3 + slot);
#pragma unroll
    for (int j = 0; j < 4; ++j) bf[j] = *reinterpret_cast<const v4i*>(Bs + (wn + 32 * j + r32) * SK3 + slot);
  };
  auto mfmas = [&](const v4i (&af)[4], const v4i (&bf)[4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(bf[j], af[i], acc[i][j], 0, 0, 0);
  };
  auto wait_stage = [&](int s) {
    if constexpr (MODE == 0) {
      const int later = min(ns - 1, s + 2) - s;
      if (later >= 2) vmwait<16>();
      else if (later == 1) vmwait<8>();
      else vmwait<0>();
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  };
  v4i ca[4], cb[4], na[4], nb[4];
  if constexpr (MODE == 0) {
    for (int s = 0; s < min(ns, 3); ++s) stage(s);
    wait_stage(0);
    if (ns > 3) stage(3);
  } else if constexpr (MODE == 1) {
    gload(0, rg[0]);
    if (ns > 1) gload(1, rg[1]);
    vmwait<0>();
    lwrite(0, rg[0]);
    if (ns > 2) gload(2, rg[0]);
    wait_stage(0);
  } else {
    wait_stage(0);
  }
  frags(0, 0, ca, cb);
  for (int s = 0; s < ns; ++s) {
    mfmas(ca, cb);
    frags(s, 1, na, nb);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
    __builtin_amdgcn_sched_barrier(0);
    if (s + 1 < ns) {
      if constexpr (MODE == 1) {
        // stage s + 1's registers (loaded two iterations ago) into buffer (s + 1) % 3, whose
        // last reads (stage s - 2) every wave finished before the previous barrier
        if (s + 2 < ns) vmwait<8>(); else vmwait<0>();
        lwrite(s + 1, rg[(s + 1) & 1]);
        if (s + 3 < ns) gload(s + 3, rg[(s + 1) & 1]);
      }
      wait_stage(s + 1);
      if constexpr (MODE == 0)
        if (s + 4 < ns) stage(s + 4);
      frags(s + 1, 0, ca, cb);
    }
    __builtin_amdgcn_sched_barrier(0);
    mfmas(na, nb);
    __builtin_amdgcn_sched_barrier(0);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const long long m = (long long)ti * T3 + wm + 32 * i + r32;
        const long long n = (long long)tj * T3 + wn + 32 * j + (r & 3) + 8 * (r >> 2) + 4 * h;
        C[m + n * ldc] = acc[i][j][r];
      }
}

int main(int argc, char** argv) {
  const int big = argc > 1 ? atoi(argv[1]) : 8192;
  const int var = argc > 2 ? atoi(argv[2]) : 0;
  if (var == 2) {
    int* o;
    CK(hipMalloc(&o, 2048 * 256 * 4));
    const int iters = 4096;
    for (int wpc : {4, 8, 16}) {   // workgroups of 4 waves per CU: 1 or 2 waves per SIMD
      const int g = 256 * wpc / 4;
      hipLaunchKernelGGL(k_i8peak, dim3(g), dim3(256), 0, 0, o, iters);
      CK(hipDeviceSynchronize());
      hipEvent_t e0, e1;
      CK(hipEventCreate(&e0));
      CK(hipEventCreate(&e1));
      CK(hipEventRecord(e0));
      hipLaunchKernelGGL(k_i8peak, dim3(g), dim3(256), 0, 0, o, iters);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double ops = 2.0 * 16 * 16 * 64 * 16.0 * iters * g * 4;
      printf("MFMA-only i8 16x16x64, %d waves per SIMD: %.1f TOPS\n", wpc / 4, ops / (ms * 1e-3) / 1e12);
      hipLaunchKernelGGL(k_i8peak32, dim3(g), dim3(256), 0, 0, o, iters);
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0));
      hipLaunchKernelGGL(k_i8peak32, dim3(g), dim3(256), 0, 0, o, iters);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double ops32 = 2.0 * 32 * 32 * 32 * 8.0 * iters * g * 4;
      printf("MFMA-only i8 32x32x32, %d waves per SIMD: %.1f TOPS\n", wpc / 4, ops32 / (ms * 1e-3) / 1e12);
      {
        v4i* rnd;
        const size_t nr = (size_t)g * 16 * 256;
        CK(hipMalloc(&rnd, nr * sizeof(v4i)));
        std::vector<int> hr(nr * 4);
        for (auto& v : hr) v = rand() * 2 + (rand() & 1);
        CK(hipMemcpy(rnd, hr.data(), nr * sizeof(v4i), hipMemcpyHostToDevice));
        hipLaunchKernelGGL(k_i8peak32r, dim3(g), dim3(256), 0, 0, rnd, o, iters);
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int rr = 0; rr < 5; ++rr) hipLaunchKernelGGL(k_i8peak32r, dim3(g), dim3(256), 0, 0, rnd, o, iters);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("MFMA-only i8 32x32x32 RANDOM operands, %d waves per SIMD: %.1f TOPS\n", wpc / 4, 5 * ops32 / (ms * 1e-3) / 1e12);
        CK(hipFree(rnd));
      }
    }
    return 0;
  }
  for (int pass = 0; pass < 2; ++pass) {
    const int M = pass ? big : 256, N = M, K = pass ? big : 1024;
    std::vector<int8_t> ha((size_t)M * K), hb((size_t)N * K);
    srand(1 + pass);
    for (auto& v : ha) v = (int8_t)((rand() % 255) - 127);
    for (auto& v : hb) v = (int8_t)((rand() % 255) - 127);
    int8_t *da, *db;
    int* dc;
    CK(hipMalloc(&da, ha.size()));
    CK(hipMalloc(&db, hb.size()));
    CK(hipMalloc(&dc, (size_t)M * N * 4));
    CK(hipMemcpy(da, ha.data(), ha.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(db, hb.data(), hb.size(), hipMemcpyHostToDevice));
    const int TT = var >= 3 ? T3 : (var ? TB : T);
    const int mt = M / TT, nt = N / TT;
    const size_t lds = var >= 3 ? NBUF3 * 2 * OP3 : (var ? 4 * OPND2 : 4 * OPND);
    auto run = [&]() {
      if (var == 7) hipLaunchKernelGGL(k_i8gemm_p<0>, dim3(mt * nt), dim3(256), lds, 0, da, 0ll, db, 0ll, dc, (long long)M, K, mt);
      else if (var == 4) hipLaunchKernelGGL(k_i8gemm_p<0>, dim3(mt * nt), dim3(256), lds, 0, da, (long long)K, db, (long long)K, dc, (long long)M, K, mt);
      else if (var == 5) hipLaunchKernelGGL(k_i8gemm_p<1>, dim3(mt * nt), dim3(256), lds, 0, da, (long long)K, db, (long long)K, dc, (long long)M, K, mt);
      else if (var == 6) hipLaunchKernelGGL(k_i8gemm_p<2>, dim3(mt * nt), dim3(256), lds, 0, da, (long long)K, db, (long long)K, dc, (long long)M, K, mt);
      else if (var == 3) hipLaunchKernelGGL(k_i8gemm_c, dim3(mt * nt), dim3(256), lds, 0, da, (long long)K, db, (long long)K, dc, (long long)M, K, mt);
      else if (var) hipLaunchKernelGGL(k_i8gemm_b, dim3(mt * nt), dim3(256), lds, 0, da, (long long)K, db, (long long)K, dc, (long long)M, K, mt);
      else hipLaunchKernelGGL(k_i8gemm, dim3(mt * nt), dim3(256), lds, 0, da, (long long)K, db, (long long)K, dc, (long long)M, K, mt);
    };
    run();
    CK(hipDeviceSynchronize());
    if (!pass) {
      std::vector<int> hc((size_t)M * N);
      CK(hipMemcpy(hc.data(), dc, hc.size() * 4, hipMemcpyDeviceToHost));
      long long bad = 0;
      for (int m = 0; m < M; ++m)
        for (int n = 0; n < N; ++n) {
          long long s = 0;
          for (int k = 0; k < K; ++k) s += (long long)ha[(size_t)m * K + k] * hb[(size_t)n * K + k];
          if (s != hc[m + (size_t)n * M]) ++bad;
        }
      printf("check M=N=%d K=%d: %lld mismatches\n", M, K, bad);
    } else {
      hipEvent_t e0, e1;
      CK(hipEventCreate(&e0));
      CK(hipEventCreate(&e1));
      const int reps = 20;
      CK(hipEventRecord(e0));
      for (int r = 0; r < reps; ++r) run();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double ops = 2.0 * M * N * (double)K;
      printf("variant %d M=N=K=%d: %.3f ms per GEMM, %.1f TOPS (int8 dense peak ~5000)\n", var, M, ms / reps, ops / (ms / reps * 1e-3) / 1e12);
    }
    CK(hipFree(da));
    CK(hipFree(db));
    CK(hipFree(dc));
  }
  return 0;
}
