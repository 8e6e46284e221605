// gpemu_tiny.hpp -- the objective of a training set of at most 128 points (one 128 x 128
// tile: the reference's examples, toy-sim's 60 and toysim3D's 100 points) in ONE launch of
// k_tiny instead of the general path's ~20 small launches and copies.
//
// Workgroup 0 (everything after the first staging in LDS): K's image in (built by the
//   helpers), db_factor_invert (L and X = L^-1 assembled in LDS), X's image out to the
//   helpers, Z = X [f H] (16 x 16 x 4 fp64 MFMA on X's blocks), the Gram Z^T Z.  Value only:
//   stop there (Gram, log|L| and the failed column go to the host, whose q x q algebra gives
//   the LLH).  With the gradient, on: Y = X^T Z (MFMA); the q x q algebra of the host's
//   small_from_gram / small_t2 (Cholesky of Q = H^T A^-1 H one column per barrier, beta and
//   sqrt(c), Kq^-1 one column per lane); W = Y T2 = X^T (Z T2) = [sqrt(c) alpha,
//   Kq^-1-scaled L^-T L^-1 H] (MFMA), out to the helpers.
// TINY_NH helper workgroups, wave w of helper h owning lower 16 x 16 block 4h + w: its K-build
//   entries (k_pairs' arithmetic); then, once X is out, its block of X^T X (MFMA) and, once W
//   is out, - W W^T and the contraction of its entries in the accumulators into the d + 3 sums
//   of k_contract (<M, E (.) D_k>, <M, E>, tr M, sum M_ii r_i); each helper's partial sums go
//   to the host, which adds them in helper order.
// The host computes the LLH from the Gram with the same small_from_gram as the general path,
// and the gradient from the d + 3 sums with the same small_grad.
// The arithmetic of every quantity is the general path's formula (the K-build's entries are
// k_pairs' to the bit: same scaled coordinates, same fma order, same selects); products and
// sums run in other orders than the general path's GEMMs and k_contract, so results agree to
// rounding.
// Global -> LDS staging issues every load of a thread before its first LDS store (a load /
// store pair per loop iteration put one memory latency per iteration in sequence).
// Limits: n <= 128, d <= 32, q + 1 <= 32 (the host takes the general path otherwise).
#pragma once

namespace gpe {

constexpr int TINY_DM = 32;   // basis columns held per row
// LDS row pitches of the row-major [i][k] images: an odd number of doubles, so 16 or 64
// lanes reading 16 or 64 different rows spread over the banks (a pitch of 16 or 32
// doubles put 32 or 64 lanes of a wave on one bank: ~100 us per launch in a first version)
constexpr int TINY_ZP = TINY_DM + 1;
template <int DM> struct TinyPitch { static constexpr int v = DM + 1; };
// the q x q algebra in zs once Z is consumed: Gram (P x P), Q's Cholesky (q x q, pitch 32),
// its diagonal, u, T2 ([k][p], pitch TINY_ZP)
constexpr int TY_G = 0, TY_Q = 1024, TY_QD = 2048, TY_B = 2080, TY_T2 = 2112;
static_assert(TY_T2 + TINY_DM * TINY_ZP <= 128 * TINY_ZP, "algebra fits in zs");

// dev-tool phase clocks (tools/hip/tiny_bench.hip): -DTINY_TIMING
#ifdef TINY_TIMING
__device__ unsigned long long tiny_tsc[12], tiny_clk[12];   // 100 MHz wall clock, shader clock
#define TINY_T(s) do { __syncthreads(); if (threadIdx.x == 0) { tiny_tsc[s] = wall_clock64(); tiny_clk[s] = clock64(); } } while (0)
#else
#define TINY_T(s) do {} while (0)
#endif

struct TinyArgs {
  const double* X;      // n_pad x d raw points, row-major (rows >= n zero)
  const double* F;      // [f H], 128 x P column-major (rows >= n zero)
  const double* r;      // per-point nugget added on the diagonal (rscale r_i), or null
  const double* rdiag;  // the std kernel's sigma-gradient r (sum M_ii r_i), or null
  double* xw;           // out: scaled points (128 x d)
  double* L;            // out: L (ld 128)
  double* Xo;           // out: X = L^-1 (ld 128, zero upper)
  double* Z;            // out: Z = L^-1 [f H] (ld 128, P columns)
  double* small;        // out (pinned host memory): Gram (P x P) | log|L| | failed column |
                        // (d + 3) | Q not PD | the helpers' partial sums (TINY_NH x 64,
                        // slot 63 of each: the call's tag once the helper's sums are in)
  double* K;            // the helpers' K-build in the block-packed image's layout; L's buffer
  double* Xp;           // X's LDS image (block-packed, 36 x DB_BS doubles)
  double* Wg;           // W for the helpers (128 x 32, row-major)
  int* sync;            // [0] K-build count, [1] X flag, [2] W flag: monotone over the
                        // context's calls (zeroed after a failed one)
  int* abort_flag;      // the failed column (or 1: Q not positive definite); zero on entry
  int ek, eg;           // this call's ordinal among all calls / gradient calls since the zeroing
  int n, d, P, want_grad, mucm;
  int dbg_skip;         // dev switch (tests): this helper gives up its first wait; else -1
  double tag;           // this call's tag (never repeats in a context) for the helpers' sums
  double s2, coff, cdiag, rscale;
  double invd[32];
};

constexpr int TINY_NH = 9;
constexpr int TINY_SYNC_INTS = 3;

// Hand-offs between the workgroups of one k_tiny launch without agent fences (each a
// write-back or invalidate of ~1.7-6.5 us on the chain, three of them in a row before): every
// handed-off byte stored and loaded `sc1` (global_store/load ... sc1: L2, not L1), every
// storing wave's vmcnt(0) wait and the workgroup's barrier before ONE lane's counter add or
// sc1 flag store; the consumer polls sc1, then a barrier before its loads (the MI355X
// guide's measured sc1 hand-off form, one workgroup per CU).
typedef __attribute__((address_space(1))) double tiny_gdouble;
typedef __attribute__((address_space(1))) int tiny_gint;
__device__ __forceinline__ void tiny_st(double* p, double v) {
  __hip_atomic_store((tiny_gdouble*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double tiny_ld(const double* p) {
  return __hip_atomic_load((tiny_gdouble*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int tiny_ldi(const int* p) {
  return __hip_atomic_load((tiny_gint*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// sc1 load through a buffer descriptor over [base, base + 4 GB): an ordinary load the compiler
// batches (an atomic load is issued and waited for one at a time); the consumer form of the
// sc1 hand-off ("buffer_load ... sc1", aux 16)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t tiny_rsrc(const double* base) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, -1, 0x00020000);
}
__device__ __forceinline__ double tiny_bld(__amdgpu_buffer_rsrc_t r, long long idx) {
  const auto v = __builtin_amdgcn_raw_buffer_load_b64(r, (int)(idx * 8), 0, 16);
  return __longlong_as_double(((long long)v[1] << 32) | v[0]);
}
// every wave's stores landed, then one lane signals (add 1, or store v when v > 0)
__device__ __forceinline__ void tiny_signal(int* p, int v) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    if (v > 0) __hip_atomic_store((tiny_gint*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else __hip_atomic_fetch_add((tiny_gint*)p, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
// one lane polls until *p >= want (1) or the launch aborted (2); 0 after ~1 s (never
// expected: the waiter then raises the abort flag itself, so every other waiter of the
// launch stops at its next poll instead of running out its own budget); the result in *st
// for every thread after the barrier.  The two words are loaded together each poll.
// skip (the dev switch GPEMU_DEBUG_SKIP_WAIT, tests only): give up at once, as a timeout.
__device__ __forceinline__ int tiny_wait(const int* p, int want, int* abort_flag, int* st, bool skip = false) {
  if (threadIdx.x == 0) {
    int v = 0;
    for (long it = skip ? (1l << 22) : 0; it < (1l << 22); ++it) {
      const int x = tiny_ldi(p);
      const int ab = abort_flag ? tiny_ldi(abort_flag) : 0;
      if (x >= want) { v = 1; break; }
      if (ab) { v = 2; break; }
      __builtin_amdgcn_s_sleep(2);
    }
    if (v == 0 && abort_flag) atomicCAS(abort_flag, 0, GEMM_WAIT_TIMEOUT);
    *st = v;
  }
  __syncthreads();
  const int v = *st;
  __syncthreads();
  return v;
}
__host__ __device__ constexpr int tiny_tri_row(int b) {   // row of lower-triangle entry b
  int r = 0;
  while ((r + 1) * (r + 2) / 2 <= b) ++r;
  return r;
}   // helper workgroups: 4 waves each, one lower 16 x 16 block per wave

// N pieces per thread (index threadIdx.x + 256 u): every load, then every store
template <int N, class Ld, class St>
__device__ __forceinline__ void tiny_stage(Ld ld, St st) {
  double v[N];
#pragma unroll
  for (int u = 0; u < N; ++u) v[u] = ld((int)threadIdx.x + 256 * u);
#pragma unroll
  for (int u = 0; u < N; ++u) st((int)threadIdx.x + 256 * u, v[u]);
}

// k_contract's sums over the pairs (i >= j) of M: the diagonal to tr and the r sum, an
// off-diagonal pair to <M, E> and <M, E (.) D_k>
template <int DM>
struct TinySums {
  double acc[DM];
  double e, t, r;
  __device__ void zero() {
#pragma unroll
    for (int k = 0; k < DM; ++k) acc[k] = 0.0;
    e = t = r = 0.0;
  }
  // workgroup sum (fixed order) into out[0 .. d+3): the DM + 3 values of a thread in one
  // shuffle tree, the four waves' partials added by d + 3 threads; red: 4 (DM + 3) doubles
  __device__ void reduce(int d, double* red, double* out) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    double v[DM + 3];
#pragma unroll
    for (int k = 0; k < DM; ++k) v[k] = acc[k];
    v[DM] = e;
    v[DM + 1] = t;
    v[DM + 2] = r;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1)
#pragma unroll
      for (int k = 0; k < DM + 3; ++k) v[k] += __shfl_down(v[k], off, 64);
    if (lane == 0)
#pragma unroll
      for (int k = 0; k < DM + 3; ++k) red[wave * (DM + 3) + k] = v[k];
    __syncthreads();
    if (tid < d + 3) {
      const int k = tid < d ? tid : DM + (tid - d);
      out[tid] = (red[k] + red[(DM + 3) + k]) + (red[2 * (DM + 3) + k] + red[3 * (DM + 3) + k]);
    }
  }
};

// s - sum_{k0 <= k < k1} a[k sa] b[k sb], eight loads of each in flight per step (a plain
// loop with a run-time trip count waits one LDS latency per term); terms past k1 masked
// (their reads stay inside the kernel's LDS)
__device__ __forceinline__ double tiny_dot(double s, const double* a, int sa, const double* b, int sb, int k0, int k1) {
  for (int c = k0; c < k1; c += 8) {
    double x[8], y[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      x[u] = a[(c + u) * sa];
      y[u] = b[(c + u) * sb];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const bool in = c + u < k1;
      s = fma(-(in ? x[u] : 0.0), in ? y[u] : 0.0, s);
    }
  }
  return s;
}

// s -= sum_{k < k1} x[k]^2 and t -= sum_{k < k1} y[k] x[k] together (two chains in flight)
__device__ __forceinline__ void tiny_dot2(double& s, double& t, const double* x, const double* y, int k1) {
  for (int c = 0; c < k1; c += 8) {
    double xv[8], yv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      xv[u] = x[c + u];
      yv[u] = y[c + u];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const bool in = c + u < k1;
      const double xm = in ? xv[u] : 0.0;
      s = fma(-xm, xm, s);
      t = fma(-(in ? yv[u] : 0.0), xm, t);
    }
  }
}

typedef double tiny_d4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ tiny_d4 tiny_mfma(double a, double b, tiny_d4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// A helper workgroup (blockIdx 1 .. TINY_NH): wave w of helper h owns lower block b = 4h + w
// = (bi, bj) of the 16 x 16 grid.  First its 256 entries of the K-build (k_pairs' training
// mode, in the MFMA accumulator layout: lane -> rows 16 bi + lane / 16 + 4 r, column
// 16 bj + lane % 16), written to K and their exp(-s) kept; then, once workgroup 0 has
// published W, M(bi, bj) = X^T X - W W^T (MFMA, X and W from L2) contracted into the d + 3
// sums; each helper's partial sums go to the host.
template <int DM>
__device__ void tiny_helper(const TinyArgs& a, double* lds) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = blockIdx.x - 1;
  const int m16 = lane & 15, k4 = lane >> 4;
  const int n = a.n, d = a.d, P = a.P;
  int bi = 0;
  const int b = 4 * h + wave;
  while ((bi + 1) * (bi + 2) / 2 <= b) ++bi;
  const int bj = b - bi * (bi + 1) / 2;
  const int j = 16 * bj + m16;
  auto coord = [&](int i, int k) { return (k < d && i < n) ? a.X[i * d + k] * a.invd[k] : 0.0; };
  double xj[DM];
#pragma unroll
  for (int k = 0; k < DM; ++k) xj[k] = coord(j, k);
  double xi[4][DM];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int k = 0; k < DM; ++k) xi[r][k] = coord(16 * bi + k4 + 4 * r, k);
  double ex[4];
  {
    const double pre = a.s2 * a.coff;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = 16 * bi + k4 + 4 * r;
      double s = 0.0;
#pragma unroll
      for (int k = 0; k < DM; ++k) {
        const double df = xi[r][k] - xj[k];
        s = fma(df, df, s);
      }
      ex[r] = exp(-s);
      double v = pre * ex[r];
      const bool pad = i >= n || j >= n;
      const bool diag = i == j;
      double vd = a.s2 * a.cdiag;
      if (a.r && i < n) vd += a.rscale * a.r[i];
      v = pad ? (diag ? 1.0 : 0.0) : (diag ? vd : v);
      if (i >= j) tiny_st(a.K + db_blk(bi, bj) + db_e(i & 15, m16), v);
    }
  }
  tiny_signal(&a.sync[0], 0);
  if (!a.want_grad) return;
  int* st = reinterpret_cast<int*>(lds);
  const auto rXp = tiny_rsrc(a.Xp), rWg = tiny_rsrc(a.Wg);
  // M(bi, bj) = X^T X (as soon as workgroup 0 has published X) - W W^T (once W is out)
  if (tiny_wait(&a.sync[1], a.eg, a.abort_flag, st, h == a.dbg_skip) != 1) return;
  tiny_d4 acc = {0.0, 0.0, 0.0, 0.0};
  {
    double av[8][4], bv[8][4];   // X's blocks (kb, bi) and (kb, bj): 4 operands per lane each
#pragma unroll
    for (int kb = 0; kb < 8; ++kb)
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        // X(16 kb + k, 16 bi + m) (zero above the diagonal of a diagonal block)
        const int k = 4 * s + k4;
        // (every load unconditional, so they issue back to back; out-of-range blocks read block 0)
        const bool ia = kb >= bi && !(kb == bi && k < m16), ib = kb >= bi && !(kb == bj && k < m16);
        const double va = tiny_bld(rXp, (kb >= bi ? db_blk(kb, bi) : 0) + db_e(k, m16));
        const double vb = tiny_bld(rXp, (kb >= bi ? db_blk(kb, bj) : 0) + db_e(k, m16));
        av[kb][s] = ia ? va : 0.0;
        bv[kb][s] = ib ? vb : 0.0;
      }
#pragma unroll
    for (int kb = 0; kb < 8; ++kb)
      if (kb >= bi)
#pragma unroll
        for (int s = 0; s < 4; ++s) acc = tiny_mfma(av[kb][s], bv[kb][s], acc);
  }
  if (tiny_wait(&a.sync[2], a.eg, a.abort_flag, st) != 1) return;   // (aborted: Q failed)
  {
    const int ks = (P + 3) >> 2;
    double av[8], bv[8];
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const double va = tiny_bld(rWg, (16 * bi + m16) * 32 + 4 * s + k4), vb = tiny_bld(rWg, (16 * bj + m16) * 32 + 4 * s + k4);
      av[s] = s < ks ? -va : 0.0;
      bv[s] = s < ks ? vb : 0.0;
    }
#pragma unroll
    for (int s = 0; s < 8; ++s)
      if (s < ks) acc = tiny_mfma(av[s], bv[s], acc);
  }
  TinySums<DM> sm;
  sm.zero();
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = 16 * bi + k4 + 4 * r;
    const bool ok = i < n && j < n && i >= j;
    const double m = ok ? acc[r] : 0.0;
    const bool dg = i == j;
    double df2[DM];
#pragma unroll
    for (int k = 0; k < DM; ++k) {
      const double df = xi[r][k] - xj[k];
      df2[k] = df * df;
    }
    sm.t += dg ? m : 0.0;
    sm.r += (dg && ok && a.rdiag) ? m * a.rdiag[i] : 0.0;
    const double me = dg ? 0.0 : m * ex[r];
    sm.e += me;
#pragma unroll
    for (int k = 0; k < DM; ++k) sm.acc[k] = fma(me, df2[k], sm.acc[k]);
  }
  double* red = lds + 8;   // (past st)
  sm.reduce(d, red, red + 4 * (DM + 3));
  // this helper's partial sums straight to the host, which adds the nine in helper order,
  // then the call's tag (the host refuses a helper whose slot does not carry it)
  if (tid < d + 3) a.small[P * P + 2 + d + 4 + h * 64 + tid] = red[4 * (DM + 3) + tid];
  if (tid == 0) a.small[P * P + 2 + d + 4 + h * 64 + 63] = a.tag;
#ifdef TINY_TIMING
  if (tid == 0) atomicMax(&tiny_tsc[7], wall_clock64());
#endif
}

template <int DM>
static __global__ void __launch_bounds__(256) k_tiny(TinyArgs a) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  if (blockIdx.x > 0) {
    tiny_helper<DM>(a, lds);
    return;
  }
  constexpr int ZP = TINY_ZP;
  double* lb = lds;                              // db_factor_invert's image + extras
  double* r1 = lds + G_LDS_LAUNCH_DOUBLES;       // 128 x ZP: [f H], Y, W
  double* zs = r1 + TILE * ZP;                   // 128 x ZP: Z, the q x q algebra
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int m16 = lane & 15, k4 = lane >> 4;     // MFMA operand lane -> (row m16, k k4)
  const int n = a.n, d = a.d, P = a.P, q = P - 1;
  const int npb = (P + 15) >> 4;                 // 16-column blocks of [f H]
  TINY_T(0);
  // the scaled points (k_scale_points' product) for the later calls, while the helpers
  // build K
  tiny_stage<TILE * DM / 256>([&](int e) {
    const int i = e / DM, k = e - i * DM;
    return (k < d && i < n) ? a.X[i * d + k] * a.invd[k] : 0.0;
  }, [&](int e, double v) {
    const int i = e / DM, k = e - i * DM;
    if (k < d) a.xw[i * d + k] = v;
  });
  // [f H] -> r1 ([i][p], pitch ZP; columns P .. 16 npb zero), also while the helpers build K
  tiny_stage<TILE * TINY_DM / 256>([&](int e) {
    const int i = e / TINY_DM, p = e - i * TINY_DM;
    return p < P ? a.F[i + p * TILE] : 0.0;
  }, [&](int e, double v) { r1[(e / TINY_DM) * ZP + e % TINY_DM] = v; });
  TINY_T(1);
  {
    if (tiny_wait(&a.sync[0], TINY_NH * a.ek, a.abort_flag, reinterpret_cast<int*>(zs)) != 1) {   // (never expected)
      if (tid == 0) a.small[P * P + 1] = -1.0;   // (tiny_wait raised the abort flag)
      return;
    }
  }
  // the helpers' image of K's lower half (the diagonal blocks' upper entries unused)
  const auto rK = tiny_rsrc(a.K);
  tiny_stage<36 * DB_BS / 256 + 1>([&](int e) { return tiny_bld(rK, min(e, 36 * DB_BS - 1)); },
                                   [&](int e, double v) { if (e < 36 * DB_BS) lb[e] = v; });
  __syncthreads();
  TINY_T(2);
  const int bad = db_factor_invert(lb, a.L, TILE, a.Xo, TILE, a.small + P * P, [] {}, true);
  if (bad) {
    if (tid == 0) {
      a.small[P * P + 1] = (double)bad;
      if (a.abort_flag) atomicCAS(a.abort_flag, 0, bad);
    }
    return;
  }
  TINY_T(3);
  __syncthreads();   // (the assembled image complete)
  // X's element (i, k) from the image; the diagonal blocks hold other values across their
  // diagonal, read as zero (lower: k > i, or as X^T: k < i)
  auto xlo = [&](int bi, int bk, int i, int k) {   // X(16 bi + i, 16 bk + k), lower
    const double v = lb[db_blk(bi, bk) + db_e(i, k)];
    return (bi == bk && k > i) ? 0.0 : v;
  };
  // Z = X F: blocks (bi, bp), wave w rows bi = w and 7 - w (the same k-length, 9 blocks)
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int bi = u ? 7 - wave : wave;
    for (int bp = 0; bp < npb; ++bp) {
      tiny_d4 acc = {0.0, 0.0, 0.0, 0.0};
      for (int kb = 0; kb <= bi; ++kb) {
        double av[4], bv[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          av[s] = xlo(bi, kb, m16, 4 * s + k4);
          bv[s] = r1[(16 * kb + 4 * s + k4) * ZP + 16 * bp + m16];
        }
#pragma unroll
        for (int s = 0; s < 4; ++s) acc = tiny_mfma(av[s], bv[s], acc);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = 16 * bi + k4 + 4 * r, p = 16 * bp + m16;
        zs[i * ZP + p] = acc[r];
        if (p < P) a.Z[i + p * TILE] = acc[r];
      }
    }
  }
  __syncthreads();
  TINY_T(4);
  // Gram (lower pairs p >= q', mirrored); kept in registers for the algebra below
  double gv[3];
  for (int u = 0; u < 3; ++u) {
    const int e = tid + 256 * u;
    gv[u] = 0.0;
    if (e < P * (P + 1) / 2) {
      int p = 0;
      while ((p + 1) * (p + 2) / 2 <= e) ++p;
      const int qq = e - p * (p + 1) / 2;
      double s = 0.0;
      for (int i = 0; i < TILE; ++i) s = fma(zs[i * ZP + p], zs[i * ZP + qq], s);
      a.small[p * P + qq] = s;
      a.small[qq * P + p] = s;
      gv[u] = s;
    }
  }
  if (tid == 0) a.small[P * P + 1] = 0.0;
  TINY_T(5);
  if (!a.want_grad) return;
  // X's image for the helpers (off the chain until here: they need it only some 20 us before W)
  for (int e = tid; e < 36 * DB_BS; e += 256) tiny_st(a.Xp + e, lb[e]);
  tiny_signal(&a.sync[1], a.eg);
  // Y = X^T Z: blocks (bi, bp) over kb >= bi; written over [f H] (read before the barrier
  // above)
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int bi = u ? 7 - wave : wave;
    for (int bp = 0; bp < npb; ++bp) {
      tiny_d4 acc = {0.0, 0.0, 0.0, 0.0};
      for (int kb = bi; kb < 8; ++kb) {
        double av[4], bv[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          av[s] = xlo(kb, bi, 4 * s + k4, m16);   // X^T(16 bi + m, 16 kb + k)
          bv[s] = zs[(16 * kb + 4 * s + k4) * ZP + 16 * bp + m16];
        }
#pragma unroll
        for (int s = 0; s < 4; ++s) acc = tiny_mfma(av[s], bv[s], acc);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) r1[(16 * bi + k4 + 4 * r) * ZP + 16 * bp + m16] = acc[r];
    }
  }
  __syncthreads();   // Z consumed: zs takes the algebra
  TINY_T(8);
  double* G = zs + TY_G;
  double* Qa = zs + TY_Q;
  double* Qd = zs + TY_QD;
  double* bt = zs + TY_B;
  double* t2 = zs + TY_T2;
  for (int u = 0; u < 3; ++u) {
    const int e = tid + 256 * u;
    if (e < P * (P + 1) / 2) {
      int p = 0;
      while ((p + 1) * (p + 2) / 2 <= e) ++p;
      const int qq = e - p * (p + 1) / 2;
      G[p * P + qq] = gv[u];
      G[qq * P + p] = gv[u];
    }
  }
  for (int e = tid; e < TINY_DM * ZP; e += 256) t2[e] = 0.0;
  __syncthreads();
  for (int e = tid; e < 32 * 32; e += 256) {   // Q = G[1:, 1:] (pitch 32)
    const int i = e >> 5, k = e & 31;
    Qa[e] = (i < q && k < q) ? G[(i + 1) * P + k + 1] : 0.0;
  }
  __syncthreads();
  // Cholesky of Q (small_chol's order of terms): column j by the threads of its rows, the
  // pivot by every thread
  for (int j = 0; j < q; ++j) {
    // the pivot's sum (every thread) and row tid's (threads j < tid < q) in one pass
    const int ti = (tid > j && tid < q) ? tid : j;
    double s = Qa[j * 32 + j], t = Qa[ti * 32 + j];
    tiny_dot2(s, t, Qa + j * 32, Qa + ti * 32, j);
    if (!(s > 0.0)) {   // (uniform) H^T A^-1 H not positive definite
      if (tid == 0) {
        a.small[P * P + 2 + d + 3] = 1.0;
        __hip_atomic_store((tiny_gint*)a.abort_flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // helpers stop
      }
      return;
    }
    const double dj = sqrt(s);
    if (tid > j && tid < q) Qa[tid * 32 + j] = t / dj;
    if (tid == 0) Qd[j] = dj;
    __syncthreads();
  }
  TINY_T(9);
  // T2 = [[sqrt(c), 0], [-sqrt(c) beta, Kq^-T]] (small_t2): Kq^-1 one column per lane
  // (small_trinv's forward substitution) into T2(c + 1, 1 + i) = Kq^-1(i, c); then
  // u = Kq^-1 wz, beta = Kq^-T u and quad = zz - |u|^2 (= zz - wz^T Q^-1 wz)
  if (tid < q) {
    const int c = tid;
    double* e = t2 + (c + 1) * ZP + 1;
    for (int i = c; i < q; ++i) e[i] = tiny_dot(i == c ? 1.0 : 0.0, Qa + i * 32, 1, e, 1, c, i) / Qd[i];
  }
  __syncthreads();
  if (tid < q) bt[tid] = -tiny_dot(0.0, t2 + 1 + tid + ZP, ZP, G + P, P, 0, tid + 1);   // u_i
  __syncthreads();
  {
    const double quad = tiny_dot(G[0], bt, 1, bt, 1, 0, q);
    double cfac = 1.0;
    if (a.mucm) {
      const double sig2 = quad / ((double)n - q - 2.0);
      cfac = ((double)n - q) / (sig2 * ((double)n - q - 2.0));
    }
    const double sc = sqrt(cfac);
    if (tid < q) t2[(tid + 1) * ZP] = sc * tiny_dot(0.0, t2 + (tid + 1) * ZP + 1, 1, bt, 1, tid, q);   // -sc beta_i
    if (tid == 0) t2[0] = sc;
  }
  __syncthreads();
  TINY_T(10);
  // W = Y T2 (blocks (bi, bp), wave w rows 2w, 2w + 1), over Y once every wave has read it
  const int ks = (P + 3) >> 2;
  {
    tiny_d4 wacc[2][2];
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int bp = 0; bp < 2; ++bp) {
        wacc[u][bp] = tiny_d4{0.0, 0.0, 0.0, 0.0};
        if (bp < npb)
          for (int s = 0; s < ks; ++s)
            wacc[u][bp] = tiny_mfma(r1[(16 * (2 * wave + u) + m16) * ZP + 4 * s + k4],
                                    t2[(4 * s + k4) * ZP + 16 * bp + m16], wacc[u][bp]);
      }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int bp = 0; bp < 2; ++bp)
        if (bp < npb)
#pragma unroll
          for (int r = 0; r < 4; ++r) r1[(16 * (2 * wave + u) + k4 + 4 * r) * ZP + 16 * bp + m16] = wacc[u][bp][r];
  }
  // W to L2 for the helpers, then the flag
  for (int e = tid; e < TILE * 32; e += 256) {
    const int i = e >> 5, k = e & 31;
    tiny_st(a.Wg + e, k < 16 * npb ? r1[i * ZP + k] : 0.0);
  }
  if (tid == 0) a.small[P * P + 2 + d + 3] = 0.0;
  tiny_signal(&a.sync[2], a.eg);
  TINY_T(6);
}

}  // namespace gpe
