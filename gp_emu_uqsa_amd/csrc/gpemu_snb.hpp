// gpemu_snb.hpp -- the objective of 128 < n <= 512 points (2 to 4 tiles: the reference's
// history-matching waves, noisefit2D's 500 points) in ONE launch, the n <= 128 design of
// gpemu_tiny.hpp carried over tile by tile.
//
// Workgroup 0 runs the chain: for each diagonal tile k, the updated tile into LDS,
// db_factor_invert (L(k,k), X(k,k) = L(k,k)^-1 in LDS), X(k,k) out; at the end the Gram of
// Z = L^-1 [f H] and, with the gradient, the q x q algebra (T2) as in k_tiny.
// SNB_NH helper workgroups (4 waves each) do the rest as 16 x 16 block tasks, one wave per
// task, every product on the fp64 MFMA with all of a task's loads of a k-chunk in flight:
//   K-build (lower tiles; [f H]^T into the augmented rows Zt);
//   per step k: panel L(i,k) = A(i,k) X(k,k)^T for i > k and the augmented row's
//     Z_k^T = Zt(:, k) X(k,k)^T; then the trailing update A(i,j) -= L(i,k) L(j,k)^T,
//     Zt(:, j) -= Z_k^T L(j,k)^T (k < j <= i);
//   with the gradient: X = L^-1 by levels l = i - j (T = sum_m L(i,m) X(m,j), then
//     X(i,j) = -X(i,i) T), W = (X^T Z) T2 by row blocks, and M = X^T X - W W^T block by
//     block, contracted in the accumulators into the d + 3 sums of k_contract (as k_tiny's
//     helpers); each helper's partial sums go to the host, which adds them in helper order.
// Hand-offs as k_tiny's (sc1 stores and loads, a barrier and one lane's counter add or
// flag store): a helper counter hc (each helper workgroup adds 1 per finished phase) and a
// main flag mf; both count up over a context's calls (bases in the arguments).
// X and X^T (Xt) are both kept so every operand load has its 16 lanes on consecutive rows.
// Limits: 128 < n <= 512, d <= 32, q + 1 <= 32.
#pragma once

namespace gpe {

constexpr int SNB_NH = 48;          // helper workgroups
constexpr int SNB_MAXNB = 4;        // tiles
constexpr int SNB_SYNC_INTS = 2;    // hc, mf
// dynamic LDS: workgroup 0's factor image + 2 x 128 x 33 (k_tiny's); a helper's flag, partial
// sums, Y rows (64 + 4 x 16 x 33) and the scaled points (512 x 33 at most)
constexpr int SNB_LDS_DOUBLES = 64 + 4 * 16 * 33 + 512 * 33;
static_assert(SNB_LDS_DOUBLES >= G_LDS_LAUNCH_DOUBLES + 2 * TILE * TINY_ZP, "workgroup 0 fits");
static_assert(SNB_LDS_DOUBLES * 8 <= 160 * 1024, "LDS");

// dev-tool clocks (tools/hip/snb_bench.hip): -DTINY_TIMING.  Workgroup 0: [4k .. 4k+3] step k's
// wait begin / tile in LDS / factor done / X published, [16..18] Gram wait done / Gram done /
// T2 published; helpers: [20 + p] the latest end of helper phase p.
#ifdef TINY_TIMING
__device__ unsigned long long snb_tsc[48];
#define SNB_T(s) do { __syncthreads(); if (threadIdx.x == 0) snb_tsc[s] = wall_clock64(); } while (0)
#define SNB_TH(p) do { if (threadIdx.x == 0) atomicMax(&snb_tsc[20 + (p)], wall_clock64()); } while (0)
#else
#define SNB_T(s) do {} while (0)
#define SNB_TH(p) do {} while (0)
#endif

struct SnbArgs {
  const double* X;      // raw points, n_pad x d row-major (rows >= n zero)
  const double* F;      // [f H], n_pad x P column-major (rows >= n zero)
  const double* r;      // per-point nugget added on the diagonal (rscale r_i), or null
  const double* rdiag;  // the std kernel's sigma-gradient r, or null
  double* xw;           // out: scaled points (n_pad x d)
  double* A;            // n_pad^2 (ld np): K-build, updated tiles; then X = L^-1 (lower tiles)
  double* Lb;           // n_pad^2 (ld np): L (lower tiles); T^T of the X levels (upper tiles)
  double* Xt;           // n_pad^2 (ld np): X^T
  double* Zt;           // 32 x n_pad (ld 32): [f H]^T, updated by the steps
  double* Zo;           // 32 x n_pad (ld 32): Z^T = (L^-1 [f H])^T
  double* Wg;           // n_pad x 32 row-major: W
  double* T2g;          // 32 x 33: T2 (row k, column p) from workgroup 0
  double* Xscr;         // 128 x 128: db_factor_invert's own X stores (read by nobody)
  double* small;        // out (pinned host memory): Gram (P x P) | log|L(k,k)| (NB) | failed
                        // column | (d + 3) | Q not PD | the helpers' partial sums (SNB_NH x 64,
                        // slot 63 of each: the call's tag once the helper's sums are in)
  int* sync;            // [0] hc, [1] mf (count up over calls)
  int* abort_flag;      // zero on entry; a wait that runs out raises it (GEMM_WAIT_TIMEOUT)
  int n, np, NB, d, P, want_grad, mucm;
  int dbg_skip;         // dev switch (tests): this helper gives up its first wait; else -1
  double tag;           // this call's tag (never repeats in a context) for the helpers' sums
  int hcb, mfb;         // the counters' values before this call (hc in phases)
  double s2, coff, cdiag, rscale;
  double invd[32];
};

// acc += sum over k in [k0, k1) of A(m16, k) B(k, m16) (this lane's operands from fa / fb),
// 4 SNB_CH k (2 SNB_CH loads per lane) in flight at a time: every load unconditional (past k1
// it reads k1 - 1 and is dropped), so they issue back to back; k0, k1 multiples of 4
#ifndef SNB_CH
#define SNB_CH 16
#endif
template <class FA, class FB>
__device__ __forceinline__ tiny_d4 snb_mma(tiny_d4 acc, int k0, int k1, FA fa, FB fb) {
  const int k4 = (threadIdx.x & 63) >> 4;
  for (int c = k0; c < k1; c += 4 * SNB_CH) {
    double av[SNB_CH], bv[SNB_CH];
#pragma unroll
    for (int s = 0; s < SNB_CH; ++s) {
      const int k = min(c + 4 * s + k4, k1 - 1);
      av[s] = fa(k);
      bv[s] = fb(k);
    }
#pragma unroll
    for (int s = 0; s < SNB_CH; ++s)
      if (c + 4 * s < k1) acc = tiny_mfma(av[s], bv[s], acc);
  }
  return acc;
}

template <int DM>
__device__ void snb_helper(const SnbArgs& a, double* lds) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int m16 = lane & 15, k4 = lane >> 4;
  const int gw = (blockIdx.x - 1) * 4 + wave, NW = SNB_NH * 4;
  const int n = a.n, d = a.d, P = a.P, NB = a.NB, NBB = 8 * NB;
  const long long np = a.np;
  const int npb = (P + 15) >> 4;
  int* st = reinterpret_cast<int*>(lds);
  const auto rA = tiny_rsrc(a.A), rL = tiny_rsrc(a.Lb), rXt = tiny_rsrc(a.Xt), rZt = tiny_rsrc(a.Zt),
             rZo = tiny_rsrc(a.Zo), rW = tiny_rsrc(a.Wg), rT2 = tiny_rsrc(a.T2g);
  int ph = 0;   // helper phases finished in this call
  auto next_phase = [&]() {
    tiny_signal(&a.sync[0], 0);   // (add 1)
    SNB_TH(ph);
    ++ph;
  };
  // (a wait that runs out raises the abort flag: every other waiter stops, workgroup 0
  // reports the call as failed, and this helper's sums never carry the call's tag)
  const bool skip = (int)blockIdx.x - 1 == a.dbg_skip;
  auto wait_hc = [&]() { return tiny_wait(&a.sync[0], (a.hcb + ph) * SNB_NH, a.abort_flag, st) == 1; };
  auto wait_mf = [&](int v) { return tiny_wait(&a.sync[1], a.mfb + v, a.abort_flag, st, skip && v == 1) == 1; };
  // the scaled points (k_scale_points' product) staged in LDS once per workgroup (rows of
  // DM + 1 doubles, zero past d and n): the K-build's and the contraction's coordinates
  double* xs = lds + 64 + 4 * 16 * 33;   // (past st, red and the W phase's Y rows)
  constexpr int XP = DM + 1;
  for (int e = tid; e < (int)np * DM; e += 256) {
    const int i = e / DM, k = e - i * DM;
    xs[i * XP + k] = (k < d && i < n) ? a.X[i * d + k] * a.invd[k] : 0.0;
  }
  __syncthreads();
  auto coord = [&](int i, int k) { return xs[i * XP + k]; };
  auto tri = [](int t, int& bi, int& bj) {
    bi = 0;
    while ((bi + 1) * (bi + 2) / 2 <= t) ++bi;
    bj = t - bi * (bi + 1) / 2;
  };
  // ---- K-build (lower blocks), [f H]^T into Zt, the scaled points
  {
    const double pre = a.s2 * a.coff;
    for (int t = gw; t < NBB * (NBB + 1) / 2; t += NW) {
      int bi, bj;
      tri(t, bi, bj);
      // lane rows i = 16 bi + lane % 16 (a store instruction writes 128-byte column runs),
      // columns j = 16 bj + lane / 16 + 4 r
      const int i = 16 * bi + m16;
      double xi[DM], xj[4][DM];   // (every coordinate load before the first store)
#pragma unroll
      for (int k = 0; k < DM; ++k) xi[k] = coord(i, k);
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int k = 0; k < DM; ++k) xj[r][k] = coord(16 * bj + k4 + 4 * r, k);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int j = 16 * bj + k4 + 4 * r;
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < DM; ++k) {
          const double df = xi[k] - xj[r][k];
          s = fma(df, df, s);
        }
        double v = pre * exp(-s);
        const bool pad = i >= n || j >= n;
        const bool diag = i == j;
        double vd = a.s2 * a.cdiag;
        if (a.r && i < n) vd += a.rscale * a.r[i];
        v = pad ? (diag ? 1.0 : 0.0) : (diag ? vd : v);
        if (i >= j) tiny_st(a.A + i + j * np, v);
      }
    }
    for (long long e = (long long)gw * 64 + lane; e < 32 * np; e += (long long)NW * 64) {
      const int p = (int)(e & 31), i = (int)(e >> 5);
      tiny_st(a.Zt + e, p < P ? a.F[i + p * np] : 0.0);
    }
    for (long long e = (long long)gw * 64 + lane; e < np * d; e += (long long)NW * 64) {
      const int i = (int)(e / d), k = (int)(e - (long long)i * d);
      a.xw[e] = xs[i * XP + k];
    }
    next_phase();
  }
  for (int k = 0; k < NB; ++k) {
    // ---- panel k: L(i, k) = A(i, k) X(k,k)^T (i > k), Z_k^T = Zt(:, k) X(k,k)^T
    if (!wait_mf(k + 1)) return;
    {
      const long long c0 = 128ll * k;
      const int nreg = (NB - 1 - k) * 64, ntask = nreg + npb * 8;
      for (int t = gw; t < ntask; t += NW) {
        const bool aug = t >= nreg;
        const int tt = aug ? t - nreg : t;
        const int bc = tt & 7, br = aug ? tt >> 3 : (tt & 63) >> 3, i = aug ? 0 : k + 1 + (tt >> 6);
        // the transposed product X(k,k) A(i,k)^T: acc[r] = L(i,k)(16 br + lane % 16, 16 bc +
        // lane / 16 + 4 r), so each store writes 128-byte column runs
        tiny_d4 acc = {0.0, 0.0, 0.0, 0.0};
        auto fa = [&](int kk) { return tiny_bld(rA, (c0 + 16 * bc + m16) + (c0 + kk) * np); };   // X(k,k)(c, kk)
        if (aug)
          acc = snb_mma(acc, 0, 16 * bc + 16, fa, [&](int kk) { return tiny_bld(rZt, (16 * br + m16) + 32 * (c0 + kk)); });
        else
          acc = snb_mma(acc, 0, 16 * bc + 16, fa, [&](int kk) { return tiny_bld(rA, (128ll * i + 16 * br + m16) + (c0 + kk) * np); });
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const long long col = c0 + 16 * bc + k4 + 4 * r;
          if (aug) tiny_st(a.Zo + (16 * br + m16) + 32 * col, acc[r]);
          else tiny_st(a.Lb + (128ll * i + 16 * br + m16) + col * np, acc[r]);
        }
      }
    }
    next_phase();
    // ---- update k: A(i, j) -= L(i,k) L(j,k)^T, Zt(:, j) -= Z_k^T L(j,k)^T  (k < j <= i)
    if (k < NB - 1) {
      if (!wait_hc()) return;
      const long long c0 = 128ll * k;
      int pairs = 0;
      for (int j = k + 1; j < NB; ++j) pairs += NB - j;
      const int nreg = pairs * 64, ntask = nreg + (NB - 1 - k) * npb * 8;
      for (int t = gw; t < ntask; t += NW) {
        const bool aug = t >= nreg;
        int i = 0, j = 0, br, bc;
        if (!aug) {
          int q = t >> 6;
          for (j = k + 1; q >= NB - j; ++j) q -= NB - j;
          i = j + q;
          br = (t & 63) >> 3;
          bc = t & 7;
          if (i == j && br < bc) continue;   // (upper half of a diagonal tile)
        } else {
          const int tt = t - nreg;
          j = k + 1 + tt / (npb * 8);
          br = (tt % (npb * 8)) >> 3;
          bc = tt & 7;
        }
        // transposed as the panel's: acc[r] = (L(i,k) L(j,k)^T)(16 br + lane % 16, 16 bc + lane / 16 + 4 r)
        double old[4];   // (the block's current values, loaded beside the product's operands)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const long long col = 128ll * j + 16 * bc + k4 + 4 * r;
          old[r] = aug ? tiny_bld(rZt, (16 * br + m16) + 32 * col) : tiny_bld(rA, (128ll * i + 16 * br + m16) + col * np);
        }
        tiny_d4 acc = {0.0, 0.0, 0.0, 0.0};
        auto fa = [&](int kk) { return tiny_bld(rL, (128ll * j + 16 * bc + m16) + (c0 + kk) * np); };   // L(j,k)(c, kk)
        if (aug)
          acc = snb_mma(acc, 0, 128, fa, [&](int kk) { return tiny_bld(rZo, (16 * br + m16) + 32 * (c0 + kk)); });
        else
          acc = snb_mma(acc, 0, 128, fa, [&](int kk) { return tiny_bld(rL, (128ll * i + 16 * br + m16) + (c0 + kk) * np); });
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const long long col = 128ll * j + 16 * bc + k4 + 4 * r;
          const long long o = aug ? (16 * br + m16) + 32 * col : (128ll * i + 16 * br + m16) + col * np;
          tiny_st((aug ? a.Zt : a.A) + o, old[r] - acc[r]);
        }
      }
      next_phase();
    }
    // ---- with the gradient, row k of X = L^-1 below the diagonal while workgroup 0 factors the
    // next tile (every X(m, j), m < k, is out by now): T(k, j) = sum_{m = j}^{k-1} L(k, m) X(m, j),
    // stored transposed in Lb's upper tile (j, k), then X(k, j) = -X(k, k) T(k, j)
    if (a.want_grad && k > 0) {
      const int i = k;
      if (!wait_hc()) return;
      for (int t = gw; t < k * 64; t += NW) {
        const int j = t >> 6, br = (t & 63) >> 3, bc = t & 7;
        tiny_d4 acc = {0.0, 0.0, 0.0, 0.0};
        acc = snb_mma(acc, 128 * j + 16 * bc, 128 * i,   // (X(m, j) is zero above X(j, j)'s diagonal blocks)
                      [&](int kk) { return tiny_bld(rL, (128ll * i + 16 * br + m16) + (long long)kk * np); },
                      [&](int kk) { return tiny_bld(rXt, (128ll * j + 16 * bc + m16) + (long long)kk * np); });
#pragma unroll
        for (int r = 0; r < 4; ++r)
          tiny_st(a.Lb + (128ll * j + 16 * bc + m16) + (128ll * i + 16 * br + k4 + 4 * r) * np, acc[r]);
      }
      next_phase();
      if (!wait_hc()) return;
      for (int t = gw; t < k * 64; t += NW) {
        const int j = t >> 6, br = (t & 63) >> 3, bc = t & 7;
        tiny_d4 acc = {0.0, 0.0, 0.0, 0.0};
        acc = snb_mma(acc, 0, 16 * br + 16,
                      [&](int kk) { return tiny_bld(rA, (128ll * i + 16 * br + m16) + (128ll * i + kk) * np); },
                      [&](int kk) { return tiny_bld(rL, (128ll * j + 16 * bc + m16) + (128ll * i + kk) * np); });
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const long long row = 128ll * i + 16 * br + k4 + 4 * r, col = 128ll * j + 16 * bc + m16;
          tiny_st(a.A + row + col * np, -acc[r]);
          tiny_st(a.Xt + col + row * np, -acc[r]);
        }
      }
      next_phase();
    }
  }
  if (!a.want_grad) return;
  // ---- W = (X^T Z) T2, one 16-row block per helper workgroup: its four waves split the rows k
  // of the sum X^T Z, the partials are added in wave order in LDS, wave 0 multiplies by T2
  if (!wait_hc() || !wait_mf(NB + 1)) return;
  {
    const int ks = (P + 3) >> 2;
    double* yp = lds + 64;   // the waves' partials, 16 x 33 each
    for (int bj = blockIdx.x - 1; bj < NBB; bj += SNB_NH) {
      const int nkb = NBB - bj, b0 = bj + (wave * nkb) / 4, b1 = bj + ((wave + 1) * nkb) / 4;
      for (int bp = 0; bp < npb; ++bp) {
        tiny_d4 acc = {0.0, 0.0, 0.0, 0.0};
        if (b1 > b0)
          acc = snb_mma(acc, 16 * b0, 16 * b1,
                        [&](int kk) { return tiny_bld(rXt, (16 * bj + m16) + (long long)kk * np); },
                        [&](int kk) { return tiny_bld(rZo, (16 * bp + m16) + 32ll * kk); });
#pragma unroll
        for (int r = 0; r < 4; ++r) yp[wave * 528 + (k4 + 4 * r) * 33 + 16 * bp + m16] = acc[r];
      }
      __syncthreads();
      if (wave == 0) {
        for (int e = lane; e < 16 * 32; e += 64) {
          const int o = (e >> 5) * 33 + (e & 31);
          if ((e & 31) < 16 * npb) yp[o] = ((yp[o] + yp[528 + o]) + yp[2 * 528 + o]) + yp[3 * 528 + o];
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);   // (lgkmcnt(0): the wave's LDS stores landed)
        __builtin_amdgcn_wave_barrier();
        for (int bq = 0; bq < npb; ++bq) {
          tiny_d4 acc = {0.0, 0.0, 0.0, 0.0};
          for (int s4 = 0; s4 < ks; ++s4)
            acc = tiny_mfma(yp[m16 * 33 + 4 * s4 + k4], tiny_bld(rT2, (4 * s4 + k4) * 33 + 16 * bq + m16), acc);
#pragma unroll
          for (int r = 0; r < 4; ++r) tiny_st(a.Wg + (16 * bj + k4 + 4 * r) * 32 + 16 * bq + m16, acc[r]);
        }
      }
      __syncthreads();   // (yp reused by the next block)
    }
    next_phase();   // (W's columns past 16 npb are never read: 4 ceil(P / 4) <= 16 npb)
  }
  // ---- M = X^T X - W W^T by lower 16 x 16 blocks, contracted in place.  The contraction is
  // linear in M, so a block's sum over k is split into pieces of <= SNB_PK rows, each piece
  // contracted on its own (the -W W^T part rides with piece 0): a task is one piece, and no
  // wave waits for more than two chunks of loads per task
  if (!wait_hc()) return;
  TinySums<DM> sm;
  sm.zero();
  {
    constexpr int SNB_PK = 128;
    const int ks = (P + 3) >> 2;
    const int nbv = (n + 15) >> 4;   // blocks holding a valid row
    auto npc = [&](int bi) { return ((int)np - 16 * bi + SNB_PK - 1) / SNB_PK; };
    int ntask = 0;
    for (int bi = 0; bi < nbv; ++bi) ntask += (bi + 1) * npc(bi);
    // (tasks in block-row order, i.e. of decreasing length, dealt snake-wise over the rounds)
    for (int round = 0; round * NW < ntask; ++round) {
      int t = round * NW + ((round & 1) ? NW - 1 - gw : gw);
      if (t >= ntask) continue;
      int bi = 0;
      while (t >= (bi + 1) * npc(bi)) {
        t -= (bi + 1) * npc(bi);
        ++bi;
      }
      const int bj = t / npc(bi), pc = t - bj * npc(bi);
      const int k0 = 16 * bi + pc * SNB_PK, k1 = min(k0 + SNB_PK, (int)np);
      tiny_d4 acc = {0.0, 0.0, 0.0, 0.0};
      acc = snb_mma(acc, k0, k1,
                    [&](int kk) { return tiny_bld(rXt, (16 * bi + m16) + (long long)kk * np); },
                    [&](int kk) { return tiny_bld(rXt, (16 * bj + m16) + (long long)kk * np); });
      if (pc == 0)
        acc = snb_mma(acc, 0, 4 * ks, [&](int kk) { return -tiny_bld(rW, (16 * bi + m16) * 32 + kk); },
                      [&](int kk) { return tiny_bld(rW, (16 * bj + m16) * 32 + kk); });
      const int j = 16 * bj + m16;
      double xj[DM];
#pragma unroll
      for (int k = 0; k < DM; ++k) xj[k] = coord(j, k);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = 16 * bi + k4 + 4 * r;
        const bool ok = i < n && j < n && i >= j;
        const double m = ok ? acc[r] : 0.0;
        const bool dg = i == j;
        double df2[DM], s = 0.0;
#pragma unroll
        for (int k = 0; k < DM; ++k) {
          const double df = coord(i, k) - xj[k];
          df2[k] = df * df;
          s += df2[k];
        }
        sm.t += dg ? m : 0.0;
        sm.r += (dg && ok && a.rdiag) ? m * a.rdiag[i] : 0.0;
        const double me = dg ? 0.0 : m * exp(-s);
        sm.e += me;
#pragma unroll
        for (int k = 0; k < DM; ++k) sm.acc[k] = fma(me, df2[k], sm.acc[k]);
      }
    }
  }
  const int h = blockIdx.x - 1;
  double* red = lds + 8;
  sm.reduce(d, red, red + 4 * (DM + 3));
  // this helper's partial sums straight to the host, which adds them in helper order (no
  // cross-workgroup pass on the kernel's tail)
  if (tid < d + 3) a.small[P * P + NB + 1 + d + 4 + h * 64 + tid] = red[4 * (DM + 3) + tid];
  if (tid == 0) a.small[P * P + NB + 1 + d + 4 + h * 64 + 63] = a.tag;
}

template <int DM>
static __global__ void __launch_bounds__(256) k_snb(SnbArgs a) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  if (blockIdx.x > 0) {
    snb_helper<DM>(a, lds);
    return;
  }
  constexpr int ZP = TINY_ZP;
  double* lb = lds;
  const int tid = threadIdx.x;
  const int n = a.n, d = a.d, P = a.P, q = P - 1, NB = a.NB;
  const long long np = a.np;
  int* st = reinterpret_cast<int*>(lds + G_LDS_LAUNCH_DOUBLES);
  const auto rA = tiny_rsrc(a.A), rZo = tiny_rsrc(a.Zo);
  for (int k = 0; k < NB; ++k) {
    // the step's tile, updated by every earlier step, into the block-packed image
    SNB_T(4 * k);
    // (helper phases up to update k - 1: the K-build, a panel and an update per step, and with
    // the gradient the two X-row phases of steps 1 .. k - 2)
    const int upd = 1 + 2 * k + (a.want_grad ? 2 * max(0, k - 2) : 0);
    if (tiny_wait(&a.sync[0], (a.hcb + upd) * SNB_NH, a.abort_flag, st) != 1) {
      // (a helper's wait ran out, or this one did: the abort flag is up either way; only
      // workgroup 0 itself raises it otherwise, after this loop)
      if (tid == 0) a.small[P * P + NB] = -1.0;
      return;
    }
    const long long c0 = 128ll * k;
    {
      double v[36];
#pragma unroll
      for (int b = 0; b < 36; ++b) {
        const int bi = tiny_tri_row(b), bj = b - bi * (bi + 1) / 2;
        const int i = 16 * bi + (tid & 15), c = 16 * bj + (tid >> 4);
        v[b] = i >= c ? tiny_bld(rA, (c0 + i) + (c0 + c) * np) : 0.0;
      }
#pragma unroll
      for (int b = 0; b < 36; ++b) {
        const int bi = tiny_tri_row(b), bj = b - bi * (bi + 1) / 2;
        lb[db_blk(bi, bj) + db_e(tid & 15, tid >> 4)] = v[b];
      }
    }
    __syncthreads();
    SNB_T(4 * k + 1);
    const int bad = db_factor_invert(lb, a.Lb + c0 + c0 * np, np, a.Xscr, TILE, a.small + P * P + k, [] {}, true);
    if (bad) {
      if (tid == 0) {
        a.small[P * P + NB] = (double)(c0 + bad);
        if (a.abort_flag) atomicCAS(a.abort_flag, 0, (int)(c0 + bad));
      }
      return;
    }
    __syncthreads();
    SNB_T(4 * k + 2);
    // X(k, k) (zero above the diagonal) into A's tile and, with the gradient, into Xt (each
    // store run along consecutive addresses)
    // (the lower 16 x 16 blocks only, the diagonal blocks with their zeros: no reader goes
    // above them)
#pragma unroll
    for (int b = 0; b < 36; ++b) {   // rows along the lanes
      const int bi = tiny_tri_row(b), bj = b - bi * (bi + 1) / 2, il = tid & 15, cl = tid >> 4;
      const double v = lb[db_blk(bi, bj) + db_e(il, cl)];
      tiny_st(a.A + (c0 + 16 * bi + il) + (c0 + 16 * bj + cl) * np, (bi == bj && il < cl) ? 0.0 : v);
    }
    if (a.want_grad)
#pragma unroll
      for (int b = 0; b < 36; ++b) {   // columns along the lanes
        const int bi = tiny_tri_row(b), bj = b - bi * (bi + 1) / 2, il = tid >> 4, cl = tid & 15;
        const double v = lb[db_blk(bi, bj) + db_e(il, cl)];
        tiny_st(a.Xt + (c0 + 16 * bj + cl) + (c0 + 16 * bi + il) * np, (bi == bj && il < cl) ? 0.0 : v);
      }
    tiny_signal(&a.sync[1], a.mfb + k + 1);
    SNB_T(4 * k + 3);
  }
  // the Gram of Z = L^-1 [f H] (Z^T from the last panel) out of LDS
  // (helper phases up to the last panel: as above, and the X rows of steps 1 .. NB - 2)
  if (tiny_wait(&a.sync[0], (a.hcb + 2 * NB + (a.want_grad ? 2 * max(0, NB - 2) : 0)) * SNB_NH, a.abort_flag, st) != 1) {
    if (tid == 0) a.small[P * P + NB] = -1.0;   // (never the previous call's Gram as a success)
    return;
  }
  SNB_T(16);
  // Z^T (P x np) into LDS, rows of np + 1 doubles (the MFMA's 16 operand rows on distinct
  // banks): every load of a thread in flight, then the stores
  const int zp = (int)np + 1;
  double* zl = lds;
  {
    const int tot = P * (int)np;
    double v[64];   // (P np <= 32 x 512)
#pragma unroll
    for (int u = 0; u < 64; ++u) {
      const int e = min(tid + 256 * u, tot - 1), p = e / (int)np, i = e - p * (int)np;
      v[u] = tiny_bld(rZo, p + 32ll * i);
    }
#pragma unroll
    for (int u = 0; u < 64; ++u) {
      const int e = tid + 256 * u, p = e / (int)np, i = e - p * (int)np;
      if (e < tot) zl[p * zp + i] = v[u];
    }
  }
  __syncthreads();
  // the Gram Z^T Z on the MFMA: wave w its 16 x 16 block (w / 2, w % 2) of the (<= 32)^2; with
  // one block (P <= 16) the four waves take a quarter of the rows each, added in wave order
  const int lane = tid & 63, wave = tid >> 6, m16 = lane & 15, k4 = lane >> 4;
  const int npb = (P + 15) >> 4;
  const int gp = npb == 1 ? 0 : wave >> 1, gq = npb == 1 ? 0 : wave & 1;
  const int gk0 = npb == 1 ? wave * (int)np / 4 : 0, gk1 = npb == 1 ? (wave + 1) * (int)np / 4 : (int)np;
  tiny_d4 gacc = {0.0, 0.0, 0.0, 0.0};
  if (gp < npb && gq < npb) {
    const int pa = min(16 * gp + m16, P - 1), pb = min(16 * gq + m16, P - 1);   // (rows past P: dropped)
    for (int kk = gk0; kk < gk1; kk += 16) {
      double av[4], bv[4];
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) {
        av[s4] = zl[pa * zp + kk + 4 * s4 + k4];
        bv[s4] = zl[pb * zp + kk + 4 * s4 + k4];
      }
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) gacc = tiny_mfma(av[s4], bv[s4], gacc);
    }
  }
  if (npb == 1) {   // the four quarters, added in wave order
    double* gr = lds + 32 * 513;   // (past Z^T)
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 4; ++r) gr[wave * 256 + r * 64 + lane] = gacc[r];
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int o = r * 64 + lane;
      gacc[r] = ((gr[o] + gr[256 + o]) + gr[512 + o]) + gr[768 + o];
    }
  }
  if (gp < npb && gq < npb && (npb > 1 || wave == 0))
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int p = 16 * gp + k4 + 4 * r, qq = 16 * gq + m16;
      if (p < P && qq < P) a.small[p * P + qq] = gacc[r];
    }
  if (tid == 0) a.small[P * P + NB] = 0.0;
  SNB_T(17);
  if (!a.want_grad) return;
  __syncthreads();   // (Z^T read by every wave)
  // the q x q algebra (as k_tiny's) in LDS (Z^T consumed)
  double* zs = lds;
  double* G = zs + TY_G;
  double* Qa = zs + TY_Q;
  double* Qd = zs + TY_QD;
  double* bt = zs + TY_B;
  double* t2 = zs + TY_T2;
  if (gp < npb && gq < npb && (npb > 1 || wave == 0))
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int p = 16 * gp + k4 + 4 * r, qq = 16 * gq + m16;
      if (p < P && qq < P) G[p * P + qq] = gacc[r];
    }
  for (int e = tid; e < TINY_DM * ZP; e += 256) t2[e] = 0.0;
  __syncthreads();
  for (int e = tid; e < 32 * 32; e += 256) {
    const int i = e >> 5, k = e & 31;
    Qa[e] = (i < q && k < q) ? G[(i + 1) * P + k + 1] : 0.0;
  }
  __syncthreads();
  for (int j = 0; j < q; ++j) {
    const int ti = (tid > j && tid < q) ? tid : j;
    double s = Qa[j * 32 + j], t = Qa[ti * 32 + j];
    tiny_dot2(s, t, Qa + j * 32, Qa + ti * 32, j);
    if (!(s > 0.0)) {   // (uniform) H^T A^-1 H not positive definite: the helpers stop
      if (tid == 0) {
        a.small[P * P + NB + 1 + d + 3] = 1.0;
        __hip_atomic_store((tiny_gint*)a.abort_flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      return;
    }
    const double dj = sqrt(s);
    if (tid > j && tid < q) Qa[tid * 32 + j] = t / dj;
    if (tid == 0) Qd[j] = dj;
    __syncthreads();
  }
  if (tid < q) {
    const int c = tid;
    double* e = t2 + (c + 1) * ZP + 1;
    for (int i = c; i < q; ++i) e[i] = tiny_dot(i == c ? 1.0 : 0.0, Qa + i * 32, 1, e, 1, c, i) / Qd[i];
  }
  __syncthreads();
  if (tid < q) bt[tid] = -tiny_dot(0.0, t2 + 1 + tid + ZP, ZP, G + P, P, 0, tid + 1);
  __syncthreads();
  {
    const double quad = tiny_dot(G[0], bt, 1, bt, 1, 0, q);
    double cfac = 1.0;
    if (a.mucm) {
      const double sig2 = quad / ((double)n - q - 2.0);
      cfac = ((double)n - q) / (sig2 * ((double)n - q - 2.0));
    }
    const double sc = sqrt(cfac);
    if (tid < q) t2[(tid + 1) * ZP] = sc * tiny_dot(0.0, t2 + (tid + 1) * ZP + 1, 1, bt, 1, tid, q);
    if (tid == 0) t2[0] = sc;
  }
  __syncthreads();
  for (int e = tid; e < TINY_DM * ZP; e += 256) tiny_st(a.T2g + e, t2[e]);
  if (tid == 0) a.small[P * P + NB + 1 + d + 3] = 0.0;
  tiny_signal(&a.sync[1], a.mfb + NB + 1);
  SNB_T(18);
}

}  // namespace gpe
