// gpemu_tiny.hpp -- the objective of a training set of at most 128 points (one 128 x 128
// tile: the reference's examples, toy-sim's 60 and toysim3D's 100 points) in ONE one-
// workgroup launch instead of the general path's ~20 small launches and copies.
//
// k_tiny, with everything in LDS after the first staging:
//   scaled points; K-build straight into the block-packed LDS image of db_factor_invert
//   (rows i and 127 - i per lane, every wave the same number of entries); L and X = L^-1
//   (assembled in LDS); Z = X [f H] (16 x 16 x 4 fp64 MFMA on X's blocks); the Gram Z^T Z.
//   Value only: stop there (Gram, log|L| and the failed column go to the host, whose q x q
//   algebra gives the LLH).  With the gradient, on: Y = X^T Z (MFMA); the q x q algebra of
//   the host's small_from_gram / small_t2 (Cholesky of Q = H^T A^-1 H one column per
//   barrier, beta and sqrt(c) on one lane, Kq^-1 one column per lane); W = Y T2 =
//   X^T (Z T2) = [sqrt(c) alpha, Kq^-1-scaled L^-T L^-1 H] (MFMA); M = A^-1 - W W^T
//   = X^T X - W W^T in 16 x 16 MFMA blocks, each contracted where it sits in the
//   accumulators into the d + 3 sums of k_contract (<M, E (.) D_k>, <M, E>, tr M,
//   sum M_ii r_i), four entries at a time so their exp chains overlap.
// The host computes the LLH from the Gram with the same small_from_gram as the general
// path, and the gradient from the d + 3 sums with the same small_grad.
// The arithmetic of every quantity is the general path's formula (the K-build's entries
// are k_pairs' to the bit: same scaled coordinates, same fma order, same selects); products
// and sums run in other orders than the general path's GEMMs and k_contract, so results
// agree to rounding.
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
// the q x q algebra in zs once Z is consumed: Gram (P x P), a flag, u, T2 ([k][p], pitch
// TINY_ZP)
constexpr int TY_G = 0, TY_QD = 2048, TY_B = 2080, TY_T2 = 2112;
static_assert(TY_T2 + TINY_DM * TINY_ZP <= 128 * TINY_ZP, "algebra fits in zs");

// dev-tool phase clocks (tools/hip/tiny_bench.hip): -DTINY_TIMING
#ifdef TINY_TIMING
__device__ unsigned long long tiny_tsc[12];
#define TINY_T(s) do { __syncthreads(); if (threadIdx.x == 0) tiny_tsc[s] = wall_clock64(); } while (0)
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
  double* small;        // out: Gram (P x P) | log|L| | failed column | d + 3 sums | Q not PD
  int* abort_flag;      // set to the failed column as the general path's Cholesky does
  int n, d, P, want_grad, mucm;
  double s2, coff, cdiag, rscale;
  double invd[32];
};

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

typedef double tiny_d4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ tiny_d4 tiny_mfma(double a, double b, tiny_d4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

template <int DM>
static __global__ void __launch_bounds__(256) k_tiny(TinyArgs a) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  constexpr int XP = TinyPitch<DM>::v, ZP = TINY_ZP;
  double* lb = lds;                              // db_factor_invert's image + extras
  double* r1 = lds + G_LDS_LAUNCH_DOUBLES;       // 128 x ZP: scaled points, [f H], Y, W
  double* zs = r1 + TILE * ZP;                   // 128 x ZP: Z, the q x q algebra, scaled points
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int m16 = lane & 15, k4 = lane >> 4;     // MFMA operand lane -> (row m16, k k4)
  const int n = a.n, d = a.d, P = a.P, q = P - 1;
  const int npb = (P + 15) >> 4;                 // 16-column blocks of [f H]
  TINY_T(0);
  auto xw_ld = [&](int e) {   // scaled coordinate e = i DM + k (k_scale_points' product)
    const int i = e / DM, k = e - i * DM;
    return (k < d && i < n) ? a.X[i * d + k] * a.invd[k] : 0.0;
  };
  tiny_stage<TILE * DM / 256>(xw_ld, [&](int e, double v) {
    const int i = e / DM, k = e - i * DM;
    r1[i * XP + k] = v;
    if (k < d) a.xw[i * d + k] = v;
  });
  __syncthreads();
  TINY_T(1);
  // K-build of the lower half into the block-packed image (k_pairs' training mode): lane
  // rows ra = lane and rb = 127 - lane, wave g their columns c = g (mod 4) -- 32 or 33
  // entries per lane, KU at a time (their exp chains overlap)
  {
    const int ra = lane, rb = 127 - lane, g = wave;
    double xa[DM], xb[DM];
#pragma unroll
    for (int k = 0; k < DM; ++k) {
      xa[k] = r1[ra * XP + k];
      xb[k] = r1[rb * XP + k];
    }
    const double pre = a.s2 * a.coff;
    double va = a.s2 * a.cdiag, vb = va;
    if (a.r && ra < n) va += a.rscale * a.r[ra];
    if (a.r && rb < n) vb += a.rscale * a.r[rb];
    const int na = ra >= g ? (ra - g) / 4 + 1 : 0;
    const int tot = na + (rb - g) / 4 + 1;
    constexpr int KU = DM <= 16 ? 4 : 2;
    for (int it = 0; it < tot; it += KU) {
      double s[KU];
      int ii[KU], cc[KU];
#pragma unroll
      for (int u = 0; u < KU; ++u) {
        const int t = min(it + u, tot - 1);
        const bool inA = t < na;
        ii[u] = inA ? ra : rb;
        cc[u] = g + 4 * (inA ? t : t - na);
        s[u] = 0.0;
#pragma unroll
        for (int k = 0; k < DM; ++k) {
          const double df = (inA ? xa[k] : xb[k]) - r1[cc[u] * XP + k];
          s[u] = fma(df, df, s[u]);
        }
      }
#pragma unroll
      for (int u = 0; u < KU; ++u) {
        const int i = ii[u], c = cc[u];
        double v = pre * exp(-s[u]);
        const bool pad = i >= n || c >= n;
        const bool diag = i == c;
        v = pad ? (diag ? 1.0 : 0.0) : (diag ? (i == ra ? va : vb) : v);
        if (it + u < tot) lb[db_off(i, c)] = v;
      }
    }
  }
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
  // [f H] -> r1 ([i][p], pitch ZP; columns P .. 16 npb zero)
  tiny_stage<TILE * TINY_DM / 256>([&](int e) {
    const int i = e / TINY_DM, p = e - i * TINY_DM;
    return p < P ? a.F[i + p * TILE] : 0.0;
  }, [&](int e, double v) { r1[(e / TINY_DM) * ZP + e % TINY_DM] = v; });
  __syncthreads();
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
  // The q x q algebra on wave 0, lane i < q holding row i of Q in registers (every loop
  // over columns unrolled to 32, skipped past q): the Cholesky right-looking (each entry's
  // terms in small_chol's order), u = Kq^-1 wz and the rows of Kq^-1 (small_fwd's and
  // small_trinv's order of terms), the column entries passed by shuffles.  Kq^-1 goes to
  // T2(c + 1, 1 + i) = Kq^-1(i, c), u to bt; then beta = Kq^-T u and quad = zz - |u|^2
  // (= zz - wz^T Q^-1 wz) below.
  if (wave == 0) {
    const int i = lane;
    double qr[32];
#pragma unroll
    for (int k = 0; k < 32; ++k) qr[k] = (i < q && k < q) ? G[(i + 1) * P + k + 1] : 0.0;
    bool okq = true;
#pragma unroll
    for (int j = 0; j < 32; ++j) {
      if (j < q && okq) {
        const double piv = __shfl(qr[j], j, 64);
        if (!(piv > 0.0)) okq = false;   // (uniform over the wave)
        const double dj = sqrt(piv);
        const double l = i == j ? dj : (i > j ? qr[j] / dj : 0.0);
        qr[j] = l;
#pragma unroll
        for (int k = j + 1; k < 32; ++k)
          if (k < q) qr[k] = fma(-l, __shfl(l, k, 64), qr[k]);   // (entries k > i: unused)
      }
    }
    double acc = (i < q) ? G[(i + 1) * P] : 0.0, uval = 0.0;
    double xr[32];
#pragma unroll
    for (int c = 0; c < 32; ++c) xr[c] = i == c ? 1.0 : 0.0;
#pragma unroll
    for (int k = 0; k < 32; ++k) {
      if (k < q && okq) {
        const double dk = __shfl(qr[k], k, 64);   // L(k, k)
        const double uk = __shfl(acc / dk, k, 64);
        uval = i == k ? uk : uval;
        acc = fma(-qr[k], uk, acc);
#pragma unroll
        for (int c = 0; c <= k; ++c) {
          if (i == k) xr[c] = xr[c] / dk;
          const double xkc = __shfl(xr[c], k, 64);
          if (i > k) xr[c] = fma(-qr[k], xkc, xr[c]);
        }
      }
    }
    if (i < q) {
      bt[i] = uval;
#pragma unroll
      for (int c = 0; c < 32; ++c)
        if (c <= i) t2[(c + 1) * ZP + 1 + i] = xr[c];
    }
    if (lane == 0) Qd[0] = okq ? 0.0 : 1.0;
  }
  __syncthreads();
  if (Qd[0] != 0.0) {   // (uniform) H^T A^-1 H not positive definite
    if (tid == 0) a.small[P * P + 2 + d + 3] = 1.0;
    return;
  }
  TINY_T(9);
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
  // the scaled points again (pitch XP) in zs
  tiny_stage<TILE * DM / 256>(xw_ld, [&](int e, double v) { zs[(e / DM) * XP + e % DM] = v; });
  __syncthreads();
  TINY_T(6);
  // M = X^T X - W W^T over the 36 lower 16 x 16 blocks (wave w: rows w and 7 - w, all
  // their column blocks: 9 each), each entry (i >= j, both < n) contracted in place
  constexpr int RI = DM <= 16 ? 4 : 1;   // entries contracted together (register budget)
  TinySums<DM> sm;
  sm.zero();
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int bi = u ? 7 - wave : wave;
    if (16 * bi >= n) continue;
    for (int bj = 0; bj <= bi; ++bj) {
      if (16 * bj >= n) break;
      tiny_d4 acc = {0.0, 0.0, 0.0, 0.0};
      for (int kb = bi; kb < 8; ++kb) {
        double av[4], bv[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          av[s] = xlo(kb, bi, 4 * s + k4, m16);
          bv[s] = xlo(kb, bj, 4 * s + k4, m16);
        }
#pragma unroll
        for (int s = 0; s < 4; ++s) acc = tiny_mfma(av[s], bv[s], acc);
      }
      for (int s = 0; s < ks; ++s)
        acc = tiny_mfma(-r1[(16 * bi + m16) * ZP + 4 * s + k4], r1[(16 * bj + m16) * ZP + 4 * s + k4], acc);
      const int j = 16 * bj + m16;
      double xj[DM];
#pragma unroll
      for (int k = 0; k < DM; ++k) xj[k] = zs[j * XP + k];
#pragma unroll
      for (int r0 = 0; r0 < 4; r0 += RI) {
        double df2[RI][DM], s[RI];
#pragma unroll
        for (int rr = 0; rr < RI; ++rr) {
          const int i = 16 * bi + k4 + 4 * (r0 + rr);
          s[rr] = 0.0;
#pragma unroll
          for (int k = 0; k < DM; ++k) {
            const double df = zs[i * XP + k] - xj[k];
            df2[rr][k] = df * df;
            s[rr] += df2[rr][k];
          }
        }
#pragma unroll
        for (int rr = 0; rr < RI; ++rr) {
          const int i = 16 * bi + k4 + 4 * (r0 + rr);
          const bool ok = i < n && j < n && i >= j;
          const double m = ok ? acc[r0 + rr] : 0.0;
          const bool dg = i == j;
          sm.t += dg ? m : 0.0;
          sm.r += (dg && ok && a.rdiag) ? m * a.rdiag[i] : 0.0;
          const double me = dg ? 0.0 : m * exp(-s[rr]);
          sm.e += me;
#pragma unroll
          for (int k = 0; k < DM; ++k) sm.acc[k] = fma(me, df2[rr][k], sm.acc[k]);
        }
      }
    }
  }
  __syncthreads();   // (red below reuses r1)
  sm.reduce(d, r1, a.small + P * P + 2);
  if (tid == 0) a.small[P * P + 2 + d + 3] = 0.0;
  TINY_T(7);
}

}  // namespace gpe
