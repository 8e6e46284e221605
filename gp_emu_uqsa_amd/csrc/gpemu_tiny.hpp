// gpemu_tiny.hpp -- the objective of a training set of at most 128 points (one 128 x 128
// tile: the reference's examples, toy-sim's 60 and toysim3D's 100 points) in two one-
// workgroup launches instead of the general path's ~20 small launches and copies.
//
//   k_tiny_factor (before the host's q x q algebra): scaled points, K-build straight into
//     the block-packed LDS image of db_factor_invert, L and X = L^-1 (assembled in LDS),
//     Z = X [f H], the Gram Z^T Z; with the gradient also A^-1 = X^T X (16 x 16 MFMA blocks
//     of X from LDS), contracted where it sits in the accumulators: its part of the d + 3
//     sums of k_contract (<A^-1, E (.) D_k>, <A^-1, E>, tr A^-1, sum (A^-1)_ii r_i) -- the
//     contraction is linear in M = A^-1 - W W^T, and this part needs nothing from the host.
//     Gram, log|L|, the failed column and those sums go to the host in one copy.
//   k_tiny_grad (after the host's algebra, T2 uploaded): R2 = Z T2, W = [sqrt(c) alpha, W]
//     = X^T R2, and the -W W^T part of the same sums.  The host adds the two parts.
// The arithmetic of every quantity is the general path's formula (the K-build's entries
// are k_pairs' to the bit: same scaled coordinates, same fma order, same selects); sums
// run in other orders than the MFMA GEMMs' and k_contract's, so results agree to rounding.
// Global -> LDS staging issues every load of a thread before its first LDS store (a load /
// store pair per loop iteration put one memory latency per iteration in sequence: the
// first version spent ~90 us per launch there).
// Limits: n <= 128, d <= 32, q + 1 <= 32 (the host takes the general path otherwise).
#pragma once

namespace gpe {

constexpr int TINY_DM = 32;   // LDS pitch of the staged basis columns

struct TinyArgs {
  const double* X;      // n_pad x d raw points, row-major (rows >= n zero)
  const double* F;      // [f H], 128 x P column-major
  const double* r;      // per-point nugget added on the diagonal (rscale r_i), or null
  const double* rdiag;  // the std kernel's sigma-gradient r (sum M_ii r_i), or null
  double* xw;           // out: scaled points (128 x d)
  double* L;            // out: L (ld 128)
  double* Xo;           // out: X = L^-1 (ld 128, zero upper)
  double* Z;            // out: Z = L^-1 [f H] (ld 128, P columns)
  double* small;        // out: Gram (P x P) | log|L| | failed column | A^-1 part of the sums (d + 3)
  int* abort_flag;      // set to the failed column as the general path's Cholesky does
  int n, d, P, want_grad;
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

// k_contract's per-pair work for M(i, j) = m (i >= j): the diagonal to tr and the r sum, an
// off-diagonal pair to <M, E> and <M, E (.) D_k> (xs: scaled points, pitch DM)
template <int DM>
struct TinySums {
  double acc[DM];
  double e, t, r;
  __device__ void zero() {
#pragma unroll
    for (int k = 0; k < DM; ++k) acc[k] = 0.0;
    e = t = r = 0.0;
  }
  __device__ __forceinline__ void pair(double m, const double* xs, int i, int j, double ri) {
    double df2[DM];
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < DM; ++k) {
      const double df = xs[i * DM + k] - xs[j * DM + k];
      df2[k] = df * df;
      s += df2[k];
    }
    const bool dg = i == j;
    t += dg ? m : 0.0;
    r += dg ? m * ri : 0.0;
    const double me = dg ? 0.0 : m * exp(-s);
    e += me;
#pragma unroll
    for (int k = 0; k < DM; ++k) acc[k] = fma(me, df2[k], acc[k]);
  }
  // workgroup sum (fixed order) of the d + 3 values into out[0 .. d+3); red: 4 (DM + 3)
  __device__ void reduce(int d, double* red, double* out) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nv = d + 3;
    for (int k = 0; k < nv; ++k) {
      double v = 0.0;
#pragma unroll
      for (int kk = 0; kk < DM; ++kk)
        if (kk == k) v = acc[kk];
      if (k == d) v = e;
      if (k == d + 1) v = t;
      if (k == d + 2) v = r;
      for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
      if (lane == 0) red[wave * (DM + 3) + k] = v;
    }
    __syncthreads();
    if (tid < nv) out[tid] = (red[tid] + red[(DM + 3) + tid]) + (red[2 * (DM + 3) + tid] + red[3 * (DM + 3) + tid]);
  }
};

template <int DM>
static __global__ void __launch_bounds__(256) k_tiny_factor(TinyArgs a) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  double* lb = lds;                              // db_factor_invert's image + extras
  double* r1 = lds + G_LDS_LAUNCH_DOUBLES;       // 128 x TINY_DM: scaled points, then [f H]
  double* zs = r1 + TILE * TINY_DM;              // 128 x TINY_DM: Z, then the scaled points again
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n = a.n, d = a.d, P = a.P;
  auto xw_ld = [&](int e) {   // scaled coordinate e = i DM + k (k_scale_points' product)
    const int i = e / DM, k = e - i * DM;
    return (k < d && i < n) ? a.X[i * d + k] * a.invd[k] : 0.0;
  };
  tiny_stage<TILE * DM / 256>(xw_ld, [&](int e, double v) {
    const int i = e / DM, k = e - i * DM;
    r1[i * DM + k] = v;
    if (k < d) a.xw[i * d + k] = v;
  });
  __syncthreads();
  // K-build of the lower half into the block-packed image (k_pairs' training mode)
  {
    const int i = tid & (TILE - 1);
    double xi[DM];
#pragma unroll
    for (int k = 0; k < DM; ++k) xi[k] = r1[i * DM + k];
    const double pre = a.s2 * a.coff;
    const bool row_pad = i >= n;
    double vdiag = a.s2 * a.cdiag;
    if (a.r && !row_pad) vdiag += a.rscale * a.r[i];
    for (int c = tid >> 7; c <= i; c += 2) {
      double s = 0.0;
#pragma unroll
      for (int k = 0; k < DM; ++k) {
        const double df = xi[k] - r1[c * DM + k];
        s = fma(df, df, s);
      }
      double v = pre * exp(-s);
      const bool pad = row_pad || c >= n;
      const bool diag = i == c;
      v = pad ? (diag ? 1.0 : 0.0) : (diag ? vdiag : v);
      lb[db_off(i, c)] = v;
    }
  }
  __syncthreads();
  const int bad = db_factor_invert(lb, a.L, TILE, a.Xo, TILE, a.small + P * P, [] {}, true);
  if (bad) {
    if (tid == 0) {
      a.small[P * P + 1] = (double)bad;
      if (a.abort_flag) atomicCAS(a.abort_flag, 0, bad);
    }
    return;
  }
  // [f H] -> r1 ([i][p], pitch TINY_DM)
  tiny_stage<TILE * TINY_DM / 256>([&](int e) {
    const int i = e / TINY_DM, p = e - i * TINY_DM;
    return p < P ? a.F[i + p * TILE] : 0.0;
  }, [&](int e, double v) { r1[e] = v; });
  __syncthreads();
  // Z = X [f H]: thread (row i, half h) accumulates columns h, h + 2, ... over k <= i (X in
  // LDS, lower blocks; the diagonal blocks' lower part)
  {
    const int i = tid & (TILE - 1), h = tid >> 7;
    double z[TINY_DM / 2];
#pragma unroll
    for (int u = 0; u < TINY_DM / 2; ++u) z[u] = 0.0;
    for (int k = 0; k <= i; ++k) {
      const double x = lb[db_off(i, k)];
#pragma unroll
      for (int u = 0; u < TINY_DM / 2; ++u) z[u] = fma(x, r1[k * TINY_DM + h + 2 * u], z[u]);
    }
#pragma unroll
    for (int u = 0; u < TINY_DM / 2; ++u) {
      const int p = h + 2 * u;
      zs[i * TINY_DM + p] = z[u];
      if (p < P) a.Z[i + p * TILE] = z[u];
    }
  }
  __syncthreads();
  // Gram (lower pairs p >= q, mirrored)
  for (int e = tid; e < P * (P + 1) / 2; e += 256) {
    int p = 0;
    while ((p + 1) * (p + 2) / 2 <= e) ++p;
    const int q = e - p * (p + 1) / 2;
    double s = 0.0;
    for (int i = 0; i < TILE; ++i) s = fma(zs[i * TINY_DM + p], zs[i * TINY_DM + q], s);
    a.small[p * P + q] = s;
    a.small[q * P + p] = s;
  }
  if (tid == 0) a.small[P * P + 1] = 0.0;
  if (!a.want_grad) return;
  __syncthreads();   // every Gram read of zs done
  // the scaled points again (pitch DM) in zs
  tiny_stage<TILE * DM / 256>(xw_ld, [&](int e, double v) { zs[e] = v; });
  __syncthreads();
  // A^-1 = X^T X over the 36 lower 16 x 16 blocks (bi >= bj): sum over kb >= bi of
  // X(kb, bi)^T X(kb, bj) (X's diagonal blocks hold other values above their diagonal in
  // the image, read as zero here), each entry (i >= j, both < n) contracted at once
  TinySums<DM> sm;
  sm.zero();
  for (int b = wave; b < 36; b += 4) {
    int bi = 0;
    while ((bi + 1) * (bi + 2) / 2 <= b) ++bi;
    const int bj = b - bi * (bi + 1) / 2;
    d4 acc = d4{0.0, 0.0, 0.0, 0.0};
    for (int kb = bi; kb < 8; ++kb) {
      double av[4], bv[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int k = 4 * s + (lane >> 4), m = lane & 15;
        const double xa = lb[db_blk(kb, bi) + db_e(k, m)];
        const double xb = lb[db_blk(kb, bj) + db_e(k, m)];
        av[s] = (kb == bi && k < m) ? 0.0 : xa;   // X(kb,bi)^T(m, k) = X(16 kb + k, 16 bi + m)
        bv[s] = (kb == bj && k < m) ? 0.0 : xb;
      }
#pragma unroll
      for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[s], bv[s], acc, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = 16 * bi + (lane >> 4) + 4 * r, j = 16 * bj + (lane & 15);
      if (i < n && j < n && i >= j) sm.pair(acc[r], zs, i, j, a.rdiag ? a.rdiag[i] : 0.0);
    }
  }
  __syncthreads();   // (red below reuses r1)
  sm.reduce(d, r1, a.small + P * P + 2);
}

struct TinyGradArgs {
  const double* Xo;     // X = L^-1 (ld 128)
  const double* Z;      // L^-1 [f H] (ld 128)
  const double* T2;     // P x P column-major (small_t2)
  const double* xw;     // scaled points (128 x d)
  const double* rdiag;  // the std kernel's sigma-gradient r, or null
  double* sums;         // out: the -W W^T part of the d + 3 sums
  const int* abort_flag;
  int n, d, P;
};

template <int DM>
static __global__ void __launch_bounds__(256) k_tiny_grad(TinyGradArgs a) {
  __shared__ double zs[TILE * TINY_DM];   // Z, then R2
  __shared__ double ws[TILE * TINY_DM];   // W
  __shared__ double xs[TILE * DM];
  __shared__ double t2[TINY_DM * TINY_DM];
  __shared__ double xk[32 * TILE];        // 32 rows of X at a time ([kk][j]); then the reduction
  if (a.abort_flag && *a.abort_flag) return;
  const int tid = threadIdx.x;
  const int P = a.P, d = a.d, n = a.n;
  tiny_stage<TILE * TINY_DM / 256>([&](int e) {
    const int i = e / TINY_DM, p = e - i * TINY_DM;
    return p < P ? a.Z[i + p * TILE] : 0.0;
  }, [&](int e, double v) { zs[e] = v; });
  tiny_stage<TINY_DM * TINY_DM / 256>([&](int e) {
    const int q = e / TINY_DM, p = e - q * TINY_DM;   // t2[q][p] = T2(q, p)
    return (q < P && p < P) ? a.T2[q + p * P] : 0.0;
  }, [&](int e, double v) { t2[e] = v; });
  tiny_stage<TILE * DM / 256>([&](int e) {
    const int i = e / DM, k = e - i * DM;
    return k < d ? a.xw[i * d + k] : 0.0;
  }, [&](int e, double v) { xs[e] = v; });
  __syncthreads();
  const int i = tid & (TILE - 1), h = tid >> 7;
  // R2 = Z T2 (rows i, columns h, h + 2, ...), in place of Z once every row is read
  double rv[TINY_DM / 2];
#pragma unroll
  for (int u = 0; u < TINY_DM / 2; ++u) {
    const int p = h + 2 * u;
    double s = 0.0;
    for (int q = 0; q < P; ++q) s = fma(zs[i * TINY_DM + q], t2[q * TINY_DM + p], s);
    rv[u] = s;
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < TINY_DM / 2; ++u) zs[i * TINY_DM + h + 2 * u] = rv[u];
  // W = X^T R2: row j = i of W over rows k >= j of X, X staged 32 rows at a time
  // (coalesced: a column's 32 rows are contiguous)
  {
    double w[TINY_DM / 2];
#pragma unroll
    for (int u = 0; u < TINY_DM / 2; ++u) w[u] = 0.0;
    for (int k0 = 0; k0 < TILE; k0 += 32) {
      __syncthreads();   // R2 stored / the previous chunk consumed
      tiny_stage<32 * TILE / 256>([&](int e) { return a.Xo[k0 + (e & 31) + (e >> 5) * TILE]; },
                                  [&](int e, double v) { xk[(e & 31) * TILE + (e >> 5)] = v; });
      __syncthreads();
      for (int kk = max(0, i - k0); kk < 32; ++kk) {
        const double x = xk[kk * TILE + i];
#pragma unroll
        for (int u = 0; u < TINY_DM / 2; ++u) w[u] = fma(x, zs[(k0 + kk) * TINY_DM + h + 2 * u], w[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < TINY_DM / 2; ++u) ws[i * TINY_DM + h + 2 * u] = w[u];
  }
  __syncthreads();
  // the -W W^T part of the contraction (pairs c <= i < n, columns c = h + 2 u)
  TinySums<DM> sm;
  sm.zero();
  if (i < n) {
    double wi[TINY_DM];
#pragma unroll
    for (int k = 0; k < TINY_DM; ++k) wi[k] = ws[i * TINY_DM + k];
    const double ri = a.rdiag ? a.rdiag[i] : 0.0;
    for (int c = h; c <= i; c += 2) {
      double m = 0.0;
#pragma unroll
      for (int k = 0; k < TINY_DM; ++k) m = fma(-wi[k], ws[c * TINY_DM + k], m);
      sm.pair(m, xs, i, c, ri);
    }
  }
  sm.reduce(d, xk, a.sums);
}

}  // namespace gpe
