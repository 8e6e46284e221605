// gpemu_tiny.hpp -- the objective of a training set of at most 128 points (one 128 x 128
// tile: the reference's examples, toy-sim's 60 and toysim3D's 100 points) in two one-
// workgroup launches instead of the general path's ~20 small launches and copies.
//
//   k_tiny_factor (before the host's q x q algebra): scaled points, K-build straight into
//     the block-packed LDS image of db_factor_invert, L and X = L^-1 (assembled in LDS),
//     Z = X [f H], the Gram Z^T Z, and with the gradient A^-1 = X^T X (16 x 16 MFMA
//     blocks of X read from LDS); Gram, log|L| and the failure column go to one small
//     buffer the host reads with one copy.
//   k_tiny_grad (after it, T2 from the host): R2 = Z T2, [sqrt(c) alpha, W] = X^T R2 and
//     the contraction <M, E (.) D_k>, <M, E>, tr M, sum M_ii r_i of k_contract over the
//     tile -> d + 3 sums.
// The arithmetic of every quantity is the general path's formula (the K-build's entries
// are k_pairs' to the bit: same scaled coordinates, same fma order, same selects); sums
// over rows run in another order than the MFMA GEMMs, so results agree to rounding.
// Limits: n <= 128, d <= 32, q + 1 <= 32 (the host takes the general path otherwise).
#pragma once

namespace gpe {

constexpr int TINY_DM = 32;   // LDS pitch of the staged coordinates / basis columns

struct TinyArgs {
  const double* X;      // n_pad x d raw points, row-major (rows >= n zero)
  const double* F;      // [f H], 128 x P column-major
  const double* r;      // per-point nugget added on the diagonal (rscale r_i), or null
  double* xw;           // out: scaled points (128 x d)
  double* L;            // out: L (ld 128); with the gradient then A^-1 over it (lower)
  double* Xo;           // out: X = L^-1 (ld 128, zero upper)
  double* Z;            // out: Z = L^-1 [f H] (ld 128, P columns)
  double* small;        // out: Gram (P x P) | log|L| | failed column (0: none)
  int* abort_flag;      // set to the failed column as the general path's Cholesky does
  int n, d, P, want_grad;
  double s2, coff, cdiag, rscale;
  double invd[TINY_DM];
};

template <int DM>
static __global__ void __launch_bounds__(256) k_tiny_factor(TinyArgs a) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  double* lb = lds;                              // db_factor_invert's image + extras
  double* r1 = lds + G_LDS_LAUNCH_DOUBLES;       // 128 x TINY_DM: scaled points, then [f H]
  double* zs = r1 + TILE * TINY_DM;              // 128 x TINY_DM: Z
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // scaled points, zero-padded to DM (k_scale_points' products)
  for (int e = tid; e < TILE * DM; e += 256) {
    const int i = e / DM, k = e - i * DM;
    double v = 0.0;
    if (k < a.d) {
      v = (i < a.n) ? a.X[i * a.d + k] * a.invd[k] : 0.0;
      a.xw[i * a.d + k] = v;
    }
    r1[i * TINY_DM + k] = v;
  }
  __syncthreads();
  // K-build of the lower half into the block-packed image (k_pairs' training mode)
  {
    const int i = tid & (TILE - 1);
    double xi[DM];
#pragma unroll
    for (int k = 0; k < DM; ++k) xi[k] = r1[i * TINY_DM + k];
    const double pre = a.s2 * a.coff;
    const bool row_pad = i >= a.n;
    double vdiag = a.s2 * a.cdiag;
    if (a.r && !row_pad) vdiag += a.rscale * a.r[i];
    for (int c = tid >> 7; c <= i; c += 2) {
      double s = 0.0;
#pragma unroll
      for (int k = 0; k < DM; ++k) {
        const double df = xi[k] - r1[c * TINY_DM + k];
        s = fma(df, df, s);
      }
      double v = pre * exp(-s);
      const bool pad = row_pad || c >= a.n;
      const bool diag = i == c;
      v = pad ? (diag ? 1.0 : 0.0) : (diag ? vdiag : v);
      lb[db_off(i, c)] = v;
    }
  }
  __syncthreads();
  const int bad = db_factor_invert(lb, a.L, TILE, a.Xo, TILE, a.small + a.P * a.P, [] {}, true);
  if (bad) {
    if (tid == 0) {
      a.small[a.P * a.P + 1] = (double)bad;
      if (a.abort_flag) atomicCAS(a.abort_flag, 0, bad);
    }
    return;
  }
  // [f H] -> r1 ([i][p], pitch TINY_DM)
  for (int e = tid; e < TILE * TINY_DM; e += 256) {
    const int i = e / TINY_DM, p = e - i * TINY_DM;
    r1[e] = p < a.P ? a.F[i + p * TILE] : 0.0;
  }
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
      if (p < a.P) a.Z[i + p * TILE] = z[u];
    }
  }
  __syncthreads();
  // Gram (lower pairs p >= q, mirrored)
  for (int e = tid; e < a.P * (a.P + 1) / 2; e += 256) {
    int p = 0;
    while ((p + 1) * (p + 2) / 2 <= e) ++p;
    const int q = e - p * (p + 1) / 2;
    double s = 0.0;
    for (int i = 0; i < TILE; ++i) s = fma(zs[i * TINY_DM + p], zs[i * TINY_DM + q], s);
    a.small[p * a.P + q] = s;
    a.small[q * a.P + p] = s;
  }
  if (tid == 0) a.small[a.P * a.P + 1] = 0.0;
  if (!a.want_grad) return;
  // A^-1 = X^T X over the 36 lower 16 x 16 blocks (bi >= bj): sum over kb >= bi of
  // X(kb, bi)^T X(kb, bj); X's diagonal blocks hold other values above their diagonal in
  // the image, read as zero here.  Written over L (the contraction reads the lower half).
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
      db_gst1(a.L + i + j * TILE, acc[r]);
    }
  }
}

struct TinyGradArgs {
  const double* Ainv;   // 128 x 128 lower (ld 128)
  const double* Xo;     // X = L^-1 (ld 128)
  const double* Z;      // L^-1 [f H] (ld 128)
  const double* T2;     // P x P column-major (small_t2)
  const double* xw;     // scaled points (128 x d)
  const double* rdiag;  // the std kernel's sigma-gradient correction sum_i M_ii r_i, or null
  double* sums;         // out: d + 3 contraction sums (k_contract's order: D_k..., E, tr, r)
  const int* abort_flag;
  int n, d, P;
};

template <int DM>
static __global__ void __launch_bounds__(256) k_tiny_grad(TinyGradArgs a) {
  __shared__ double zs[TILE * TINY_DM];   // Z, then R2
  __shared__ double ws[TILE * TINY_DM];   // Wa = [sqrt(c) alpha, W]
  __shared__ double xs[TILE * DM];
  __shared__ double t2[TINY_DM * TINY_DM];
  __shared__ double xk[32 * TILE];        // 32 rows of X at a time ([kk][j])
  __shared__ double red[4 * (DM + 3)];
  if (a.abort_flag && *a.abort_flag) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int P = a.P, d = a.d;
  for (int e = tid; e < TILE * TINY_DM; e += 256) {
    const int i = e / TINY_DM, p = e - i * TINY_DM;
    zs[e] = p < P ? a.Z[i + p * TILE] : 0.0;
  }
  for (int e = tid; e < TINY_DM * TINY_DM; e += 256) {
    const int q = e / TINY_DM, p = e - q * TINY_DM;   // t2[q][p] = T2(q, p)
    t2[e] = (q < P && p < P) ? a.T2[q + p * P] : 0.0;
  }
  for (int e = tid; e < TILE * DM; e += 256) {
    const int i = e / DM, k = e - i * DM;
    xs[e] = k < d ? a.xw[i * d + k] : 0.0;
  }
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
  __syncthreads();
  // Wa = X^T R2: row j = i of Wa over rows k >= j of X, X staged 32 rows at a time
  // (coalesced: a column's 32 rows are contiguous)
  {
    double w[TINY_DM / 2];
#pragma unroll
    for (int u = 0; u < TINY_DM / 2; ++u) w[u] = 0.0;
    for (int k0 = 0; k0 < TILE; k0 += 32) {
      for (int e = tid; e < 32 * TILE; e += 256) {
        const int kk = e & 31, j = e >> 5;
        xk[kk * TILE + j] = a.Xo[k0 + kk + j * TILE];
      }
      __syncthreads();
      for (int kk = max(0, i - k0); kk < 32; ++kk) {
        const double x = xk[kk * TILE + i];
#pragma unroll
        for (int u = 0; u < TINY_DM / 2; ++u) w[u] = fma(x, zs[(k0 + kk) * TINY_DM + h + 2 * u], w[u]);
      }
      __syncthreads();
    }
#pragma unroll
    for (int u = 0; u < TINY_DM / 2; ++u) ws[i * TINY_DM + h + 2 * u] = w[u];
  }
  __syncthreads();
  // the contraction of k_contract over the tile (columns c = h + 2 u <= i, c < n)
  double xi[DM], acc[DM], wi[TINY_DM];
#pragma unroll
  for (int k = 0; k < DM; ++k) {
    xi[k] = xs[i * DM + k];
    acc[k] = 0.0;
  }
#pragma unroll
  for (int k = 0; k < TINY_DM; ++k) wi[k] = ws[i * TINY_DM + k];
  double accE = 0.0, accT = 0.0, accR = 0.0;
  const double ri = (a.rdiag && i < a.n) ? a.rdiag[i] : 0.0;
  if (i < a.n) {
    const int cend = min(i + 1, a.n);
    for (int c = h; c < cend; c += 2) {
      double mij = a.Ainv[i + c * TILE];
#pragma unroll
      for (int k = 0; k < TINY_DM; ++k) mij = fma(-wi[k], ws[c * TINY_DM + k], mij);
      double df2[DM];
      double s = 0.0;
#pragma unroll
      for (int k = 0; k < DM; ++k) {
        const double df = xi[k] - xs[c * DM + k];
        df2[k] = df * df;
        s += df2[k];
      }
      const bool dg = c == i;
      accT += dg ? mij : 0.0;
      accR += dg ? mij * ri : 0.0;
      const double me = dg ? 0.0 : mij * exp(-s);
      accE += me;
#pragma unroll
      for (int k = 0; k < DM; ++k) acc[k] = fma(me, df2[k], acc[k]);
    }
  }
  const int nv = d + 3;
  for (int k = 0; k < nv; ++k) {
    double v = 0.0;
#pragma unroll
    for (int kk = 0; kk < DM; ++kk)
      if (kk == k) v = acc[kk];
    if (k == d) v = accE;
    if (k == d + 1) v = accT;
    if (k == d + 2) v = accR;
    for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
    if (lane == 0) red[wave * (DM + 3) + k] = v;
  }
  __syncthreads();
  if (tid < nv)
    a.sums[tid] = (red[tid] + red[(DM + 3) + tid]) + (red[2 * (DM + 3) + tid] + red[3 * (DM + 3) + tid]);
}

}  // namespace gpe
