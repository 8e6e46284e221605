// gpemu_diag.hpp -- 128x128 diagonal-block Cholesky + inverse inside 72 KB of LDS.
//
// Used by the special first workgroup of each trailing-update launch (k_gemm with
// a DIAG tile entry) and by k_potrf_diag_bp for the first block: the factorisation
// of tile (k+1,k+1) then overlaps the rest of the update instead of following it.
//
// LDS: L in block-packed form -- the 36 lower 16x16 blocks (bi >= bk), block
// bi*(bi+1)/2 + bk at DB_BS*blk doubles, column-major inside the block with column j
// shifted by j & 14 (db_e) -- 78,336 B; plus a 2 KB scratch for the current leaf
// inverse.  After L is written out, X = L^-1 is assembled in place of it (X21
// overwrites L21 once T = L21 X11 is in registers) and written out.
//
// Algorithm (16-wide right-looking inside the tile, depth-1 look-ahead):
//   for jb: panel    -- L(ib,jb) = A(ib,jb) X_jb^T   (MFMA, ib > jb)
//           wave 0   -- update block (jb+1,jb+1), then factor + invert it (leaf)
//           waves 1-3-- the rest of A(ib,kb) -= L(ib,jb) L(kb,jb)^T (MFMA)
//   X assembly: X21 = -X22 (L21 X11) at 32, 64, 128 (MFMA, accumulator of T
//   reused as the B fragments of the second product).
#pragma once
#include <hip/hip_runtime.h>

namespace gpe {

typedef double d4 __attribute__((ext_vector_type(4)));

// Element (i, j) of a 16 x 16 block in LDS: column-major with column j shifted by j & 14
// doubles (block stride DB_BS).  The accumulator pattern of the MFMA code (lane ->
// (lane >> 4 + 4 r, lane & 15)) then reads conflict-free and writes 3 LDS cycles per
// 16-lane group instead of 16 (plain column-major: every lane of a ds_write_b64 group on
// one bank, reads 8-way), the operand pattern (lane -> (lane & 15, 4 s + lane >> 4)) stays
// conflict-free, and both stay affine in r and s (immediate offsets, no extra address
// registers); pairs of rows stay 16-byte aligned.
constexpr int DB_BS = 272;
__host__ __device__ constexpr int db_e(int i, int j) { return i + 16 * j + (j & 14); }
constexpr int DB_LDS_DOUBLES = 37 * DB_BS;   // block-packed L + leaf-inverse scratch (same layout)
constexpr int DB_EXTRA_DOUBLES = 128 + 8;        // X diagonal, reduction slots, flag

// dev-tool phase timing (tools/hip/db_bench.hip): -DDB_TIMING
#ifdef DB_TIMING
__device__ unsigned long long db_tsc[8];
// per-thread register accumulators (a global read-modify-write per mark would put
// an HBM round trip inside every interval); slot 7 is timed by wave 1
#define DB_T(slot) do { dbt[slot] += wall_clock64(); } while (0)
#define DB_TN(slot) do { dbt[slot] -= wall_clock64(); } while (0)
#define DB_TDECL unsigned long long dbt[8] = {0, 0, 0, 0, 0, 0, 0, 0}
#define DB_TFLUSH do { if (threadIdx.x == 0 || threadIdx.x == 64) \
    for (int s_ = 0; s_ < 8; ++s_) if ((s_ == 7) == (threadIdx.x == 64)) atomicAdd(&db_tsc[s_], dbt[s_]); } while (0)
#else
#define DB_TDECL do {} while (0)
#define DB_TFLUSH do {} while (0)
#define DB_T(slot) do {} while (0)
#define DB_TN(slot) do {} while (0)
#endif

// global-address-space stores: a FLAT store also counts in lgkmcnt, so the LDS waits
// after it would wait for the store to land
typedef double db_v2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void db_gst2(double* p, double x, double y) {
  *(__attribute__((address_space(1))) db_v2*)(p) = db_v2{x, y};
}
__device__ __forceinline__ void db_gst1(double* p, double x) { *(__attribute__((address_space(1))) double*)(p) = x; }

__device__ __forceinline__ int db_off(int i, int k) {   // i >= k
  const int bi = i >> 4, bk = k >> 4;
  return (bi * (bi + 1) / 2 + bk) * DB_BS + db_e(i & 15, k & 15);
}

__device__ __forceinline__ double db_bcast(double v, int src) {
  const unsigned long long b = __double_as_longlong(v);
  const unsigned lo = __builtin_amdgcn_readlane((unsigned)b, src);
  const unsigned hi = __builtin_amdgcn_readlane((unsigned)(b >> 32), src);
  return __longlong_as_double(((unsigned long long)hi << 32) | lo);
}

__device__ __forceinline__ double db_rsq(double p) {
  double r = __builtin_amdgcn_rsq(p);
  return r * fma(-0.5 * p * r, r, 1.5);
}

__device__ __forceinline__ double db_perm(double v, int src_lane) {
  const unsigned long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_ds_bpermute(src_lane << 2, (int)(unsigned)b);
  const int hi = __builtin_amdgcn_ds_bpermute(src_lane << 2, (int)(unsigned)(b >> 32));
  return __longlong_as_double(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}

// One wave factors and inverts diagonal block jb (16 x 16) with all 64 lanes:
// lane = i + 16 q holds row i of the block at columns k = 4k'+q (a[k']) and rows
// r = 4r'+q of column i of X = L^-1 (xc[r']).  Per column j the owners of column j
// compute L(., j) and two permutes hand every lane its row's multiplier L(i, j) and
// the four L(k, j) it needs; the same values drive the forward substitution of X.
// L -> lower part of the block, X strictly-lower -> upper part transposed
// (X(r,c) at (c,r)), X diagonal -> xdiag, X -> xs.  *flag = 1-based tile column
// of the first bad pivot.
__device__ __forceinline__ void db_leaf(double* lb, double* xs, double* xdiag, int jb, int* flag) {
  const int lane = threadIdx.x & 63;
  const int i = lane & 15, q = lane >> 4;
  const int base = (jb * (jb + 1) / 2 + jb) * DB_BS;
  double a[4], xc[4];
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) {
    const int k = 4 * kk + q;
    a[kk] = (k <= i) ? lb[base + db_e(i, k)] : 0.0;
    xc[kk] = (k == i) ? 1.0 : 0.0;
  }
  int bad = 0;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int qj = j & 3, kj = j >> 2;
    const double piv = db_bcast(a[kj], j + 16 * qj);
    if (!(piv > 0.0) && bad == 0) bad = j + 1;   // wave-uniform; later columns are NaN garbage
    const double r = db_rsq(piv);
    // owners of column j (q == qj): L(i, j) for i >= j, 0 above
    const double v = (i > j) ? a[kj] * r : (i == j ? piv * r : 0.0);
    if (q == qj) a[kj] = (i >= j) ? v : a[kj];
    const double lij = db_perm(v, i + 16 * qj);                  // L(i, j)
    double lk[4];
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) lk[kk] = db_perm(v, 4 * kk + q + 16 * qj);   // L(4kk+q, j)
    if (q == qj) xc[kj] *= r;                                    // X(j, i) final
    const double xji = db_perm(xc[kj], i + 16 * qj);
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const bool below = 4 * kk + q > j;
      const double c = below ? lk[kk] : 0.0;
      a[kk] = fma(-lij, c, a[kk]);
      xc[kk] = fma(-c, xji, xc[kk]);
    }
  }
  if (bad) {
    if (lane == 0) *flag = jb * 16 + bad;
    return;
  }
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) {
    const int k = 4 * kk + q;
    lb[base + db_e(i, k)] = (k <= i) ? a[kk] : xc[kk];   // L lower / X(k,i) at (i,k) upper
    xs[db_e(k, i)] = xc[kk];                             // X(k, i), zero for k < i
    if (k == i) xdiag[jb * 16 + i] = xc[kk];
  }
}

// The same leaf with the column updates on the MFMA pipe.  v_mfma_f64_16x16x4f64(a, b, c)
// gives D(i, j) = c(i, j) + sum_k a[lane i + 16 k] b[lane j + 16 k], D(i, j) held by lane
// j + 16 (i & 3) in register i >> 2.  The symmetric block S sits in that layout (acc), so
// row c of S -- which is column c -- is one register (c >> 2) of one lane group (c & 3),
// indexed by the lane's column j: scaled by rsq(S(c, c)) it is L(j, c), and as the a and b
// operands of one MFMA (every other lane group zero) it is the rank-1 update
// S -= L(., c) L(., c)^T, with no data moved between lanes.  X = L^-1 rides along the same
// way: Y starts as I, X(c, .) = r Y(c, .) and Y -= L(., c) X(c, .) (a second, independent
// MFMA per column).  The pivot chain per column is the MFMA, a readlane of the next pivot,
// rsq + one Newton step and the scaling, against ~325 shader cycles of bpermute round
// trips in db_leaf, and it leaves the LDS to the other waves' trailing update.
// Row c of acc is overwritten by L^T's row (L(j, c), j >= c) and row c of Y by X(c, .),
// so at the end acc's upper triangle is L^T and Y's lower triangle is X.  Same outputs
// as db_leaf.
__device__ __forceinline__ void db_leaf_mfma(double* lb, double* xs, double* xdiag, int jb, int* flag) {
  const int lane = threadIdx.x & 63;
  const int j = lane & 15, q = lane >> 4;
  const int base = (jb * (jb + 1) / 2 + jb) * DB_BS;
  d4 acc, Y;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = q + 4 * r;   // this register's row
    acc[r] = (i >= j) ? lb[base + db_e(i, j)] : lb[base + db_e(j, i)];
    Y[r] = (i == j) ? 1.0 : 0.0;
  }
  int bad = 0;
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    const int k0 = c & 3, rc = c >> 2;
    const double piv = db_bcast(acc[rc], c + 16 * k0);
    if (!(piv > 0.0) && bad == 0) bad = c + 1;   // wave-uniform; later columns are NaN garbage
    const double r = db_rsq(piv);
    const bool mine = q == k0;
    const double u = acc[rc] * r;                  // lane group k0: L(j, c) for j > c
    const double xr = Y[rc] * r;                   // lane group k0: X(c, j)
    const bool act = mine && j > c;
    const double ua = act ? -u : 0.0, ub = act ? u : 0.0;
    const double xb = mine ? xr : 0.0;
    acc[rc] = (mine && j >= c) ? (j == c ? piv * r : u) : acc[rc];   // row c -> L^T
    Y[rc] = mine ? xr : Y[rc];                                        // row c -> X(c, .)
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(ua, ub, acc, 0, 0, 0);
    Y = __builtin_amdgcn_mfma_f64_16x16x4f64(ua, xb, Y, 0, 0, 0);
  }
  if (bad) {
    if (lane == 0) *flag = jb * 16 + bad;
    return;
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int c = q + 4 * r;   // this register's row of acc / Y: L(j, c) or X(c, j)
    lb[base + db_e(j, c)] = (j >= c) ? acc[r] : Y[r];   // L lower / X(c, j) at (j, c), upper
    xs[db_e(c, j)] = Y[r];                              // X(c, j), zero for j > c
    if (j == c) xdiag[jb * 16 + c] = Y[r];
  }
}


// The leaf by 4-column blocks: per block p the 4 x 4 diagonal block is broadcast (its 10
// values by readlane) and factored and inverted by every lane on uniform values (Li =
// L_pp^-1, four dependent rsq's), and everything else is four MFMAs on the accumulator
// layout of db_leaf_mfma.  Rows 4p .. 4p+3 of S are register p of the four lane groups
// (lane j + 16 q holds S(4p + q, j)), so with a[lane i + 16 k] = Li(i - 4p, k) (rows of
// the block only) and b = acc[p]:
//   MFMA(a, acc[p])   = Li S(block rows, .)  -> rows 4p.. of L^T (the block and the panel)
//   MFMA(a, Y[p])     = Li Y(block rows, .)  -> rows 4p.. of X = L^-1
//   S -= P P^T, Y -= P X(block rows, .)     (P = the new acc[p] past the block: the panel)
// Two MFMAs and the 4 x 4 factor per four columns on the pivot chain, against one MFMA
// and a rsq per column in db_leaf_mfma.  Same outputs as db_leaf.
__device__ __forceinline__ void db_leaf_blk(double* lb, double* xs, double* xdiag, int jb, int* flag) {
  const int lane = threadIdx.x & 63;
  const int j = lane & 15, q = lane >> 4;
  const int base = (jb * (jb + 1) / 2 + jb) * DB_BS;
  d4 acc, Y;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = q + 4 * r;   // this register's row
    acc[r] = (i >= j) ? lb[base + db_e(i, j)] : lb[base + db_e(j, i)];
    Y[r] = (i == j) ? 1.0 : 0.0;
  }
  int bad = 0;
  const d4 z4 = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int c0 = 4 * p;
    // S(c0 + k, c0 + l), l <= k: lane c0 + l of group k, register p
    const double a00 = db_bcast(acc[p], c0);
    const double a10 = db_bcast(acc[p], c0 + 16), a11 = db_bcast(acc[p], c0 + 17);
    const double a20 = db_bcast(acc[p], c0 + 32), a21 = db_bcast(acc[p], c0 + 33), a22 = db_bcast(acc[p], c0 + 34);
    const double a30 = db_bcast(acc[p], c0 + 48), a31 = db_bcast(acc[p], c0 + 49), a32 = db_bcast(acc[p], c0 + 50),
                 a33 = db_bcast(acc[p], c0 + 51);
    // 4 x 4 Cholesky (uniform values) and its inverse Li
    if (!(a00 > 0.0) && bad == 0) bad = c0 + 1;
    const double r0 = db_rsq(a00);
    const double l10 = a10 * r0, l20 = a20 * r0, l30 = a30 * r0;
    const double d1 = fma(-l10, l10, a11);
    if (!(d1 > 0.0) && bad == 0) bad = c0 + 2;
    const double r1 = db_rsq(d1);
    const double l21 = fma(-l20, l10, a21) * r1, l31 = fma(-l30, l10, a31) * r1;
    const double d2 = fma(-l21, l21, fma(-l20, l20, a22));
    if (!(d2 > 0.0) && bad == 0) bad = c0 + 3;
    const double r2 = db_rsq(d2);
    const double l32 = fma(-l31, l21, fma(-l30, l20, a32)) * r2;
    const double d3 = fma(-l32, l32, fma(-l31, l31, fma(-l30, l30, a33)));
    if (!(d3 > 0.0) && bad == 0) bad = c0 + 4;
    const double r3 = db_rsq(d3);
    const double i10 = -l10 * r0 * r1;
    const double i21 = -l21 * r1 * r2;
    const double i20 = -(l20 * r0 + l21 * i10) * r2;
    const double i32 = -l32 * r2 * r3;
    const double i31 = -(l31 * r1 + l32 * i21) * r3;
    const double i30 = -(l30 * r0 + l31 * i10 + l32 * i20) * r3;
    // a[lane i + 16 k] = Li(i - c0, k) for rows i of the block
    const int ib = j - c0;   // row of Li this lane supplies (valid 0..3)
    double li;
    if (q == 0) li = ib == 0 ? r0 : (ib == 1 ? i10 : (ib == 2 ? i20 : i30));
    else if (q == 1) li = ib == 1 ? r1 : (ib == 2 ? i21 : i31);
    else if (q == 2) li = ib == 2 ? r2 : i32;
    else li = r3;
    const double aL = (ib >= q && ib < 4) ? li : 0.0;
    const d4 Lr = __builtin_amdgcn_mfma_f64_16x16x4f64(aL, acc[p], z4, 0, 0, 0);   // rows c0.. of L^T
    const d4 Xr = __builtin_amdgcn_mfma_f64_16x16x4f64(aL, Y[p], z4, 0, 0, 0);     // rows c0.. of X
    const double pv = Lr[p];                      // L(j, c0 + q) for j past the block
    const double pa = j >= c0 + 4 ? pv : 0.0;
    acc[p] = (j >= c0) ? pv : acc[p];             // rows c0.. -> L^T (upper part)
    Y[p] = Xr[p];
    if (p < 3) {
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64(-pa, pa, acc, 0, 0, 0);
      Y = __builtin_amdgcn_mfma_f64_16x16x4f64(-pa, Y[p], Y, 0, 0, 0);
    }
  }
  if (bad) {
    if (lane == 0) *flag = jb * 16 + bad;
    return;
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int c = q + 4 * r;   // this register's row of acc / Y: L(j, c) or X(c, j)
    lb[base + db_e(j, c)] = (j >= c) ? acc[r] : Y[r];   // L lower / X(c, j) at (j, c), upper
    xs[db_e(c, j)] = Y[r];                              // X(c, j), zero for j > c
    if (j == c) xdiag[jb * 16 + c] = Y[r];
  }
}

// the leaf of db_factor_invert (dev A/B: -DDB_LEAF_PERMUTE the bpermute leaf, -DDB_LEAF_COLUMN
// the rank-1 MFMA leaf)
#if defined(DB_LEAF_PERMUTE)
#define DB_LEAF db_leaf
#elif defined(DB_LEAF_COLUMN)
#define DB_LEAF db_leaf_mfma
#else
#define DB_LEAF db_leaf_blk
#endif

// A(po) -= L(pa) L(pb)^T for 16 x 16 blocks at LDS offsets pa, pb, po (one wave)
__device__ __forceinline__ void db_syrk_block(double* lb, int pa, int pb, int po) {
  const int lane = threadIdx.x & 63;
  d4 acc = d4{0.0, 0.0, 0.0, 0.0};
  double av[4], bv[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int k = 4 * s + (lane >> 4);
    av[s] = lb[pa + db_e(lane & 15, k)];
    bv[s] = lb[pb + db_e(lane & 15, k)];          // L(kb,jb)^T(k, n) = L(kb,jb)(n, k)
  }
#pragma unroll
  for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[s], bv[s], acc, 0, 0, 0);
#pragma unroll
  for (int r = 0; r < 4; ++r) lb[po + db_e((lane >> 4) + 4 * r, lane & 15)] -= acc[r];
}

// Two independent blocks of the trailing update at once (the second only if has1): both
// blocks' operand reads, then both MFMA chains, then both read-modify-writes, so each LDS
// round trip is paid once per pair
__device__ __forceinline__ void db_syrk_pair(double* lb, int pa0, int pb0, int po0, int pa1, int pb1, int po1,
                                             bool has1) {
  const int lane = threadIdx.x & 63;
  double av0[4], bv0[4], av1[4], bv1[4], c0[4], c1[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int k = 4 * s + (lane >> 4);
    av0[s] = lb[pa0 + db_e(lane & 15, k)];
    bv0[s] = lb[pb0 + db_e(lane & 15, k)];
    if (has1) {
      av1[s] = lb[pa1 + db_e(lane & 15, k)];
      bv1[s] = lb[pb1 + db_e(lane & 15, k)];
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    c0[r] = lb[po0 + db_e((lane >> 4) + 4 * r, lane & 15)];
    if (has1) c1[r] = lb[po1 + db_e((lane >> 4) + 4 * r, lane & 15)];
  }
  d4 acc0 = d4{0.0, 0.0, 0.0, 0.0}, acc1 = acc0;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(av0[s], bv0[s], acc0, 0, 0, 0);
    if (has1) acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(av1[s], bv1[s], acc1, 0, 0, 0);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    lb[po0 + db_e((lane >> 4) + 4 * r, lane & 15)] = c0[r] - acc0[r];
    if (has1) lb[po1 + db_e((lane >> 4) + 4 * r, lane & 15)] = c1[r] - acc1[r];
  }
}

// X-level of the in-place inverse: for each instance of size 2h (offset o, o2 = o+h),
// X21 = -X22 (L21 X11), X21 written over L21.  Work item = (instance, column block).
template <int H>
__device__ __forceinline__ void db_xlevel(double* lb) {
  constexpr int NBH = H / 16, NINST = 128 / (2 * H);
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // diagonal blocks hold X in their lower part only
  auto xop = [&](int bi, int bk, int r, int c) -> double {
    const int off = (bi * (bi + 1) / 2 + bk) * DB_BS + db_e(r, c);
    return (bi > bk || r >= c) ? lb[off] : 0.0;
  };
  constexpr int ITEMS = NINST * NBH;   // 4 for every level
  static_assert(ITEMS == 4, "one item per wave");
  const int inst = wave / NBH, cb = wave % NBH;
  const int ob = inst * 2 * NBH, ob2 = ob + NBH;      // block offsets
  d4 T[NBH];
#pragma unroll
  for (int ib = 0; ib < NBH; ++ib) {
    T[ib] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int kb = 0; kb < NBH; ++kb) {
      if (kb < cb) continue;
      double av[4], bv[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int k = 4 * s + (lane >> 4);
        const int bi = ob2 + ib, bk = ob + kb;
        av[s] = lb[(bi * (bi + 1) / 2 + bk) * DB_BS + db_e(lane & 15, k)];   // L21(m, k)
        bv[s] = xop(ob + kb, ob + cb, k, lane & 15);                          // X11(k, n)
      }
#pragma unroll
      for (int s = 0; s < 4; ++s) T[ib] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[s], bv[s], T[ib], 0, 0, 0);
    }
  }
  __syncthreads();    // every L21 read before any X21 write
#pragma unroll
  for (int ib = 0; ib < NBH; ++ib) {
    d4 acc = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int kb = 0; kb <= ib; ++kb) {
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const double av = xop(ob2 + ib, ob2 + kb, lane & 15, 4 * s + (lane >> 4));   // X22(m, k)
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, T[kb][s], acc, 0, 0, 0);
      }
    }
    const int bi = ob2 + ib, bk = ob + cb;
#pragma unroll
    for (int r = 0; r < 4; ++r)
      lb[(bi * (bi + 1) / 2 + bk) * DB_BS + db_e((lane >> 4) + 4 * r, lane & 15)] = -acc[r];
  }
  __syncthreads();
}

// One wave stores 16 x 16 block (at lb[off], db_e layout) to G (its top-left element):
// lane = 8 columns x 8 row pairs per 16-byte store.  MODE 0: whole block; 1: lower
// part with the diagonal only (L's diagonal blocks, whose upper part holds X^T);
// 2: lower part and zeros above (X's diagonal blocks).
template <int MODE>
__device__ __forceinline__ void db_put_block(const double* lb, int off, double* G, long long ld) {
  const int lane = threadIdx.x & 63;
  const int r = (lane & 7) * 2;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int c = (lane >> 3) + 8 * h;
    double2 v = *reinterpret_cast<const double2*>(lb + off + db_e(r, c));
    double* gp = G + r + (long long)c * ld;
    if (MODE == 1) {
      if (r >= c) db_gst2(gp, v.x, v.y);
      else if (r + 1 == c) db_gst1(gp + 1, v.y);
    } else {
      if (MODE == 2) {
        if (r < c) v.x = 0.0;
        if (r + 1 < c) v.y = 0.0;
      }
      db_gst2(gp, v.x, v.y);
    }
  }
}

__device__ __forceinline__ int db_blk(int bi, int bk) { return (bi * (bi + 1) / 2 + bk) * DB_BS; }

// row of entry b of a row-major lower triangle (b = r (r + 1) / 2 + c), b < 28: a packed
// table of 3-bit rows for b < 21, row 6 beyond -- a few scalar operations instead of a loop
__host__ __device__ constexpr unsigned long long db_tri_rows() {
  unsigned long long t = 0;
  for (int b = 0, r = 0; b < 21; ++b) {
    while ((r + 1) * (r + 2) / 2 <= b) ++r;
    t |= (unsigned long long)r << (3 * b);
  }
  return t;
}
__device__ __forceinline__ int db_tri_row(int b) {
  return b >= 21 ? 6 : (int)((db_tri_rows() >> (3 * b)) & 7);
}

// Factor + invert the tile held block-packed in lb[0 .. 36*DB_BS).  Writes L (lower)
// to Lg, X = L^-1 (full tile, zero upper) to Xg, returns 0 or the 1-based column
// of the first bad pivot; *logdet_out (thread 0) = sum log L_jj.
// LDS: lb[0, DB_LDS_DOUBLES) plus DB_EXTRA_DOUBLES after it.
// The global stores ride beside the arithmetic: X's zero upper blocks while wave 0
// factors the first leaf, each column block of L once its panel step is done (waves
// 1-3, behind their share of the trailing update), X's blocks as each level of the
// assembly finishes them -- so only the last level's 16 blocks follow the arithmetic.
// on_factored(): called by every thread once L and X's diagonal blocks are stored (only
// with a good factor), before the rest of X is assembled -- the fused Cholesky's panel
// tiles need no more than those (their block substitution, k_gemm G_PANEL).
// assemble = false: return there; the rest of X is assembled later, off the Cholesky's
// chain, for all diagonal tiles at once (k_xasm: it reads L and the stored leaf inverses).
template <class OnFactored>
__device__ __forceinline__ int db_factor_invert(double* lb, double* Lg, long long ldl, double* Xg,
                                                long long ldx, double* logdet_out, OnFactored on_factored,
                                                bool assemble = true) {
  // the wave index as a scalar: derived from tid >> 6 the compiler treats it as divergent,
  // and the trailing update's block loop ran under exec masks with its MFMA pairs split
  // by branches (s_nop between dependent MFMAs)
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  double* xs = lb + 36 * DB_BS;           // current leaf inverse, 16 x 16 (db_e)
  double* xdiag = lb + DB_LDS_DOUBLES;    // 128 diagonal entries of X
  double* red = xdiag + 128;              // 4
  int* flag = reinterpret_cast<int*>(red + 4);
  auto lg_at = [&](int bi, int bk) { return Lg + bi * 16 + (long long)(bk * 16) * ldl; };
  auto xg_at = [&](int bi, int bk) { return Xg + bi * 16 + (long long)(bk * 16) * ldx; };
  if (tid == 0) *flag = 0;
  DB_TDECL;
  __syncthreads();
  DB_TN(0);
  DB_TN(1);
  if (wave == 0) {
    DB_LEAF(lb, xs, xdiag, 0, flag);
  } else {
    // X's 28 strictly-upper blocks are zero
    for (int b = wave - 1; b < 28; b += 3) {
      int bk = 1;
      while (bk * (bk + 1) / 2 <= b) ++bk;            // b = bk(bk-1)/2 + bi, bi < bk
      const int bi = b - bk * (bk - 1) / 2;
      const int r = (lane & 7) * 2;
#pragma unroll
      for (int h = 0; h < 2; ++h)
        db_gst2(xg_at(bi, bk) + r + (long long)((lane >> 3) + 8 * h) * ldx, 0.0, 0.0);
    }
  }
  __syncthreads();
  DB_T(1);
  for (int jb = 0; jb < 8; ++jb) {
    if (*flag) return *flag;
    DB_TN(2);
    // ---- panel: L(ib,jb) = A(ib,jb) X_jb^T, one 16x16 block per wave
    for (int ib = jb + 1 + wave; ib < 8; ib += 4) {
      const int bo = db_blk(ib, jb);
      d4 acc = d4{0.0, 0.0, 0.0, 0.0};
      double av[4], bv[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int k = 4 * s + (lane >> 4);
        av[s] = lb[bo + db_e(lane & 15, k)];          // A(ib,jb)(m, k)
        bv[s] = xs[db_e(lane & 15, k)];               // X^T(k, n) = X(n, k)
      }
#pragma unroll
      for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[s], bv[s], acc, 0, 0, 0);
#pragma unroll
      for (int r = 0; r < 4; ++r) lb[bo + db_e((lane >> 4) + 4 * r, lane & 15)] = acc[r];
    }
    __syncthreads();
    DB_T(2);
    if (jb == 7) break;
    // ---- wave 0: update diagonal block jb+1 and factor it (look-ahead);
    //      waves 1-3: the rest of the trailing update A(ib,kb) -= L(ib,jb) L(kb,jb)^T,
    //      then column block jb of L out
    DB_TN(1);
    if (wave == 0) {
      const int p1 = db_blk(jb + 1, jb);
      DB_TN(6);
      db_syrk_block(lb, p1, p1, db_blk(jb + 1, jb + 1));
      DB_T(6);
      DB_TN(5);
#ifndef DB_NO_LEAF   // dev probe: the update without the leaf beside it (wrong results)
      DB_LEAF(lb, xs, xdiag, jb + 1, flag);
#endif
      DB_T(5);
    } else {
      DB_TN(7);
      const int m = 7 - jb, cnt = m * (m + 1) / 2;
#ifdef DB_NO_UPDATE
      if (cnt < 0)   // dev probe: the leaf without the concurrent update (wrong results)
#endif
      // blocks b = wave, wave + 3, ... (b = 0, the diagonal block, is wave 0's), two at a
      // time (one at a time, the update's LDS round trips held wave 0's leaf at twice its
      // stand-alone time: factor 78.7 -> 73.4 us with pairs, tools/hip/db_bench.hip)
      for (int b = wave; b < cnt; b += 6) {
        const int rr = db_tri_row(b);
        const int ib = jb + 1 + rr, kb = jb + 1 + (b - rr * (rr + 1) / 2);
        const int b1 = b + 3;
        const bool has1 = b1 < cnt;
        const int r1 = db_tri_row(b1);
        const int ib1 = jb + 1 + r1, kb1 = jb + 1 + (b1 - r1 * (r1 + 1) / 2);
        // without a second block the first one goes twice: db_syrk_pair reads both C blocks
        // before writing either, so both write the same values -- and the pair stays
        // branch-free (under has1 its loads and MFMAs were split by ~20 branches: a pair
        // took 2000 shader cycles against 860 in a loop of this shape, tools/hip/syrk_probe.hip;
        // the factor 1-1.5 us faster, profiles/db_probe_r05f.log)
        db_syrk_pair(lb, db_blk(ib, jb), db_blk(kb, jb), db_blk(ib, kb), db_blk(has1 ? ib1 : ib, jb),
                     db_blk(has1 ? kb1 : kb, jb), has1 ? db_blk(ib1, kb1) : db_blk(ib, kb), true);
      }
      for (int ib = jb + wave - 1; ib < 8; ib += 3) {
        if (ib == jb) db_put_block<1>(lb, db_blk(jb, jb), lg_at(jb, jb), ldl);
        else db_put_block<0>(lb, db_blk(ib, jb), lg_at(ib, jb), ldl);
      }
      DB_T(7);
    }
    __syncthreads();
    DB_T(1);
  }
  DB_TN(4);
  // ---- last diagonal block of L out, log-determinant
  if (wave == 1) db_put_block<1>(lb, db_blk(7, 7), lg_at(7, 7), ldl);
  double lg = (tid < 128) ? log(lb[db_off(tid, tid)]) : 0.0;
  for (int off = 32; off > 0; off >>= 1) lg += __shfl_down(lg, off, 64);
  if ((tid & 63) == 0) red[tid >> 6] = lg;
  __syncthreads();
  if (tid == 0) db_gst1(logdet_out, (red[0] + red[1]) + (red[2] + red[3]));
  // ---- diagonal blocks -> X leaves (lower part): X(i,c) stored at (c,i), diag in xdiag
  {
    const int jb = tid >> 5, t = tid & 31;          // 8 blocks x 32 threads
    const int base = db_blk(jb, jb);
    for (int e = t; e < 256; e += 32) {
      const int i = e & 15, c = e >> 4;
      if (i > c) lb[base + db_e(i, c)] = lb[base + db_e(c, i)];
      else if (i == c) lb[base + db_e(i, c)] = xdiag[jb * 16 + i];
    }
  }
  __syncthreads();
  DB_T(4);
  DB_TN(3);
  for (int b = wave; b < 8; b += 4) db_put_block<2>(lb, db_blk(b, b), xg_at(b, b), ldx);
  on_factored();
  if (!assemble) {
    DB_T(3);
    DB_T(0);
    DB_TFLUSH;
    return 0;
  }
  db_xlevel<16>(lb);
  db_put_block<0>(lb, db_blk(2 * wave + 1, 2 * wave), xg_at(2 * wave + 1, 2 * wave), ldx);
  db_xlevel<32>(lb);
#pragma unroll
  for (int h = 0; h < 2; ++h) {                       // rows {2,3} x cols {0,1}, rows {6,7} x cols {4,5}
    const int q = wave * 2 + h, o = (q >> 2) * 4;
    const int bi = o + 2 + ((q >> 1) & 1), bk = o + (q & 1);
    db_put_block<0>(lb, db_blk(bi, bk), xg_at(bi, bk), ldx);
  }
  db_xlevel<64>(lb);
  DB_T(3);
  DB_TN(4);
#pragma unroll
  for (int h = 0; h < 4; ++h) {                       // rows 4-7 x cols 0-3
    const int bi = 4 + wave, bk = h;
    db_put_block<0>(lb, db_blk(bi, bk), xg_at(bi, bk), ldx);
  }
  DB_T(4);
  DB_T(0);
  DB_TFLUSH;
  return 0;
}

}  // namespace gpe
