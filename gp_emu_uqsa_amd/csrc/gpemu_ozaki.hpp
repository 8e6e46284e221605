// gpemu_ozaki.hpp -- A^-1 = X^T X (the LAUUM of the objective's gradient, X = L^-1 lower
// triangular) on the int8 matrix cores, exact integer products reconstructed to fp64 by the
// Chinese remainder theorem (the Ozaki scheme II construction: Ozaki, Uchino, Imamura 2024).
//
// Why: on gfx950 the 32 x 32 x 32 i8 MFMA does 32768 integer multiply-adds per 32 cycles per
// SIMD against 2048 flops per 64 cycles for the 16 x 16 x 4 f64 MFMA: 32 x the fp64 rate per
// clock (measured on random operands, where the chip holds a lower clock: 2.2-2.4 POPS against
// the fp64 GEMM's 70 TF/s, tools/hip/i8_probe.hip).  With N = 16 moduli the product is exact
// and the operands carry 53 bits: the result has fp64 accuracy.
//
// The arithmetic, per column j of X (the rows of both operands of X^T X):
//   e_j     = 52 - ilogb(max_k |X(k,j)|), so X'(k,j) = rint(X(k,j) 2^e_j) is an integer with
//             |X'| <= 2^53 (beta bits: 53, or fewer for n > 16384, see oz_beta on the host);
//   C'(i,j) = sum_k X'(k,i) X'(k,j), exact, |C'| <= n 2^(2 beta) < M / 2 (M = prod m_l);
//   for each modulus m_l (pairwise coprime, <= 256): X'_l = X' mod m_l in [-128, 127]
//             (int8), C'_l = X'_l^T X'_l on the i8 MFMA (int32, exact: |.| <= n 2^14 < 2^31),
//             c_l = C'_l mod m_l (centred, stored as one byte);
//   C'/M    = sum_l c_l y_l / m_l  (mod 1), y_l = (M / m_l)^-1 mod m_l: the centred fraction
//             v of that sum, formed exactly on a 2^-41 grid (hi parts) plus the lo parts,
//             gives C' = v M and A^-1(i,j) = v M 2^-(e_i + e_j).
// Kernels: k_oz_colexp (e_j), k_oz_split (X -> N int8 planes, lower 256-column panels),
// k_oz_gemm (grouped over moduli: 256 x 256 tiles of the lower triangle, K from the tile
// row's diagonal block), k_oz_crt (N residue bytes per element -> fp64, lower 128-tiles).
#pragma once

namespace gpe {

constexpr int OZ_T = 256;                  // output tile, and the planes' column panels
constexpr int OZ_SK = 64;                  // k (bytes) per LDS stage: two 32-deep k-steps
constexpr int OZ_NBUF = 4;                 // stage ring (loads issued 3 stages ahead)
constexpr int OZ_OPND = OZ_T * OZ_SK;      // one operand's stage image (16 KB)
constexpr int OZ_LDS = OZ_NBUF * 2 * OZ_OPND;   // 128 KB: one workgroup per CU
constexpr int OZ_MAXMOD = 16;

// moduli (pairwise coprime; the odd ones <= 253 so a rounded centred residue stays in int8)
// and the reconstruction constants (host: oz_consts)
struct OzConst {
  int m[OZ_MAXMOD];        // modulus
  int c16[OZ_MAXMOD];      // 2^16 mod m
  float inv[OZ_MAXMOD];    // 1 / m
  double rhi[OZ_MAXMOD];   // y / m rounded to a multiple of 2^-41 (y = (M / m)^-1 mod m)
  double rlo[OZ_MAXMOD];   // y / m - rhi
  double Md;               // M = prod m (rounded)
  int nmod;
  int beta;                // operand bits
};

typedef int oz_v4i __attribute__((ext_vector_type(4)));
typedef int oz_v16i __attribute__((ext_vector_type(16)));

// A row (or column) holding a NaN or an infinity gets the exponent OZ_EX_NAN: its planes are
// zero and every product entry in its row (column) comes out NaN, as an fp64 GEMM's would
// (k_oz_il_to_ex: an atomically max-ed OZ_IL_BAD)
constexpr int OZ_EX_NAN = -(1 << 20), OZ_IL_BAD = 1 << 29;
// max that keeps a NaN of either side
__device__ __forceinline__ double oz_pmax(double a, double b) { return (a > b || a != a) ? a : b; }
__device__ __forceinline__ int oz_ex_of(double mx, int beta) {
  return !(mx <= 1.7976931348623157e308) ? OZ_EX_NAN : (mx > 0.0 ? (beta - 1) - ilogb(mx) : 0);
}

// byte offset of column-panel cb in the planes: panel cb holds columns [256 cb, 256 cb + 256),
// rows [256 cb, np2), column-major with ld np2 - 256 cb
__host__ __device__ __forceinline__ long long oz_panel_off(int cb, int np2) {
  return (long long)OZ_T * ((long long)cb * np2 - (long long)OZ_T * cb * (cb - 1) / 2);
}
__host__ __device__ __forceinline__ long long oz_plane_bytes(int np2) { return oz_panel_off(np2 / OZ_T, np2); }

// e_j for every column j < np2 (one wave per column, rows k >= j; columns past np: 0)
static __global__ void __launch_bounds__(256) k_oz_colexp(const double* __restrict__ X, long long ldx, int np,
                                                          int np2, int beta, int* __restrict__ ex) {
  const int lane = threadIdx.x & 63, j = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (j >= np2) return;
  double mx = 0.0;
  if (j < np)
    for (int k = j + lane; k < np; k += 64) mx = oz_pmax(mx, fabs(X[k + (long long)j * ldx]));
  for (int off = 32; off > 0; off >>= 1) mx = oz_pmax(mx, __shfl_xor(mx, off, 64));
  if (lane == 0) ex[j] = oz_ex_of(mx, beta);
}

// X -> the N int8 planes: thread = 8 consecutive rows of one column (a wave reads 4 KB of
// the column and writes 512 contiguous bytes per plane); entries above the diagonal (and past
// np) are zero
constexpr int OZ_SPLIT_ROWS = 8;
static __global__ void __launch_bounds__(256) k_oz_split(const double* __restrict__ X, long long ldx, int np,
                                                         int np2, const int* __restrict__ ex, int8_t* __restrict__ planes,
                                                         long long plane_bytes, OzConst cst) {
  const int j = blockIdx.x;
  const int cb = j / OZ_T, r0 = cb * OZ_T;
  const int k0 = r0 + OZ_SPLIT_ROWS * ((int)blockIdx.y * 256 + (int)threadIdx.x);
  if (k0 >= np2) return;
  const int e = ex[j];
  double xs[OZ_SPLIT_ROWS];
  if (j < np && k0 + OZ_SPLIT_ROWS <= np && k0 >= j) {   // (16-byte loads: k0 is a multiple of 8)
#pragma unroll
    for (int u = 0; u < OZ_SPLIT_ROWS; u += 2) {
      const double2 v = *reinterpret_cast<const double2*>(X + k0 + u + (long long)j * ldx);
      xs[u] = v.x;
      xs[u + 1] = v.y;
    }
  } else {
#pragma unroll
    for (int u = 0; u < OZ_SPLIT_ROWS; ++u) {
      const int k = k0 + u;
      xs[u] = (k >= j && k < np && j < np) ? X[k + (long long)j * ldx] : 0.0;
    }
  }
#pragma unroll
  for (int u = 0; u < OZ_SPLIT_ROWS; ++u) xs[u] = e == OZ_EX_NAN ? 0.0 : rint(ldexp(xs[u], e));   // |.| <= 2^beta
  const long long ld = np2 - r0;
  int8_t* dst = planes + oz_panel_off(cb, np2) + (long long)(j - r0) * ld + (k0 - r0);
  for (int l = 0; l < cst.nmod; ++l) {
    const double m = (double)cst.m[l], im = 1.0 / m;
    unsigned w[2] = {0u, 0u};
#pragma unroll
    for (int u = 0; u < OZ_SPLIT_ROWS; ++u) {
      // centred residue: x - m rint(x / m) is exact (|x| <= 2^53, the product q m an integer
      // below 2^53), |.| <= m / 2 + 1; the m = 256 one wraps into int8 congruently
      const double q = rint(xs[u] * im);
      int r = (int)fma(-q, m, xs[u]);
      r = r > 127 ? r - cst.m[l] : (r < -128 ? r + cst.m[l] : r);
      w[u >> 2] |= ((unsigned)r & 0xffu) << (8 * (u & 3));
    }
    *reinterpret_cast<uint2*>(dst + (long long)l * plane_bytes) = make_uint2(w[0], w[1]);
  }
}

__device__ __forceinline__ void oz_glds16(const int8_t* src, int8_t* dst) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
}
template <int N> __device__ __forceinline__ void oz_vmwait() { asm volatile("s_waitcnt vmcnt(%0)" :: "n"(N) : "memory"); }

// One operand of a product, as int8 planes (one per modulus, plane_bytes apart): row r of
// 256-row tile t at depth k is
//   packed (the LAUUM's lower column panels of X): oz_panel_off(t, np2) + r (np2 - 256 t) + k - 256 t
//   rectangular: (256 t + r) ld + k
struct OzOpnd {
  const int8_t* p;
  long long plane_bytes;
  long long ld;    // rectangular row pitch (bytes); 0: packed
  int np2;         // packed: the padded order
};
__device__ __forceinline__ const int8_t* oz_tile_rows(const OzOpnd& o, int t, int k, long long& ld) {
  if (o.ld == 0) {
    ld = o.np2 - OZ_T * t;
    return o.p + oz_panel_off(t, o.np2) + (k - OZ_T * t);
  }
  ld = o.ld;
  return o.p + (long long)OZ_T * t * o.ld + k;
}

// A product C'_l = A'_l B'_l^T over the 256 x 256 tiles of a list (entries ti << 16 | tj, the
// list's length a multiple of 8 so position % 8 is the XCD under round-robin dispatch,
// 0xffffffff padding the bins), blockIdx.x = l * list_len + position.  K range of tile
// (ti, tj): from 0, 256 ti, 256 tj or 128 floor(2 ti / kdiv) (kbeg 0 / 1 / 2 / 3) to K or
// 256 (ti + 1) (kend 0 / 1): the triangular operands' nonzero k (kbeg 3: the rows of a
// lower-triangular X dealt cyclically by 128-row tiles over kdiv ranks, seen from one rank).
// Tile rows from ti0 (the residues of tile (ti, tj) at its index less that of (ti0, 0)).
struct OzGemm {
  OzOpnd a, b;
  const unsigned* list;
  int list_len;
  int K, kbeg, kend;
  int tri, ntj;    // residue tile of (ti, tj): ti (ti + 1) / 2 + tj (tri) or ti ntj + tj
  int8_t* res;
  long long res_bytes;
  int kdiv = 1;
  int ti0 = 0;
};
__device__ __forceinline__ long long oz_res_tile(int tri, int ntj, int ti, int tj) {
  return tri ? (long long)ti * (ti + 1) / 2 + tj : (long long)ti * ntj + tj;
}

// 4 waves of 128 x 128 (4 x 4 blocks of the 32 x 32 x 32 i8 MFMA, operands swapped so lane &
// 31 runs along the tile's rows); stages of 64 k through a 4-deep LDS ring filled by direct
// global -> LDS loads.  The stage image of each operand is [row][64 B] with granule g of row
// r at slot g ^ ((r >> 2) & 3): conflict-free for ds_read_b128's lane groups.  Output: the
// centred residue of every entry, one byte, in the MFMA's own order (lane l of block b of
// wave w: 16 bytes at ((w 16 + b) 64 + l) 16 of the tile's 64 KB).
static __global__ void __launch_bounds__(256, 1) k_oz_gemm(OzGemm g, OzConst cst) {
  extern __shared__ __attribute__((aligned(16))) double lds_d[];
  int8_t* lds = reinterpret_cast<int8_t*>(lds_d);
  const int l = (int)blockIdx.x / g.list_len;
  const unsigned ent = g.list[(int)blockIdx.x - l * g.list_len];
  if (ent == 0xffffffffu) return;
  const int ti = (int)(ent >> 16), tj = (int)(ent & 0xffffu);
  const int kb = g.kbeg == 1 ? OZ_T * ti : (g.kbeg == 2 ? OZ_T * tj : (g.kbeg == 3 ? 128 * ((2 * ti) / g.kdiv) : 0));
  const int ke = g.kend == 1 ? min(g.K, OZ_T * (ti + 1)) : g.K;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = (wave >> 1) * 128, wn = (wave & 1) * 128;
  OzOpnd oa = g.a, ob = g.b;
  oa.p += (long long)l * oa.plane_bytes;
  ob.p += (long long)l * ob.plane_bytes;
  long long lda, ldb;
  const int kp = (lane & 3) ^ ((lane >> 4) & 3);
  const int8_t* sa = oz_tile_rows(oa, ti, kb, lda);
  const int8_t* sb = oz_tile_rows(ob, tj, kb, ldb);
  sa += (long long)(16 * wave + (lane >> 2)) * lda + 16 * kp;
  sb += (long long)(16 * wave + (lane >> 2)) * ldb + 16 * kp;
  auto stage = [&](int s) {
    int8_t* As = lds + (s & (OZ_NBUF - 1)) * 2 * OZ_OPND;
    int8_t* Bs = As + OZ_OPND;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int w = wave + 4 * p;   // wave-instruction index: rows 16 w .. 16 w + 15
      oz_glds16(sa + (long long)p * 64 * lda + (long long)s * OZ_SK, As + 16 * w * OZ_SK);
      oz_glds16(sb + (long long)p * 64 * ldb + (long long)s * OZ_SK, Bs + 16 * w * OZ_SK);
    }
  };
  oz_v16i acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = oz_v16i{};
  const int ns = max(0, ke - kb) / OZ_SK;
  const int r32 = lane & 31, h = lane >> 5, sw = (r32 >> 2) & 3;
  // the 8 fragments (4 of A, 4 of B) of k-step ks of stage s
  auto frags = [&](int s, int ks, oz_v4i (&af)[4], oz_v4i (&bf)[4]) {
    const int8_t* As = lds + (s & (OZ_NBUF - 1)) * 2 * OZ_OPND;
    const int8_t* Bs = As + OZ_OPND;
    const int slot = ((2 * ks + h) ^ sw) * 16;
#pragma unroll
    for (int i = 0; i < 4; ++i) af[i] = *reinterpret_cast<const oz_v4i*>(As + (wm + 32 * i + r32) * OZ_SK + slot);
#pragma unroll
    for (int j = 0; j < 4; ++j) bf[j] = *reinterpret_cast<const oz_v4i*>(Bs + (wn + 32 * j + r32) * OZ_SK + slot);
  };
  auto mfmas = [&](const oz_v4i (&af)[4], const oz_v4i (&bf)[4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(bf[j], af[i], acc[i][j], 0, 0, 0);
  };
  // wait until stage s has landed (this wave's loads; the barrier makes it every wave's):
  // the stages issued after it, up to s + 3, may stay in flight (loads retire in order)
  auto wait_stage = [&](int s) {
    const int later = min(ns - 1, s + 2) - s;
    if (later >= 2) oz_vmwait<16>();
    else if (later == 1) oz_vmwait<8>();
    else oz_vmwait<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  };
  if (ns > 0) {
    // Software pipeline, one barrier per stage: the next k-step's fragments are read while
    // the current k-step's 16 MFMAs issue.  Stage s + 4 goes into the buffer of stage s,
    // whose last fragment reads every wave finished before the barrier of stage s + 1.
    for (int s = 0; s < min(ns, 3); ++s) stage(s);
    oz_v4i ca[4], cb[4], na[4], nb[4];
    wait_stage(0);
    if (ns > 3) stage(3);
    frags(0, 0, ca, cb);
    for (int s = 0; s < ns; ++s) {
      // this k-step's MFMAs with the next k-step's 8 fragment reads between the first 8 (an
      // MFMA leaves the wave's issue free for most of its 32 cycles; the reads issued ahead
      // of the MFMAs made the first MFMA wait for all of them: lgkmcnt(0))
      mfmas(ca, cb);
      frags(s, 1, na, nb);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // one MFMA
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);   // one LDS read
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
      __builtin_amdgcn_sched_barrier(0);
      if (s + 1 < ns) {
        wait_stage(s + 1);
        if (s + 4 < ns) stage(s + 4);
        frags(s + 1, 0, ca, cb);
      }
      __builtin_amdgcn_sched_barrier(0);
      mfmas(na, nb);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  // centred residues: t = (acc >> 16) (2^16 mod m) + (acc & 0xffff) is exact in fp32
  // (|t| < 2^20), q = rint(t / m) to within 3e-4, r = t - q m in [-m/2 - 1, m/2 + 1];
  // m = 256: the low byte itself
  const int m = cst.m[l], c16 = cst.c16[l];
  const float inv = cst.inv[l];
  int8_t* out = g.res + (long long)l * g.res_bytes +
                (oz_res_tile(g.tri, g.ntj, ti, tj) - oz_res_tile(g.tri, g.ntj, g.ti0, 0)) * (OZ_T * OZ_T) +
                ((long long)(wave * 16) * 64 + lane) * 16;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      unsigned w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int a = acc[i][j][r];
        int v = a;
        if (m != 256) {
          const int t = __mul24(a >> 16, c16) + (a & 0xffff);
          const int q = (int)rintf((float)t * inv);
          v = t - __mul24(q, m);
        }
        w[r >> 2] |= ((unsigned)v & 0xffu) << (8 * (r & 3));
      }
      *reinterpret_cast<oz_v4i*>(out + (long long)(4 * i + j) * 64 * 16) = oz_v4i{(int)w[0], (int)w[1], (int)w[2], (int)w[3]};
    }
}

// fp64 entries from the residues: C(r, c) = alpha v M 2^-(exr[r] + exc[c]), v = C'/M the
// centred fraction of sum_l c_l y_l / m_l.  Thread u of tile t (16 workgroups per tile) =
// wave u / 1024, block (u / 64) % 16, lane u % 64 of k_oz_gemm's order, 16 entries; rows
// < rows and columns < cols only, and with lower128 only the lower 128-tiles.  Tile rows
// from ti0 (as OzGemm); row gm of the product goes to row gm - 256 ti0 of C.
struct OzCrt {
  const int8_t* res;
  long long res_bytes;
  int tri, ntj;
  const int* exr;
  const int* exc;
  double* C;
  long long ldc;
  int rows, cols, lower128;
  double alpha;
  int ti0 = 0;
};
static __global__ void __launch_bounds__(256) k_oz_crt(OzCrt g, OzConst cst) {
  const int t = (int)blockIdx.x >> 4;
  const int u = ((int)blockIdx.x & 15) * 256 + (int)threadIdx.x;
  int ti, tj;
  if (g.tri) {
    const int ta = t + g.ti0 * (g.ti0 + 1) / 2;
    ti = g.ti0;
    while ((ti + 1) * (ti + 2) / 2 <= ta) ++ti;
    tj = ta - ti * (ti + 1) / 2;
  } else {
    ti = g.ti0 + t / g.ntj;
    tj = t % g.ntj;
  }
  const int wave = u >> 10, blk = (u >> 6) & 15, lane = u & 63;
  const int i = blk >> 2, j = blk & 3;
  const int gm = OZ_T * ti + (wave >> 1) * 128 + 32 * i + (lane & 31);
  const int gn0 = OZ_T * tj + (wave & 1) * 128 + 32 * j + 4 * (lane >> 5);
  if (gm >= g.rows || gn0 >= g.cols) return;
  double shi[16], slo[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) shi[r] = slo[r] = 0.0;
  const int8_t* src = g.res + (long long)t * (OZ_T * OZ_T) + (long long)u * 16;
  for (int l = 0; l < cst.nmod; ++l) {
    const oz_v4i w = *reinterpret_cast<const oz_v4i*>(src + (long long)l * g.res_bytes);
    const double rh = cst.rhi[l], rl = cst.rlo[l];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const double cv = (double)(int)(int8_t)((unsigned)w[r >> 2] >> (8 * (r & 3)));
      shi[r] = fma(cv, rh, shi[r]);   // exact: multiples of 2^-41 below 2^11
      slo[r] = fma(cv, rl, slo[r]);
    }
  }
  const int em = g.exr[gm];
  const double sc = g.alpha * cst.Md;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int gn = gn0 + (r & 3) + 8 * (r >> 2);
    if (gn >= g.cols || (g.lower128 && (gm >> 7) < (gn >> 7))) continue;
    const double v = (shi[r] - rint(shi[r])) + slo[r];   // C' / M, centred
    const int en = g.exc[gn];
    g.C[gm - OZ_T * g.ti0 + (long long)gn * g.ldc] =
        (em == OZ_EX_NAN || en == OZ_EX_NAN) ? __builtin_nan("") : v * ldexp(sc, -(em + en));
  }
}

// ---- rectangular operands (the TRTRI's products): op(r, k) of an fp64 block src (ld) is
// src[k + r ld] (TRANS false: the rows are the block's columns) or src[r + k ld] (TRANS
// true), r < R, k < Kv; zero outside, and (mask) where k < r (1) or k > r (2): the lower
// triangle's nonzeros seen from a column (1) or a row (2).
__device__ __forceinline__ bool oz_keep(int mask, int r, int k) {
  return mask == 1 ? k >= r : (mask == 2 ? k <= r : true);
}

// per-row exponents e_r = beta - 1 - ilogb(max_k |op(r, k)|), rows r < Rp (0 past R or for a
// zero row).  TRANS false: one wave per row.  TRANS true: workgroup = 64 rows x 256 k (the
// lanes along r: coalesced), its maximum's ilogb + 2048 atomically max-ed into il (zeroed
// before), then k_oz_il_to_ex.
template <bool TRANS>
static __global__ void __launch_bounds__(256) k_oz_rowexp(const double* __restrict__ src, long long ld, int R, int Rp,
                                                          int Kv, int mask, int beta, int* __restrict__ ex) {
  if constexpr (!TRANS) {
    const int lane = threadIdx.x & 63, r = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= Rp) return;
    double mx = 0.0;
    if (r < R)
      for (int k = lane; k < Kv; k += 64)
        if (oz_keep(mask, r, k)) mx = oz_pmax(mx, fabs(src[k + (long long)r * ld]));
    for (int off = 32; off > 0; off >>= 1) mx = oz_pmax(mx, __shfl_xor(mx, off, 64));
    if (lane == 0) ex[r] = oz_ex_of(mx, beta);
  } else {
    __shared__ double red[4][64];
    const int rl = threadIdx.x & 63, q = threadIdx.x >> 6, r = blockIdx.x * 64 + rl;
    const int k0 = blockIdx.y * 256;
    double mx = 0.0;
    if (r < R)
#pragma unroll 8
      for (int u = 0; u < 64; ++u) {
        const int k = k0 + 4 * u + q;
        if (k < Kv && oz_keep(mask, r, k)) mx = oz_pmax(mx, fabs(src[r + (long long)k * ld]));
      }
    red[q][rl] = mx;
    __syncthreads();
    if (q == 0 && r < R) {
      mx = oz_pmax(oz_pmax(red[0][rl], red[1][rl]), oz_pmax(red[2][rl], red[3][rl]));
      if (!(mx <= 1.7976931348623157e308)) atomicMax(ex + r, OZ_IL_BAD);
      else if (mx > 0.0) atomicMax(ex + r, ilogb(mx) + 2048);
    }
  }
}
static __global__ void __launch_bounds__(256) k_oz_il_to_ex(int* __restrict__ ex, int Rp, int beta) {
  const int r = blockIdx.x * 256 + threadIdx.x;
  if (r < Rp) ex[r] = ex[r] >= OZ_IL_BAD ? OZ_EX_NAN : (ex[r] > 0 ? (beta - 1) - (ex[r] - 2048) : 0);
}

// x (an integer-valued double, |x| <= 2^53) -> its centred residue mod m as one byte
__device__ __forceinline__ unsigned oz_res8(double x, double m, double im, int mi) {
  // x - m rint(x / m) is exact (the product q m an integer below 2^53), |.| <= m / 2 + 1;
  // the m = 256 one wraps into int8 congruently
  const double q = rint(x * im);
  int r = (int)fma(-q, m, x);
  r = r > 127 ? r - mi : (r < -128 ? r + mi : r);
  return (unsigned)r & 0xffu;
}

// op -> the N int8 planes, rectangular (row r at r ldp + k, k < Kp; zero past R / Kv and
// masked).  TRANS false: thread = 8 consecutive k of one row (contiguous in src: four 16-byte
// loads when the 8 are in range and on one side of the mask's diagonal).  TRANS true:
// workgroup = 64 rows x 64 k, thread = 2 adjacent rows x 8 consecutive k (each load 16 bytes,
// the lanes along r); each plane's 64 x 64 bytes go through LDS so the stores run along k
// (4 threads per row, 16 bytes each).
template <bool TRANS>
static __global__ void __launch_bounds__(256) k_oz_split_rect(const double* __restrict__ src, long long ld, int R,
                                                              int Kv, int mask, const int* __restrict__ ex,
                                                              int8_t* __restrict__ planes, long long plane_bytes,
                                                              long long ldp, int Kp, OzConst cst) {
  if constexpr (!TRANS) {
    const int r = blockIdx.x;
    const int k0 = ((int)blockIdx.y * 256 + (int)threadIdx.x) * 8;
    if (k0 >= Kp) return;
    const int e = ex[r];
    double xs[8];
    const double* p = src + k0 + (long long)r * ld;
    // the mask's diagonal k = r: all 8 kept (1), all dropped (0), or mixed (2)
    const int side = mask == 1 ? (k0 >= r ? 1 : (k0 + 7 < r ? 0 : 2))
                   : (mask == 2 ? (k0 + 7 <= r ? 1 : (k0 > r ? 0 : 2)) : 1);
    if (r < R && k0 + 8 <= Kv && side == 1 && ((reinterpret_cast<uintptr_t>(p) & 15) == 0)) {
#pragma unroll
      for (int u = 0; u < 8; u += 2) {
        const double2 v = *reinterpret_cast<const double2*>(p + u);
        xs[u] = v.x;
        xs[u + 1] = v.y;
      }
    } else {
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int k = k0 + u;
        xs[u] = (side != 0 && r < R && k < Kv && oz_keep(mask, r, k)) ? p[u] : 0.0;
      }
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) xs[u] = e == OZ_EX_NAN ? 0.0 : rint(ldexp(xs[u], e));
    int8_t* dst = planes + (long long)r * ldp + k0;
    for (int l = 0; l < cst.nmod; ++l) {
      const double m = (double)cst.m[l], im = 1.0 / m;
      unsigned w0 = 0u, w1 = 0u;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        w0 |= oz_res8(xs[u], m, im, cst.m[l]) << (8 * u);
        w1 |= oz_res8(xs[u + 4], m, im, cst.m[l]) << (8 * u);
      }
      *reinterpret_cast<uint2*>(dst + (long long)l * plane_bytes) = make_uint2(w0, w1);
    }
  } else {
    __shared__ __attribute__((aligned(16))) unsigned tr[64 * 20];   // [row][16 words + 4 pad]
    const int lane = threadIdx.x & 63, rp = lane & 31, kg = (int)threadIdx.x >> 5;
    const int r = (int)blockIdx.x * 64 + 2 * rp;          // rows r, r + 1
    const int k0 = (int)blockIdx.y * 64 + 8 * kg;         // k0 .. k0 + 7
    const int e0 = ex[r], e1 = ex[r + 1];
    double x0[8], x1[8];
    const double* p = src + r + (long long)k0 * ld;
    const bool vec = r + 1 < R && ((reinterpret_cast<uintptr_t>(src + r) & 15) == 0) && (ld & 1) == 0;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int k = k0 + u;
      double a = 0.0, b = 0.0;
      if (k < Kv) {
        if (vec) {
          const double2 v = *reinterpret_cast<const double2*>(p + (long long)u * ld);
          a = v.x;
          b = v.y;
        } else {
          if (r < R) a = p[(long long)u * ld];
          if (r + 1 < R) b = p[(long long)u * ld + 1];
        }
      }
      x0[u] = oz_keep(mask, r, k) ? a : 0.0;
      x1[u] = oz_keep(mask, r + 1, k) ? b : 0.0;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      x0[u] = e0 == OZ_EX_NAN ? 0.0 : rint(ldexp(x0[u], e0));
      x1[u] = e1 == OZ_EX_NAN ? 0.0 : rint(ldexp(x1[u], e1));
    }
    const int wr = (int)threadIdx.x >> 2, wp = (int)threadIdx.x & 3;   // row wr, piece wp of the block
    int8_t* dst = planes + ((long long)blockIdx.x * 64 + wr) * ldp + (long long)blockIdx.y * 64 + 16 * wp;
    for (int l = 0; l < cst.nmod; ++l) {
      const double m = (double)cst.m[l], im = 1.0 / m;
      unsigned a0 = 0u, a1 = 0u, b0 = 0u, b1 = 0u;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        a0 |= oz_res8(x0[u], m, im, cst.m[l]) << (8 * u);
        a1 |= oz_res8(x0[u + 4], m, im, cst.m[l]) << (8 * u);
        b0 |= oz_res8(x1[u], m, im, cst.m[l]) << (8 * u);
        b1 |= oz_res8(x1[u + 4], m, im, cst.m[l]) << (8 * u);
      }
      if (l > 0) __syncthreads();   // (the previous plane's reads done)
      *reinterpret_cast<uint2*>(tr + (2 * rp) * 20 + 2 * kg) = make_uint2(a0, a1);
      *reinterpret_cast<uint2*>(tr + (2 * rp + 1) * 20 + 2 * kg) = make_uint2(b0, b1);
      __syncthreads();
      *reinterpret_cast<uint4*>(dst + (long long)l * plane_bytes) = *reinterpret_cast<const uint4*>(tr + wr * 20 + 4 * wp);
    }
  }
}

// ---- host side (gpemu.hip, gpemu_dist.hip)

// moduli and reconstruction constants for operand sums of length up to np2
inline OzConst oz_consts(int nmod, int np2) {
  static const int mods[OZ_MAXMOD] = {256, 253, 251, 247, 241, 239, 233, 229, 227, 223, 217, 211, 199, 197, 193, 191};
  OzConst k{};
  k.nmod = nmod;
  double log2M = 0.0, Md = 1.0;
  for (int l = 0; l < nmod; ++l) {
    log2M += std::log2((double)mods[l]);
    Md *= (double)mods[l];
  }
  k.Md = Md;
  // |C'| <= np2 2^(2 beta) < M / 2
  k.beta = std::min(53, (int)std::floor((log2M - 1.0 - std::log2((double)np2) - 1e-9) / 2.0));
  for (int l = 0; l < nmod; ++l) {
    const int m = mods[l];
    k.m[l] = m;
    k.c16[l] = 65536 % m;
    k.inv[l] = 1.0f / (float)m;
    long long Mm = 1;   // (M / m) mod m
    for (int j = 0; j < nmod; ++j)
      if (j != l) Mm = (Mm * (mods[j] % m)) % m;
    int y = 1;          // its inverse mod m
    while ((Mm * y) % m != 1) ++y;
    // y / m = rhi + rlo, rhi on the 2^-41 grid (exact products and sums in k_oz_crt)
    const long long num = (long long)y << 41;
    const long long Q = num / m, R = num - Q * m;
    k.rhi[l] = std::ldexp((double)Q, -41);
    k.rlo[l] = std::ldexp((double)R / (double)m, -41);
  }
  return k;
}

// A product's tile list: blocks of OZ_BR tile rows x OZ_BC tile columns (8 x 4; GPEMU_OZ_BLOCK
// "RxC" for A/B runs: 4 x 8, 16 x 2 and 8 x 8 measured within 1%, the LAUUM ~0.15 ms slower
// at 4 x 8, profiles/ozblock_ab_r06*.log) (clipped to the lower
// triangle when lower), heaviest first, greedily binned by work into 8 XCD bins, interleaved
// position by position (bin = position % 8, the XCD under round-robin dispatch), bins padded
// to one length with 0xffffffff; tile rows ti0 .. ti0 + nti - 1.  An XCD's 32 CUs then run one
// block at a time: its tiles share 8 A panels and 4 B panels (a whole tile row on one XCD
// shared one A panel among 32 different B panels: L2 hit rate ~0.5)
template <class W>
std::vector<unsigned> oz_list(int nti, int ntj, bool lower, W work, int ti0 = 0) {
  static const std::pair<int, int> blk = [] {   // (A/B: GPEMU_OZ_BLOCK="RxC")
    int r = 8, c = 4;
    if (const char* e = std::getenv("GPEMU_OZ_BLOCK")) {
      const int rr = std::atoi(e);
      const char* x = std::strchr(e, 'x');
      if (rr > 0 && x && std::atoi(x + 1) > 0) { r = rr; c = std::atoi(x + 1); }
    }
    return std::make_pair(r, c);
  }();
  const int OZ_BR = blk.first, OZ_BC = blk.second;
  struct Blk { double w; std::vector<unsigned> t; };
  std::vector<Blk> blks;
  for (int r0 = ti0; r0 < ti0 + nti; r0 += OZ_BR)
    for (int c0 = 0; c0 < ntj && (!lower || c0 <= r0 + OZ_BR - 1); c0 += OZ_BC) {
      Blk b{0.0, {}};
      for (int ti = r0; ti < std::min(ti0 + nti, r0 + OZ_BR); ++ti)
        for (int tj = c0; tj < std::min(lower ? ti + 1 : ntj, c0 + OZ_BC); ++tj) {
          b.t.push_back(((unsigned)ti << 16) | (unsigned)tj);
          b.w += work(ti, tj);
        }
      if (!b.t.empty()) blks.push_back(std::move(b));
    }
  std::stable_sort(blks.begin(), blks.end(), [](const Blk& x, const Blk& y) { return x.w / x.t.size() > y.w / y.t.size(); });
  std::vector<std::vector<unsigned>> bins(8);
  std::vector<double> load(8, 0.0);
  for (const Blk& b : blks) {
    const int x = (int)(std::min_element(load.begin(), load.end()) - load.begin());
    load[x] += b.w;
    bins[x].insert(bins[x].end(), b.t.begin(), b.t.end());
  }
  size_t longest = 0;
  for (auto& b : bins) longest = std::max(longest, b.size());
  std::vector<unsigned> list(8 * longest, 0xffffffffu);
  for (int x = 0; x < 8; ++x)
    for (size_t q = 0; q < bins[x].size(); ++q) list[8 * q + x] = bins[x][q];
  return list;
}

// ---- one block pair (t0, h, t1) of a TRTRI level (tile units of 128) on the int8 cores:
// the blocks X11 = X(t0:h, t0:h) and X22 = X(h:t1, h:t1) already inverted, L21 = L(h:t1,
// t0:h):
//   T   = L21 X11      (rows of L21 against columns of X11, k >= the column: kbeg = 256 tj)
//   X21 = -X22 T       (rows of X22, k <= the row: kend = 256 (ti + 1), against columns of T)
// T goes to a scratch block (column-major, ld Pb, so its columns are the second product's
// rows).  Plan (host): the rows of each block (Ra, Rb), padded to 256 (Pa, Pb), the two tile
// lists' offsets in a list array, and the products' int8 operations (every modulus).
struct OzTriPair {
  int t0, h, t1, Ra, Rb, Pa, Pb;
  long long la_off, lb_off;
  int la_len, lb_len;
  double ops_a, ops_b;
  size_t planes_bytes(int N) const { return (size_t)N * Pa * (Pa + Pb); }
  size_t resid_bytes(int N) const { return (size_t)N * Pa * Pb; }
};
inline OzTriPair oz_tri_pair_plan(int t0, int h, int t1, int N, std::vector<unsigned>& lists) {
  OzTriPair q;
  q.t0 = t0; q.h = h; q.t1 = t1;
  q.Ra = (h - t0) * TILE;
  q.Rb = (t1 - h) * TILE;
  q.Pa = (q.Ra + OZ_T - 1) / OZ_T * OZ_T;
  q.Pb = (q.Rb + OZ_T - 1) / OZ_T * OZ_T;
  const int nti = q.Pb / OZ_T, ntj = q.Pa / OZ_T;
  const std::vector<unsigned> la = oz_list(nti, ntj, false, [&](int, int tj) { return (double)(q.Pa - OZ_T * tj); });
  const std::vector<unsigned> lb = oz_list(nti, ntj, false, [&](int ti, int) { return (double)(OZ_T * (ti + 1)); });
  q.ops_a = q.ops_b = 0.0;
  for (int tj = 0; tj < ntj; ++tj) q.ops_a += 2.0 * OZ_T * OZ_T * nti * (double)(q.Pa - OZ_T * tj) * N;
  for (int ti = 0; ti < nti; ++ti) q.ops_b += 2.0 * OZ_T * OZ_T * ntj * (double)(OZ_T * (ti + 1)) * N;
  q.la_off = (long long)lists.size();
  q.la_len = (int)la.size();
  lists.insert(lists.end(), la.begin(), la.end());
  q.lb_off = (long long)lists.size();
  q.lb_len = (int)lb.size();
  lists.insert(lists.end(), lb.begin(), lb.end());
  return q;
}

// the first product's L21 side: row exponents (into ex[0, Pb)) and planes of L21's rows
inline void oz_l21_launch(hipStream_t st, const OzConst& k, const OzTriPair& q, const double* L21, long long ld,
                          int8_t* planes, int* ex) {
  const long long pA = (long long)q.Pb * q.Pa;
  (void)hipMemsetAsync(ex, 0, q.Pb * sizeof(int), st);
  hipLaunchKernelGGL(k_oz_rowexp<true>, dim3(q.Pb / 64, (q.Ra + 255) / 256), dim3(256), 0, st, L21, ld, q.Rb, q.Pb,
                     q.Ra, 0, k.beta, ex);
  hipLaunchKernelGGL(k_oz_il_to_ex, dim3((q.Pb + 255) / 256), dim3(256), 0, st, ex, q.Pb, k.beta);
  hipLaunchKernelGGL(k_oz_split_rect<true>, dim3(q.Pb / 64, q.Pa / 64), dim3(256), 0, st, L21, ld, q.Rb, q.Ra, 0,
                     ex, planes, pA, (long long)q.Pa, q.Pa, k);
}

// both products of the pair on stream st (X blocks and L21 with leading dimension ld; T:
// Pb x Pa doubles; planes: q.planes_bytes(N); res: q.resid_bytes(N); ex: Pa + Pb ints;
// lists: the list array of oz_tri_pair_plan, on the device).  l21_done: oz_l21_launch already
// ran (ordered before st's work by the caller).  gc(g, r, nti, ops, flops64) launches one
// k_oz_gemm + k_oz_crt pair.
template <class GC>
void oz_tri_pair_launches(hipStream_t st, const OzConst& k, const OzTriPair& q, const unsigned* lists, const double* L21,
                          const double* X11, const double* X22, double* X21, long long ld, double* T, int8_t* planes,
                          int8_t* res, int* ex, bool l21_done, GC gc) {
  int* exA = ex;
  int* exB = ex + q.Pb;
  const int nti = q.Pb / OZ_T, ntj = q.Pa / OZ_T;
  const long long rb = (long long)nti * ntj * OZ_T * OZ_T;
  {   // T = L21 X11
    const long long pA = (long long)q.Pb * q.Pa, pB = (long long)q.Pa * q.Pa;
    int8_t* PA = planes;
    int8_t* PB = planes + (size_t)k.nmod * pA;
    if (!l21_done) oz_l21_launch(st, k, q, L21, ld, PA, exA);
    hipLaunchKernelGGL(k_oz_rowexp<false>, dim3(q.Pa / 4), dim3(256), 0, st, X11, ld, q.Ra, q.Pa, q.Ra, 1, k.beta, exB);
    hipLaunchKernelGGL(k_oz_split_rect<false>, dim3(q.Pa, (q.Pa + 2047) / 2048), dim3(256), 0, st, X11, ld, q.Ra, q.Ra,
                       1, exB, PB, pB, (long long)q.Pa, q.Pa, k);
    OzGemm g;
    g.a = OzOpnd{PA, pA, q.Pa, 0};
    g.b = OzOpnd{PB, pB, q.Pa, 0};
    g.list = lists + q.la_off;
    g.list_len = q.la_len;
    g.K = q.Pa;
    g.kbeg = 2;
    g.kend = 0;
    g.tri = 0;
    g.ntj = ntj;
    g.res = res;
    g.res_bytes = rb;
    OzCrt r{res, rb, 0, ntj, exA, exB, T, (long long)q.Pb, q.Rb, q.Ra, 0, 1.0};
    gc(g, r, nti, q.ops_a, (double)q.Ra * q.Ra * q.Rb);
  }
  {   // X21 = -X22 T
    const long long pA = (long long)q.Pb * q.Pb, pB = (long long)q.Pa * q.Pb;
    int8_t* PA = planes;
    int8_t* PB = planes + (size_t)k.nmod * pA;
    (void)hipMemsetAsync(exA, 0, q.Pb * sizeof(int), st);
    hipLaunchKernelGGL(k_oz_rowexp<true>, dim3(q.Pb / 64, (q.Rb + 255) / 256), dim3(256), 0, st, X22, ld, q.Rb, q.Pb,
                       q.Rb, 2, k.beta, exA);
    hipLaunchKernelGGL(k_oz_il_to_ex, dim3((q.Pb + 255) / 256), dim3(256), 0, st, exA, q.Pb, k.beta);
    hipLaunchKernelGGL(k_oz_rowexp<false>, dim3(q.Pa / 4), dim3(256), 0, st, T, (long long)q.Pb, q.Ra, q.Pa, q.Rb, 0,
                       k.beta, exB);
    hipLaunchKernelGGL(k_oz_split_rect<true>, dim3(q.Pb / 64, q.Pb / 64), dim3(256), 0, st, X22, ld, q.Rb, q.Rb, 2,
                       exA, PA, pA, (long long)q.Pb, q.Pb, k);
    hipLaunchKernelGGL(k_oz_split_rect<false>, dim3(q.Pa, (q.Pb + 2047) / 2048), dim3(256), 0, st, T, (long long)q.Pb,
                       q.Ra, q.Rb, 0, exB, PB, pB, (long long)q.Pb, q.Pb, k);
    OzGemm g;
    g.a = OzOpnd{PA, pA, q.Pb, 0};
    g.b = OzOpnd{PB, pB, q.Pb, 0};
    g.list = lists + q.lb_off;
    g.list_len = q.lb_len;
    g.K = q.Pb;
    g.kbeg = 0;
    g.kend = 1;
    g.tri = 0;
    g.ntj = ntj;
    g.res = res;
    g.res_bytes = rb;
    OzCrt r{res, rb, 0, ntj, exA, exB, X21, ld, q.Rb, q.Ra, 0, -1.0};
    gc(g, r, nti, q.ops_b, (double)q.Rb * q.Rb * q.Ra);
  }
}

}  // namespace gpe
