// gpemu_kernels.hpp -- gfx950 (CDNA4) device kernels of the GP-emulator hot path.
//
// Storage conventions (see DESIGN.md "Data layout in HBM"):
//  * every n x n matrix is column-major fp64 with ld = n_pad (n rounded up to a
//    multiple of TILE = 128); the padded block is the identity, so Cholesky,
//    inverse and logdet of the padded matrix equal those of the real one;
//  * only lower tiles (ti >= tj) carry data; strictly-upper tiles are scratch;
//  * point sets (X scaled by 1/delta) are row-major n_pad x d, padded rows 0;
//  * skinny right-hand sides ([f H], [u w], ...) are column-major n_pad x P.
//
// Kernels (reference call they replace):
//  k_pairs          K.var / K.covar pair kernel (pdist+exp+squareform, a1,a2,a11)
//  k_gemm<AK,BK>    grouped fp64 MFMA GEMM (v_mfma_f64_16x16x4_f64), used for the
//                   trailing SYRK, panel TRSM, recursive TRTRI and LAUUM; its fused
//                   instance also factors the 128x128 diagonal tiles (gpemu_diag.hpp)
//  k_skinny_mfma    L^-1 x [f H] and L^-T x [u w] (the n x q solves of a7)
//  k_contract       fused <M, dA/dtheta> for all d+2 hyperparameters (a4,a5,a7)
//  small kernels    Gram, reductions, apply q x q transform, column norms
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <cstdlib>

#include "gpemu_diag.hpp"

namespace gpe {

constexpr int TILE = 128;

typedef double d4 __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------------------
// pair kernel: out(i,j) = s2*coff*exp(-|xr_i - xc_j|^2)   (x already / delta)
// mode bit0: lower tiles only (grid enumerates ti >= tj)
// mode bit1: "training" diagonal/padding rules: gi==gj -> s2*cdiag + rscale*r[gi];
//            gi or gj >= n_valid -> identity.  Without bit1 padded -> 0.
// mode bit2: mirror: also write out(j,i) (full symmetric materialisation)
// mode bit3: zero diagonal (the reference's dA matrices, _emulatorkernels.py:53-71)
// fcol: if set, every entry is also multiplied by ((fcol[gi] - fcol[gj]) * fscale)^2
// (dA/d(2 log delta_i): the per-dimension squared distance, :53-63)
// ---------------------------------------------------------------------------
struct PairArgs {
  const double* xr;   // rows point set, row-major [*, d]
  const double* xc;   // cols point set, row-major [*, d]
  double* out;        // column-major
  long long ld;
  int d, nr_valid, nc_valid, mt, nt, mode;
  double s2, coff, cdiag, rscale;
  const double* r;
  const double* fcol = nullptr;
  double fscale = 0.0;
  int csplit = 1;     // k_pairs: workgroups per tile, each a contiguous share of its columns
};

__device__ inline void tri_decode(int e, int& ti, int& tj) {
  int r = (int)((sqrtf(8.0f * (float)e + 1.0f) - 1.0f) * 0.5f);
  while ((r + 1) * (r + 2) / 2 <= e) ++r;
  while (r * (r + 1) / 2 > e) --r;
  ti = r;
  tj = e - r * (r + 1) / 2;
}

// Coordinates are zero-padded to DMAX in registers and LDS, so the distance loop has
// no per-dimension branch; the padded terms are fma(0, 0, s) = s, so the sum over
// k = 0..d-1 is bit-identical to the unpadded one.  Padding, diagonal and zeroed
// entries are selected after the general formula (no divergent paths per entry).
template <int DMAX>
static __global__ void __launch_bounds__(256) k_pairs(PairArgs a) {
  __shared__ double xs_col[TILE * DMAX];
  int ti, tj;
  const int part = (int)blockIdx.x % a.csplit, blk = (int)blockIdx.x / a.csplit;
  if (a.mode & 1) tri_decode(blk, ti, tj);
  else { ti = blk % a.mt; tj = blk / a.mt; }
  const int tid = threadIdx.x;
  const int d = a.d;
  for (int e = tid; e < TILE * DMAX; e += 256) {
    const int c = e / DMAX, k = e - c * DMAX;
    xs_col[e] = k < d ? a.xc[(long long)(tj * TILE + c) * d + k] : 0.0;
  }
  const int r = tid & (TILE - 1);
  const int gi = ti * TILE + r;
  double xi[DMAX];
#pragma unroll
  for (int k = 0; k < DMAX; ++k) xi[k] = (k < d) ? a.xr[(long long)gi * d + k] : 0.0;
  __syncthreads();
  const double pre = a.s2 * a.coff;
  const bool train = (a.mode & 2) != 0;
  const bool zero_diag = (a.mode & 8) != 0;
  const bool row_pad = gi >= a.nr_valid;
  double vdiag = a.s2 * a.cdiag;
  if (train && a.r && ti == tj && !row_pad) vdiag += a.rscale * a.r[gi];
  const double fi = a.fcol ? a.fcol[gi] : 0.0;
  double* out = a.out + gi;
  const int cw = TILE / a.csplit, cend = (part + 1) * cw;
  for (int c = part * cw + (tid >> 7); c < cend; c += 2) {
    const int gj = tj * TILE + c;
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < DMAX; ++k) {
      const double df = xi[k] - xs_col[c * DMAX + k];
      s = fma(df, df, s);
    }
    double v = pre * exp(-s);
    if (a.fcol) {
      const double df = (fi - a.fcol[gj]) * a.fscale;
      v *= df * df;
    }
    const bool pad = row_pad || gj >= a.nc_valid;
    const bool diag = gi == gj;
    if (train) v = pad ? (diag ? 1.0 : 0.0) : (diag ? vdiag : v);
    else v = pad ? 0.0 : v;
    if (zero_diag && diag) v = 0.0;
    out[(long long)gj * a.ld] = v;
    if ((a.mode & 4) && ti != tj) a.out[(long long)gj + (long long)gi * a.ld] = v;
  }
}

// k_pairs for any d (the reference's kernel takes any number of inputs,
// _emulatorkernels.py:39-50): coordinates staged through LDS 32 dimensions at a
// time, each thread keeping the running squared distances of its 64 columns.  The
// sum over k = 0..d-1 is taken in the same order with the same fma as k_pairs.
constexpr int PW_CH = 32;
static __global__ void __launch_bounds__(256) k_pairs_wide(PairArgs a) {
  __shared__ double xs_col[TILE * PW_CH];
  int ti, tj;
  if (a.mode & 1) tri_decode(blockIdx.x, ti, tj);
  else { ti = blockIdx.x % a.mt; tj = blockIdx.x / a.mt; }
  const int tid = threadIdx.x, h = tid >> 7;
  const int d = a.d;
  const int r = tid & (TILE - 1);
  const int gi = ti * TILE + r;
  double s[TILE / 2];
#pragma unroll
  for (int u = 0; u < TILE / 2; ++u) s[u] = 0.0;
  for (int k0 = 0; k0 < d; k0 += PW_CH) {
    __syncthreads();
    for (int e = tid; e < TILE * PW_CH; e += 256) {
      const int c = e / PW_CH, k = e - c * PW_CH;
      xs_col[e] = k0 + k < d ? a.xc[(long long)(tj * TILE + c) * d + k0 + k] : 0.0;
    }
    double xi[PW_CH];
#pragma unroll
    for (int k = 0; k < PW_CH; ++k) xi[k] = (k0 + k < d) ? a.xr[(long long)gi * d + k0 + k] : 0.0;
    __syncthreads();
#pragma unroll
    for (int u = 0; u < TILE / 2; ++u) {
      const int c = h + 2 * u;
#pragma unroll
      for (int k = 0; k < PW_CH; ++k) {
        const double df = xi[k] - xs_col[c * PW_CH + k];
        s[u] = fma(df, df, s[u]);
      }
    }
  }
  const double pre = a.s2 * a.coff;
  const bool train = (a.mode & 2) != 0;
  const bool zero_diag = (a.mode & 8) != 0;
  const bool row_pad = gi >= a.nr_valid;
  double vdiag = a.s2 * a.cdiag;
  if (train && a.r && ti == tj && !row_pad) vdiag += a.rscale * a.r[gi];
  const double fi = a.fcol ? a.fcol[gi] : 0.0;
  double* out = a.out + gi;
#pragma unroll
  for (int u = 0; u < TILE / 2; ++u) {
    const int c = h + 2 * u;
    const int gj = tj * TILE + c;
    double v = pre * exp(-s[u]);
    if (a.fcol) {
      const double df = (fi - a.fcol[gj]) * a.fscale;
      v *= df * df;
    }
    const bool pad = row_pad || gj >= a.nc_valid;
    const bool diag = gi == gj;
    if (train) v = pad ? (diag ? 1.0 : 0.0) : (diag ? vdiag : v);
    else v = pad ? 0.0 : v;
    if (zero_diag && diag) v = 0.0;
    out[(long long)gj * a.ld] = v;
    if ((a.mode & 4) && ti != tj) a.out[(long long)gj + (long long)gi * a.ld] = v;
  }
}

// ---------------------------------------------------------------------------
// grouped fp64 MFMA GEMM:  C(m,n) = alpha * sum_k opA(m,k) opB(k,n) + beta * C(m,n)
// over 128x128 output tiles; each problem of a group may skip upper tiles
// (G_CLOWER) and restrict its K range to a triangular operand's support.
// AK: opA(m,k) at A[k + m*lda] (K-contiguous) else A[m + k*lda]
// BK: opB(k,n) at B[k + n*ldb] (K-contiguous) else B[n + k*ldb]
// C (m,n) at C[m + n*ldc].  256 threads = 4 waves in 2x2, 64x64 per wave =
// 4x4 v_mfma_f64_16x16x4_f64 accumulators.  K staged 16 deep, double-buffered
// LDS ([k][m], pitch 144 doubles: conflict-free fragment reads).
// ---------------------------------------------------------------------------
// G_DIAG: a single diagonal tile whose updated value is then factored and inverted
// in LDS by the same workgroup (gpemu_diag.hpp): L over C, L^-1 into X,
// sum log L_jj into *logdet, info = diag_col0 + bad column on failure.
// G_PANEL: a panel tile updated like any other, then (after the G_DIAG workgroup of
// the same launch released *flag) solved against the factored diagonal tile by block
// substitution: L = (C - L L^T) L_tt^-T (panel_subst; Ld / X point at L_tt and at
// L_tt^-1's diagonal 16 x 16 blocks).
// G_DQUAD: the pending update of a G_DIAG tile split over DQ_N = 10 workgroups, one per
// 32 x 32 block of its lower half (dq_update); each posts *post when stored, and the
// G_DIAG workgroup (K = 0) waits for all of them, then loads the updated tile.
// G_PHALF0 / G_PHALF1 (with G_PANEL): every panel tile is two workgroups, one per 64-row
// half of its substitution.  The G_PHALF0 workgroup runs the tile's pending update, stores
// it and posts *cpost, then substitutes rows 0-63; the G_PHALF1 workgroup (K = 0) waits
// for all of its step's G_PHALF0 tiles to post (pre0), then substitutes rows 64-127.
enum : int { G_CLOWER = 1, G_KBEG_TI = 2, G_KEND_TI = 4, G_DIAG = 8, G_PANEL = 16, G_DQUAD = 32,
             G_PHALF0 = 64, G_PHALF1 = 128 };

struct GemmProb {
  const double* A;
  const double* B;
  double* C;
  long long lda, ldb, ldc;
  int mt, nt, K, flags;
  double alpha, beta;
  int tile_begin, ntiles;
  double* X;          // G_DIAG: X = L^-1 out; G_PANEL: X's diagonal 16 x 16 blocks in
  long long ldx;
  // G_PANEL: the factored diagonal tile L (its strictly lower 16 x 16 blocks), for the
  // block substitution P = C L^-T (G_DIAG with a flag releases the panel tiles as soon as
  // L and X's diagonal blocks are out)
  const double* Ld;
  long long ldd;
  double* logdet;
  int diag_col0;
  int* flag;          // G_DIAG releases, G_PANEL waits
  // counted hand-offs inside one launch (the group schedule of the fused Cholesky):
  // before reading anything the tile waits until *pre0 >= pre0_n and *pre1 >= pre1_n;
  // when its results are stored it adds 1 to *post.  Every awaited tile sits earlier in
  // the launch's tile list (dispatch order), so the earliest unfinished tile can always run.
  int* pre0;
  int* pre1;
  int* post;
  int pre0_n, pre1_n;
  int* cpost;         // G_PHALF0: counted once the tile's pending update is stored
  // split K (plain instances, beta = 0, implicit tile order): ksplit workgroups per tile,
  // each over a contiguous share of the K stages; each stores its partial 128 x 128 sum
  // in part (slot tile * ksplit + kpart) and counts itself in tcnt[tile]; the last to
  // arrive adds the ksplit partials in index order (deterministic) and stores C, then
  // resets the counter.  For launches with fewer tiles than the chip has slots (small n,
  // the TRTRI's small levels): each tile's K loop on one CU is the launch's latency.
  int ksplit;
  double* part;
  int* tcnt;
  // G_KEND_TI: row tile ti's K ends at (ti kti_mul + kti_off + 1) x 128 (1, 0: the
  // triangle's own rows; the row-block TRTRI: a rank's rows ti of a cyclic partition)
  int kti_mul, kti_off;
};

// dev-tool per-tile timeline (-DGEMM_TTRACE build only, tools/hip/tile_probe.hip): per
// workgroup, [0] start, [1] C and first stage landed, [2] K loop done, [3] stores done,
// [4] hardware id, [5] XCC id
// Entries are numbered in start order across launches (gemm_ttrace_n, reset by the host),
// so a whole sweep of launches fits: up to GEMM_TTRACE_MAX workgroups.
#ifdef GEMM_TTRACE
constexpr unsigned GEMM_TTRACE_MAX = 262144;
__device__ unsigned long long gemm_ttrace[8 * GEMM_TTRACE_MAX];
__device__ unsigned gemm_ttrace_n;
__shared__ unsigned gemm_tslot;
#define TTRACE(slot) do { if (threadIdx.x == 0 && gemm_tslot < GEMM_TTRACE_MAX) gemm_ttrace[gemm_tslot * 8 + (slot)] = wall_clock64(); } while (0)
#else
#define TTRACE(slot) do {} while (0)
#endif

// wave index as a scalar: the compiler treats threadIdx.x >> 6 as divergent, so every
// wave-derived address (stage loads, LDS destinations, C corner) would be VALU math
__device__ __forceinline__ int gemm_wave() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

constexpr int GK = 16;
constexpr int GP = 144;    // [k][m] image of an M-contiguous operand: pitch 144 doubles
constexpr int GQ = 18;     // [m][k] image of a K-contiguous operand: pitch 18 doubles
                           // (16-B aligned rows, conflict-free fragment reads)
constexpr int G_OPND = GK * GP;                  // 2304 doubles >= 128 * GQ
constexpr int G_LDS_DOUBLES = 2 * 2 * G_OPND;    // 9216 doubles = 73,728 B
// launch size: also holds the G_DIAG factorisation (block-packed L + scratch +
// flag/reduction slots) -- 2 workgroups per CU still fit in 160 KB
constexpr int G_LDS_LAUNCH_DOUBLES = DB_LDS_DOUBLES + DB_EXTRA_DOUBLES;
static_assert(G_LDS_LAUNCH_DOUBLES >= G_LDS_DOUBLES, "LDS");

// MFMA f64 16x16x4 accumulator layout: lane l, register r -> (row, col) of D
__device__ inline int mfma64_row(int lane, int r) { return (lane >> 4) + 4 * r; }

// K-stage staging of the grouped GEMM: each of the 256 threads moves four 16-byte
// pieces of the A tile (128 x 16) and four of the B tile into registers, then
// into the [k][m] LDS image (pitch GP).
// operands live in global memory: address space 1 gives global_load (vmcnt only)
// instead of flat_load, whose lgkmcnt share would make every LDS-fragment wait
// also wait for the next stage's HBM loads
typedef double gvec2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ double2 gld2(const double* p) {
  const gvec2 v = *(__attribute__((address_space(1))) const gvec2*)(p);
  return make_double2(v.x, v.y);
}
__device__ __forceinline__ double gld1(const double* p) {
  return *(__attribute__((address_space(1))) const double*)(p);
}
__device__ __forceinline__ void gst1(double* p, double v) {
  *(__attribute__((address_space(1))) double*)(p) = v;
}
__device__ __forceinline__ void gst2(double* p, double x, double y) {
  *(__attribute__((address_space(1))) gvec2*)(p) = gvec2{x, y};
}
// value held by lane l ^ 1 (DPP quad_perm [1,0,3,2], two 32-bit moves)
__device__ __forceinline__ double dpp_xor1(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp((int)b, 0xB1, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), 0xB1, 0xF, 0xF, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

template <bool AK, bool BK>
__device__ __forceinline__ void gemm_gload(const double* __restrict__ Ab,
                                           const double* __restrict__ Bb, long long lda,
                                           long long ldb, int k0, int tid, double (&ra)[8],
                                           double (&rb)[8]) {
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int c = tid + 256 * s;
    double2 va, vb;
    if (!AK) {
      const int kk = c >> 6, mm = (c & 63) * 2;
      va = gld2(Ab + mm + (long long)(k0 + kk) * lda);
    } else {
      const int mm = c >> 3, kk = (c & 7) * 2;
      va = gld2(Ab + (long long)mm * lda + k0 + kk);
    }
    if (!BK) {
      const int kk = c >> 6, nn = (c & 63) * 2;
      vb = gld2(Bb + nn + (long long)(k0 + kk) * ldb);
    } else {
      const int nn = c >> 3, kk = (c & 7) * 2;
      vb = gld2(Bb + (long long)nn * ldb + k0 + kk);
    }
    ra[2 * s] = va.x;
    ra[2 * s + 1] = va.y;
    rb[2 * s] = vb.x;
    rb[2 * s + 1] = vb.y;
  }
}

template <bool AK, bool BK>
__device__ __forceinline__ void gemm_sstore(double* lds, int buf, int tid, const double (&ra)[8],
                                            const double (&rb)[8]) {
  double* As = lds + buf * (2 * G_OPND);
  double* Bs = As + G_OPND;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int c = tid + 256 * s;
    if (!AK) {
      const int kk = c >> 6, mm = (c & 63) * 2;
      *reinterpret_cast<double2*>(As + kk * GP + mm) = make_double2(ra[2 * s], ra[2 * s + 1]);
    } else {
      const int mm = c >> 3, kk = (c & 7) * 2;
      *reinterpret_cast<double2*>(As + mm * GQ + kk) = make_double2(ra[2 * s], ra[2 * s + 1]);
    }
    if (!BK) {
      const int kk = c >> 6, nn = (c & 63) * 2;
      *reinterpret_cast<double2*>(Bs + kk * GP + nn) = make_double2(rb[2 * s], rb[2 * s + 1]);
    } else {
      const int nn = c >> 3, kk = (c & 7) * 2;
      *reinterpret_cast<double2*>(Bs + nn * GQ + kk) = make_double2(rb[2 * s], rb[2 * s + 1]);
    }
  }
}

// Direct global -> LDS staging (global_load_lds_dwordx4, no VGPR round trip; the
// default unless GEMM_REGSTAGE).  One wave-instruction writes 64 x 16 B contiguous
// from a wave-uniform LDS base, so:
// - M-contiguous operand: one instruction = one k-row of 128 doubles, into the same
//   [k][m] image (pitch GP) as the register path;
// - K-contiguous operand: one instruction = 8 rows m of 16 doubles, into a [m][16]
//   image whose 16-byte granules are XOR-swizzled (granule kp of row m at slot
//   kp ^ ((m >> 1) & 7)); the swizzle is applied to the per-lane SOURCE address and
//   undone by the fragment reads (kc_idx), which keeps ds_read_b64 conflict-free.
__device__ __forceinline__ int kc_idx(int m, int k) {
  return m * GK + (((((k >> 1) ^ (m >> 1)) & 7)) << 1) + (k & 1);
}

__device__ __forceinline__ void glds16(const double* src, double* lds_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_base, 16, 0, 0);
}

// Per-thread source of the stage loads: the lane-dependent part of the address, computed
// once per tile; each stage then adds a uniform offset (one 64-bit add per load instead of
// a per-lane 64-bit multiply).  K-contiguous operand: row m = 8 w + (lane >> 3) with
// w = wave + 4 s, whose swizzle (m >> 1) & 7 = (4 wave + (lane >> 4)) & 7 does not depend
// on s.
template <bool K_CONTIG>
__device__ __forceinline__ const double* glds_lane_base(const double* P, long long ld, int lane, int wave) {
  if constexpr (!K_CONTIG) return P + 2 * lane + (long long)wave * ld;
  const int kp = (lane & 7) ^ ((4 * wave + (lane >> 4)) & 7);
  return P + (long long)(8 * wave + (lane >> 3)) * ld + 2 * kp;
}

// Ast / Bst: this stage's lane sources (lane base + the stage's K offset); piece s adds
// s * sa (sa = 4 ld for an M-contiguous operand, 32 ld for a K-contiguous one).
template <bool AK, bool BK>
__device__ __forceinline__ void gemm_glds(const double* __restrict__ Ast, const double* __restrict__ Bst,
                                          long long sa, long long sb, double* lds, int buf) {
  double* As = lds + buf * (2 * G_OPND);
  double* Bs = As + G_OPND;
  const int wave = gemm_wave();   // the LDS targets (M0) are wave-uniform: scalar math
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int w = wave + 4 * s;   // wave-instruction index 0..15
    glds16(Ast + s * sa, AK ? As + 8 * w * GK : As + w * GP);
    glds16(Bst + s * sb, BK ? Bs + 8 * w * GK : Bs + w * GP);
  }
}

// Optional tile list: entry = problem (8 bits) | ti (12 bits) | tj (12 bits), one per
// workgroup, in the order the host chose (longest-first, rows grouped per XCD under
// round-robin dispatch).  Speed only: any order gives the same result.
__device__ __forceinline__ void tile_unpack(unsigned v, int& p, int& ti, int& tj) {
  p = (int)(v >> 24);
  ti = (int)((v >> 12) & 0xfffu);
  tj = (int)(v & 0xfffu);
}

// fragments of k-step ks (4 deep) from the LDS stage at As/Bs
template <bool AK, bool BK>
__device__ __forceinline__ void gemm_frags(const double* As, const double* Bs, int ks, int lane, int wm,
                                           int wn, double (&af)[4], double (&bf)[4]) {
  const int krow = ks * 4 + (lane >> 4);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = wm + i * 16 + (lane & 15);
#ifdef GEMM_REGSTAGE
    af[i] = AK ? As[m * GQ + krow] : As[krow * GP + m];
#else
    af[i] = AK ? As[kc_idx(m, krow)] : As[krow * GP + m];
#endif
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = wn + j * 16 + (lane & 15);
#ifdef GEMM_REGSTAGE
    bf[j] = BK ? Bs[n * GQ + krow] : Bs[krow * GP + n];
#else
    bf[j] = BK ? Bs[kc_idx(n, krow)] : Bs[krow * GP + n];
#endif
  }
}

// MFMAs u0 <= u < u1 of one k-step (u = 4 i + j); operands swapped: D = (A B)^T
template <int U0, int U1>
__device__ __forceinline__ void gemm_mfmas(d4 (&acc)[4][4], const double (&af)[4], const double (&bf)[4]) {
#pragma unroll
  for (int u = U0; u < U1; ++u)
    acc[u >> 2][u & 3] = __builtin_amdgcn_mfma_f64_16x16x4f64(bf[u & 3], af[u >> 2], acc[u >> 2][u & 3], 0, 0, 0);
}

// C added inside the K loop (beta != 0, >= 10 stages), in eight chunks of two
// accumulator blocks (chunk c = blocks (c >> 1, 2 (c & 1) + {0, 1}), 8 values per lane):
// chunk c is loaded in stage c after that stage's operand loads, into buffer c & 1, and
// added at the top of stage c + 2.  The stage-end wait lets the chunk just issued stay in
// flight (vmcnt counts in issue order), so each chunk has ~1.5 stages to arrive.  The
// tile's first MFMA then waits only for its first stage, not for the 128 KB of C: the
// up-front preload costs ~11 us per tile at K = 512 (tools/hip/tile_probe.hip), and with
// one stage of slack the chunks stall the loop by as much.  Chunk indices are template
// constants (the first ten stages are unrolled): no register is indexed at run time.
// WIDE: the 16-byte form of gemm_store (DPP exchange at the add).
// stage tag: v = C chunk index (-1: none), p = the stage's buffer parity (-1: from s)
#ifndef GEMM_HOLD
#define GEMM_HOLD 12   // MFMAs of a stage's last k-step issued before its barrier (the rest after)
#endif
template <int V, int P = -1> struct gemm_ic { static constexpr int v = V, p = P < 0 ? (V < 0 ? -1 : (V & 1)) : P; };
constexpr int C_CHUNKS = 8;
// host: a launch holding this problem uses the CDEF instance of k_gemm (tiles with fewer
// than C_CHUNKS + 2 stages still preload C there)
// (ldc bound: the chunk loads' 32-bit buffer offsets reach 64 columns of C)
// (GPEMU_NO_CDEF=1: dev A/B switch, every launch preloads C)
inline bool gemm_cdef(const GemmProb& p) {
  static const bool off = std::getenv("GPEMU_NO_CDEF") != nullptr;
  return !off && p.beta != 0.0 && p.K >= (C_CHUNKS + 2) * GK && p.ldc <= (1ll << 21);
}

// The chunk loads are buffer loads off one per-wave resource (SGPRs), one per-lane byte
// offset (one VGPR) and a scalar offset per load: with 64-bit per-load addresses the
// straight-line prologue keeps every chunk's addresses live and spills.
struct CSrc {
  __amdgpu_buffer_rsrc_t rsrc;   // C tile + this wave's (wm, wn) corner
  int voff;                      // lane part of the element offset, bytes
  int ldc8;                      // ldc in bytes
};

template <bool WIDE>
__device__ __forceinline__ CSrc c_src(const double* Cb, long long ldc, int lane, int wm, int wn) {
  CSrc c;
  const double* base = Cb + __builtin_amdgcn_readfirstlane(wm) + (long long)__builtin_amdgcn_readfirstlane(wn) * ldc;
  c.rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, -1, 0x00020000);
  const int ml = WIDE ? (lane & 14) : (lane & 15);
  const int nl = (lane >> 4) + (WIDE ? 4 * (lane & 1) : 0);   // WIDE: odd lanes read row r + 1
  c.voff = (int)((ml + (long long)nl * ldc) * 8);
  c.ldc8 = (int)(ldc * 8);
  return c;
}

template <int CI, bool WIDE>
__device__ __forceinline__ void c_chunk_load(const CSrc& c, double (&ct)[8]) {
  constexpr int I = CI >> 1;
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int j = 2 * (CI & 1) + q;
    if constexpr (WIDE) {
#pragma unroll
      for (int r = 0; r < 4; r += 2) {
        const int so = I * 16 * 8 + (j * 16 + 4 * r) * c.ldc8;
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(c.rsrc, c.voff, so, 0);
        ct[4 * q + r] = __longlong_as_double(((long long)v[1] << 32) | v[0]);
        ct[4 * q + r + 1] = __longlong_as_double(((long long)v[3] << 32) | v[2]);
      }
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int so = I * 16 * 8 + (j * 16 + 4 * r) * c.ldc8;
        const auto v = __builtin_amdgcn_raw_buffer_load_b64(c.rsrc, c.voff, so, 0);
        ct[4 * q + r] = __longlong_as_double(((long long)v[1] << 32) | v[0]);
      }
    }
  }
}

// use == false (a tile of a CDEF launch whose C is preloaded or absent): add nothing,
// by selection rather than a branch (a branch here costs the stage-end wait its count)
template <int CI, bool WIDE>
__device__ __forceinline__ void c_chunk_add(d4 (&acc)[4][4], int lane, bool use, double sc, const double (&ct)[8]) {
  constexpr int I = CI >> 1;
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    d4& a = acc[I][2 * (CI & 1) + q];
    if constexpr (WIDE) {
      const bool odd = lane & 1;
#pragma unroll
      for (int r = 0; r < 4; r += 2) {
        const double x = ct[4 * q + r], y = ct[4 * q + r + 1];
        const double got = dpp_xor1(odd ? x : y);
        a[r] += use ? sc * (odd ? got : x) : 0.0;
        a[r + 1] += use ? sc * (odd ? y : got) : 0.0;
      }
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r) a[r] += use ? sc * ct[4 * q + r] : 0.0;
    }
    // pin the adds here, ahead of the stage's loads: sunk past the `if (more)` loads they
    // would sit at a join point where the waitcnt pass falls back to vmcnt(0)
#pragma unroll
    for (int r = 0; r < 4; ++r) asm volatile("" : "+v"(a[r]));
  }
}

// K loop of one 128x128 output tile: acc += opA(Ab) opB(Bb) over nk stages of GK.
// Software pipeline (source order): the fragments of the next k-step are read while
// the 16 MFMAs of the current one issue; at a stage boundary the last 4 MFMAs are
// held back until the next stage's first fragments are in flight.
// Order pins between the MFMA clusters: needed by the register-staging path, whose
// fragment reads the compiler otherwise sinks behind the MFMAs; with direct global->LDS
// staging the compiler's own schedule is ~1% faster, so no pins.
#ifdef GEMM_REGSTAGE
#define GEMM_SB() __builtin_amdgcn_sched_barrier(0)
#else
#define GEMM_SB() do {} while (0)
#endif
template <bool AK, bool BK, bool WIDE = true, bool CDEF = false, bool SW = true>
__device__ __forceinline__ void gemm_kloop(const double* Ab, const double* Bb,
                                           long long lda, long long ldb, int kbeg, int nk, double* lds,
                                           d4 (&acc)[4][4], bool cuse = false, const double* Cb = nullptr,
                                           long long ldc = 0, double sc = 0.0) {
  // SW: the wave index as a scalar (gemm_wave); the fused kernel keeps it in a VGPR (with
  // SGPR wave math its factor / panel paths spill ~100 more VGPRs)
  const int tid = threadIdx.x, lane = tid & 63, wave = SW ? gemm_wave() : tid >> 6;
  const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;
  double fa0[4], fb0[4], fa1[4], fb1[4];
  // stage-load sources (gemm_glds): lane base at kbeg, advanced by one stage of K per stage
  const long long sa = AK ? 32 * lda : 4 * lda, sb = BK ? 32 * ldb : 4 * ldb;
  const long long da = AK ? GK : GK * lda, db = BK ? GK : GK * ldb;
  const double* Al = glds_lane_base<AK>(Ab, lda, lane, wave) + (AK ? kbeg : kbeg * lda);
  const double* Bl = glds_lane_base<BK>(Bb, ldb, lane, wave) + (BK ? kbeg : kbeg * ldb);
  double ct0[8], ct1[8];   // CDEF: C chunks in flight (buffer c & 1)
  CSrc csrc;
  if constexpr (CDEF) csrc = c_src<WIDE>(Cb, ldc, lane, wm, wn);
#ifdef GEMM_REGSTAGE
  double ra[8], rb[8];
  gemm_gload<AK, BK>(Ab, Bb, lda, ldb, kbeg, tid, ra, rb);
  gemm_sstore<AK, BK>(lds, 0, tid, ra, rb);
#else
  gemm_glds<AK, BK>(Al, Bl, sa, sb, lds, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
  __syncthreads();
  TTRACE(1);
  gemm_frags<AK, BK>(lds, lds + G_OPND, 0, lane, wm, wn, fa0, fb0);
  // stage s; CI >= 0 (CDEF's first 10 stages, unrolled): C chunk CI is loaded here
  // and chunk CI - 2 added (nothing added unless cuse).  CDEF is a kernel template
  // parameter, not a branch: two inlined K loops in one kernel push the allocator past
  // 256 VGPRs, and run-time branches around the chunks cost the waitcnt pass its counts.
  auto stage = [&](int s, auto cc) {
    constexpr int CI = decltype(cc)::v, PAR = decltype(cc)::p;
    const int cur = PAR >= 0 ? PAR : (s & 1), nxt = cur ^ 1;   // this stage's / the next one's buffer
    const bool more = (CI >= 0 && CI + 2 < C_CHUNKS + 2) || s + 1 < nk;   // prologue: nk >= C_CHUNKS + 2
    if constexpr (CI >= 0) __builtin_amdgcn_sched_barrier(0);   // prologue stages stay apart
    if constexpr (CDEF && CI >= 2) c_chunk_add<CI - 2, WIDE>(acc, lane, cuse, sc, (CI & 1) ? ct1 : ct0);
#ifdef GEMM_REGSTAGE
    if (more) gemm_gload<AK, BK>(Ab, Bb, lda, ldb, kbeg + (s + 1) * GK, tid, ra, rb);
#else
    if (more) {
      Al += da;
      Bl += db;
      gemm_glds<AK, BK>(Al, Bl, sa, sb, lds, nxt);
    }
#endif
    constexpr bool CLOAD = CDEF && CI >= 0 && CI < C_CHUNKS;
    if constexpr (CLOAD) {
      __builtin_amdgcn_sched_barrier(0);   // the chunk's loads issue after the stage's
      c_chunk_load<CI, WIDE>(csrc, (CI & 1) ? ct1 : ct0);
      __builtin_amdgcn_sched_barrier(0);
    }
    const double* As = lds + cur * (2 * G_OPND);
    const double* Bs = As + G_OPND;
    gemm_frags<AK, BK>(As, Bs, 1, lane, wm, wn, fa1, fb1);
    gemm_mfmas<0, 16>(acc, fa0, fb0);
    GEMM_SB();
    gemm_frags<AK, BK>(As, Bs, 2, lane, wm, wn, fa0, fb0);
    gemm_mfmas<0, 16>(acc, fa1, fb1);
    GEMM_SB();
    gemm_frags<AK, BK>(As, Bs, 3, lane, wm, wn, fa1, fb1);
    gemm_mfmas<0, 16>(acc, fa0, fb0);
    GEMM_SB();
    gemm_mfmas<0, GEMM_HOLD>(acc, fa1, fb1);
    GEMM_SB();
    if (more) {
#ifdef GEMM_REGSTAGE
      gemm_sstore<AK, BK>(lds, nxt, tid, ra, rb);
      __syncthreads();
#else
      // this wave's stage s+1 pieces landed; a chunk issued after them may stay in flight
      if constexpr (CLOAD && WIDE) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else if constexpr (CLOAD) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      // bare barrier: __syncthreads' workgroup fence would add a vmcnt(0) (the chunk in
      // flight); this stage's fragment reads were all consumed by its MFMAs, and the
      // clobber keeps the compiler from moving LDS accesses across
      asm volatile("s_barrier" ::: "memory");
#endif
      const double* An = lds + nxt * (2 * G_OPND);
      gemm_frags<AK, BK>(An, An + G_OPND, 0, lane, wm, wn, fa0, fb0);
    }
    GEMM_SB();
    gemm_mfmas<GEMM_HOLD, 16>(acc, fa1, fb1);
    GEMM_SB();
    if constexpr (CI >= 0) __builtin_amdgcn_sched_barrier(0);
  };
  // CDEF prologue: the first C_CHUNKS + 2 stages as straight-line code (no branch between
  // a chunk's load and its add, so the waitcnt pass keeps its counts; at a join it falls
  // back to vmcnt(0)); shorter tiles (never cuse) take the loop alone
  int s0 = 0;
  if constexpr (CDEF) {
    static_assert(C_CHUNKS == 8, "prologue length");
    if (nk >= C_CHUNKS + 2) {
      stage(0, gemm_ic<0>{});
      stage(1, gemm_ic<1>{});
      stage(2, gemm_ic<2>{});
      stage(3, gemm_ic<3>{});
      stage(4, gemm_ic<4>{});
      stage(5, gemm_ic<5>{});
      stage(6, gemm_ic<6>{});
      stage(7, gemm_ic<7>{});
      stage(8, gemm_ic<8>{});
      stage(9, gemm_ic<9>{});
      s0 = C_CHUNKS + 2;
    }
  }
  // s0 is even: the loop runs stage pairs whose buffers are compile-time constants
  int s = s0;
  for (; s + 1 < nk; s += 2) {
    stage(s, gemm_ic<-1, 0>{});
    stage(s + 1, gemm_ic<-1, 1>{});
  }
  if (s < nk) stage(s, gemm_ic<-1, 0>{});
  if constexpr (!SW) __syncthreads();   // the fused kernel's factor / panel paths reuse the staging LDS
}

// Epilogue and C preload move 16 B per lane: in the MFMA layout lanes l and l ^ 1 hold
// rows m and m ^ 1 of the same columns, so for each register pair (r, r + 1) the even
// lane trades its column-(r + 1) value for the odd lane's column-r value (one DPP
// exchange) and each lane then owns rows (m & ~1, m | 1) of one column: half the store
// (load) instructions of the 8-byte form, same bytes and addresses.
// The fused Cholesky's kernel (k_gemm FUSED) keeps the 8-byte form: there the exchange's
// live values push the factor/panel paths past 256 VGPRs (~150 spilled).
template <bool WIDE = true>
__device__ __forceinline__ void gemm_store(double* Cb, long long ldc, double alpha, const d4 (&acc)[4][4]) {
  const int lane = threadIdx.x & 63, wave = WIDE ? gemm_wave() : (int)(threadIdx.x >> 6);   // narrow: fused
  const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;
  if constexpr (!WIDE) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = wm + i * 16 + (lane & 15);
          const int n = wn + j * 16 + mfma64_row(lane, r);
          gst1(Cb + m + (long long)n * ldc, alpha * acc[i][j][r]);
        }
    return;
  }
  const bool odd = lane & 1;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; r += 2) {
        const int m = wm + i * 16 + (lane & 14);
        const int n = wn + j * 16 + mfma64_row(lane, odd ? r + 1 : r);
        const double a = acc[i][j][r], b = acc[i][j][r + 1];
        const double got = dpp_xor1(odd ? a : b);
        gst2(Cb + m + (long long)n * ldc, alpha * (odd ? got : a), alpha * (odd ? b : got));
      }
}

// Cross-workgroup hand-off inside one launch (MI355X guide, inter-workgroup
// visibility): producer = plain stores, every storing wave s_waitcnt vmcnt(0),
// barrier, one lane: agent release fence, s_waitcnt, relaxed sc1 flag store;
// consumer = relaxed sc1 poll, one agent acquire fence, s_waitcnt, barrier.
__device__ __forceinline__ void gemm_publish_flag(int* flag, int v) {   // one lane, after the barrier
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __hip_atomic_store(flag, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// bounded wait (one lane) for a G_DIAG workgroup's flag (1 = ready, 2 = failed);
// returns the flag, or 0 after ~seconds (never expected: reported as an error)
// (an abort raised meanwhile -- a bad pivot elsewhere -- ends the wait as failed)
__device__ __forceinline__ int gemm_wait_flag(const int* flag, const int* abort_flag) {
  int v = 0;
  for (long it = 0; it < (1l << 22) && v == 0; ++it) {
    v = __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (v == 0 && abort_flag && __hip_atomic_load(abort_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) v = 2;
    if (v == 0) __builtin_amdgcn_s_sleep(8);
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  return v;
}

constexpr int GEMM_WAIT_TIMEOUT = 0x7fffffff;   // info value after a flag wait timed out

// bounded wait (one lane) until *cnt >= n: 1 reached, 2 the launch aborted meanwhile,
// 0 after ~seconds (never expected: reported as an error)
__device__ __forceinline__ int gemm_wait_count(const int* cnt, int n, const int* abort_flag) {
  int st = 0;
  for (long it = 0; it < (1l << 22); ++it) {
    if (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= n) { st = 1; break; }
    if (abort_flag && __hip_atomic_load(abort_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) { st = 2; break; }
    __builtin_amdgcn_s_sleep(8);
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  return st;
}

// every wave's stores of this tile done, then one lane releases them and counts the tile
__device__ __forceinline__ void gemm_post_count(int* cnt) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// dev-tool timeline of the fused Cholesky (-DGEMM_TRACE build only): per column
// step t, slots [t*8 + 0..3] = diagonal workgroup start / update done / factor
// done / flag published, [t*8 + 4..7] = first panel workgroup start / update done /
// flag seen / multiply done (wall_clock64, 100 MHz).
#ifdef GEMM_TRACE
__device__ unsigned long long gemm_trace[8 * 4096];
#define GTRACE(P, slot) do { if (threadIdx.x == 0 && (P).flag && (P).diag_col0 >= 0) gemm_trace[(P).diag_col0 / TILE * 8 + (slot)] = wall_clock64(); } while (0)
#else
#define GTRACE(P, slot) do {} while (0)
#endif

// One 32 x 32 block (qr, qc) of a diagonal tile's lower half (DQ_N = 10 of them, ti =
// qr (qr + 1) / 2 + qc) of its pending update, C -= L_r L_c^T over K (L_r / L_c: rows
// 32 qr / 32 qc of the tile row's pending columns, A = their top-left, column-major,
// lda), by one workgroup: the diagonal tile's update is on the Cholesky's critical chain,
// and on one CU its 128 x 128 x K product (4.2 MFLOP at K = 128, ~14 us at one CU's fp64
// MFMA rate, plus the cold C preload) was the chain step's second-longest link; ten
// workgroups take 0.26 MFLOP each.  Waves 2 x 2, 16 x 16 each.  K staged 64 deep through
// two LDS slots ([k][m] images, pitch 32, global_load_lds: one wave instruction = four k
// rows of 32 doubles); at K = 128 (the width-1 steps) both chunks are requested at once.
// The block's C is loaded before the first chunk and added after the K loop; diagonal
// blocks skip their upper-right 16 x 16 (never read: only the tile's lower half is factored).
constexpr int DQ_N = 10;
constexpr int DQ_KC = 64;              // k per chunk
constexpr int DQ_P = 32;               // image pitch (doubles)
constexpr int DQ_IMG = DQ_KC * DQ_P;   // one operand image, 2048 doubles
constexpr int DQ_SLOT = 2 * DQ_IMG;    // A + B: 32 KB
static_assert(2 * DQ_SLOT <= G_LDS_DOUBLES, "dq slots");
__device__ __forceinline__ void dq_stage(const double* La, const double* Lb, long long lda, int k0, double* lds,
                                         int slot, int lane) {
  const int wave = gemm_wave();   // the LDS targets (M0) are wave-uniform
  double* As = lds + slot * DQ_SLOT;
  double* Bs = As + DQ_IMG;
#pragma unroll
  for (int h = 0; h < 4; ++h) {   // wave instruction w = 4 wave + h: k rows 4w .. 4w + 3
    const int w = 4 * wave + h;
    const long long off = 2 * (lane & 15) + (long long)(k0 + 4 * w + (lane >> 4)) * lda;
    glds16(La + off, As + w * 4 * DQ_P);
    glds16(Lb + off, Bs + w * 4 * DQ_P);
  }
}

template <class Prob>
__device__ __forceinline__ void dq_update(const Prob& P, int quad, double* lds) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int qr = 0;
  while ((qr + 1) * (qr + 2) / 2 <= quad) ++qr;
  const int qc = quad - qr * (qr + 1) / 2;
  const int wm = (wave >> 1) * 16, wn = (wave & 1) * 16;
  const bool skip = qr == qc && wm < wn;   // upper-right 16 x 16 of a diagonal block
  const double* La = P.A + 32 * qr;
  const double* Lb = P.A + 32 * qc;
  double* Cq = P.C + 32 * qr + (long long)(32 * qc) * P.ldc;
  const int nk = P.K / DQ_KC;   // K is a multiple of 128
  double cv[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) cv[r] = gld1(Cq + (wm + (lane & 15)) + (long long)(wn + mfma64_row(lane, r)) * P.ldc);
  dq_stage(La, Lb, P.lda, 0, lds, 0, lane);
  if (nk > 1) dq_stage(La, Lb, P.lda, DQ_KC, lds, 1, lane);
  d4 acc = d4{0.0, 0.0, 0.0, 0.0};
  for (int c = 0; c < nk; ++c) {
    // chunk c landed (8 loads per wave per chunk; chunk c + 1 may stay in flight)
    if (c + 1 < nk) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();   // every wave's pieces of chunk c
    const double* As = lds + (c & 1) * DQ_SLOT;
    const double* Bs = As + DQ_IMG;
    if (!skip) {
#pragma unroll
      for (int ks = 0; ks < DQ_KC / 4; ++ks) {
        const int krow = 4 * ks + (lane >> 4);
        const double af = As[krow * DQ_P + wm + (lane & 15)];
        const double bf = Bs[krow * DQ_P + wn + (lane & 15)];
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(bf, af, acc, 0, 0, 0);
      }
    }
    __syncthreads();   // every wave is done with slot c & 1
    if (c + 2 < nk) dq_stage(La, Lb, P.lda, (c + 2) * DQ_KC, lds, c & 1, lane);
  }
  if (skip) return;
#pragma unroll
  for (int r = 0; r < 4; ++r)
    gst1(Cq + (wm + (lane & 15)) + (long long)(wn + mfma64_row(lane, r)) * P.ldc, P.beta * cv[r] + P.alpha * acc[r]);
}

// Panel tile of the fused Cholesky by block substitution: P = C L^-T for a 128 x 128
// tile C (in place, ldc) against the factored diagonal tile L (ldd) and its diagonal
// blocks' inverses X_b (X's diagonal 16 x 16 blocks, ldx).  As transposes, P^T(jb) =
// X_jb (C^T(jb) - sum_{kb<jb} L(jb,kb) P^T(kb)) for the eight 16-row blocks jb.
// A tile's rows are split over two workgroups (G_PHALF0 / G_PHALF1: rows row_base ..
// row_base + 63); wave w owns rows row_base + 16w .. + 15 (one 16-column block of P^T), so
// the waves never exchange data; an MFMA result (row (lane>>4)+4r, column lane&15) is
// already the B operand of the next product (k = 4s + (lane>>4), n = lane&15 at s = r).
// On one CU the substitution is its 144 MFMAs per wave (64 cycles each): two workgroups
// per tile halve the chain's panel link against one workgroup of 32 rows per wave.
// panel_subst_c: this wave's C^T blocks into pt -- issued before the flag wait (C is
// the tile's own update, stored before by the G_PHALF0 workgroup's four waves: the
// caller has them land first), so they arrive while the factor finishes.
// The tile's loads and stores are buffer accesses off one SGPR resource at the tile's
// corner: one 32-bit lane offset (row, column lane >> 4) and a uniform offset per
// (jb, r), where 64-bit per-access addresses kept all 32 of them live (and spilled).
// (Offsets fit 32 bits: n <= 2^20, so ldc * 8 * 128 < 2^31.)
struct PanelAddr {
  __amdgpu_buffer_rsrc_t rsrc;
  int voff, ldc8;
};
__device__ __forceinline__ PanelAddr panel_addr(const double* Cb, long long ldc, int row_base) {
  PanelAddr a;
  const unsigned long long cb = (unsigned long long)Cb;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)cb), hi = __builtin_amdgcn_readfirstlane((unsigned)(cb >> 32));
  a.rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)(((unsigned long long)hi << 32) | lo), 0, -1, 0x00020000);
  const int lane = threadIdx.x & 63, row0 = row_base + (threadIdx.x >> 6) * 16 + (lane & 15);
  a.ldc8 = (int)(ldc * 8);
  a.voff = row0 * 8 + (lane >> 4) * a.ldc8;
  return a;
}
__device__ __forceinline__ double panel_ld(const PanelAddr& a, int col) {   // col: jb * 16 + 4 r
  const auto v = __builtin_amdgcn_raw_buffer_load_b64(a.rsrc, a.voff, col * a.ldc8, 0);
  return __longlong_as_double(((long long)v[1] << 32) | v[0]);
}
__device__ __forceinline__ void panel_st(const PanelAddr& a, int col, double x) {
  const unsigned long long b = __double_as_longlong(x);
  __builtin_amdgcn_raw_buffer_store_b64((__attribute__((ext_vector_type(2))) unsigned){(unsigned)b, (unsigned)(b >> 32)},
                                        a.rsrc, a.voff, col * a.ldc8, 0);
}
__device__ __forceinline__ void panel_subst_c(const PanelAddr& pa, d4 (&pt)[8]) {
#pragma unroll
  for (int jb = 0; jb < 8; ++jb)
#pragma unroll
    for (int r = 0; r < 4; ++r) pt[jb][r] = panel_ld(pa, jb * 16 + 4 * r);
}

typedef double dv2 __attribute__((ext_vector_type(2)));

__host__ __device__ constexpr int tri_row(int b) {   // bi of packed lower block b = bi(bi+1)/2 + bk
  int bi = 0;
  while ((bi + 1) * (bi + 2) / 2 <= b) ++bi;
  return bi;
}

// LDS: L(jb,kb) (kb < jb) and X_jb, block-packed (256 doubles a block, plain column-major:
// this code reads only the operand pattern) -- 72 KB, the staging space;
// every thread's 18 16-byte pieces are loaded together (one round trip), then stored.
template <class Prob>
__device__ __forceinline__ void panel_subst(const PanelAddr& pa, const double* Ld, long long ldd,
                                            const double* Xd, long long ldx, double* lb, d4 (&pt)[8],
                                            const Prob& P, int ti) {
  const int tid = threadIdx.x, lane = tid & 63;
  {
    // one SGPR resource per source (L, X's diagonal blocks), a 32-bit lane offset each and
    // a uniform offset per block: no per-load 64-bit addresses live across the batch
    const int hi = tid >> 7, w = tid & 127, r = (w & 7) * 2, c = w >> 3;
    const __amdgpu_buffer_rsrc_t rl = __builtin_amdgcn_make_buffer_rsrc((void*)Ld, 0, -1, 0x00020000);
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void*)Xd, 0, -1, 0x00020000);
    const int ldd8 = (int)(ldd * 8), ldx8 = (int)(ldx * 8);
    const int vl = r * 8 + c * ldd8, vx = r * 8 + c * ldx8;
    dv2 v[18];
#pragma unroll
    for (int i = 0; i < 18; ++i) {   // block b = 2i + hi (both candidates fold at compile time)
      const int bi0 = tri_row(2 * i), bk0 = 2 * i - bi0 * (bi0 + 1) / 2;
      const int bi1 = tri_row(2 * i + 1), bk1 = 2 * i + 1 - bi1 * (bi1 + 1) / 2;
      const int bi = hi ? bi1 : bi0, bk = hi ? bk1 : bk0;   // (hi is wave-uniform)
      const bool xb = bi == bk;
      const auto u = __builtin_amdgcn_raw_buffer_load_b128(xb ? rx : rl, xb ? vx : vl,
                                                            bi * 128 + bk * 16 * (xb ? ldx8 : ldd8), 0);
      v[i] = dv2{__longlong_as_double(((long long)u[1] << 32) | u[0]), __longlong_as_double(((long long)u[3] << 32) | u[2])};
    }
#pragma unroll
    for (int i = 0; i < 18; ++i) *reinterpret_cast<dv2*>(lb + (2 * i + hi) * 256 + r + c * 16) = v[i];
  }
  __syncthreads();
#ifdef PANEL_PHASES   // dev probe: GEMM_TRACE slot 5 = staging done
  if (ti == 0) GTRACE(P, 5);
#endif
  const int ao = (lane & 15) + (lane >> 4) * 16;   // A operand (m = lane&15, k = 4s + lane>>4) at ao + 64 s
#pragma unroll
  for (int jb = 0; jb < 8; ++jb) {
    // the step's A operands first, in one batch (row block jb of L, then X_jb): a read
    // beside each product would put an LDS round trip in front of every MFMA
    double av[8][4], xv[4];
    const double* arow = lb + (jb * (jb + 1) / 2) * 256 + ao;   // blocks (jb, 0 .. jb) are contiguous
#pragma unroll
    for (int kb = 0; kb < jb; ++kb)
#pragma unroll
      for (int s = 0; s < 4; ++s) av[kb][s] = arow[kb * 256 + 64 * s];
#pragma unroll
    for (int s = 0; s < 4; ++s) xv[s] = arow[jb * 256 + 64 * s];
    // two accumulation chains (even / odd kb) keep two MFMAs in flight
    d4 t0 = d4{0.0, 0.0, 0.0, 0.0}, t1 = t0;
#pragma unroll
    for (int kb = 0; kb < jb; ++kb) {
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        if (kb & 1) t1 = __builtin_amdgcn_mfma_f64_16x16x4f64(av[kb][s], pt[kb][s], t1, 0, 0, 0);
        else t0 = __builtin_amdgcn_mfma_f64_16x16x4f64(av[kb][s], pt[kb][s], t0, 0, 0, 0);
      }
    }
    const d4 t = pt[jb] - (t0 + t1);
    d4 o = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int s = 0; s < 4; ++s) o = __builtin_amdgcn_mfma_f64_16x16x4f64(xv[s], t[s], o, 0, 0, 0);
    pt[jb] = o;
    // buffer stores (a FLAT store would also count in lgkmcnt, and the next step's LDS
    // wait would wait for it to land)
#pragma unroll
    for (int r = 0; r < 4; ++r) panel_st(pa, jb * 16 + 4 * r, o[r]);
  }
}

// FUSED (only <false, false, true>): the fused Cholesky's launches, whose problems may be
// G_DIAG / G_PANEL; the other instances hold no factor / panel code, so they stay well
// inside the register budget and use the 16-byte C preload and epilogue.
// ticket (FUSED launches with a tile list and in-launch waits): each workgroup claims its
// list position with an atomic ticket when it starts, instead of taking blockIdx.x.  A
// tile waits only on tiles earlier in the list (build_plan checks it), and every earlier
// position was claimed by a workgroup that is already running, so the earliest unfinished
// tile can always make progress whatever order the hardware dispatches the workgroups in
// and whatever else occupies the CUs (other streams, other contexts' launches).
template <bool AK, bool BK, bool FUSED = false, bool CDEF = false>
static __global__ void __launch_bounds__(256, 2) k_gemm(const GemmProb* __restrict__ probs, int nprob,
                                                  const unsigned* __restrict__ tiles,
                                                  int* __restrict__ abort_flag, int* __restrict__ ticket) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  unsigned pos = blockIdx.x;
  if constexpr (FUSED) {
    if (ticket) {   // (LDS slot G_LDS_LAUNCH_DOUBLES - 3 is used by nothing else)
      int* slot = reinterpret_cast<int*>(lds + G_LDS_LAUNCH_DOUBLES - 3);
      if (threadIdx.x == 0)
        *slot = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __syncthreads();
      pos = (unsigned)*slot;
    }
  }
  if (abort_flag && *abort_flag) return;
  int p = 0, ti, tj;
  if (tiles) {
    tile_unpack(tiles[pos], p, ti, tj);
  } else {
    // last problem whose tile_begin <= blockIdx.x (tile_begin is non-decreasing)
    int lo = 0, hi = nprob - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if ((int)pos >= probs[mid].tile_begin) lo = mid;
      else hi = mid - 1;
    }
    p = lo;
  }
  const GemmProb P = probs[p];
  int kpart = 0, tl = 0;   // split K: this workgroup's share and its tile's index in the problem
  if (!tiles) {
    int local = (int)pos - P.tile_begin;
    if (!FUSED && P.ksplit > 1) {
      kpart = local % P.ksplit;
      local /= P.ksplit;
      tl = local;
    }
    if (P.flags & G_CLOWER) {
      tri_decode(local, ti, tj);
    } else if ((P.flags & G_KEND_TI) && nprob == 1) {
      // triangle times a full block (the posterior's L^-1 K*, noise_fit's L U^T):
      // row ti has K = (ti+1)*128, so rows go longest first, and with mt % 8 == 0
      // XCD b % 8 takes whole rows (its A panel stays in that XCD's L2); as k_gemm_f32
      if ((P.mt & 7) == 0) {
        const int x = local & 7, r = local >> 3;
        ti = P.mt - 1 - (x + 8 * (r / P.nt));
        tj = r % P.nt;
      } else {
        ti = P.mt - 1 - local / P.nt;
        tj = local % P.nt;
      }
    } else {
      ti = local % P.mt;
      tj = local / P.mt;
    }
  }
  int kbeg = 0, kend = P.K;
  if (P.flags & G_KBEG_TI) kbeg = ti * TILE;
  if (P.flags & G_KEND_TI) kend = min(kend, (ti * P.kti_mul + P.kti_off + 1) * TILE);
  if (!FUSED && P.ksplit > 1) {   // this share of the tile's K stages
    const int ns = max(0, kend - kbeg) / GK;
    const int s0 = kpart * ns / P.ksplit, s1 = (kpart + 1) * ns / P.ksplit;
    kend = kbeg + s1 * GK;
    kbeg += s0 * GK;
  }

  const int tid = threadIdx.x;
  if constexpr (FUSED) {
    if (P.pre0 || P.pre1) {   // the group schedule's in-launch hand-offs (see GemmProb)
      int* ready = reinterpret_cast<int*>(lds + G_LDS_LAUNCH_DOUBLES - 2);
      if (tid == 0) {
        int st = 1;
        if (P.pre0) st = gemm_wait_count(P.pre0, P.pre0_n, abort_flag);
        if (st == 1 && P.pre1) st = gemm_wait_count(P.pre1, P.pre1_n, abort_flag);
        *ready = st;
      }
      __syncthreads();
      const int st = *ready;
      __syncthreads();
      if (st != 1) {
        if (st == 0 && tid == 0 && abort_flag) atomicCAS(abort_flag, 0, GEMM_WAIT_TIMEOUT);
        return;
      }
    }
  }
  const int lane = tid & 63, wave = FUSED ? (tid >> 6) : gemm_wave();   // as gemm_kloop's SW
  const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;
#ifdef GEMM_TTRACE
  if (tid == 0) gemm_tslot = atomicAdd(&gemm_ttrace_n, 1u);
  __syncthreads();
  TTRACE(0);
  if (threadIdx.x == 0 && gemm_tslot < GEMM_TTRACE_MAX) {
    const unsigned e = gemm_tslot * 8;
    gemm_ttrace[e + 4] = __builtin_amdgcn_s_getreg((31 << 11) | 4);
    gemm_ttrace[e + 5] = __builtin_amdgcn_s_getreg((31 << 11) | 20);
    // [6] kind (0 plain tile, 1 diagonal, 2 panel) + 4 x blockIdx, [7] K of its own product
    gemm_ttrace[e + 6] = ((P.flags & G_DIAG) ? 1 : ((P.flags & G_PANEL) ? 2 : 0)) + 4ull * pos;
    gemm_ttrace[e + 7] = (unsigned long long)(kend - kbeg);
  }
#endif
  if constexpr (FUSED) {
    if (P.flags & G_DQUAD) {   // one quadrant of a diagonal tile's pending update
      dq_update(P, ti, lds);
      if (P.post) gemm_post_count(P.post);
      return;
    }
  }
  if (P.flags & G_DIAG) GTRACE(P, 0);
  if ((P.flags & G_PHALF0) && ti == 0) GTRACE(P, 4);

  const double* Ab = AK ? P.A + (long long)ti * TILE * P.lda : P.A + (long long)ti * TILE;
  const double* Bb = BK ? P.B + (long long)tj * TILE * P.ldb : P.B + (long long)tj * TILE;

  // operands are swapped in the MFMA, so D = (A B)^T: lane&15 -> m, row map -> n.
  // beta != 0: with >= 10 K stages C is added inside the K loop (c_chunk_load); shorter
  // tiles start the accumulators at (beta/alpha) C, loaded in one burst.
  double* Cb = P.C + (long long)ti * TILE + (long long)tj * TILE * P.ldc;
  const int nk = (kend - kbeg) / GK;
  // beta != 0 with >= 10 stages: C is added chunk by chunk inside the K loop (c_chunk_load)
  // (the ldc bound of gemm_cdef again: the chunk loads' 32-bit buffer offsets; a CDEF
  // launch may mix problems, and one over the bound preloads C instead)
  const bool cdefer = CDEF && P.beta != 0.0 && nk >= C_CHUNKS + 2 && P.ldc <= (1ll << 21);
  d4 acc[4][4];
  if (cdefer) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = d4{0.0, 0.0, 0.0, 0.0};
  } else if (P.beta != 0.0 && FUSED) {   // the fused kernel keeps the 8-byte form (see gemm_store)
    const double sc = P.beta / P.alpha;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = wm + i * 16 + (lane & 15);
          const int n = wn + j * 16 + mfma64_row(lane, r);
          acc[i][j][r] = sc * gld1(Cb + m + (long long)n * P.ldc);
        }
  } else if (P.beta != 0.0) {
    const double sc = P.beta / P.alpha;
    const bool odd = lane & 1;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; r += 2) {   // 16-B loads, the inverse of gemm_store's exchange
          const int m = wm + i * 16 + (lane & 14);
          const int n = wn + j * 16 + mfma64_row(lane, odd ? r + 1 : r);
          const double2 v = gld2(Cb + m + (long long)n * P.ldc);
          const double got = dpp_xor1(odd ? v.x : v.y);
          acc[i][j][r] = sc * (odd ? got : v.x);
          acc[i][j][r + 1] = sc * (odd ? v.y : got);
        }
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = d4{0.0, 0.0, 0.0, 0.0};
  }

  if (nk > 0) gemm_kloop<AK, BK, !FUSED, CDEF, !FUSED>(Ab, Bb, P.lda, P.ldb, kbeg, nk, lds, acc, cdefer, Cb, P.ldc,
                                               P.beta / P.alpha);
  TTRACE(2);

  if constexpr (FUSED) {
    if (P.flags & G_DIAG) {
      GTRACE(P, 1);
      // updated diagonal tile -> block-packed LDS (lower half), then factor + invert;
      // then release the panel workgroups of this launch waiting on *P.flag
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int m = wm + i * 16 + (lane & 15);
            const int n = wn + j * 16 + mfma64_row(lane, r);
            if (m >= n) lds[db_off(m, n)] = P.alpha * acc[i][j][r];
          }
      __syncthreads();
      // the panel tiles (block substitution with L and X's diagonal blocks) are released
      // once those are out, before the rest of X is assembled
      const int bad = db_factor_invert(lds, Cb, P.ldc, P.X, P.ldx, P.logdet, [&] {
        if (P.flag) {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every wave's L / X-block stores done
          __syncthreads();
          if (tid == 0) { gemm_publish_flag(P.flag, 1); GTRACE(P, 2); }
        }
      }, P.flag == nullptr);   // the single-GPU sweep (with flags) assembles X later (k_xasm)
      if (bad && tid == 0 && abort_flag) atomicCAS(abort_flag, 0, P.diag_col0 + bad);
      if (P.flag && bad) {   // (on_factored is not called for a bad factor)
        __syncthreads();
        if (tid == 0) gemm_publish_flag(P.flag, 2);
      }
      GTRACE(P, 3);
      TTRACE(3);
      return;
    }
    if (P.flags & G_PANEL) {
      // G_PHALF0: updated panel tile -> C, posted; both halves: wait for the diagonal
      // factor of this launch, then L = C L_tt^-T over their 64 rows by block substitution
      const bool h0 = (P.flags & G_PHALF0) != 0;
      const int row_base = h0 ? 0 : 64;
      if (h0) {
        if (ti == 0) GTRACE(P, 5);
        gemm_store<false>(Cb, P.ldc, P.alpha, acc);
        gemm_post_count(P.cpost);   // (every wave's stores landed: the barrier inside)
      }
      d4 pt[8];
      // the C^T rows span every wave's stores: all of them landed, and no stale L1 line
      __syncthreads();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      const PanelAddr pa = panel_addr(Cb, P.ldc, row_base);
      panel_subst_c(pa, pt);
      int* ready = reinterpret_cast<int*>(lds + G_LDS_LAUNCH_DOUBLES - 1);   // staging is idle here
      if (tid == 0) *ready = gemm_wait_flag(P.flag, abort_flag);
      __syncthreads();
      const int st = *ready;
      __syncthreads();
      if (h0 && ti == 0) GTRACE(P, 6);
      if (st != 1) {
        if (st == 0 && tid == 0 && abort_flag) atomicCAS(abort_flag, 0, GEMM_WAIT_TIMEOUT);
        return;
      }
      TTRACE(1);   // (panel tiles: [1] = the diagonal inverse seen)
      panel_subst(pa, P.Ld, P.ldd, P.X, P.ldx, lds, pt, P, ti);
      if (h0 && ti == 0) GTRACE(P, 7);
      if (P.post) gemm_post_count(P.post);
#ifdef GEMM_TTRACE
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      TTRACE(3);
#endif
      return;
    }
  }
  if constexpr (!FUSED) {
    if (P.ksplit > 1) {
      // partial out (value-major: coalesced across the workgroup), count, and the last
      // workgroup of the tile sums the partials in index order
      const int ks = P.ksplit;
      double* slot = P.part + ((long long)tl * ks + kpart) * (TILE * TILE);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) gst1(slot + ((i * 4 + j) * 4 + r) * 256 + tid, acc[i][j][r]);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      int* last = reinterpret_cast<int*>(lds + G_LDS_LAUNCH_DOUBLES - 3);
      if (tid == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        *last = __hip_atomic_fetch_add(P.tcnt + tl, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ks - 1;
      }
      __syncthreads();
      if (!*last) return;
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      const double* p0 = P.part + (long long)tl * ks * (TILE * TILE);
      // partial by partial, each one's 64 loads issued together (a load-add chain per
      // element put ~ks x 64 dependent load latencies in front of the store: a 4-way split
      // of a 16-tile TRTRI level took 70 us)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[i][j][r] = gld1(p0 + ((i * 4 + j) * 4 + r) * 256 + tid);
      for (int c = 1; c < ks; ++c) {
        const double* pc = p0 + (long long)c * (TILE * TILE);
        double t[4][4][4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) t[i][j][r] = gld1(pc + ((i * 4 + j) * 4 + r) * 256 + tid);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[i][j][r] += t[i][j][r];
      }
      if (tid == 0) __hip_atomic_store(P.tcnt + tl, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  gemm_store<!FUSED>(Cb, P.ldc, P.alpha, acc);
  if constexpr (FUSED) {
    if (P.post) gemm_post_count(P.post);
  }
#ifdef GEMM_TTRACE
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  TTRACE(3);
#endif
}

// X_tt = L_tt^-1 for every diagonal tile t (blockIdx.x) of a factorisation, after the
// fused Cholesky (whose diagonal workgroups store L and the eight 16 x 16 leaf inverses,
// release the panel tiles and stop there: db_factor_invert(assemble = false)).  The
// assembly (db_xlevel at 16, 32, 64) was ~12 us of each step's diagonal workgroup, which
// in the width-1 steps outlived the panel substitution and held the launch open; here it
// runs once for all tiles, off the chain.  X's strictly-upper blocks are already zero.
static __global__ void __launch_bounds__(256) k_xasm(const double* __restrict__ A, double* __restrict__ B,
                                                     long long ld) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const long long t0 = (long long)blockIdx.x * TILE * (ld + 1);
  const double* L = A + t0;
  double* X = B + t0;
  for (int e = threadIdx.x; e < 36 * 256; e += 256) {
    const int b = e >> 8, w = e & 255, bi = tri_row(b), bk = b - bi * (bi + 1) / 2;
    const long long g = (bi * 16 + (w & 15)) + (long long)(bk * 16 + (w >> 4)) * ld;
    lds[b * DB_BS + db_e(w & 15, w >> 4)] = gld1((bi == bk ? X : L) + g);   // leaf inverse (zeros above) / L block
  }
  __syncthreads();
  db_xlevel<16>(lds);
  db_xlevel<32>(lds);
  db_xlevel<64>(lds);
  const int wave = threadIdx.x >> 6;
  for (int b = wave; b < 36; b += 4) {
    const int bi = tri_row(b), bk = b - bi * (bi + 1) / 2;
    if (bi != bk) db_put_block<0>(lds, b * DB_BS, X + bi * 16 + (long long)(bk * 16) * ld, ld);
  }
}

// ---------------------------------------------------------------------------
// fp32 GEMM for the posterior's V = L^-1 K* at precision 32 (BASELINE C5):
// C(m,n) = sum_k A(m,k) B(k,n), A M-contiguous (the triangle, G_KEND_TI), B
// K-contiguous (K*), fp32 in and out, v_mfma_f32_16x16x4_f32.  Same tiling as
// k_gemm: 128x128 tile, 4 waves of 64x64, K staged 32 deep in double-buffered
// LDS: [k][m] pitch 144 floats and [n][k] pitch 36 floats, both conflict-free for
// ds_read_b32 (lane -> bank is a permutation).  Operands swapped as in k_gemm so
// the stores are M-contiguous; f32 C/D map: row = 4 (lane >> 4) + reg.
// ---------------------------------------------------------------------------
constexpr int F32_GK = 32;
constexpr int F32_PA = 144;   // [k][m]
constexpr int F32_PB = 36;    // [n][k]
constexpr int F32_STAGE = F32_GK * F32_PA + TILE * F32_PB;   // floats per stage (9216)
typedef float f4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float4 gld4f(const float* p) {
  const f4v v = *(__attribute__((address_space(1))) const f4v*)(p);
  return make_float4(v.x, v.y, v.z, v.w);
}

// pa / pb: this thread's sources for the stage (lane part + the stage's K offset, see
// k_gemm_f32); piece u adds u * sa (sa = 8 lda: k rows) / u * sb (sb = 32 ldb: n rows)
__device__ __forceinline__ void g32_gload(const float* pa, const float* pb, long long sa, long long sb,
                                          float (&ra)[16], float (&rb)[16]) {
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const float4 a = gld4f(pa + u * sa);
    const float4 b = gld4f(pb + u * sb);
    ra[4 * u] = a.x; ra[4 * u + 1] = a.y; ra[4 * u + 2] = a.z; ra[4 * u + 3] = a.w;
    rb[4 * u] = b.x; rb[4 * u + 1] = b.y; rb[4 * u + 2] = b.z; rb[4 * u + 3] = b.w;
  }
}

__device__ __forceinline__ void g32_sstore(float* st, int tid, const float (&ra)[16], const float (&rb)[16]) {
  float* As = st;
  float* Bs = st + F32_GK * F32_PA;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int c = tid + 256 * u;
    const int kk = c >> 5, mm = (c & 31) * 4;
    *reinterpret_cast<float4*>(As + kk * F32_PA + mm) = make_float4(ra[4 * u], ra[4 * u + 1], ra[4 * u + 2], ra[4 * u + 3]);
    const int nn = c >> 3, k2 = (c & 7) * 4;
    *reinterpret_cast<float4*>(Bs + nn * F32_PB + k2) = make_float4(rb[4 * u], rb[4 * u + 1], rb[4 * u + 2], rb[4 * u + 3]);
  }
}

static __global__ void __launch_bounds__(256, 2) k_gemm_f32(const float* A, long long lda, const float* B,
                                                             long long ldb, float* C, long long ldc, int mt,
                                                             int K, int kend_ti) {
  extern __shared__ __attribute__((aligned(16))) float lds32[];
  // Tile order: with the triangle (kend_ti), row ti has K = (ti+1)*128, so rows go
  // longest first (no long tile starts last).  When mt % 8 == 0, workgroup b runs on
  // XCD b % 8 under round-robin dispatch and that XCD takes rows mt-1-(b%8), -8, ...
  // whole, so each row's A panel is read into one XCD's L2.
  const int nt = gridDim.x / mt;
  int ti, tj;
  if ((mt & 7) == 0) {
    const int x = blockIdx.x & 7, r = blockIdx.x >> 3;
    ti = mt - 1 - (x + 8 * (r / nt));
    tj = r % nt;
  } else {
    ti = mt - 1 - (int)blockIdx.x / nt;
    tj = (int)blockIdx.x % nt;
  }
  const int kend = kend_ti ? min(K, (ti + 1) * TILE) : K;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;
  const float* Ab = A + (long long)ti * TILE;
  const float* Bb = B + (long long)tj * TILE * ldb;
  typedef float f4 __attribute__((ext_vector_type(4)));
  f4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  const int nk = kend / F32_GK;
  float ra[16], rb[16];
  // fragments of k-step ks (4 deep) of the stage at As/Bs
  auto frags = [&](const float* As, const float* Bs, int ks, float (&af)[4], float (&bf)[4]) {
    const int krow = 4 * ks + (lane >> 4);
#pragma unroll
    for (int i = 0; i < 4; ++i) af[i] = As[krow * F32_PA + wm + i * 16 + (lane & 15)];
#pragma unroll
    for (int j = 0; j < 4; ++j) bf[j] = Bs[(wn + j * 16 + (lane & 15)) * F32_PB + krow];
  };
  // MFMAs u0 <= u < u1 (u = 4 i + j) of one k-step
  auto mfmas = [&](int u0, int u1, const float (&af)[4], const float (&bf)[4]) {
#pragma unroll
    for (int u = 0; u < 16; ++u)
      if (u >= u0 && u < u1)
        acc[u >> 2][u & 3] = __builtin_amdgcn_mfma_f32_16x16x4f32(bf[u & 3], af[u >> 2], acc[u >> 2][u & 3], 0, 0, 0);
  };
  float fa0[4], fb0[4], fa1[4], fb1[4];
  // stage-load sources: lane part once per tile (A: k row tid >> 5, m (tid & 31) * 4; B: n row
  // tid >> 3, k (tid & 7) * 4), then one uniform step of F32_GK per stage
  const float* pa = Ab + (tid & 31) * 4 + (long long)(tid >> 5) * lda;
  const float* pb = Bb + (long long)(tid >> 3) * ldb + (tid & 7) * 4;
  const long long sa = 8 * lda, sb = 32 * ldb, da = F32_GK * lda;
  if (nk > 0) {
    g32_gload(pa, pb, sa, sb, ra, rb);
    g32_sstore(lds32, tid, ra, rb);
    __syncthreads();
    frags(lds32, lds32 + F32_GK * F32_PA, 0, fa0, fb0);
  }
  // Software pipeline (as gemm_kloop): the fragments of k-step ks+1 are read before
  // the 16 MFMAs of k-step ks issue, so their LDS latency hides behind them; at the
  // stage boundary the last 4 MFMAs wait until the next stage's first fragments
  // are in flight.  sched_barrier keeps the compiler from regrouping.
  // stages run in pairs so each stage's buffer is a compile-time constant (as gemm_kloop)
  auto stage = [&](int s, auto par) {
    constexpr int cur = decltype(par)::v, nxt = cur ^ 1;
    const bool more = s + 1 < nk;
    if (more) {
      pa += da;
      pb += F32_GK;
      g32_gload(pa, pb, sa, sb, ra, rb);
    }
    const float* As = lds32 + cur * F32_STAGE;
    const float* Bs = As + F32_GK * F32_PA;
#pragma unroll
    for (int ks = 0; ks < F32_GK / 4; ks += 2) {
      frags(As, Bs, ks + 1, fa1, fb1);
      __builtin_amdgcn_sched_barrier(0);
      mfmas(0, 16, fa0, fb0);
      __builtin_amdgcn_sched_barrier(0);
      if (ks + 2 < F32_GK / 4) {
        frags(As, Bs, ks + 2, fa0, fb0);
        __builtin_amdgcn_sched_barrier(0);
        mfmas(0, 16, fa1, fb1);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    mfmas(0, 12, fa1, fb1);
    __builtin_amdgcn_sched_barrier(0);
    if (more) {
      g32_sstore(lds32 + nxt * F32_STAGE, tid, ra, rb);
      __syncthreads();
      const float* An = lds32 + nxt * F32_STAGE;
      frags(An, An + F32_GK * F32_PA, 0, fa0, fb0);
    }
    __builtin_amdgcn_sched_barrier(0);
    mfmas(12, 16, fa1, fb1);
    __builtin_amdgcn_sched_barrier(0);
  };
  int s = 0;
  for (; s + 1 < nk; s += 2) {
    stage(s, gemm_ic<0>{});
    stage(s + 1, gemm_ic<1>{});
  }
  if (s < nk) stage(s, gemm_ic<0>{});
  float* Cb = C + (long long)ti * TILE + (long long)tj * TILE * ldc;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = wm + i * 16 + (lane & 15);
        const int n = wn + j * 16 + 4 * (lane >> 4) + r;
        Cb[m + (long long)n * ldc] = acc[i][j][r];
      }
}

// out (fp32, ld_out) = in (fp64, ld_in) over rows x cols
static __global__ void __launch_bounds__(256) k_to_f32(const double* in, long long ld_in, float* out,
                                                        long long ld_out, long long rows, int cols) {
  const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
  if (e >= rows * cols) return;
  const long long i = e % rows, j = e / rows;
  out[i + j * ld_out] = (float)in[i + j * ld_in];
}

// out[j] = sum_i V(i, j)^2 over fp32 V, fp64 accumulation (4 columns per block)
static __global__ void __launch_bounds__(256) k_colnorm2_f32(const float* V, long long ldv, int nrows,
                                                              int ncols, double* out) {
  const int j = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (j >= ncols) return;
  const float* col = V + (long long)j * ldv;
  double s = 0.0;
  for (int i = lane; i < nrows; i += 64) {
    const double v = col[i];
    s = fma(v, v, s);
  }
  for (int off = 32; off > 0; off >>= 1) s += __shfl_down(s, off, 64);
  if (lane == 0) out[j] = s;
}

// ---------------------------------------------------------------------------
// skinny products with a lower-triangular (or full) tiled matrix M (ld = ldm),
// k_skinny_mfma below:
//   TR = false : part[ch] = M[rows it, cols k in chunk] x R[k, 0:P]
//   TR = true  : part[ch] = M[rows k in chunk, cols it]^T x R[k, 0:P]
// R column-major (ld = ldr), partials column-major [ch][P][ldp].
// Chunks of CH k-tiles bound the partial buffer; k_reduce_chunks sums them
// in a fixed order (bitwise reproducible).
// ---------------------------------------------------------------------------
constexpr int SK_CH = 16;
constexpr int SK_PMAX = 32;

struct SkinnyArgs {
  const double* M;
  long long ldm;
  const double* R;
  long long ldr;
  double* part;
  long long ldp;       // rows of one partial column
  long long pstride;   // doubles between chunk partials
  int P, ntr;          // columns of R; number of row tiles of M (k extent, t-kernel)
  int lower;           // 1: M lower-triangular by tiles
  int nit;             // output tiles
  const int* abort_flag;
  int chk;             // k tiles per chunk (<= SK_CH; fewer for launches of few output tiles)
};

// ---------------------------------------------------------------------------
// Z = L^-1 F by blocked forward substitution, without forming L^-1: the value-only
// objective and gpe_beta need only L, L^-1 f and L^-1 H (_emulatoroptimise.py:382-408,
// :425-442, :497-504).  L lower by 128-row tiles (ld), D_t = L_tt^-1 the diagonal-tile
// inverses the fused Cholesky leaves in the second buffer (Dinv, ld), F / Z column-major
// n_pad x P (P <= TS_PM; the host runs wider F in column chunks).
// One workgroup per tile row i: acc = F_i - sum_{j<i} L_ij Z_j, taking each Z_j as soon
// as row j is published, then Z_i = D_i acc, published by raising the row counter
// *flags to i + 1.  Rows publish in order (row i only after reading *flags >= i), so the
// counter is monotone, one poll tells a lagging row every tile it may take, and every
// wait is on a row claimed (by ticket) before the waiting one's (no dispatch-order deadlock).
// Thread (r, h), 512 threads: row r of the tile row, k quarter h of every 128 x 128 x P
// product (L_ij's 32 values are loaded before the wait; D_i's 32 are held from the
// start), partial sums combined through LDS.  L is read once (n^2/2 x 8 B, HBM-bound);
// the chain per tile row is one flag hop, the Z_{i-1} staging, one tile product and the
// D_i product (~1.7 us each at one CU's fp64 rate).
// ---------------------------------------------------------------------------
constexpr int TS_PM = 16;
constexpr int TS_Q = 4;             // k quarters
constexpr int TS_KQ = TILE / TS_Q;  // 32

// sum the TS_Q quarters' v[PM] into quarter 0's threads (two tree rounds through LDS
// buffers b0, b1, each TILE x PM; callers sync before reusing them)
__device__ __forceinline__ void ts_reduce(double (&v)[TS_PM], double* b0, double* b1, int r, int h) {
  if (h >= 2) {
    double* b = (h == 2) ? b0 : b1;
#pragma unroll
    for (int p = 0; p < TS_PM; ++p) b[r * TS_PM + p] = v[p];
  }
  __syncthreads();
  if (h < 2) {
    const double* b = (h == 0) ? b0 : b1;
#pragma unroll
    for (int p = 0; p < TS_PM; ++p) v[p] += b[r * TS_PM + p];
  }
  __syncthreads();
  if (h == 1) {
#pragma unroll
    for (int p = 0; p < TS_PM; ++p) b0[r * TS_PM + p] = v[p];
  }
  __syncthreads();
  if (h == 0) {
#pragma unroll
    for (int p = 0; p < TS_PM; ++p) v[p] += b0[r * TS_PM + p];
  }
}

static __global__ void __launch_bounds__(512) k_trsv_lower(const double* __restrict__ L, long long ld,
                                                   const double* __restrict__ Dinv,
                                                   const double* __restrict__ F, long long ldf, double* Z,
                                                   long long ldz, int P, int* flags, int* ticket,
                                                   int* abort_flag) {
  constexpr int PM = TS_PM, KQ = TS_KQ;
  __shared__ double Zs[2][TILE * PM];   // [k][p]; after the loop: reduction buffers
  __shared__ int st, row;
  if (abort_flag && *abort_flag) return;   // set by an earlier launch: every workgroup sees it
  // the tile row by ticket, not blockIdx.x: every row this one waits on was claimed by a
  // workgroup that is already running (no dependence on the hardware's dispatch order)
  if (threadIdx.x == 0) row = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const int i = row;
  const int tid = threadIdx.x, r = tid & (TILE - 1), h = tid >> 7;
  // D_i(r, k) for this thread's k quarter (the upper triangle is stored as zeros)
  double dv[KQ];
  {
    const double* drow = Dinv + (long long)i * TILE + r + (long long)(i * TILE + h * KQ) * ld;
#pragma unroll
    for (int k = 0; k < KQ; ++k) dv[k] = drow[(long long)k * ld];
  }
  double acc[PM];
  const double* frow = F + (long long)i * TILE + r;
#pragma unroll
  for (int p = 0; p < PM; ++p) acc[p] = (h == 0 && p < P) ? frow[(long long)p * ldf] : 0.0;
  const double* lrow = L + (long long)i * TILE + r + (long long)(h * KQ) * ld;
  int ready = 0;   // rows [0, ready) known published (lane 0 of wave 0 only)
  for (int j = 0; j < i; ++j) {
    double lv[KQ];
    const double* lt = lrow + (long long)j * TILE * ld;
#pragma unroll
    for (int k = 0; k < KQ; ++k) lv[k] = lt[(long long)k * ld];
    if (tid == 0 && j >= ready) {   // one poll and one acquire per batch of published rows
      int v = 0;
      for (long it = 0; it < (1l << 22); ++it) {
        v = __hip_atomic_load(flags, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (v > j) break;
        __builtin_amdgcn_s_sleep(4);
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      ready = v;
      st = v > j ? 1 : 0;
    }
    __syncthreads();
    if (st != 1) {   // timed out (never expected): report once, stop
      if (tid == 0 && st == 0 && abort_flag) atomicCAS(abort_flag, 0, GEMM_WAIT_TIMEOUT);
      return;
    }
    double* zs = Zs[j & 1];
    for (int e = tid; e < TILE * PM; e += 512) {
      const int kk = e & (TILE - 1), p = e >> 7;
      zs[kk * PM + p] = p < P ? Z[(long long)j * TILE + kk + (long long)p * ldz] : 0.0;
    }
    __syncthreads();
    const double* zh = zs + h * KQ * PM;
#pragma unroll   // lv stays in registers only when every index is a constant
    for (int k = 0; k < KQ; ++k) {
      const double x = lv[k];
#pragma unroll
      for (int p = 0; p < PM; ++p) acc[p] = fma(-x, zh[k * PM + p], acc[p]);
    }
  }
  __syncthreads();
  ts_reduce(acc, Zs[0], Zs[1], r, h);   // the full acc in quarter 0
  double* S = Zs[1];                    // acc as [k][p]
  if (h == 0) {
#pragma unroll
    for (int p = 0; p < PM; ++p) S[r * PM + p] = acc[p];
  }
  __syncthreads();
  // Z_i(r, p) = sum_k D_i(r, k) S(k, p): quarter h takes k in [h KQ, h KQ + KQ)
  double out[PM];
#pragma unroll
  for (int p = 0; p < PM; ++p) out[p] = 0.0;
  const double* sh = S + h * KQ * PM;
#pragma unroll
  for (int k = 0; k < KQ; ++k)
#pragma unroll
    for (int p = 0; p < PM; ++p) out[p] = fma(dv[k], sh[k * PM + p], out[p]);
  __syncthreads();   // every quarter has read S
  ts_reduce(out, Zs[0], Zs[1], r, h);
  // Z_i leaves through sc1 (write-through) stores, so the flag needs no L2 write-back
  // (MI355X guide, valid hand-off forms: sc1 payload, every storing wave's vmcnt(0),
  // a barrier, then one lane's flag store; the consumer keeps its agent acquire)
  if (h == 0) {
#pragma unroll
    for (int p = 0; p < PM; ++p)
      if (p < P)
        __hip_atomic_store(Z + (long long)i * TILE + r + (long long)p * ldz, out[p], __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) __hip_atomic_store(flags, i + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The skinny products on MFMA (grid: blockIdx.x = it + nit * ch; partials as
// described above): D(p, i) = sum_k R(k, p) op(M)(k, i) on v_mfma_f64_16x16x4_f64,
// p = rows of the MFMA tile (P <= PM, zero-padded), i = 128 output rows per
// workgroup (32 per wave).  TR: op(M)(k,i) = M(k,i) (k contiguous: LDS image [i][k],
// pitch 34); else op(M)(k,i) = M(i,k) (i contiguous: image [k][i], pitch 144).
// 32 k per stage, registers prefetch the next stage.  HBM-bound by design.
constexpr int SKM_GK = 32;
constexpr int SKM_PT = 34;     // [i][k] / [p][k] pitch (doubles)
constexpr int SKM_PN = 144;    // [k][i] pitch (doubles)

template <int PM, bool TR>
__device__ __forceinline__ void skm_gload(const double* Mb, long long ldm, const double* R, long long ldr,
                                          int P, int k0, int tid, double (&mv)[16], double (&rv)[PM / 8]) {
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int c = tid + 256 * u;
    if (TR) {   // column i = c >> 4, k pair (c & 15) * 2
      const int i = c >> 4, kk = (c & 15) * 2;
      const double2 v = *reinterpret_cast<const double2*>(Mb + (long long)i * ldm + k0 + kk);
      mv[2 * u] = v.x;
      mv[2 * u + 1] = v.y;
    } else {    // row k = c >> 6, i pair (c & 63) * 2
      const int kk = c >> 6, i = (c & 63) * 2;
      const double2 v = *reinterpret_cast<const double2*>(Mb + i + (long long)(k0 + kk) * ldm);
      mv[2 * u] = v.x;
      mv[2 * u + 1] = v.y;
    }
  }
#pragma unroll
  for (int u = 0; u < PM / 8; ++u) {
    const int e = tid + 256 * u;           // PM * 32 entries
    const int kk = e & (SKM_GK - 1), pp = e >> 5;
    rv[u] = (pp < P) ? R[(long long)(k0 + kk) + (long long)pp * ldr] : 0.0;
  }
}

template <int PM, bool TR>
__device__ __forceinline__ void skm_sstore(double* Ms, double* Rs, int tid, const double (&mv)[16],
                                           const double (&rv)[PM / 8]) {
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int c = tid + 256 * u;
    if (TR) {
      const int i = c >> 4, kk = (c & 15) * 2;
      *reinterpret_cast<double2*>(Ms + i * SKM_PT + kk) = make_double2(mv[2 * u], mv[2 * u + 1]);
    } else {
      const int kk = c >> 6, i = (c & 63) * 2;
      *reinterpret_cast<double2*>(Ms + kk * SKM_PN + i) = make_double2(mv[2 * u], mv[2 * u + 1]);
    }
  }
#pragma unroll
  for (int u = 0; u < PM / 8; ++u) {
    const int e = tid + 256 * u;
    const int kk = e & (SKM_GK - 1), pp = e >> 5;
    Rs[pp * SKM_PT + kk] = rv[u];
  }
}

template <int PM, bool TR>
static __global__ void __launch_bounds__(256) k_skinny_mfma(SkinnyArgs a) {
  constexpr int MIMG = TR ? TILE * SKM_PT : SKM_GK * SKM_PN;
  __shared__ __attribute__((aligned(16))) double Ms[MIMG];
  __shared__ __attribute__((aligned(16))) double Rs[PM * SKM_PT];
  if (a.abort_flag && *a.abort_flag) return;
  const int it = blockIdx.x % a.nit, ch = blockIdx.x / a.nit;
  int kt0, kt1;
  if (TR) {
    const int kbase = a.lower ? it : 0;
    kt0 = kbase + ch * a.chk;
    if (kt0 >= a.ntr) return;
    kt1 = min(kt0 + a.chk, a.ntr);
  } else {
    const int kend = a.lower ? it + 1 : a.ntr;
    kt0 = ch * a.chk;
    if (kt0 >= kend) return;
    kt1 = min(kt0 + a.chk, kend);
  }
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int P = a.P;
  const double* Mb = TR ? a.M + (long long)(it * TILE) * a.ldm : a.M + (long long)it * TILE;
  constexpr int NPT = PM / 16;
  d4 acc[NPT][2];
#pragma unroll
  for (int u = 0; u < NPT; ++u) acc[u][0] = acc[u][1] = d4{0.0, 0.0, 0.0, 0.0};
  double mv[16];
  double rv[PM / 8];
  const int kb = kt0 * TILE, ke = kt1 * TILE;
  skm_gload<PM, TR>(Mb, a.ldm, a.R, a.ldr, P, kb, tid, mv, rv);
  for (int k0 = kb; k0 < ke; k0 += SKM_GK) {
    __syncthreads();
    skm_sstore<PM, TR>(Ms, Rs, tid, mv, rv);
    __syncthreads();
    if (k0 + SKM_GK < ke) skm_gload<PM, TR>(Mb, a.ldm, a.R, a.ldr, P, k0 + SKM_GK, tid, mv, rv);
#pragma unroll
    for (int s = 0; s < SKM_GK / 4; ++s) {
      const int kk = 4 * s + (lane >> 4);
      double bf[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int i = wave * 32 + j * 16 + (lane & 15);
        bf[j] = TR ? Ms[i * SKM_PT + kk] : Ms[kk * SKM_PN + i];
      }
#pragma unroll
      for (int u = 0; u < NPT; ++u) {
        const double af = Rs[(u * 16 + (lane & 15)) * SKM_PT + kk];
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[u][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(af, bf[j], acc[u][j], 0, 0, 0);
      }
    }
  }
  double* out = a.part + (long long)ch * a.pstride + it * TILE;
#pragma unroll
  for (int u = 0; u < NPT; ++u)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int pp = u * 16 + mfma64_row(lane, r);
        const int i = wave * 32 + j * 16 + (lane & 15);
        if (pp < P) out[i + (long long)pp * a.ldp] = acc[u][j][r];
      }
}

// out[i + p*ldp] = sum_{ch < nch(i)} part[ch][i + p*ldp], fixed order
// nch(i) for the n-kernel (lower): ceil((it+1)/CH); t-kernel lower: ceil((ntr-it)/CH)
static __global__ void k_reduce_chunks(const double* part, long long pstride, double* out,
                                long long ldp, int P, int nrows, int ntr, int mode,
                                const int* abort_flag, int chk) {
  if (abort_flag && *abort_flag) return;
  long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (long long)nrows * P) return;
  int i = (int)(e % nrows), p = (int)(e / nrows);
  int it = i / TILE;
  int nch;
  if (mode == 0) nch = (it + chk) / chk;                 // lower, n-kernel
  else if (mode == 1) nch = (ntr - it + chk - 1) / chk;  // lower, t-kernel
  else nch = (ntr + chk - 1) / chk;                      // full
  double s = 0.0;
  for (int ch = 0; ch < nch; ++ch) s += part[ch * pstride + i + (long long)p * ldp];
  out[i + (long long)p * ldp] = s;
}

// ---------------------------------------------------------------------------
// Gram: part[blk][a + b P] = sum_{rows in blk} Z(row,a) Z(row,b); rows 256 per block.
// Any P: blockIdx.y enumerates pairs of 32-column chunks (ca <= cb); a pair of
// different chunks writes its block and the mirror.  With P <= 32 there is one pair
// and the sums are those of the single-chunk form.
// ---------------------------------------------------------------------------
static __global__ void __launch_bounds__(256) k_gram(const double* Z, long long ldz, int P, int nrows,
                                              double* part, const int* abort_flag) {
  __shared__ double za[256 * (SK_PMAX + 1)];
  __shared__ double zb[256 * (SK_PMAX + 1)];
  if (abort_flag && *abort_flag) return;
  const int tid = threadIdx.x;
  const int r0 = blockIdx.x * 256;
  const int nch = (P + SK_PMAX - 1) / SK_PMAX;
  int pi = blockIdx.y, ca = 0;
  while (pi >= nch - ca) { pi -= nch - ca; ++ca; }
  const int cb = ca + pi;
  const int a0 = ca * SK_PMAX, pa = min(SK_PMAX, P - a0);
  const int b0 = cb * SK_PMAX, pb = min(SK_PMAX, P - b0);
  for (int e = tid; e < 256 * pa; e += 256) {
    int rr = e & 255, p = e >> 8;
    int row = r0 + rr;
    za[rr * (SK_PMAX + 1) + p] = (row < nrows) ? Z[row + (long long)(a0 + p) * ldz] : 0.0;
  }
  if (cb != ca)
    for (int e = tid; e < 256 * pb; e += 256) {
      int rr = e & 255, p = e >> 8;
      int row = r0 + rr;
      zb[rr * (SK_PMAX + 1) + p] = (row < nrows) ? Z[row + (long long)(b0 + p) * ldz] : 0.0;
    }
  __syncthreads();
  const double* zy = cb != ca ? zb : za;
  double* out = part + (long long)blockIdx.x * P * P;
  for (int e = tid; e < pa * pb; e += 256) {
    int x = e % pa, y = e / pa;
    double s = 0.0;
    for (int rr = 0; rr < 256; ++rr) s = fma(za[rr * (SK_PMAX + 1) + x], zy[rr * (SK_PMAX + 1) + y], s);
    out[(a0 + x) + (long long)(b0 + y) * P] = s;
    if (cb != ca) out[(b0 + y) + (long long)(a0 + x) * P] = s;
  }
}

// Y(i, :) = Z(i, :) x T for any P (k_apply_small holds a row of Z in registers, P <= 32)
static __global__ void k_apply_big(const double* Z, long long ldz, int P, const double* T, int Pout, double* Y,
                                   long long ldy, int nrows, const int* abort_flag) {
  if (abort_flag && *abort_flag) return;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nrows) return;
  for (int o = 0; o < Pout; ++o) {
    double s = 0.0;
    for (int p = 0; p < P; ++p) s = fma(Z[i + (long long)p * ldz], T[p + o * P], s);
    Y[i + (long long)o * ldy] = s;
  }
}

// out[j] = sum_w part[w*len + j]; one block per j, fixed tree -> reproducible
static __global__ void __launch_bounds__(256) k_reduce_rows(const double* part, int nw, int len,
                                                     double* out) {
  __shared__ double red[256];
  const int j = blockIdx.x, tid = threadIdx.x;
  double s = 0.0;
  for (int w = tid; w < nw; w += 256) s += part[(long long)w * len + j];
  red[tid] = s;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if (tid < off) red[tid] += red[tid + off];
    __syncthreads();
  }
  if (tid == 0) out[j] = red[0];
}

// Y(i, :) = Z(i, :) x T   (T P x Pout column-major, Z/Y column-major)
static __global__ void k_apply_small(const double* Z, long long ldz, int P, const double* T,
                              int Pout, double* Y, long long ldy, int nrows,
                              const int* abort_flag) {
  if (abort_flag && *abort_flag) return;
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nrows) return;
  double z[SK_PMAX];
#pragma unroll
  for (int p = 0; p < SK_PMAX; ++p) z[p] = (p < P) ? Z[i + (long long)p * ldz] : 0.0;
  for (int o = 0; o < Pout; ++o) {
    double s = 0.0;
#pragma unroll
    for (int p = 0; p < SK_PMAX; ++p)
      if (p < P) s = fma(z[p], T[p + o * P], s);
    Y[i + (long long)o * ldy] = s;
  }
}

// colsum2[j] = sum_i V(i, j)^2  (one wave per column)
static __global__ void __launch_bounds__(256) k_colnorm2(const double* V, long long ldv, int nrows,
                                                  int ncols, double* out) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int j = blockIdx.x * 4 + wave;
  if (j >= ncols) return;
  const double* col = V + (long long)j * ldv;
  double s = 0.0;
  for (int i = lane; i < nrows; i += 64) s = fma(col[i], col[i], s);
  for (int off = 32; off > 0; off >>= 1) s += __shfl_down(s, off, 64);
  if (lane == 0) out[j] = s;
}

// ---------------------------------------------------------------------------
// gradient contraction over the lower tiles of A^-1:
//   M(i,j) = Ainv(i,j) - sum_p Wa(i,p) Wa(j,p)     (Wa = [sqrt(c) alpha, W], q+1 cols,
//            column-major, ld = ldw)
//   off-diagonal (i>j):  accE += M E,  acc_k += M E (x_ik - x_jk)^2 / delta_k^2
//   diagonal:            accT += M(i,i)
// E recomputed from the scaled points (no n x n exp cache, no n x n dA).
// part[blk][0:d] = acc_k, [d] = accE, [d+1] = accT, [d+2] = accR = sum_i M(i,i) r_i
// (rdiag non-null: the reference's sigma gradient subtracts diag(r) from A for every
// kernel, _emulatoroptimise.py:476-478, while make_A adds r only for alt-nugget)
// Slabs: the launch covers lower tiles blk0 .. blk0 + gridDim.x - 1 (row-major tile
// order) and Ainv holds global rows row0 .. (A^-1 row gi at Ainv[gi - row0]).
// ---------------------------------------------------------------------------
template <int DMAX, int QMAX>
static __global__ void __launch_bounds__(256) k_contract(const double* Ainv, long long lda,
                                                  const double* xw, int d,
                                                  const double* Wa, long long ldw, int q1,
                                                  int n_valid, double* part,
                                                  const int* abort_flag, int blk0 = 0,
                                                  long long row0 = 0, const double* rdiag = nullptr,
                                                  int csplit = 1) {
  __shared__ double xs[TILE * DMAX];
  __shared__ double ws[TILE * QMAX];
  __shared__ double red[4 * (DMAX + 3)];
  if (abort_flag && *abort_flag) return;
  int ti, tj;
  // csplit workgroups per tile (launches of few tiles), each a contiguous share of its
  // columns with a partial of its own: part row blk * csplit + share
  const int share = (int)blockIdx.x % csplit;
  const int blk = blk0 + (int)blockIdx.x / csplit;
  tri_decode(blk, ti, tj);
  const int tid = threadIdx.x;
  // zero-padded to DMAX / QMAX: the padded terms are exact no-ops (fma(-0, 0, m) = m,
  // s + 0 = s), so the inner loops carry no per-dimension branch
  for (int e = tid; e < TILE * DMAX; e += 256) {
    const int c = e / DMAX, k = e - c * DMAX;
    xs[e] = k < d ? xw[(long long)(tj * TILE + c) * d + k] : 0.0;
  }
  for (int e = tid; e < TILE * QMAX; e += 256) {
    const int c = e / QMAX, k = e - c * QMAX;
    ws[e] = k < q1 ? Wa[(long long)(tj * TILE + c) + (long long)k * ldw] : 0.0;
  }
  const int r = tid & (TILE - 1);
  const int gi = ti * TILE + r;
  double xi[DMAX], wi[QMAX], acc[DMAX];
#pragma unroll
  for (int k = 0; k < DMAX; ++k) {
    xi[k] = (k < d) ? xw[(long long)gi * d + k] : 0.0;
    acc[k] = 0.0;
  }
#pragma unroll
  for (int k = 0; k < QMAX; ++k) wi[k] = (k < q1) ? Wa[gi + (long long)k * ldw] : 0.0;
  double accE = 0.0, accT = 0.0, accR = 0.0;
  const double ri = (rdiag && gi < n_valid && ti == tj) ? rdiag[gi] : 0.0;
  __syncthreads();
  if (gi < n_valid) {
    const double* acol = Ainv + (gi - row0) + (long long)tj * TILE * lda;
    const int cw = TILE / csplit, cbeg = share * cw;
    const int cend = min(min((ti == tj) ? r + 1 : TILE, n_valid - tj * TILE), cbeg + cw);
    // columns c = (tid >> 7) + 2u, four loads in flight ahead of the arithmetic
    for (int c0 = cbeg + (tid >> 7); c0 < cend; c0 += 8) {
      double mv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int c = c0 + 2 * u;
        mv[u] = (c < cend) ? acol[(long long)c * lda] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int c = c0 + 2 * u;
        if (c >= cend) break;
        const int gj = tj * TILE + c;
        double mij = mv[u];
#pragma unroll
        for (int k = 0; k < QMAX; ++k) mij = fma(-wi[k], ws[c * QMAX + k], mij);
        double df2[DMAX];
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < DMAX; ++k) {
          const double df = xi[k] - xs[c * DMAX + k];
          df2[k] = df * df;
          s += df2[k];
        }
        // the diagonal entry goes to accT; adding the zeros the selects leave is exact
        const bool dg = gj == gi;
        accT += dg ? mij : 0.0;
        accR += dg ? mij * ri : 0.0;
        const double me = dg ? 0.0 : mij * exp(-s);
        accE += me;
#pragma unroll
        for (int k = 0; k < DMAX; ++k) acc[k] = fma(me, df2[k], acc[k]);
      }
    }
  }
  // block reduction, fixed order
  const int nv = d + 3;
  const int lane = tid & 63, wave = tid >> 6;
  for (int k = 0; k < nv; ++k) {
    double v = 0.0;
#pragma unroll
    for (int kk = 0; kk < DMAX; ++kk)
      if (kk == k) v = acc[kk];
    if (k == d) v = accE;
    if (k == d + 1) v = accT;
    if (k == d + 2) v = accR;
    for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
    if (lane == 0) red[wave * (DMAX + 3) + k] = v;
  }
  __syncthreads();
  if (tid < nv) {
    const double s = (red[tid] + red[(DMAX + 3) + tid]) +
                     (red[2 * (DMAX + 3) + tid] + red[3 * (DMAX + 3) + tid]);
    part[((long long)blk * csplit + share) * nv + tid] = s;
  }
}

// k_contract for any d and q (d > 32 or q + 1 > 33): the same sums, with the
// coordinates and the columns of Wa staged through LDS 32 at a time.  Per pass over
// a chunk of 32 per-dimension accumulators, each thread walks its 64 columns in four
// groups of 16 (distances, M(i,j), then M E times the chunk's squared differences);
// passes beyond the first recompute E (d / 32 passes in all).
constexpr int CW_CH = 32;
static __global__ void __launch_bounds__(256) k_contract_wide(const double* Ainv, long long lda,
                                                             const double* xw, int d,
                                                             const double* Wa, long long ldw, int q1,
                                                             int n_valid, double* part,
                                                             const int* abort_flag, int blk0,
                                                             long long row0, const double* rdiag) {
  __shared__ double st[TILE * CW_CH];
  __shared__ double red[4 * CW_CH];
  if (abort_flag && *abort_flag) return;
  int ti, tj;
  const int blk = blk0 + (int)blockIdx.x;
  tri_decode(blk, ti, tj);
  const int tid = threadIdx.x, h = tid >> 7, lane = tid & 63, wave = tid >> 6;
  const int r = tid & (TILE - 1);
  const int gi = ti * TILE + r;
  const bool rv = gi < n_valid;
  const int cend = rv ? min((ti == tj) ? r + 1 : TILE, n_valid - tj * TILE) : 0;
  const double ri = (rdiag && rv && ti == tj) ? rdiag[gi] : 0.0;
  const int nv = d + 3;
  double accE = 0.0, accT = 0.0, accR = 0.0;
  // wave sum of v into red[wave][k]; the caller adds the four waves in fixed order
  auto block_sum = [&](double v, int k) {
    for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
    if (lane == 0) red[wave * CW_CH + k] = v;
  };
  for (int a0 = 0; a0 < d; a0 += CW_CH) {
    double acc[CW_CH];
#pragma unroll
    for (int k = 0; k < CW_CH; ++k) acc[k] = 0.0;
    for (int cg = 0; cg < 4; ++cg) {
      double sd[16], m[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int c = h + 2 * (cg * 16 + u);
        sd[u] = 0.0;
        m[u] = (c < cend) ? Ainv[(gi - row0) + (long long)(tj * TILE + c) * lda] : 0.0;
      }
      for (int k0 = 0; k0 < d; k0 += CW_CH) {   // squared distances over every dimension
        __syncthreads();
        for (int e = tid; e < TILE * CW_CH; e += 256) {
          const int c = e / CW_CH, k = e - c * CW_CH;
          st[e] = k0 + k < d ? xw[(long long)(tj * TILE + c) * d + k0 + k] : 0.0;
        }
        double xi[CW_CH];
#pragma unroll
        for (int k = 0; k < CW_CH; ++k) xi[k] = (k0 + k < d) ? xw[(long long)gi * d + k0 + k] : 0.0;
        __syncthreads();
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          const int c = h + 2 * (cg * 16 + u);
#pragma unroll
          for (int k = 0; k < CW_CH; ++k) {
            const double df = xi[k] - st[c * CW_CH + k];
            sd[u] += df * df;
          }
        }
      }
      for (int p0 = 0; p0 < q1; p0 += CW_CH) {  // M(i,j) = A^-1(i,j) - sum_p Wa(i,p) Wa(j,p)
        __syncthreads();
        for (int e = tid; e < TILE * CW_CH; e += 256) {
          const int c = e / CW_CH, k = e - c * CW_CH;
          st[e] = p0 + k < q1 ? Wa[(long long)(tj * TILE + c) + (long long)(p0 + k) * ldw] : 0.0;
        }
        double wi[CW_CH];
#pragma unroll
        for (int k = 0; k < CW_CH; ++k) wi[k] = (p0 + k < q1) ? Wa[gi + (long long)(p0 + k) * ldw] : 0.0;
        __syncthreads();
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          const int c = h + 2 * (cg * 16 + u);
#pragma unroll
          for (int k = 0; k < CW_CH; ++k) m[u] = fma(-wi[k], st[c * CW_CH + k], m[u]);
        }
      }
      // M E off the diagonal; trace terms once (first pass)
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int c = h + 2 * (cg * 16 + u);
        const bool valid = c < cend, dg = tj * TILE + c == gi;
        if (a0 == 0) {
          accT += (valid && dg) ? m[u] : 0.0;
          accR += (valid && dg) ? m[u] * ri : 0.0;
        }
        sd[u] = (valid && !dg) ? m[u] * exp(-sd[u]) : 0.0;   // now M E
        if (a0 == 0) accE += sd[u];
      }
      // this pass's dimensions: acc_k += M E (x_ik - x_jk)^2
      __syncthreads();
      for (int e = tid; e < TILE * CW_CH; e += 256) {
        const int c = e / CW_CH, k = e - c * CW_CH;
        st[e] = a0 + k < d ? xw[(long long)(tj * TILE + c) * d + a0 + k] : 0.0;
      }
      double xi[CW_CH];
#pragma unroll
      for (int k = 0; k < CW_CH; ++k) xi[k] = (a0 + k < d) ? xw[(long long)gi * d + a0 + k] : 0.0;
      __syncthreads();
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int c = h + 2 * (cg * 16 + u);
#pragma unroll
        for (int k = 0; k < CW_CH; ++k) {
          const double df = xi[k] - st[c * CW_CH + k];
          acc[k] = fma(sd[u], df * df, acc[k]);
        }
      }
    }
    // this pass's per-dimension sums
    const int kn = min(CW_CH, d - a0);
#pragma unroll
    for (int k = 0; k < CW_CH; ++k)
      if (k < kn) block_sum(acc[k], k);
    __syncthreads();
    if (tid < kn)
      part[(long long)blk * nv + a0 + tid] =
          (red[tid] + red[CW_CH + tid]) + (red[2 * CW_CH + tid] + red[3 * CW_CH + tid]);
    __syncthreads();
  }
  block_sum(accE, 0);
  block_sum(accT, 1);
  block_sum(accR, 2);
  __syncthreads();
  if (tid < 3)
    part[(long long)blk * nv + d + tid] =
        (red[tid] + red[CW_CH + tid]) + (red[2 * CW_CH + tid] + red[3 * CW_CH + tid]);
}

// ---------------------------------------------------------------------------
// sensitivity pair sums (reference sensitivity/_sensitivityclasses.py:90-102 Rtt,
// :599-626 P_prod / Pw): J Gaussian pair kernels on the raw training inputs x,
//   K_j(k,l) = u_j[k] u_j[l] exp(-sum_i w_j[i] (x_ki - x_li)^2),
// never stored: each is contracted with A^-1 (lower tiles; off-diagonal pairs
// twice) and applied to Z (n x p, column-major): V = K_j Z, quad = Z^T V.
// grid (NB, J, CS): row block ti of 128 rows, column slice z of CS (each slice a
// multiple of SP_CT columns), two threads per row split the slice's columns.
// part[((ti*CS + z)*4 + wave) * ldp + j*(1+p*p)] = trace part, then the p*p quad part.
// Z columns zc0 .. zc0 + pc (pc <= PMAX) per launch: V = K Z[:, zc0:] and quad(a, zc0 + b)
// for every a < p; the host covers any p in such column chunks (the trace part is the
// same in each).
// ---------------------------------------------------------------------------
constexpr int SP_CT = 64;   // columns staged in LDS per pass
template <int DMAX, int PMAX>
static __global__ void __launch_bounds__(256) k_sense_pairs(const double* Ainv, long long lda, const double* x,
                                                           int d, const double* w, const double* u,
                                                           long long ldu, const double* Z, long long ldz,
                                                           int p, int n_valid, int cslice, double* part,
                                                           long long ldp, int zc0, int pc) {
  __shared__ double xs[SP_CT * DMAX];
  __shared__ double zs[SP_CT * PMAX];
  __shared__ double us[SP_CT];
  const int ti = blockIdx.x, j = blockIdx.y, tid = threadIdx.x;
  const int r = tid & (TILE - 1), h = tid >> 7;
  const int gi = ti * TILE + r;
  const bool rv = gi < n_valid;
  double xi[DMAX], wj[DMAX], v[PMAX];
#pragma unroll
  for (int k = 0; k < DMAX; ++k) {
    xi[k] = (k < d && rv) ? x[(long long)gi * d + k] : 0.0;
    wj[k] = (k < d) ? w[j * d + k] : 0.0;
  }
#pragma unroll
  for (int q = 0; q < PMAX; ++q) v[q] = 0.0;
  const double ui = rv ? u[j * ldu + gi] : 0.0;
  double acc = 0.0;
  const int cbeg = blockIdx.z * cslice, cfin = min(n_valid, cbeg + cslice);
  for (int c0 = cbeg; c0 < cfin; c0 += SP_CT) {
    __syncthreads();
    // zero-padded to DMAX / PMAX, so the loops below carry no per-dimension branch
    for (int e = tid; e < SP_CT * DMAX; e += 256) {
      const int c = e / DMAX, k = e - c * DMAX, g = c0 + c;
      xs[e] = (k < d && g < n_valid) ? x[(long long)g * d + k] : 0.0;
    }
    for (int e = tid; e < SP_CT * PMAX; e += 256) {   // Z columns zc0 .. zc0 + pc
      const int c = e % SP_CT, k = e / SP_CT, g = c0 + c;
      zs[c * PMAX + k] = (k < pc && g < n_valid) ? Z[g + (long long)(zc0 + k) * ldz] : 0.0;
    }
    if (tid < SP_CT) us[tid] = (c0 + tid < n_valid) ? u[j * ldu + c0 + tid] : 0.0;
    __syncthreads();
    if (rv) {
      const int cend = min(SP_CT, cfin - c0);
      for (int c = h; c < cend; c += 2) {
        const int gj = c0 + c;
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < DMAX; ++k) {
          const double df = xi[k] - xs[c * DMAX + k];
          s = fma(wj[k] * df, df, s);
        }
        const double K = ui * us[c] * exp(-s);
#pragma unroll
        for (int q = 0; q < PMAX; ++q) v[q] = fma(K, zs[c * PMAX + q], v[q]);
        // lower triangle only (the upper one is not stored): a masked load, then an
        // exact no-op fma(0, 0, acc) above the diagonal
        const double av = gj <= gi ? Ainv[gi + (long long)gj * lda] : 0.0;
        acc = fma(gj < gi ? 2.0 * K : (gj == gi ? K : 0.0), av, acc);
      }
    }
  }
  // per-wave partials: trace, then quad(a, b) = sum_rows Z(row, a) V(row, b)
  const int lane = tid & 63, wave = tid >> 6;
  double* out = part + (long long)((ti * gridDim.z + blockIdx.z) * 4 + wave) * ldp + (long long)j * (1 + p * p);
  double t = acc;
  for (int off = 32; off > 0; off >>= 1) t += __shfl_down(t, off, 64);
  if (lane == 0) out[0] = t;
  for (int a = 0; a < p; ++a) {
    const double za = rv ? Z[gi + (long long)a * ldz] : 0.0;
#pragma unroll
    for (int b = 0; b < PMAX; ++b) {
      if (b < pc) {
        double s = za * v[b];
        for (int off = 32; off > 0; off >>= 1) s += __shfl_down(s, off, 64);
        if (lane == 0) out[1 + a * p + zc0 + b] = s;
      }
    }
  }
}

// k_sense_pairs for any d (> 32): the slice's columns are staged SPW_CT at a time and
// their coordinates SPW_DC dimensions at a time (LDS), each thread keeping the running
// squared distances of its SPW_CT / 2 columns; the distances accumulate dimension by
// dimension in the same fma order as k_sense_pairs, so the pair values are the same.
constexpr int SPW_CT = 32, SPW_DC = 32;
template <int PMAX>
static __global__ void __launch_bounds__(256) k_sense_pairs_wide(const double* Ainv, long long lda, const double* x,
                                                                int d, const double* w, const double* u,
                                                                long long ldu, const double* Z, long long ldz,
                                                                int p, int n_valid, int cslice, double* part,
                                                                long long ldp, int zc0, int pc) {
  __shared__ double xs[SPW_CT * SPW_DC];
  __shared__ double wsh[SPW_DC];
  __shared__ double zs[SPW_CT * PMAX];
  __shared__ double us[SPW_CT];
  constexpr int CM = SPW_CT / 2;   // columns per thread per stage
  const int ti = blockIdx.x, j = blockIdx.y, tid = threadIdx.x;
  const int r = tid & (TILE - 1), h = tid >> 7;
  const int gi = ti * TILE + r;
  const bool rv = gi < n_valid;
  double v[PMAX];
#pragma unroll
  for (int q = 0; q < PMAX; ++q) v[q] = 0.0;
  const double ui = rv ? u[j * ldu + gi] : 0.0;
  double acc = 0.0;
  const int cbeg = blockIdx.z * cslice, cfin = min(n_valid, cbeg + cslice);
  for (int c0 = cbeg; c0 < cfin; c0 += SPW_CT) {
    double sd[CM];
#pragma unroll
    for (int m = 0; m < CM; ++m) sd[m] = 0.0;
    for (int k0 = 0; k0 < d; k0 += SPW_DC) {
      __syncthreads();
      for (int e = tid; e < SPW_CT * SPW_DC; e += 256) {
        const int c = e / SPW_DC, k = e - c * SPW_DC, g = c0 + c;
        xs[e] = (k0 + k < d && g < n_valid) ? x[(long long)g * d + k0 + k] : 0.0;
      }
      if (tid < SPW_DC) wsh[tid] = (k0 + tid < d) ? w[j * d + k0 + tid] : 0.0;
      __syncthreads();
      double xi[SPW_DC];
#pragma unroll
      for (int k = 0; k < SPW_DC; ++k) xi[k] = (k0 + k < d && rv) ? x[(long long)gi * d + k0 + k] : 0.0;
#pragma unroll
      for (int m = 0; m < CM; ++m) {
        const int c = h + 2 * m;
#pragma unroll
        for (int k = 0; k < SPW_DC; ++k) {
          const double df = xi[k] - xs[c * SPW_DC + k];
          sd[m] = fma(wsh[k] * df, df, sd[m]);
        }
      }
    }
    __syncthreads();
    for (int e = tid; e < SPW_CT * PMAX; e += 256) {   // Z columns zc0 .. zc0 + pc
      const int c = e % SPW_CT, k = e / SPW_CT, g = c0 + c;
      zs[c * PMAX + k] = (k < pc && g < n_valid) ? Z[g + (long long)(zc0 + k) * ldz] : 0.0;
    }
    if (tid < SPW_CT) us[tid] = (c0 + tid < n_valid) ? u[j * ldu + c0 + tid] : 0.0;
    __syncthreads();
    if (rv) {
#pragma unroll
      for (int m = 0; m < CM; ++m) {
        const int c = h + 2 * m, gj = c0 + c;
        if (gj < cfin) {
          const double K = ui * us[c] * exp(-sd[m]);
#pragma unroll
          for (int q = 0; q < PMAX; ++q) v[q] = fma(K, zs[c * PMAX + q], v[q]);
          const double av = gj <= gi ? Ainv[gi + (long long)gj * lda] : 0.0;
          acc = fma(gj < gi ? 2.0 * K : (gj == gi ? K : 0.0), av, acc);
        }
      }
    }
  }
  const int lane = tid & 63, wave = tid >> 6;
  double* out = part + (long long)((ti * gridDim.z + blockIdx.z) * 4 + wave) * ldp + (long long)j * (1 + p * p);
  double t = acc;
  for (int off = 32; off > 0; off >>= 1) t += __shfl_down(t, off, 64);
  if (lane == 0) out[0] = t;
  for (int a = 0; a < p; ++a) {
    const double za = rv ? Z[gi + (long long)a * ldz] : 0.0;
#pragma unroll
    for (int b = 0; b < PMAX; ++b) {
      if (b < pc) {
        double s = za * v[b];
        for (int off = 32; off > 0; off >>= 1) s += __shfl_down(s, off, 64);
        if (lane == 0) out[1 + a * p + zc0 + b] = s;
      }
    }
  }
}

// Gauss transform over the training inputs (main / interaction effects,
// _sensitivityclasses.py:628-633 Tw summed against e):
//   out[t] = sum_k a[k] exp(-sum_s c[s] (Y[t,s] - x[k, dims[s]])^2),  one wave per t
struct GaussArgs {
  const double* x;
  const double* a;
  const double* Y;
  double* out;
  int d, n, m, ns;
  int dims[4];
  double c[4];
};
static __global__ void __launch_bounds__(256) k_gauss_transform(GaussArgs g) {
  const int lane = threadIdx.x & 63;
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= g.m) return;
  double y[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) y[s] = s < g.ns ? g.Y[t * g.ns + s] : 0.0;
  double acc = 0.0;
  for (int k = lane; k < g.n; k += 64) {
    double q = 0.0;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      if (s < g.ns) {
        const double df = y[s] - g.x[(long long)k * g.d + g.dims[s]];
        q = fma(g.c[s] * df, df, q);
      }
    }
    acc = fma(g.a[k], exp(-q), acc);
  }
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_down(acc, off, 64);
  if (lane == 0) g.out[t] = acc;
}

// xw(i,k) = X(i,k) / delta_k  for i < n, 0 for padded rows
static __global__ void k_scale_points(const double* X, const double* inv_delta, int d, int n,
                               int n_pad, double* xw) {
  long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (long long)n_pad * d) return;
  int i = (int)(e / d), k = (int)(e % d);
  xw[e] = (i < n) ? X[e] * inv_delta[k] : 0.0;
}

// The augmented tile row of the fused Cholesky: [f H]^T as rows under the matrix
// (TILE x n_pad, ld = TILE): Faug(p, i) = F(i, p) for p < P, rows P..127 zero.  The
// sweep leaves (L^-1 [f H])^T there (build_plan).
static __global__ void k_aug_init(const double* F, long long ldf, int P, long long n_pad, double* Faug) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n_pad * TILE) return;
  const int p = (int)(e & (TILE - 1));
  const long long i = e >> 7;
  Faug[e] = p < P ? F[i + (long long)p * ldf] : 0.0;
}

// Z(i, p) = Faug(p, i): the augmented row back as a column-major n_pad x P block
static __global__ void k_aug_to_cols(const double* Faug, int P, long long n_pad, double* Z, long long ldz) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n_pad * P) return;
  const long long i = e % n_pad;
  const int p = (int)(e / n_pad);
  Z[i + (long long)p * ldz] = Faug[p + i * TILE];
}

// set tile (t,t) of M to the identity for t >= t0 (padding blocks of the inverse)
static __global__ void k_identity_tiles(double* M, long long ld, int t0) {
  const int t = t0 + blockIdx.x;
  double* base = M + (long long)t * TILE * (ld + 1);
  for (int e = threadIdx.x; e < TILE * TILE; e += blockDim.x) {
    int i = e & (TILE - 1), j = e >> 7;
    base[i + (long long)j * ld] = (i == j) ? 1.0 : 0.0;
  }
}

// zero the strictly-upper part of every diagonal tile (t,t) of a factored matrix, so
// a G_KEND_TI GEMM can read it as the triangle L
static __global__ void k_zero_upper_diag_tiles(double* M, long long ld) {
  double* base = M + (long long)blockIdx.x * TILE * (ld + 1);
  for (int e = threadIdx.x; e < TILE * TILE; e += blockDim.x) {
    int i = e & (TILE - 1), j = e >> 7;
    if (i < j) base[i + (long long)j * ld] = 0.0;
  }
}

// z_i = sum_{j<s} 0.5 (e_i - Y(i,j))^2, Y column-major (ld), one thread per row:
// consecutive threads read consecutive rows of each column (coalesced).  The sum
// runs in the reference's order j = 0..s-1 (noise_fit.py:134-137).
static __global__ void __launch_bounds__(256) k_noise_sq(const double* Y, long long ld, int s,
                                                         const double* e, int m, double* z) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  const double ei = e[i];
  double acc = 0.0;
  for (int j = 0; j < s; ++j) {
    const double r = ei - Y[i + (long long)j * ld];
    acc += 0.5 * (r * r);
  }
  z[i] = acc;
}

// ---- oLHC "maximin" selection (design_inputs.py:54-67): np.argmin(pdist(xt, 'sqeuclidean'))
// per candidate design, xt = [x_k; fextra] (m = n + ne points).  Ordering key of a pair is
// (distance, condensed index), NaN distances first -- np.argmin's first occurrence of the
// minimum, with NaN as the minimum.
__device__ __forceinline__ bool lhc_less(double a, long long ia, double b, long long ib) {
  return a < b || (a == b && ia < ib);
}

__device__ __forceinline__ void lhc_block_min(double& bd, long long& bi, double* sd, long long* si) {
  for (int off = 32; off > 0; off >>= 1) {
    const double od = __shfl_down(bd, off, 64);
    const long long oi = __shfl_down(bi, off, 64);
    if (lhc_less(od, oi, bd, bi)) { bd = od; bi = oi; }
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) { sd[w] = bd; si[w] = bi; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 1; k < (int)(blockDim.x >> 6); ++k)
      if (lhc_less(sd[k], si[k], bd, bi)) { bd = sd[k]; bi = si[k]; }
  }
}

// One block per (tile of LHC_R consecutive rows i, design k): rows [row0 + x R, +R) against
// every j > i.  Each thread walks j = i0+1+tid, +256, ..., loads point j once and forms the
// distances of all R rows from it (row points staged in LDS, read as broadcasts).  Point j
// is row j of design k for j < n, else row j-n of E.  The squared distance is summed over
// dimensions in order with separate multiply and add (no FMA), as scipy's pdist does, so
// every distance is bit-identical to the host's.  Writes the tile's (min, index).
// kLds = false (dim above LHC_LDS_DIM): the row points are read from global memory instead.
constexpr int LHC_R = 8;
constexpr int LHC_LDS_DIM = 512;
template <bool kLds>
static __global__ void __launch_bounds__(256) k_lhc_rowmin(const double* __restrict__ D, long long dstride,
                                                           int n, const double* __restrict__ E, int ne,
                                                           int dim, int row0, int row_end,
                                                           double* __restrict__ out_d,
                                                           long long* __restrict__ out_i) {
#pragma clang fp contract(off)
  extern __shared__ double lhc_sm[];  // LHC_R * dim row points
  __shared__ double sd[4];
  __shared__ long long si[4];
  const int m = n + ne;
  const double* Dk = D + (long long)blockIdx.y * dstride;
  const int i0 = row0 + (int)blockIdx.x * LHC_R;
  const int nr = min(LHC_R, row_end - i0);
  const double* prow[LHC_R];
#pragma unroll
  for (int r = 0; r < LHC_R; ++r) {
    const int i = min(i0 + r, m - 1);
    prow[r] = i < n ? Dk + (long long)i * dim : E + (long long)(i - n) * dim;
  }
  if (kLds) {
    for (int t = threadIdx.x; t < nr * dim; t += blockDim.x) {
      const int r = t / dim, k = t - r * dim, i = i0 + r;
      lhc_sm[t] = i < n ? Dk[(long long)i * dim + k] : E[(long long)(i - n) * dim + k];
    }
    __syncthreads();
  }
  double bd = __builtin_inf();
  long long bi = 0x7fffffffffffffffLL;
  double s[LHC_R];
  for (int j = i0 + 1 + (int)threadIdx.x; j < m; j += blockDim.x) {
    const double* pj = j < n ? Dk + (long long)j * dim : E + (long long)(j - n) * dim;
#pragma unroll
    for (int r = 0; r < LHC_R; ++r) s[r] = 0.0;
    for (int k = 0; k < dim; ++k) {
      const double xj = pj[k];
#pragma unroll
      for (int r = 0; r < LHC_R; ++r) {
        const double t = (kLds ? lhc_sm[r * dim + k] : prow[r][k]) - xj;
        s[r] = s[r] + t * t;
      }
    }
#pragma unroll
    for (int r = 0; r < LHC_R; ++r) {
      const int i = i0 + r;
      if (r < nr && j > i) {
        const double v = (s[r] != s[r]) ? -__builtin_inf() : s[r];
        const long long idx = (long long)m * i - (long long)i * (i + 1) / 2 + (j - i - 1);
        if (lhc_less(v, idx, bd, bi)) { bd = v; bi = idx; }
      }
    }
  }
  lhc_block_min(bd, bi, sd, si);
  if (threadIdx.x == 0) {
    const long long o = (long long)blockIdx.y * gridDim.x + blockIdx.x;
    out_d[o] = bd;
    out_i[o] = bi;
  }
}

// One block per design: the minimum over its nb tile results, and over the (design
// independent) fextra-fextra minimum (fd, fi) when given.  Writes the condensed index
// (and the distance key, when out_d is given).
static __global__ void __launch_bounds__(256) k_lhc_reduce(const double* __restrict__ in_d,
                                                           const long long* __restrict__ in_i, int nb,
                                                           const double* fd, const long long* fi,
                                                           double* out_d, long long* __restrict__ out_i) {
  __shared__ double sd[4];
  __shared__ long long si[4];
  double bd = __builtin_inf();
  long long bi = 0x7fffffffffffffffLL;
  const long long base = (long long)blockIdx.x * nb;
  for (int t = threadIdx.x; t < nb; t += blockDim.x)
    if (lhc_less(in_d[base + t], in_i[base + t], bd, bi)) { bd = in_d[base + t]; bi = in_i[base + t]; }
  lhc_block_min(bd, bi, sd, si);
  if (threadIdx.x == 0) {
    if (fd && lhc_less(*fd, *fi, bd, bi)) { bd = *fd; bi = *fi; }
    if (out_d) out_d[blockIdx.x] = bd;
    out_i[blockIdx.x] = bi;
  }
}

}  // namespace gpe
