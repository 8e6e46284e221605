// gpemu_dist.hip -- row-block distributed objective over RCCL (include/gpemu_dist.h).
//
// Partition: 128-row tile rows dealt cyclically, tile row t on rank t mod P (the
// trailing matrix shrinks evenly on every rank); rank r stores its tile rows of
// the lower triangle in one column-major buffer (local tile row li <-> global
// t = li P + r).  Tile row NB (below the n_pad x n_pad matrix) holds [f H]^T: the
// sweep turns it into (L^-1 [f H])^T and its diagonal tile into -Gram.
//
// Step k (k = 0 .. NB-1) in column group [gb, ge) (widths as the single-GPU fused
// Cholesky, one wider: 8 while > 160 tile columns remain, then 4, 2, 1), every rank:
//   owner(k): A(k,k) -= L(k,gb:k) L(k,gb:k)^T, -> L_kk (in place), Dinv = L_kk^-1
//             (k_gemm G_DIAG, 1 workgroup); every rank: its panel tiles
//             A(i,k) -= L(i,gb:k) L(k,gb:k)^T (same launch; row k from the gathered panels)
//   broadcast of Dinv from owner(k)                          (128 KB)
//   panel:   L(i,k) = A(i,k) Dinv^T for its rows i > k      (k_gemm)
//   pack its panel tiles, all-gather, unpermute into the group's panel block k-gb
//   k = ge-1: A(i,j) -= L(i,gb:ge) L(j,gb:ge)^T, its rows, ge <= j <= i
//             (k_gemm, tile list, K = 128 (ge-gb))
//
// Gradient (want_grad), same partition, no n x n collective, O(n^2 / P) memory:
//   X = L^-1 by the single-GPU path's recursive TRTRI (block pairs, levels of doubling
//     width), each level's two GEMMs over each rank's own tile rows: M^T = X11^T L21^T
//     after an all-gather of X11, X21 = -X22 M after an all-gather of M (in column
//     chunks that fit the slab; X(k,k) = Dinv_k kept from the sweep).
//   A^-1 = X^T X = sum_r X_r^T X_r over each rank's rows.  The contraction
//   <M, dA/dtheta> is linear in A^-1, so rank r contracts its own partial X_r^T X_r,
//   formed slab by slab (a few tile rows of the lower triangle at a time, never the
//   whole n x n), and rank 0 also carries the -W W^T term; W = [sqrt(c) alpha, W] is
//   all-reduced (n x (q+1)) and then only the d+3 sums.
//
// Look-ahead: the chain of a column group (diagonal factor, Dinv broadcast, panels,
// all-gather) runs on a critical stream; the group's trailing update is split into
// the next group's columns (queued first) and the rest, on the compute stream.  The
// next group's chain waits only for the first part, so its collectives overlap the
// rest of the update.  The panel buffer is double-buffered by group parity.
//
// Every logical rank owns all of its buffers (tile rows, Dinv, panel, all-gather
// buffer, Gram, log-det, X rows, broadcast row, W, slab, sums).  The two transports
// differ only in the collective call (coll_* below): RCCL on this process's one
// rank, or loopback -- all P logical ranks in this process on one GPU, each
// collective a set of device copies (and an add kernel for the all-reduce) between
// the ranks' buffers.  The replicated inputs (points, [f H], r) and the abort flag
// are shared by the loopback ranks.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <map>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/gpemu.h"
#include "../../include/gpemu_dist.h"
#include "gpemu_kernels.hpp"
#include "gpemu_small.hpp"
#include "gpemu_ozaki.hpp"

using namespace gpe;

namespace {

struct DistPairArgs {
  const double* xw;   // scaled points, n_pad x d row-major (zero rows >= n)
  const double* F;    // [f H], n_pad x Pc column-major (zero rows >= n)
  const double* r;    // nugget vector or null
  double* out;        // local tile rows, column-major
  long long ld, ldF;
  int d, n_valid, NB, nranks, rank, nloc, Pc;
  double s2, coff, cdiag, rscale;
};

// K-build of one rank's tile rows: tile (li, tj), tj <= t = li P + rank; the
// training matrix s2 coff exp(-|x_i - x_j|^2), diagonal s2 cdiag + rscale r_i,
// identity on padded rows; tile row NB = [f H]^T (zero beyond Pc rows, (NB,NB) = 0).
template <int DMAX>
__global__ void __launch_bounds__(256) k_dist_kbuild(DistPairArgs a) {
  __shared__ double xs_col[TILE * DMAX];
  const int li = blockIdx.x % a.nloc, tj = blockIdx.x / a.nloc;
  const int gt = li * a.nranks + a.rank;
  if (tj > gt) return;
  const int tid = threadIdx.x, r = tid & (TILE - 1);
  double* out = a.out + (long long)li * TILE + (long long)tj * TILE * a.ld;
  if (gt >= a.NB) {   // augmented tile row u = gt - NB: [f H] columns 128 u .., transposed
    const int pr = r + (gt - a.NB) * TILE;
    for (int c = tid >> 7; c < TILE; c += 2) {
      const int gj = tj * TILE + c;
      const double v = (tj < a.NB && pr < a.Pc) ? a.F[gj + (long long)pr * a.ldF] : 0.0;
      out[r + (long long)c * a.ld] = v;
    }
    return;
  }
  // coordinates zero-padded to DMAX (exact no-op terms), entries selected, not branched:
  // the same sums and values as the single-GPU k_pairs
  const int d = a.d;
  for (int e = tid; e < TILE * DMAX; e += 256) {
    const int c = e / DMAX, k = e - c * DMAX;
    xs_col[e] = k < d ? a.xw[(long long)(tj * TILE + c) * d + k] : 0.0;
  }
  const int gi = gt * TILE + r;
  double xi[DMAX];
#pragma unroll
  for (int k = 0; k < DMAX; ++k) xi[k] = (k < d) ? a.xw[(long long)gi * d + k] : 0.0;
  __syncthreads();
  const double pre = a.s2 * a.coff;
  const bool row_pad = gi >= a.n_valid;
  double vdiag = a.s2 * a.cdiag;
  if (a.r && gt == tj && !row_pad) vdiag += a.rscale * a.r[gi];
  for (int c = tid >> 7; c < TILE; c += 2) {
    const int gj = tj * TILE + c;
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < DMAX; ++k) {
      const double df = xi[k] - xs_col[c * DMAX + k];
      s = fma(df, df, s);
    }
    double v = pre * exp(-s);
    const bool diag = gi == gj;
    v = (row_pad || gj >= a.n_valid) ? (diag ? 1.0 : 0.0) : (diag ? vdiag : v);
    out[r + (long long)c * a.ld] = v;
  }
}

// k_dist_kbuild for d > 32: coordinates staged through LDS 32 dimensions at a time
// (as k_pairs_wide; the same sums in the same order)
__global__ void __launch_bounds__(256) k_dist_kbuild_wide(DistPairArgs a) {
  __shared__ double xs_col[TILE * PW_CH];
  const int li = blockIdx.x % a.nloc, tj = blockIdx.x / a.nloc;
  const int gt = li * a.nranks + a.rank;
  if (tj > gt) return;
  const int tid = threadIdx.x, r = tid & (TILE - 1), h = tid >> 7;
  double* out = a.out + (long long)li * TILE + (long long)tj * TILE * a.ld;
  if (gt >= a.NB) {   // augmented tile row u = gt - NB: [f H] columns 128 u .., transposed
    const int pr = r + (gt - a.NB) * TILE;
    for (int c = h; c < TILE; c += 2) {
      const int gj = tj * TILE + c;
      const double v = (tj < a.NB && pr < a.Pc) ? a.F[gj + (long long)pr * a.ldF] : 0.0;
      out[r + (long long)c * a.ld] = v;
    }
    return;
  }
  const int d = a.d;
  const int gi = gt * TILE + r;
  double s[TILE / 2];
#pragma unroll
  for (int u = 0; u < TILE / 2; ++u) s[u] = 0.0;
  for (int k0 = 0; k0 < d; k0 += PW_CH) {
    __syncthreads();
    for (int e = tid; e < TILE * PW_CH; e += 256) {
      const int c = e / PW_CH, k = e - c * PW_CH;
      xs_col[e] = k0 + k < d ? a.xw[(long long)(tj * TILE + c) * d + k0 + k] : 0.0;
    }
    double xi[PW_CH];
#pragma unroll
    for (int k = 0; k < PW_CH; ++k) xi[k] = (k0 + k < d) ? a.xw[(long long)gi * d + k0 + k] : 0.0;
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
  const bool row_pad = gi >= a.n_valid;
  double vdiag = a.s2 * a.cdiag;
  if (a.r && gt == tj && !row_pad) vdiag += a.rscale * a.r[gi];
#pragma unroll
  for (int u = 0; u < TILE / 2; ++u) {
    const int c = h + 2 * u;
    const int gj = tj * TILE + c;
    double v = pre * exp(-s[u]);
    const bool diag = gi == gj;
    v = (row_pad || gj >= a.n_valid) ? (diag ? 1.0 : 0.0) : (diag ? vdiag : v);
    out[r + (long long)c * a.ld] = v;
  }
}

// panel tiles (local rows li0 .. li0+cnt-1, column k) -> dst, 128x128 column-major each
__global__ void __launch_bounds__(256) k_dist_pack(const double* Aloc, long long ld, int li0, int k,
                                                   double* dst) {
  const int t = blockIdx.x;
  const double* src = Aloc + (long long)(li0 + t) * TILE + (long long)k * TILE * ld;
  double* o = dst + (long long)t * TILE * TILE;
  for (int e = threadIdx.x; e < TILE * TILE / 2; e += 256) {
    const int i = (e & 63) * 2, c = e >> 6;
    *reinterpret_cast<double2*>(o + i + c * TILE) =
        *reinterpret_cast<const double2*>(src + i + (long long)c * ld);
  }
}

// one 128 x 128 tile src (ld lds) -> dst (ld ldd): 16 workgroups of 8 columns, 16-byte
// accesses (a hipMemcpy2DAsync of the same tile: 16 us per step on the chain)
__device__ __forceinline__ void k_dist_tile_body(const double* src, long long lds, double* dst, long long ldd) {
  const int c = blockIdx.x * 8 + (threadIdx.x >> 5), i = (threadIdx.x & 31) * 4;
  const double2* s = reinterpret_cast<const double2*>(src + i + c * lds);
  double2* o = reinterpret_cast<double2*>(dst + i + c * ldd);
  const double2 a = s[0], b = s[1];
  o[0] = a;
  o[1] = b;
}
__global__ void __launch_bounds__(256) k_dist_tile(const double* src, long long lds, double* dst, long long ldd) {
  k_dist_tile_body(src, lds, dst, ldd);
}

// P = 1: the factors' leaf-inverse tiles (one per step, ld 128) -> X's diagonal tiles, all
// NB at once after the sweep (per step on the chain, k_dist_tile averaged 20 us: its 16
// workgroups waited for slots behind the trailing updates)
__global__ void __launch_bounds__(256) k_dist_leaves(const double* src, double* X, long long ld) {
  const long long t = blockIdx.y;
  k_dist_tile_body(src + t * TILE * TILE, (long long)TILE, X + t * TILE + t * TILE * ld, ld);
}

// gathered segment of rank r (blockIdx.y), tile t -> panel rows of global tile (li0_r + t) P + r
__global__ void __launch_bounds__(256) k_dist_unpermute(const double* recv, long long seg,
                                                        const int* li0, const int* cnt, int P,
                                                        double* panel, long long ldp) {
  const int r = blockIdx.y, t = blockIdx.x;
  if (t >= cnt[r]) return;
  const int gt = (li0[r] + t) * P + r;
  const double* src = recv + (long long)r * seg + (long long)t * TILE * TILE;
  double* o = panel + (long long)gt * TILE;
  for (int e = threadIdx.x; e < TILE * TILE / 2; e += 256) {
    const int i = (e & 63) * 2, c = e >> 6;
    *reinterpret_cast<double2*>(o + i + (long long)c * ldp) =
        *reinterpret_cast<const double2*>(src + i + c * TILE);
  }
}

// columns p0 .. p0+pc of Z = L^-1 [f H] (n_pad x Pc, column-major) out of an augmented
// tile row (local row li)
__global__ void __launch_bounds__(256) k_dist_take_z(const double* Aloc, long long ld, int li, long long np,
                                                     int p0, int pc, double* Z) {
  const long long j = (long long)blockIdx.x * 256 + threadIdx.x;
  if (j >= np) return;
  const double* src = Aloc + (long long)li * TILE + j * ld;
  for (int p = 0; p < pc; ++p) Z[j + (p0 + p) * np] = src[p];
}

// rows of R2 (n_pad x Pc) at rank `rank`'s tile rows -> out (local rows, ld ldo)
__global__ void __launch_bounds__(256) k_dist_rows(const double* R2, long long ldr, int Pc, int P, int rank,
                                                   int nlx, double* out, long long ldo) {
  const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
  if (e >= (long long)nlx * TILE) return;
  const int li = (int)(e / TILE), rr = (int)(e % TILE);
  const long long g = (long long)(li * P + rank) * TILE + rr;
  for (int p = 0; p < Pc; ++p) out[e + p * ldo] = R2[g + p * ldr];
}

// loopback all-reduce: dst += src
__global__ void __launch_bounds__(256) k_dist_add(double* dst, const double* src, long long count) {
  for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < count; e += (long long)gridDim.x * 256)
    dst[e] += src[e];
}

// Tile moves of the recursive TRTRI's gathers: dst tile (ti, tj) of a rows x cols block
// <- src.  perm = 0: src tile (ti, tj).  perm = 1 (2): the block's tile rows (columns) are
// the global tile rows g = g0 + ti (g0 + tj), which arrive by rank, in the all-gather
// segment of g's owner (g mod P, seg doubles apart), as that rank's j-th such row:
// src tile (j, tj) ((ti, j)) of that segment.
struct MoveDesc {
  const double* src;
  double* dst;
  long long lds, ldd, seg;
  int rows, cols, tile_begin, perm, g0, P;
};

__global__ void __launch_bounds__(256) k_dist_move(const MoveDesc* __restrict__ d, int nd) {
  int lo = 0, hi = nd - 1;   // last descriptor whose tile_begin <= blockIdx.x
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if ((int)blockIdx.x >= d[mid].tile_begin) lo = mid;
    else hi = mid - 1;
  }
  const MoveDesc D = d[lo];
  const int local = (int)blockIdx.x - D.tile_begin;
  const int ti = local % D.rows, tj = local / D.rows;
  int si = ti, sj = tj;
  const double* s = D.src;
  if (D.perm) {
    const int g = D.g0 + (D.perm == 1 ? ti : tj), r = g % D.P;
    const int first = D.g0 + (r - D.g0 % D.P + D.P) % D.P;   // the owner's first row >= g0
    const int j = (g - first) / D.P;
    s += (long long)r * D.seg;
    (D.perm == 1 ? si : sj) = j;
  }
  s += (long long)si * TILE + (long long)sj * TILE * D.lds;
  double* o = D.dst + (long long)ti * TILE + (long long)tj * TILE * D.ldd;
  for (int e = threadIdx.x; e < TILE * TILE / 2; e += 256) {
    const int i = (e & 63) * 2, c = e >> 6;
    *reinterpret_cast<double2*>(o + i + (long long)c * D.ldd) =
        *reinterpret_cast<const double2*>(s + i + (long long)c * D.lds);
  }
}

struct Rank {              // one rank's buffers (one per process over RCCL, P in loopback)
  int rank = 0, nloc = 0;
  long long ld = 0;
  int nlx = 0;             // tile rows of the matrix proper (without the [f H] row)
  // sweep
  double* A = nullptr;     // nloc*128 x (NB+1)*128, column-major
  double* logdet = nullptr;   // NB+1 (own steps; all-reduced)
  // the step's broadcast block, 128 x (Kp + 128), ld 128: [-M | Dinv] with Dinv = L_kk^-1 and
  // M = Dinv L(k, gb:k) (Kp = 128 (k - gb) pending columns of the group; P = 1: Dinv alone)
  double* dinv = nullptr;
  double* panel = nullptr; // 2 x (NB+1)*128 x wmax*128: gathered panels of a group (by group parity)
  double* recv = nullptr;  // all-gather buffer, P segments of the largest panel
  double* gram = nullptr;  // Pc x Pc
  // gradient
  double* X = nullptr;     // L^-1 rows, ld as A, NB*128 columns (zero above the diagonal)
  double* g1 = nullptr;    // P > 1: a TRTRI chunk's gathered X11 blocks (global row order)
  double* trecv = nullptr; // P > 1: the TRTRI's all-gather buffer (X11 rows, then M^T columns)
  double* dZ = nullptr;    // n_pad x Pc: L^-1 [f H] (broadcast)
  double* dR2 = nullptr;   // n_pad x Pc
  double* r2loc = nullptr; // local rows of R2, 128 columns (zero beyond Pc)
  double* wpart = nullptr; // n_pad x 128: [sqrt(c) alpha, W] (all-reduced)
  long long slab_doubles = 0;
  double* slab = nullptr;  // slab*128 x n_pad: tile rows of this rank's partial X_r^T X_r
                           // (first, the TRTRI chunks' M^T blocks)
  double* csum = nullptr;  // d+3 contraction sums (all-reduced)
  size_t bytes = 0;        // device bytes held for this rank
};

struct DLaunch {           // one grouped k_gemm launch
  int first = 0, count = 0, tiles = 0;
  long long list = -1;
  int kind = 0;            // 0 <false,false> (the fused instance: G_DIAG problems), 1 <false,true>,
                           // 2 <true,true>, 3 <true,false>, 4 <false,false> (plain)
  bool cdef = false;       // k_gemm's CDEF instance (gemm_cdef of some problem)
  int* ticket = nullptr;   // FUSED launches with in-launch waits: list positions by atomic
                           // ticket (k_gemm), so progress never depends on dispatch order
};

// one column chunk of one level of the recursive TRTRI (see ensure_grad)
struct TriChunk {
  DLaunch m, x;            // M^T = X11^T L21^T ; X21 = -X22 M
  int pack0 = 0, npack = 0, pack_tiles = 0;   // P > 1: move descriptors and their tiles
  int unp1 = 0, nunp1 = 0, unp1_tiles = 0;
  int unp2 = 0, nunp2 = 0, unp2_tiles = 0;
  size_t seg1 = 0, seg2 = 0;                  // all-gather segments (doubles)
  int s = 0, cw = 0;                          // its level (pairs of s tile columns), chunk width
  std::vector<OzTriPair> oz;                  // P = 1: the level's pairs on the int8 cores
};

struct SlabLaunch {        // one slab of a rank's partial of A^-1: GEMM + contraction
  DLaunch gemm;
  int a0 = 0, a1 = 0;      // tile rows [a0, a1)
};

constexpr int DIST_DESC_MAX = 1 << 20;
constexpr size_t SLAB_DOUBLES = (size_t)1 << 26;   // 512 MiB per rank for the A^-1 slab

int nloc_of(int NB, int P, int r) { return r <= NB ? (NB - r) / P + 1 : 0; }
// first local row of rank r whose global tile row exceeds k
int li0_of(int k, int P, int r) { return k < r ? 0 : (k - r) / P + 1; }

}  // namespace

struct gpe_dist {
  int device = 0, P = 1, rank = 0;
  bool loop = true;
  ncclComm_t comm = nullptr;
  hipStream_t stream = nullptr;   // compute stream (bulk updates, everything outside the sweeps)
  hipStream_t crit = nullptr;     // critical stream (a group's chain and its collectives)
  hipStream_t cs = nullptr;       // the stream launches and collectives are issued on
  std::string err;

  long long n = 0, n_pad = 0;
  int d = 0, q = 0, NB = 0;
  int NA = 1;              // augmented tile rows NB .. NB+NA-1: [f H]^T, 128 basis columns each
  bool has_r = false;
  // replicated inputs (one copy shared by the loopback ranks)
  double* dX = nullptr;    // n_pad x d raw
  double* dXw = nullptr;   // scaled
  double* dF = nullptr;    // n_pad x (q+1)
  double* dr = nullptr;
  double* dinvdelta = nullptr;
  int* dinfo = nullptr;    // abort flag / failed pivot (all-reduced with max over RCCL)
  int* dq = nullptr;       // 6 x NB counters: the diagonal tiles' pending-update blocks (G_DQUAD);
                           // P = 1: the diagonal flags and the panel halves' stored updates;
                           // the diagonal launches' tickets; P = 1: the fused update launches'
                           // tickets and their first columns' stored tiles (fuse_next_factor)
  double* cpart = nullptr; // contraction partials (scratch, stream-ordered)
  std::vector<Rank> ranks;   // local ranks (all P in loopback, one otherwise)

  // column groups: {width, min remaining tile columns}, first match wins, else 1
  // (GPEMU_DIST_W="8:160,4:80,2:40" style).  Width 4 to the end: with the next group's
  // update on the chain stream, the narrower tail groups of round 5 (2 and 1 wide) cost
  // more in launches than their shorter pending updates saved (P = 1, n = 16384: value
  // 30.7-30.9 -> 30.2-30.3 ms, gradient 75.4-75.5 -> 74.6-74.8, profiles/dist_w_r05z.log)
  std::vector<std::pair<int, int>> groups = {{8, 160}, {4, 0}};
  std::vector<int> gstart;   // per step: first column of its group
  std::vector<int> gid;      // per step: index of its group
  std::vector<int> gs;       // group starts, then NB
  int wmax = 1;
  size_t panel_sz = 0;       // doubles per panel buffer (two per rank)
  std::vector<hipEvent_t> ev_chain, ev_next;   // per group (sweep or TRTRI, reused)
  std::vector<hipEvent_t> ev_near, ev_far;     // per group: the sweep's near / far updates done
  hipEvent_t ev_join = nullptr, ev_end = nullptr;
  bool next_on_chain = true;                   // GPEMU_DIST_NEXT_ON_CHAIN=0: round-5 schedule
  bool fuse_next = false;                      // P = 1: a group's first factor inside the update
                                               // before it (GPEMU_DIST_FUSE_NEXT=1; measured no
                                               // faster)
  int* dli0 = nullptr;       // [NB][P] first local row with global row > k
  int* dcnt = nullptr;       // [NB][P] panel tiles of rank r at step k
  GemmProb* dprobs = nullptr;
  unsigned* dtiles = nullptr;
  std::vector<DLaunch> diag, mrow, panel_l, upd_next, upd_near, upd_far;   // per step (updates: group ends)
  std::vector<int> maxT;                       // per step: max panel tiles over ranks
  size_t recv_tiles = 0;                       // P > 1: tiles per rank segment of the group all-gather
  double* hpin = nullptr;
  size_t hpin_cap = 0;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  std::vector<hipEvent_t> cev;
  int ev = 0;                                  // event pairs used by this objective call
  double total_ms = 0.0, comm_ms = 0.0;
  size_t shared_bytes = 0;

  // gradient (allocated on the first want_grad call after gpe_dist_set_data)
  bool grad_ready = false, grad_now = false;
  int slab_rows = 1;                           // tile rows per slab of A^-1
  double* dT2 = nullptr;
  GemmProb* gprobs = nullptr;
  double* wsplit = nullptr;                    // split-K partials of the W launch
  int* wcnt = nullptr;                         // its per-tile arrival counters
  unsigned* gtiles = nullptr;                  // tile lists of the gradient launches
  std::vector<DLaunch> wa_l;
  std::vector<TriChunk> tri;                   // the recursive TRTRI, level by level
  MoveDesc* dmoves = nullptr;
  std::vector<std::vector<SlabLaunch>> slabs;  // per local rank
  // the A^-1 partial X_r^T X_r on the int8 cores (gpemu_ozaki.hpp, as the single-GPU LAUUM;
  // GPEMU_OZAKI=0: fp64 k_gemm slabs).  The buffers serve one rank at a time (the loopback
  // ranks' partials run one after another on the compute stream)
  bool oz_on = true;
  int oz_nmod = OZ_MAXMOD;
  bool oz_now = false;                         // this data's partial on the int8 cores
  long long oz_cap_mb = 16384;                 // at most this many MiB of planes per rank
  int oz_min_np = 6144;                        // from this n_pad (as gpemu.hip; GPEMU_OZAKI_MIN_NP)
  int oz_tri_min = 8192;                       // P = 1: TRTRI levels of blocks this tall on the
                                               // int8 cores (GPEMU_OZAKI_TRI_MIN, as gpemu.hip)
  int oz_np2 = 0, oz_kp = 0;                   // planes: oz_np2 rows (columns of X_r) x oz_kp k
  OzConst oz_c{};
  int8_t* ozp = nullptr;                       // N planes of X_r^T
  int8_t* ozr = nullptr;                       // N residue images of one slab's 256-tiles
  long long oz_res_bytes = 0;
  int* ozx = nullptr;                          // column exponents of X_r
  unsigned* ozl = nullptr;                     // the slabs' tile lists
  std::vector<std::pair<long long, int>> oz_lists;   // per slab: offset, length
};

namespace {

#define DCHK_HIP(h, expr)                                                          \
  do {                                                                             \
    hipError_t e_ = (expr);                                                        \
    if (e_ != hipSuccess) {                                                        \
      (h)->err = std::string(#expr) + ": " + hipGetErrorString(e_);                \
      return GPE_ERR_HIP;                                                          \
    }                                                                              \
  } while (0)

#define DCHK_NCCL(h, expr)                                                         \
  do {                                                                             \
    ncclResult_t e_ = (expr);                                                      \
    if (e_ != ncclSuccess) {                                                       \
      (h)->err = std::string(#expr) + ": " + ncclGetErrorString(e_);               \
      return GPE_ERR_HIP;                                                          \
    }                                                                              \
  } while (0)

#define DCHK(expr)                   \
  do {                               \
    int rc_ = (expr);                \
    if (rc_ != GPE_OK) return rc_;   \
  } while (0)

int dfail(gpe_dist* h, int code, const std::string& m) {
  h->err = m;
  return code;
}

template <typename T>
void dfree(T** p) {
  if (*p) (void)hipFree(*p);
  *p = nullptr;
}

template <typename T>
int dalloc(gpe_dist* h, T** p, size_t count, size_t* acct = nullptr) {
  dfree(p);
  if (count == 0) return GPE_OK;
  if (hipMalloc((void**)p, count * sizeof(T)) != hipSuccess) {
    *p = nullptr;
    return dfail(h, GPE_ERR_ALLOC, "hipMalloc failed (" + std::to_string(count * sizeof(T)) + " bytes)");
  }
  if (acct) *acct += count * sizeof(T);
  return GPE_OK;
}

void free_rank(Rank& R) {
  if (R.trecv == R.recv) R.trecv = nullptr;   // aliased (ensure_grad)
  double** bufs[] = {&R.A, &R.logdet, &R.dinv, &R.panel, &R.recv, &R.gram, &R.X, &R.g1, &R.trecv,
                     &R.dZ, &R.dR2, &R.r2loc, &R.wpart, &R.slab, &R.csum};
  for (double** b : bufs) dfree(b);
  R.bytes = 0;
}

int pinned(gpe_dist* h, size_t doubles) {
  if (doubles <= h->hpin_cap) return GPE_OK;
  if (h->hpin) (void)hipHostFree(h->hpin);
  h->hpin = nullptr;
  const size_t cap = std::max<size_t>(doubles, 1 << 14);
  DCHK_HIP(h, hipHostMalloc((void**)&h->hpin, cap * sizeof(double), hipHostMallocDefault));
  h->hpin_cap = cap;
  return GPE_OK;
}

GemmProb dprob(const double* A, long long lda, const double* B, long long ldb, double* C, long long ldc,
               int mt, int nt, int K, int flags, double alpha, double beta) {
  GemmProb p;
  std::memset(&p, 0, sizeof(p));
  p.A = A; p.B = B; p.C = C;
  p.lda = lda; p.ldb = ldb; p.ldc = ldc;
  p.mt = mt; p.nt = nt; p.K = K; p.flags = flags;
  p.alpha = alpha; p.beta = beta;
  p.kti_mul = 1;
  return p;
}

Rank* rank_slot(gpe_dist* h, int r) {   // the local slot of rank r, or null (another process)
  for (Rank& R : h->ranks)
    if (R.rank == r) return &R;
  return nullptr;
}

// ---------------------------------------------------------------------------
// Collectives.  Arguments name a buffer member of Rank plus an element offset;
// over RCCL they act on this process's one rank, in loopback on the P logical
// ranks' buffers.  Each is bracketed by an event pair (comm time).
// ---------------------------------------------------------------------------
int ensure_events(gpe_dist* h, size_t n) {
  while (h->cev.size() < n) {
    hipEvent_t e;
    DCHK_HIP(h, hipEventCreate(&e));
    h->cev.push_back(e);
  }
  return GPE_OK;
}

int comm_begin(gpe_dist* h) {
  DCHK(ensure_events(h, (size_t)h->ev + 2));
  DCHK_HIP(h, hipEventRecord(h->cev[h->ev], h->cs));
  return GPE_OK;
}

int comm_end(gpe_dist* h) {
  DCHK_HIP(h, hipEventRecord(h->cev[h->ev + 1], h->cs));
  h->ev += 2;
  return GPE_OK;
}

// broadcast count doubles at (Rank::*buf + off) from rank root
int coll_bcast(gpe_dist* h, double* Rank::*buf, long long off, size_t count, int root) {
  DCHK(comm_begin(h));
  if (!h->loop) {
    double* p = h->ranks[0].*buf + off;
    DCHK_NCCL(h, ncclBroadcast(p, p, count, ncclDouble, root, h->comm, h->cs));
  } else {
    const double* src = rank_slot(h, root)->*buf + off;
    for (Rank& R : h->ranks) {
      if (R.rank == root) continue;
      DCHK_HIP(h, hipMemcpyAsync(R.*buf + off, src, count * sizeof(double), hipMemcpyDeviceToDevice, h->cs));
    }
  }
  return comm_end(h);
}

// in-place all-gather: rank r's segment of seg doubles at offset r*seg
int coll_allgather(gpe_dist* h, double* Rank::*buf, size_t seg) {
  DCHK(comm_begin(h));
  if (!h->loop) {
    double* p = h->ranks[0].*buf;
    DCHK_NCCL(h, ncclAllGather(p + (size_t)h->rank * seg, p, seg, ncclDouble, h->comm, h->cs));
  } else {
    for (Rank& D : h->ranks)
      for (const Rank& S : h->ranks) {
        if (S.rank == D.rank) continue;
        const size_t o = (size_t)S.rank * seg;
        DCHK_HIP(h, hipMemcpyAsync(D.*buf + o, S.*buf + o, seg * sizeof(double), hipMemcpyDeviceToDevice,
                                   h->cs));
      }
  }
  return comm_end(h);
}

// all-reduce (sum) of count doubles at (Rank::*buf + off)
int coll_allreduce_sum(gpe_dist* h, double* Rank::*buf, long long off, size_t count) {
  DCHK(comm_begin(h));
  if (!h->loop) {
    double* p = h->ranks[0].*buf + off;
    DCHK_NCCL(h, ncclAllReduce(p, p, count, ncclDouble, ncclSum, h->comm, h->cs));
  } else if (h->ranks.size() > 1) {
    double* acc = h->ranks[0].*buf + off;
    const unsigned g = (unsigned)std::min<size_t>((count + 255) / 256, 2048);
    for (size_t s = 1; s < h->ranks.size(); ++s) {
      hipLaunchKernelGGL(k_dist_add, dim3(g), dim3(256), 0, h->cs, acc, h->ranks[s].*buf + off,
                         (long long)count);
      DCHK_HIP(h, hipGetLastError());
    }
    for (size_t s = 1; s < h->ranks.size(); ++s)
      DCHK_HIP(h, hipMemcpyAsync(h->ranks[s].*buf + off, acc, count * sizeof(double), hipMemcpyDeviceToDevice,
                                 h->cs));
  }
  return comm_end(h);
}

// all-reduce (max) of the abort flag: over RCCL each process has its own; the
// loopback ranks share one (their launches are batched), so it is already reduced
int coll_info_max(gpe_dist* h) {
  if (h->loop) return GPE_OK;
  DCHK(comm_begin(h));
  DCHK_NCCL(h, ncclAllReduce(h->dinfo, h->dinfo, 1, ncclInt32, ncclMax, h->comm, h->cs));
  return comm_end(h);
}

// Column groups [gb, ge): step k = gb + w applies the pending update by the group's
// earlier columns [gb, k) to its own diagonal tile and panel tiles (K = 128 w, in the
// diagonal launch, before the Dinv broadcast), and the step that closes the group
// applies the whole group to the trailing matrix in one K = 128 (ge - gb) update.
void build_groups(gpe_dist* h) {
  const int NB = h->NB;
  h->gstart.assign(NB, 0);
  h->gid.assign(NB, 0);
  h->gs.clear();
  h->wmax = 1;
  for (int g = 0; g < NB;) {
    int w = 1;
    for (const auto& r : h->groups)
      if (NB - g > r.second) { w = r.first; break; }
    w = std::max(1, std::min(w, NB - g));
    for (int k = g; k < g + w; ++k) {
      h->gstart[k] = g;
      h->gid[k] = (int)h->gs.size();
    }
    h->gs.push_back(g);
    h->wmax = std::max(h->wmax, w);
    g += w;
  }
  h->gs.push_back(NB);
}

int group_end(const gpe_dist* h, int k) {   // one past the last column of k's group
  return h->gs[h->gid[k] + 1];
}

// one past the last column of the group after k's (NB when k's group is the last)
int next_group_end(const gpe_dist* h, int k) {
  const int g = h->gid[k];
  return g + 2 < (int)h->gs.size() ? h->gs[g + 2] : h->NB;
}

// the panel buffer of step k's group (double-buffered by group parity); with one rank the
// gathered panels would be the rank's own columns in the same layout: its tile rows
int gather_panels(const gpe_dist* h) { return h->P > 1; }
double* panel_of(const gpe_dist* h, const Rank& R, int k) {
  if (!gather_panels(h)) return R.A + (long long)h->gstart[k] * TILE * R.ld;
  return R.panel + (size_t)(h->gid[k] & 1) * h->panel_sz;
}

// XCD-aware order of a launch's tiles (as gpemu.hip order_tiles): rows (problem, ti) -- one
// A panel each -- longest tiles first, greedily packed into 8 bins of equal work, the bins
// interleaved tile by tile.  Under round-robin dispatch each row's tiles then run on one
// XCD and its A panel stays in that XCD's L2: in implicit order (ti fastest) every XCD
// streams every panel, and a K = 8192 TRTRI level ran 2.7x over its MFMA time.
std::vector<unsigned> xcd_order(const GemmProb* probs, const std::vector<unsigned>& tiles) {
  struct Row { double w = 0.0, tw = 0.0; std::vector<unsigned> t; };
  std::map<std::pair<int, int>, Row> rows;
  for (unsigned code : tiles) {
    const int p = (int)(code >> 24), ti = (int)((code >> 12) & 0xfff);
    const GemmProb& P = probs[p];
    int kb = 0, ke = P.K;
    if (P.flags & G_KBEG_TI) kb = ti * TILE;
    if (P.flags & G_KEND_TI) ke = std::min(ke, (ti * P.kti_mul + P.kti_off + 1) * TILE);
    Row& r = rows[{p, ti}];
    r.tw = (double)std::max(ke - kb, 0) + 2.0 * GK;   // + fixed per-tile cost
    r.w += r.tw;
    r.t.push_back(code);
  }
  std::vector<const Row*> order;
  for (const auto& kv : rows) order.push_back(&kv.second);
  std::stable_sort(order.begin(), order.end(), [](const Row* a, const Row* b) { return a->tw > b->tw; });
  constexpr int NX = 8;
  std::vector<std::vector<unsigned>> bins(NX);
  std::vector<double> load(NX, 0.0);
  for (const Row* r : order) {
    const int x = (int)(std::min_element(load.begin(), load.end()) - load.begin());
    load[x] += r->w;
    bins[x].insert(bins[x].end(), r->t.begin(), r->t.end());
  }
  std::vector<unsigned> out;
  size_t longest = 0;
  for (auto& b : bins) longest = std::max(longest, b.size());
  for (size_t j = 0; j < longest; ++j)
    for (int x = 0; x < NX; ++x)
      if (j < bins[x].size()) out.push_back(bins[x][j]);
  return out;
}

// every tile of a plain launch's problems, XCD-ordered, appended to tiles as L's list
// (launches of more than 256 problems, which the list code cannot name, keep the
// implicit order)
void list_launch(DLaunch& L, const std::vector<GemmProb>& probs, std::vector<unsigned>& tiles) {
  if (L.count == 0 || L.count > 256) return;
  std::vector<unsigned> all;
  for (int p = 0; p < L.count; ++p) {
    const GemmProb& P = probs[L.first + p];
    for (int tj = 0; tj < P.nt; ++tj)
      for (int ti = 0; ti < P.mt; ++ti)
        if (!(P.flags & G_CLOWER) || tj <= ti) all.push_back(((unsigned)p << 24) | ((unsigned)ti << 12) | (unsigned)tj);
  }
  const std::vector<unsigned> ord = xcd_order(probs.data() + L.first, all);
  L.list = (long long)tiles.size();
  tiles.insert(tiles.end(), ord.begin(), ord.end());
}

// P = 1 (round-6 verdict item 4): the first step of each group after the first is started
// inside the update launch before it (the previous group's update of the group's columns, A),
// on tile counts, as the single-GPU fused sweep does: that launch's tiles of column ge count
// themselves when stored, the factor of tile (ge, ge) and the panel tiles' first halves wait
// for all of them, and the rest of the update runs beside the factorisation.  The group's
// first step has no pending columns (no G_DQUAD blocks), and its launch drops out of the chain
// (one dependent launch and its idle gap fewer per group).  List order: column ge's tiles,
// the factor, the other columns' tiles, the panel halves; every wait points to an earlier
// list position (checked), and positions are claimed by ticket.
int fuse_next_factor(gpe_dist* h, std::vector<GemmProb>& probs, std::vector<unsigned>& tiles) {
  const int NB = h->NB;
  for (int k = 0; k + 1 < NB; ++k) {
    const int ge = k + 1;
    if (group_end(h, k) != ge) continue;
    DLaunch& ul = h->upd_next[k];
    DLaunch& dl = h->diag[ge];
    if (ul.count != 1 || ul.tiles == 0 || ul.list < 0 || dl.count == 0 || dl.list >= 0) continue;
    int* cnt = h->dq + 5 * NB + ge;
    DLaunch f;
    f.kind = 0;
    f.first = (int)probs.size();
    GemmProb pc = probs[ul.first], pr = probs[ul.first];
    pc.post = cnt;
    std::vector<unsigned> col, rest;
    for (int i = 0; i < ul.tiles; ++i) {
      const unsigned code = tiles[(size_t)ul.list + i], tj = code & 0xfffu;
      (tj == (unsigned)ge ? col : rest).push_back((tj == (unsigned)ge ? 0u : 1u << 24) | (code & 0xffffffu));
    }
    if (col.empty()) continue;
    probs.push_back(pc);
    probs.push_back(pr);
    std::vector<unsigned> fac, halves;
    for (int p = 0; p < dl.count; ++p) {
      GemmProb q = probs[dl.first + p];
      if (q.flags & G_DQUAD) return dfail(h, GPE_ERR_STATE, "internal error: a group's first step with pending columns");
      if (q.flags & (G_DIAG | G_PHALF0)) {
        q.pre0 = cnt;
        q.pre0_n = (int)col.size();
      }
      const unsigned pi = (unsigned)(2 + p);
      for (int ti = 0; ti < q.mt; ++ti)
        ((q.flags & G_DIAG) ? fac : halves).push_back((pi << 24) | ((unsigned)ti << 12));
      f.cdef = f.cdef || gemm_cdef(q);
      probs.push_back(q);
    }
    f.count = 2 + dl.count;
    f.cdef = f.cdef || gemm_cdef(pc);
    std::vector<unsigned> order = col;
    order.insert(order.end(), fac.begin(), fac.end());
    order.insert(order.end(), rest.begin(), rest.end());
    order.insert(order.end(), halves.begin(), halves.end());
    {   // every wait on an earlier position (counts complete before the waiter's slot)
      std::map<const int*, size_t> last_post;
      size_t diag_at = order.size();
      for (size_t i = 0; i < order.size(); ++i) {
        const GemmProb& q = probs[f.first + (order[i] >> 24)];
        if (q.post) last_post[q.post] = i;
        if (q.cpost) last_post[q.cpost] = i;
        if (q.flags & G_DIAG) diag_at = i;
      }
      for (size_t i = 0; i < order.size(); ++i) {
        const GemmProb& q = probs[f.first + (order[i] >> 24)];
        const bool ok = (!q.pre0 || (last_post.count(q.pre0) && last_post[q.pre0] < i)) &&
                        (!(q.flags & G_PANEL) || diag_at < i);
        if (!ok) return dfail(h, GPE_ERR_STATE, "internal error: fused launch waits on a later tile");
      }
    }
    f.list = (long long)tiles.size();
    tiles.insert(tiles.end(), order.begin(), order.end());
    f.tiles = (int)order.size();
    f.ticket = h->dq + 4 * NB + k;
    ul = f;
    dl = DLaunch();   // (step ge launches nothing for its factor)
  }
  return GPE_OK;
}

// every per-step GEMM descriptor and tile list, for the current n and partition
int build_schedule(gpe_dist* h) {
  const int NB = h->NB, P = h->P, NT = NB + h->NA;
  const long long ldp = (long long)NT * TILE;
  std::vector<GemmProb> probs;
  std::vector<unsigned> tiles;
  h->diag.assign(NB, DLaunch());
  h->mrow.assign(NB, DLaunch());
  h->panel_l.assign(NB, DLaunch());
  h->upd_next.assign(NB, DLaunch());
  h->upd_near.assign(NB, DLaunch());
  h->upd_far.assign(NB, DLaunch());
  h->maxT.assign(NB, 0);
  std::vector<int> li0((size_t)NB * P), cnt((size_t)NB * P);
  for (int k = 0; k < NB; ++k) {
    const int gb = h->gstart[k], ge = group_end(h, k);
    const int Kp = (k - gb) * TILE;   // pending columns [gb, k)
    for (int r = 0; r < P; ++r) {
      li0[(size_t)k * P + r] = li0_of(k, P, r);
      cnt[(size_t)k * P + r] = std::max(0, nloc_of(NT - 1, P, r) - li0_of(k, P, r));
      h->maxT[k] = std::max(h->maxT[k], cnt[(size_t)k * P + r]);
    }
    // diagonal tile: owner's local row k / P, column k, less the pending update
    // L(k, gb:k) L(k, gb:k)^T from its own row; then factored and inverted into its Dinv
    // (the Dinv block of the step's broadcast block)
    const bool gath = gather_panels(h);
    DLaunch dl;
    dl.first = (int)probs.size();
    if (Rank* R = rank_slot(h, k % P)) {
      double* Ckk = R->A + (long long)(k / P) * TILE + (long long)k * TILE * R->ld;
      const double* Lk = R->A + (long long)(k / P) * TILE + (long long)gb * TILE * R->ld;
      // the pending update as DQ_N 32 x 32-block workgroups (as the single-GPU sweep), which
      // the G_DIAG workgroup waits for (they precede it in the launch)
      if (Kp > 0) {
        GemmProb q = dprob(Lk, R->ld, nullptr, 0, Ckk, R->ld, DQ_N, 1, Kp, G_DQUAD, -1.0, 1.0);
        q.post = h->dq + k;
        q.diag_col0 = k * TILE;
        q.tile_begin = dl.tiles;
        q.ntiles = DQ_N;
        dl.tiles += DQ_N;
        probs.push_back(q);
        ++dl.count;
      }
      GemmProb p = dprob(nullptr, R->ld, nullptr, R->ld, Ckk, R->ld, 1, 1, 0, G_DIAG, 1.0, 1.0);
      if (Kp > 0) {
        p.pre0 = h->dq + k;
        p.pre0_n = DQ_N;
      }
      p.X = gath ? R->dinv + (long long)Kp * TILE : R->dinv + (long long)k * TILE * TILE;
      p.ldx = TILE;
      p.logdet = R->logdet + k;
      p.diag_col0 = k * TILE;
      // P = 1: the factor releases this launch's panel tiles through a flag once L and
      // the leaf inverses are stored (X is assembled after the sweep, k_xasm)
      if (!gath) p.flag = h->dq + NB + k;
      p.tile_begin = dl.tiles;
      p.ntiles = 1;
      dl.tiles += 1;
      dl.cdef = dl.cdef || gemm_cdef(p);
      probs.push_back(p);
      ++dl.count;
    }
    // P = 1 (the rank holds every row): the panel tiles ride in the same launch, as the
    // single-GPU fused sweep's: each G_PHALF0 workgroup applies the pending update
    // A(i,k) -= L(i, gb:k) L(k, gb:k)^T, stores it and posts, waits for the flag and solves
    // rows 0-63 of L(i,k) = A(i,k) L_kk^-T by block substitution; each G_PHALF1 workgroup
    // waits for the step's G_PHALF0 posts and solves rows 64-127.  (Dispatch follows the
    // problem order: every wait points to earlier workgroups.)  P > 1: the panel launch
    // after the broadcast applies the update and the inverse in one product.
    if (!gath) {
      Rank& R = h->ranks[0];
      const int a = li0_of(k, P, R.rank), c = std::max(0, R.nloc - a);
      if (c > 0) {
        double* Ckk = R.A + (long long)k * TILE + (long long)k * TILE * R.ld;
        GemmProb q = dprob(Kp ? R.A + (long long)a * TILE + (long long)gb * TILE * R.ld : nullptr, R.ld,
                           Kp ? R.A + (long long)k * TILE + (long long)gb * TILE * R.ld : nullptr, R.ld,
                           R.A + (long long)a * TILE + (long long)k * TILE * R.ld, R.ld, c, 1, Kp,
                           G_PANEL | G_PHALF0, Kp ? -1.0 : 1.0, 1.0);
        q.cpost = h->dq + 2 * NB + k;
        q.X = R.dinv + (long long)k * TILE * TILE;
        q.ldx = TILE;
        q.flag = h->dq + NB + k;
        q.diag_col0 = -TILE;   // (no GEMM_TRACE slot)
        q.Ld = Ckk;
        q.ldd = R.ld;
        q.tile_begin = dl.tiles;
        q.ntiles = c;
        dl.tiles += c;
        dl.cdef = dl.cdef || gemm_cdef(q);
        probs.push_back(q);
        ++dl.count;
        GemmProb q1 = q;
        q1.flags = G_PANEL | G_PHALF1;
        q1.A = q1.B = nullptr;
        q1.K = 0;
        q1.alpha = 1.0;
        q1.beta = 0.0;
        q1.pre0 = q.cpost;
        q1.pre0_n = c;
        q1.cpost = nullptr;
        q1.tile_begin = dl.tiles;
        dl.tiles += c;
        probs.push_back(q1);
        ++dl.count;
      }
    }
    // in-launch waits (quadrants -> factor, factor -> panel halves, halves -> halves): the
    // workgroups take their positions by ticket, as the single-GPU sweep's
    if (dl.count > 1) dl.ticket = h->dq + 3 * NB + k;
    h->diag[k] = dl;
    // P > 1, Kp > 0: the owner's M block of the broadcast, -Dinv L(k, gb:k) (its own row)
    if (gath && Kp > 0)
      if (Rank* R = rank_slot(h, k % P)) {
        DLaunch ml;
        ml.first = (int)probs.size();
        GemmProb p = dprob(R->dinv + (long long)Kp * TILE, TILE,
                           R->A + (long long)(k / P) * TILE + (long long)gb * TILE * R->ld, R->ld, R->dinv, TILE,
                           1, Kp / TILE, TILE, 0, -1.0, 0.0);
        p.tile_begin = 0;
        p.ntiles = Kp / TILE;
        ml.tiles = p.ntiles;
        ml.count = 1;
        ml.kind = 1;
        probs.push_back(p);
        h->mrow[k] = ml;
      }
    // panel over each local rank's rows i > k: P = 1, L(i,k) = A(i,k) Dinv^T (pending update
    // applied in the diagonal launch); P > 1, L(i,k) = [L(i, gb:k) A(i,k)] [-M Dinv]^T =
    // (A(i,k) - L(i, gb:k) L(k, gb:k)^T) Dinv^T, one product with K = Kp + 128 over the
    // row's columns gb..k (in place: each tile reads only its own rows before storing)
    DLaunch pl;
    pl.first = (int)probs.size();
    for (Rank& R : h->ranks) {
      const int a = li0_of(k, P, R.rank), c = std::max(0, R.nloc - a);
      if (c == 0 || !gath) continue;
      double* Aik = R.A + (long long)a * TILE + (long long)k * TILE * R.ld;
      GemmProb p = gath ? dprob(R.A + (long long)a * TILE + (long long)gb * TILE * R.ld, R.ld, R.dinv, TILE, Aik,
                                R.ld, c, 1, Kp + TILE, 0, 1.0, 0.0)
                        : dprob(Aik, R.ld, R.dinv + (long long)Kp * TILE, TILE, Aik, R.ld, c, 1, TILE, 0, 1.0, 0.0);
      p.tile_begin = pl.tiles;
      p.ntiles = c;
      pl.tiles += c;
      probs.push_back(p);
      ++pl.count;
    }
    pl.kind = 4;
    h->panel_l[k] = pl;
    // the step closing a group: trailing update of each local rank's rows by the
    // whole group, columns ge <= j <= i, K = 128 (ge - gb), in three launches: the next
    // group's columns ge <= j < ge2 (its chain waits for these), the group after it
    // (ge2 <= j < ge3: the next chain's own next-group update waits for these), then the rest
    if (k + 1 != ge) continue;
    const int ge2 = next_group_end(h, k);
    const int ge3 = ge2 < NB ? next_group_end(h, ge2 - 1) : NB;
    for (int part = 0; part < 3; ++part) {
      const int j0 = part == 0 ? ge : (part == 1 ? ge2 : ge3), j1 = part == 0 ? ge2 : (part == 1 ? ge3 : NT);
      DLaunch ul;
      ul.first = (int)probs.size();
      ul.list = (long long)tiles.size();
      int pi = 0;
      for (Rank& R : h->ranks) {
        const int a = li0_of(k, P, R.rank);
        if (a >= R.nloc) continue;
        GemmProb p = dprob(R.A + (long long)gb * TILE * R.ld, R.ld, panel_of(h, R, k), ldp, R.A, R.ld,
                           R.nloc, NT, (ge - gb) * TILE, 0, -1.0, 1.0);
        for (int li = a; li < R.nloc; ++li) {
          const int gt = li * P + R.rank;
          for (int j = j0; j < j1 && j <= gt; ++j)
            tiles.push_back(((unsigned)pi << 24) | ((unsigned)li << 12) | (unsigned)j);
        }
        ul.cdef = ul.cdef || gemm_cdef(p);
        probs.push_back(p);
        ++pi;
        ++ul.count;
      }
      ul.tiles = (int)(tiles.size() - ul.list);
      if (ul.tiles == 0) ul.count = 0;
      if (ul.tiles > 0) {   // (at most 256 problems: one per local rank)
        const std::vector<unsigned> mine(tiles.begin() + ul.list, tiles.end());
        const std::vector<unsigned> ord = xcd_order(probs.data() + ul.first, mine);
        std::copy(ord.begin(), ord.end(), tiles.begin() + ul.list);
      }
      ul.kind = 4;
      (part == 0 ? h->upd_next : (part == 1 ? h->upd_near : h->upd_far))[k] = ul;
    }
  }
  if (!gather_panels(h) && h->next_on_chain && h->fuse_next) DCHK(fuse_next_factor(h, probs, tiles));
  if ((int)probs.size() > DIST_DESC_MAX) return dfail(h, GPE_ERR_UNSUPPORTED, "distributed schedule too large");
  DCHK(dalloc(h, &h->dprobs, probs.size()));
  DCHK_HIP(h, hipMemcpy(h->dprobs, probs.data(), probs.size() * sizeof(GemmProb), hipMemcpyHostToDevice));
  DCHK(dalloc(h, &h->dtiles, std::max<size_t>(tiles.size(), 1)));
  if (!tiles.empty())
    DCHK_HIP(h, hipMemcpy(h->dtiles, tiles.data(), tiles.size() * sizeof(unsigned), hipMemcpyHostToDevice));
  DCHK(dalloc(h, &h->dli0, li0.size()));
  DCHK(dalloc(h, &h->dcnt, cnt.size()));
  DCHK_HIP(h, hipMemcpy(h->dli0, li0.data(), li0.size() * sizeof(int), hipMemcpyHostToDevice));
  DCHK_HIP(h, hipMemcpy(h->dcnt, cnt.data(), cnt.size() * sizeof(int), hipMemcpyHostToDevice));
  return GPE_OK;
}

// the sweep's launches (dprobs / dtiles), or the gradient's (gprobs / gtiles) with grad
int launch(gpe_dist* h, const DLaunch& L, bool grad = false) {
  if (L.count == 0 || L.tiles == 0) return GPE_OK;
  const size_t lds = G_LDS_LAUNCH_DOUBLES * sizeof(double);
  const unsigned* tl = L.list >= 0 ? (grad ? h->gtiles : h->dtiles) + L.list : nullptr;
  const GemmProb* pr = (grad ? h->gprobs : h->dprobs) + L.first;
  const dim3 g(L.tiles);
  const dim3 b(256);
  if (L.cdef) {
    switch (L.kind) {
      case 1: hipLaunchKernelGGL((k_gemm<false, true, false, true>), g, b, lds, h->cs, pr, L.count, tl, h->dinfo, nullptr); break;
      case 2: hipLaunchKernelGGL((k_gemm<true, true, false, true>), g, b, lds, h->cs, pr, L.count, tl, h->dinfo, nullptr); break;
      case 3: hipLaunchKernelGGL((k_gemm<true, false, false, true>), g, b, lds, h->cs, pr, L.count, tl, h->dinfo, nullptr); break;
      case 4: hipLaunchKernelGGL((k_gemm<false, false, false, true>), g, b, lds, h->cs, pr, L.count, tl, h->dinfo, nullptr); break;
      default:   // kind 0 launches may carry G_DIAG / G_PANEL problems
        hipLaunchKernelGGL((k_gemm<false, false, true, true>), g, b, lds, h->cs, pr, L.count, tl, h->dinfo, L.ticket); break;
    }
  } else {
    switch (L.kind) {
      case 1: hipLaunchKernelGGL((k_gemm<false, true>), g, b, lds, h->cs, pr, L.count, tl, h->dinfo, nullptr); break;
      case 2: hipLaunchKernelGGL((k_gemm<true, true>), g, b, lds, h->cs, pr, L.count, tl, h->dinfo, nullptr); break;
      case 3: hipLaunchKernelGGL((k_gemm<true, false>), g, b, lds, h->cs, pr, L.count, tl, h->dinfo, nullptr); break;
      case 4: hipLaunchKernelGGL((k_gemm<false, false>), g, b, lds, h->cs, pr, L.count, tl, h->dinfo, nullptr); break;
      default:   // kind 0 launches may carry G_DIAG / G_PANEL problems
        hipLaunchKernelGGL((k_gemm<false, false, true>), g, b, lds, h->cs, pr, L.count, tl, h->dinfo, L.ticket); break;
    }
  }
  DCHK_HIP(h, hipGetLastError());
  return GPE_OK;
}

// first local tile row of rank r whose global row is >= a
int lstart_of(int a, int P, int r) { return a <= r ? 0 : (a - r + P - 1) / P; }

// ---- the A^-1 partial on the int8 cores.  Rank r's partial X_r^T X_r is the product of
// op = X_r^T with itself: op's rows are the columns of X_r (np2 of them, 256-row tiles),
// its k the rank's rows (oz_kp = rank 0's, the most).  Column c of X_r is zero on the local
// rows whose global tile row is below c's, so the tiles of op-row tile ti start at local
// row 128 floor(2 ti / P) (OzGemm kbeg 3).  One launch pair (k_oz_gemm, k_oz_crt) per slab
// of tile rows [a0, a1) writes the slab's lower tiles, in place of the fp64 slab launch.
int oz_prepare(gpe_dist* h) {
  const int NB = h->NB, P = h->P, N = h->oz_nmod;
  const int np2 = (int)((h->n_pad + OZ_T - 1) / OZ_T * OZ_T), Kp = ((NB - 1) / P + 1) * TILE;
  h->oz_np2 = np2;
  h->oz_kp = Kp;
  h->oz_c = oz_consts(N, Kp);
  std::vector<unsigned> all;
  h->oz_lists.clear();
  long long maxt = 0;
  for (const SlabLaunch& sl : h->slabs[0]) {   // (the same slab bounds on every rank)
    const int ti0 = sl.a0 / 2, ti1 = (sl.a1 + 1) / 2;
    const std::vector<unsigned> l = oz_list(ti1 - ti0, ti1, true, [&](int ti, int) {
      return (double)std::max(0, Kp - 128 * ((2 * ti) / P));
    }, ti0);
    h->oz_lists.push_back({(long long)all.size(), (int)l.size()});
    all.insert(all.end(), l.begin(), l.end());
    maxt = std::max(maxt, (long long)ti1 * (ti1 + 1) / 2 - (long long)ti0 * (ti0 + 1) / 2);
  }
  h->oz_res_bytes = maxt * OZ_T * OZ_T;
  // P = 1: the TRTRI levels whose blocks have at least oz_tri_min rows, each in one chunk,
  // as the single-GPU path's int8 pairs (oz_tri_pair_launches: T in the slab, in place of
  // the M^T blocks); the partial's buffers are the larger
  const size_t slab_doubles = (size_t)h->ranks[0].slab_doubles;
  for (TriChunk& tc : h->tri) {
    tc.oz.clear();
    const int a = tc.s / 2;
    if (P != 1 || tc.cw != a || (long long)a * TILE < h->oz_tri_min) continue;
    std::vector<unsigned> lists = all;
    std::vector<OzTriPair> prs;
    bool fits = true;
    for (int t0 = 0; t0 + a < NB; t0 += tc.s) {
      const OzTriPair q = oz_tri_pair_plan(t0, t0 + a, std::min(t0 + tc.s, NB), N, lists);
      fits = fits && q.planes_bytes(N) <= (size_t)N * np2 * Kp && q.resid_bytes(N) <= (size_t)N * h->oz_res_bytes &&
             (size_t)q.Pa * q.Pb <= slab_doubles && q.Pa + q.Pb <= np2;
      prs.push_back(q);
    }
    if (!fits) continue;
    all = lists;
    tc.oz = prs;
  }
  DCHK(dalloc(h, &h->ozp, (size_t)N * np2 * Kp, &h->shared_bytes));
  DCHK(dalloc(h, &h->ozr, (size_t)N * h->oz_res_bytes, &h->shared_bytes));
  DCHK(dalloc(h, &h->ozx, (size_t)np2, &h->shared_bytes));
  DCHK(dalloc(h, &h->ozl, all.size(), &h->shared_bytes));
  DCHK_HIP(h, hipMemcpy(h->ozl, all.data(), all.size() * sizeof(unsigned), hipMemcpyHostToDevice));
  return GPE_OK;
}

// rank R's column exponents and planes of X_r^T (rows past n_pad and k past its rows: zero)
int oz_split_rank(gpe_dist* h, const Rank& R) {
  const int np2 = h->oz_np2, Kp = h->oz_kp, Kv = R.nlx * TILE;
  const OzConst& k = h->oz_c;
  hipLaunchKernelGGL(k_oz_rowexp<false>, dim3(np2 / 4), dim3(256), 0, h->stream, R.X, R.ld, (int)h->n_pad, np2, Kv,
                     0, k.beta, h->ozx);
  hipLaunchKernelGGL(k_oz_split_rect<false>, dim3(np2, (Kp + 2047) / 2048), dim3(256), 0, h->stream, R.X, R.ld,
                     (int)h->n_pad, Kv, 0, h->ozx, h->ozp, (long long)np2 * Kp, (long long)Kp, Kp, k);
  DCHK_HIP(h, hipGetLastError());
  return GPE_OK;
}

// slab si of rank R's partial: tile rows [a0, a1) (a0 even), their lower tiles into R.slab
int oz_slab(gpe_dist* h, const Rank& R, const SlabLaunch& sl, size_t si) {
  const int np2 = h->oz_np2, Kp = h->oz_kp;
  const int ti0 = sl.a0 / 2, ti1 = (sl.a1 + 1) / 2;
  const OzConst& k = h->oz_c;
  OzGemm g;
  g.a = g.b = OzOpnd{h->ozp, (long long)np2 * Kp, (long long)Kp, 0};
  g.list = h->ozl + h->oz_lists[si].first;
  g.list_len = h->oz_lists[si].second;
  g.K = Kp;
  g.kbeg = 3;
  g.kdiv = h->P;
  g.kend = 0;
  g.tri = 1;
  g.ntj = 0;
  g.res = h->ozr;
  g.res_bytes = h->oz_res_bytes;
  g.ti0 = ti0;
  hipLaunchKernelGGL(k_oz_gemm, dim3(k.nmod * g.list_len), dim3(256), OZ_LDS, h->stream, g, k);
  const int rows = sl.a1 * TILE;
  OzCrt r{h->ozr, h->oz_res_bytes, 1, 0, h->ozx, h->ozx, R.slab, (long long)h->slab_rows * TILE, rows, rows, 1, 1.0, ti0};
  const long long nt = (long long)ti1 * (ti1 + 1) / 2 - (long long)ti0 * (ti0 + 1) / 2;
  hipLaunchKernelGGL(k_oz_crt, dim3((unsigned)(nt * 16)), dim3(256), 0, h->stream, r, k);
  DCHK_HIP(h, hipGetLastError());
  return GPE_OK;
}

// gradient buffers and GEMM descriptors (TRTRI steps, W partial, A^-1 slabs)
int ensure_grad(gpe_dist* h) {
  if (h->grad_ready) return GPE_OK;
  const int NB = h->NB, P = h->P, Pc = h->q + 1, d = h->d;
  const long long np = h->n_pad;
  // slab of the A^-1 partial (and the TRTRI's gathered blocks): as many tile rows as
  // fit SLAB_DOUBLES, or GPEMU_DIST_SLAB_MB MiB (at least one tile row)
  long long slab_doubles = (long long)SLAB_DOUBLES;
  // when the whole lower triangle's tile rows take at most 4x that (n <= 16384), a slab
  // of 1/P of them (at P = 1 the partial then forms in one launch, as the single-GPU
  // LAUUM; per-rank memory stays O(n^2 / P): at P >= 4 the slab is the default)
  const long long whole = (long long)NB * TILE * np;
  if (whole <= 4 * (long long)SLAB_DOUBLES) slab_doubles = std::max(slab_doubles, whole / P);
  if (const char* e = std::getenv("GPEMU_DIST_SLAB_MB")) slab_doubles = std::max(1ll, std::atoll(e)) << 17;
  h->slab_rows = (int)std::max<long long>(1, std::min<long long>(NB, slab_doubles / (TILE * np)));
  const int tri_rows = h->slab_rows;   // the TRTRI's gathered blocks fit tri_rows tile rows
  // the int8 partial (oz_slab): products of sums over a rank's rows, oz_kp <= 2^17 keeps the
  // int32 accumulators exact; its 256-row tiles need every slab but the last to start at an
  // even tile row.  Its planes take 2 x the bytes of the rank's rows of L^-1: on only while
  // they fit oz_cap_mb (16 GiB; GPEMU_DIST_OZAKI_MB), so a rank of C4 takes them from P = 8
  const int nlx0 = (NB - 1) / P + 1;
  const double oz_planes = (double)h->oz_nmod * ((np + OZ_T - 1) / OZ_T * OZ_T) * nlx0 * TILE;
  h->oz_now = h->oz_on && np >= h->oz_min_np && (long long)nlx0 * TILE < (1 << 17) &&
              oz_planes <= (double)h->oz_cap_mb * (1 << 20);
  if (h->oz_now && h->slab_rows < NB && (h->slab_rows & 1)) h->slab_rows = std::max(2, h->slab_rows - 1);
  const long long lds = (long long)h->slab_rows * TILE;
  for (Rank& R : h->ranks) {
    R.nlx = R.rank <= NB - 1 ? (NB - 1 - R.rank) / P + 1 : 0;
    DCHK(dalloc(h, &R.X, (size_t)R.ld * NB * TILE, &R.bytes));
    DCHK(dalloc(h, &R.dZ, (size_t)np * Pc, &R.bytes));
    DCHK(dalloc(h, &R.dR2, (size_t)np * Pc, &R.bytes));
    DCHK(dalloc(h, &R.r2loc, (size_t)R.ld * h->NA * TILE, &R.bytes));
    DCHK_HIP(h, hipMemset(R.r2loc, 0, (size_t)R.ld * h->NA * TILE * sizeof(double)));
    DCHK(dalloc(h, &R.wpart, (size_t)np * h->NA * TILE, &R.bytes));
    R.slab_doubles = (long long)std::max(h->slab_rows, tri_rows) * TILE * np;
    DCHK(dalloc(h, &R.slab, (size_t)R.slab_doubles, &R.bytes));
    DCHK(dalloc(h, &R.csum, (size_t)d + 3, &R.bytes));
  }
  DCHK(dalloc(h, &h->dT2, (size_t)Pc * Pc, &h->shared_bytes));
  DCHK(dalloc(h, &h->cpart, (size_t)NB * (NB + 1) / 2 * (d + 3), &h->shared_bytes));

  // X = L^-1 by the recursive TRTRI of the single-GPU path (gpemu.hip build_plan), level
  // by level (block pairs [t0, h), [h, t1) of s tile columns, s = 2, 4, ...; the
  // diagonal tiles X(t,t) = Dinv_t were kept from the sweep), on the tile rows each rank
  // owns:
  //   M^T = X11^T L21^T  X11 = X(t0:h, t0:h) gathered from every rank, L21 the rank's
  //                      rows of L(h:t1, t0:h): its columns of M^T (its rows of M)
  //   X21 = -X22 M       M gathered; the rank's rows of X22 (finished a level earlier)
  // in column chunks [c0, c0 + cw) of [t0, h), as wide as the gathered blocks fit the
  // slab (X11's rows c0:h of the chunk's columns, M^T's chunk rows).  Two all-gathers
  // per chunk; none at P = 1, where X11 is read in place and M^T lands in the slab.
  std::vector<GemmProb> probs;
  std::vector<MoveDesc> moves;
  h->tri.clear();
  const long long cap = (long long)tri_rows * TILE * np, T2 = (long long)TILE * TILE;
  struct Pair { int t0, h, t1; };
  std::vector<std::pair<int, int>> lev;   // per level: {s, chunk width}
  long long g1_need = 0, rv_need = 0;
  for (int s = 2; s / 2 < NB; s *= 2) {
    const int a = s / 2;
    long long g1 = 0, s1 = 0, g2 = 0, s2 = 0;   // per unit of chunk width
    for (int t0 = 0; t0 + a < NB; t0 += s) {
      const int b = std::min(t0 + s, NB) - (t0 + a);
      g1 += a; s1 += (a + P - 1) / P; g2 += b; s2 += (b + P - 1) / P;
    }
    // (M^T's blocks live in the slab: g2 <= NB tiles always fits; the gathered X11 and the
    // all-gather buffer are sized to the slab as well, except at width 1, where the
    // segments' per-pair rounding to ceil(rows / P) may take them past it at small levels)
    int cc = a;
    auto fits = [&](long long w) {
      return g2 * w * T2 <= cap && (P == 1 || (g1 * w * T2 <= cap && P * s1 * w * T2 <= cap && P * s2 * w * T2 <= cap));
    };
    while (cc > 1 && !fits(cc)) cc = (cc + 1) / 2;
    if (g2 * cc * T2 > cap) return dfail(h, GPE_ERR_UNSUPPORTED, "distributed TRTRI blocks exceed the slab");
    lev.push_back({s, cc});
    if (P > 1) {
      g1_need = std::max(g1_need, g1 * cc * T2);
      rv_need = std::max({rv_need, P * s1 * cc * T2, P * s2 * cc * T2});
    }
  }
  for (Rank& R : h->ranks) {
    DCHK(dalloc(h, &R.g1, (size_t)g1_need, &R.bytes));
    // the TRTRI's all-gather buffer runs after the sweep: it shares the sweep's group
    // all-gather buffer when that is large enough (stream order separates their uses)
    if (R.trecv == R.recv) R.trecv = nullptr;
    if (R.recv && (size_t)rv_need <= (size_t)P * h->recv_tiles * TILE * TILE) {
      dfree(&R.trecv);
      R.trecv = R.recv;
    } else {
      DCHK(dalloc(h, &R.trecv, (size_t)rv_need, &R.bytes));
    }
  }
  for (const auto& lv : lev) {
    const int s = lv.first, a = s / 2, cc = lv.second;
    std::vector<Pair> pairs;
    for (int t0 = 0; t0 + a < NB; t0 += s) pairs.push_back({t0, t0 + a, std::min(t0 + s, NB)});
    for (int j0 = 0; j0 < a; j0 += cc) {
      const int cw = std::min(cc, a - j0), rows1 = a - j0, mx1 = (rows1 + P - 1) / P;
      TriChunk tc;
      tc.s = s;
      tc.cw = cw;
      // per pair: offsets in the all-gather segments (o1, o2) and the gathered blocks (og1, og2)
      std::vector<long long> o1, og1, o2, og2;
      long long s1 = 0, gg1 = 0, s2 = 0, gg2 = 0;
      for (const Pair& pr : pairs) {
        const int b = pr.t1 - pr.h;
        o1.push_back(s1 * T2); s1 += (long long)mx1 * cw;
        og1.push_back(gg1 * T2); gg1 += (long long)rows1 * cw;
        o2.push_back(s2 * T2); s2 += (long long)cw * ((b + P - 1) / P);
        og2.push_back(gg2 * T2); gg2 += (long long)cw * b;
      }
      tc.seg1 = (size_t)(s1 * T2);
      tc.seg2 = (size_t)(s2 * T2);
      auto add_move = [&](MoveDesc m, int& tiles) {
        if (m.rows <= 0 || m.cols <= 0) return;
        m.tile_begin = tiles;
        tiles += m.rows * m.cols;
        moves.push_back(m);
      };
      if (P > 1) {   // the rank's rows c0:h of X11's chunk columns into its segment, then out by rows
        tc.pack0 = (int)moves.size();
        for (Rank& R : h->ranks)
          for (size_t p = 0; p < pairs.size(); ++p) {
            const int c0 = pairs[p].t0 + j0, ls = lstart_of(c0, P, R.rank);
            const int nown = std::min(R.nlx, lstart_of(pairs[p].h, P, R.rank)) - ls;
            add_move({R.X + (long long)ls * TILE + (long long)c0 * TILE * R.ld, R.trecv + R.rank * tc.seg1 + o1[p],
                      R.ld, (long long)mx1 * TILE, 0, nown, cw, 0, 0, 0, P}, tc.pack_tiles);
          }
        tc.npack = (int)moves.size() - tc.pack0;
        tc.unp1 = (int)moves.size();
        for (Rank& R : h->ranks)
          for (size_t p = 0; p < pairs.size(); ++p)
            add_move({R.trecv + o1[p], R.g1 + og1[p], (long long)mx1 * TILE, (long long)rows1 * TILE,
                      (long long)tc.seg1, rows1, cw, 0, 1, pairs[p].t0 + j0, P}, tc.unp1_tiles);
        tc.nunp1 = (int)moves.size() - tc.unp1;
      }
      // M^T(c0:c0+cw, the rank's rows of h:t1) = X11(c0:h, c0:c0+cw)^T L21(rows, c0:h)^T
      // (X11 triangular: K from the output's row tile, G_KBEG_TI)
      tc.m.kind = 3;
      tc.m.first = (int)probs.size();
      for (Rank& R : h->ranks)
        for (size_t p = 0; p < pairs.size(); ++p) {
          const int c0 = pairs[p].t0 + j0, ls = lstart_of(pairs[p].h, P, R.rank);
          const int n2 = std::min(R.nlx, lstart_of(pairs[p].t1, P, R.rank)) - ls;
          if (n2 <= 0) continue;
          const double* A = P == 1 ? R.X + (long long)c0 * TILE + (long long)c0 * TILE * R.ld : R.g1 + og1[p];
          double* C = P == 1 ? R.slab + og2[p] : R.trecv + R.rank * tc.seg2 + o2[p];
          GemmProb q = dprob(A, P == 1 ? R.ld : (long long)rows1 * TILE,
                             R.A + (long long)ls * TILE + (long long)c0 * TILE * R.ld, R.ld, C, (long long)cw * TILE,
                             cw, n2, rows1 * TILE, G_KBEG_TI, 1.0, 0.0);
          q.tile_begin = tc.m.tiles;
          q.ntiles = cw * n2;
          tc.m.tiles += q.ntiles;
          ++tc.m.count;
          probs.push_back(q);
        }
      if (P > 1) {   // M^T's columns out of the segments, in global row order
        tc.unp2 = (int)moves.size();
        for (Rank& R : h->ranks)
          for (size_t p = 0; p < pairs.size(); ++p)
            add_move({R.trecv + o2[p], R.slab + og2[p], (long long)cw * TILE, (long long)cw * TILE,
                      (long long)tc.seg2, cw, pairs[p].t1 - pairs[p].h, 0, 2, pairs[p].h, P}, tc.unp2_tiles);
        tc.nunp2 = (int)moves.size() - tc.unp2;
      }
      // X21(i, c0:c0+cw) = -X22(i, h:i+1) M(h:i+1, c0:c0+cw) for the rank's rows i of
      // [h, t1): one problem per pair, local row ti = global row (ls + ti) P + rank with K
      // up to its diagonal (G_KEND_TI with kti_mul = P)
      tc.x.kind = 4;
      tc.x.first = (int)probs.size();
      for (Rank& R : h->ranks)
        for (size_t p = 0; p < pairs.size(); ++p) {
          const int c0 = pairs[p].t0 + j0, hh = pairs[p].h;
          const int ls = lstart_of(hh, P, R.rank);
          const int le = std::min(R.nlx, lstart_of(pairs[p].t1, P, R.rank));
          if (le <= ls) continue;
          double* row = R.X + (long long)ls * TILE;
          GemmProb q = dprob(row + (long long)hh * TILE * R.ld, R.ld, R.slab + og2[p], (long long)cw * TILE,
                             row + (long long)c0 * TILE * R.ld, R.ld, le - ls, cw, (pairs[p].t1 - hh) * TILE,
                             G_KEND_TI, -1.0, 0.0);
          q.kti_mul = P;
          q.kti_off = ls * P + R.rank - hh;
          q.tile_begin = tc.x.tiles;
          q.ntiles = (le - ls) * cw;
          tc.x.tiles += q.ntiles;
          ++tc.x.count;
          probs.push_back(q);
        }
      h->tri.push_back(tc);
    }
  }
  std::vector<unsigned> gt;
  for (TriChunk& tc : h->tri) {
    list_launch(tc.m, probs, gt);
    list_launch(tc.x, probs, gt);
  }
  if (!moves.empty()) {
    DCHK(dalloc(h, &h->dmoves, moves.size(), &h->shared_bytes));
    DCHK_HIP(h, hipMemcpy(h->dmoves, moves.data(), moves.size() * sizeof(MoveDesc), hipMemcpyHostToDevice));
  }
  {   // the W launch's split-K scratch (shared by the local ranks' launches, stream-ordered)
    const int ntw = NB * h->NA, ks = std::max(1, std::min(8, 512 / std::max(ntw, 1)));
    if (ks > 1) {
      DCHK(dalloc(h, &h->wsplit, (size_t)ntw * ks * TILE * TILE, &h->shared_bytes));
      DCHK(dalloc(h, &h->wcnt, (size_t)ntw, &h->shared_bytes));
      DCHK_HIP(h, hipMemset(h->wcnt, 0, (size_t)ntw * sizeof(int)));
    }
  }
  h->wa_l.assign(h->ranks.size(), DLaunch());
  h->slabs.assign(h->ranks.size(), std::vector<SlabLaunch>());
  for (size_t s = 0; s < h->ranks.size(); ++s) {
    Rank& R = h->ranks[s];
    DLaunch wl;
    wl.kind = 2;
    wl.first = (int)probs.size();
    // W(a) = X_r(:, a)^T R2_r over its rows >= a: one tile row of W per a, K up to n -- a
    // launch of NB tiles, so K is split over up to 8 workgroups per tile (last-arriver
    // reduction in index order, as the single-GPU split_k)
    const int ntw = (R.nlx > 0 ? NB : 0) * h->NA;
    const int ks = ntw > 0 ? std::max(1, std::min(8, 512 / ntw)) : 1;
    for (int a = 0; a < NB; ++a) {
      const int ls = lstart_of(a, P, R.rank), K = (R.nlx - ls) * TILE;
      if (K <= 0) continue;
      GemmProb p = dprob(R.X + (long long)ls * TILE + (long long)a * TILE * R.ld, R.ld,
                         R.r2loc + (long long)ls * TILE, R.ld, R.wpart + (long long)a * TILE, np,
                         1, h->NA, K, 0, 1.0, 0.0);
      if (ks > 1) {
        p.ksplit = ks;
        p.part = h->wsplit + (size_t)wl.tiles * ks * TILE * TILE;
        p.tcnt = h->wcnt + wl.tiles;
      }
      p.tile_begin = wl.tiles * ks;
      p.ntiles = h->NA * ks;
      wl.tiles += h->NA;
      ++wl.count;
      probs.push_back(p);
    }
    wl.tiles *= ks;
    h->wa_l[s] = wl;
    // partial of A^-1 by slabs of tile rows [a0, a1): P_r(a, 0:a+1) = X_r(:, a)^T X_r(:, 0:a+1)
    // over its rows >= a (K = 0 writes zeros), into slab row a - a0
    for (int a0 = 0; a0 < NB; a0 += h->slab_rows) {
      SlabLaunch sl;
      sl.a0 = a0;
      sl.a1 = std::min(NB, a0 + h->slab_rows);
      sl.gemm.kind = 2;
      sl.gemm.first = (int)probs.size();
      for (int a = sl.a0; a < sl.a1; ++a) {
        const int ls = lstart_of(a, P, R.rank), K = std::max(0, (R.nlx - ls) * TILE);
        GemmProb p = dprob(R.X + (long long)ls * TILE + (long long)a * TILE * R.ld, R.ld,
                           R.X + (long long)ls * TILE, R.ld, R.slab + (long long)(a - a0) * TILE, lds,
                           1, a + 1, K, 0, 1.0, 0.0);
        p.tile_begin = sl.gemm.tiles;
        p.ntiles = a + 1;
        sl.gemm.tiles += a + 1;
        ++sl.gemm.count;
        probs.push_back(p);
      }
      h->slabs[s].push_back(sl);
    }
  }
  for (auto& v : h->slabs)
    for (SlabLaunch& sl : v) list_launch(sl.gemm, probs, gt);
  if ((int)probs.size() > DIST_DESC_MAX) return dfail(h, GPE_ERR_UNSUPPORTED, "distributed gradient schedule too large");
  if (h->oz_now) DCHK(oz_prepare(h));
  DCHK(dalloc(h, &h->gtiles, std::max<size_t>(gt.size(), 1), &h->shared_bytes));
  if (!gt.empty())
    DCHK_HIP(h, hipMemcpy(h->gtiles, gt.data(), gt.size() * sizeof(unsigned), hipMemcpyHostToDevice));
  DCHK(dalloc(h, &h->gprobs, probs.size(), &h->shared_bytes));
  DCHK_HIP(h, hipMemcpy(h->gprobs, probs.data(), probs.size() * sizeof(GemmProb), hipMemcpyHostToDevice));
  h->grad_ready = true;
  return GPE_OK;
}

int move_launch(gpe_dist* h, int first, int count, int tiles) {
  if (count == 0 || tiles == 0) return GPE_OK;
  hipLaunchKernelGGL(k_dist_move, dim3(tiles), dim3(256), 0, h->cs, h->dmoves + first, count);
  DCHK_HIP(h, hipGetLastError());
  return GPE_OK;
}

// the recursive TRTRI (ensure_grad), chunk by chunk on the compute stream
int trtri_all(gpe_dist* h) {
  h->cs = h->stream;
  for (const TriChunk& tc : h->tri) {
    if (!tc.oz.empty()) {   // P = 1, int8 pairs (oz_prepare)
      Rank& R = h->ranks[0];
      auto tile = [&](double* M, int i, int j) { return M + (long long)i * TILE + (long long)j * TILE * R.ld; };
      const OzConst& k = h->oz_c;
      for (const OzTriPair& q : tc.oz)
        oz_tri_pair_launches(h->stream, k, q, h->ozl, tile(R.A, q.h, q.t0), tile(R.X, q.t0, q.t0), tile(R.X, q.h, q.h),
                             tile(R.X, q.h, q.t0), R.ld, R.slab, h->ozp, h->ozr, h->ozx, false,
                             [&](const OzGemm& g, const OzCrt& r, int nti, double, double) {
                               hipLaunchKernelGGL(k_oz_gemm, dim3(k.nmod * g.list_len), dim3(256), OZ_LDS, h->stream, g, k);
                               hipLaunchKernelGGL(k_oz_crt, dim3((unsigned)(nti * g.ntj * 16)), dim3(256), 0, h->stream,
                                                  r, k);
                             });
      DCHK_HIP(h, hipGetLastError());
      continue;
    }
    if (h->P > 1) {
      DCHK(move_launch(h, tc.pack0, tc.npack, tc.pack_tiles));
      DCHK(coll_allgather(h, &Rank::trecv, tc.seg1));
      DCHK(move_launch(h, tc.unp1, tc.nunp1, tc.unp1_tiles));
    }
    DCHK(launch(h, tc.m, true));
    if (h->P > 1) {
      DCHK(coll_allgather(h, &Rank::trecv, tc.seg2));
      DCHK(move_launch(h, tc.unp2, tc.nunp2, tc.unp2_tiles));
    }
    DCHK(launch(h, tc.x, true));
  }
  return GPE_OK;
}

int kbuild(gpe_dist* h, int kernel, double nu, double s2, double rscale) {
  double coff, cdiag;
  if (kernel == GPE_KERNEL_ALT_NUG) {
    coff = 1.0;
    cdiag = 1.0 + nu * nu;
  } else {
    coff = 1.0 - nu;
    cdiag = 1.0;
  }
  for (Rank& R : h->ranks) {
    if (R.nloc == 0) continue;   // more ranks than tile rows
    DistPairArgs a;
    a.xw = h->dXw; a.F = h->dF; a.r = (h->has_r && rscale != 0.0) ? h->dr : nullptr; a.out = R.A;
    a.ld = R.ld; a.ldF = h->n_pad; a.d = h->d; a.n_valid = (int)h->n; a.NB = h->NB; a.nranks = h->P;
    a.rank = R.rank; a.nloc = R.nloc; a.Pc = h->q + 1;
    a.s2 = s2; a.coff = coff; a.cdiag = cdiag; a.rscale = rscale;
    const dim3 grid((unsigned)(R.nloc * (h->NB + h->NA)));
    if (h->d <= 4) hipLaunchKernelGGL(k_dist_kbuild<4>, grid, dim3(256), 0, h->stream, a);
    else if (h->d <= 8) hipLaunchKernelGGL(k_dist_kbuild<8>, grid, dim3(256), 0, h->stream, a);
    else if (h->d <= 10) hipLaunchKernelGGL(k_dist_kbuild<10>, grid, dim3(256), 0, h->stream, a);
    else if (h->d <= 16) hipLaunchKernelGGL(k_dist_kbuild<16>, grid, dim3(256), 0, h->stream, a);
    else if (h->d <= 20) hipLaunchKernelGGL(k_dist_kbuild<20>, grid, dim3(256), 0, h->stream, a);
    else if (h->d <= 32) hipLaunchKernelGGL(k_dist_kbuild<32>, grid, dim3(256), 0, h->stream, a);
    else hipLaunchKernelGGL(k_dist_kbuild_wide, grid, dim3(256), 0, h->stream, a);
    DCHK_HIP(h, hipGetLastError());
  }
  return GPE_OK;
}

// one column step of a group's chain: diag (the owner's factor), [the owner's M block],
// ONE broadcast of [-M | Dinv] (128 KB x (1 + pending columns)), panel
int step(gpe_dist* h, int k) {
  const int P = h->P, owner = k % P;
  const long long Kp = (long long)(k - h->gstart[k]) * TILE;
  DCHK(launch(h, h->diag[k]));
  DCHK(launch(h, h->mrow[k]));
  if (gather_panels(h)) DCHK(coll_bcast(h, &Rank::dinv, 0, (size_t)TILE * (Kp + TILE), owner));
  if (h->grad_now && gather_panels(h)) {
    if (Rank* O = rank_slot(h, owner)) {   // the diagonal tile of X = L^-1 (Dinv)
      hipLaunchKernelGGL(k_dist_tile, dim3(TILE / 8), dim3(256), 0, h->cs, O->dinv + Kp * TILE, (long long)TILE,
                         O->X + (long long)(k / P) * TILE + (long long)k * TILE * O->ld, (long long)O->ld);
      DCHK_HIP(h, hipGetLastError());
    }
  }
  return launch(h, h->panel_l[k]);
}

// P > 1, at the end of the group [gb, ge): every rank packs its tile rows below the group
// (global rows >= ge) of the group's W columns, tile row by tile row; ONE all-gather; the
// segments are unpermuted into the group's panel buffer in global row order, which the
// trailing update reads (rows >= ge only: the chain needed no gathered rows)
int gather_group(gpe_dist* h, int gb, int ge) {
  if (!gather_panels(h)) return GPE_OK;
  const int P = h->P, k = ge - 1, W = ge - gb, T = h->maxT[k];
  if (T <= 0) return GPE_OK;
  const long long ldp = (long long)(h->NB + h->NA) * TILE;
  const size_t blk = (size_t)T * TILE * TILE, seg = (size_t)W * blk;
  for (Rank& R : h->ranks) {
    const int a = li0_of(k, P, R.rank), c = std::max(0, R.nloc - a);
    if (c == 0) continue;
    for (int w = 0; w < W; ++w) {
      hipLaunchKernelGGL(k_dist_pack, dim3(c), dim3(256), 0, h->cs, R.A, R.ld, a, gb + w,
                         R.recv + (size_t)R.rank * seg + (size_t)w * blk);
      DCHK_HIP(h, hipGetLastError());
    }
  }
  DCHK(coll_allgather(h, &Rank::recv, seg));
  for (Rank& R : h->ranks)
    for (int w = 0; w < W; ++w) {
      hipLaunchKernelGGL(k_dist_unpermute, dim3(T, P), dim3(256), 0, h->cs, R.recv + (size_t)w * blk, (long long)seg,
                         h->dli0 + (size_t)k * P, h->dcnt + (size_t)k * P, P,
                         panel_of(h, R, k) + (long long)w * TILE * ldp, ldp);
      DCHK_HIP(h, hipGetLastError());
    }
  return GPE_OK;
}

int ensure_group_events(gpe_dist* h, size_t ng) {
  while (h->ev_chain.size() < ng) {
    hipEvent_t a, b, c, d;
    DCHK_HIP(h, hipEventCreateWithFlags(&a, hipEventDisableTiming));
    DCHK_HIP(h, hipEventCreateWithFlags(&b, hipEventDisableTiming));
    DCHK_HIP(h, hipEventCreateWithFlags(&c, hipEventDisableTiming));
    DCHK_HIP(h, hipEventCreateWithFlags(&d, hipEventDisableTiming));
    h->ev_chain.push_back(a);
    h->ev_next.push_back(b);
    h->ev_near.push_back(c);
    h->ev_far.push_back(d);
  }
  return GPE_OK;
}

// The column groups with one group of look-ahead.  Group g's chain (its steps) runs on
// the critical stream; its trailing update is three launches by columns: the next
// group's (A), the group after it (B) and the rest (C).  A runs on the critical stream
// right behind the chain, after B of the previous group (the only earlier update of
// those columns still possibly running: everything before it on the compute stream is
// done), so the next chain never queues behind the far update C of the previous group;
// B and C run on the compute stream after the chain, overlapping the next chains.
// Writers of one column's tiles never overlap: A(g) waits for B(g-1), which follows C(g-2)
// on the compute stream.  A group's gather (P > 1) refills the panel buffer of group g-2
// and waits for that group's C.  The compute stream finally waits for the critical one,
// so work queued on it afterwards follows the whole sweep.
// GPEMU_DIST_NEXT_ON_CHAIN=0: the round-5 schedule (A on the compute stream behind the
// previous group's B and C; the next chain waits for it).
int group_sweep(gpe_dist* h) {
  const int ng = (int)h->gs.size() - 1;
  DCHK(ensure_group_events(h, (size_t)ng));
  DCHK_HIP(h, hipEventRecord(h->ev_join, h->stream));
  DCHK_HIP(h, hipStreamWaitEvent(h->crit, h->ev_join, 0));
  if (h->next_on_chain) {
    for (int g = 0; g < ng; ++g) {
      const int gb = h->gs[g], ge = h->gs[g + 1];
      h->cs = h->crit;
      for (int k = gb; k < ge; ++k) DCHK(step(h, k));
      if (g >= 2 && gather_panels(h)) DCHK_HIP(h, hipStreamWaitEvent(h->crit, h->ev_far[g - 2], 0));
      DCHK(gather_group(h, gb, ge));
      DCHK_HIP(h, hipEventRecord(h->ev_chain[g], h->crit));
      h->cs = h->stream;
      DCHK_HIP(h, hipStreamWaitEvent(h->stream, h->ev_chain[g], 0));
      DCHK(launch(h, h->upd_near[ge - 1]));
      DCHK_HIP(h, hipEventRecord(h->ev_near[g], h->stream));
      DCHK(launch(h, h->upd_far[ge - 1]));
      DCHK_HIP(h, hipEventRecord(h->ev_far[g], h->stream));
      h->cs = h->crit;
      if (g >= 1) DCHK_HIP(h, hipStreamWaitEvent(h->crit, h->ev_near[g - 1], 0));
      DCHK(launch(h, h->upd_next[ge - 1]));
    }
    DCHK_HIP(h, hipEventRecord(h->ev_end, h->crit));
    DCHK_HIP(h, hipStreamWaitEvent(h->stream, h->ev_end, 0));
    h->cs = h->stream;
    return GPE_OK;
  }
  for (int g = 0; g < ng; ++g) {
    const int gb = h->gs[g], ge = h->gs[g + 1];
    h->cs = h->crit;
    if (g > 0) DCHK_HIP(h, hipStreamWaitEvent(h->crit, h->ev_next[g - 1], 0));
    for (int k = gb; k < ge; ++k) DCHK(step(h, k));
    DCHK(gather_group(h, gb, ge));
    DCHK_HIP(h, hipEventRecord(h->ev_chain[g], h->crit));
    h->cs = h->stream;
    DCHK_HIP(h, hipStreamWaitEvent(h->stream, h->ev_chain[g], 0));
    DCHK(launch(h, h->upd_next[ge - 1]));
    DCHK_HIP(h, hipEventRecord(h->ev_next[g], h->stream));
    DCHK(launch(h, h->upd_near[ge - 1]));
    DCHK(launch(h, h->upd_far[ge - 1]));
  }
  h->cs = h->stream;
  return GPE_OK;
}

void contract_launch(gpe_dist* h, const double* slab, long long lds, long long row0, int blk0, int nblk,
                     const double* wpart, int q1, const double* rdiag) {
  const int d = h->d, Pc = h->q + 1, bucket = std::max(d, Pc);
  const long long np = h->n_pad;
  const dim3 g(nblk);
  const int nv = (int)h->n;
  if (d > 32 || Pc > 33)
    hipLaunchKernelGGL(k_contract_wide, g, dim3(256), 0, h->stream, slab, lds, h->dXw, d, wpart, np, q1, nv, h->cpart, h->dinfo, blk0, row0, rdiag);
  else if (d == 10 && Pc <= 13)
    hipLaunchKernelGGL((k_contract<10, 13>), g, dim3(256), 0, h->stream, slab, lds, h->dXw, d, wpart, np, q1, nv, h->cpart, h->dinfo, blk0, row0, rdiag);
  else if (d == 20 && Pc <= 21)   // BASELINE configs[3]
    hipLaunchKernelGGL((k_contract<20, 21>), g, dim3(256), 0, h->stream, slab, lds, h->dXw, d, wpart, np, q1, nv, h->cpart, h->dinfo, blk0, row0, rdiag);
  else if (bucket <= 8)
    hipLaunchKernelGGL((k_contract<8, 9>), g, dim3(256), 0, h->stream, slab, lds, h->dXw, d, wpart, np, q1, nv, h->cpart, h->dinfo, blk0, row0, rdiag);
  else if (bucket <= 16)
    hipLaunchKernelGGL((k_contract<16, 17>), g, dim3(256), 0, h->stream, slab, lds, h->dXw, d, wpart, np, q1, nv, h->cpart, h->dinfo, blk0, row0, rdiag);
  else
    hipLaunchKernelGGL((k_contract<32, 33>), g, dim3(256), 0, h->stream, slab, lds, h->dXw, d, wpart, np, q1, nv, h->cpart, h->dinfo, blk0, row0, rdiag);
}

}  // namespace

extern "C" {

int gpe_dist_unique_id(uint8_t* out, int32_t len) {
  if (!out || len < (int32_t)sizeof(ncclUniqueId)) return GPE_ERR_ARG;
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return GPE_ERR_HIP;
  std::memcpy(out, &id, sizeof(id));
  return GPE_OK;
}

int32_t gpe_dist_owner(int32_t nranks, int32_t tile_row) {
  if (nranks <= 0 || tile_row < 0) return -1;
  return tile_row % nranks;
}

int32_t gpe_dist_local_rows(int64_t n, int32_t q, int32_t nranks, int32_t rank) {
  if (n <= 0 || q < 0 || nranks <= 0 || rank < 0 || rank >= nranks) return -1;
  const int NB = (int)((n + TILE - 1) / TILE);
  const int NA = (q + 1 + TILE - 1) / TILE;   // augmented [f H]^T tile rows (set_data)
  return nloc_of(NB + NA - 1, nranks, rank);
}

gpe_dist* gpe_dist_create(int32_t device, int32_t nranks, int32_t rank, const uint8_t* unique_id) {
  if (nranks <= 0 || nranks > 256 || (unique_id && (rank < 0 || rank >= nranks))) return nullptr;
  if (hipSetDevice(device) != hipSuccess) return nullptr;
  gpe_dist* h = new gpe_dist();
  h->device = device;
  h->P = nranks;
  h->rank = unique_id ? rank : 0;
  h->loop = unique_id == nullptr;
  if (const char* e = std::getenv("GPEMU_DIST_NEXT_ON_CHAIN")) h->next_on_chain = std::atoi(e) != 0;
  if (const char* e = std::getenv("GPEMU_DIST_FUSE_NEXT")) h->fuse_next = std::atoi(e) != 0;
  if (const char* e = std::getenv("GPEMU_OZAKI")) h->oz_on = std::atoi(e) != 0;
  if (const char* e = std::getenv("GPEMU_DIST_OZAKI_MB")) h->oz_cap_mb = std::max(0ll, std::atoll(e));
  if (const char* e = std::getenv("GPEMU_OZAKI_MIN_NP")) h->oz_min_np = std::max(512, std::atoi(e));
  if (const char* e = std::getenv("GPEMU_OZAKI_TRI_MIN")) h->oz_tri_min = std::max(512, std::atoi(e));
  if (const char* e = std::getenv("GPEMU_OZAKI_MODULI")) h->oz_nmod = std::max(8, std::min(OZ_MAXMOD, std::atoi(e)));
  // one rank: 8 wide while 64 tile columns remain (n = 16384, value 29.95-30.43 -> 29.49-29.60 ms,
  // gradient 66.1 -> 65.8-65.9; n = 65536 unchanged); with more ranks 8:160 stays (two loopback
  // ranks 44.6-44.8 against 47.6-47.9 ms for 8:64; profiles/dist_w_r06*.log)
  if (nranks == 1) h->groups = {{8, 64}, {4, 0}};
  if (const char* e = std::getenv("GPEMU_DIST_W")) {   // "4:80,2:40": {width, min remaining}
    h->groups.clear();
    std::string spec(e);
    size_t pos = 0;
    while (pos < spec.size()) {
      size_t end = spec.find(',', pos);
      if (end == std::string::npos) end = spec.size();
      const std::string item = spec.substr(pos, end - pos);
      const size_t colon = item.find(':');
      const int w = std::atoi(item.substr(0, colon).c_str());
      const int lim = colon == std::string::npos ? 0 : std::atoi(item.substr(colon + 1).c_str());
      if (w >= 1 && w <= 16) h->groups.push_back({w, lim});
      pos = end + 1;
    }
  }
  int lo = 0, hi = 0;   // the critical stream at the highest priority the device offers
  bool ok = hipDeviceGetStreamPriorityRange(&lo, &hi) == hipSuccess &&
            hipStreamCreateWithPriority(&h->crit, hipStreamNonBlocking, hi) == hipSuccess &&
            hipEventCreateWithFlags(&h->ev_join, hipEventDisableTiming) == hipSuccess &&
            hipEventCreateWithFlags(&h->ev_end, hipEventDisableTiming) == hipSuccess &&
            hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) == hipSuccess &&
            hipEventCreate(&h->e0) == hipSuccess && hipEventCreate(&h->e1) == hipSuccess &&
            hipMalloc((void**)&h->dinfo, sizeof(int)) == hipSuccess;
  if (ok && !h->loop) {
    ncclUniqueId id;
    std::memcpy(&id, unique_id, sizeof(id));
    ok = ncclCommInitRank(&h->comm, nranks, id, rank) == ncclSuccess;
  }
  if (!ok) {
    gpe_dist_destroy(h);
    return nullptr;
  }
  return h;
}

void gpe_dist_destroy(gpe_dist* h) {
  if (!h) return;
  (void)hipSetDevice(h->device);
  if (h->stream) (void)hipStreamSynchronize(h->stream);
  if (h->crit) (void)hipStreamSynchronize(h->crit);
  if (h->comm) (void)ncclCommDestroy(h->comm);
  for (Rank& R : h->ranks) free_rank(R);
  double** bufs[] = {&h->dX, &h->dXw, &h->dF, &h->dr, &h->dinvdelta, &h->cpart, &h->dT2};
  for (double** b : bufs) dfree(b);
  dfree(&h->dinfo);
  dfree(&h->dq);
  dfree(&h->dli0);
  dfree(&h->dcnt);
  dfree(&h->dprobs);
  dfree(&h->dtiles);
  dfree(&h->gprobs);
  dfree(&h->gtiles);
  dfree(&h->dmoves);
  dfree(&h->wsplit);
  dfree(&h->wcnt);
  dfree(&h->ozp);
  dfree(&h->ozr);
  dfree(&h->ozx);
  dfree(&h->ozl);
  if (h->hpin) (void)hipHostFree(h->hpin);
  for (hipEvent_t e : h->cev) (void)hipEventDestroy(e);
  if (h->e0) (void)hipEventDestroy(h->e0);
  if (h->e1) (void)hipEventDestroy(h->e1);
  for (hipEvent_t e : h->ev_chain) (void)hipEventDestroy(e);
  for (hipEvent_t e : h->ev_next) (void)hipEventDestroy(e);
  for (hipEvent_t e : h->ev_near) (void)hipEventDestroy(e);
  for (hipEvent_t e : h->ev_far) (void)hipEventDestroy(e);
  if (h->ev_join) (void)hipEventDestroy(h->ev_join);
  if (h->ev_end) (void)hipEventDestroy(h->ev_end);
  if (h->stream) (void)hipStreamDestroy(h->stream);
  if (h->crit) (void)hipStreamDestroy(h->crit);
  delete h;
}

const char* gpe_dist_last_error(gpe_dist* h) { return h ? h->err.c_str() : "null handle"; }

int gpe_dist_set_data(gpe_dist* h, int64_t n, int32_t d, int32_t q, const double* X, const double* f,
                      const double* H, const double* r) {
  if (!h) return GPE_ERR_ARG;
  // [f H]^T rides in the tile rows under the matrix (NB .. NB+NA-1), 128 columns each
  if (n <= 0 || d <= 0 || q < 0 || !X || !f || (q > 0 && !H))
    return dfail(h, GPE_ERR_ARG, "bad shapes");
  DCHK_HIP(h, hipSetDevice(h->device));
  DCHK_HIP(h, hipStreamSynchronize(h->stream));
  DCHK_HIP(h, hipStreamSynchronize(h->crit));
  h->n = n;
  h->d = d;
  h->q = q;
  h->NB = (int)((n + TILE - 1) / TILE);
  h->n_pad = (long long)h->NB * TILE;
  h->NA = (q + 1 + TILE - 1) / TILE;
  if (h->NB + h->NA > 4095) return dfail(h, GPE_ERR_UNSUPPORTED, "n too large for the tile list");
  const long long np = h->n_pad;
  const int Pc = q + 1;
  for (Rank& R : h->ranks) free_rank(R);
  h->ranks.clear();
  h->grad_ready = false;
  h->shared_bytes = 0;
  dfree(&h->cpart);
  dfree(&h->dT2);
  dfree(&h->gprobs);
  dfree(&h->gtiles);
  dfree(&h->dmoves);
  dfree(&h->wsplit);
  dfree(&h->wcnt);
  dfree(&h->ozp);
  dfree(&h->ozr);
  dfree(&h->ozx);
  dfree(&h->ozl);
  DCHK(pinned(h, (size_t)np * std::max(d, Pc) + 16));
  // X (row-major, zero padded)
  DCHK(dalloc(h, &h->dX, (size_t)np * d, &h->shared_bytes));
  DCHK(dalloc(h, &h->dXw, (size_t)np * d, &h->shared_bytes));
  std::memset(h->hpin, 0, (size_t)np * d * sizeof(double));
  std::memcpy(h->hpin, X, (size_t)n * d * sizeof(double));
  DCHK_HIP(h, hipMemcpy(h->dX, h->hpin, (size_t)np * d * sizeof(double), hipMemcpyHostToDevice));
  // [f H] column-major, zero padded
  DCHK(dalloc(h, &h->dF, (size_t)np * Pc, &h->shared_bytes));
  std::memset(h->hpin, 0, (size_t)np * Pc * sizeof(double));
  for (long long i = 0; i < n; ++i) {
    h->hpin[i] = f[i];
    for (int k = 0; k < q; ++k) h->hpin[i + (long long)(k + 1) * np] = H[i * q + k];
  }
  DCHK_HIP(h, hipMemcpy(h->dF, h->hpin, (size_t)np * Pc * sizeof(double), hipMemcpyHostToDevice));
  h->has_r = r != nullptr;
  dfree(&h->dr);
  if (r) {
    DCHK(dalloc(h, &h->dr, (size_t)np, &h->shared_bytes));
    std::memset(h->hpin, 0, (size_t)np * sizeof(double));
    std::memcpy(h->hpin, r, (size_t)n * sizeof(double));
    DCHK_HIP(h, hipMemcpy(h->dr, h->hpin, (size_t)np * sizeof(double), hipMemcpyHostToDevice));
  }
  DCHK(dalloc(h, &h->dinvdelta, (size_t)d, &h->shared_bytes));
  // local ranks and their sweep buffers
  build_groups(h);
  DCHK(dalloc(h, &h->dq, 6 * (size_t)h->NB, &h->shared_bytes));
  const int NT = h->NB + h->NA;
  h->panel_sz = (size_t)NT * TILE * TILE * h->wmax;
  // the group all-gather's segment: W column blocks of the most tile rows below the group
  // any rank holds (rows >= ge)
  h->recv_tiles = 0;
  for (size_t g = 0; g + 1 < h->gs.size(); ++g) {
    const int ge = h->gs[g + 1], W = ge - h->gs[g];
    int T = 0;
    for (int rr = 0; rr < h->P; ++rr) T = std::max(T, std::max(0, nloc_of(NT - 1, h->P, rr) - li0_of(ge - 1, h->P, rr)));
    h->recv_tiles = std::max(h->recv_tiles, (size_t)T * W);
  }
  for (int rr = 0; rr < h->P; ++rr) {
    if (!h->loop && rr != h->rank) continue;
    Rank R;
    R.rank = rr;
    R.nloc = nloc_of(NT - 1, h->P, rr);
    R.ld = (long long)std::max(R.nloc, 1) * TILE;
    h->ranks.push_back(R);
    Rank& B = h->ranks.back();
    DCHK(dalloc(h, &B.A, (size_t)B.ld * (size_t)NT * TILE, &B.bytes));
    DCHK(dalloc(h, &B.logdet, (size_t)h->NB + 1, &B.bytes));
    // P = 1: one leaf-inverse tile per step (the factors write them there; k_dist_leaves
    // moves all of them into X after the sweep, off the chain)
    DCHK(dalloc(h, &B.dinv, (size_t)TILE * TILE * (gather_panels(h) ? h->wmax : h->NB), &B.bytes));
    if (gather_panels(h)) {
      DCHK(dalloc(h, &B.panel, 2 * h->panel_sz, &B.bytes));
      DCHK(dalloc(h, &B.recv, (size_t)h->P * h->recv_tiles * TILE * TILE, &B.bytes));
    }
    DCHK(dalloc(h, &B.gram, (size_t)Pc * Pc, &B.bytes));
  }
  DCHK(build_schedule(h));
  DCHK(ensure_events(h, (size_t)8 * h->NB + 32));
  return GPE_OK;
}

int gpe_dist_objective(gpe_dist* h, int32_t variant, int32_t kernel, const double* hp, int32_t n_hp,
                       double nu_fixed, int32_t want_grad, double* llh_out, double* grad_out,
                       double* sigma2_out) {
  if (!h) return GPE_ERR_ARG;
  if (h->n <= 0) return dfail(h, GPE_ERR_STATE, "gpe_dist_set_data has not been called");
  if (!hp || !llh_out) return dfail(h, GPE_ERR_ARG, "null argument");
  if (want_grad && !grad_out) return dfail(h, GPE_ERR_ARG, "grad_out is NULL");
  if (variant != GPE_GP4ML && variant != GPE_MUCM) return dfail(h, GPE_ERR_ARG, "bad variant");
  if (kernel != GPE_KERNEL_STD && kernel != GPE_KERNEL_ALT_NUG) return dfail(h, GPE_ERR_ARG, "bad kernel");
  DCHK_HIP(h, hipSetDevice(h->device));
  // a previous call that failed inside group_sweep may have left chain work queued on the
  // critical stream, never joined into the compute stream: drain it before this call's
  // host staging and memsets (idle in the normal case)
  DCHK_HIP(h, hipStreamSynchronize(h->crit));
  const int d = h->d, q = h->q, Pc = q + 1, P = h->P, NB = h->NB;
  const long long np = h->n_pad;
  const bool gp4ml = variant == GPE_GP4ML;
  const int base = gp4ml ? d + 1 : d;
  if (n_hp != base && n_hp != base + 1) return dfail(h, GPE_ERR_ARG, "n_hp inconsistent with d");
  const bool fitnug = n_hp == base + 1;
  const double nu = fitnug ? hp[d] : nu_fixed;
  const double sigma = gp4ml ? hp[n_hp - 1] : 1.0;
  const double s2 = gp4ml ? sigma * sigma : 1.0;
  const double rscale = (gp4ml && kernel == GPE_KERNEL_ALT_NUG) ? 1.0 : 0.0;
  if (want_grad) DCHK(ensure_grad(h));
  h->grad_now = want_grad != 0;
  h->ev = 0;
  h->cs = h->stream;
  Rank& R0 = h->ranks[0];   // every rank holds the reduced results; read this process's first

  DCHK(pinned(h, (size_t)NB + 1 + (size_t)Pc * Pc + (size_t)(d + 3) + 64));
  for (int k = 0; k < d; ++k) {
    if (!(hp[k] > 0.0) && !(hp[k] < 0.0))   // as the single-GPU path: not positive definite
      return dfail(h, GPE_NOT_PD, "length scale delta[" + std::to_string(k) + "] is zero or NaN");
    h->hpin[k] = 1.0 / hp[k];
  }
  DCHK_HIP(h, hipEventRecord(h->e0, h->stream));
  DCHK_HIP(h, hipMemcpyAsync(h->dinvdelta, h->hpin, d * sizeof(double), hipMemcpyHostToDevice, h->stream));
  DCHK_HIP(h, hipMemsetAsync(h->dinfo, 0, sizeof(int), h->stream));
  const long long tot = np * d;
  hipLaunchKernelGGL(k_scale_points, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, h->stream, h->dX,
                     h->dinvdelta, d, (int)h->n, (int)np, h->dXw);
  DCHK_HIP(h, hipGetLastError());
  for (Rank& R : h->ranks) {
    DCHK_HIP(h, hipMemsetAsync(R.logdet, 0, (size_t)(NB + 1) * sizeof(double), h->stream));
    if (h->grad_now && R.nlx > 0)
      DCHK_HIP(h, hipMemsetAsync(R.X, 0, (size_t)R.ld * NB * TILE * sizeof(double), h->stream));
  }
  DCHK(kbuild(h, kernel, nu, s2, rscale));
  DCHK_HIP(h, hipMemsetAsync(h->dq, 0, 6 * (size_t)NB * sizeof(int), h->stream));
  DCHK(group_sweep(h));
  // P = 1: the sweep's factors stored L and the leaf inverses only (flag mode): the
  // TRTRI's leaves X(t, t) are assembled here for every diagonal tile at once
  if (h->grad_now && !gather_panels(h))
    for (Rank& R : h->ranks) {
      if (R.nlx == 0) continue;
      hipLaunchKernelGGL(k_dist_leaves, dim3(TILE / 8, NB), dim3(256), 0, h->stream, R.dinv, R.X, R.ld);
      hipLaunchKernelGGL(k_xasm, dim3(NB), dim3(256), DB_LDS_DOUBLES * sizeof(double), h->stream, R.A, R.X, R.ld);
      DCHK_HIP(h, hipGetLastError());
    }

  // Gram of L^-1 [f H] = -(the augmented rows' diagonal block; its lower tiles), and
  // Z = L^-1 [f H], from the owners of the augmented tile rows: each places its rows of
  // the Gram (the rest zero) for an all-reduce, and broadcasts its columns of Z
  for (Rank& R : h->ranks) DCHK_HIP(h, hipMemsetAsync(R.gram, 0, (size_t)Pc * Pc * sizeof(double), h->stream));
  for (int u = 0; u < h->NA; ++u) {
    const int gt = NB + u, p0 = u * TILE, pc = std::min(Pc - p0, TILE);
    if (Rank* O = rank_slot(h, gt % P)) {
      const double* t = O->A + (long long)(gt / P) * TILE + (long long)NB * TILE * O->ld;
      DCHK_HIP(h, hipMemcpy2DAsync(O->gram + p0, Pc * sizeof(double), t, O->ld * sizeof(double), pc * sizeof(double),
                                   p0 + pc, hipMemcpyDeviceToDevice, h->stream));
      if (h->grad_now) {
        hipLaunchKernelGGL(k_dist_take_z, dim3((unsigned)((np + 255) / 256)), dim3(256), 0, h->stream, O->A,
                           O->ld, gt / P, np, p0, pc, O->dZ);
        DCHK_HIP(h, hipGetLastError());
      }
    }
  }
  DCHK(coll_allreduce_sum(h, &Rank::gram, 0, (size_t)Pc * Pc));
  DCHK(coll_allreduce_sum(h, &Rank::logdet, 0, (size_t)NB + 1));
  DCHK(coll_info_max(h));
  if (h->grad_now)
    for (int u = 0; u < h->NA; ++u) {
      const int p0 = u * TILE, pc = std::min(Pc - p0, TILE);
      DCHK(coll_bcast(h, &Rank::dZ, (long long)p0 * np, (size_t)np * pc, (NB + u) % P));
    }
  // host reads behind an event; the triangular inverse (independent of the host
  // algebra) is queued first so the GPU does not idle over the round trip
  double* hld = h->hpin;
  double* hgram = h->hpin + (NB + 1);
  DCHK_HIP(h, hipMemcpyAsync(hld, R0.logdet, (NB + 1) * sizeof(double), hipMemcpyDeviceToHost, h->stream));
  DCHK_HIP(h, hipMemcpyAsync(hgram, R0.gram, (size_t)Pc * Pc * sizeof(double), hipMemcpyDeviceToHost, h->stream));
  DCHK_HIP(h, hipMemcpyAsync(hgram + Pc * Pc, h->dinfo, sizeof(int), hipMemcpyDeviceToHost, h->stream));
  DCHK_HIP(h, hipEventRecord(h->e1, h->stream));
  if (h->grad_now) DCHK(trtri_all(h));
  DCHK_HIP(h, hipEventSynchronize(h->e1));
  int info = 0;
  std::memcpy(&info, hgram + Pc * Pc, sizeof(int));
  if (info == GEMM_WAIT_TIMEOUT) {
    (void)hipStreamSynchronize(h->stream);
    return dfail(h, GPE_ERR_HIP, "internal error: flag wait timed out");
  }
  if (info != 0) {
    (void)hipStreamSynchronize(h->stream);   // the queued inverse steps skip themselves (abort flag)
    h->err = "matrix not positive definite (pivot " + std::to_string(info) + ")";
    return GPE_NOT_PD;
  }
  double logdetA = 0.0;
  for (int k = 0; k < NB; ++k) logdetA += hld[k];
  logdetA *= 2.0;
  std::vector<double> G((size_t)Pc * Pc);
  for (int i = 0; i < Pc; ++i)   // from the lower triangle (tiles above the diagonal are not formed)
    for (int j = 0; j < Pc; ++j) G[(size_t)i * Pc + j] = -hgram[std::max(i, j) + (size_t)std::min(i, j) * Pc];
  SmallAlgebra sa = small_from_gram(G, Pc);
  if (!sa.ok) {
    (void)hipStreamSynchronize(h->stream);
    h->err = "H^T A^-1 H not positive definite";
    return GPE_NOT_PD;
  }
  const double n = (double)h->n;
  double llh, sig2, cfac, gscale;
  if (gp4ml) {
    llh = 0.5 * (sa.quad + logdetA + sa.logdetQ + (n - q) * std::log(2.0 * M_PI));
    sig2 = s2;
    cfac = 1.0;
    gscale = s2;
  } else {
    sig2 = sa.quad / (n - q - 2.0);
    llh = 0.5 * ((n - q) * std::log(sig2) + logdetA + sa.logdetQ);
    cfac = (n - q) / (sig2 * (n - q - 2.0));
    gscale = sig2;
  }
  *llh_out = llh;
  if (sigma2_out) *sigma2_out = sig2;

  if (h->grad_now) {
    // R2 = Z T2; [sqrt(c) alpha, W] = X^T R2 = sum over ranks of X_r^T R2_r
    const std::vector<double> T2 = small_t2(sa, q, cfac);
    std::memcpy(h->hpin, T2.data(), T2.size() * sizeof(double));
    DCHK_HIP(h, hipMemcpyAsync(h->dT2, h->hpin, T2.size() * sizeof(double), hipMemcpyHostToDevice, h->stream));
    for (size_t s = 0; s < h->ranks.size(); ++s) {
      Rank& R = h->ranks[s];
      DCHK_HIP(h, hipMemsetAsync(R.wpart, 0, (size_t)np * h->NA * TILE * sizeof(double), h->stream));
      if (R.nlx == 0) continue;
      if (Pc <= SK_PMAX)
        hipLaunchKernelGGL(k_apply_small, dim3((unsigned)((np + 255) / 256)), dim3(256), 0, h->stream, R.dZ, np, Pc,
                           h->dT2, Pc, R.dR2, np, (int)np, h->dinfo);
      else
        hipLaunchKernelGGL(k_apply_big, dim3((unsigned)((np + 255) / 256)), dim3(256), 0, h->stream, R.dZ, np, Pc,
                           h->dT2, Pc, R.dR2, np, (int)np, h->dinfo);
      DCHK_HIP(h, hipGetLastError());
      const long long e = (long long)R.nlx * TILE;
      hipLaunchKernelGGL(k_dist_rows, dim3((unsigned)((e + 255) / 256)), dim3(256), 0, h->stream, R.dR2, np, Pc,
                         P, R.rank, R.nlx, R.r2loc, R.ld);
      DCHK_HIP(h, hipGetLastError());
      DCHK(launch(h, h->wa_l[s], true));
    }
    DCHK(coll_allreduce_sum(h, &Rank::wpart, 0, (size_t)np * Pc));
    // each rank: its partial of A^-1 slab by slab, each slab contracted at once
    const int nblk = NB * (NB + 1) / 2;
    const long long lds = (long long)h->slab_rows * TILE;
    // sum_i M_ii r_i for the std kernel's sigma gradient when r is set (small_grad)
    const double* rdiag = (gp4ml && kernel == GPE_KERNEL_STD && h->has_r) ? h->dr : nullptr;
    for (size_t s = 0; s < h->ranks.size(); ++s) {
      Rank& R = h->ranks[s];
      DCHK_HIP(h, hipMemsetAsync(R.csum, 0, (size_t)(d + 3) * sizeof(double), h->stream));
      if (R.nlx == 0) continue;
      const int q1 = R.rank == 0 ? Pc : 0;   // the -W W^T term once
      if (h->oz_now) DCHK(oz_split_rank(h, R));
      for (size_t si = 0; si < h->slabs[s].size(); ++si) {
        const SlabLaunch& sl = h->slabs[s][si];
        if (h->oz_now) DCHK(oz_slab(h, R, sl, si));
        else DCHK(launch(h, sl.gemm, true));
        const int b0 = sl.a0 * (sl.a0 + 1) / 2, b1 = sl.a1 * (sl.a1 + 1) / 2;
        contract_launch(h, R.slab, lds, (long long)sl.a0 * TILE, b0, b1 - b0, R.wpart, q1, rdiag);
        DCHK_HIP(h, hipGetLastError());
      }
      hipLaunchKernelGGL(k_reduce_rows, dim3(d + 3), dim3(256), 0, h->stream, h->cpart, nblk, d + 3, R.csum);
      DCHK_HIP(h, hipGetLastError());
    }
    DCHK(coll_allreduce_sum(h, &Rank::csum, 0, (size_t)d + 3));
  }
  DCHK_HIP(h, hipEventRecord(h->e1, h->stream));
  if (h->grad_now)
    DCHK_HIP(h, hipMemcpyAsync(h->hpin, R0.csum, (size_t)(d + 3) * sizeof(double), hipMemcpyDeviceToHost,
                               h->stream));
  DCHK_HIP(h, hipStreamSynchronize(h->stream));
  if (h->grad_now) {
    double coff, cdiag;
    if (kernel == GPE_KERNEL_ALT_NUG) {
      coff = 1.0;
      cdiag = 1.0 + nu * nu;
    } else {
      coff = 1.0 - nu;
      cdiag = 1.0;
    }
    std::vector<double> red(h->hpin, h->hpin + d + 3);
    small_grad(red.data(), d, kernel == GPE_KERNEL_ALT_NUG, nu, fitnug, gp4ml, gscale, s2, coff, cdiag, n_hp,
               grad_out, gp4ml && kernel == GPE_KERNEL_STD && h->has_r);
  }
  {
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, h->e0, h->e1);
    h->total_ms = ms;
    double c = 0.0;
    for (int i = 0; i + 1 < h->ev; i += 2) {
      ms = 0.f;
      (void)hipEventElapsedTime(&ms, h->cev[i], h->cev[i + 1]);
      c += ms;
    }
    h->comm_ms = c;
  }
  return GPE_OK;
}

int gpe_dist_times(gpe_dist* h, double* total_ms, double* comm_ms) {
  if (!h) return GPE_ERR_ARG;
  if (total_ms) *total_ms = h->total_ms;
  if (comm_ms) *comm_ms = h->comm_ms;
  return GPE_OK;
}

int gpe_dist_rank_bytes(gpe_dist* h, int32_t rank, int64_t* bytes_out) {
  if (!h || !bytes_out) return GPE_ERR_ARG;
  for (const Rank& R : h->ranks)
    if (R.rank == rank) {
      *bytes_out = (int64_t)(R.bytes + h->shared_bytes);
      return GPE_OK;
    }
  return dfail(h, GPE_ERR_ARG, "rank " + std::to_string(rank) + " is not held by this process");
}

}  // extern "C"
