// Latency of one 16x16 leaf factor + inverse (db_leaf / db_leaf_sc) on one wave (dev tool).
// hipcc --offload-arch=gfx950 -O3 -w tools/hip/leaf_probe.hip -o tools/hip/leaf_probe_bin
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include "../../gp_emu_uqsa_amd/csrc/gpemu_diag.hpp"
using namespace gpe;

// Same contract as db_leaf, with the column chain carried by scalar broadcasts:
// lanes 0-15 hold row i of the block (v[k] = A(i, k), k <= i), lanes 16-31 hold
// column c of X (v[k] = X(k, c), starting as e_c).  Per column j every lane forms
// own = v[j] * rsq(pivot) (L(i, j), or X(j, c)), the 15 - j multipliers L(k, j) come
// back as uniform readlanes of lane k's own, and v[k] -= own * L(k, j) is the
// right-looking update on the factor lanes and the forward substitution on the X
// lanes in the same instruction.  No LDS round trip inside the 16 columns.
__device__ __forceinline__ void db_leaf_sc(double* lb, double* xs, double* xdiag, int jb, int* flag) {
  const int lane = threadIdx.x & 63;
  const int base = (jb * (jb + 1) / 2 + jb) * 256;
  const bool frow = lane < 16, xcol = (lane >= 16) && (lane < 32);
  const int i = lane & 15;
  const int lim = frow ? i : (xcol ? 15 : -1);    // columns j <= lim produce a nonzero own
  double v[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    double a = 0.0;
    if (frow && k <= i) a = lb[base + db_e(i, k)];
    if (xcol && k == i) a = 1.0;
    v[k] = a;
  }
  int bad = 0;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const double piv = db_bcast(v[j], j);
    if (!(piv > 0.0) && bad == 0) bad = j + 1;      // wave-uniform; later columns are NaN garbage
    const double r = db_rsq(piv);
    const double own = (j <= lim) ? v[j] * r : 0.0;
    v[j] = own;
#pragma unroll
    for (int k = j + 1; k < 16; ++k) v[k] = fma(-own, db_bcast(own, k), v[k]);
  }
  if (bad) {
    if (lane == 0) *flag = jb * 16 + bad;
    return;
  }
  if (frow) {
#pragma unroll
    for (int k = 0; k < 16; ++k)
      if (k <= i) lb[base + db_e(i, k)] = v[k];          // L lower
  } else if (xcol) {
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      if (k > i) lb[base + db_e(i, k)] = v[k];           // X(k, c) at (c, k), upper
      xs[db_e(k, i)] = v[k];                             // X(k, c), zero for k < c
    }
    xdiag[jb * 16 + i] = v[i];
  }
}


// software-pipelined readlane leaf: the next pivot's chain (its one update, broadcast, rsq)
// is issued before the rest of the current column's updates
template <int SPLIT>
__device__ __forceinline__ void leaf_sc2(double* lb, double* xs, double* xdiag, int jb, int* flag) {
  const int lane = threadIdx.x & 63;
  const int base = (jb * (jb + 1) / 2 + jb) * 256;
  const bool frow = lane < 16, xcol = (lane >= 16) && (lane < 32);
  const int i = lane & 15;
  const int lim = frow ? i : (xcol ? 15 : -1);
  double v[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    double a = 0.0;
    if (frow && k <= i) a = lb[base + db_e(i, k)];
    if (xcol && k == i) a = 1.0;
    v[k] = a;
  }
  int bad = 0;
  double piv = db_bcast(v[0], 0);
  double r = db_rsq(piv);
  if (!(piv > 0.0)) bad = 1;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const double own = (j <= lim) ? v[j] * r : 0.0;
    v[j] = own;
    if (j < 15) {
      v[j + 1] = fma(-own, db_bcast(own, j + 1), v[j + 1]);
      const double pn = db_bcast(v[j + 1], j + 1);
      const double r0 = __builtin_amdgcn_rsq(pn);
      __builtin_amdgcn_sched_barrier(0);
      constexpr int dummy = 0; (void)dummy;
      const int mid = j + 2 + (14 - j) / 2;
#pragma unroll
      for (int k = j + 2; k < 16; ++k) {
        if (SPLIT && k == mid) __builtin_amdgcn_sched_barrier(0);
        v[k] = fma(-own, db_bcast(own, k), v[k]);
      }
      __builtin_amdgcn_sched_barrier(0);
      r = r0 * fma(-0.5 * pn * r0, r0, 1.5);
      if (!(pn > 0.0) && bad == 0) bad = j + 2;
    }
  }
  if (bad) {
    if (lane == 0) *flag = jb * 16 + bad;
    return;
  }
  if (frow) {
#pragma unroll
    for (int k = 0; k < 16; ++k)
      if (k <= i) lb[base + db_e(i, k)] = v[k];
  } else if (xcol) {
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      if (k > i) lb[base + db_e(i, k)] = v[k];
      xs[db_e(k, i)] = v[k];
    }
    xdiag[jb * 16 + i] = v[i];
  }
}

// LDS broadcast of the column: the factor lanes write own to a 16-double slot, every lane
// reads L(k, j) back with uniform-address loads; the next pivot's chain stays on readlanes
__device__ __forceinline__ void leaf_lds(double* lb, double* xs, double* xdiag, int jb, int* flag, double* col) {
  const int lane = threadIdx.x & 63;
  const int base = (jb * (jb + 1) / 2 + jb) * 256;
  const bool frow = lane < 16, xcol = (lane >= 16) && (lane < 32);
  const int i = lane & 15;
  const int lim = frow ? i : (xcol ? 15 : -1);
  double v[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    double a = 0.0;
    if (frow && k <= i) a = lb[base + db_e(i, k)];
    if (xcol && k == i) a = 1.0;
    v[k] = a;
  }
  int bad = 0;
  double piv = db_bcast(v[0], 0);
  double r = db_rsq(piv);
  if (!(piv > 0.0)) bad = 1;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const double own = (j <= lim) ? v[j] * r : 0.0;
    v[j] = own;
    if (j < 15) {
      if (frow) col[j * 16 + i] = own;
      v[j + 1] = fma(-own, db_bcast(own, j + 1), v[j + 1]);
      const double pn = db_bcast(v[j + 1], j + 1);
      const double r0 = __builtin_amdgcn_rsq(pn);
      double l[16];
#pragma unroll
      for (int k = j + 2; k < 16; ++k) l[k] = col[j * 16 + k];
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int k = j + 2; k < 16; ++k) v[k] = fma(-own, l[k], v[k]);
      __builtin_amdgcn_sched_barrier(0);
      r = r0 * fma(-0.5 * pn * r0, r0, 1.5);
      if (!(pn > 0.0) && bad == 0) bad = j + 2;
    }
  }
  if (bad) {
    if (lane == 0) *flag = jb * 16 + bad;
    return;
  }
  if (frow) {
#pragma unroll
    for (int k = 0; k < 16; ++k)
      if (k <= i) lb[base + db_e(i, k)] = v[k];
  } else if (xcol) {
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      if (k > i) lb[base + db_e(i, k)] = v[k];
      xs[db_e(k, i)] = v[k];
    }
    xdiag[jb * 16 + i] = v[i];
  }
}


// probes of the MFMA leaf's chain (db_leaf_mfma): VARIANT 1 drops the X (Y) MFMA,
// VARIANT 2 drops both MFMAs (the pivot chain alone: readlane, rsq, scaling)
template <int VARIANT>
__device__ __forceinline__ void leaf_mfma_probe(double* lb, double* xs, double* xdiag, int jb, int* flag) {
  const int lane = threadIdx.x & 63;
  const int j = lane & 15, q = lane >> 4;
  const int base = (jb * (jb + 1) / 2 + jb) * 256;
  d4 acc, Y;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = q + 4 * r;
    acc[r] = (i >= j) ? lb[base + db_e(i, j)] : lb[base + db_e(j, i)];
    Y[r] = (i == j) ? 1.0 : 0.0;
  }
  int bad = 0;
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    const int k0 = c & 3, rc = c >> 2;
    const double piv = db_bcast(acc[rc], c + 16 * k0);
    if (!(piv > 0.0) && bad == 0) bad = c + 1;
    const double r = db_rsq(piv);
    const bool mine = q == k0;
    const double u = acc[rc] * r;
    const double xr = Y[rc] * r;
    const bool act = mine && j > c;
    const double ua = act ? -u : 0.0, ub = act ? u : 0.0;
    const double xb = mine ? xr : 0.0;
    acc[rc] = (mine && j >= c) ? (j == c ? piv * r : u) : acc[rc];
    Y[rc] = mine ? xr : Y[rc];
    if (VARIANT < 2) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(ua, ub, acc, 0, 0, 0);
    else acc[(rc + 1) & 3] = acc[(rc + 1) & 3] - ua * ub;   // keep a dependence on the column
    if (VARIANT < 1) Y = __builtin_amdgcn_mfma_f64_16x16x4f64(ua, xb, Y, 0, 0, 0);
  }
  if (bad) {
    if (lane == 0) *flag = jb * 16 + bad;
    return;
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int c = q + 4 * r;
    lb[base + db_e(j, c)] = (j >= c) ? acc[r] : Y[r];
    xs[db_e(c, j)] = Y[r];
    if (j == c) xdiag[jb * 16 + c] = Y[r];
  }
}

// mode 0: db_leaf (permutes), 1: db_leaf_sc (readlanes), 2: loads + stores only,
// 3/4: leaf_sc2 (pipelined next pivot; 4 also splits the update run), 5: leaf_lds,
// 6: db_leaf_mfma (column updates as rank-1 MFMAs in the accumulator layout), 7: its chain
// without the X MFMA, 8: without either MFMA (wrong results: chain latency only),
// 9: db_leaf_blk (4-column blocks: 4 x 4 factor on uniform values, four MFMAs per block)
template <int MODE>
__global__ void __launch_bounds__(64) k_leaf(const double* A, double* out, unsigned long long* t, int reps) {
  __shared__ __attribute__((aligned(16))) double lb[DB_LDS_DOUBLES + DB_EXTRA_DOUBLES];
  const int lane = threadIdx.x;
  double* xs = lb + 36 * 256;
  double* xdiag = lb + DB_LDS_DOUBLES;
  int* flag = reinterpret_cast<int*>(xdiag + 132);
  if (lane == 0) *flag = 0;
  unsigned long long acc = 0, accs = 0;
  for (int r = 0; r < reps; ++r) {
    for (int e = lane; e < 256; e += 64) lb[db_e(e & 15, e >> 4)] = A[e];     // block (0,0)
    __syncthreads();
    const unsigned long long t0 = wall_clock64();
    const unsigned long long s0 = clock64();
    if (MODE == 0) db_leaf(lb, xs, xdiag, 0, flag);
    else if (MODE == 1) db_leaf_sc(lb, xs, xdiag, 0, flag);
    else if (MODE == 3) leaf_sc2<0>(lb, xs, xdiag, 0, flag);
    else if (MODE == 4) leaf_sc2<1>(lb, xs, xdiag, 0, flag);
    else if (MODE == 5) leaf_lds(lb, xs, xdiag, 0, flag, lb + 1024);
    else if (MODE == 6) db_leaf_mfma(lb, xs, xdiag, 0, flag);
    else if (MODE == 7) leaf_mfma_probe<1>(lb, xs, xdiag, 0, flag);
    else if (MODE == 8) leaf_mfma_probe<2>(lb, xs, xdiag, 0, flag);
    else if (MODE == 9) db_leaf_blk(lb, xs, xdiag, 0, flag);
    else {
      double v = lb[lane] + lb[lane + 64];
      xs[lane] = v;
    }
    __syncthreads();
    const unsigned long long s1 = clock64();
    const unsigned long long t1 = wall_clock64();
    acc += t1 - t0;
    accs += s1 - s0;
  }
  for (int e = lane; e < 256; e += 64) out[e] = lb[db_e(e & 15, e >> 4)], out[256 + e] = xs[db_e(e & 15, e >> 4)];
  if (lane == 0) t[0] = acc, t[1] = accs;
}

int main() {
  double h[256];
  for (int c = 0; c < 16; ++c)
    for (int r = 0; r < 16; ++r) h[r + 16 * c] = std::exp(-0.01 * (r - c) * (r - c)) + (r == c ? 1.0 : 0.0);
  double *A, *out;
  unsigned long long* t;
  hipMalloc(&A, 256 * 8); hipMalloc(&out, 512 * 8); hipMalloc(&t, 16);
  hipMemcpy(A, h, 256 * 8, hipMemcpyHostToDevice);
  const int reps = 200;
  for (int m = 0; m < 10; ++m) {
    for (int it = 0; it < 2; ++it) {
      if (m == 0) hipLaunchKernelGGL(k_leaf<0>, dim3(1), dim3(64), 0, 0, A, out, t, reps);
      if (m == 1) hipLaunchKernelGGL(k_leaf<1>, dim3(1), dim3(64), 0, 0, A, out, t, reps);
      if (m == 2) hipLaunchKernelGGL(k_leaf<2>, dim3(1), dim3(64), 0, 0, A, out, t, reps);
      if (m == 3) hipLaunchKernelGGL(k_leaf<3>, dim3(1), dim3(64), 0, 0, A, out, t, reps);
      if (m == 4) hipLaunchKernelGGL(k_leaf<4>, dim3(1), dim3(64), 0, 0, A, out, t, reps);
      if (m == 5) hipLaunchKernelGGL(k_leaf<5>, dim3(1), dim3(64), 0, 0, A, out, t, reps);
      if (m == 6) hipLaunchKernelGGL(k_leaf<6>, dim3(1), dim3(64), 0, 0, A, out, t, reps);
      if (m == 7) hipLaunchKernelGGL(k_leaf<7>, dim3(1), dim3(64), 0, 0, A, out, t, reps);
      if (m == 8) hipLaunchKernelGGL(k_leaf<8>, dim3(1), dim3(64), 0, 0, A, out, t, reps);
      if (m == 9) hipLaunchKernelGGL(k_leaf<9>, dim3(1), dim3(64), 0, 0, A, out, t, reps);
      hipDeviceSynchronize();
    }
    unsigned long long th[2];
    double o[512];
    hipMemcpy(th, t, 16, hipMemcpyDeviceToHost);
    hipMemcpy(o, out, 512 * 8, hipMemcpyDeviceToHost);
    // check L L^T = A and X L = I on the lower part
    double e1 = 0, e2 = 0;
    for (int i = 0; i < 16; ++i)
      for (int j = 0; j <= i; ++j) {
        double s = 0, s2 = 0;
        for (int k = 0; k <= j; ++k) s += o[i + 16 * k] * o[j + 16 * k];
        for (int k = j; k <= i; ++k) s2 += o[256 + k + 16 * i] * o[k + 16 * j];   // xs(k, i) = X(k, i)? (column-major X)
        e1 = fmax(e1, fabs(s - h[i + 16 * j]));
        (void)s2;
      }
    // X from xs: X(r, c) = xs[r + 16 c]; check X L = I
    for (int i = 0; i < 16; ++i)
      for (int j = 0; j < 16; ++j) {
        double s = 0;
        for (int k = 0; k < 16; ++k) s += o[256 + i + 16 * k] * (k >= j ? o[k + 16 * j] : 0.0);
        e2 = fmax(e2, fabs(s - (i == j ? 1.0 : 0.0)));
      }
    printf("mode %d: %.3f us/leaf (wall), %.0f shader cycles/leaf  |LL^T-A| %.1e |XL-I| %.1e\n", m,
           th[0] * 0.01 / reps, (double)th[1] / reps, e1, e2);
  }
  return 0;
}
