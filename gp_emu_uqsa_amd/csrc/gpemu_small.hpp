// gpemu_small.hpp -- host-side q x q algebra on the Gram matrix of [L^-1 f, L^-1 H]
// (shared by the single-GPU and the distributed objective).
#pragma once
#include <cmath>
#include <vector>

namespace gpe {

// dense Cholesky of a small SPD matrix (row-major), false if not PD
inline bool small_chol(std::vector<double>& a, int q) {
  for (int j = 0; j < q; ++j) {
    double s = a[j * q + j];
    for (int k = 0; k < j; ++k) s -= a[j * q + k] * a[j * q + k];
    if (!(s > 0.0)) return false;
    const double dj = std::sqrt(s);
    a[j * q + j] = dj;
    for (int i = j + 1; i < q; ++i) {
      double t = a[i * q + j];
      for (int k = 0; k < j; ++k) t -= a[i * q + k] * a[j * q + k];
      a[i * q + j] = t / dj;
    }
    for (int k = j + 1; k < q; ++k) a[j * q + k] = 0.0;
  }
  return true;
}

// solve K y = b (K lower, row-major)
inline void small_fwd(const std::vector<double>& K, int q, double* b) {
  for (int i = 0; i < q; ++i) {
    double s = b[i];
    for (int k = 0; k < i; ++k) s -= K[i * q + k] * b[k];
    b[i] = s / K[i * q + i];
  }
}
inline void small_bwd(const std::vector<double>& K, int q, double* b) {
  for (int i = q - 1; i >= 0; --i) {
    double s = b[i];
    for (int k = i + 1; k < q; ++k) s -= K[k * q + i] * b[k];
    b[i] = s / K[i * q + i];
  }
}
// inverse of lower-triangular K (row-major)
inline std::vector<double> small_trinv(const std::vector<double>& K, int q) {
  std::vector<double> X((size_t)q * q, 0.0);
  for (int c0 = 0; c0 < q; ++c0) {
    std::vector<double> e(q, 0.0);
    e[c0] = 1.0;
    small_fwd(K, q, e.data());
    for (int i = 0; i < q; ++i) X[i * q + c0] = e[i];
  }
  return X;
}

struct SmallAlgebra {
  double zz = 0, quad = 0, logdetQ = 0;
  std::vector<double> Kq, beta;  // Kq row-major lower (q x q)
  bool ok = false;
};

inline SmallAlgebra small_from_gram(const std::vector<double>& G, int P) {
  // G over [z w]: zz = G00, wz = G[1:,0], Q = G[1:,1:]
  SmallAlgebra s;
  const int q = P - 1;
  s.zz = G[0];
  std::vector<double> Q((size_t)q * q), wz(q);
  for (int i = 0; i < q; ++i) {
    wz[i] = G[(i + 1) * P + 0];
    for (int j = 0; j < q; ++j) Q[i * q + j] = G[(i + 1) * P + (j + 1)];
  }
  if (!small_chol(Q, q)) return s;
  s.Kq = Q;
  s.beta = wz;
  small_fwd(Q, q, s.beta.data());
  small_bwd(Q, q, s.beta.data());
  double wzB = 0.0;
  for (int i = 0; i < q; ++i) wzB += wz[i] * s.beta[i];
  s.quad = s.zz - wzB;
  s.logdetQ = 0.0;
  for (int i = 0; i < q; ++i) s.logdetQ += 2.0 * std::log(Q[i * q + i]);
  s.ok = true;
  return s;
}

// T2 (P x P, column-major) with R2 = [z w] T2 = [sqrt(c)(z - w beta), w Kq^-T]:
// L^-T R2 = [sqrt(c) alpha, W], the two low-rank terms of the gradient's M
inline std::vector<double> small_t2(const SmallAlgebra& sa, int q, double cfac) {
  const int P = q + 1;
  std::vector<double> Kinv = small_trinv(sa.Kq, q);   // row-major
  std::vector<double> T2((size_t)P * P, 0.0);
  const double sc = std::sqrt(cfac);
  T2[0] = sc;
  for (int i = 0; i < q; ++i) T2[(i + 1) + 0 * P] = -sc * sa.beta[i];
  for (int o = 0; o < q; ++o)
    for (int i = 0; i < q; ++i) T2[(i + 1) + (o + 1) * P] = Kinv[o * q + i];   // (Kq^-T)(i,o)
  return T2;
}

// gradient from the contraction sums red[0:d] = sum M E dx_k^2, red[d] = sum_{i>j} M E,
// red[d+1] = tr M (the d+2 outputs of k_contract); coff/cdiag as the K-build's
// red = [S_1..S_d, E, T, R] from k_contract; std_r: the std kernel with a per-point r,
// whose sigma derivative the reference takes as A - diag(r) although A carries no r
// (_emulatoroptimise.py:476-478 vs _emulatorclasses.py:572-575): -1/2 sum_i M_ii r_i
inline void small_grad(const double* red, int d, bool alt_nug, double nu, bool fitnug, bool gp4ml,
                       double gscale, double s2, double coff, double cdiag, int n_hp, double* grad,
                       bool std_r = false) {
  const double pref = alt_nug ? 1.0 : (1.0 - nu);
  const double SE = 2.0 * red[d], Tr = red[d + 1];
  for (int k = 0; k < d; ++k) grad[k] = 0.5 * gscale * pref * 2.0 * red[k];
  if (fitnug) grad[d] = alt_nug ? 0.5 * gscale * nu * nu * Tr : 0.5 * gscale * (-0.5 * nu) * SE;
  if (gp4ml) grad[n_hp - 1] = 0.5 * s2 * (coff * SE + cdiag * Tr) - (std_r ? 0.5 * red[d + 2] : 0.0);
}

}  // namespace gpe
