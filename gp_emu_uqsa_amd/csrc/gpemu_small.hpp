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

}  // namespace gpe
