"""CPU oracle for noise_fit's noise-estimation step -- TEST INFRASTRUCTURE ONLY.

A NumPy restatement of gp_emu_uqsa/noise_fit/noise_fit.py (MathThyMod/GP_emu_UQSA,
read-only at /root/reference in the build container, never shipped).  Only ``tests/``
may import it; the product module ``gp_emu_uqsa_amd.noise_fit`` never does.
Pinned against the reference's own seeded noisefit() run: tests/golden/noise_fit.npz
(make_golden.py G9), which records every posterior, Cholesky factor, randn draw and
'zp-outputs' array of the noise loop.
"""
from __future__ import annotations

import numpy as np

from . import gp_oracle as orc


def posterior_ref(x, f, H, A, xs, Hs, beta, sigma, delta, nu, kind, rs_new=None):
    """Posterior(Dnew, Dold, ...) with Dnew.A = K.var(xs) + rs_new on the diagonal
    (Dnew.set_r(r); Dnew.make_A(s2): rs_new = r / s2, alt-nugget only;
    _emulatorclasses.py:572-575, :607-631)."""
    covar = orc.kernel_covar_ref(x, xs, delta, nu, kind)
    from scipy import linalg as sla
    mean = Hs.dot(beta) + covar.T.dot(sla.solve(A, f - H.dot(beta)))
    invA_H = sla.solve(A, H)
    t1 = Hs - covar.T.dot(invA_H)
    t2 = H.T.dot(invA_H)
    Ass, _ = orc.kernel_var_ref(xs, delta, nu, kind, True)
    if rs_new is not None and kind == orc.ALT:
        Ass[np.diag_indices_from(Ass)] += rs_new
    t3 = Ass - covar.T.dot(sla.solve(A, covar))
    var = sigma ** 2 * (t3 + t1.dot(sla.solve(t2, t1.T)))
    return mean, var


def noise_estimate_ref(mean, var, t, U):
    """z' = log( sum_j 0.5 (t - (mean + L u_j))^2 / s ), L = chol(var), u_j = U[j]
    (noise_fit.py:130-138, the loop kept as the reference runs it)."""
    L = np.linalg.cholesky(var)
    z = np.zeros(np.size(t))
    for u in U:
        tij = mean + L.dot(u)
        z = z + 0.5 * (t - tij) ** 2
    return np.log(z / float(len(U)))
