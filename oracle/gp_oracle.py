"""CPU oracle for the GP-emulator hot path -- TEST INFRASTRUCTURE ONLY.

This module is a NumPy/SciPy restatement of the reference algorithm
(MathThyMod/GP_emu_UQSA, mounted read-only at /root/reference in the build
container, never shipped).  It exists to CHECK the HIP path, never to run it:
only ``tests/``, ``__graft_entry__.smoke()``, the ``cpu_baseline`` leg of
``bench.py`` and the dev timing tools that time the reference's CPU path beside the
GPU (``tools/cpu_ref_c3.py``, ``tools/example_train_time.py``) may import it.  The product package ``gp_emu_uqsa_amd`` never
imports this module and fails loudly when its HIP library is missing.

Two restatements live here:

* ``*_ref`` functions restate the reference op-for-op (pdist/squareform,
  ``np.linalg.cholesky`` then ``np.linalg.solve`` -- a general LU -- for every
  triangular solve, one dense dA per hyperparameter).  They are pinned against
  golden vectors produced by the reference itself (``tests/golden``) and are
  the timed CPU baseline (``cpu_baseline.kind == "port"``).
* ``*_fast`` functions compute the same quantities the way the GPU path does:
  Cholesky, explicit inverse, and the gradient as a Frobenius contraction
  0.5 * <M, dA/dtheta> with M = A^-1 - A^-1 H Q^-1 H^T A^-1 - c * alpha alpha^T.

Conventions follow the reference: hyperparameters are untransformed
(delta[d], [nu], [sigma]); the objective returns the NEGATIVE log marginal
likelihood and its gradient w.r.t. the transformed parameters x = 2 log(hp)
(reference ``_emulatorkernels.py:31-36``).
"""
from __future__ import annotations

import numpy as np
from scipy import linalg as _sla
from scipy.spatial import distance as _dist

STD = 0   # (1-nu) exp(-r^2) + nu on the diagonal      (_emulatorkernels.py:10-79)
ALT = 1   # exp(-r^2) + nu^2 on the diagonal            (_emulatorkernels.py:83-152)
GP4ML = 0  # sigma is a hyperparameter                  (_emulatoroptimise.py:412-493)
MUCM = 1   # sigma analytic, gradient scaled by sig2    (_emulatoroptimise.py:305-378)


# --------------------------------------------------------------------------
# kernel (a1, a2, a4, a5, a11 of SURVEY section 8a)
# --------------------------------------------------------------------------
def kernel_var_ref(X, delta, nu, kind, predict=True):
    """K.var(X, predict) -> (A, exp_save).  _emulatorkernels.py:39-50 / :112-123."""
    X = np.asarray(X, dtype=np.float64)
    inv_len = 1.0 / np.asarray(delta, dtype=np.float64)
    cond = _dist.pdist(X * inv_len, "sqeuclidean")
    e = np.exp(-cond)
    if kind == ALT:
        A = _dist.squareform(e)
        np.fill_diagonal(A, 1.0 + nu ** 2 if predict else 1.0)
    else:
        A = _dist.squareform((1.0 - nu) * e)
        np.fill_diagonal(A, 1.0 if predict else 1.0 - nu)
    return A, e


def kernel_covar_ref(XT, XV, delta, nu, kind):
    """K.covar(XT, XV) -> n x m.  _emulatorkernels.py:75-79 / :148-152."""
    inv_len = 1.0 / np.asarray(delta, dtype=np.float64)
    c = np.exp(-_dist.cdist(np.asarray(XT) * inv_len, np.asarray(XV) * inv_len,
                            "sqeuclidean"))
    return c if kind == ALT else (1.0 - nu) * c


def grad_delta_ref(xcol, delta_i, nu, exp_save, s2, kind):
    """dA/d(2 log delta_i), dense n x n.  _emulatorkernels.py:53-63 / :126-136."""
    n = xcol.size
    w = 1.0 / delta_i
    p = _dist.pdist((xcol * w).reshape(n, 1), "sqeuclidean")
    pref = s2 if kind == ALT else (1.0 - nu) * s2
    return _dist.squareform(pref * p * exp_save)


def grad_nugget_ref(n, nu, exp_save, s2, kind):
    """dA/d(2 log nu), dense n x n.  _emulatorkernels.py:66-71 / :139-144."""
    if kind == ALT:
        g = np.zeros((n, n))
        np.fill_diagonal(g, nu ** 2 * s2)
        return g
    return _dist.squareform((-0.5 * nu * s2) * exp_save)


def make_A_ref(X, delta, nu, kind, r=None, s2=1.0, predict=True):
    """Data.make_A(s2, predict).  _emulatorclasses.py:572-575.

    r is only added for the alt-nugget kernel (the reference adds it only
    when ``alt_nugget == 'T'``)."""
    A, e = kernel_var_ref(X, delta, nu, kind, predict)
    if kind == ALT and r is not None:
        A[np.diag_indices_from(A)] += np.asarray(r, dtype=np.float64) / s2
    return A, e


def split_hp(hp, d, variant, fit_nugget):
    """Untransformed hp vector -> (delta, nu_or_None, sigma_or_None).

    Layout follows _emulatoroptimise.py:193-203 and the set_params rule
    (_emulatorkernels.py:20-24): delta first, then nugget (if fitted), then
    sigma (gp4ml only)."""
    hp = np.asarray(hp, dtype=np.float64)
    delta = hp[:d]
    nu = hp[d] if fit_nugget else None
    sigma = hp[-1] if variant == GP4ML else None
    return delta, nu, sigma


def _common_solves_ref(A, H, f):
    """The chain at _emulatoroptimise.py:425-438 (LU solves, as the reference)."""
    L = np.linalg.cholesky(A)
    w = np.linalg.solve(L, H)
    Q = w.T.dot(w)
    Kq = np.linalg.cholesky(Q)
    invA_f = np.linalg.solve(L.T, np.linalg.solve(L, f))
    invA_H = np.linalg.solve(L.T, np.linalg.solve(L, H))
    sKH = np.linalg.solve(Kq, H.T)
    B = np.linalg.solve(Kq.T, sKH.dot(invA_f))
    return L, Q, Kq, invA_f, invA_H, sKH, B


def _grad_term_ref(L, dA, f, invA_f, invA_H_B, H_B, Kq, sKH, invA_H, factor):
    """One gradient component, _emulatoroptimise.py:452-460 / :347-357."""
    P = np.linalg.solve(L.T, np.linalg.solve(L, dA))
    sam = P.dot(invA_H_B)
    return -0.5 * (-np.trace(P)
                   + factor * (f.T.dot(P).dot(invA_f) + (-2.0 * f.T + H_B).dot(sam))
                   + np.trace(np.linalg.solve(Kq.T, sKH.dot(P)).dot(invA_H)))


def objective_ref(X, f, H, hp, variant, kind, fit_nugget, r=None, want_grad=True,
                  nu_fixed=0.0):
    """Op-for-op restatement of loglikelihood_gp4ml / loglikelihood_mucm.

    gp4ml: _emulatoroptimise.py:412-493; mucm: :305-378.
    hp is UNtransformed.  Returns (LLH, grad, sig2) or None when the
    Cholesky fails (the reference prints and returns None, :374-376/:489-491).
    sig2 is sigma^2 for gp4ml and the analytic sigma-hat^2 for mucm."""
    X = np.asarray(X, np.float64)
    f = np.asarray(f, np.float64)
    H = np.asarray(H, np.float64)
    n, d = X.shape
    q = H.shape[1]
    delta, nu, sigma = split_hp(hp, d, variant, fit_nugget)
    nu_eff = nu if nu is not None else float(nu_fixed)
    if variant == GP4ML:
        s2 = sigma ** 2
        A, e = make_A_ref(X, delta, nu_eff, kind, r, s2)
        A = s2 * A
    else:
        s2 = 1.0
        A, e = make_A_ref(X, delta, nu_eff, kind, None, 1.0)
    try:
        L, Q, Kq, invA_f, invA_H, sKH, B = _common_solves_ref(A, H, f)
    except np.linalg.LinAlgError:
        return None
    logdetA = 2.0 * np.sum(np.log(np.diag(L)))
    invA_H_B = invA_H.dot(B)
    quad = f.T.dot(invA_f - invA_H_B)
    if variant == GP4ML:
        llh = -0.5 * (-quad - logdetA - np.log(_sla.det(Q)) - (n - q) * np.log(2.0 * np.pi))
        sig2 = s2
        factor = 1.0
        gs2 = s2
    else:
        sig2 = quad / (n - q - 2.0)
        llh = -0.5 * (-(n - q) * np.log(sig2) - logdetA - np.log(np.linalg.det(Q)))
        factor = (n - q) / (sig2 * (n - q - 2))
        gs2 = sig2
    if not want_grad:
        return llh, None, sig2
    H_B = H.dot(B).T
    n_hp = np.asarray(hp).size
    grad = np.empty(n_hp)
    for i in range(d):
        dA = grad_delta_ref(X[:, i], delta[i], nu_eff, e, gs2, kind)
        grad[i] = _grad_term_ref(L, dA, f, invA_f, invA_H_B, H_B, Kq, sKH, invA_H, factor)
    if fit_nugget:
        dA = grad_nugget_ref(n, nu_eff, e, gs2, kind)
        grad[d] = _grad_term_ref(L, dA, f, invA_f, invA_H_B, H_B, Kq, sKH, invA_H, factor)
    if variant == GP4ML:
        # :476-478 subtracts data.r for every kernel, though make_A adds r only for
        # the alt-nugget kernel (:572-575): for the std kernel with r set, dA = A - diag(r)
        dA = A.copy()
        if r is not None:
            dA[np.diag_indices_from(dA)] -= r
        grad[-1] = _grad_term_ref(L, dA, f, invA_f, invA_H_B, H_B, Kq, sKH, invA_H, factor)
    return llh, grad, sig2


# --------------------------------------------------------------------------
# fast restatement (what the GPU computes; not the reference's op order)
# --------------------------------------------------------------------------
def objective_fast(X, f, H, hp, variant, kind, fit_nugget, r=None, want_grad=True,
                   nu_fixed=0.0):
    """Cholesky + explicit inverse + Frobenius-contraction gradient.

    Same mathematics as objective_ref; see DESIGN.md section 'Objective'."""
    X = np.asarray(X, np.float64)
    f = np.asarray(f, np.float64)
    H = np.asarray(H, np.float64)
    n, d = X.shape
    q = H.shape[1]
    delta, nu, sigma = split_hp(hp, d, variant, fit_nugget)
    nu_eff = nu if nu is not None else float(nu_fixed)
    s2 = sigma ** 2 if variant == GP4ML else 1.0
    C, e = kernel_var_ref(X, delta, nu_eff, kind, True)
    A = s2 * C
    if variant == GP4ML and kind == ALT and r is not None:
        A[np.diag_indices_from(A)] += r
    try:
        L = np.linalg.cholesky(A)
    except np.linalg.LinAlgError:
        return None
    Linv = _sla.solve_triangular(L, np.eye(n), lower=True)
    z = Linv @ f
    w = Linv @ H
    Q = w.T @ w
    Kq = np.linalg.cholesky(Q)
    B = _sla.cho_solve((Kq, True), w.T @ z)
    u = z - w @ B
    quad = float(u @ u)
    logdetA = 2.0 * np.sum(np.log(np.diag(L)))
    logdetQ = 2.0 * np.sum(np.log(np.diag(Kq)))
    if variant == GP4ML:
        llh = 0.5 * (quad + logdetA + logdetQ + (n - q) * np.log(2.0 * np.pi))
        sig2 = s2
        c = 1.0
        gscale = 1.0
    else:
        sig2 = quad / (n - q - 2.0)
        llh = 0.5 * ((n - q) * np.log(sig2) + logdetA + logdetQ)
        c = (n - q) / (sig2 * (n - q - 2.0))
        gscale = sig2          # reference quirk: MUCM gradient is sig2 x true
    if not want_grad:
        return llh, None, sig2
    Ainv = Linv.T @ Linv
    alpha = Linv.T @ u
    G = Linv.T @ w
    W = _sla.solve_triangular(Kq, G.T, lower=True).T       # G K^-T
    M = Ainv - W @ W.T - c * np.outer(alpha, alpha)
    offd = np.ones((n, n)) - np.eye(n)
    Eful = _dist.squareform(e)
    grad = np.empty(np.asarray(hp).size)
    pre = s2 if kind == ALT else (1.0 - nu_eff) * s2
    for i in range(d):
        Di = (X[:, i, None] - X[None, :, i]) ** 2 / delta[i] ** 2
        grad[i] = 0.5 * gscale * np.sum(M * pre * Di * Eful)
    if fit_nugget:
        if kind == ALT:
            grad[d] = 0.5 * gscale * s2 * nu_eff ** 2 * np.trace(M)
        else:
            grad[d] = 0.5 * gscale * np.sum(M * (-0.5 * nu_eff * s2) * Eful * offd)
    if variant == GP4ML:
        grad[-1] = 0.5 * np.sum(M * (s2 * C))
        if kind == STD and r is not None:      # the reference's A - diag(r) (objective_ref)
            grad[-1] -= 0.5 * float(np.diag(M) @ np.asarray(r, dtype=np.float64))
    return llh, grad, sig2


# --------------------------------------------------------------------------
# posterior (a11-a14)
# --------------------------------------------------------------------------
def posterior_ref(XT, fT, HT, A, Xs, Hs, beta, sigma, delta, nu, kind):
    """Posterior mean / full variance. _emulatorclasses.py:607-631.

    A is the training Data.A the reference holds at that point."""
    covar = kernel_covar_ref(XT, Xs, delta, nu, kind)
    mean = Hs.dot(beta) + covar.T.dot(_sla.solve(A, fT - HT.dot(beta)))
    invA_H = _sla.solve(A, HT)
    t1 = Hs - covar.T.dot(invA_H)
    t2 = HT.T.dot(invA_H)
    Ass, _ = kernel_var_ref(Xs, delta, nu, kind, True)
    t3 = Ass - covar.T.dot(_sla.solve(A, covar))
    var = sigma ** 2 * (t3 + t1.dot(_sla.solve(t2, t1.T)))
    return mean, var


def optimal_beta_ref(A, H, f):
    """GLS beta, _emulatoroptimise.py:497-504."""
    L = np.linalg.cholesky(A)
    w = np.linalg.solve(L, H)
    Kq = np.linalg.cholesky(w.T.dot(w))
    invA_f = np.linalg.solve(L.T, np.linalg.solve(L, f))
    return np.linalg.solve(Kq.T, np.linalg.solve(Kq, H.T).dot(invA_f))


# --------------------------------------------------------------------------
# synthetic measurement data
# --------------------------------------------------------------------------
def olhc_design(n, d, seed):
    """Latin hypercube x_ij = (pi_j(i) + U(0,1)) / n, one design, RandomState(seed).

    Restates design_inputs.py:54-64 (one design; the 'maximin' selection is
    skipped as SURVEY 8d prescribes); then min-max scaling per column as
    _emulatorclasses.py:457-471."""
    rs = np.random.RandomState(seed)
    x = np.empty((n, d))
    for i in range(d):
        u = rs.uniform(0.0, 1.0, n)
        b = np.arange(n)
        rs.shuffle(b)
        x[:, i] = (b + u) / float(n)
    lo = x.min(axis=0)
    hi = x.max(axis=0)
    return (x - lo) / (hi - lo)


def toysim_outputs(X, seed):
    """toysim3D-style output (examples/sensitivity_multi_outputs/toysim3D.py:16)
    plus 0.1 sin(2 pi x_k) for k>=3 and 0.01 N(0,1) noise."""
    rs = np.random.RandomState(seed + 1000)
    x = X.T
    y = 3.0 * x[0] ** 3
    if X.shape[1] > 1:
        y = y + np.exp(np.cos(10.0 * x[1]) * np.cos(5.0 * x[0]) ** 2)
    if X.shape[1] > 2:
        y = y + np.exp(np.sin(7.5 * x[2]))
    for k in range(3, X.shape[1]):
        y = y + 0.1 * np.sin(2.0 * np.pi * x[k])
    return y + 0.01 * rs.standard_normal(X.shape[0])


def linear_basis(X):
    """H = [1, x_0, ..., x_{d-1}]  (basis_str '1.0 x x ...')."""
    return np.hstack([np.ones((X.shape[0], 1)), X])


def synthetic_problem(n, d, seed=0):
    X = olhc_design(n, d, seed)
    f = toysim_outputs(X, seed)
    return X, f, linear_basis(X)
