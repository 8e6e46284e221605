"""CPU oracle for the case2 sensitivity / uncertainty analysis -- TEST INFRASTRUCTURE ONLY.

A NumPy restatement of the reference's sensitivity/_sensitivityclasses.py
(MathThyMod/GP_emu_UQSA, read-only at /root/reference in the build container, never
shipped).  Only ``tests/`` may import it; the product module
``gp_emu_uqsa_amd.sensitivity`` never does.

Restatement rules: every quantity is formed with the reference's own matrices and
formulas (B = inv(diag(v)), C = diag(1/delta^2), the same np.linalg.solve / det /
sqrt-of-matrix calls).  The reference's per-point and per-pair Python loops become
broadcasts over the same per-point solves.  So the n x n x d arrays of P_prod_calc
(:599-607) are formed here too, and this module is only for the small n of the tests.
Pinned against the reference's own run: tests/golden/sensitivity_*.npz
(make_golden.py G8).
"""
from __future__ import annotations

import numpy as np


def _quad_cols(V, M):
    """v^T M v for every column v of V (d x N)."""
    return np.einsum("in,ij,jn->n", V, M, V)


def setup_ref(x, f, H, A, beta, sigma, nugget, delta, m, v):
    """Sensitivity.__init__ + UPSQRT_const (:8-52, :519-552)."""
    m = np.asarray(m, dtype=float)
    v = np.asarray(v, dtype=float)
    s = {"x": x, "f": f, "H": H, "A": A, "beta": np.asarray(beta, float), "sigma": float(sigma),
         "nugget": float(nugget), "m": m, "v": v}
    B = np.linalg.inv(np.diag(v))
    C = np.diag(1.0 / (np.asarray(delta, dtype=float) ** 2))
    s["B"], s["C"] = B, C
    nu = s["nugget"]
    T1 = np.sqrt(B.dot(np.linalg.inv(B + 2.0 * C)))
    T2 = 0.5 * 2.0 * C.dot(B).dot(np.linalg.inv(B + 2.0 * C))
    T3 = (x - m) ** 2
    s["Tk_b4_prod"] = np.exp(-T3.dot(T2.T)).dot(T1.T)          # row k: T1 . exp(-T2 . T3[k])
    s["T"] = (1.0 - nu) * np.prod(s["Tk_b4_prod"], axis=1)
    s["R"] = np.append([1.0], m)
    s["Q"] = np.outer(s["R"].T, s["R"])
    s["U"] = (1.0 - nu) * np.prod(np.diag(np.sqrt(B.dot(np.linalg.inv(B + 4.0 * C)))))
    s["P1"] = B.dot(np.linalg.inv(B + 2.0 * C))
    s["P2"] = 0.5 * 2.0 * C.dot(B).dot(np.linalg.inv(B + 2.0 * C))
    s["P3"] = T3
    s["P4"] = np.sqrt(B.dot(np.linalg.inv(B + 4.0 * C)))
    s["P5"] = 0.5 * np.linalg.inv(B + 4.0 * C)
    s["e"] = np.linalg.solve(A, f - H.dot(s["beta"]))
    s["W"] = np.linalg.inv(H.T.dot(np.linalg.solve(A, H)))
    s["G"] = np.linalg.solve(A, H)
    return s


def uncertainty_ref(s):
    """Sensitivity.uncertainty (:54-203)."""
    x, m, B, C, nu = s["x"], s["m"], s["B"], s["C"], s["nugget"]
    n, d = x.shape
    A, G, W, e, beta = s["A"], s["G"], s["W"], s["e"], s["beta"]
    r = {}
    Rh = np.append([1.0], m)
    Rhh = np.zeros([1 + d, 1 + d])
    Rhh[0, 0] = 1.0
    Rhh[0, 1:] = m
    Rhh[1:, 0] = m
    Rhh[1:, 1:] = np.outer(m, m) + np.linalg.inv(np.diag(np.diag(B)))
    # R integrals: one (2C+B) solve per point (:79-88)
    mpk = np.linalg.solve(2.0 * C + B, 2.0 * C.dot(x.T) + B.dot(m)[:, None])
    Qk = 2.0 * _quad_cols(mpk - x.T, C) + _quad_cols(mpk - m[:, None], B)
    Rt = (1.0 - nu) * np.sqrt(np.linalg.det(B) / np.linalg.det(2.0 * C + B)) * np.exp(-0.5 * Qk)
    Rht = Rt[None, :] * np.vstack([np.ones(n), mpk])
    # Rtt: one (4C+B) solve per pair (:90-102)
    cx = 2.0 * C.dot(x.T)
    rhs = cx[:, :, None] + cx[:, None, :] + B.dot(m)[:, None, None]
    mpkl = np.linalg.solve(4.0 * C + B, rhs.reshape(d, -1)).reshape(d, n, n)
    a1 = mpkl - x.T[:, :, None]
    a2 = mpkl - x.T[:, None, :]
    a3 = mpkl - m[:, None, None]
    Qkl = (2.0 * np.einsum("ikl,ij,jkl->kl", a1, C, a1) + 2.0 * np.einsum("ikl,ij,jkl->kl", a2, C, a2)
           + np.einsum("ikl,ij,jkl->kl", a3, B, a3))
    Rtt = ((1.0 - nu) ** 2) * np.sqrt(np.linalg.det(B) / np.linalg.det(4.0 * C + B)) * np.exp(-0.5 * Qkl)
    # U integrals (:105-160)
    Bbold = np.block([[2.0 * C + B, -2.0 * C], [-2.0 * C, 2.0 * C + B]])
    U2 = (1.0 - nu) * np.linalg.det(B) / np.sqrt(np.linalg.det(Bbold))
    Bboldk = np.block([[2.0 * C + B, -2.0 * C], [-2.0 * C, 4.0 * C + B]])
    Ufact = ((1.0 - nu) ** 2) * np.linalg.det(B) / np.sqrt(np.linalg.det(Bboldk))
    mpkvec = np.vstack([np.repeat(B.dot(m)[:, None], n, axis=1), 2.0 * C.dot(x.T) + B.dot(m)[:, None]])
    mp = np.linalg.solve(Bboldk, mpkvec)
    mp1, mp2 = mp[:d], mp[d:]
    Qku = (2.0 * _quad_cols(mp2 - x.T, C) + 2.0 * _quad_cols(mp1 - mp2, C)
           + _quad_cols(mp1 - m[:, None], B) + _quad_cols(mp2 - m[:, None], B))
    Ut = Ufact * np.exp(-0.5 * Qku)
    Uht = Ut[None, :] * np.vstack([np.ones(n), mp1, mp2])
    Bboldkl = np.block([[4.0 * C + B, -2.0 * C], [-2.0 * C, 4.0 * C + B]])
    Ufact2 = ((1.0 - nu) ** 3) * np.linalg.det(B) / np.sqrt(np.linalg.det(Bboldkl))
    Utt = Ufact2 * np.exp(-0.5 * (Qk[:, None] + Qk[None, :]))
    # S integrals (:163-181)
    Smat = np.zeros([3 * d, 3 * d])
    Smat[:d, :d] = 4.0 * C + B
    Smat[d:2 * d, d:2 * d] = 2.0 * C + B
    Smat[2 * d:, 2 * d:] = 2.0 * C + B
    Smat[:d, d:2 * d] = -2.0 * C
    Smat[:d, 2 * d:] = -2.0 * C
    Smat[d:2 * d, :d] = -2.0 * C
    Smat[2 * d:, :d] = -2.0 * C
    Smat2 = np.block([[4.0 * C + B, -4.0 * C], [-4.0 * C, 4.0 * C + B]])
    S = ((1.0 - nu) ** 2) * ((np.sqrt(np.linalg.det(B))) ** 3) / np.sqrt(np.linalg.det(Smat))
    Stild = (1.0 - nu) * np.linalg.det(B) / np.sqrt(np.linalg.det(Smat2))
    # the measures (:185-203)
    s2 = s["sigma"] ** 2
    uE = Rh.T.dot(beta) + Rt.T.dot(e)
    uV = s2 * (U2 - Rt.T.dot(np.linalg.solve(A, Rt))
               + (Rh - G.T.dot(Rt)).T.dot(W).dot(Rh - G.T.dot(Rt)))
    I1 = s2 * (1.0 - np.trace(np.linalg.solve(A, Rtt))
               + np.trace(W.dot(Rhh - 2.0 * Rht.dot(G) + G.T.dot(Rtt).dot(G))))
    I2 = beta.T.dot(Rhh).dot(beta) + 2.0 * beta.T.dot(Rht).dot(e) + e.T.dot(Rtt).dot(e)
    uEV = (I1 - uV) + (I2 - uE ** 2)
    r.update(Rh=Rh, Rhh=Rhh, Rt=Rt, Rht=Rht, Rtt=Rtt, U2=U2, Uh=U2 * Rh, Uhh=U2 * Rhh, Ut=Ut, Uht=Uht,
             Utt=Utt, S=S, Stild=Stild, uE=uE, uV=uV, I1=I1, I2=I2, uEV=uEV)
    return r


def _w_terms_ref(s, w):
    """Qw, Estar, Uw, Sw, Pw for index set w (:554-626)."""
    x, m, B, C, nu = s["x"], s["m"], s["B"], s["C"], s["nugget"]
    n, d = x.shape
    wb = [k for k in range(d) if k not in w]
    Qw = np.zeros([1 + d, 1 + d])
    Qw[0, 0] = 1.0
    for i in wb + w:
        Qw[0, 1 + i] = m[i]
        Qw[1 + i, 0] = m[i]
    for i in wb + w:
        for j in wb + w:
            Qw[1 + i, 1 + j] = m[i] * m[j]
    Bww = np.diag(np.diag(B)[w])
    mwB = np.outer(m[w], m[w]) + np.linalg.inv(Bww)
    for a, i in enumerate(w):
        for b, j in enumerate(w):
            Qw[1 + i, 1 + j] = mwB[a, b]
    Estar = np.zeros([1 + d, n])
    Estar[0] = 1.0
    for kn in range(d):
        if kn in wb:
            Estar[1 + kn] = m[kn]
        if kn in w:
            Estar[1 + kn] = (2 * C[kn, kn] * x[:, kn] + B[kn, kn] * m[kn]) / (2 * C[kn, kn] + B[kn, kn])
    Uw_b4 = np.diag(np.sqrt(B.dot(np.linalg.inv(B + 4.0 * C))))
    Uw = (1.0 - nu) * np.prod(Uw_b4[wb])
    S1 = np.sqrt(B.dot(np.linalg.inv(B + 2.0 * C)))
    S2 = 0.5 * (2.0 * C * B).dot(np.linalg.inv(B + 2.0 * C))
    Sw_b4 = np.exp(-s["P3"].dot(S2.T)).dot(S1.T)
    Sw = (1.0 - nu) * Estar * np.prod(Sw_b4, axis=1)[None, :]
    P3 = s["P3"]
    P3kl = P3[:, None, :] + P3[None, :, :]                           # n x n x d
    P_prod = np.exp(-np.einsum("ij,klj->kli", s["P2"], P3kl))
    dx2 = (x[:, None, :] - x[None, :, :]) ** 2
    inner = np.einsum("ij,klj->kli", 4.0 * (C * C), dx2) + np.einsum("ij,klj->kli", 2.0 * (C * B), P3kl)
    P_b4 = np.einsum("ij,klj->kli", s["P4"], np.exp(-np.einsum("ij,klj->kli", s["P5"], inner)))
    P1P = np.einsum("ij,klj->kli", s["P1"], P_prod)
    Pw = ((1.0 - nu) ** 2) * np.prod(P1P[:, :, wb], axis=2) * np.prod(P_b4[:, :, w], axis=2)
    return Qw, Estar, Uw, Sw, Pw


def _evint_ref(s, w):
    """EEE - EE2 (:481-506)."""
    A, H, G, W, e, beta, T, R, U = s["A"], s["H"], s["G"], s["W"], s["e"], s["beta"], s["T"], s["R"], s["U"]
    Qw, Estar, Uw, Sw, Pw = _w_terms_ref(s, w)
    s2 = s["sigma"] ** 2
    EEE = s2 * (Uw - np.trace(np.linalg.solve(A, Pw))
                + np.trace(W.dot(Qw - Sw.dot(np.linalg.solve(A, H)) - H.T.dot(np.linalg.solve(A, Sw.T))
                                 + H.T.dot(np.linalg.solve(A, Pw)).dot(np.linalg.solve(A, H))))) \
        + e.T.dot(Pw).dot(e) + 2.0 * beta.T.dot(Sw).dot(e) + beta.T.dot(Qw).dot(beta)
    EE2 = s2 * (U - T.dot(np.linalg.solve(A, T.T))
                + (R - T.dot(np.linalg.solve(A, H))).dot(W).dot((R - T.dot(np.linalg.solve(A, H)).T))) \
        + (R.dot(beta) + T.dot(e)) ** 2
    return EEE - EE2


def sensitivity_ref(s):
    """Sensitivity.sensitivity (:466-516): senseindex[P] = E(V_P)."""
    return np.array([_evint_ref(s, [P]) for P in range(s["x"].shape[1])])


def totaleffectvariance_ref(s, uEV):
    """Sensitivity.totaleffectvariance (:405-463).  Qw/Sw/Pw/Uw are formed for w = [P]
    before the reference swaps w and wb, so EVaaa equals senseindex[P]."""
    ev = sensitivity_ref(s)
    return ev, uEV - ev


def _tw_ref(s, w, xw):
    """Tw for index set w at xw (:628-633)."""
    x, C, nu = s["x"], s["C"], s["nugget"]
    wb = [k for k in range(x.shape[1]) if k not in w]
    Cww = np.diag(np.diag(C)[w])
    val = np.prod(s["Tk_b4_prod"][:, wb], axis=1)
    dx = np.asarray(xw, float)[None, :] - x[:, w]
    return (1.0 - nu) * val * np.exp(-0.5 * np.einsum("ki,ij,kj->k", dx, 2.0 * Cww, dx))


def _rw_ref(s, w, xw):
    Rwno1 = np.array(s["m"])
    Rwno1[w] = xw
    return np.append([1.0], Rwno1)


def main_effect_ref(s, input_range, points=100, w=None):
    """Sensitivity.main_effect without the plot (:238-285): (effect, mean_effect)."""
    d = s["x"].shape[1]
    effect = np.zeros([d, points])
    mean_effect = np.zeros([d, points])
    for P in (range(d) if not w else w):
        for j, xw in enumerate(np.linspace(input_range[P][0], input_range[P][1], points)):
            Tw = _tw_ref(s, [P], [xw])
            Rw = _rw_ref(s, [P], xw)
            mean_effect[P, j] = Rw.dot(s["beta"]) + Tw.dot(s["e"])
            effect[P, j] = (Rw - s["R"]).dot(s["beta"]) + (Tw - s["T"]).dot(s["e"])
    return effect, mean_effect


def interaction_ref(s, input_range, i, j, points=25):
    """Sensitivity.interaction_effect without the plot (:327-373)."""
    effect, mean_effect = main_effect_ref(s, input_range, points, w=[i, j])
    inter = np.zeros([points, points])
    for ic, xwi in enumerate(np.linspace(input_range[i][0], input_range[i][1], points)):
        for jc, xwj in enumerate(np.linspace(input_range[j][0], input_range[j][1], points)):
            xw = np.array([xwi, xwj])
            Tw = _tw_ref(s, [i, j], xw)
            Rw = _rw_ref(s, [i, j], xw)
            inter[ic, jc] = ((Rw + s["R"]).dot(s["beta"]) + (Tw + s["T"]).dot(s["e"])
                             - mean_effect[i, ic] - mean_effect[j, jc])
    return inter, effect, mean_effect
