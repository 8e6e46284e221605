"""Uncertainty and sensitivity analysis, MUCM case2 (reference:
gp_emu_uqsa/sensitivity/sensitivityfunctions.py and _sensitivityclasses.py).

Same entry points, messages, attributes and output file as the reference:
``setup(emul, m, v)``, ``Sensitivity.uncertainty / sensitivity / main_effect /
interaction_effect / totaleffectvariance / to_file`` and ``sense_table``.

Where the work goes:
* The O(n^2) part runs on the GPU with the emulator's resident factor of
  training.A (the same one Posterior uses).
  - `gpe_sense_pairs` gives tr(A^-1 K) and [e G]^T K [e G] for the n x n
    Gaussian-integral matrices Rtt (:90-102) and, for every input P, Pw
    (:599-626). The reference builds these, and the n x n x d arrays behind
    Pw, with Python loops; here they are never formed.
  - `gpe_solve` gives e, G, A^-1 Rt and A^-1 T (:40-44, :187, :451).
  - `gpe_gauss_transform` gives the Tw . e sums of the main and interaction
    effects (:277-285, :353-373).
* The host keeps the O(n d) per-point factors. They are in closed form: B and C
  are diagonal, so every per-point (2C+B) / (4C+B) solve of the reference is
  elementwise. The host also keeps the small (d+1)-sized algebra.

Every pair matrix has the form K(k,l) = u_k u_l exp(-sum_i w_i (x_ki - x_li)^2):
  Rtt: w_i = 2 c_i^2 / (4 c_i + b_i),
       u_k = (1-nu) (prod b/(4c+b))^(1/4) exp(-sum_i c_i b_i (x_ki-m_i)^2 / (4c_i+b_i))
  Pw (w = [P]): w_P = 2 c_P^2 / (b_P + 4 c_P), w_i = 0 otherwise,
       u_k = (1-nu) sqrt(prod_{i!=P} P1_i . P4_P)
             exp(-sum_{i!=P} P2_i (x_ki-m_i)^2 - c_P b_P (x_kP-m_P)^2 / (b_P+4c_P))
with b = 1/v, c = 1/delta^2, P1 = b/(b+2c), P2 = c b/(b+2c), P4 = sqrt(b/(b+4c)).
(Minimising the quadratic of the reference's per-pair solve gives these exponents.)

The reference's totaleffectvariance (:405-463) forms Qw/Sw/Pw/Uw for w = [P]
before swapping w and wb, so its E(V) is senseindex[P] and EVTw[P] = uEV -
senseindex[P]. This is reproduced as is.
"""
from __future__ import annotations

import numpy as np

from .model import upload_training

__all__ = ["setup", "sense_table", "Sensitivity"]


def setup(emul, m, v, case="case2"):
    """Sensitivity instance for emulator `emul`, input means m and variances v
    (reference sensitivityfunctions.py:7-54)."""
    print("\n*** Initialising Sensitivity class ***")
    if not isinstance(m, list) or not isinstance(v, list):
        print("ERROR: 2nd and 3rd arguments must be lists of floats. "
              "Return None.")
        return None
    if case == "case2":
        if len(emul.par.beta) != emul.training.inputs[0].size + 1 \
                or False in [i == 'x' for i in emul.beliefs.basis_str[1:]]:
            print("The case2 sensitivity routines only work for emulators "
                  "with a gaussian kernel and linear mean. "
                  "This mean function will not work. Return None.")
            return None
        if len(m) != len(emul.par.beta) - 1 or len(v) != len(emul.par.beta) - 1:
            print("Mean and Variance lists must both contain as many items "
                  "as there are input dimensions. Return None.")
            return None
    else:
        print("Only case2 of MUCM's U & S analysis is implemented. Return None.")
        return None
    return Sensitivity(emul, np.array(m), np.array(v))


class Sensitivity:
    """Reference _sensitivityclasses.py:7-662 (case2)."""

    def __init__(self, emul, m, v):
        self.v = v
        self.m = m
        self.x = emul.training.inputs
        self.input_range = emul.all_data.input_range
        self.minmax = emul.all_data.minmax
        self.B = np.linalg.inv(np.diag(self.v))
        self.C = np.diag(1.0 / (np.array(emul.par.delta) ** 2))
        self.f = emul.training.outputs
        self.H = emul.training.H
        self.beta = emul.par.beta
        self.sigma = emul.par.sigma
        self.nugget = emul.par.nugget
        self._training = emul.training
        self._K = emul.K
        self._b = np.diag(self.B).copy()
        self._c = np.diag(self.C).copy()
        self.UPSQRT_const()
        Z = self._gpu().solve(np.column_stack([self.f - self.H.dot(self.beta), self.H]))
        self.e = Z[:, 0].copy()
        self.G = Z[:, 1:].copy()
        self.W = np.linalg.inv(self.H.T.dot(self.G))
        self._Z = Z                           # [e G] = A^-1 [f - H beta, H]
        self._AinvT = self._gpu().solve(self.T)
        self._evint_cache = None
        self.done_uncertainty = False
        self.done_sensitivity = False
        self.done_main_effect = False
        self.done_interaction = False
        self.done_totaleffectvar = False

    def _gpu(self):
        """The context with this emulator's training set and factor of training.A resident
        (as Posterior holds it); another emulator's analysis may have replaced them."""
        ctx = upload_training(self._training)
        K = self._K
        ctx.ensure_factor(K.kind, K.d, float(K.n), 1.0, self._training.r_scale())
        return ctx

    @property
    def A(self):
        """training.A as the reference holds it (formed on request only)."""
        return self._training.A

    # ------------------------------------------------------------ constants
    def UPSQRT_const(self):
        """T, R, Q, S, U and the per-point factors (:519-552), elementwise."""
        b, c, nu = self._b, self._c, self.nugget
        self.T1 = np.sqrt(self.B.dot(np.linalg.inv(self.B + 2.0 * self.C)))
        self.T2 = 0.5 * 2.0 * self.C.dot(self.B).dot(np.linalg.inv(self.B + 2.0 * self.C))
        self.T3 = (self.x - self.m) ** 2
        self.Tk_b4_prod = np.sqrt(b / (b + 2.0 * c))[None, :] * np.exp(-self.T3 * (c * b / (b + 2.0 * c))[None, :])
        self.T = (1.0 - nu) * np.prod(self.Tk_b4_prod, axis=1)
        self.R = np.append([1.0], self.m)
        self.Q = np.outer(self.R.T, self.R)
        self.S = np.outer(self.R.T, self.T)
        self.U = (1.0 - nu) * np.prod(np.diag(np.sqrt(self.B.dot(np.linalg.inv(self.B + 4.0 * self.C)))))
        self.Sw_b4_prod = self.Tk_b4_prod
        self.P1 = self.B.dot(np.linalg.inv(self.B + 2.0 * self.C))
        self.P2 = 0.5 * 2.0 * self.C.dot(self.B).dot(np.linalg.inv(self.B + 2.0 * self.C))
        self.P3 = self.T3
        self.P4 = np.sqrt(self.B.dot(np.linalg.inv(self.B + 4.0 * self.C)))
        self.P5 = 0.5 * np.linalg.inv(self.B + 4.0 * self.C)

    # ------------------------------------------------------------ uncertainty
    def uncertainty(self):
        """E*[E[f(X)]], var*[E[f(X)]], E*[var[f(X)]] (:54-203)."""
        print("\n*** Uncertainty measures ***")
        self.done_uncertainty = True
        m, b, c, nu = self.m, self._b, self._c, self.nugget
        d = m.size
        self.w = list(range(d))
        self.Rh = np.append([1.0], np.array(m[self.w]))
        self.Rhh = np.zeros([1 + d, 1 + d])
        self.Rhh[0, 0] = 1.0
        self.Rhh[0, 1:] = m
        self.Rhh[1:, 0] = m
        self.Rhh[1:, 1:] = np.outer(m, m) + np.linalg.inv(np.diag(b))
        # R integrals: the per-point (2C+B) solve is elementwise (:79-88)
        mpk = (2.0 * c * self.x + b * m) / (2.0 * c + b)
        Qk = (2.0 * ((mpk - self.x) ** 2).dot(c) + ((mpk - m) ** 2).dot(b))
        self.Rt = (1.0 - nu) * np.sqrt(np.linalg.det(self.B) / np.linalg.det(2.0 * self.C + self.B)) \
            * np.exp(-0.5 * Qk)
        self.Rht = self.Rt[None, :] * np.vstack([np.ones(self.x.shape[0]), mpk.T])
        # U integrals (:105-160)
        Bbold = np.block([[2.0 * self.C + self.B, -2.0 * self.C], [-2.0 * self.C, 2.0 * self.C + self.B]])
        self.U2 = (1.0 - nu) * np.linalg.det(self.B) / np.sqrt(np.linalg.det(Bbold))
        self.Uh = self.U2 * self.Rh
        self.Uhh = self.U2 * self.Rhh
        Bboldk = np.block([[2.0 * self.C + self.B, -2.0 * self.C], [-2.0 * self.C, 4.0 * self.C + self.B]])
        Ufact = ((1.0 - nu) ** 2) * np.linalg.det(self.B) / np.sqrt(np.linalg.det(Bboldk))
        n = self.x.shape[0]
        rhs = np.vstack([np.repeat(self.B.dot(m)[:, None], n, axis=1),
                         2.0 * self.C.dot(self.x.T) + self.B.dot(m)[:, None]])
        mp = np.linalg.solve(Bboldk, rhs)
        mp1, mp2 = mp[:d], mp[d:]
        Qku = (2.0 * ((mp2 - self.x.T) ** 2).T.dot(c) + 2.0 * ((mp1 - mp2) ** 2).T.dot(c)
               + ((mp1 - m[:, None]) ** 2).T.dot(b) + ((mp2 - m[:, None]) ** 2).T.dot(b))
        self.Ut = Ufact * np.exp(-0.5 * Qku)
        self.Uht = self.Ut[None, :] * np.vstack([np.ones(n), mp1, mp2])
        Bboldkl = np.block([[4.0 * self.C + self.B, -2.0 * self.C], [-2.0 * self.C, 4.0 * self.C + self.B]])
        self._Ufact2 = ((1.0 - nu) ** 3) * np.linalg.det(self.B) / np.sqrt(np.linalg.det(Bboldkl))
        self._hk = np.exp(-0.5 * Qk)
        self.Utild = 1
        # S integrals (:163-181)
        Smat = np.zeros([3 * d, 3 * d])
        Smat[:d, :d] = 4.0 * self.C + self.B
        Smat[d:2 * d, d:2 * d] = 2.0 * self.C + self.B
        Smat[2 * d:, 2 * d:] = 2.0 * self.C + self.B
        Smat[:d, d:2 * d] = -2.0 * self.C
        Smat[:d, 2 * d:] = -2.0 * self.C
        Smat[d:2 * d, :d] = -2.0 * self.C
        Smat[2 * d:, :d] = -2.0 * self.C
        Smat2 = np.block([[4.0 * self.C + self.B, -4.0 * self.C], [-4.0 * self.C, 4.0 * self.C + self.B]])
        self.S = ((1.0 - nu) ** 2) * ((np.sqrt(np.linalg.det(self.B))) ** 3) / np.sqrt(np.linalg.det(Smat))
        self.Stild = (1.0 - nu) * np.linalg.det(self.B) / np.sqrt(np.linalg.det(Smat2))
        # Rtt on the GPU: tr(A^-1 Rtt) and [e G]^T Rtt [e G]
        w0 = 2.0 * c * c / (4.0 * c + b)
        u0 = (1.0 - nu) * np.prod(b / (4.0 * c + b)) ** 0.25 \
            * np.exp(-((self.x - m) ** 2).dot(c * b / (4.0 * c + b)))
        tr, quad = self._gpu().sense_pairs(w0[None, :], u0[None, :], self._Z)
        trRtt, eRe, GRG = tr[0], quad[0, 0, 0], quad[0, 1:, 1:]
        AinvRt = self._gpu().solve(self.Rt)
        s2 = self.sigma ** 2
        G, W, e, beta = self.G, self.W, self.e, self.beta
        self.uE = self.Rh.T.dot(beta) + self.Rt.T.dot(e)
        self.uV = s2 * (self.U2 - self.Rt.T.dot(AinvRt)
                        + (self.Rh - G.T.dot(self.Rt)).T.dot(W).dot(self.Rh - G.T.dot(self.Rt)))
        self.I1 = s2 * (self.Utild - trRtt + np.trace(W.dot(self.Rhh - 2.0 * self.Rht.dot(G) + GRG)))
        self.I2 = beta.T.dot(self.Rhh).dot(beta) + 2.0 * beta.T.dot(self.Rht).dot(e) + eRe
        self.uEV = (self.I1 - self.uV) + (self.I2 - self.uE ** 2)
        print("E*[ E[f(X)] ]  :", self.uE)
        print("var*[ E[f(X)] ]:", self.uV)
        print("E*[ var[f(X)] ]:", self.uEV)

    @property
    def Utt(self):
        """Ufact2 exp(-(Qk + Ql)/2) (:146-159): rank one, formed on request."""
        return self._Ufact2 * np.outer(self._hk, self._hk)

    # ------------------------------------------------------------ w / wb terms
    def setup_w_wb(self, P):
        self.w = [P]
        self.wb = [k for k in range(len(self.m)) if k not in self.w]

    def _qw(self, w):
        """Qw (:554-582): R R^T with v_w added on the w diagonal."""
        Qw = np.outer(self.R, self.R)
        for i in w:
            Qw[1 + i, 1 + i] += self.v[i]
        return Qw

    def _estar(self, w):
        """Estar (:584-596)."""
        b, c = self._b, self._c
        E = np.repeat(self.R[:, None], self.x.shape[0], axis=1)
        for kn in w:
            E[1 + kn] = (2 * c[kn] * self.x[:, kn] + b[kn] * self.m[kn]) / (2 * c[kn] + b[kn])
        return E

    def _uw(self, wb):
        return (1.0 - self.nugget) * np.prod(np.diag(np.sqrt(self.B.dot(np.linalg.inv(self.B + 4.0 * self.C))))[wb])

    def _pw_factors(self):
        """(w, u) of Pw for w = [P], every P (see the module docstring)."""
        b, c, nu, m = self._b, self._c, self.nugget, self.m
        d = m.size
        P1, P2, P4 = b / (b + 2.0 * c), c * b / (b + 2.0 * c), np.sqrt(b / (b + 4.0 * c))
        dm2 = (self.x - m) ** 2
        W = np.zeros((d, d))
        Uf = np.zeros((d, self.x.shape[0]))
        for P in range(d):
            wb = [i for i in range(d) if i != P]
            W[P, P] = 2.0 * c[P] ** 2 / (b[P] + 4.0 * c[P])
            const = (1.0 - nu) * np.sqrt(np.prod(P1[wb]) * P4[P])
            Uf[P] = const * np.exp(-dm2[:, wb].dot(P2[wb]) - dm2[:, P] * c[P] * b[P] / (b[P] + 4.0 * c[P]))
        return W, Uf

    def _evint_all(self):
        """EEE - EE2 for w = [P], every P (:481-506); one pair-kernel call for all P."""
        if self._evint_cache is not None:
            return self._evint_cache
        d = self.m.size
        W, Uf = self._pw_factors()
        trPw, quad = self._gpu().sense_pairs(W, Uf, self._Z)
        s2 = self.sigma ** 2
        G, Wm, e, beta, T, R = self.G, self.W, self.e, self.beta, self.T, self.R
        TG = T.dot(G)
        EE2 = s2 * (self.U - T.dot(self._AinvT) + (R - TG).dot(Wm).dot(R - TG)) + (R.dot(beta) + T.dot(e)) ** 2
        out = np.zeros(d)
        for P in range(d):
            w = [P]
            wb = [k for k in range(d) if k not in w]
            Qw = self._qw(w)
            Sw = self._estar(w) * T[None, :]      # (1-nu) Estar prod(Sw_b4_prod) (:615-619)
            SwG = Sw.dot(G)
            EEE = s2 * (self._uw(wb) - trPw[P]
                        + np.trace(Wm.dot(Qw - SwG - SwG.T + quad[P, 1:, 1:]))) \
                + quad[P, 0, 0] + 2.0 * beta.T.dot(Sw).dot(e) + beta.T.dot(Qw).dot(beta)
            out[P] = EEE - EE2
        self._evint_cache = out
        return out

    # ------------------------------------------------------------ public measures
    def sensitivity(self):
        """Sensitivity indices E(V_w) for each input (:466-516)."""
        print("\n*** Calculate sensitivity indices ***")
        self.done_sensitivity = True
        ev = self._evint_all()
        self.senseindex = np.zeros([self.m.size])
        for P in range(self.m.size):
            self.setup_w_wb(P)
            self.EVint = ev[P]
            if self.done_uncertainty:
                print("E(V" + str(self.w) + ")/EV:", self.EVint / self.uEV)
            else:
                print("E(V" + str(self.w) + "):", self.EVint)
            self.senseindex[P] = self.EVint
        if self.done_uncertainty:
            print("Sum of Sensitivities:", np.sum(self.senseindex / self.uEV))

    def totaleffectvariance(self):
        """Total effect variances as the reference computes them (:405-463)."""
        self.done_totaleffectvar = True
        print("\n*** Calculate total effect variance ***")
        self.senseindexwb = np.zeros([self.m.size])
        self.EVTw = np.zeros([self.m.size])
        self.EVf = self.uEV
        print("E*[ var[f(X)] ]:", self.EVf)
        ev = self._evint_all()
        for P in range(self.m.size):
            self.EVaaa = ev[P]
            self.senseindexwb[P] = self.EVaaa
            self.EVTw[P] = self.EVf - self.EVaaa
            print("E(V[T" + str(P) + "]):", self.EVTw[P])

    def _line_sums(self, w, Y):
        """Tw . e for index set w at the rows of Y (len(w) columns)."""
        wb = [k for k in range(self.m.size) if k not in w]
        a = (1.0 - self.nugget) * np.prod(self.Tk_b4_prod[:, wb], axis=1) * self.e
        return self._gpu().gauss_transform(w, self._c[w], Y, a)

    def main_effect(self, plot=False, points=100, customKey=[], customLabels=[], plotShrink=0.9, w=[],
                    black_white=False):
        """Main effects of each input over its range (:238-324)."""
        print("\n*** Main effect measures ***")
        self.done_main_effect = True
        self.effect = np.zeros([self.m.size, points])
        self.mean_effect = np.zeros([self.m.size, points])
        if w == []:
            w = range(0, len(self.m))
        if plot:
            import matplotlib.pyplot as plt
            from cycler import cycler
            fig = plt.figure()
            ax = plt.subplot(111)
            if black_white:
                ax.set_prop_cycle(cycler('linestyle', ['-', '--', '-.', ':']))
                colors = plt.get_cmap('plasma')(np.linspace(0, 1.0, len(w)))
            else:
                colors = plt.get_cmap('jet')(np.linspace(0, 1.0, len(w)))
        base = self.R.dot(self.beta) + self.T.dot(self.e)
        cn = 0
        for P in w:
            print("Main effect measures for input", P, "range", self.input_range[P])
            self.setup_w_wb(P)
            xs = np.linspace(self.input_range[P][0], self.input_range[P][1], points)
            Twe = self._line_sums([P], xs[:, None])
            Rwb = self.R.dot(self.beta) + self.beta[1 + P] * (xs - self.m[P])
            self.mean_effect[P] = Rwb + Twe
            self.effect[P] = self.mean_effect[P] - base
            if plot:
                label = 'x' + str(P)
                if customKey != []:
                    try:
                        label = str(customKey[P])
                    except IndexError:
                        pass
                ax.plot(np.linspace(0.0, 1.0, points), self.effect[P], linewidth=2.0, label=label,
                        color=colors[cn])
            cn = cn + 1
        if plot:
            box = ax.get_position()
            ax.set_position([box.x0, box.y0, box.width * plotShrink, box.height])
            ax.legend(loc='center left', bbox_to_anchor=(1, 0.5))
            xl, yl = "xw", "Main Effect"
            if customLabels != []:
                xl = customLabels[0] if len(customLabels) > 0 else xl
                yl = customLabels[1] if len(customLabels) > 1 else yl
            plt.xlabel(xl)
            plt.ylabel(yl)
            print("Plotting main effects...")
            plt.show()

    def interaction_effect(self, i, j, points=25, customLabels=[]):
        """Interaction effect of inputs i and j on a points x points grid (:327-401)."""
        print("\n*** Interaction effects ***")
        self.done_interaction = True
        self.interaction = np.zeros([points, points])
        print("Recalculating main effect with", points, "points...")
        self.main_effect(plot=False, points=points, w=[i, j])
        self.w = [i, j]
        self.wb = [k for k in range(len(self.m)) if k not in self.w]
        ra_i = self.input_range[i]
        ra_j = self.input_range[j]
        print("\nCalculating", points * points, "interaction effects...")
        xi = np.linspace(ra_i[0], ra_i[1], points)
        xj = np.linspace(ra_j[0], ra_j[1], points)
        Y = np.column_stack([np.repeat(xi, points), np.tile(xj, points)])
        Twe = self._line_sums([i, j], Y).reshape(points, points)
        Rwb = (self.R.dot(self.beta) + self.beta[1 + i] * (xi - self.m[i])[:, None]
               + self.beta[1 + j] * (xj - self.m[j])[None, :])
        self.interaction = (Rwb + self.R.dot(self.beta)) + (Twe + self.T.dot(self.e)) \
            - self.mean_effect[i][:, None] - self.mean_effect[j][None, :]
        import matplotlib.pyplot as plt
        plt.figure()
        ax = plt.gca()
        im = ax.imshow(self.interaction, origin='lower', cmap=plt.get_cmap('hot'),
                       extent=(ra_i[0], ra_i[1], ra_j[0], ra_j[1]))
        plt.colorbar(im)
        xl, yl = "input " + str(self.w[0]), "input " + str(self.w[1])
        if customLabels != []:
            xl = customLabels[0] if len(customLabels) > 0 else xl
            yl = customLabels[1] if len(customLabels) > 1 else yl
        plt.xlabel(xl)
        plt.ylabel(yl)
        extent = ax.get_images()[0].get_extent()
        ax.set_aspect(abs((extent[1] - extent[0]) / (extent[3] - extent[2])) / 1.0)
        plt.show()

    def to_file(self, filename):
        """Results file in the reference's format (:641-662)."""
        print("Sensitivity & Uncertainty results to file...")
        with open(filename, 'w') as f:
            if self.done_uncertainty:
                f.write("EE " + str(self.uE) + "\n")
                f.write("VE " + str(self.uV) + "\n")
                f.write("EV " + str(self.uEV) + "\n")
            if self.done_sensitivity:
                f.write("EVw " + ' '.join(map(str, self.senseindex)) + "\n")
            if self.done_totaleffectvar:
                f.write("EVTw " + ' '.join(map(str, self.EVTw)) + "\n")
            if self.done_main_effect:
                f.write("xw " + ' '.join(map(str, [i for i in np.linspace(0.0, 1.0, self.effect[0].size)])) + "\n")
                for i in range(0, len(self.m)):
                    f.write("ME" + str(i) + " " + ' '.join(map(str, self.effect[i])) + "\n")


def sense_table(sense_list, inputNames=[], outputNames=[], rowHeight=6):
    """Table plot of sensitivity indices, one row per Sensitivity instance
    (reference sensitivityfunctions.py:57-148)."""
    import matplotlib.pyplot as plt
    print("\n*** Creating sensitivity table ***")
    if not isinstance(sense_list, list):
        print("ERROR: first argument must be list e.g. [s] or [s,] or [s1, s2]. "
              "Return None.")
        return None
    rows = len(sense_list)
    cols = len(sense_list[0].m) + 1
    for s in sense_list:
        if len(s.m) != cols - 1:
            print("Each emulator must be built with the same number of inputs.")
            return None
    for s in sense_list:
        if not s.done_uncertainty:
            s.uncertainty()
        if not s.done_sensitivity:
            s.sensitivity()
    if inputNames == []:
        inputNames = ["input " + str(i) for i in range(cols - 1)]
    inputNames.append("Sum")
    if outputNames == []:
        outputNames = ["output " + str(i) for i in range(rows)]
    cells = np.zeros([rows, cols])
    for si, s in enumerate(sense_list):
        cells[si, 0:cols - 1] = s.senseindex / s.uEV
        cells[si, cols - 1] = np.sum(s.senseindex / s.uEV)
    tab_2 = [['%.3f' % j for j in i] for i in cells]
    fig = plt.figure(figsize=(16, 8))
    fig.add_subplot(111, frameon=False, xticks=[], yticks=[])
    img = plt.imshow(cells, cmap="hot", vmin=0.0, vmax=1.0)
    img.set_visible(False)
    tb = plt.table(cellText=tab_2, colLabels=inputNames, rowLabels=outputNames, loc='center',
                   cellColours=img.to_rgba(cells))
    tb.scale(1, rowHeight)
    for i in range(1, rows + 1):
        for j in range(0, cols):
            tb._cells[(i, j)]._text.set_color('green')
    plt.show()
    return None
