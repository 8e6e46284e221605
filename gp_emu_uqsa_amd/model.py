"""Emulator data structures with the reference's interface
(_emulatorclasses.py: Emulator :14, Hyperparams :254, Basis :263, TV_config :321,
All_Data :379, Data :539, Posterior :588).

Host-only bookkeeping (file reading, scaling, shuffling, the T/V split) keeps the
reference's semantics and its np.random consumption order; every covariance,
factorisation and solve goes through the HIP library (gp_emu_uqsa_amd.native).
``Data.A`` is materialised on the GPU only when a caller reads it.
"""
from __future__ import annotations

import numpy as np

from . import native


class Emulator:
    """Keeps instances of the other classes together (reference :14-29)."""

    def __init__(self, config, beliefs, par, basis, tv_conf, all_data,
                 training, validation, post, opt_T, K):
        self.config = config
        self.beliefs = beliefs
        self.par = par
        self.basis = basis
        self.tv_conf = tv_conf
        self.all_data = all_data
        self.training = training
        self.validation = validation
        self.post = post
        self.opt_T = opt_T
        self.K = K


class Hyperparams:
    def __init__(self, beliefs):
        self.beta = np.array(beliefs.beta)
        self.delta = np.array(beliefs.delta)
        self.sigma = beliefs.sigma
        self.nugget = beliefs.nugget


class Basis:
    """Mean-function basis h_0 = const, h_j(x) on input basis_inf[j-1] (reference
    :263-317).  Each basis_str entry is an expression in x, as in the reference
    (which exec()s it); numpy is available as np."""

    def __init__(self, beliefs):
        if beliefs.active != []:
            for i in range(len(beliefs.basis_inf)):
                if beliefs.basis_inf[i] not in beliefs.active:
                    print("WARNING: basis_inf specifies non-active inputs")
                    raise SystemExit(1)
            # drop basis terms on inactive inputs (the reference's in-place walk)
            keep_inf, keep_str = [], [beliefs.basis_str[0]]
            for i, inf in enumerate(beliefs.basis_inf):
                if inf in beliefs.active:
                    keep_inf.append(inf)
                    keep_str.append(beliefs.basis_str[i + 1])
                else:
                    print("Input", inf, "not active")
            beliefs.basis_inf[:] = keep_inf
            beliefs.basis_str[:] = keep_str
        beliefs.basis_inf = list(range(0, len(beliefs.basis_inf)))
        self.h = [self._compile(expr) for expr in beliefs.basis_str]
        self.exprs = list(beliefs.basis_str)
        self._print_mean_function(beliefs.basis_inf, beliefs.basis_str, beliefs.active)
        self.basis_inf = beliefs.basis_inf

    @staticmethod
    def _compile(expr):
        return eval("lambda x: " + expr, {"np": np, "numpy": np, "_np": np})

    def make_h(self, basis_str):
        """Append one basis function per expression (reference :293-299)."""
        self.h.extend(self._compile(expr) for expr in basis_str)

    def print_mean_function(self, basis_inf, basis_str, include):
        """(reference :301-317)"""
        self._print_mean_function(basis_inf, basis_str, include)

    def _print_mean_function(self, basis_inf, basis_str, include):
        meanf = "m(x) ="
        for i in range(len(self.h)):
            if i == 0:
                meanf += " b"
            else:
                idx = basis_inf[i - 1] if include == [] else include[i - 1]
                meanf += " + b" + str(idx) + basis_str[i] + "[" + str(idx) + "]"
        self.meanf = meanf
        print(meanf)

    def design_matrix(self, X):
        """H = (h(x_1), h(x_2), ...), n x q (reference Data.make_H :558-566)."""
        X = np.asarray(X, dtype=float)
        n = X.shape[0]
        H = np.empty((n, len(self.h)))
        H[:, 0] = self.h[0](1.0)
        for j in range(1, len(self.h)):
            col = X[:, self.basis_inf[j - 1]]
            try:
                H[:, j] = np.broadcast_to(np.asarray(self.h[j](col), dtype=float), (n,))
            except Exception:
                H[:, j] = [self.h[j](v) for v in col]
        return H


class TV_config:
    """Training/validation rounds (reference :321-375); interactive prompts kept."""

    def __init__(self, k, c, noV):
        self.k = k
        self.c = c
        self.noV = noV
        self.retrain = "y"
        self.no_of_trains = 0
        self.auto = False
        self.no_retrain = False

    def auto_train(self, auto, no_retrain):
        self.auto = bool(auto)
        self.no_retrain = no_retrain is not False

    def next_train(self):
        self.no_of_trains += 1

    def next_Vset(self):
        self.c += 1

    def check_still_training(self):
        if self.no_of_trains < self.noV:
            if not self.auto and self.no_of_trains >= 1:
                self.retrain = input("Retrain with V in T against new V? y/[n]: ")
            else:
                self.retrain = "n" if self.no_retrain else "y"
        else:
            self.retrain = "n"
        return self.retrain == "y"

    def doing_training(self):
        if self.no_of_trains < self.noV and self.retrain == "y":
            self.next_train()
            return True
        return False

    def do_final_build(self):
        if not self.auto:
            self.retrain = input("\nRetrain with V in T? y/[n]: ")
        else:
            self.retrain = "n" if self.no_retrain else "y"
        return self.retrain == "y"


class All_Data:
    """All data, scaled to [0,1], shuffled, split into T and V (reference :379-535)."""

    def __init__(self, all_inputs, all_outputs, tv, beliefs, par, datashuffle, scaleinputs):
        print("\n*** Reading data files ***")
        print("Reading inputs file:", all_inputs)
        try:
            self.x_full = np.loadtxt(all_inputs)
        except OSError:
            print("ERROR: Problem reading file.")
            raise SystemExit(1)
        if "output_index" in beliefs.beliefs:
            print("Emulator was trained on output_index", beliefs.output_index)
        print("Reading outputs file:", all_outputs)
        try:
            try:
                self.y_full = np.loadtxt(all_outputs, usecols=[beliefs.output]).T
                print("Using output", beliefs.output, "(relative to outputs file)")
            except IndexError:
                print("ERROR: output (column)", beliefs.output, "not in outputs file")
                raise SystemExit(1)
        except OSError:
            print("ERROR: Problem reading file.")
            raise SystemExit(1)
        self.dim = self.x_full[0].size
        if self.dim == 1:
            self.x_full = np.array([self.x_full]).T
        self.numpoints = self.x_full.shape[0]
        if self.x_full.shape[0] != self.y_full.size:
            print("WARNING: different number of data points in input and output files.")
            raise SystemExit(1)
        if "active_index" in beliefs.beliefs:
            print("Emulator was trained on active_index", beliefs.active_index)
        if beliefs.active != []:
            print("Including input dimensions", beliefs.active)
            self.x_full = self.x_full[:, beliefs.active]
        if len(par.delta) != self.x_full.shape[1]:
            print("WARNING: different number of delta than input dimensions.")
            raise SystemExit(1)
        self.input_minmax = beliefs.input_minmax
        self.map_inputs_0to1(par, scaleinputs)
        self.data_shuffle(datashuffle)
        self.T = 0
        self.V = 0
        self.tv = tv
        self.split_T_V_config()

    def map_inputs_0to1(self, par, scaleinputs):
        d = self.x_full.shape[1]
        if not scaleinputs:
            print("Input scaling off")
            self.minmax = np.array([(0.0, 1.0)] * d)
        elif self.input_minmax == []:
            print("Input scaling based on data")
            mm = [(np.amin(self.x_full[:, i]), np.amax(self.x_full[:, i])) for i in range(d)]
            self.minmax = np.array(mm)
            self.input_minmax = [list(t) for t in mm]
        else:
            print('Input scaling based on "input_minmax" in beliefs file')
            self.minmax = np.array(self.input_minmax)
        for i in range(d):
            span = self.minmax[i, 1] - self.minmax[i, 0]
            self.x_full[:, i] = (self.x_full[:, i] - self.minmax[i, 0]) / span
            print("Dim", i, "scaled by %", span)
        self.input_range = [[np.amin(self.x_full[:, i]), np.amax(self.x_full[:, i])]
                            for i in range(d)]

    def data_shuffle(self, datashuffle):
        if datashuffle:
            n, d = self.x_full.shape
            print("Shuffling", n, "data points")
            z = np.zeros((n, d + 1))
            z[:, :d] = self.x_full
            z[:, d] = self.y_full
            np.random.shuffle(z)            # same RNG consumption as the reference
            self.x_full[:, :] = z[:, :d]
            self.y_full = z[:, d]
        else:
            print("Data shuffling turned off")

    def split_T_V_config(self):
        n = self.x_full.shape[0]
        print("Split data into", self.tv.k, "sets")
        self.T = int((n / self.tv.k) * (self.tv.k - self.tv.noV))
        self.V = int((n / self.tv.k) * 1)
        self.remainder = n - (self.T + self.tv.noV * self.V)
        print("Remainder", self.remainder, "added to T-set")
        self.T = self.T + self.remainder
        print("T-set size:", self.T, ", V-set size:", self.V, ", V sets:", self.tv.noV)

    def choose_T(self):
        rows = list(range(0, self.tv.c * self.V)) + \
            list(range((self.tv.c + self.tv.noV) * self.V, self.tv.k * self.V + self.remainder))
        return self.x_full[rows, :], self.y_full[rows]

    def choose_V(self):
        rows = list(range(self.tv.c * self.V, (self.tv.c + 1) * self.V))
        return self.x_full[rows, :], self.y_full[rows]

    def choose_new_V(self, validation):
        rows = list(range(self.tv.c * self.V, (self.tv.c + 1) * self.V))
        validation.inputs = self.x_full[rows, :]
        validation.outputs = self.y_full[rows]


class Data:
    """A data set with its basis matrix H and covariance A (reference :539-584).

    ``make_A(s2, predict)`` records how A is defined -- K.var(inputs, predict),
    plus r/s2 on the diagonal for the alt-nugget kernel -- and ``A`` is built on
    the GPU when read.  The objective and the posterior never need it on the host.
    """

    def __init__(self, inputs, outputs, basis, par, beliefs, K):
        self.inputs = inputs
        self.outputs = outputs
        self.basis = basis
        self.beliefs = beliefs
        self.par = par
        self.K = K
        self.r = 0
        self.make_H()
        self.make_A()

    def remake(self):
        self.make_H()
        self.make_A()

    def make_H(self):
        self.H = self.basis.design_matrix(self.inputs)

    def make_E(self):
        self.E = self.H.dot(self.par.beta)

    def make_A(self, s2=1.0, predict=True):
        self._A_def = (float(s2), bool(predict))
        self._A_cache = None

    def r_scale(self):
        """Coefficient of diag(r) in A (reference :574-575: r/s2, alt-nugget only)."""
        if self.beliefs.alt_nugget != "T" or np.isscalar(self.r):
            return 0.0
        return 1.0 / self._A_def[0]

    @property
    def A(self):
        if self._A_cache is None:
            s2, predict = self._A_def
            rs = self.r_scale()
            self._A_cache = native.default_context().kernel_var(
                self.K.kind, self.K.d, float(self.K.n), self.inputs, predict=predict,
                r=None if rs == 0.0 else self.r, r_scale=rs)
        return self._A_cache

    @A.setter
    def A(self, value):
        self._A_cache = value

    def set_r(self, r, message=True):
        if len(r) == self.inputs.shape[0]:
            if message:
                print("\n*** Updating array 'r' of constant variances***")
            self.r = r
            self._A_cache = None
        else:
            print("\nWARNING: length of 'r' does not match number of data points")
            raise SystemExit(1)


def upload_training(D):
    """Make D (inputs, outputs, H, r) the resident training set of the context."""
    ctx = native.default_context()
    r = None if np.isscalar(D.r) else D.r
    ctx.ensure_data(D.inputs, D.outputs, D.H, r)
    return ctx


class Posterior:
    """Posterior mean and variance at Dnew given Dold (reference :588-676).

    mean = H* beta + K*^T A^-1 (f - H beta)
    var  = sigma^2 (A** - K*^T A^-1 K* + T (H^T A^-1 H)^-1 T^T),  T = H* - K*^T A^-1 H
    with A = Dold.A as the reference holds it and A** = Dnew.A (K.var plus Dnew's r/s2
    for the alt-nugget kernel).  ``full_var=False`` returns only the
    diagonal (what plot / history matching use) and supports any number of points.
    The reference's ``predict`` flag has no effect (its use is commented out, :621).
    """

    def __init__(self, Dnew, Dold, par, beliefs, K, predict=True, full_var=True):
        self.Dnew = Dnew
        self.Dold = Dold
        self.par = par
        self.beliefs = beliefs
        self.K = K
        self.predict = predict
        self.full_var = full_var
        self.remake()

    def remake(self):
        self._covar = None
        ctx = upload_training(self.Dold)
        ctx.ensure_factor(self.K.kind, self.K.d, float(self.K.n), 1.0, self.Dold.r_scale())
        self.mean, self.var = ctx.posterior(self.Dnew.inputs, self.Dnew.H, self.par.beta,
                                            float(self.par.sigma), full_var=self.full_var)
        rs = self.Dnew.r_scale()
        if rs != 0.0:
            # Dnew.A carries Dnew's own r/s2 on its diagonal (:572-575), so sigma^2 r/s2 is
            # part of var (:625-631); noise_fit sets it (noise_fit.py:118-121)
            add = float(self.par.sigma) ** 2 * rs * np.asarray(self.Dnew.r, dtype=float)
            if self.var.ndim == 2:
                self.var[np.diag_indices_from(self.var)] += add
            else:
                self.var = self.var + add

    # reference-compatible pieces
    def make_covar(self):
        self._covar = self.K.covar(self.Dold.inputs, self.Dnew.inputs)

    @property
    def covar(self):
        if self._covar is None:
            self.make_covar()
        return self._covar

    def make_mean(self):
        self.remake()

    def make_var(self):
        self.remake()

    def _diag(self):
        return np.diag(self.var) if self.var.ndim == 2 else self.var

    def interval(self):
        sd = np.sqrt(np.abs(self._diag()))
        self.LI = self.mean - 1.96 * sd
        self.UI = self.mean + 1.96 * sd

    def indiv_standard_error(self, ise=2.0):
        retrain = False
        e = (self.Dnew.outputs - self.mean) / np.sqrt(self._diag())
        for i in range(e.size):
            if np.abs(e[i]) >= ise:
                print("  Bad predictions:", self.Dnew.inputs[i, :], "ise:", np.round(e[i], decimals=4))
                retrain = True
        return retrain

    def mahalanobis_distance(self):
        MDtheo = self.Dnew.outputs.size
        try:
            MDtheovar = 2 * self.Dnew.outputs.size * \
                (self.Dnew.outputs.size + self.Dold.outputs.size - self.par.beta.size - 2.0) / \
                (self.Dold.outputs.size - self.par.beta.size - 4.0)
            print("theoretical Mahalanobis_distance (mean, var):(", MDtheo, ",", MDtheovar, ")")
        except ZeroDivisionError:
            print("theoretical Mahalanobis_distance mean:", MDtheo, "(too few data for variance)")
        resid = self.Dnew.outputs - self.mean
        MD = resid.T.dot(np.linalg.solve(self.var, resid))
        print("calculated Mahalanobis_distance:", MD)
        return True

    def incVinT(self):
        self.Dold.inputs = np.append(self.Dnew.inputs, self.Dold.inputs, axis=0)
        self.Dold.outputs = np.append(self.Dnew.outputs, self.Dold.outputs)
        print("Include V into T, T-set size:", self.Dold.inputs.shape[0])
        n, q = self.Dold.inputs.shape[0], len(self.Dold.basis.h)
        self.Dold.H = np.zeros([n, q])
        self.Dold.A = None          # rebuilt lazily after the caller's remake()

    def final_design_points(self, E, final=False):
        suffix = "f" if final else ""
        n = str(E.tv_conf.no_of_trains)
        o = str(E.beliefs.output)
        i_file = E.config.inputs + "-o" + o + "-" + n + suffix
        o_file = E.config.outputs + "-o" + o + "-" + n + suffix
        data = np.copy(self.Dold.inputs)
        mm = E.all_data.minmax
        for i in range(data.shape[1]):
            data[:, i] = data[:, i] * (mm[i, 1] - mm[i, 0]) + mm[i, 0]
        print("Writing T-data to:", i_file)
        try:
            np.savetxt(i_file, data, delimiter=" ", fmt="%.8f")
        except OSError:
            print("ERROR: Problem writing to file.")
            raise SystemExit(1)
        print("Writing T-data to:", o_file)
        try:
            np.savetxt(o_file, self.Dold.outputs, delimiter=" ", fmt="%.8f")
        except OSError:
            print("ERROR: Problem writing to file.")
            raise SystemExit(1)
