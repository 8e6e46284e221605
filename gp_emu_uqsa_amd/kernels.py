"""Covariance kernel objects with the reference's duck-typed interface
(_emulatorkernels.py:10-79 ``kernel``, :83-152 ``kernel_alt_nug``): state
``d`` (length scales delta) and ``n`` (nugget), ``set_hp``, ``set_params``,
``transform``/``untransform`` (x = 2 log hp), ``var``, ``covar``, ``grad_delta_A`` and
``grad_nugget_A``.

``var`` / ``covar`` / the gradients are evaluated on the GPU (gpe_kernel_var /
gpe_kernel_covar / gpe_kernel_grad); the objective never materialises them -- it
builds the covariance and contracts the gradient inside gpe_objective.  ``kind`` is
the C-ABI kernel code.
"""
from __future__ import annotations

import numpy as _np

from . import native

# the reference sets NumPy's global print options when its kernel, optimiser and
# plotting modules are imported (_emulatorkernels.py:6-7, _emulatoroptimise.py:19-20,
# _emulatorplotting.py:6-7); its printed arrays (hyperparameters, "Bad predictions")
# depend on them
_np.set_printoptions(precision=6)
_np.set_printoptions(suppress=True)


class _GaussianBase:
    kind = native.KERNEL_STD

    def __init__(self, dim, par):
        self.d = _np.asarray(par.delta, dtype=float)
        self.n = par.nugget

    def set_hp(self, d, s, n):
        self.d = d
        self.n = n

    def set_params(self, x):
        """delta = x[:d]; nugget = x[-1] when x is longer (reference :20-24)."""
        x = _np.asarray(x, dtype=float)
        size = _np.asarray(self.d).size
        self.d = x[0:size]
        if x.size > size:
            self.n = x[-1]

    def print_kernel(self):
        print("delta:", self.d)
        print("nugget:", self.n)

    @staticmethod
    def transform(hp):
        return 2.0 * _np.log(hp)

    @staticmethod
    def untransform(hp):
        return _np.exp(_np.asarray(hp) / 2.0)

    def var(self, X, predict=True):
        """K(X, X): off-diagonal (1-nu) exp(-r^2) / exp(-r^2), diagonal per kind."""
        X = _np.asarray(X, dtype=float)
        if X.ndim == 1:
            X = X.reshape(-1, 1)
        self.A = native.default_context().kernel_var(self.kind, self.d, float(self.n), X,
                                                     predict=predict)
        # what the reference's exp_save holds: the points and length scales of this call
        self._var_X = X.copy()
        self._var_d = _np.array(self.d, dtype=float, copy=True)
        return self.A

    def _exp_state(self):
        try:
            return self._var_X, self._var_d
        except AttributeError:   # the reference fails the same way: no exp_save before var()
            raise AttributeError("'%s' object has no attribute 'exp_save'" % type(self).__name__) from None

    def grad_delta_A(self, X, di, s2):
        """dA/d(2 log delta_di) (reference :53-63, alt :126-136): s2 (1-nu) ((x_k - x_l)/delta_di)^2
        exp_save (alt: no (1-nu)), zero diagonal; X is the input column, exp_save that of
        the preceding var()."""
        Xv, dv = self._exp_state()
        pre = s2 if self.kind == native.KERNEL_ALT_NUG else (1.0 - self.n) * s2
        return native.default_context().kernel_grad(dv, Xv, _np.asarray(X, dtype=float).ravel(),
                                                    1.0 / float(self.d[di]), pre)

    def grad_nugget_A(self, X, s2):
        """dA/d(2 log nu) (reference :66-71): -nu s2 / 2 exp_save off the diagonal;
        alt-nugget (:139-144): s2 nu^2 on the diagonal only."""
        X = _np.asarray(X, dtype=float)
        if self.kind == native.KERNEL_ALT_NUG:
            f = _np.zeros((X.shape[0], X.shape[0]))
            _np.fill_diagonal(f, (self.n ** 2) * s2)
            return f
        Xv, dv = self._exp_state()
        return native.default_context().kernel_grad(dv, Xv, None, 0.0, 0.5 * (-self.n) * s2)

    def covar(self, XT, XV):
        return native.default_context().kernel_covar(self.kind, self.d, float(self.n), XT, XV)


class kernel(_GaussianBase):
    """(1-nugget) exp(-sum((x-x')/delta)^2), nugget added back on the diagonal."""
    kind = native.KERNEL_STD


class kernel_alt_nug(_GaussianBase):
    """exp(-sum((x-x')/delta)^2), nugget^2 added on the diagonal."""
    kind = native.KERNEL_ALT_NUG
