"""Covariance kernel objects with the reference's duck-typed interface
(_emulatorkernels.py:10-79 ``kernel``, :83-152 ``kernel_alt_nug``): state
``d`` (length scales delta) and ``n`` (nugget), ``set_hp``, ``set_params``,
``transform``/``untransform`` (x = 2 log hp), ``var`` and ``covar``.

``var`` / ``covar`` are evaluated on the GPU (gpe_kernel_var / gpe_kernel_covar);
the objective never materialises them -- it builds the covariance inside
gpe_objective.  ``kind`` is the C-ABI kernel code.
"""
from __future__ import annotations

import numpy as _np

from . import native


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
        return self.A

    def covar(self, XT, XV):
        return native.default_context().kernel_covar(self.kind, self.d, float(self.n), XT, XV)


class kernel(_GaussianBase):
    """(1-nugget) exp(-sum((x-x')/delta)^2), nugget added back on the diagonal."""
    kind = native.KERNEL_STD


class kernel_alt_nug(_GaussianBase):
    """exp(-sum((x-x')/delta)^2), nugget^2 added on the diagonal."""
    kind = native.KERNEL_ALT_NUG
