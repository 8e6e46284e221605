"""Synthetic measurement inputs: an oLHC-style design, toysim3D-
style outputs and the linear basis, for bench.py and the tools.

Design: column j is a random permutation of 0..n-1 plus U(0,1), divided by n
(one design of design_inputs.py:54-64; the maximin choice among several designs
is skipped, as 8d prescribes), then min-max scaled per column like
_emulatorclasses.py:457-471.  Outputs: 3 x0^3 + exp(cos(10 x1) cos^2(5 x0)) +
exp(sin(7.5 x2)) + sum_{k>=3} 0.1 sin(2 pi xk) + 0.01 N(0,1)
(examples/sensitivity_multi_outputs/toysim3D.py:16 extended to d inputs).
The random streams are numpy RandomState(seed) for the design and
RandomState(seed + 1000) for the noise.
"""
from __future__ import annotations

import numpy as np


def design(n: int, d: int, seed: int = 0) -> np.ndarray:
    rs = np.random.RandomState(seed)
    cols = []
    for _ in range(d):
        jitter = rs.uniform(0.0, 1.0, n)
        perm = np.arange(n)
        rs.shuffle(perm)
        cols.append((perm + jitter) / float(n))
    x = np.stack(cols, axis=1)
    lo, hi = x.min(axis=0), x.max(axis=0)
    return (x - lo) / (hi - lo)


def outputs(X: np.ndarray, seed: int = 0) -> np.ndarray:
    noise = np.random.RandomState(seed + 1000).standard_normal(X.shape[0])
    d = X.shape[1]
    y = 3.0 * X[:, 0] ** 3
    if d > 1:
        y = y + np.exp(np.cos(10.0 * X[:, 1]) * np.cos(5.0 * X[:, 0]) ** 2)
    if d > 2:
        y = y + np.exp(np.sin(7.5 * X[:, 2]))
    for k in range(3, d):
        y = y + 0.1 * np.sin(2.0 * np.pi * X[:, k])
    return y + 0.01 * noise


def linear_basis(X: np.ndarray) -> np.ndarray:
    """H = [1, x_0, ..., x_{d-1}]  (basis_str '1.0 x x ...')."""
    return np.hstack([np.ones((X.shape[0], 1)), X])


def problem(n: int, d: int, seed: int = 0):
    """(X, f, H) for n points in d dimensions."""
    X = design(n, d, seed)
    return X, outputs(X, seed), linear_basis(X)
