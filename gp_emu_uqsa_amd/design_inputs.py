"""Optimised Latin hypercube designs (reference: design_inputs/design_inputs.py:13-77).

Behaviour kept for drop-in parity with the reference:
- the same np.random consumption: per design k and dimension i, uniform(0, 1, n) then
  shuffle(arange(n));
- the same selection rule. The reference records `argmin(pdist(...))`, the INDEX of the closest
  pair, as "maximin", and keeps the design whose index is largest (:62-67). It is not the design
  with the largest minimum distance, but it is what reference runs produce, so it is reproduced;
- the same unscaling to `minmax` and the same '%.8f' text file.

Only the removed `np.int` alias (:54) is replaced by `int`.
"""
from __future__ import annotations

import numpy as _np
import scipy.spatial.distance as _dist


def optLatinHyperCube(dim=None, n=None, N=None, minmax=None, filename="inputs", fextra=None):
    """Design n points in `dim` dimensions, pick one of N oLHC designs, save to `filename`."""
    print('dim:', dim)
    print('n:', n)
    print('N:', N)
    print('minmax:', minmax)
    print('filename:', filename)
    if dim is None or n is None or N is None or minmax is None:
        print("Please supply values for function arguments (default for filename is \"inputs\")")
    if len(minmax) != dim:
        print("WARNING: length of 'minmax' (list of lists) must equal 'dim'")
        raise SystemExit
    what = "combining with supplied extra data, " if fextra is not None else ""
    print("\nGenerating", N, "oLHC samples of", n, "points,", what +
          "and checking maximin criterion (pick design with maximum minimum distance between design points)...")
    u = _np.zeros((n, dim))
    b = _np.zeros((n, dim), dtype=int)
    x = _np.zeros((n, dim))
    best_D, best_k, best_maximin = None, 0, None
    for k in range(N):
        for i in range(dim):
            u[:, i] = _np.random.uniform(0.0, 1.0, n)
            b[:, i] = _np.arange(0, n, 1)
            _np.random.shuffle(b[:, i])
            x[:, i] = (b[:, i] + u[:, i]) / float(n)
        xt = _np.concatenate([x, fextra]) if fextra is not None else x
        maximin = _np.argmin(_dist.pdist(xt, 'sqeuclidean'))
        if k == 0 or maximin > best_maximin:
            best_D = _np.copy(x)
            best_k = k
            best_maximin = maximin
    D = best_D
    print("Optimal LHC design was no.", best_k)
    print("Saving inputs to file...")
    lim = _np.array(minmax, dtype=float)
    for i in range(dim):
        D[:, i] = D[:, i] * (lim[i, 1] - lim[i, 0]) + lim[i, 0]
    _np.savetxt(filename, D, delimiter=" ", fmt='%.8f')
    print("DONE!")
    return None
