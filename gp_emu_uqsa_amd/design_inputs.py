"""Optimised Latin hypercube designs (reference: design_inputs/design_inputs.py:13-77).

Behaviour kept for drop-in parity with the reference:
- the same np.random consumption: per design k and dimension i, uniform(0, 1, n) then
  shuffle(arange(n));
- the same selection rule. The reference records `argmin(pdist(...))`, the INDEX of the closest
  pair, as "maximin", and keeps the design whose index is largest (:62-67). It is not the design
  with the largest minimum distance, but it is what reference runs produce, so it is reproduced;
- the same unscaling to `minmax` and the same '%.8f' text file.

Only the removed `np.int` alias (:54) is replaced by `int`.

The selection statistic, argmin(pdist([x_k; fextra])) over every candidate design, is
computed on the GPU (gpe_lhc_maximin: all N designs batched, the fextra-fextra pairs once)
with distances bit-identical to pdist's.  The designs are drawn on the host first, in the
reference's RNG order, in batches of at most _BATCH doubles.
"""
from __future__ import annotations

import numpy as _np

from . import native as _native

_BATCH = 1 << 25


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
    xe = None if fextra is None else _np.asarray(fextra, dtype=float).reshape(-1, dim)
    if n + (0 if xe is None else xe.shape[0]) < 2:
        raise ValueError("attempt to get argmin of an empty sequence")
    u = _np.zeros((n, dim))
    b = _np.zeros((n, dim), dtype=int)
    best_D, best_k, best_maximin = None, 0, None
    per = max(1, _BATCH // (n * dim))
    ctx = _native.default_context()
    for k0 in range(0, N, per):
        kb = min(per, N - k0)
        xs = _np.empty((kb, n, dim))
        for k in range(kb):
            for i in range(dim):
                u[:, i] = _np.random.uniform(0.0, 1.0, n)
                b[:, i] = _np.arange(0, n, 1)
                _np.random.shuffle(b[:, i])
                xs[k, :, i] = (b[:, i] + u[:, i]) / float(n)
        maximin = ctx.lhc_maximin(xs, xe)
        for k in range(kb):
            if k0 + k == 0 or maximin[k] > best_maximin:
                best_D = _np.copy(xs[k])
                best_k = k0 + k
                best_maximin = maximin[k]
    D = best_D
    print("Optimal LHC design was no.", best_k)
    print("Saving inputs to file...")
    lim = _np.array(minmax, dtype=float)
    for i in range(dim):
        D[:, i] = D[:, i] * (lim[i, 1] - lim[i, 0]) + lim[i, 0]
    _np.savetxt(filename, D, delimiter=" ", fmt='%.8f')
    print("DONE!")
    return None
