"""CPU oracle of the oLHC selection statistic -- TEST INFRASTRUCTURE ONLY (only tests/
may import it; the product computes it with gpe_lhc_maximin).

design_inputs.py:62 of the reference (MathThyMod/GP_emu_UQSA) evaluates, per candidate
design x_k, ``argmin(pdist(concatenate([x_k, fextra]), 'sqeuclidean'))`` -- scipy's
condensed pair order, numpy's first occurrence on ties and NaN as the minimum.  This is
that expression, op for op, over a batch of designs.  Pinned by the reference's own
designs (tests/golden/history_match.npz, G7: the designs imp_plot wrote).
"""
from __future__ import annotations

import numpy as np
from scipy.spatial import distance as _dist


def lhc_maximin_ref(designs, fextra=None):
    """designs: N x n x dim -> int64[N], the reference's per-design "maximin" index."""
    out = np.empty(len(designs), dtype=np.int64)
    for k, x in enumerate(designs):
        xt = np.concatenate([x, fextra]) if fextra is not None else x
        out[k] = np.argmin(_dist.pdist(xt, "sqeuclidean"))
    return out


class OracleContext:
    """Stands in for native.Context in host-logic tests on machines without a GPU."""

    def lhc_maximin(self, designs, fextra=None):
        return lhc_maximin_ref(designs, fextra)
