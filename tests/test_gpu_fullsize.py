"""Parity at BASELINE.json's full sizes through size-independent properties (the CPU
oracle cannot run there: the reference takes ~1230 s per evaluation at n=16384).

- C3 (n=16384, d=10): the single-GPU objective (fused Cholesky, recursive TRTRI,
  LAUUM, fused contraction) against the row-block distributed objective on loopback
  ranks (different partition, schedule and reduction order; the row TRTRI and
  per-rank A^-1 partials), value and gradient; and the gradient against central
  differences of the value in the transformed coordinates x = 2 log hp.
- C4 (n=65536, d=20): the single-GPU value and gradient against the loopback
  distributed path at P=8 (eight logical ranks, each with its own buffers, through
  the pack / all-gather / unpermute and broadcast-row path), and every rank's device
  memory within 12 GB (its tile rows of A and of L^-1 plus one slab of its A^-1
  partial: O(n^2 / P)).
Tolerances: value 1e-10 relative; gradient 1e-8 of max|g| between the two exact
paths; finite differences 1e-4 of max|g| (step 1e-4, LLH ~ 4e5 carries ~1e-10
relative rounding at cond(A) ~ 1e6).
"""
import numpy as np
import pytest

from gp_emu_uqsa_amd import native, synthetic

pytestmark = pytest.mark.gpu


def _hp(d):
    return np.concatenate([np.ones(d), [1e-3, 1.0]])


def test_c3_fullsize_objective():
    n, d = 16384, 10
    X, f, H = synthetic.problem(n, d, seed=0)
    hp = _hp(d)
    ctx = native.Context(0)
    ctx.set_data(X, f, H)
    llh, g, _ = ctx.objective(native.GP4ML, native.KERNEL_STD, hp)
    assert np.isfinite(llh) and np.all(np.isfinite(g))
    # distributed loopback, 2 ranks
    dc = native.DistContext(0, 2)
    dc.set_data(X, f, H)
    llh2, g2, _ = dc.objective(native.GP4ML, native.KERNEL_STD, hp, want_grad=True)
    dc.close()
    assert abs(llh2 - llh) <= 1e-10 * abs(llh), (llh, llh2)
    scale = np.max(np.abs(g))
    assert np.max(np.abs(g2 - g)) <= 1e-8 * scale, np.max(np.abs(g2 - g)) / scale
    # central differences in x = 2 log hp for delta_0, nu and sigma
    h = 1e-4
    for k in (0, d, d + 1):
        xp, xm = hp.copy(), hp.copy()
        xp[k] *= np.exp(h / 2)
        xm[k] *= np.exp(-h / 2)
        fp = ctx.objective(native.GP4ML, native.KERNEL_STD, xp, want_grad=False)[0]
        fm = ctx.objective(native.GP4ML, native.KERNEL_STD, xm, want_grad=False)[0]
        fd = (fp - fm) / (2 * h)
        assert abs(fd - g[k]) <= 1e-4 * scale, (k, fd, g[k], scale)
    ctx.close()


def test_c4_fullsize_objective():
    n, d = 65536, 20
    X, f, H = synthetic.problem(n, d, seed=0)
    hp = _hp(d)
    ctx = native.Context(0)
    ctx.set_data(X, f, H)
    llh, g, _ = ctx.objective(native.GP4ML, native.KERNEL_STD, hp)
    ctx.close()
    del ctx
    dc = native.DistContext(0, 8)
    dc.set_data(X, f, H)
    llh8, _ = dc.objective(native.GP4ML, native.KERNEL_STD, hp)
    assert abs(llh8 - llh) <= 1e-10 * abs(llh), (llh, llh8)
    llh8g, g8, _ = dc.objective(native.GP4ML, native.KERNEL_STD, hp, want_grad=True)
    per_rank = [dc.rank_bytes(r) for r in range(8)]
    dc.close()
    assert llh8g == llh8
    scale = np.max(np.abs(g))
    assert np.max(np.abs(g8 - g)) <= 1e-8 * scale, np.max(np.abs(g8 - g)) / scale
    # rows of A and L^-1, slab and buffers under 12 GB; plus the int8 partial's buffers
    # (gpemu_dist.hip oz_prepare): 16 planes of X_r^T (65536 x 64 tile rows of 128) and 16
    # residue images of the largest 8-row slab's 256-tiles (tile rows 252-255, 1018 tiles)
    oz = 16 * 65536 * 64 * 128 + 16 * 1018 * 256 * 256
    assert max(per_rank) <= 12e9 + oz, per_rank
