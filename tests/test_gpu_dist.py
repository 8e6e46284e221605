"""Row-block distributed objective and gradient (include/gpemu_dist.h) on the GPU:
the loopback transport (P logical ranks in one process, each with its own
buffers, running the device code of the RCCL path -- pack, all-gather buffer,
unpermute, broadcast rows, all-reduced partials -- with copies for the
collectives) for P = 1..8, and a 1-rank RCCL communicator, against the oracle
(reference op order) and the single-GPU path.

Gradient tolerance as tests/test_gpu_objective.py:
|g - g_ref| <= 1e-7 (|g_ref| + max|g_ref|)."""
import numpy as np
import pytest

from gp_emu_uqsa_amd import native
from oracle import gp_oracle as orc

pytestmark = pytest.mark.gpu


def _hp(d, fit_nug=True, gp4ml=True):
    hp = [0.6 + 0.1 * k for k in range(d)]
    if fit_nug:
        hp.append(1e-2)
    if gp4ml:
        hp.append(0.9)
    return np.array(hp)


@pytest.mark.parametrize("P", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("n", [300, 1000])
def test_loopback_matches_oracle(P, n):
    X, f, H = orc.synthetic_problem(n, 3, seed=1)
    hp = _hp(3)
    ctx = native.DistContext(0, P)
    ctx.set_data(X, f, H)
    llh, s2 = ctx.objective(native.GP4ML, native.KERNEL_STD, hp)
    ref = orc.objective_ref(X, f, H, hp, orc.GP4ML, orc.STD, True, want_grad=False)[0]
    assert abs(llh - ref) <= 1e-9 * abs(ref), (llh, ref)
    assert abs(s2 - hp[-1] ** 2) < 1e-15
    ctx.close()


@pytest.mark.parametrize("variant,kernel,use_r", [(native.MUCM, native.KERNEL_STD, False),
                                                  (native.GP4ML, native.KERNEL_ALT_NUG, True)])
def test_loopback_variants_match_single_gpu(ctx, variant, kernel, use_r):
    n, d = 777, 4
    X, f, H = orc.synthetic_problem(n, d, seed=2)
    r = np.random.RandomState(5).uniform(1e-4, 1e-3, size=n) if use_r else None
    hp = _hp(d, gp4ml=variant == native.GP4ML)
    ctx.set_data(X, f, H, r)
    ref, _, s2ref = ctx.objective(variant, kernel, hp, want_grad=False)
    dc = native.DistContext(0, 3)
    dc.set_data(X, f, H, r)
    llh, s2 = dc.objective(variant, kernel, hp)
    assert abs(llh - ref) <= 1e-10 * abs(ref), (llh, ref)
    assert abs(s2 - s2ref) <= 1e-10 * abs(s2ref)
    dc.close()


def _grad_ok(g, gref, tol=1e-7):
    g, gref = np.asarray(g), np.asarray(gref)
    err = np.abs(g - gref)
    return bool(np.all(err <= tol * (np.abs(gref) + np.abs(gref).max()))), err.max()


@pytest.mark.parametrize("P", [1, 2, 3, 5, 8])
@pytest.mark.parametrize("n", [300, 1000])
def test_loopback_gradient_matches_oracle(P, n):
    d = 3
    X, f, H = orc.synthetic_problem(n, d, seed=1)
    hp = _hp(d)
    ctx = native.DistContext(0, P)
    ctx.set_data(X, f, H)
    llh, g, s2 = ctx.objective(native.GP4ML, native.KERNEL_STD, hp, want_grad=True)
    ref, gref = orc.objective_ref(X, f, H, hp, orc.GP4ML, orc.STD, True)[:2]
    assert abs(llh - ref) <= 1e-9 * abs(ref), (llh, ref)
    ok, err = _grad_ok(g, gref)
    assert ok, (g, gref, err)
    # value-only call after a gradient call reuses the same buffers
    llh2, _ = ctx.objective(native.GP4ML, native.KERNEL_STD, hp)
    assert llh2 == llh
    ctx.close()


@pytest.mark.parametrize("variant,kernel,use_r,d,P", [(native.MUCM, native.KERNEL_STD, False, 4, 3),
                                                       (native.GP4ML, native.KERNEL_ALT_NUG, True, 4, 2),
                                                       (native.GP4ML, native.KERNEL_STD, True, 4, 3),
                                                       (native.GP4ML, native.KERNEL_STD, False, 10, 4),
                                                       (native.GP4ML, native.KERNEL_STD, False, 20, 3)])
def test_loopback_gradient_matches_single_gpu(ctx, variant, kernel, use_r, d, P):
    n = 1100
    X, f, H = orc.synthetic_problem(n, d, seed=6)
    r = np.random.RandomState(5).uniform(1e-4, 1e-3, size=n) if use_r else None
    hp = _hp(d, gp4ml=variant == native.GP4ML)
    ctx.set_data(X, f, H, r)
    ref, gref, s2ref = ctx.objective(variant, kernel, hp, want_grad=True)
    dc = native.DistContext(0, P)
    dc.set_data(X, f, H, r)
    llh, g, s2 = dc.objective(variant, kernel, hp, want_grad=True)
    assert abs(llh - ref) <= 1e-10 * abs(ref), (llh, ref)
    assert abs(s2 - s2ref) <= 1e-10 * abs(s2ref)
    ok, err = _grad_ok(g, gref)
    assert ok, (g, gref, err)
    dc.close()


def test_loopback_not_pd():
    X, f, H = orc.synthetic_problem(400, 2, seed=3)
    X[1] = X[0]                                   # duplicate point, no nugget
    dc = native.DistContext(0, 2)
    dc.set_data(X, f, H)
    with pytest.raises(native.NotPositiveDefinite):
        dc.objective(native.GP4ML, native.KERNEL_STD, np.array([0.5, 0.5, 1.0]), nu_fixed=0.0)
    with pytest.raises(native.NotPositiveDefinite):
        dc.objective(native.GP4ML, native.KERNEL_STD, np.array([0.5, 0.5, 1.0]), nu_fixed=0.0, want_grad=True)
    dc.close()


def test_rccl_single_rank():
    n, d = 2000, 10
    X, f, H = orc.synthetic_problem(n, d, seed=4)
    hp = _hp(d)
    dc = native.DistContext(0, 1, 0, native.dist_unique_id())
    dc.set_data(X, f, H)
    llh, _ = dc.objective(native.GP4ML, native.KERNEL_STD, hp)
    ref, gref = orc.objective_ref(X, f, H, hp, orc.GP4ML, orc.STD, True)[:2]
    assert abs(llh - ref) <= 1e-9 * abs(ref), (llh, ref)
    llh_g, g, _ = dc.objective(native.GP4ML, native.KERNEL_STD, hp, want_grad=True)
    assert llh_g == llh
    ok, err = _grad_ok(g, gref)
    assert ok, (g, gref, err)
    t = dc.times()
    assert t["total_ms"] > 0.0
    dc.close()


@pytest.mark.parametrize("groups", ["4:0", "3:0", "2:0,1:0"])
@pytest.mark.parametrize("P", [1, 3])
def test_loopback_column_groups(ctx, monkeypatch, groups, P):
    """Column groups (pending updates inside the group, one K = 128 W trailing update
    per group; GPEMU_DIST_W forces widths on a small matrix): value and gradient equal
    the single-GPU path, incl. the augmented [f H] row and a ragged last group."""
    monkeypatch.setenv("GPEMU_DIST_W", groups)
    n, d = 1000, 4
    X, f, H = orc.synthetic_problem(n, d, seed=3)
    hp = _hp(d)
    ctx.set_data(X, f, H)
    ref, gref, _ = ctx.objective(native.GP4ML, native.KERNEL_STD, hp)
    dc = native.DistContext(0, P)
    dc.set_data(X, f, H)
    llh, g, _ = dc.objective(native.GP4ML, native.KERNEL_STD, hp, want_grad=True)
    dc.close()
    assert abs(llh - ref) <= 1e-10 * abs(ref), (llh, ref)
    ok, err = _grad_ok(g, gref, 1e-8)
    assert ok, err


@pytest.mark.parametrize("P", [1, 3])
def test_loopback_gradient_chunked_trtri(ctx, monkeypatch, P):
    """A one-tile-row slab (GPEMU_DIST_SLAB_MB=1) splits the recursive TRTRI's upper
    levels into column chunks of 1-2 tiles (each with its own pair of all-gathers) and
    the A^-1 partial into one-row slabs: value and gradient as the single-GPU path."""
    monkeypatch.setenv("GPEMU_DIST_SLAB_MB", "1")
    n, d = 3000, 4
    X, f, H = orc.synthetic_problem(n, d, seed=11)
    hp = _hp(d)
    ctx.set_data(X, f, H)
    ref, gref, _ = ctx.objective(native.GP4ML, native.KERNEL_STD, hp, want_grad=True)
    dc = native.DistContext(0, P)
    dc.set_data(X, f, H)
    llh, g, _ = dc.objective(native.GP4ML, native.KERNEL_STD, hp, want_grad=True)
    dc.close()
    assert abs(llh - ref) <= 1e-10 * abs(ref), (llh, ref)
    ok, err = _grad_ok(g, gref)
    assert ok, (g, gref, err)


@pytest.mark.parametrize("n,P", [(4000, 2), (4000, 3), (10240, 4)])
def test_loopback_rank_memory(n, P):
    """Each logical rank holds its own tile rows (of A and, after a gradient call, of
    L^-1): the per-rank bytes follow the partition, not n^2.  Upper bound after the
    gradient: its rows of L^-1 plus at most three slab-sized buffers (the A^-1 partial's
    slab, the TRTRI's gathered X11 and all-gather buffer), the slab being the whole
    triangle's tile rows / P (at least 512 MiB, at most the whole) -- at n = 10240, P = 4
    one n x n partial per rank (the round-4 slab) would exceed it."""
    d = 3
    X, f, H = orc.synthetic_problem(n, d, seed=1)
    dc = native.DistContext(0, P)
    dc.set_data(X, f, H)
    nb = (n + 127) // 128
    np_ = nb * 128
    val = [dc.rank_bytes(r) for r in range(P)]
    # the two gathered-panel buffers (P > 1): (NB + 1) * 128 rows x the widest column
    # group's columns, at most 8 tiles -- O(n), not O(n^2)
    panels = 2 * (nb + 1) * 128 * 8 * 128 * 8
    for r in range(P):
        rows = native.dist_local_rows(n, P, r, d + 1)
        assert val[r] >= rows * 128 * (nb + 1) * 128 * 8            # its tile rows of A
        assert val[r] < (rows + 1) * 128 * (nb + 1) * 128 * 8 + panels + (32 << 20)   # panels, inputs
    dc.objective(native.GP4ML, native.KERNEL_STD, _hp(d), want_grad=True)
    grad = [dc.rank_bytes(r) for r in range(P)]
    whole = nb * 128 * np_
    slab = min(whole, max(1 << 26, whole // P)) * 8
    for r in range(P):
        rows = native.dist_local_rows(n, P, r, d + 1)
        xrows = rows * 128 * nb * 128 * 8
        assert grad[r] - val[r] >= xrows                            # its rows of L^-1
        assert grad[r] - val[r] <= xrows + 3 * slab + (64 << 20), (grad[r] - val[r], xrows, slab)
    with pytest.raises(RuntimeError):
        dc.rank_bytes(P)
    dc.close()
