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


def _oz_bytes(nb, P, nmod=16):
    """The int8 A^-1 partial's buffers (gpemu_dist.hip oz_prepare, shared by the loopback
    ranks): nmod planes of X_r^T (np2 x rank 0's rows) and nmod residue images of the largest
    slab's 256-tiles (slabs of an even number of tile rows)."""
    np_ = nb * 128
    if np_ < 6144:   # (the int8 partial's default start)
        return 0
    np2 = -(-np_ // 256) * 256
    kp = ((nb - 1) // P + 1) * 128
    whole = nb * 128 * np_
    sd = 1 << 26
    if whole <= 4 * sd:
        sd = max(sd, whole // P)
    sr = max(1, min(nb, sd // (128 * np_)))
    if sr < nb and sr % 2:
        sr = max(2, sr - 1)
    tri = lambda t: t * (t + 1) // 2
    maxt = max(tri((min(nb, a0 + sr) + 1) // 2) - tri(a0 // 2) for a0 in range(0, nb, sr))
    return nmod * np2 * kp + nmod * maxt * 256 * 256 + 4 * np2 + (1 << 20)


@pytest.mark.parametrize("n,P", [(4000, 2), (4000, 3), (10240, 4)])
def test_loopback_rank_memory(n, P):
    """Each logical rank holds its own tile rows (of A and, after a gradient call, of
    L^-1): the per-rank bytes follow the partition, not n^2.  Upper bound after the
    gradient: its rows of L^-1 plus at most three slab-sized buffers (the A^-1 partial's
    slab, the TRTRI's gathered X11 and all-gather buffer), the slab being the whole
    triangle's tile rows / P (at least 512 MiB, at most the whole) -- at n = 10240, P = 4
    one n x n partial per rank (the round-4 slab) would exceed it; plus the int8 partial's
    planes and residues (_oz_bytes)."""
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
        assert grad[r] - val[r] <= xrows + 3 * slab + _oz_bytes(nb, P) + (64 << 20), (grad[r] - val[r], xrows, slab)
    with pytest.raises(RuntimeError):
        dc.rank_bytes(P)
    dc.close()


@pytest.mark.parametrize("P,slab_mb", [(1, None), (2, None), (3, 16), (5, 1)])
def test_loopback_int8_partial_matches_fp64(monkeypatch, P, slab_mb):
    """The rank partials of A^-1 on the int8 cores (gpemu_dist.hip oz_slab: each rank's
    X_r^T X_r from its own rows, K from the first nonzero local row of each 256-column block)
    against the same context type with GPEMU_OZAKI=0 (fp64 k_gemm slabs): the LLH equal (it
    does not depend on A^-1), the gradient to 1e-10 of scale.  n = 3000 / 2900 pad to 24 / 23
    tile rows (the last 256-tile half past n_pad); slabs of 16 and 1 MiB (5 tile rows, rounded to 4; 1 row, raised to 2)
    split the partial into 6 and 12 slabs; against the oracle to the suite's 1e-7.  At P = 1
    the top TRTRI levels run on the int8 cores too (GPEMU_OZAKI_TRI_MIN lowered)."""
    n, d = (2900 if P == 3 else 3000), 5   # 23 / 24 tile rows
    X, f, H = orc.synthetic_problem(n, d, seed=17)
    r = np.random.RandomState(3).uniform(1e-4, 1e-3, size=n)
    hp = _hp(d)
    if slab_mb:
        monkeypatch.setenv("GPEMU_DIST_SLAB_MB", str(slab_mb))
    monkeypatch.setenv("GPEMU_OZAKI_MIN_NP", "2048")   # (default start 6144)
    # P = 1: the TRTRI levels of blocks >= 1024 rows on the int8 cores as well (pairs
    # (0, 8, 16) and (0, 16, 24) at 24 tile rows: a ragged second block)
    monkeypatch.setenv("GPEMU_OZAKI_TRI_MIN", "1024")
    out = {}
    for oz in ("0", "1"):
        monkeypatch.setenv("GPEMU_OZAKI", oz)
        dc = native.DistContext(0, P)
        dc.set_data(X, f, H, r)
        out[oz] = dc.objective(native.GP4ML, native.KERNEL_ALT_NUG, hp, want_grad=True)
        dc.close()
    (l0, g0, _), (l1, g1, _) = out["0"], out["1"]
    assert l1 == l0
    scale = np.abs(g0) + np.max(np.abs(g0))
    assert np.max(np.abs(g1 - g0) / scale) <= 1e-10, (g1, g0)
    ref = orc.objective_fast(X, f, H, hp, orc.GP4ML, orc.ALT, True, r=r)
    ok, err = _grad_ok(g1, ref[1])
    assert ok, err


def test_loopback_fused_next_factor_bit_identical(monkeypatch):
    """GPEMU_DIST_FUSE_NEXT=1 (P = 1: each group's first factor inside the update launch
    before it, on tile counts) changes the launches, not the arithmetic: LLH and gradient
    bit-identical to the default schedule, for a ragged n with 4-wide groups to the end."""
    n, d = 2500, 4
    X, f, H = orc.synthetic_problem(n, d, seed=23)
    hp = _hp(d)
    out = []
    for fz in ("0", "1"):
        monkeypatch.setenv("GPEMU_DIST_FUSE_NEXT", fz)
        dc = native.DistContext(0, 1)
        dc.set_data(X, f, H)
        out.append(dc.objective(native.GP4ML, native.KERNEL_STD, hp, want_grad=True))
        dc.close()
    assert out[0][0] == out[1][0]
    assert np.array_equal(out[0][1], out[1][1])
