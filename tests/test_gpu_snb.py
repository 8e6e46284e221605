"""The objective for 128 < n <= 512 (gpemu_snb.hpp: one launch, a factor workgroup and
SNB_NH = 48 helper workgroups) against the oracle and against the general path of the same library
(GPEMU_TINY=0), for the variants the general path's golden tests cover: gp4ml / MUCM, std /
alt-nugget kernel with per-point r, fitted / fixed nugget, the std kernel's set_r sigma
gradient, 2 to 4 tiles with ragged last tiles, d from 1 to 30, q + 1 up to 32; a non-positive-
definite matrix and the calls after it; contexts sharing the GPU.  Tolerances as
tests/test_gpu_tiny.py."""
import threading

import numpy as np
import pytest

from gp_emu_uqsa_amd import native
from oracle import gp_oracle as orc

pytestmark = pytest.mark.gpu


def _grad_ok(g, gref, tol=1e-7):
    scale = np.abs(gref) + np.max(np.abs(gref))
    return np.all(np.abs(g - gref) <= tol * scale), np.max(np.abs(g - gref) / scale)


@pytest.fixture(scope="module")
def general():
    mp = pytest.MonkeyPatch()
    mp.setenv("GPEMU_TINY", "0")
    c = native.Context(0)
    mp.undo()
    yield c
    c.close()


CASES = [   # (variant, kernel, fit nugget, r)
    (orc.GP4ML, orc.STD, True, False),
    (orc.GP4ML, orc.STD, False, False),
    (orc.MUCM, orc.STD, True, False),
    (orc.MUCM, orc.STD, False, False),
    (orc.GP4ML, orc.ALT, True, True),
    (orc.GP4ML, orc.STD, True, True),
]


def _hp(d, variant, fitn, kind):
    hp = list(np.linspace(0.3, 0.9, d))
    if fitn:
        hp.append(3e-2 if kind == orc.ALT else 2e-3)
    if variant == orc.GP4ML:
        hp.append(1.2)
    return np.array(hp)


@pytest.mark.parametrize("n,d", [(129, 5), (200, 3), (256, 10), (300, 10), (384, 2), (500, 2), (512, 16), (450, 30)])
@pytest.mark.parametrize("case", CASES, ids=["gp4ml_fit", "gp4ml_fix", "mucm_fit", "mucm_fix", "alt_r", "std_r"])
def test_snb_matches_oracle_and_general(ctx, general, n, d, case):
    variant, kind, fitn, use_r = case
    X, f, H = orc.synthetic_problem(n, d, seed=n + d)
    r = np.random.RandomState(n).uniform(1e-4, 1e-3, size=n) if use_r else None
    hp = _hp(d, variant, fitn, kind)
    nu_fixed = 5e-3 if not fitn else 0.0
    ctx.set_data(X, f, H, r)
    general.set_data(X, f, H, r)
    llh, g, s2 = ctx.objective(variant, kind, hp, nu_fixed=nu_fixed)
    v, _, vs2 = ctx.objective(variant, kind, hp, nu_fixed=nu_fixed, want_grad=False)
    ref = orc.objective_fast(X, f, H, hp, variant, kind, fitn, r=r, nu_fixed=nu_fixed)
    assert abs(llh - ref[0]) <= 1e-10 * max(1.0, abs(ref[0])), (llh, ref[0])
    assert abs(v - llh) <= 1e-12 * max(1.0, abs(llh)) and abs(vs2 - s2) <= 1e-12 * s2
    assert abs(s2 - ref[2]) <= 1e-10 * ref[2]
    ok, err = _grad_ok(g, ref[1])
    assert ok, (err, g, ref[1])
    gl, gg, gs2 = general.objective(variant, kind, hp, nu_fixed=nu_fixed)
    assert abs(llh - gl) <= 1e-11 * max(1.0, abs(gl)), (llh, gl)
    assert np.max(np.abs(g - gg)) <= 1e-9 * (1.0 + np.max(np.abs(gg))), (g, gg)
    assert abs(s2 - gs2) <= 1e-11 * gs2


def test_snb_wide_basis(ctx):
    """q + 1 = 32 basis columns (two 16-column blocks of the augmented row) at n = 300."""
    X, f, H = orc.synthetic_problem(300, 31, seed=5)
    ctx.set_data(X, f, H)
    hp = _hp(31, orc.GP4ML, True, orc.STD)
    llh, g, _ = ctx.objective(orc.GP4ML, orc.STD, hp)
    ref = orc.objective_fast(X, f, H, hp, orc.GP4ML, orc.STD, True)
    assert abs(llh - ref[0]) <= 1e-10 * abs(ref[0])
    ok, err = _grad_ok(g, ref[1])
    assert ok, err


def test_snb_not_pd_then_usable(ctx):
    """A non-positive-definite 300-point matrix (duplicated points, nugget -1) is reported;
    the next calls (value, gradient, the resident factor) are right."""
    X, f, H = orc.synthetic_problem(290, 2, seed=3)
    X = np.vstack([X, X[:10]])
    f = np.concatenate([f, f[:10]])
    H = orc.linear_basis(X)
    ctx.set_data(X, f, H)
    with pytest.raises(native.NotPositiveDefinite):
        ctx.objective(orc.GP4ML, orc.STD, np.array([0.5, 0.5, 1.0]), nu_fixed=-1.0)
    hp = np.array([0.5, 0.6, 1e-2, 1.0])
    for want in (False, True, True):
        llh, g, _ = ctx.objective(orc.GP4ML, orc.STD, hp, want_grad=want)
        ref = orc.objective_fast(X, f, H, hp, orc.GP4ML, orc.STD, True)
        assert abs(llh - ref[0]) <= 1e-10 * abs(ref[0])
        if want:
            ok, err = _grad_ok(g, ref[1])
            assert ok, err
    ctx.factor(native.KERNEL_STD, hp[:2], hp[2], 1.0, 0.0)
    beta = ctx.beta()
    A, _ = orc.kernel_var_ref(X, hp[:2], hp[2], orc.STD, True)
    assert np.max(np.abs(beta - orc.optimal_beta_ref(A, H, f))) <= 1e-8 * (1 + np.max(np.abs(beta)))


def test_snb_concurrent_contexts():
    """Two contexts on two threads (n = 300 and n = 500) and one on the n <= 128 path share
    the GPU; 30 mixed gradient / value calls each equal the same call run alone."""
    probs = [orc.synthetic_problem(n, d, seed=s) for n, d, s in ((300, 10, 41), (500, 2, 42), (100, 3, 43))]
    hps = [np.concatenate([np.linspace(0.4, 0.8, d), [1e-3, 1.1]]) for d in (10, 2, 3)]
    ctxs = [native.Context(0) for _ in range(3)]
    th = []
    try:
        alone = []
        for c, (X, f, H), hp in zip(ctxs, probs, hps):
            c.set_data(X, f, H)
            alone.append((c.objective(orc.GP4ML, orc.STD, hp), c.objective(orc.GP4ML, orc.STD, hp, want_grad=False)))
        errors = []

        def run(k):
            try:
                for it in range(30):
                    want = it % 3 != 2
                    llh, g, _ = ctxs[k].objective(orc.GP4ML, orc.STD, hps[k], want_grad=want)
                    ref = alone[k][0] if want else alone[k][1]
                    if llh != ref[0] or (want and not np.array_equal(g, ref[1])):
                        errors.append((k, it, llh, ref[0]))
            except Exception as e:   # noqa: BLE001 (reported below)
                errors.append((k, repr(e)))

        th = [threading.Thread(target=run, args=(k,)) for k in range(3)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=120)
        assert not any(t.is_alive() for t in th), "a context did not finish"
        assert not errors, errors[:5]
    finally:
        for k, c in enumerate(ctxs):
            if k >= len(th) or not th[k].is_alive():
                c.close()
