"""The objective for n <= 128 (gpemu_tiny.hpp: two one-workgroup launches) against the
oracle and against the general path of the same library (GPEMU_TINY=0), for every
variant the general path's golden tests cover: gp4ml / MUCM, std / alt-nugget kernel with
per-point r, fitted / fixed nugget, the std kernel's set_r sigma gradient, d = 1 .. 30 and
q + 1 up to 32 basis columns (the tiny path's limits; one past them the general path
runs), ragged n down to 5, a non-positive-definite matrix, and the resident-factor calls
after it.  Tolerances as tests/test_gpu_objective.py: LLH 1e-10 relative, gradient
|g - g_ref| <= 1e-7 (|g_ref| + max|g_ref|); tiny against general path 1e-11 / 1e-9 (the
sums over rows run in another order than the MFMA GEMMs')."""
import os

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
    """A context on the general path (GPEMU_TINY=0 is read when the context is created)."""
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


@pytest.mark.parametrize("n,d", [(60, 2), (100, 3), (128, 10), (97, 1), (128, 30), (40, 16), (5, 1), (80, 6)])
@pytest.mark.parametrize("case", CASES, ids=["gp4ml_fit", "gp4ml_fix", "mucm_fit", "mucm_fix", "alt_r", "std_r"])
def test_tiny_matches_oracle_and_general(ctx, general, n, d, case):
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


def test_tiny_toysim_example(ctx):
    """The reference's toy-sim example data (60 points, d = 2, scaled to [0, 1] as setup()
    does) against the op-for-op oracle (objective_ref, pinned to the reference's G2)."""
    ex = os.path.join(os.path.dirname(__file__), "golden", "examples", "toy-sim")
    X = np.loadtxt(os.path.join(ex, "toy-sim_input"))
    y = np.loadtxt(os.path.join(ex, "toy-sim_output"))
    X = (X - X.min(0)) / (X.max(0) - X.min(0))
    H = np.hstack([np.ones((X.shape[0], 1)), X])
    ctx.set_data(X, y, H)
    for hp in ([0.4, 0.7, 1e-3, 1.1], [1.5, 0.2, 1e-2, 0.6]):
        hp = np.array(hp)
        llh, g, _ = ctx.objective(orc.GP4ML, orc.STD, hp)
        ref = orc.objective_ref(X, y, H, hp, orc.GP4ML, orc.STD, True)
        assert abs(llh - ref[0]) <= 1e-10 * abs(ref[0]), (llh, ref[0])
        ok, err = _grad_ok(g, ref[1])
        assert ok, err


@pytest.mark.parametrize("n,d", [(128, 31), (129, 3)])
def test_past_the_tiny_limits(ctx, n, d):
    """q + 1 = 33 basis columns and n = 129 take the general path: still right."""
    X, f, H = orc.synthetic_problem(n, d, seed=7)
    ctx.set_data(X, f, H)
    hp = _hp(d, orc.GP4ML, True, orc.STD)
    llh, g, _ = ctx.objective(orc.GP4ML, orc.STD, hp)
    ref = orc.objective_fast(X, f, H, hp, orc.GP4ML, orc.STD, True)
    assert abs(llh - ref[0]) <= 1e-10 * abs(ref[0])
    ok, err = _grad_ok(g, ref[1])
    assert ok, err


def test_tiny_not_pd_then_usable(ctx):
    """A non-positive-definite matrix (duplicated points with nugget -1: off-diagonal 2 s2
    against s2 on the diagonal) is reported, the context
    stays usable, and the resident-factor calls (gpe_factor, beta, posterior) run after a
    tiny-path objective."""
    X, f, H = orc.synthetic_problem(50, 2, seed=3)
    X = np.vstack([X, X[:5]])
    f = np.concatenate([f, f[:5]])
    H = orc.linear_basis(X)
    ctx.set_data(X, f, H)
    with pytest.raises(native.NotPositiveDefinite):
        ctx.objective(orc.GP4ML, orc.STD, np.array([0.5, 0.5, 1.0]), nu_fixed=-1.0)
    hp = np.array([0.5, 0.6, 1e-2, 1.0])
    llh, g, _ = ctx.objective(orc.GP4ML, orc.STD, hp)
    ref = orc.objective_fast(X, f, H, hp, orc.GP4ML, orc.STD, True)
    assert abs(llh - ref[0]) <= 1e-10 * abs(ref[0])
    ctx.factor(native.KERNEL_STD, hp[:2], hp[2], 1.0, 0.0)
    beta = ctx.beta()
    A, _ = orc.kernel_var_ref(X, hp[:2], hp[2], orc.STD, True)
    assert np.max(np.abs(beta - orc.optimal_beta_ref(A, H, f))) <= 1e-8 * (1 + np.max(np.abs(beta)))
    xs = np.random.RandomState(1).uniform(size=(9, 2))
    mean, var = ctx.posterior(xs, orc.linear_basis(xs), beta, hp[-1], full_var=True)
    m_ref, v_ref = orc.posterior_ref(X, f, H, A, xs, orc.linear_basis(xs), beta, hp[-1], hp[:2], hp[2], orc.STD)
    assert np.max(np.abs(mean - m_ref)) < 1e-8 and np.max(np.abs(var - v_ref)) < 1e-8


def test_tiny_concurrent_contexts_and_big_neighbour():
    """Three contexts on three threads, each with its own stream: two run n <= 128 objectives
    (the one-launch path's cross-workgroup hand-offs then share the GPU with each other) and
    one an n = 4096 objective beside them (uneven load); every result equals the same call
    run alone, and the sync words stay consistent over 40 mixed gradient / value calls."""
    import threading
    probs = [orc.synthetic_problem(n, d, seed=s) for n, d, s in ((128, 10, 31), (77, 3, 32), (4096, 10, 33))]
    hps = [np.concatenate([np.linspace(0.4, 0.8, d), [1e-3, 1.1]]) for d in (10, 3, 10)]
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
                reps = 4 if k == 2 else 40
                for it in range(reps):
                    want = it % 3 != 2
                    llh, g, s2 = ctxs[k].objective(orc.GP4ML, orc.STD, hps[k], want_grad=want)
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
        for k, c in enumerate(ctxs):   # (a context still in use by its thread stays open)
            if k >= len(th) or not th[k].is_alive():
                c.close()
