"""Edge cases at the C-ABI and host API: one input dimension, single prediction
points, NaN hyperparameters (the reference's LinAlgError -> `return None` path),
the documented argument limits."""
import numpy as np
import pytest

from gp_emu_uqsa_amd import native
from oracle import gp_oracle as orc

pytestmark = pytest.mark.gpu


def test_one_dimension_objective_and_posterior(ctx):
    rs = np.random.RandomState(2)
    X = rs.uniform(size=(150, 1))
    f = np.sin(6 * X[:, 0]) + 0.01 * rs.randn(150)
    H = orc.linear_basis(X)
    hp = np.array([0.3, 1e-2, 0.9])
    ctx.set_data(X, f, H)
    llh, g, _ = ctx.objective(native.GP4ML, native.KERNEL_STD, hp)
    ref = orc.objective_ref(X, f, H, hp, orc.GP4ML, orc.STD, True)
    assert abs(llh - ref[0]) <= 1e-9 * abs(ref[0])
    assert np.max(np.abs(g - ref[1])) <= 1e-7 * (np.max(np.abs(ref[1])) + 1.0)
    ctx.factor(native.KERNEL_STD, hp[:1], hp[1], 1.0, 0.0)
    beta = ctx.beta()
    xs = np.array([[0.37]])
    mean, var = ctx.posterior(xs, orc.linear_basis(xs), beta, hp[-1], full_var=True)
    A, _ = orc.kernel_var_ref(X, hp[:1], hp[1], orc.STD, True)
    m_ref, v_ref = orc.posterior_ref(X, f, H, A, xs, orc.linear_basis(xs), beta, hp[-1], hp[:1], hp[1],
                                     orc.STD)
    assert mean.shape == (1,) and var.shape == (1, 1)
    assert abs(mean[0] - m_ref[0]) < 1e-8 and abs(var[0, 0] - v_ref[0, 0]) < 1e-8


def test_nan_hyperparameter_is_not_pd(ctx):
    X, f, H = orc.synthetic_problem(200, 3, seed=1)
    ctx.set_data(X, f, H)
    with pytest.raises(native.NotPositiveDefinite):
        ctx.objective(native.GP4ML, native.KERNEL_STD, np.array([0.5, np.nan, 0.7, 1e-2, 1.0]))
    # the context stays usable
    llh, _, _ = ctx.objective(native.GP4ML, native.KERNEL_STD, np.array([0.5, 0.6, 0.7, 1e-2, 1.0]))
    assert np.isfinite(llh)


def _wide_problem(n, d, seed):
    rs = np.random.RandomState(seed)
    X = rs.uniform(size=(n, d))
    f = np.sin(X @ rs.normal(size=d) / np.sqrt(d)) + 0.01 * rs.normal(size=n)
    return X, f, orc.linear_basis(X)


def test_any_d_and_basis_width(ctx):
    """No input-dimension or basis-width limit, as in the reference
    (_emulatorkernels.py:39-50 takes any d): d = 150 inputs with the linear mean's
    151 basis columns, beyond the 128 the context's small buffers start at
    (GPE_MAX_DIMS / GPE_MAX_COLS, include/gpemu.h).  Value, gradient and sigma^2
    against the oracle (the value path without the augmented row, which holds 128
    columns), then the kernel matrix at d = 129, and the row-block path (2 and 3 loopback
    ranks) with all 151 basis columns: [f H]^T rides in two augmented tile rows there,
    owned by different ranks."""
    n, d = 400, 150
    X, f, H = _wide_problem(n, d, seed=8)
    hp = np.concatenate([np.linspace(2.5, 4.0, d), [1e-2, 0.9]])
    ctx.set_data(X, f, H)
    llh, g, s2 = ctx.objective(native.GP4ML, native.KERNEL_STD, hp)
    ref = orc.objective_fast(X, f, H, hp, orc.GP4ML, orc.STD, True)
    assert abs(llh - ref[0]) <= 1e-10 * abs(ref[0]), (llh, ref[0])
    scale = np.max(np.abs(ref[1])) + 1.0
    assert np.max(np.abs(g - ref[1])) <= 1e-7 * scale, np.max(np.abs(g - ref[1]))
    v = ctx.objective(native.GP4ML, native.KERNEL_STD, hp, want_grad=False)[0]
    assert abs(v - ref[0]) <= 1e-10 * abs(ref[0])
    X2 = np.random.RandomState(9).uniform(size=(50, 129))
    A = ctx.kernel_var(native.KERNEL_STD, np.full(129, 3.0), 1e-3, X2)
    Aref, _ = orc.kernel_var_ref(X2, np.full(129, 3.0), 1e-3, orc.STD, True)
    assert np.max(np.abs(A - Aref)) <= 1e-13
    for P in (2, 3):
        dc = native.DistContext(0, P)
        try:
            dc.set_data(X, f, H)
            llh_d, g_d, s2_d = dc.objective(native.GP4ML, native.KERNEL_STD, hp, want_grad=True)
            v_d = dc.objective(native.GP4ML, native.KERNEL_STD, hp)[0]
        finally:
            dc.close()
        assert abs(llh_d - ref[0]) <= 1e-10 * abs(ref[0]), (P, llh_d, ref[0])
        assert v_d == llh_d
        assert np.max(np.abs(g_d - ref[1])) <= 1e-7 * scale, (P, np.max(np.abs(g_d - ref[1])))


def test_noise_sample_single_point(ctx):
    rs = np.random.RandomState(3)
    X = rs.uniform(size=(80, 2))
    f = np.cos(3 * X[:, 0])
    ctx.set_data(X, f, np.ones((80, 1)))
    ctx.factor(native.KERNEL_STD, np.array([0.4, 0.5]), 1e-3, 1.0, 0.0)
    xs = np.array([[0.2, 0.3]])
    U = rs.randn(7, 1)
    mean, z = ctx.noise_sample(xs, np.ones((1, 1)), np.array([0.1]), 0.8, np.array([0.5]), U)
    _, V = ctx.posterior(xs, np.ones((1, 1)), np.array([0.1]), 0.8, full_var=True)
    ref = np.sum(0.5 * (0.5 - mean[0] - np.sqrt(V[0, 0]) * U[:, 0]) ** 2)
    assert abs(z[0] - ref) <= 1e-12 * abs(ref)
