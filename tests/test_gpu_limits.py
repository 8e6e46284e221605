"""Shapes beyond the register-resident kernels (the reference takes any d and any
basis, _emulatorkernels.py:39-50, _emulatorclasses.py:263-317, and forms the full
m x m posterior covariance for any m, :618-631):

- d = 40 inputs with the linear mean (q = 41, so [f H] has 42 columns): the K-build,
  contraction, skinny products, Gram and q x q transforms run their chunked forms;
  objective (gp4ml / MUCM / alt-nugget with r), kernel pieces and posterior against the
  oracle; the row-block distributed objective on 2 loopback ranks;
- d = 3 with a 40-column polynomial basis (many basis columns, few inputs);
- sensitivity pair sums with p = 45 columns of Z (chunks of 32), and at d = 40 inputs
  (coordinates staged through LDS: k_sense_pairs_wide);
- the full posterior covariance at m = 16384 + 300 points (two chunks: its off-diagonal
  blocks are formed on the device and written to the host), against the oracle on
  points drawn from both chunks;
- noise_fit's estimation step (gpe_noise_sample) at m = 16384 + 500 points: the
  covariance is formed block by block in the factorisation workspace, factored and
  drawn from on the device (noise_fit.py:130-150 has no bound on m).
Tolerances as the small-d tests: LLH 1e-9 relative, gradient 1e-7 of (|g| + max|g|),
posterior 1e-8 absolute."""
import numpy as np
import pytest

from gp_emu_uqsa_amd import native
from oracle import gp_oracle as orc

pytestmark = pytest.mark.gpu


def _grad_ok(g, gref, tol=1e-7):
    scale = np.abs(gref) + np.max(np.abs(gref))
    return np.all(np.abs(g - gref) <= tol * scale), np.max(np.abs(g - gref) / scale)


def _wide_problem(n=600, d=40, seed=5):
    X, f, H = orc.synthetic_problem(n, d, seed=seed)
    return X, f, H


@pytest.mark.parametrize("variant,kind,use_r", [(orc.GP4ML, orc.STD, False), (orc.MUCM, orc.STD, False),
                                                (orc.GP4ML, orc.ALT, True)])
def test_objective_d40(ctx, variant, kind, use_r):
    X, f, H = _wide_problem()
    d = X.shape[1]
    assert H.shape[1] == d + 1
    r = np.random.RandomState(3).uniform(1e-4, 1e-3, size=X.shape[0]) if use_r else None
    hp = np.concatenate([np.linspace(2.0, 4.0, d), [2e-3]] + ([[0.9]] if variant == orc.GP4ML else []))
    ctx.set_data(X, f, H, r)
    llh, g, s2 = ctx.objective(variant, kind, hp)
    ref = orc.objective_ref(X, f, H, hp, variant, kind, True, r)
    assert abs(llh - ref[0]) <= 1e-9 * abs(ref[0]), (llh, ref[0])
    ok, err = _grad_ok(g, ref[1])
    assert ok, err
    if variant == orc.MUCM:
        assert abs(s2 - ref[2]) <= 1e-9 * abs(ref[2])


def test_kernel_pieces_d40(ctx):
    X, f, H = _wide_problem(n=300)
    d = X.shape[1]
    delta = np.linspace(2.0, 4.0, d)
    ctx.set_data(X, f, H)
    A = ctx.kernel_var(native.KERNEL_STD, delta, 2e-3, X)
    Aref, _ = orc.kernel_var_ref(X, delta, 2e-3, orc.STD, True)
    assert np.max(np.abs(A - Aref)) <= 4e-15
    xv = np.random.RandomState(8).uniform(size=(70, d))
    C = ctx.kernel_covar(native.KERNEL_STD, delta, 2e-3, X, xv)
    assert np.max(np.abs(C - orc.kernel_covar_ref(X, xv, delta, 2e-3, orc.STD))) <= 4e-15


def test_posterior_d40(ctx):
    X, f, H = _wide_problem(n=500)
    d = X.shape[1]
    delta, nu, sigma = np.linspace(2.0, 4.0, d), 2e-3, 0.8
    ctx.set_data(X, f, H)
    ctx.factor(native.KERNEL_STD, delta, nu, 1.0, 0.0)
    beta = ctx.beta()
    A, _ = orc.kernel_var_ref(X, delta, nu, orc.STD, True)
    assert np.max(np.abs(beta - orc.optimal_beta_ref(A, H, f))) <= 1e-8 * (1 + np.max(np.abs(beta)))
    xs = np.random.RandomState(4).uniform(size=(40, d))
    hs = orc.linear_basis(xs)
    mean, var = ctx.posterior(xs, hs, beta, sigma, full_var=True)
    mref, vref = orc.posterior_ref(X, f, H, A, xs, hs, beta, sigma, delta, nu, orc.STD)
    assert np.max(np.abs(mean - mref)) < 1e-8 and np.max(np.abs(var - vref)) < 1e-8


def test_distributed_d40(ctx):
    X, f, H = _wide_problem(n=700)
    d = X.shape[1]
    hp = np.concatenate([np.linspace(2.0, 4.0, d), [2e-3, 0.9]])
    ctx.set_data(X, f, H)
    ref, gref, _ = ctx.objective(native.GP4ML, native.KERNEL_STD, hp)
    dc = native.DistContext(0, 2)
    dc.set_data(X, f, H)
    llh, g, _ = dc.objective(native.GP4ML, native.KERNEL_STD, hp, want_grad=True)
    dc.close()
    assert abs(llh - ref) <= 1e-10 * abs(ref)
    ok, err = _grad_ok(g, gref, 1e-8)
    assert ok, err


def test_many_basis_columns(ctx):
    rs = np.random.RandomState(6)
    n, d = 500, 3
    X = rs.uniform(size=(n, d))
    f = np.sin(4 * X[:, 0]) + X[:, 1] ** 2 + 0.01 * rs.randn(n)
    # a 40-column basis in the three inputs: 1, x_k, sin / cos(pi j x_k), j = 1..6
    cols = [np.ones(n)] + [X[:, k] for k in range(d)]
    for j in range(1, 7):
        for k in range(d):
            cols += [np.sin(np.pi * j * X[:, k]), np.cos(np.pi * j * X[:, k])]
    H = np.stack(cols, axis=1)
    assert H.shape[1] == 40
    hp = np.array([0.7, 0.8, 0.9, 1e-2, 1.1])
    ctx.set_data(X, f, H)
    llh, g, _ = ctx.objective(native.GP4ML, native.KERNEL_STD, hp)
    ref = orc.objective_ref(X, f, H, hp, orc.GP4ML, orc.STD, True)
    assert abs(llh - ref[0]) <= 1e-9 * abs(ref[0]), (llh, ref[0])
    ok, err = _grad_ok(g, ref[1])
    assert ok, err


def test_sense_pairs_many_columns(ctx):
    rs = np.random.RandomState(7)
    n, d = 400, 3
    X = rs.uniform(size=(n, d))
    f = np.cos(3 * X[:, 0])
    ctx.set_data(X, f, orc.linear_basis(X))
    delta, nu = np.array([0.5, 0.6, 0.7]), 1e-2
    ctx.factor(native.KERNEL_STD, delta, nu)
    Ainv = np.linalg.inv(orc.kernel_var_ref(X, delta, nu, orc.STD)[0])
    W = rs.uniform(0.0, 4.0, size=(2, d))
    U = rs.uniform(0.5, 1.5, size=(2, n))
    Z = rs.normal(size=(n, 45))
    tr, quad = ctx.sense_pairs(W, U, Z)
    for j in range(2):
        D = ((X[:, None, :] - X[None, :, :]) ** 2 * W[j]).sum(-1)
        K = U[j][:, None] * U[j][None, :] * np.exp(-D)
        assert abs(tr[j] - np.sum(Ainv * K)) <= 1e-9 * np.sum(np.abs(Ainv * K))
        np.testing.assert_allclose(quad[j], Z.T @ K @ Z, rtol=0, atol=1e-11 * np.abs(Z).sum(0).max() ** 2 * 2.25)


def test_full_covariance_beyond_one_chunk(ctx):
    n, d = 400, 3
    X, f, H = orc.synthetic_problem(n, d, seed=9)
    delta, nu, sigma = np.array([0.3, 0.4, 0.5]), 1e-3, 0.7
    ctx.set_data(X, f, H)
    ctx.factor(native.KERNEL_STD, delta, nu, 1.0, 0.0)
    beta = ctx.beta()
    m = 16384 + 300
    xs = np.random.RandomState(10).uniform(size=(m, d))
    hs = orc.linear_basis(xs)
    mean, var = ctx.posterior(xs, hs, beta, sigma, full_var=True)
    assert var.shape == (m, m)
    np.testing.assert_array_equal(var, var.T)
    sel = np.concatenate([np.arange(0, 16384, 211), np.arange(16384, m, 7)])
    A, _ = orc.kernel_var_ref(X, delta, nu, orc.STD, True)
    mref, vref = orc.posterior_ref(X, f, H, A, xs[sel], hs[sel], beta, sigma, delta, nu, orc.STD)
    assert np.max(np.abs(mean[sel] - mref)) < 1e-8
    assert np.max(np.abs(var[np.ix_(sel, sel)] - vref)) < 1e-8
    _, vdiag = ctx.posterior(xs, hs, beta, sigma, full_var=False)
    assert np.max(np.abs(np.diag(var) - vdiag)) < 1e-10


@pytest.mark.parametrize("p", [5, 12, 37])
def test_sense_pairs_d40(ctx, p):
    """gpe_sense_pairs beyond 32 input dimensions (sensitivity/_sensitivityclasses.py
    :599-626 takes any d): d = 40, Z widths in each column bucket and over a chunk."""
    rs = np.random.RandomState(11)
    n, d = 300, 40
    X = rs.uniform(size=(n, d))
    f = np.cos(3 * X[:, 0]) + X[:, 1]
    ctx.set_data(X, f, orc.linear_basis(X))
    delta, nu = np.linspace(2.0, 4.0, d), 1e-2
    ctx.factor(native.KERNEL_STD, delta, nu)
    Ainv = np.linalg.inv(orc.kernel_var_ref(X, delta, nu, orc.STD)[0])
    W = rs.uniform(0.0, 0.2, size=(3, d))
    U = rs.uniform(0.5, 1.5, size=(3, n))
    Z = rs.normal(size=(n, p))
    tr, quad = ctx.sense_pairs(W, U, Z)
    for j in range(3):
        D = ((X[:, None, :] - X[None, :, :]) ** 2 * W[j]).sum(-1)
        K = U[j][:, None] * U[j][None, :] * np.exp(-D)
        assert abs(tr[j] - np.sum(Ainv * K)) <= 1e-9 * np.sum(np.abs(Ainv * K))
        np.testing.assert_allclose(quad[j], Z.T @ K @ Z, rtol=0, atol=1e-11 * np.abs(Z).sum(0).max() ** 2 * 2.25)


def test_noise_sample_beyond_one_chunk(ctx):
    from oracle import noise_oracle as nor
    rs = np.random.RandomState(12)
    n, m, s = 300, 16384 + 500, 6
    x = rs.uniform(size=(n, 2))
    f = np.cos(3 * x[:, 0]) + x[:, 1] ** 2 + 0.1 * rs.randn(n)
    r = 0.01 + 0.05 * x[:, 1]
    delta, nu, sig, beta = np.array([0.3, 0.4]), 1e-3, 0.8, np.array([0.2])
    ctx.set_data(x, f, np.ones((n, 1)), r)
    ctx.factor(native.KERNEL_ALT_NUG, delta, nu, 1.0, 1.0)
    xs = rs.uniform(size=(m, 2))
    rn = 0.01 + 0.05 * xs[:, 1]
    t = rs.randn(m)
    U = rs.randn(s, m)
    mean, zsum = ctx.noise_sample(xs, np.ones((m, 1)), beta, sig, t, U, r_new=rn, r_scale=1.0 / sig ** 2)
    A, _ = orc.kernel_var_ref(x, delta, nu, orc.ALT, True)
    A[np.diag_indices(n)] += r
    mref, vref = nor.posterior_ref(x, f, np.ones((n, 1)), A, xs, np.ones((m, 1)), beta, sig, delta, nu,
                                   orc.ALT, rs_new=rn / sig ** 2)
    assert np.max(np.abs(mean - mref)) <= 1e-10 * (np.max(np.abs(mref)) + 1.0)
    zref = np.exp(nor.noise_estimate_ref(mref, vref, t, U)) * s
    assert np.max(np.abs(zsum - zref) / zref) <= 1e-8, np.max(np.abs(zsum - zref) / zref)
