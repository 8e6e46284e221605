"""GPU posterior mean/variance vs the reference's reconstructed emulators (G3).
North-star tolerance: posterior mean within 1e-8 of SciPy (absolute)."""
import os

import numpy as np
import pytest

from oracle import gp_oracle as orc

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.mark.parametrize("tag", ["toysim", "toysim3d_o0", "toysim3d_o1"])
@pytest.mark.parametrize("full", [True, False])
def test_posterior_golden(ctx, tag, full):
    z = np.load(os.path.join(GOLD, f"posterior_{tag}.npz"))
    kind = orc.ALT if bool(z["alt"]) else orc.STD
    ctx.set_data(z["XT"], z["fT"], z["HT"])
    ctx.factor(kind, z["delta"], float(z["nu"]), 1.0, 0.0)
    Hs = np.hstack([np.ones((z["xs"].shape[0], 1)), z["xs"]])[:, :z["HT"].shape[1]]
    mean, var = ctx.posterior(z["xs"], Hs, z["beta"], float(z["sigma"]), full_var=full)
    assert np.max(np.abs(mean - z["mean"])) < 1e-8
    vref = z["var"] if full else np.diag(z["var"])
    assert np.max(np.abs(var - vref)) < 1e-8 * max(1.0, np.max(np.abs(vref)))


@pytest.mark.parametrize("tag", ["toysim", "toysim3d_o0"])
def test_beta_golden(ctx, tag):
    z = np.load(os.path.join(GOLD, f"posterior_{tag}.npz"))
    kind = orc.ALT if bool(z["alt"]) else orc.STD
    ctx.set_data(z["XT"], z["fT"], z["HT"])
    ctx.factor(kind, z["delta"], float(z["nu"]), 1.0, 0.0)
    assert np.max(np.abs(ctx.beta() - z["beta_opt"])) < 1e-9 * (1 + np.max(np.abs(z["beta_opt"])))


@pytest.mark.parametrize("kind", [orc.STD, orc.ALT])
def test_kernel_var_covar_golden(ctx, kind):
    z = np.load(os.path.join(GOLD, "kernel_std.npz" if kind == orc.STD else "kernel_alt.npz"))
    for pred, key in ((True, "A_pred"), (False, "A_est")):
        A = ctx.kernel_var(kind, z["delta"], float(z["nu"]), z["X"], predict=pred)
        assert np.max(np.abs(A - z[key])) < 1e-15 * 4
    C = ctx.kernel_covar(kind, z["delta"], float(z["nu"]), z["X"], z["Xs"])
    assert np.max(np.abs(C - z["covar"])) < 1e-15 * 4


def test_posterior_large_m_chunked(ctx):
    X, f, H = orc.synthetic_problem(700, 3, seed=4)
    ctx.set_data(X, f, H)
    delta, nu = np.array([0.5, 0.6, 0.7]), 1e-3
    ctx.factor(orc.STD, delta, nu, 1.0, 0.0)
    beta = ctx.beta()
    xs = np.random.RandomState(1).uniform(size=(9000, 3))
    hs = orc.linear_basis(xs)
    mean, var = ctx.posterior(xs, hs, beta, 0.8, full_var=False)
    A, _ = orc.kernel_var_ref(X, delta, nu, orc.STD, True)
    sel = np.arange(0, 9000, 97)
    m_ref, v_ref = orc.posterior_ref(X, f, H, A, xs[sel], hs[sel], beta, 0.8, delta, nu, orc.STD)
    assert np.max(np.abs(mean[sel] - m_ref)) < 1e-8
    assert np.max(np.abs(var[sel] - np.diag(v_ref))) < 1e-8


@pytest.mark.parametrize("oz", ["1", "0"])
def test_posterior_precision32_diagonal(monkeypatch, oz):
    """precision 32 (config C5): L^-1 K* as exact int8 products of 24-bit operands (8 moduli,
    posterior_oz), or with GPEMU_OZAKI=0 on fp32 MFMA.  The mean is fp64 and must equal the
    fp64 path; the diagonal variance sigma^2 (1 - |L^-1 k*|^2 + ...) loses ~fp32 eps *
    |L^-1 k*|^2 to cancellation, tolerance 2e-5 * sigma^2."""
    from gp_emu_uqsa_amd import native, synthetic
    monkeypatch.setenv("GPEMU_OZAKI", oz)
    monkeypatch.setenv("GPEMU_OZAKI_MIN_NP", "2048")   # (the int8 product's default start: 4096)
    ctx = native.Context(0)
    X, f, H = synthetic.problem(2000, 6, seed=3)
    ctx.set_data(X, f, H)
    delta = np.full(6, 0.8)
    ctx.factor(native.KERNEL_STD, delta, 1e-3, 1.0, 0.0)
    beta = ctx.beta()
    xs = synthetic.design(10000, 6, seed=9)
    hs = synthetic.linear_basis(xs)
    m64, v64 = ctx.posterior(xs, hs, beta, 0.9, full_var=False, precision=64)
    m32, v32 = ctx.posterior(xs, hs, beta, 0.9, full_var=False, precision=32)
    assert np.array_equal(m32, m64)
    assert np.max(np.abs(v32 - v64)) < 2e-5 * 0.81, np.max(np.abs(v32 - v64))
    with pytest.raises(RuntimeError):
        ctx.posterior(xs[:10], hs[:10], beta, 0.9, full_var=True, precision=32)
    ctx.close()


def test_posterior_int8_matches_fp64(monkeypatch):
    """V = L^-1 K* on the int8 cores (posterior_oz, started from n_pad 2048 here) against the fp64 k_gemm
    product (GPEMU_OZAKI=0) and the oracle: precision 64 (16 moduli, 53-bit operands) to
    1e-11 sigma^2 in the diagonal and in the full covariance, precision 32 (8 moduli, 24-bit
    operands) to 4e-6 sigma^2, below the fp32 GEMM's own error on these inputs; ragged n (2200: 9 tiles of 256) and chunks (9000 points: a full
    8192-point chunk and a ragged one)."""
    from gp_emu_uqsa_amd import native, synthetic
    n, d, s2 = 2200, 5, 0.9 ** 2
    X, f, H = synthetic.problem(n, d, seed=5)
    delta = np.full(d, 0.7)
    xs = synthetic.design(9000, d, seed=8)
    hs = synthetic.linear_basis(xs)
    out = {}
    monkeypatch.setenv("GPEMU_OZAKI_MIN_NP", "2048")   # (the int8 product's default start: 4096)
    for oz in ("0", "1"):
        monkeypatch.setenv("GPEMU_OZAKI", oz)
        c = native.Context(0)
        c.set_data(X, f, H)
        c.factor(native.KERNEL_STD, delta, 1e-3, 1.0, 0.0)
        beta = c.beta()
        out[oz] = (c.posterior(xs, hs, beta, 0.9, full_var=False, precision=64),
                   c.posterior(xs, hs, beta, 0.9, full_var=False, precision=32),
                   c.posterior(xs[:300], hs[:300], beta, 0.9, full_var=True, precision=64), beta)
        c.close()
    (m0, v0), _, (mf0, vf0), beta = out["0"]
    (m1, v1), (m132, v132), (mf1, vf1), _ = out["1"]
    assert np.array_equal(m1, m0) and np.array_equal(m132, m0)
    assert np.max(np.abs(v1 - v0)) < 1e-11 * s2, np.max(np.abs(v1 - v0))
    # (the fp32 GEMM, GPEMU_OZAKI=0, is 7.9e-6 off on these inputs: tools/post_err_r06.py)
    assert np.max(np.abs(v132 - v0)) < 4e-6 * s2, np.max(np.abs(v132 - v0))
    assert np.max(np.abs(vf1 - vf0)) < 1e-11 * s2, np.max(np.abs(vf1 - vf0))
    A, _ = orc.kernel_var_ref(X, delta, 1e-3, orc.STD, True)
    sel = np.arange(0, 9000, 450)
    m_ref, v_ref = orc.posterior_ref(X, f, H, A, xs[sel], hs[sel], beta, 0.9, delta, 1e-3, orc.STD)
    assert np.max(np.abs(m1[sel] - m_ref)) < 1e-8
    assert np.max(np.abs(v1[sel] - np.diag(v_ref))) < 1e-8


def test_posterior_int8_nan_point(monkeypatch):
    """A NaN prediction point gives a NaN mean and variance on the int8 product as on the fp64 one
    (its K* row gets the OZ_EX_NAN exponent: zero planes, NaN out of the CRT), and leaves every
    other point's variance as it is without it."""
    from gp_emu_uqsa_amd import native, synthetic
    n, d, s2 = 2200, 5, 0.9 ** 2
    X, f, H = synthetic.problem(n, d, seed=5)
    delta = np.full(d, 0.7)
    xs = synthetic.design(600, d, seed=8)
    xs[17, 2] = np.nan
    hs = synthetic.linear_basis(xs)
    monkeypatch.setenv("GPEMU_OZAKI_MIN_NP", "2048")
    out = {}
    for oz in ("0", "1"):
        monkeypatch.setenv("GPEMU_OZAKI", oz)
        c = native.Context(0)
        c.set_data(X, f, H)
        c.factor(native.KERNEL_STD, delta, 1e-3, 1.0, 0.0)
        beta = c.beta()
        out[oz] = [c.posterior(xs, hs, beta, 0.9, full_var=False, precision=p) for p in (64, 32)]
        c.close()
    ok = np.ones(600, bool)
    ok[17] = False
    for p in range(2):
        for oz in ("0", "1"):
            m, v = out[oz][p]
            assert np.isnan(m[17]) and np.isnan(v[17]), (oz, p)
            assert np.all(np.isfinite(m[ok])) and np.all(np.isfinite(v[ok])), (oz, p)
    (m0, v0), (m1, v1) = out["0"][0], out["1"][0]
    assert np.max(np.abs(v1[ok] - v0[ok])) < 1e-11 * s2
    assert np.array_equal(m1[ok], m0[ok])


@pytest.mark.parametrize("kind", [orc.STD, orc.ALT])
def test_kernel_gradients_golden(kind):
    """kernel.grad_delta_A / grad_nugget_A through the kernel objects (gpe_kernel_grad)
    against the reference's own matrices (G1): exp_save from the preceding var()."""
    from gp_emu_uqsa_amd import kernels

    z = np.load(os.path.join(GOLD, "kernel_std.npz" if kind == orc.STD else "kernel_alt.npz"))

    class Par:
        delta = z["delta"]
        nugget = float(z["nu"])

    K = (kernels.kernel if kind == orc.STD else kernels.kernel_alt_nug)(3, Par)
    X, s2 = z["X"], float(z["s2"])
    with pytest.raises(AttributeError):
        K.grad_delta_A(X[:, 0], 0, s2)          # no var() yet: the reference has no exp_save
    K.var(X, False)
    for i in range(3):
        G = K.grad_delta_A(X[:, i], i, s2)
        ref = z["grad_delta"][i]
        assert np.max(np.abs(G - ref)) <= 1e-14 * np.max(np.abs(ref)), i
    Gn = K.grad_nugget_A(X, s2)
    refn = z["grad_nugget"]
    assert np.max(np.abs(Gn - refn)) <= 1e-14 * np.max(np.abs(refn))


def test_posterior_int8_full_covariance_two_chunks(monkeypatch):
    """The full posterior covariance beyond one chunk (m = 16500: two 16384-point chunks whose V
    = L^-1 K* the int8 product writes into the device-resident V of all points, then the m x m
    blocks) at n_pad = 4224 (the int8 product's default range), against GPEMU_OZAKI=0."""
    from gp_emu_uqsa_amd import native, synthetic
    n, d, m = 4100, 3, 16500
    X, f, H = synthetic.problem(n, d, seed=21)
    xs = synthetic.design(m, d, seed=22)
    hs = synthetic.linear_basis(xs)
    out = {}
    for oz in ("0", "1"):
        monkeypatch.setenv("GPEMU_OZAKI", oz)
        c = native.Context(0)
        c.set_data(X, f, H)
        c.factor(native.KERNEL_STD, np.full(d, 0.5), 1e-3, 1.0, 0.0)
        beta = c.beta()
        out[oz] = c.posterior(xs, hs, beta, 0.9, full_var=True)
        c.close()
    (m0, v0), (m1, v1) = out["0"], out["1"]
    assert np.array_equal(m0, m1)
    err = float(np.max(np.abs(v1 - v0)))
    del out, v0, v1
    assert err < 1e-11 * 0.81, err
