"""GPU parity of the objective (LLH + gradient) against the reference's golden
vectors (tests/golden, produced by make_golden.py from GP_emu_UQSA itself).

Tolerances (fp64 end to end): LLH relative max(1e-10, 4 eps cond(A)); gradient
|g - g_ref| <= 1e-7 * (|g_ref| + max|g_ref|)  -- the gradient components are
differences of O(n) trace terms, so the bound is relative to the largest one.
The cond(A) term matters only for the alt-nugget point with nu^2 = 1e-6 on the
diagonal (cond 1.3e8): there LAPACK's own Cholesky of A and of A padded to 256
(identity block) already differ by 2.6e-10 relative in LLH, so 1e-10 is below
the problem's rounding floor.
"""
import os

import numpy as np
import pytest

from gp_emu_uqsa_amd import native
from oracle import gp_oracle as orc

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")

CASES = [
    ("std_gp4ml_fitnug", orc.STD, orc.GP4ML, True, False),
    ("std_gp4ml_fixnug", orc.STD, orc.GP4ML, False, False),
    ("std_mucm_fitnug", orc.STD, orc.MUCM, True, False),
    ("std_mucm_fixnug", orc.STD, orc.MUCM, False, False),
    ("alt_gp4ml_fitnug", orc.ALT, orc.GP4ML, True, False),
    ("alt_gp4ml_fixnug", orc.ALT, orc.GP4ML, False, False),
    ("alt_gp4ml_fitnug_r", orc.ALT, orc.GP4ML, True, True),
    # std kernel with Data.set_r: the reference's sigma gradient uses A - diag(r)
    ("std_gp4ml_fitnug_r", orc.STD, orc.GP4ML, True, True),
    ("std_gp4ml_fixnug_r", orc.STD, orc.GP4ML, False, True),
]


def _cond(X, hp, kind, variant, fitn, nu_fixed):
    d = X.shape[1]
    delta, nu, _ = orc.split_hp(hp, d, variant, fitn)
    A, _ = orc.kernel_var_ref(X, delta, nu if nu is not None else nu_fixed, kind, True)
    return np.linalg.cond(A)


def _grad_ok(g, gref, tol=1e-7):
    scale = np.abs(gref) + np.max(np.abs(gref))
    return np.all(np.abs(g - gref) <= tol * scale), np.max(np.abs(g - gref) / scale)


@pytest.mark.parametrize("fname", ["objective_n200_d3.npz", "objective_n1024_d10.npz"])
@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
@pytest.mark.parametrize("point", [0, 1])
@pytest.mark.parametrize("value_only", [False, True], ids=["grad", "value"])
def test_objective_golden(ctx, fname, case, point, value_only):
    """value_only: want_grad=0 runs the forward substitution with the Cholesky's
    diagonal inverses instead of L^-1 (sigma_analytic_mucm, :382-408)."""
    z = np.load(os.path.join(GOLD, fname))
    tag, kind, variant, fitn, use_r = case
    X, f = z["X"], z["f"]
    H = orc.linear_basis(X)
    ctx.set_data(X, f, H, z["r"] if use_r else None)
    key = f"{tag}_p{point}"
    hp = z[key + "_hp"]
    llh, grad, s2 = ctx.objective(variant, kind, hp, nu_fixed=float(z[key + "_nufixed"]),
                                  want_grad=not value_only)
    ref = float(z[key + "_llh"])
    rtol = max(1e-10, 4 * np.finfo(float).eps * _cond(X, hp, kind, variant, fitn,
                                                      float(z[key + "_nufixed"])))
    assert abs(llh - ref) <= rtol * max(1.0, abs(ref)), (llh, ref, rtol)
    if value_only:
        assert grad is None
    else:
        ok, err = _grad_ok(grad, z[key + "_grad"])
        assert ok, (err, grad, z[key + "_grad"])
    assert abs(s2 - float(z[key + "_sig2"])) <= 1e-10 * abs(float(z[key + "_sig2"]))


@pytest.mark.parametrize("fname", ["objective_n200_d3.npz", "objective_n1024_d10.npz"])
def test_objective_not_pd(ctx, fname):
    z = np.load(os.path.join(GOLD, fname))
    X, f = z["X"], z["f"]
    ctx.set_data(X, f, orc.linear_basis(X))
    with pytest.raises(native.NotPositiveDefinite):
        ctx.objective(orc.GP4ML, orc.STD, z["nonpd_hp"], nu_fixed=0.0)


@pytest.mark.parametrize("n,d", [(500, 4), (129, 2), (1000, 20), (3000, 40)])
def test_objective_value_only_matches(ctx, n, d):
    """The value-only path (forward substitution, no L^-1) against the gradient path
    (L^-1 [f H]) and the oracle: ragged n, and [f H] wider than one 16-column pass of
    k_trsv_lower (d = 20: 22 columns, d = 40: 42)."""
    X, f, H = orc.synthetic_problem(n, d, seed=9)
    ctx.set_data(X, f, H)
    hp = np.concatenate([np.linspace(0.5, 1.1, d), [1e-3, 1.3]])
    a = ctx.objective(orc.GP4ML, orc.STD, hp, want_grad=True)
    b = ctx.objective(orc.GP4ML, orc.STD, hp, want_grad=False)
    assert b[1] is None
    assert abs(a[0] - b[0]) <= 1e-12 * abs(a[0]), (a[0], b[0])
    ref = orc.objective_fast(X, f, H, hp, orc.GP4ML, orc.STD, True)[0]
    assert abs(b[0] - ref) <= 1e-10 * abs(ref), (b[0], ref)
    # MUCM's value is a difference of O(n) terms ((n - q) log sigma^2 against log|A|; 36 out
    # of terms near 10^3 at n = 3000, d = 40): 1e-11 of it is ~1e-13 of the terms.  Both
    # GPU paths are also pinned to the oracle's MUCM value and sigma-hat^2, to 1e-10 of the
    # largest cancelling term (so the looser cross-path bound cannot hide a drift of one)
    m = ctx.objective(orc.MUCM, orc.STD, hp[:-1], want_grad=False)
    mg = ctx.objective(orc.MUCM, orc.STD, hp[:-1], want_grad=True)
    assert abs(m[0] - mg[0]) <= 1e-11 * abs(mg[0]) and abs(m[2] - mg[2]) <= 1e-12 * mg[2]
    mref, _, s2ref = orc.objective_fast(X, f, H, hp[:-1], orc.MUCM, orc.STD, True, want_grad=False)
    A, _ = orc.kernel_var_ref(X, hp[:d], hp[d], orc.STD, True)
    logdet_a = np.linalg.slogdet(A)[1]
    q = H.shape[1]
    terms = 0.5 * max(abs((n - q) * np.log(s2ref)), abs(logdet_a))
    for got in (m, mg):
        assert abs(got[0] - mref) <= 1e-10 * terms, (got[0], mref, terms)
        assert abs(got[2] - s2ref) <= 1e-10 * s2ref, (got[2], s2ref)


def test_value_only_not_pd(ctx):
    """A non-positive-definite matrix is reported by the value-only path too, and the
    context stays usable (the substitution's workgroups stop on the abort flag)."""
    z = np.load(os.path.join(GOLD, "objective_n1024_d10.npz"))
    X, f = z["X"], z["f"]
    ctx.set_data(X, f, orc.linear_basis(X))
    with pytest.raises(native.NotPositiveDefinite):
        ctx.objective(orc.GP4ML, orc.STD, z["nonpd_hp"], nu_fixed=0.0, want_grad=False)
    key = "std_gp4ml_fitnug_p0"
    llh = ctx.objective(orc.GP4ML, orc.STD, z[key + "_hp"], want_grad=False)[0]
    assert abs(llh - float(z[key + "_llh"])) <= 1e-10 * abs(float(z[key + "_llh"]))


def test_scale_point_4096(ctx):
    """G5: n=4096, d=10 gp4ml at the measurement point (reference: ~42 s on CPU)."""
    z = np.load(os.path.join(GOLD, "scale_4096.npz"))
    X, f, H = orc.synthetic_problem(int(z["n"]), int(z["d"]), seed=int(z["seed"]))
    assert abs(X.sum() - float(z["X_sum"])) < 1e-9 and abs(f.sum() - float(z["f_sum"])) < 1e-9
    ctx.set_data(X, f, H)
    llh, grad, _ = ctx.objective(orc.GP4ML, orc.STD, z["hp"])
    assert abs(llh - float(z["llh"])) <= 1e-10 * abs(float(z["llh"])), (llh, float(z["llh"]))
    ok, err = _grad_ok(grad, z["grad"])   # (1e-7 of scale, as every other size)
    assert ok, (err, grad, z["grad"])


@pytest.mark.parametrize("n,d", [(129, 2), (383, 5), (640, 20)])
def test_objective_vs_oracle_ragged(ctx, n, d):
    """Sizes that are not multiples of the 128 tile (padding path), d up to 20."""
    X, f, H = orc.synthetic_problem(n, d, seed=n)
    ctx.set_data(X, f, H)
    hp = np.concatenate([np.linspace(0.4, 1.2, d), [5e-3, 0.8]])
    llh, grad, _ = ctx.objective(orc.GP4ML, orc.STD, hp)
    ref = orc.objective_fast(X, f, H, hp, orc.GP4ML, orc.STD, True)
    assert abs(llh - ref[0]) <= 1e-10 * abs(ref[0])
    ok, err = _grad_ok(grad, ref[1])
    assert ok, err


def test_forward_substitution_fallback(monkeypatch):
    """Without the augmented [f H]^T row in the Cholesky (GPEMU_AUG=0; the row is also
    absent beyond 128 basis columns) L^-1 [f H] for the value-only objective and beta comes
    from the ticketed, flag-chained forward substitution (k_trsv_lower) over the diagonal-
    tile inverses.  Value, gradient, beta and the gpe_factor path against the oracle,
    ragged n over 11 tile rows."""
    monkeypatch.setenv("GPEMU_AUG", "0")
    c = native.Context(0)
    try:
        X, f, H = orc.synthetic_problem(1300, 5, seed=4)
        c.set_data(X, f, H)
        hp = np.array([0.6, 0.7, 0.8, 0.9, 1.0, 2e-3, 1.2])
        llh_v = c.objective(orc.GP4ML, orc.STD, hp, want_grad=False)[0]
        llh, g, _ = c.objective(orc.GP4ML, orc.STD, hp)
        ref = orc.objective_fast(X, f, H, hp, orc.GP4ML, orc.STD, True)
        assert abs(llh_v - ref[0]) <= 1e-10 * abs(ref[0]) and abs(llh - ref[0]) <= 1e-10 * abs(ref[0])
        ok, err = _grad_ok(g, ref[1])
        assert ok, err
        c.factor(native.KERNEL_STD, hp[:5], hp[5], 1.0, 0.0)
        A, _ = orc.kernel_var_ref(X, hp[:5], hp[5], orc.STD, True)
        beta = c.beta()
        bref = orc.optimal_beta_ref(A, H, f)
        assert np.max(np.abs(beta - bref)) <= 1e-8 * (1 + np.max(np.abs(bref)))
        # [f H] wider than one 16-column pass of the substitution (d = 20: 22 columns)
        X2, f2, H2 = orc.synthetic_problem(700, 20, seed=6)
        c.set_data(X2, f2, H2)
        hp2 = np.concatenate([np.linspace(1.5, 3.0, 20), [2e-3, 0.9]])
        v2 = c.objective(orc.GP4ML, orc.STD, hp2, want_grad=False)[0]
        r2 = orc.objective_fast(X2, f2, H2, hp2, orc.GP4ML, orc.STD, True)[0]
        assert abs(v2 - r2) <= 1e-10 * abs(r2), (v2, r2)
    finally:
        c.close()


# schedules that run the same tiles with the same K ranges, only in other launches, list
# positions or streams: every tile's arithmetic is the same, so the results are bit-identical
# (train() relies on it: `auto` picks the group or the per-step launches per call, by what
# else is in flight on the device)
_SAME_ARITHMETIC = [
    {"GPEMU_POTRF": "fused"},
    {"GPEMU_POTRF": "group"},
    {"GPEMU_CHOL_PRIO": "0"},
    {"GPEMU_POTRF": "group", "GPEMU_GROUP_STRIDE": "0", "GPEMU_GROUP_P0": "1"},
    {"GPEMU_POTRF": "group", "GPEMU_GROUP_STRIDE": "5000"},
]
# other column-group widths (other K splits of the trailing updates) and the value path
# without the augmented row: the same results up to rounding
_OTHER_ARITHMETIC = [
    {"GPEMU_POTRF_W": "8:40,3:20", "GPEMU_GROUP_STRIDE": "300"},
    {"GPEMU_POTRF_W": "8:40,3:20", "GPEMU_POTRF": "fused"},
    {"GPEMU_AUG": "0"},
    # super-blocks: every group updating the whole trailing matrix (round 4), and super-
    # blocks of three groups (far updates of K = 1536), both schedules
    {"GPEMU_POTRF_SB": "1"},
    {"GPEMU_POTRF_SB": "1", "GPEMU_POTRF": "fused"},
    {"GPEMU_POTRF_SB": "3"},
    {"GPEMU_POTRF_SB": "3", "GPEMU_POTRF": "fused", "GPEMU_POTRF_W": "4:8,2:4"},
]


@pytest.fixture(scope="module")
def schedule_problem():
    """n = 8448 (66 tile columns: groups of width 4, 2 and 1), d = 10, with the default
    schedule's results."""
    X, f, H = orc.synthetic_problem(8448, 10, seed=12)
    hp = np.concatenate([np.linspace(0.8, 1.6, 10), [3e-3, 0.9]])
    c = native.Context(0)
    try:
        c.set_data(X, f, H)
        v = c.objective(orc.GP4ML, orc.STD, hp, want_grad=False)[0]
        llh, g, s2 = c.objective(orc.GP4ML, orc.STD, hp)
    finally:
        c.close()
    ref = orc.objective_fast(X, f, H, hp, orc.GP4ML, orc.STD, True)   # the default, pinned
    assert abs(llh - ref[0]) <= 1e-10 * abs(ref[0]) and abs(v - ref[0]) <= 1e-10 * abs(ref[0])
    ok, err = _grad_ok(g, ref[1])
    assert ok, err
    return X, f, H, hp, v, llh, g, s2


def _run_schedule(monkeypatch, schedule_problem, env):
    X, f, H, hp = schedule_problem[:4]
    for k, val in env.items():
        monkeypatch.setenv(k, val)
    c = native.Context(0)
    try:
        c.set_data(X, f, H)
        v = c.objective(orc.GP4ML, orc.STD, hp, want_grad=False)[0]
        llh, g, s2 = c.objective(orc.GP4ML, orc.STD, hp)
        vm, _, s2m = c.objective(orc.MUCM, orc.STD, hp[:-1], want_grad=False)
    finally:
        c.close()
    return v, llh, g, s2, vm, s2m


@pytest.mark.parametrize("env", _SAME_ARITHMETIC, ids=lambda e: ",".join(f"{k[6:]}={v}" for k, v in e.items()))
def test_schedule_switches_bit_identical(monkeypatch, schedule_problem, env):
    """The Cholesky's stream, one launch per step or per column group, and the group
    launch's chain positions give bit-identical value, gradient and
    sigma^2 (gp4ml) and MUCM value and sigma-hat^2."""
    X, f, H, hp, v0, llh0, g0, s20 = schedule_problem
    base = _run_schedule(monkeypatch, schedule_problem, {})
    got = _run_schedule(monkeypatch, schedule_problem, env)
    assert base[0] == v0 and base[1] == llh0 and np.array_equal(base[2], g0) and base[3] == s20
    assert got[0] == base[0], (got[0], base[0])
    assert got[1] == base[1], (got[1], base[1])
    assert np.array_equal(got[2], base[2]), (got[2] - base[2])
    assert got[3] == base[3] and got[4] == base[4] and got[5] == base[5]


@pytest.mark.parametrize("env", _OTHER_ARITHMETIC, ids=lambda e: ",".join(f"{k[6:]}={v}" for k, v in e.items()))
def test_schedule_widths_match_default(monkeypatch, schedule_problem, env):
    """Other column-group widths (the trailing updates' K split differently) and the value
    path without the augmented row: the default's results to rounding."""
    X, f, H, hp, v0, llh0, g0, s20 = schedule_problem
    v, llh, g, s2, _, _ = _run_schedule(monkeypatch, schedule_problem, env)
    assert abs(v - v0) <= 1e-11 * abs(v0), (v, v0)
    assert abs(llh - llh0) <= 1e-11 * abs(llh0), (llh, llh0)
    assert abs(s2 - s20) <= 1e-11 * abs(s20)
    assert np.max(np.abs(g - g0)) <= 1e-9 * (1.0 + np.max(np.abs(g0))), (g, g0)
