"""Pin the CPU oracle (oracle/gp_oracle.py) to the reference's golden vectors.
CPU only; the n=4096 point (G5, ~45 s) is checked on its value-only part."""
import os

import numpy as np
import pytest

from oracle import gp_oracle as orc

GOLD = os.path.join(os.path.dirname(__file__), "golden")
CASES = [
    ("std_gp4ml_fitnug", orc.STD, orc.GP4ML, True, False),
    ("std_gp4ml_fixnug", orc.STD, orc.GP4ML, False, False),
    ("std_mucm_fitnug", orc.STD, orc.MUCM, True, False),
    ("std_mucm_fixnug", orc.STD, orc.MUCM, False, False),
    ("alt_gp4ml_fitnug", orc.ALT, orc.GP4ML, True, False),
    ("alt_gp4ml_fixnug", orc.ALT, orc.GP4ML, False, False),
    ("alt_gp4ml_fitnug_r", orc.ALT, orc.GP4ML, True, True),
    ("std_gp4ml_fitnug_r", orc.STD, orc.GP4ML, True, True),
    ("std_gp4ml_fixnug_r", orc.STD, orc.GP4ML, False, True),
]


@pytest.mark.parametrize("kind,tag", [(orc.STD, "std"), (orc.ALT, "alt")])
def test_kernel_pieces(kind, tag):
    z = np.load(os.path.join(GOLD, f"kernel_{tag}.npz"))
    X, Xs, delta, nu, s2 = z["X"], z["Xs"], z["delta"], float(z["nu"]), float(z["s2"])
    A, e = orc.kernel_var_ref(X, delta, nu, kind, True)
    np.testing.assert_array_equal(A, z["A_pred"])
    np.testing.assert_array_equal(e, z["exp_save"])
    np.testing.assert_array_equal(orc.kernel_var_ref(X, delta, nu, kind, False)[0], z["A_est"])
    np.testing.assert_array_equal(orc.kernel_covar_ref(X, Xs, delta, nu, kind), z["covar"])
    for i in range(3):
        np.testing.assert_array_equal(orc.grad_delta_ref(X[:, i], delta[i], nu, e, s2, kind),
                                      z["grad_delta"][i])
    np.testing.assert_array_equal(orc.grad_nugget_ref(X.shape[0], nu, e, s2, kind), z["grad_nugget"])


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
@pytest.mark.parametrize("point", [0, 1])
def test_objective_ref_bitwise_n200(case, point):
    z = np.load(os.path.join(GOLD, "objective_n200_d3.npz"))
    tag, kind, variant, fitn, use_r = case
    X, f = z["X"], z["f"]
    H = orc.linear_basis(X)
    k = f"{tag}_p{point}"
    res = orc.objective_ref(X, f, H, z[k + "_hp"], variant, kind, fitn, z["r"] if use_r else None,
                            nu_fixed=float(z[k + "_nufixed"]))
    assert res[0] == float(z[k + "_llh"])
    np.testing.assert_allclose(res[1], z[k + "_grad"], rtol=1e-12, atol=1e-12 * np.abs(z[k + "_grad"]).max())


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_objective_fast_matches_reference(case):
    """The formulation the GPU uses (Cholesky, explicit inverse, <M, dA>)."""
    z = np.load(os.path.join(GOLD, "objective_n200_d3.npz"))
    tag, kind, variant, fitn, use_r = case
    X, f = z["X"], z["f"]
    H = orc.linear_basis(X)
    for point in (0, 1):
        k = f"{tag}_p{point}"
        res = orc.objective_fast(X, f, H, z[k + "_hp"], variant, kind, fitn,
                                 z["r"] if use_r else None, nu_fixed=float(z[k + "_nufixed"]))
        ref = float(z[k + "_llh"])
        assert abs(res[0] - ref) <= 1e-9 * abs(ref)
        g = z[k + "_grad"]
        assert np.all(np.abs(res[1] - g) <= 1e-8 * (np.abs(g) + np.abs(g).max()))


def test_objective_non_pd_is_none():
    z = np.load(os.path.join(GOLD, "objective_n200_d3.npz"))
    X, f = z["X"], z["f"]
    assert orc.objective_ref(X, f, orc.linear_basis(X), z["nonpd_hp"], orc.GP4ML, orc.STD,
                             False, nu_fixed=0.0) is None


def test_synthetic_generator_pinned():
    z = np.load(os.path.join(GOLD, "scale_4096.npz"))
    X, f, H = orc.synthetic_problem(int(z["n"]), int(z["d"]), seed=int(z["seed"]))
    assert abs(X.sum() - float(z["X_sum"])) < 1e-9
    assert abs((X ** 2).sum() - float(z["X_sq"])) < 1e-9
    assert abs(f.sum() - float(z["f_sum"])) < 1e-9


@pytest.mark.parametrize("tag", ["toysim", "toysim3d_o0", "toysim3d_o1"])
def test_posterior_ref(tag):
    z = np.load(os.path.join(GOLD, f"posterior_{tag}.npz"))
    kind = orc.ALT if bool(z["alt"]) else orc.STD
    A, _ = orc.kernel_var_ref(z["XT"], z["delta"], float(z["nu"]), kind, True)
    assert abs(np.trace(A) - float(z["A_trace"])) < 1e-12 and abs(A.sum() - float(z["A_sum"])) < 1e-9
    Hs = np.hstack([np.ones((20, 1)), z["xs"]])[:, :z["HT"].shape[1]]
    m, v = orc.posterior_ref(z["XT"], z["fT"], z["HT"], A, z["xs"], Hs, z["beta"],
                             float(z["sigma"]), z["delta"], float(z["nu"]), kind)
    np.testing.assert_allclose(m, z["mean"], rtol=0, atol=1e-12)
    np.testing.assert_allclose(v, z["var"], rtol=0, atol=1e-12)
    np.testing.assert_allclose(orc.optimal_beta_ref(A, z["HT"], z["fT"]), z["beta_opt"], atol=1e-10)


def test_product_generator_equals_oracle_generator():
    """bench.py/tools draw their inputs from gp_emu_uqsa_amd.synthetic; the oracle
    keeps its own copy for the checks -- both must give the same data."""
    from gp_emu_uqsa_amd import synthetic
    for n, d, seed in [(50, 1, 0), (300, 3, 1), (1000, 10, 2)]:
        a = synthetic.problem(n, d, seed)
        b = orc.synthetic_problem(n, d, seed)
        for u, v in zip(a, b):
            assert np.array_equal(u, v)
