"""Sensitivity / UQ on the GPU.

* The reference's sensitivity_rebuild.py sequence (uncertainty, sensitivity,
  main_effect(100), to_file, interaction_effect(0, 1), totaleffectvariance) on
  the two reconstructed toysim3D emulators and on the synthetic n=300, d=4
  emulator, against the reference's own run (tests/golden/sensitivity_*.npz, G8).
  Both toysim3D analyses are set up before either runs, so the second one's
  resident factor must be swapped back in.
* The three primitives (gpe_solve, gpe_sense_pairs, gpe_gauss_transform) against
  dense NumPy at n=700, and a size-independent property at n=16384
  (w = 0, u = 1: tr(A^-1 1 1^T) = 1^T A^-1 1 and Z^T 1 1^T Z = (sum Z)(sum Z)^T).

Tolerances: the measures are differences of O(1) terms, compared to 1e-9 of the
largest term (|uE|^2 + |I2|), as in tests/test_sense_oracle.py; per-point arrays
to 1e-10 relative.
"""
import os
import shutil

import numpy as np
import pytest

import gp_emu_uqsa_amd as g
from gp_emu_uqsa_amd import native
from gp_emu_uqsa_amd import sensitivity as sa
from oracle import gp_oracle as orc

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture()
def mpl(monkeypatch):
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    monkeypatch.setattr(plt, "show", lambda *a, **k: None)
    yield
    plt.close("all")


def _gold(fn, t):
    z = np.load(os.path.join(GOLD, fn))
    return {k[len(t):]: z[k] for k in z.files if k.startswith(t) and k != "meta"}


def _rel(a, b):
    return np.max(np.abs(np.asarray(a, float) - np.asarray(b, float))) / max(np.max(np.abs(b)), 1e-300)


def _run_and_check(s, gd, out_file):
    s.uncertainty()
    s.sensitivity()
    s.main_effect(plot=False, points=100)
    eff100, meff100 = s.effect.copy(), s.mean_effect.copy()
    s.to_file(out_file)
    s.interaction_effect(0, 1)
    s.totaleffectvariance()
    assert np.array_equal(s.x, gd["x"])
    scale = abs(float(gd["uE"])) ** 2 + abs(float(gd["I2"]))
    for k in ("uE", "uV", "uEV", "I1", "I2"):
        assert abs(getattr(s, k) - float(gd[k])) < 1e-9 * scale, (k, getattr(s, k), float(gd[k]))
    for k in ("senseindex", "senseindexwb", "EVTw"):
        assert np.max(np.abs(getattr(s, k) - gd[k])) < 1e-9 * scale, (k, getattr(s, k), gd[k])
    assert np.max(np.abs(eff100 - gd["effect100"])) < 1e-10 * scale
    assert np.max(np.abs(meff100 - gd["mean_effect100"])) < 1e-10 * scale
    assert np.max(np.abs(s.interaction - gd["interaction"])) < 1e-10 * scale
    assert np.max(np.abs(s.mean_effect[:2] - gd["mean_effect25"][:2])) < 1e-10 * scale
    for k in ("Rh", "Rhh", "Rt", "Rht", "Ut", "Uht", "U2", "Uh", "Uhh", "S", "Stild", "T", "U", "R", "Q",
              "e", "G", "W"):
        assert _rel(getattr(s, k), gd[k]) < 1e-10, k
    assert _rel(s.Utt[0], gd["Utt"]) < 1e-10
    # the results file: same keys, same number of values, same values
    mine = [l.split() for l in open(out_file).read().splitlines()]
    ref = [l.split() for l in str(gd["to_file"]).splitlines()]
    assert [l[0] for l in mine] == [l[0] for l in ref]
    for a, b in zip(mine, ref):
        assert len(a) == len(b)
        np.testing.assert_allclose(np.array(a[1:], float), np.array(b[1:], float), rtol=0,
                                   atol=1e-9 * scale)


def test_toysim3d_reconstructed(tmp_path, monkeypatch, mpl):
    d = tmp_path / "w"
    shutil.copytree(os.path.join(GOLD, "examples", "sensitivity_recon"), d, copy_function=shutil.copyfile)
    monkeypatch.chdir(d)
    sens = []
    for i in range(2):
        np.random.seed(0)
        emul = g.setup(f"toysim3D_config{i}_recon", datashuffle=True, scaleinputs=True)
        sens.append(sa.setup(emul, [0.50, 0.50, 0.50], [0.02, 0.02, 0.02]))
    for i in range(2):
        _run_and_check(sens[i], _gold("sensitivity_toysim3d.npz", f"o{i}_"), f"sense_file{i}")
    sa.sense_table(sens, [], ["y[0]", "y[1]"], rowHeight=4)


def test_synthetic_emulator(tmp_path, monkeypatch, mpl):
    gd = _gold("sensitivity_synthetic.npz", "")
    monkeypatch.chdir(tmp_path)
    np.savetxt("syn_input", gd["X"], fmt="%.10f")
    np.savetxt("syn_output", gd["f"].reshape(-1, 1), fmt="%.10f")
    with open("syn_config", "w") as fh:
        fh.write("beliefs syn_beliefs\ninputs syn_input\noutputs syn_output\ntv_config 10 0 0\n"
                 "delta_bounds [ ]\nnugget_bounds [ ]\nsigma_bounds [ ]\ntries 1\nconstraints bounds\n")
    with open("syn_beliefs", "w") as fh:
        fh.write("active all\noutput 0\nbasis_str 1.0 x x x x\nbasis_inf NA 0 1 2 3\n"
                 "beta 0.3 1.1 0.4 -0.2 -0.1\ndelta 0.45 0.6 0.8 0.7\nsigma 0.9\n"
                 "nugget 0.002\nfix_nugget T\nmucm F\n")
    np.random.seed(0)
    emul = g.setup("syn_config", datashuffle=False, scaleinputs=False)
    s = sa.setup(emul, list(gd["m"]), list(gd["v"]))
    _run_and_check(s, gd, "sense_out")


def test_setup_rejects_like_reference(tmp_path, monkeypatch, mpl):
    d = tmp_path / "w"
    shutil.copytree(os.path.join(GOLD, "examples", "sensitivity_recon"), d, copy_function=shutil.copyfile)
    monkeypatch.chdir(d)
    emul = g.setup("toysim3D_config0_recon", datashuffle=True, scaleinputs=True)
    assert sa.setup(emul, (0.5, 0.5, 0.5), [0.02] * 3) is None         # not lists
    assert sa.setup(emul, [0.5, 0.5], [0.02, 0.02]) is None             # wrong length
    assert sa.setup(emul, [0.5] * 3, [0.02] * 3, case="case1") is None  # only case2


def _dense_pairs(x, w, u):
    dx2 = (x[:, None, :] - x[None, :, :]) ** 2
    return u[:, None] * u[None, :] * np.exp(-(dx2 * w).sum(-1))


def test_primitives_match_dense(ctx):
    n, d = 700, 3
    X, f, H = orc.synthetic_problem(n, d, seed=11)
    delta, nu = np.array([0.5, 0.7, 0.9]), 1e-3
    ctx.set_data(X, f, H)
    ctx.factor(native.KERNEL_STD, delta, nu)
    A = orc.kernel_var_ref(X, delta, nu, orc.STD)[0]
    Ainv = np.linalg.inv(A)
    rng = np.random.RandomState(3)
    B = rng.normal(size=(n, 5))
    np.testing.assert_allclose(ctx.solve(B), np.linalg.solve(A, B), rtol=0,
                               atol=1e-9 * np.max(np.abs(np.linalg.solve(A, B))))
    W = rng.uniform(0.0, 4.0, size=(3, d))
    W[1, 1:] = 0.0                                   # a one-dimensional kernel, as Pw
    U = rng.uniform(0.5, 1.5, size=(3, n))
    Z = rng.normal(size=(n, 6))
    tr, quad = ctx.sense_pairs(W, U, Z)
    for j in range(3):
        K = _dense_pairs(X, W[j], U[j])
        ref_tr = np.sum(Ainv * K)
        ref_q = Z.T.dot(K).dot(Z)
        assert abs(tr[j] - ref_tr) <= 1e-9 * np.sum(np.abs(Ainv * K)), (j, tr[j], ref_tr)
        np.testing.assert_allclose(quad[j], ref_q, rtol=0, atol=1e-11 * np.abs(Z).sum(0).max() ** 2 * U.max() ** 2)
    a = rng.normal(size=n)
    Y = rng.uniform(size=(40, 2))
    out = ctx.gauss_transform([2, 0], [1.7, 0.6], Y, a)
    ref = np.array([np.sum(a * np.exp(-1.7 * (y[0] - X[:, 2]) ** 2 - 0.6 * (y[1] - X[:, 0]) ** 2)) for y in Y])
    np.testing.assert_allclose(out, ref, rtol=0, atol=1e-12 * np.abs(a).sum())


def test_pairs_ones_property_n16384(ctx):
    n, d = 16384, 10
    X, f, H = orc.synthetic_problem(n, d, seed=0)
    ctx.set_data(X, f, H)
    ctx.factor(native.KERNEL_STD, np.full(d, 0.8), 1e-3)
    Z = np.random.RandomState(1).normal(size=(n, 12))
    tr, quad = ctx.sense_pairs(np.zeros((1, d)), np.ones((1, n)), Z)
    one = ctx.solve(np.ones(n))
    assert abs(tr[0] - one.sum()) <= 1e-9 * np.abs(one).sum()
    sz = Z.sum(0)
    np.testing.assert_allclose(quad[0], np.outer(sz, sz), rtol=0, atol=1e-10 * np.abs(Z).sum(0).max() ** 2)
