"""End-to-end drop-in parity on the GPU: the reference's own example emulators.

* g.train() on examples/toy-sim with np.random.seed(s) must follow the
  reference's L-BFGS-B trajectory (G4): same objective call sequence (1e-6) and
  the same trained hyperparameters, sigma and beta (1e-6 relative).
  The same again with the objective routed through the row-block distributed
  path (distributed.enable_objective, loopback transport, 3 logical ranks).
* g.posterior() on the reconstructed emulators (G3) within 1e-8, and the seeded
  posterior_sample, interval, indiv_standard_error and mahalanobis_distance (a14).
"""
import json
import os
import shutil

import numpy as np
import pytest

import gp_emu_uqsa_amd as g

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
EX = os.path.join(GOLD, "examples")


@pytest.fixture()
def workdir(tmp_path, monkeypatch):
    def make(sub):
        d = tmp_path / os.path.basename(sub)
        shutil.copytree(os.path.join(EX, sub), d)
        monkeypatch.chdir(d)
        return d
    return make


@pytest.fixture(params=["single", "rowblock3"])
def objective_path(request):
    from gp_emu_uqsa_amd import distributed
    if request.param == "rowblock3":
        distributed.enable_objective(loopback=3)
    yield request.param
    distributed.disable_objective()


@pytest.mark.parametrize("seed", [0, 1])
def test_train_toysim_trajectory(workdir, seed, monkeypatch, objective_path):
    z = np.load(os.path.join(GOLD, f"train_toysim_seed{seed}.npz"))
    workdir("toy-sim")
    np.random.seed(seed)
    E = g.setup("toy-sim_config")
    calls = []
    orig = E.opt_T.loglikelihood_mucm

    def rec(x):
        res = orig(x)
        calls.append((np.array(x, float), None if res is None else res[0]))
        return res
    monkeypatch.setattr(E.opt_T, "loglikelihood_mucm", rec)
    g.train(E, auto=True)
    ref_x = z["call_x"]
    n = min(len(calls), len(ref_x))
    assert n >= 100
    xs = np.array([c[0] for c in calls[:100]])
    assert np.max(np.abs(xs - ref_x[:100])) < 1e-6
    np.testing.assert_allclose(E.par.delta, z["delta"], rtol=1e-6)
    np.testing.assert_allclose(E.par.sigma, float(z["sigma"]), rtol=1e-6)
    np.testing.assert_allclose(E.par.beta, z["beta"], rtol=1e-6)
    assert E.training.inputs.shape[0] == int(z["n_train"])
    # checkpoint files: same names, same hyperparameter lines
    ref_files = json.loads(str(z["beliefs_json"]))
    for name, text in ref_files.items():
        mine = open(name).read().splitlines()
        ref = text.splitlines()
        assert [l.split(" ")[0] for l in mine] == [l.split(" ")[0] for l in ref]
        for a, b in zip(mine, ref):
            if a.split(" ")[0] in ("delta", "sigma", "beta", "nugget"):
                np.testing.assert_allclose([float(v) for v in a.split()[1:]],
                                           [float(v) for v in b.split()[1:]], rtol=1e-5)
    pm, pv = g.posterior(E, z["xs_post"])
    assert np.max(np.abs(pm - z["post_mean"])) < 1e-5
    assert np.max(np.abs(pv - z["post_var"])) < 1e-5


@pytest.mark.parametrize("sub,conf,tag", [
    ("toy-sim/reconstruct", "toy-sim_config_recon", "toysim"),
    ("sensitivity_recon", "toysim3D_config0_recon", "toysim3d_o0"),
    ("sensitivity_recon", "toysim3D_config1_recon", "toysim3d_o1")])
def test_reconstructed_posterior(workdir, sub, conf, tag):
    z = np.load(os.path.join(GOLD, f"posterior_{tag}.npz"))
    workdir(sub)
    E = g.setup(conf, datashuffle=False)
    np.testing.assert_array_equal(E.training.inputs, z["XT"])
    mean, var = g.posterior(E, z["xs"])
    assert np.max(np.abs(mean - z["mean"])) < 1e-8
    assert np.max(np.abs(var - z["var"])) < 1e-8
    A = E.training.A
    assert abs(np.trace(A) - float(z["A_trace"])) < 1e-10
    assert abs(A.sum() - float(z["A_sum"])) < 1e-8 * abs(float(z["A_sum"]))


def test_plot_and_sample(workdir, monkeypatch):
    monkeypatch.setenv("MPLBACKEND", "Agg")
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    monkeypatch.setattr(plt, "show", lambda *a, **k: None)
    workdir("toy-sim/reconstruct")
    E = g.setup("toy-sim_config_recon", datashuffle=False)
    post = g.plot(E, [0, 1], [], [], "var")
    assert post.var.shape == (900,) and np.all(post.var > -1e-12)
    g.plot(E, [0], [1], [0.3], "mean")
    np.random.seed(3)
    s = g.posterior_sample(E, np.random.uniform(size=(15, 2)))
    assert s.shape == (15,) and np.all(np.isfinite(s))


@pytest.mark.parametrize("sub,conf,tag", [
    ("toy-sim/reconstruct", "toy-sim_config_recon", "toysim"),
    ("sensitivity_recon", "toysim3D_config0_recon", "toysim3d_o0"),
    ("sensitivity_recon", "toysim3D_config1_recon", "toysim3d_o1")])
def test_sample_interval_diagnostics_golden(workdir, capsys, sub, conf, tag):
    """a14 against the reference's own outputs (G3): the seeded posterior_sample
    (emulatorfunctions.py:255-286: mean + chol(var) randn), and on a validation-style
    set Posterior.interval, indiv_standard_error (flagged points and their printed
    lines) and mahalanobis_distance (_emulatorclasses.py:635-676).  Tolerance 1e-8 on
    values; the printed text must match (its numbers are rounded by the reference)."""
    from gp_emu_uqsa_amd import model
    z = np.load(os.path.join(GOLD, f"posterior_{tag}.npz"))
    workdir(sub)
    E = g.setup(conf, datashuffle=False)
    xs = z["xs"]
    np.random.seed(int(z["sample_seed"]))
    s = g.posterior_sample(E, xs)
    assert np.max(np.abs(s - z["sample"])) < 1e-8, np.max(np.abs(s - z["sample"]))
    Dv = model.Data(xs.copy(), z["ys"].copy(), E.basis, E.par, E.beliefs, E.K)
    p = model.Posterior(Dv, E.training, E.par, E.beliefs, E.K)
    p.interval()
    assert np.max(np.abs(p.LI - z["LI"])) < 1e-8 and np.max(np.abs(p.UI - z["UI"])) < 1e-8
    capsys.readouterr()
    assert p.indiv_standard_error(ise=2.0) == bool(z["ise_retrain"])
    assert capsys.readouterr().out == str(z["ise_text"])
    p.mahalanobis_distance()
    out = capsys.readouterr().out
    ref_lines, lines = str(z["md_text"]).splitlines(), out.splitlines()
    assert lines[0] == ref_lines[0]                         # theoretical mean / variance
    md = float(lines[1].split(":")[1])
    assert abs(md - float(z["md"])) <= 1e-8 * abs(float(z["md"])), (md, float(z["md"]))
