"""noise_fit on the GPU (gp_emu_uqsa_amd/noise_fit.py, gpe_noise_sample) against the
reference's seeded noisefit() run (G9, make_golden.py).

- The estimation step alone: with the reference's trained emulator state and its randn
  draws, gpe_noise_sample's z' (posterior covariance, Cholesky and the s draws on the
  GPU) must equal what the reference wrote to 'zp-outputs' to 1e-9 absolute (z' is a log;
  the covariance's entries agree with SciPy's LU-based ones to ~1e-12 relative).
- The whole loop: noisefit(stopat=2) from the same seed.  Each training is an
  L-BFGS-B run, and the GPU's objective differs from the reference's in the last bits,
  so trained hyperparameters and outputs agree to 1e-5 relative, not bitwise.
"""
import os

import numpy as np
import pytest

from gp_emu_uqsa_amd import native
from gp_emu_uqsa_amd import noise_fit as nf

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
G9 = np.load(os.path.join(HERE, "golden", "noise_fit.npz"))


def _post(i):
    return {k[len(f"p{i}_"):]: G9[k] for k in G9.files if k.startswith(f"p{i}_")}


def _draw_blocks():
    sizes, flat = G9["draw_sizes"], G9["draws"]
    blocks, pos, i = [], 0, 0
    while i < len(sizes):
        j = i
        while j < len(sizes) and sizes[j] == sizes[i]:
            j += 1
        blocks.append(flat[pos:pos + (j - i) * sizes[i]].reshape(j - i, sizes[i]))
        pos += (j - i) * sizes[i]
        i = j
    return blocks


@pytest.mark.parametrize("it", [0, 1])
def test_estimation_step_matches_reference(ctx, it):
    """Iteration it's training-set and validation-set estimation steps."""
    blocks = _draw_blocks()
    for k, pi in enumerate([(0, 1), (4, 5)][it]):
        p = _post(pi)
        x, f = p["x"], p["f"]
        alt = bool(p["alt"])
        kern = native.KERNEL_ALT_NUG if alt else native.KERNEL_STD
        r = p["r"] if p["r"].size == x.shape[0] else None
        ctx.set_data(x, f, np.ones((x.shape[0], 1)), r)
        ctx.factor(kern, p["delta"], float(p["nugget"]), 1.0, 1.0 if r is not None else 0.0)
        xs = p["xs"]
        m = xs.shape[0]
        sig = float(p["sigma"])
        rn = p["rs"] if p["rs"].size == m else None
        # t: the outputs of the set the step estimates (noise_fit.py:99/101)
        t = f if m == x.shape[0] else G9["zp0"][:0]
        if m != x.shape[0]:
            # the validation rows are the first V rows of the shuffled full set; find them in x
            idx = [int(np.argmin(np.sum((x - xi) ** 2, axis=1))) for xi in xs]
            t = f[idx]
        U = blocks[2 * it + k]
        mean, zsum = ctx.noise_sample(xs, np.ones((m, 1)), p["beta"], sig, t, U,
                                      r_new=rn, r_scale=0.0 if rn is None else 1.0 / sig ** 2)
        assert np.max(np.abs(mean - p["mean"])) <= 1e-10 * (np.max(np.abs(p["mean"])) + 1.0)
        z = np.log(zsum / float(U.shape[0]))
        if k == 0:
            ref = G9[f"zp{it + 1}"]
        else:   # the reference does not save the validation z'; restate it from its draws
            L = G9[f"chol{2 * it + 1}"]
            acc = np.zeros(m)
            for u in U:
                acc = acc + 0.5 * (t - (p["mean"] + L.dot(u))) ** 2
            ref = np.log(acc / float(U.shape[0]))
        assert np.max(np.abs(z - ref)) <= 1e-9, np.max(np.abs(z - ref))


def test_noise_sample_not_pd(ctx):
    """A covariance that is not positive definite raises like np.linalg.cholesky."""
    rs = np.random.RandomState(4)
    x = rs.uniform(size=(40, 2))
    f = np.sin(4 * x[:, 0])
    ctx.set_data(x, f, np.ones((40, 1)))
    ctx.factor(native.KERNEL_STD, np.array([0.4, 0.5]), 1e-3, 1.0, 0.0)
    xs = np.vstack([x[:5], x[:5]])      # repeated points: a singular covariance
    with pytest.raises(native.NotPositiveDefinite):
        ctx.noise_sample(xs, np.ones((10, 1)), np.array([0.1]), -1.0, np.zeros(10), rs.randn(3, 10),
                         r_new=-np.ones(10), r_scale=1.0)


def test_noise_sample_large_property(ctx):
    """m = 3000 (24 tiles): the sum over draws equals sum_j 0.5 (e - L u_j)^2 with L the
    library's own Cholesky of the covariance (gpe_posterior + gpe_cholesky), 1e-9 rel."""
    rs = np.random.RandomState(5)
    n, m, s = 2000, 3000, 37
    x = rs.uniform(size=(n, 2))
    f = np.cos(3 * x[:, 0]) + x[:, 1] ** 2 + 0.1 * rs.randn(n)
    r = 0.01 + 0.05 * x[:, 1]
    ctx.set_data(x, f, np.ones((n, 1)), r)
    ctx.factor(native.KERNEL_ALT_NUG, np.array([0.3, 0.4]), 1e-3, 1.0, 1.0)
    xs = rs.uniform(size=(m, 2))
    rn = 0.01 + 0.05 * xs[:, 1]
    t = rs.randn(m)
    U = rs.randn(s, m)
    mean, zsum = ctx.noise_sample(xs, np.ones((m, 1)), np.array([0.2]), 0.8, t, U, r_new=rn,
                                  r_scale=1.0 / 0.64)
    mean2, V = ctx.posterior(xs, np.ones((m, 1)), np.array([0.2]), 0.8, full_var=True)
    V[np.diag_indices(m)] += 0.64 * rn / 0.64
    L = ctx.cholesky(V, want=("L",))["L"]
    ref = np.sum(0.5 * ((t - mean2)[:, None] - L.dot(U.T)) ** 2, axis=1)
    assert np.max(np.abs(mean - mean2)) == 0.0
    assert np.max(np.abs(zsum - ref) / ref) <= 1e-9


def _write_inputs():
    np.savetxt("INPUTS", G9["X"])
    np.savetxt("OUTPUTS", G9["y"])
    for f in ("config-data", "config-noise", "beliefs-data", "beliefs-noise"):
        with open(f, "w") as fh:
            fh.write(str(G9["in_" + f.replace("-", "_")]))


def _beliefs(text):
    out = {}
    for line in str(text).splitlines():
        k, _, v = line.partition(" ")
        if k in ("beta", "delta", "sigma", "nugget"):
            out[k] = np.array([float(t) for t in v.split()])
    return out


def test_noisefit_replay(tmp_path, monkeypatch, capsys):
    monkeypatch.chdir(tmp_path)
    _write_inputs()
    np.random.seed(9)
    nf.noisefit("config-data", "config-noise", stopat=2, olhcmult=10, samples=50)
    assert np.array_equal(np.loadtxt("x_range_input"), G9["x_range"])
    assert np.array_equal(np.loadtxt("noise-inputs"), G9["noise_inputs"])
    np.testing.assert_allclose(np.loadtxt("zp-outputs"), G9["zp2"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(np.loadtxt("noise-outputs"), G9["noise_outputs"], rtol=1e-5, atol=1e-8)
    for f in ("beliefs-data-0f", "beliefs-noise-0f"):
        got = _beliefs(open(f).read())
        ref = _beliefs(G9[f.replace("-", "_")])
        for k in ref:
            np.testing.assert_allclose(got[k], ref[k], rtol=1e-5, err_msg=f + " " + k)
