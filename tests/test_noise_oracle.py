"""noise_fit oracle pinned to the reference's seeded noisefit() run (G9), CPU only."""
import os

import numpy as np
import pytest

from oracle import gp_oracle as orc
from oracle import noise_oracle as nor

G9 = np.load(os.path.join(os.path.dirname(__file__), "golden", "noise_fit.npz"))


def _post(i):
    return {k[len(f"p{i}_"):]: G9[k] for k in G9.files if k.startswith(f"p{i}_")}


def _draw_blocks():
    """The randn draws split per estimation step: (samples x m) blocks."""
    sizes = G9["draw_sizes"]
    flat = G9["draws"]
    blocks, pos, i = [], 0, 0
    while i < len(sizes):
        m = sizes[i]
        j = i
        while j < len(sizes) and sizes[j] == m:
            j += 1
        cnt = j - i
        blocks.append(flat[pos:pos + cnt * m].reshape(cnt, m))
        pos += cnt * m
        i = j
    return blocks


def _rebuild(p):
    """(A = Dold.A, rs_new) as the reference held them for posterior p."""
    kind = orc.ALT if bool(p["alt"]) else orc.STD
    r = p["r"] if p["r"].size == p["x"].shape[0] else None
    A, _ = orc.make_A_ref(p["x"], p["delta"], float(p["nugget"]), kind, r=r, s2=1.0)
    rs = None
    if p["rs"].size == p["xs"].shape[0] and kind == orc.ALT:
        # Dnew.make_A(s2 = sigma^2) after set_r (noise_fit.py:118-121)
        rs = p["rs"] / float(p["sigma"]) ** 2
    return kind, A, rs


@pytest.mark.parametrize("i", range(9))
def test_posteriors_match_reference(i):
    p = _post(i)
    kind, A, rs = _rebuild(p)
    np.testing.assert_allclose(np.diag(A), p["A_diag"], rtol=0, atol=1e-14)
    m = p["xs"].shape[0]
    Hs = np.ones((m, 1))
    H = np.ones((p["x"].shape[0], 1))
    mean, var = nor.posterior_ref(p["x"], p["f"], H, A, p["xs"], Hs, p["beta"], float(p["sigma"]),
                                  p["delta"], float(p["nugget"]), kind, rs)
    scale = np.max(np.abs(p["mean"])) + 1.0
    assert np.max(np.abs(mean - p["mean"])) <= 1e-10 * scale
    vs = np.max(np.abs(p["var"])) + 1e-300
    assert np.max(np.abs(var - p["var"])) <= 1e-9 * vs


def test_estimation_steps_match_reference():
    """Each iteration's z' written to zp-outputs equals the oracle's restatement fed
    with the reference's posterior (training points) and its randn draws."""
    blocks = _draw_blocks()
    assert len(blocks) == 4            # 2 iterations x (T, V)
    for it, (pi, zk) in enumerate([(0, "zp1"), (4, "zp2")]):
        p = _post(pi)
        z = nor.noise_estimate_ref(p["mean"], p["var"], p["f"], blocks[2 * it])
        np.testing.assert_allclose(z, G9[zk], rtol=1e-13, atol=1e-13)


def test_cholesky_of_recorded_variances():
    """The noise loop's np.linalg.cholesky inputs are the training/validation
    posterior covariances, in order."""
    assert int(G9["n_chol"]) == 4
    for c, pi in enumerate([0, 1, 4, 5]):
        L = np.linalg.cholesky(_post(pi)["var"])
        np.testing.assert_allclose(L, G9[f"chol{c}"], rtol=0, atol=1e-14)
