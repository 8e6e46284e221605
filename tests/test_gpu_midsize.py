"""Objective parity against the CPU oracle (objective_fast: LAPACK Cholesky, explicit
inverse, dense contraction) at sizes where the GPU schedule is the full-size one:
n = 10300 (81 tiles, ragged) runs the Cholesky's 4-wide and 2-wide column groups and the
single-column tail, all TRTRI recursion levels and the LAUUM tile lists of C3; n = 5200
(41 tiles) the 2-wide groups, with the MUCM variant and the alt-nugget kernel, and the
row-block distributed objective on 2 and 3 loopback ranks.
Tolerances as tests/test_gpu_objective.py: LLH 1e-10 relative, gradient 1e-7 of
(|g| + max|g|)."""
import numpy as np
import pytest

from gp_emu_uqsa_amd import native
from oracle import gp_oracle as orc

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,d,kind,variant", [(10300, 10, orc.STD, orc.GP4ML),
                                              (5200, 6, orc.STD, orc.MUCM),
                                              (5200, 6, orc.ALT, orc.GP4ML)],
                         ids=["n10300_std_gp4ml", "n5200_std_mucm", "n5200_alt_gp4ml"])
def test_objective_midsize_vs_oracle(n, d, kind, variant):
    X, f, H = orc.synthetic_problem(n, d, seed=n + d)
    hp = np.concatenate([np.linspace(0.6, 1.1, d), [2e-3]] + ([[0.9]] if variant == orc.GP4ML else []))
    ctx = native.Context(0)
    try:
        ctx.set_data(X, f, H)
        llh, g, s2 = ctx.objective(variant, kind, hp)
    finally:
        ctx.close()
    ref = orc.objective_fast(X, f, H, hp, variant, kind, True)
    assert abs(llh - ref[0]) <= 1e-10 * abs(ref[0]), (llh, ref[0])
    scale = np.abs(ref[1]) + np.max(np.abs(ref[1]))
    assert np.all(np.abs(g - ref[1]) <= 1e-7 * scale), np.max(np.abs(g - ref[1]) / scale)
    if variant == orc.MUCM:
        assert abs(s2 - ref[2]) <= 1e-10 * abs(ref[2])


@pytest.mark.parametrize("P,variant", [(3, orc.GP4ML), (2, orc.MUCM)])
def test_distributed_midsize_vs_oracle(P, variant):
    """The row-block distributed objective (loopback ranks) at n = 5200: column groups,
    grouped row TRTRI and per-rank A^-1 partials against the oracle."""
    n, d = 5200, 6
    X, f, H = orc.synthetic_problem(n, d, seed=n + d)
    hp = np.concatenate([np.linspace(0.6, 1.1, d), [2e-3]] + ([[0.9]] if variant == orc.GP4ML else []))
    dc = native.DistContext(0, P)
    try:
        dc.set_data(X, f, H)
        llh, g, _ = dc.objective(variant, orc.STD, hp, want_grad=True)
    finally:
        dc.close()
    ref = orc.objective_fast(X, f, H, hp, variant, orc.STD, True)
    assert abs(llh - ref[0]) <= 1e-10 * abs(ref[0]), (llh, ref[0])
    scale = np.abs(ref[1]) + np.max(np.abs(ref[1]))
    assert np.all(np.abs(g - ref[1]) <= 1e-7 * scale), np.max(np.abs(g - ref[1]) / scale)
