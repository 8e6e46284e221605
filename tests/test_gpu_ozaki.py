"""The objective's A^-1 = L^-T L^-1 on the int8 matrix cores (gpemu_ozaki.hpp: 16 moduli,
53-bit operands, exact integer products reconstructed by the Chinese remainder theorem)
against the fp64 LAUUM of the same library (GPEMU_OZAKI=0) and against the oracle, for
every variant the gradient has: gp4ml / MUCM, std / alt-nugget kernel with per-point r,
fitted / fixed nugget, ragged n whose padded size is an odd number of 128-tiles (the
int8 path's 256-tiles then run past n_pad), d up to 20.  The LLH does not depend on A^-1
(it comes from the Cholesky sweep): it must agree to the last bits.  Gradient: 1e-7 of
scale against the oracle (the suite's tolerance), 1e-10 against the fp64 path."""
import numpy as np
import pytest

from gp_emu_uqsa_amd import native
from oracle import gp_oracle as orc

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def oz():
    """A context with the int8 products from n_pad 2048 (their default start is 6144, where
    they begin to pay; these sizes keep the oracle checks quick)."""
    mp = pytest.MonkeyPatch()
    mp.setenv("GPEMU_OZAKI_MIN_NP", "2048")
    c = native.Context(0)
    mp.undo()
    yield c
    c.close()


@pytest.fixture(scope="module")
def fp64():
    mp = pytest.MonkeyPatch()
    mp.setenv("GPEMU_OZAKI", "0")
    c = native.Context(0)
    mp.undo()
    yield c
    c.close()


def _scale(g):
    return np.abs(g) + np.max(np.abs(g))


CASES = [   # (variant, kernel, fit nugget, r)
    (orc.GP4ML, orc.STD, True, False),
    (orc.MUCM, orc.STD, False, False),
    (orc.GP4ML, orc.ALT, True, True),
    (orc.GP4ML, orc.STD, True, True),
]


@pytest.mark.parametrize("n,d", [(2048, 10), (2200, 5), (3000, 20)])
@pytest.mark.parametrize("case", CASES, ids=["gp4ml_fit", "mucm_fix", "alt_r", "std_r"])
def test_ozaki_gradient(oz, fp64, n, d, case):
    variant, kind, fitn, use_r = case
    X, f, H = orc.synthetic_problem(n, d, seed=n + d)
    r = np.random.RandomState(n).uniform(1e-4, 1e-3, size=n) if use_r else None
    hp = list(np.linspace(0.5, 1.1, d))
    if fitn:
        hp.append(3e-2 if kind == orc.ALT else 1e-3)
    if variant == orc.GP4ML:
        hp.append(1.1)
    hp = np.array(hp)
    nu_fixed = 5e-3 if not fitn else 0.0
    oz.set_data(X, f, H, r)
    fp64.set_data(X, f, H, r)
    llh, g, s2 = oz.objective(variant, kind, hp, nu_fixed=nu_fixed)
    llh64, g64, s64 = fp64.objective(variant, kind, hp, nu_fixed=nu_fixed)
    assert llh == llh64 and s2 == s64
    err64 = np.max(np.abs(g - g64) / _scale(g64))
    assert err64 <= 1e-10, (err64, g, g64)
    ref = orc.objective_fast(X, f, H, hp, variant, kind, fitn, r=r, nu_fixed=nu_fixed)
    assert abs(llh - ref[0]) <= 1e-10 * max(1.0, abs(ref[0]))
    err = np.max(np.abs(g - ref[1]) / _scale(ref[1]))
    assert err <= 1e-7, (err, g, ref[1])


def test_ozaki_fewer_moduli_still_accurate(fp64):
    """GPEMU_OZAKI_MODULI=12 (beta = 41 bits at n_pad = 4096): the gradient still within
    1e-9 of the fp64 path (the truncated operands' error, not a wrong reconstruction)."""
    mp = pytest.MonkeyPatch()
    mp.setenv("GPEMU_OZAKI_MODULI", "12")
    mp.setenv("GPEMU_OZAKI_MIN_NP", "2048")
    c = native.Context(0)
    mp.undo()
    try:
        X, f, H = orc.synthetic_problem(4096, 10, seed=3)
        hp = np.concatenate([np.ones(10), [1e-3, 1.0]])
        c.set_data(X, f, H)
        fp64.set_data(X, f, H)
        _, g, _ = c.objective(orc.GP4ML, orc.STD, hp)
        _, g64, _ = fp64.objective(orc.GP4ML, orc.STD, hp)
        assert np.max(np.abs(g - g64) / _scale(g64)) <= 1e-9
    finally:
        c.close()
