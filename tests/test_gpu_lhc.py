"""gpe_lhc_maximin (the oLHC selection statistic, design_inputs.py:54-64) against the CPU
oracle np.argmin(pdist([x_k; fextra], 'sqeuclidean')): bit-exact indices.  Cases: the
reference's own designs (G7), random batches with and without fextra, exact ties
(duplicated points, repeated designs), NaN inputs, one design point plus fextra, dim 1,
and a history-matching-sized case (n 1000 with 4096 extra points)."""
import os

import numpy as np
import pytest

from gp_emu_uqsa_amd import design_inputs, native
from oracle.lhc_oracle import lhc_maximin_ref

pytestmark = pytest.mark.gpu
G = np.load(os.path.join(os.path.dirname(__file__), "golden", "history_match.npz"))


@pytest.fixture(scope="module")
def ctx():
    c = native.Context(0)
    yield c
    c.close()


def _designs(rng, N, n, dim):
    """oLHC candidates as the generator draws them."""
    xs = np.empty((N, n, dim))
    for k in range(N):
        for i in range(dim):
            xs[k, :, i] = (rng.permutation(n) + rng.uniform(0, 1, n)) / n
    return xs


@pytest.mark.parametrize("N,n,dim,ne", [(10, 20, 1, 0), (7, 33, 3, 0), (5, 17, 4, 50), (3, 64, 10, 257),
                                        (4, 9, 2, 1), (2, 300, 6, 0), (6, 1, 3, 12)])
def test_lhc_maximin_random(ctx, N, n, dim, ne):
    rng = np.random.RandomState(N * 1000 + n)
    xs = _designs(rng, N, n, dim)
    fe = rng.uniform(0, 1, (ne, dim)) if ne else None
    assert np.array_equal(ctx.lhc_maximin(xs, fe), lhc_maximin_ref(xs, fe))


def test_lhc_maximin_ties_and_nan(ctx):
    rng = np.random.RandomState(3)
    xs = _designs(rng, 6, 25, 2)
    xs[1, 7] = xs[1, 3]            # zero distance, and a second one later
    xs[1, 20] = xs[1, 11]
    xs[2] = xs[0]                  # identical designs give identical indices
    xs[3, 5, 1] = np.nan           # NaN distances are the minimum (first occurrence)
    fe = rng.uniform(0, 1, (30, 2))
    fe[4] = xs[4, 9]               # a design point duplicated in fextra
    fe[10] = fe[2]                 # a zero inside fextra: loses to the earlier design pair
    got, ref = ctx.lhc_maximin(xs, fe), lhc_maximin_ref(xs, fe)
    assert np.array_equal(got, ref), (got, ref)
    assert got[0] == got[2]


def test_lhc_maximin_fextra_minimum_wins(ctx):
    """The closest pair lies among the fextra points for every design."""
    rng = np.random.RandomState(4)
    xs = _designs(rng, 5, 12, 3)
    fe = rng.uniform(0, 1, (40, 3))
    fe[31] = fe[17] + 1e-9
    got = ctx.lhc_maximin(xs, fe)
    assert np.array_equal(got, lhc_maximin_ref(xs, fe))
    assert np.all(got == got[0])


def test_lhc_maximin_history_matching_size(ctx):
    rng = np.random.RandomState(5)
    xs = _designs(rng, 3, 1000, 8)
    fe = rng.uniform(0, 1, (4096, 8))
    assert np.array_equal(ctx.lhc_maximin(xs, fe), lhc_maximin_ref(xs, fe))


def test_lhc_maximin_bad_args(ctx):
    with pytest.raises(RuntimeError):
        ctx.lhc_maximin(np.zeros((2, 1, 3)))       # one point: no pairs


def test_lhc_maximin_wide_points(ctx):
    """dim above the LDS staging limit (512): row points read from global memory."""
    rng = np.random.RandomState(6)
    xs = _designs(rng, 3, 40, 600)
    fe = rng.uniform(0, 1, (20, 600))
    assert np.array_equal(ctx.lhc_maximin(xs, fe), lhc_maximin_ref(xs, fe))


def test_olhc_reference_designs_on_gpu(tmp_path, capsys):
    np.random.seed(21)
    for tag in ("0_1", "0_2", "1_2"):
        f = str(tmp_path / ("imp_input_" + tag))
        design_inputs.optLatinHyperCube(1, 20, 10, [[0.0, 1.0]], f)
        assert np.array_equal(np.loadtxt(f), G["design_" + tag]), tag


def test_lhc_maximin_more_designs_than_one_launch(ctx):
    """N above the 65535 designs of one launch: the native loop runs two batches."""
    rng = np.random.RandomState(8)
    xs = rng.uniform(0, 1, (70000, 3, 2))
    fe = rng.uniform(0, 1, (2, 2))
    got = ctx.lhc_maximin(xs, fe)
    ref = lhc_maximin_ref(xs[::997], fe)
    assert np.array_equal(got[::997], ref)
    assert np.array_equal(got[65530:65540], lhc_maximin_ref(xs[65530:65540], fe))
