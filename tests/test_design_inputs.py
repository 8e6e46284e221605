"""oLHC design restatement (gp_emu_uqsa_amd/design_inputs.py) against the designs the
reference wrote inside imp_plot (G7: np.random.seed(21), pairs (0,1), (0,2), (1,2),
dim 1, n 20, N 10 -- design_inputs.py:13-77, including its argmin-index selection)."""
import os

import numpy as np

from gp_emu_uqsa_amd import design_inputs

G = np.load(os.path.join(os.path.dirname(__file__), "golden", "history_match.npz"))


def test_olhc_matches_reference_designs(tmp_path, capsys):
    np.random.seed(21)
    for tag in ("0_1", "0_2", "1_2"):
        f = str(tmp_path / ("imp_input_" + tag))
        design_inputs.optLatinHyperCube(1, 20, 10, [[0.0, 1.0]], f)
        assert np.array_equal(np.loadtxt(f), G["design_" + tag]), tag


def test_olhc_file_and_ranges(tmp_path, capsys):
    np.random.seed(3)
    f = str(tmp_path / "d")
    design_inputs.optLatinHyperCube(3, 12, 4, [[0.0, 1.0], [2.0, 4.0], [-1.0, 0.0]], f)
    D = np.loadtxt(f)
    assert D.shape == (12, 3)
    for k, (lo, hi) in enumerate([[0.0, 1.0], [2.0, 4.0], [-1.0, 0.0]]):
        assert D[:, k].min() >= lo and D[:, k].max() <= hi
        # one point per stratum in every dimension
        assert sorted(np.floor((D[:, k] - lo) / (hi - lo) * 12).astype(int)) == list(range(12))
