"""The sensitivity oracle (oracle/sense_oracle.py) against the reference's own run
(tests/golden/sensitivity_*.npz, make_golden.py G8): the two reconstructed toysim3D
emulators and the synthetic n=300, d=4 emulator.

Tolerances: 1e-12 relative on per-point arrays; the measures are differences of
O(1) terms (I1 = s2 (1 - tr(A^-1 Rtt) + ...), EEE - EE2), so they are compared to
1e-9 of the largest term (uE^2 + I2 scale) -- the synthetic A has cond ~1e6."""
import os

import numpy as np
import pytest

from oracle import sense_oracle as so

GOLD = os.path.join(os.path.dirname(__file__), "golden")
CASES = [("sensitivity_toysim3d.npz", "o0_"), ("sensitivity_toysim3d.npz", "o1_"),
         ("sensitivity_synthetic.npz", "")]


def _load(fn, t):
    z = np.load(os.path.join(GOLD, fn))
    return {k[len(t):]: z[k] for k in z.files if k.startswith(t) and k != "meta"}


def _setup(g):
    return so.setup_ref(g["x"], g["f"], g["H"], g["A"], g["beta"], float(g["sigma"]), float(g["nugget"]),
                        g["delta"], g["m"], g["v"])


def _rel(a, b):
    return np.max(np.abs(np.asarray(a) - np.asarray(b))) / max(np.max(np.abs(b)), 1e-300)


@pytest.mark.parametrize("fn,t", CASES)
def test_oracle_matches_reference_run(fn, t):
    g = _load(fn, t)
    s = _setup(g)
    for k in ("T", "U", "e", "W", "G", "R", "Q"):
        assert _rel(s[k], g[k]) < 1e-12, k
    u = so.uncertainty_ref(s)
    for k in ("Rh", "Rhh", "Rt", "Rht", "Ut", "Uht", "U2", "S", "Stild", "Uh", "Uhh"):
        assert _rel(u[k], g[k]) < 1e-12, k
    assert _rel(u["Utt"][0], g["Utt"]) < 1e-12
    if "Rtt" in g:
        assert _rel(u["Rtt"], g["Rtt"]) < 1e-12
    scale = abs(float(g["uE"])) ** 2 + abs(float(g["I2"]))
    for k in ("uE", "uV", "uEV", "I1", "I2"):
        assert abs(u[k] - float(g[k])) < 1e-9 * scale, k
    ev, evt = so.totaleffectvariance_ref(s, u["uEV"])
    assert np.max(np.abs(ev - g["senseindex"])) < 1e-9 * scale
    assert np.max(np.abs(ev - g["senseindexwb"])) < 1e-9 * scale
    assert np.max(np.abs(evt - g["EVTw"])) < 1e-9 * scale
    eff, meff = so.main_effect_ref(s, g["input_range"], 100)
    assert np.max(np.abs(eff - g["effect100"])) < 1e-12 * scale
    assert np.max(np.abs(meff - g["mean_effect100"])) < 1e-12 * scale
    inter, e25, m25 = so.interaction_ref(s, g["input_range"], 0, 1, 25)
    assert np.max(np.abs(inter - g["interaction"])) < 1e-12 * scale
    assert np.max(np.abs(m25[:2] - g["mean_effect25"][:2])) < 1e-12 * scale
