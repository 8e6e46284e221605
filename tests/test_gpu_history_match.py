"""History matching with batched posteriors (gp_emu_uqsa_amd/history_match.py)
replayed against the reference's run (G7): imp_plot (grid 4, olhcmult 20, maxno 2)
IMP/ODP grids, nonimp_data, new_wave_design, same seeds and files.  Tolerances:
IMP (implausibility minima) 1e-7 relative -- posterior mean/variance differ from
SciPy's LU solves at ~1e-10; ODP (fractions of n=20 points) exact."""
import os
import shutil

import numpy as np
import pytest

import gp_emu_uqsa_amd as g
from gp_emu_uqsa_amd import history_match as hm

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
G = np.load(os.path.join(HERE, "golden", "history_match.npz"))


@pytest.fixture()
def workdir(tmp_path, monkeypatch):
    shutil.copytree(os.path.join(HERE, "golden", "examples", "sensitivity_recon"), tmp_path / "w",
                    copy_function=shutil.copyfile)          # the checkout may be read-only
    os.chmod(tmp_path / "w", 0o755)
    monkeypatch.chdir(tmp_path / "w")
    for i in range(2):   # as make_golden.py G7: the line final_beliefs writes
        with open(f"toysim3D_beliefs{i}-1f", "a") as fh:
            fh.write("active_index 0 1 2\n")
    np.savetxt("toysim3D_input", G["data_in"])
    np.savetxt("toysim3D_output", G["data_out"])
    return tmp_path / "w"


def test_history_match_replay(workdir, capsys):
    emuls = [g.setup(f"toysim3D_config{i}_recon", datashuffle=False, scaleinputs=True) for i in range(2)]
    zs, ve, cm = list(G["zs"]), list(G["var_extra"]), float(G["cm"])
    np.random.seed(21)
    hm.imp_plot(emuls, zs, cm, ve, maxno=2, olhcmult=20, grid=4, plot=False)
    for tag in ("0_1", "0_2", "1_2"):
        assert np.array_equal(np.loadtxt("imp_input_" + tag), G["design_" + tag])
        for m in (1, 2):
            imp = np.loadtxt(f"{m}_IMP_" + tag)
            ref = G[f"IMP{m}_" + tag]
            assert np.allclose(imp, ref, rtol=1e-7, atol=1e-9), (tag, m, np.max(np.abs(imp - ref)))
            assert np.array_equal(np.loadtxt(f"{m}_ODP_" + tag), G[f"ODP{m}_" + tag]), (tag, m)
    din, dout = "toysim3D_input", "toysim3D_output"
    count = hm.nonimp_data(emuls, zs, cm, ve, [din, dout], maxno=1)
    assert count == int(G["nonimp_count"])
    assert np.allclose(np.loadtxt("nonimp_" + din), G["nonimp_in"], rtol=0, atol=1e-15)
    assert np.array_equal(np.loadtxt("noninp_" + dout), G["nonimp_out"])
    np.random.seed(22)
    count = hm.new_wave_design(emuls, zs, cm, ve, ["nonimp_" + din, "noninp_" + dout], maxno=1, olhcmult=10)
    assert count == int(G["wave_count"])
    assert np.array_equal(np.loadtxt("olhc_des"), G["wave_olhc"])
    assert np.array_equal(np.loadtxt("nonimp_" + din), G["wave_design"])


def test_imp_plot_draws(workdir, capsys, monkeypatch):
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    monkeypatch.setattr(plt, "show", lambda: None)
    emuls = [g.setup(f"toysim3D_config{i}_recon", datashuffle=False, scaleinputs=True) for i in range(2)]
    np.random.seed(1)
    hm.imp_plot(emuls, list(G["zs"]), 3.0, list(G["var_extra"]), maxno=1, olhcmult=5, grid=3, plot=True)
    hm.imp_plot_recon(3.0, maxno=1, act=[0, 1, 2])
    assert os.path.exists("1_IMP_0_2") and os.path.exists("1_ODP_1_2")
