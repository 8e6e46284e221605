"""Host-side drop-in surface on CPU: config/beliefs parsing, data shuffle and
T/V split, basis matrix, bounds and RNG consumption vs the reference (G6)."""
import os
import shutil

import numpy as np
import pytest

from gp_emu_uqsa_amd import files, model

GOLD = os.path.join(os.path.dirname(__file__), "golden")
EX = os.path.join(GOLD, "examples")


@pytest.fixture()
def toysim_dir(tmp_path, monkeypatch):
    d = tmp_path / "toy"
    shutil.copytree(os.path.join(EX, "toy-sim"), d)
    monkeypatch.chdir(d)
    return d


def test_config_and_beliefs(toysim_dir):
    c = files.Config("toy-sim_config")
    assert c.tv_config == [10, 0, 2] and c.tries == 10 and c.constraints == "none"
    assert c.delta_bounds == [] and c.bounds == ()
    b = files.Beliefs(c.beliefs)
    assert b.active == [] and b.basis_str == ["1.0", "x"] and b.basis_inf == [0]
    assert b.fix_nugget == "T" and b.mucm == "T" and b.alt_nugget == "F"
    assert b.delta == [1.0, 1.0] and b.nugget == 0.01


def test_reconstruct_beliefs_minmax(tmp_path, monkeypatch):
    monkeypatch.chdir(os.path.join(EX, "toy-sim", "reconstruct"))
    b = files.Beliefs("toy-sim_beliefs-2f")
    assert np.allclose(b.input_minmax, [[0.0157, 0.9854], [0.0133, 0.9981]])
    assert b.fix_nugget == "F"


@pytest.mark.parametrize("text", ["[[0.1, 2*0.5]]", "[[1e-3, 1.0/3], [0.5, 2**-1 + 0.25]]",
                                  "[ [np.float64(0.1), np.pi/2] ]", "[[-1+0.5, np.sqrt(4.0)]]", "[ ]"])
def test_config_list_arithmetic_as_eval(tmp_path, monkeypatch, text):
    """Deliberate deviation, documented in files.py: the reference eval()s bound lists
    with numpy as np in scope (_emulatorclasses.py:76-78), so arithmetic in a config
    file works there; the restricted evaluator gives exactly eval's values for such
    files without executing anything else."""
    monkeypatch.chdir(tmp_path)
    (tmp_path / "cfg").write_text(f"beliefs b\ninputs i\noutputs o\ntv_config 10 0 2\ndelta_bounds {text}\n"
                                  "nugget_bounds [ ]\nsigma_bounds [[0.01, 3*1.5]]\ntries 1\nconstraints bounds\n")
    c = files.Config("cfg")
    assert c.delta_bounds == eval(text, {"np": np})   # noqa: S307 -- the reference's semantics, test input
    assert c.sigma_bounds == [[0.01, 4.5]]


@pytest.mark.parametrize("text", ["[__import__('os').getcwd()]", "[open('x')]", "[x for x in range(3)]",
                                  "[np.load('f')]", "['a', 1]"])
def test_config_list_refuses_code(text):
    """What eval() would execute (calls, names, comprehensions, strings) is refused with
    a ValueError naming the expression, instead of being run."""
    with pytest.raises(ValueError, match="unsupported expression"):
        files.literal(text)


def test_missing_key_exits(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    (tmp_path / "cfg").write_text("beliefs b\ninputs i\n")
    with pytest.raises(SystemExit):
        files.Config("cfg")


def test_setup_state_matches_reference(toysim_dir):
    """All_Data shuffle/scale/split, H and the RNG stream after setup (G6)."""
    z = np.load(os.path.join(GOLD, "host_toysim_seed0.npz"))
    np.random.seed(0)
    c = files.Config("toy-sim_config")
    b = files.Beliefs(c.beliefs)
    par = model.Hyperparams(b)
    basis = model.Basis(b)
    tv = model.TV_config(*c.tv_config)
    ad = model.All_Data(c.inputs, c.outputs, tv, b, par, True, True)
    np.testing.assert_array_equal(ad.x_full, z["x_full"])
    np.testing.assert_array_equal(ad.y_full, z["y_full"])
    np.testing.assert_array_equal(ad.minmax, z["minmax"])
    XT, fT = ad.choose_T()
    XV, _ = ad.choose_V()
    np.testing.assert_array_equal(XT, z["XT"])
    np.testing.assert_array_equal(fT, z["fT"])
    np.testing.assert_array_equal(XV, z["XV"])
    np.testing.assert_array_equal(basis.design_matrix(XT), z["HT"])
    # the reference's setup() consumes no further random numbers
    np.testing.assert_array_equal(np.random.random_sample(10), z["next_random"])


def test_final_beliefs_roundtrip(toysim_dir):
    import types
    c = files.Config("toy-sim_config")
    b = files.Beliefs(c.beliefs)
    E = types.SimpleNamespace(config=c, tv_conf=types.SimpleNamespace(no_of_trains=2),
                              par=types.SimpleNamespace(beta=np.array([0.5, 2.8]),
                                                        delta=np.array([0.2, 0.16]),
                                                        sigma=np.float64(0.61), nugget=0.03),
                              all_data=types.SimpleNamespace(input_minmax=[[np.float64(0.01), 0.98],
                                                                           [0.013, 0.99]]))
    b.final_beliefs(E, final=True)
    b2 = files.Beliefs("toy-sim_beliefs-2f")
    assert b2.delta == [0.2, 0.16] and b2.beta == [0.5, 2.8] and b2.sigma == 0.61
    assert b2.input_minmax == [[0.01, 0.98], [0.013, 0.99]]
    assert b2.active_index == [0, 1] and b2.output_index == 0


def test_concurrent_tries_policy(monkeypatch):
    """Two tries in flight for 4096 <= n <= 32768 and >= 2 tries; GPEMU_CONCURRENT_TRIES
    forces k (capped by the tries); never with a collective objective (host logic only)."""
    from gp_emu_uqsa_amd import distributed, optimize

    class D:
        def __init__(self, n):
            self.inputs = np.zeros((n, 2))

    def conc(n, tries):
        o = optimize.Optimize.__new__(optimize.Optimize)
        o.data = D(n)
        return o._concurrency(tries)

    monkeypatch.delenv("GPEMU_CONCURRENT_TRIES", raising=False)
    assert conc(16384, 4) == 2 and conc(4096, 2) == 2
    assert conc(2048, 4) == 1 and conc(65536, 4) == 1 and conc(16384, 1) == 1
    monkeypatch.setenv("GPEMU_CONCURRENT_TRIES", "3")
    assert conc(100, 5) == 3 and conc(100, 2) == 2
    monkeypatch.setenv("GPEMU_CONCURRENT_TRIES", "1")
    assert conc(16384, 4) == 1
    monkeypatch.setattr(distributed, "_OBJECTIVE", object())
    monkeypatch.setenv("GPEMU_CONCURRENT_TRIES", "4")
    assert conc(16384, 4) == 1
