"""Concurrent multistart tries (optimize.Optimize._run_concurrent): tries dealt over
host threads, each on its own context of the same GPU, give exactly the sequential
result -- every chain is the same deterministic computation."""
import os

import numpy as np
import pytest

import gp_emu_uqsa_amd as g
from gp_emu_uqsa_amd import native

pytestmark = pytest.mark.gpu


def _files(n=400, d=3, tries=4, mucm="F"):
    rs = np.random.RandomState(11)
    X = rs.uniform(size=(n, d))
    f = np.sin(3 * X[:, 0]) + X[:, 1] ** 2 - 0.5 * X[:, 2] + 0.01 * rs.randn(n)
    np.savetxt("c_input", X)
    np.savetxt("c_output", f)
    with open("c_config", "w") as fh:
        fh.write("beliefs c_beliefs\ninputs c_input\noutputs c_output\ntv_config 10 0 0\n"
                 f"delta_bounds [ ]\nnugget_bounds [ ]\nsigma_bounds [ ]\ntries {tries}\n"
                 "constraints bounds\n")
    with open("c_beliefs", "w") as fh:
        fh.write("active all\noutput 0\nbasis_str 1.0 x x x\nbasis_inf NA 0 1 2\nbeta 1.0 1.0 1.0 1.0\n"
                 f"delta 1.0 1.0 1.0\nsigma 1.0\nnugget 0.001\nfix_nugget F\nmucm {mucm}\n")


@pytest.mark.parametrize("mucm", ["F", "T"])
def test_concurrent_tries_equal_sequential(tmp_path, monkeypatch, capsys, mucm):
    monkeypatch.chdir(tmp_path)
    _files(mucm=mucm)
    out = {}
    for k in ("1", "2", "3"):
        monkeypatch.setenv("GPEMU_CONCURRENT_TRIES", k)
        np.random.seed(5)
        E = g.setup("c_config", datashuffle=True)
        g.train(E, auto=True)
        out[k] = (np.array(E.par.delta), float(E.par.nugget), float(E.par.sigma), np.array(E.par.beta),
                  open("c_beliefs-0f").read())
    for k in ("2", "3"):
        assert np.array_equal(out[k][0], out["1"][0])
        assert out[k][1] == out["1"][1] and out[k][2] == out["1"][2]
        assert np.array_equal(out[k][3], out["1"][3])
        assert out[k][4] == out["1"][4]
    assert len(native.worker_contexts(3)) == 3


def test_bound_context_routes_objective(tmp_path):
    """default_context() inside bind_context is the bound one, outside the default."""
    base = native.default_context()
    other = native.worker_contexts(2)[1]
    assert other is not base
    with native.bind_context(other):
        assert native.default_context() is other
    assert native.default_context() is base
