"""Concurrent multistart tries (optimize.Optimize._run_concurrent): tries dealt over
host threads, each on its own context of the same GPU, give exactly the sequential
result -- every chain is the same deterministic computation, whichever Cholesky
schedule (group launches or one launch per step) each call picks."""
import os
import threading

import numpy as np
import pytest

import gp_emu_uqsa_amd as g
from gp_emu_uqsa_amd import native
from oracle import gp_oracle as orc

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


@pytest.mark.parametrize("n", [400, 5200])
@pytest.mark.parametrize("mucm", ["F", "T"])
def test_concurrent_tries_equal_sequential(tmp_path, monkeypatch, capsys, mucm, n):
    """n = 5200 (41 tile columns): column groups of width 2, so a lone try runs the group
    launches and tries in flight together the per-step launches."""
    monkeypatch.chdir(tmp_path)
    _files(n=n, mucm=mucm)
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


def test_three_contexts_concurrent_group_launches(monkeypatch):
    """Three contexts evaluating at once on one GPU, two of them forced to the group
    launches (list positions claimed by ticket, in-launch hand-offs) and the third on
    `auto` (which then takes the per-step launches), at n = 10300 (81 tile columns:
    groups of width 4, 2 and 1).  No error, no timed-out wait, and every result
    bit-identical to the same context's evaluation alone."""
    X, f, H = orc.synthetic_problem(10300, 10, seed=21)
    hps = [np.concatenate([np.linspace(0.7 + 0.1 * k, 1.5, 10), [2e-3, 0.9 + 0.05 * k]]) for k in range(3)]
    ctxs = []
    th = []
    try:
        for k in range(3):
            if k < 2:
                monkeypatch.setenv("GPEMU_POTRF", "group")
            else:
                monkeypatch.delenv("GPEMU_POTRF", raising=False)
            c = native.Context(0)
            ctxs.append(c)
            c.set_data(X, f, H)
        alone = []
        for c, hp in zip(ctxs, hps):
            v = c.objective(orc.GP4ML, orc.STD, hp, want_grad=False)
            gr = c.objective(orc.GP4ML, orc.STD, hp)
            alone.append((v, gr))
        res = [[] for _ in range(3)]
        errs = []
        bar = threading.Barrier(3)

        def run(k):
            try:
                bar.wait()
                for rep in range(3):
                    res[k].append((ctxs[k].objective(orc.GP4ML, orc.STD, hps[k], want_grad=False),
                                   ctxs[k].objective(orc.GP4ML, orc.STD, hps[k])))
            except Exception as e:   # noqa: BLE001 -- reported below
                errs.append((k, e))

        th = [threading.Thread(target=run, args=(k,)) for k in range(3)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=300)
        assert not any(t.is_alive() for t in th), "concurrent evaluations did not finish"
        assert not errs, errs
        for k in range(3):
            (v0, gr0) = alone[k]
            for v, gr in res[k]:
                assert v[0] == v0[0] and v[2] == v0[2], (k, v, v0)
                assert gr[0] == gr0[0] and gr[2] == gr0[2], (k, gr[0], gr0[0])
                assert np.array_equal(gr[1], gr0[1]), (k, gr[1] - gr0[1])
    finally:
        # a context whose thread is still inside an objective call is left open (its
        # workspaces may still be in use): a hang is then reported by the assertion
        # above, not turned into a use-after-free
        busy = {k for k, t in enumerate(th) if t.is_alive()}
        for k, c in enumerate(ctxs):
            if k not in busy:
                c.close()
