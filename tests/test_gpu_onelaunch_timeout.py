"""A workgroup wait that runs out in the one-launch objectives (k_tiny, n <= 128; k_snb,
128 < n <= 512) is an error of the call (RuntimeError, GPE_ERR_HIP), never "matrix not
positive definite" (which the optimiser would take as the reference's LinAlgError and skip
the point, `_emulatoroptimise.py:374-376,489-491`) and never a result built from another
call's partial sums.  The dev switch GPEMU_DEBUG_SKIP_WAIT=h makes helper workgroup h give
up its first wait as a timeout would (`tiny_wait`'s skip): it raises the abort flag, the
other waiters stop, its partial sums never carry the call's tag, and the host refuses the
call.  A context without the switch on the same data then gives the oracle's result."""
import numpy as np
import pytest

from gp_emu_uqsa_amd import native
from oracle import gp_oracle as orc

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,d", [(100, 3), (300, 10)], ids=["tiny", "snb"])
def test_helper_wait_timeout_is_an_error(n, d):
    X, f, H = orc.synthetic_problem(n, d, seed=7)
    hp = np.concatenate([np.linspace(0.4, 0.8, d), [1e-3, 1.1]])
    mp = pytest.MonkeyPatch()
    mp.setenv("GPEMU_DEBUG_SKIP_WAIT", "2")
    bad = native.Context(0)
    mp.undo()
    good = native.Context(0)
    try:
        bad.set_data(X, f, H)
        good.set_data(X, f, H)
        ref = orc.objective_fast(X, f, H, hp, orc.GP4ML, orc.STD, True)
        for _ in range(2):   # (the call after a failed one zeroes the sync words and fails the same way)
            with pytest.raises(RuntimeError, match="timed out|did not finish"):
                bad.objective(orc.GP4ML, orc.STD, hp)
        if n <= 128:   # the value alone has no helper wait in k_tiny: it still runs
            v, _, _ = bad.objective(orc.GP4ML, orc.STD, hp, want_grad=False)
            assert abs(v - ref[0]) <= 1e-10 * abs(ref[0])
        else:          # k_snb's helpers wait for every panel: the value fails too
            with pytest.raises(RuntimeError, match="timed out"):
                bad.objective(orc.GP4ML, orc.STD, hp, want_grad=False)
        llh, g, _ = good.objective(orc.GP4ML, orc.STD, hp)
        assert abs(llh - ref[0]) <= 1e-10 * abs(ref[0])
        scale = np.abs(ref[1]) + np.max(np.abs(ref[1]))
        assert np.all(np.abs(g - ref[1]) <= 1e-7 * scale)
    finally:
        bad.close()
        good.close()
