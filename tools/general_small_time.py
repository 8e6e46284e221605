"""Host wall time of the general path (GPEMU_TINY=0) at n = 300 and 500, d = 10 (dev tool:
the baseline of the one-launch n <= 512 objective)."""
import os, sys, time
os.environ["GPEMU_TINY"] = "0"
sys.path.insert(0, ".")
import numpy as np
from gp_emu_uqsa_amd import native, synthetic
ctx = native.Context(0)
for n in (300, 500):
    X, f, H = synthetic.problem(n, 10, seed=0)
    ctx.set_data(X, f, H)
    hp = np.concatenate([np.ones(10), [1e-3, 1.0]])
    for want in (True, False):
        for _ in range(5): ctx.objective(0, 0, hp, want_grad=want)
        t = time.perf_counter()
        for _ in range(50): ctx.objective(0, 0, hp, want_grad=want)
        print("general path n", n, "grad" if want else "value", round((time.perf_counter() - t) / 50 * 1e3, 3), "ms", flush=True)
