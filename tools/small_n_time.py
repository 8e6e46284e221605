"""Per-evaluation wall time at small n (dev tool): where the typical emulator sizes
(n in the hundreds to a few thousand) spend an LLH+gradient evaluation -- GPU phases
against the host-side wall time of gpe_objective.
usage: python tools/small_n_time.py [d]"""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from gp_emu_uqsa_amd import native, synthetic  # noqa: E402

d = int(sys.argv[1]) if len(sys.argv) > 1 else 10
ctx = native.Context(0)
for n in (60, 100, 128, 200, 300, 384, 500, 640, 1024, 2048, 4096, 8192):
    X, f, H = synthetic.problem(n, d, seed=0)
    ctx.set_data(X, f, H)
    hp = np.concatenate([np.ones(d), [1e-3, 1.0]])
    for _ in range(3):
        ctx.objective(0, 0, hp)
    reps = 20
    t = time.perf_counter()
    for _ in range(reps):
        ctx.objective(0, 0, hp)
    wall = (time.perf_counter() - t) / reps * 1e3
    t = time.perf_counter()
    for _ in range(reps):
        ctx.objective(0, 0, hp, want_grad=False)
    wall_v = (time.perf_counter() - t) / reps * 1e3
    ctx.set_profiling(True)
    ctx.objective(0, 0, hp)
    ph = ctx.phase_times()
    g = ctx.gemm_stats()
    ctx.set_profiling(False)
    print(f"n {n:5d}: LLH+grad {wall:7.3f} ms wall, value only {wall_v:7.3f} ms; GPU phases "
          + " ".join(f"{k} {v:.3f}" for k, v in ph.items()) + f"; GEMM launches {g.get('launches')}", flush=True)
