import sys, time
import numpy as np
sys.path.insert(0, '.')
from gp_emu_uqsa_amd import native, synthetic
n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
ctx = native.Context(0)
X, f, H = synthetic.problem(n, 10, seed=0)
ctx.set_data(X, f, H)
hp = np.concatenate([np.ones(10), [1e-3, 1.0]])
for _ in range(4):
    t = time.perf_counter(); r = ctx.objective(0, 0, hp, want_grad=False); print("vo", time.perf_counter() - t, flush=True)
