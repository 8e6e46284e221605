"""Quick timing of one objective eval (LLH+grad) at size n (dev tool)."""
import sys, time
import numpy as np
sys.path.insert(0, '.')
from gp_emu_uqsa_amd import native
from gp_emu_uqsa_amd import synthetic
n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
d = int(sys.argv[2]) if len(sys.argv) > 2 else 10
ctx = native.Context(0)
X, f, H = synthetic.problem(n, d, seed=0)
ctx.set_data(X, f, H)
hp = np.concatenate([np.ones(d), [1e-3, 1.0]])
ctx.objective(0, 0, hp)
ts = []
for _ in range(3):
    t = time.perf_counter(); r = ctx.objective(0, 0, hp); ts.append(time.perf_counter() - t)
print("n", n, "llh", r[0], "eval s", ts, flush=True)
ctx.set_profiling(True)
ctx.objective(0, 0, hp)
print("phases ms", ctx.phase_times())
g = ctx.gemm_stats(); print("gemm", g, "TF/s", g['flops'] / g['ms'] / 1e9)
ctx.set_profiling(False)
ctx.objective(0, 0, hp, want_grad=False)
tv = []
for _ in range(3):
    t = time.perf_counter(); rv = ctx.objective(0, 0, hp, want_grad=False); tv.append(time.perf_counter() - t)
print("value-only s", tv, "llh", rv[0], "rel diff vs grad path", abs(rv[0] - r[0]) / abs(r[0]), flush=True)
