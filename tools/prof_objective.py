"""Run K objective evals at size n for rocprofv3 (dev tool)."""
import sys
import numpy as np
sys.path.insert(0, '.')
from gp_emu_uqsa_amd import native
from gp_emu_uqsa_amd import synthetic
n = int(sys.argv[1]); d = int(sys.argv[2]); reps = int(sys.argv[3])
ctx = native.Context(0)
X, f, H = synthetic.problem(n, d, seed=0)
ctx.set_data(X, f, H)
hp = np.concatenate([np.ones(d), [1e-3, 1.0]])
for _ in range(reps):
    r = ctx.objective(0, 0, hp)
print("llh", r[0])
