"""Value-only objective evaluations at n = 16384, d = 10 on one GPU (dev tool: the single-GPU
side of a kernel-trace comparison with tools/dist_objective.py --loopback 1).
usage: python tools/value_only_evals.py [reps]"""
import sys

import numpy as np

sys.path.insert(0, ".")
from gp_emu_uqsa_amd import native, synthetic  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
ctx = native.Context(0)
X, f, H = synthetic.problem(16384, 10, seed=0)
ctx.set_data(X, f, H)
hp = np.concatenate([np.ones(10), [1e-3, 1.0]])
for _ in range(reps):
    print(ctx.objective(0, 0, hp, want_grad=False)[0], flush=True)
