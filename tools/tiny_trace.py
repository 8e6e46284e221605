"""n <= 128 objective under rocprofv3 --kernel-trace (dev tool): 200 LLH + gradient
evaluations and 200 value-only at n = 128, d = 10.  usage: python tools/tiny_trace.py [n]"""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from gp_emu_uqsa_amd import native, synthetic  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 128
ctx = native.Context(0)
X, f, H = synthetic.problem(n, 10, seed=0)
ctx.set_data(X, f, H)
hp = np.concatenate([np.ones(10), [1e-3, 1.0]])
for want in (True, False):
    ctx.objective(0, 0, hp, want_grad=want)
    t = time.perf_counter()
    for _ in range(200):
        ctx.objective(0, 0, hp, want_grad=want)
    print("grad" if want else "value", (time.perf_counter() - t) / 200 * 1e3, "ms", flush=True)
