"""K-build A/B (dev tool): k_pairs (d-sum serial in one lane) against k_pairs_shfl
(GPEMU_KPAIRS=shuffle: d-sum over 8 lanes + shuffle tree) at n=16384, d=10; the
K-build phase time of 5 objective evaluations each (profiling events)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CODE = r"""
import sys, numpy as np
sys.path.insert(0, %r)
from gp_emu_uqsa_amd import native, synthetic
c = native.Context(0)
X, f, H = synthetic.problem(16384, 10, seed=0)
c.set_data(X, f, H)
hp = np.concatenate([np.ones(10), [1e-3, 1.0]])
c.set_profiling(True)
ts = []
for _ in range(6):
    c.objective(0, 0, hp, want_grad=False)
    ts.append(c.phase_times()["kbuild"])
print("kbuild_ms", sorted(ts[1:])[2])
""" % ROOT
for mode in ("default", "shuffle"):
    env = dict(os.environ)
    env.pop("GPEMU_KPAIRS", None)
    if mode == "shuffle":
        env["GPEMU_KPAIRS"] = "shuffle"
    r = subprocess.run([sys.executable, "-c", CODE], env=env, capture_output=True, text=True)
    print(mode, r.stdout.strip(), r.stderr.strip()[-300:], flush=True)
