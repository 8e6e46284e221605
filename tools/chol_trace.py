"""Fused-Cholesky chain timeline from the GEMM_TRACE dev build (dev tool).
  hipcc ... -DGEMM_TRACE -o gp_emu_uqsa_amd/libgpemu_trace.so
  GPEMU_LIB=gp_emu_uqsa_amd/libgpemu_trace.so python tools/chol_trace.py [n]
Per column step (us): diagonal workgroup update / factor / publish, first panel
workgroup update / wait / multiply, and the gap to the next step's diagonal start."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gp_emu_uqsa_amd import native, synthetic  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
ctx = native.Context(0)
X, f, H = synthetic.problem(n, 10, seed=0)
ctx.set_data(X, f, H)
hp = np.concatenate([np.ones(10), [1e-3, 1.0]])
for _ in range(2):
    ctx.objective(0, 0, hp)
lib = native.load_library()
buf = (ctypes.c_uint64 * (8 * 4096))()
assert lib.gpe_debug_trace(buf, 8 * 4096) == 0
NB = (n + 127) // 128
t = np.array(buf[:8 * NB], dtype=np.float64).reshape(NB, 8) / 100.0   # us
rows = []
for k in range(NB):
    d0, d1, d2, d3, p0, p1, p2, p3 = t[k]
    nxt = t[k + 1][0] - max(d3, p3 if p3 > 0 else d3) if k + 1 < NB else 0
    rows.append((k, d1 - d0, d2 - d1, d3 - d2, (p1 - p0) if p0 else 0, (p2 - p1) if p0 else 0,
                 (p3 - p2) if p0 else 0, (p2 - d3) if p0 else 0, nxt, (t[k + 1][0] - d0) if k + 1 < NB else 0))
if os.environ.get("PANEL_PHASES"):   # libgpemu_trace built with -DPANEL_PHASES: slot 5 = staged
    first = [t[k][5] - t[k][6] for k in range(NB - 1)]
    second = [t[k][7] - t[k][5] for k in range(NB - 1)]
    print("panel substitution: staging %.1f us, products + stores %.1f us (mean over steps)"
          % (np.mean(first[1:]), np.mean(second[1:])))
print(" k   d.upd  d.fac  d.pub  p.upd  p.wait  p.mul  seen-pub  gap   step")
show = sorted(set(list(range(min(3, NB))) + list(range(60, min(63, NB))) + list(range(100, min(103, NB)))
                  + list(range(max(0, NB - 6), NB))))
for k in show:
    r = rows[k]
    print("%3d " % r[0] + " ".join("%6.1f" % v for v in r[1:]))
segs = ((1, 48), (48, 88), (88, NB - 1)) if NB >= 96 else ((1, NB - 1),)
for lo, hi in segs:
    seg = np.array([r[1:] for r in rows[lo:hi]])
    if len(seg):
        print("mean over steps %3d..%3d:" % (lo, hi - 1), " ".join("%6.1f" % v for v in seg.mean(axis=0)))
