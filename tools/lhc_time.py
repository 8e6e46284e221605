"""oLHC selection at history-matching scale: gpe_lhc_maximin vs the reference's
per-design scipy pdist + argmin (timed on 2 designs, scaled to N).
usage: python tools/lhc_time.py N n dim ne"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gp_emu_uqsa_amd import native  # noqa: E402
from oracle.lhc_oracle import lhc_maximin_ref  # noqa: E402

N, n, dim, ne = (int(a) for a in sys.argv[1:5])
rng = np.random.RandomState(0)
xs = (np.argsort(rng.rand(N, n, dim), axis=1) + rng.rand(N, n, dim)) / n
fe = rng.rand(ne, dim) if ne else None
ctx = native.Context(0)
ctx.lhc_maximin(xs[:2], fe)
t0 = time.perf_counter()
got = ctx.lhc_maximin(xs, fe)
t_gpu = time.perf_counter() - t0
t0 = time.perf_counter()
ref = lhc_maximin_ref(xs[:2], fe)
t_cpu = (time.perf_counter() - t0) / 2 * N
m = n + ne
pairs = N * (n * (n - 1) / 2 + n * ne) + ne * (ne - 1) / 2
print(json.dumps({"N": N, "n": n, "dim": dim, "ne": ne, "gpu_s": t_gpu, "cpu_ref_s_scaled": t_cpu,
                  "speedup": t_cpu / t_gpu, "gpu_pairs_per_s": pairs / t_gpu,
                  "match_first2": bool(np.array_equal(got[:2], ref))}))
