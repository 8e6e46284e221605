"""Aggregate LLH+grad throughput with k independent evaluations in flight on one GPU
(dev tool): k contexts (own HIP stream and buffers), one host thread each (ctypes
drops the GIL during library calls), each evaluating the objective `reps` times
at its own hyperparameters, as concurrent multistart tries would.
usage: python tools/concurrent_evals.py [n] [k] [reps] [stagger_ms]
stagger_ms: try i starts i * stagger_ms later (so the tries' phases are offset); the
rate then discounts the stagger (k * reps / (span - (k-1) * stagger)), and each
try's own rate is printed."""
import sys
import threading
import time

import numpy as np

sys.path.insert(0, ".")
from gp_emu_uqsa_amd import native, synthetic  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
k = int(sys.argv[2]) if len(sys.argv) > 2 else 2
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
stagger = float(sys.argv[4]) / 1e3 if len(sys.argv) > 4 else 0.0
d = 10
X, f, H = synthetic.problem(n, d, seed=0)
ctxs = []
for i in range(k):
    c = native.Context(0)
    c.set_data(X, f, H)
    ctxs.append(c)
hps = [np.concatenate([np.full(d, 1.0 + 0.05 * i), [1e-3, 1.0]]) for i in range(k)]
for c, hp in zip(ctxs, hps):
    c.objective(0, 0, hp)
res = [None] * k
span = [[0.0, 0.0] for _ in range(k)]


def work(i):
    time.sleep(i * stagger)
    span[i][0] = time.perf_counter()
    for _ in range(reps):
        res[i] = ctxs[i].objective(0, 0, hps[i])
    span[i][1] = time.perf_counter()


for trial in range(2):
    th = [threading.Thread(target=work, args=(i,)) for i in range(k)]
    t0 = time.perf_counter()
    for t in th:
        t.start()
    for t in th:
        t.join()
    dt = time.perf_counter() - t0 - (k - 1) * stagger
    own = " ".join(f"{reps / (e - b):.2f}" for b, e in span)
    print(f"k={k} n={n} stagger {stagger * 1e3:.0f} ms: {k * reps} evals -> {k * reps / dt:.2f} evals/s "
          f"({dt / reps * 1e3:.1f} ms per round of {k}); per try {own}", flush=True)
single = native.Context(0)
single.set_data(X, f, H)
single.objective(0, 0, hps[0])
t0 = time.perf_counter()
for _ in range(reps):
    r = single.objective(0, 0, hps[0])
dt = time.perf_counter() - t0
print(f"sequential: {reps / dt:.2f} evals/s; llh match {abs(r[0] - res[0][0])}", flush=True)
