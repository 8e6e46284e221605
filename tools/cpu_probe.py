"""Where the CPU reference's time goes on this host (dev tool): the op-for-op oracle
objective at n (default 4096) under cProfile, with the BLAS limited as bench.py does,
and one n x n np.linalg.solve with the real Cholesky factor and with a synthetic one."""
import cProfile
import os
import pstats
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import gp_oracle as orc  # noqa: E402
from threadpoolctl import threadpool_info, threadpool_limits  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
threads = int(sys.argv[2]) if len(sys.argv) > 2 else 16
print("threadpools before:", [(i["internal_api"], i["num_threads"]) for i in threadpool_info()], flush=True)
with threadpool_limits(limits=threads, user_api="blas"):
    print("threadpools:", [(i["internal_api"], i["num_threads"]) for i in threadpool_info()], flush=True)
    d = 10
    X, f, H = orc.synthetic_problem(n, d, seed=0)
    hp = np.concatenate([np.ones(d), [1e-3, 1.0]])
    pr = cProfile.Profile()
    pr.enable()
    t = time.time()
    orc.objective_ref(X, f, H, hp, orc.GP4ML, orc.STD, True)
    print("objective_ref total", time.time() - t, flush=True)
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(6)
    A, _ = orc.make_A_ref(X, hp[:d], hp[d], orc.STD, None, 1.0)
    L = np.linalg.cholesky(A)
    B = np.random.rand(n, n)
    for name, M in (("real L", L), ("synthetic L", np.tril(np.random.RandomState(0).uniform(-1, 1, (n, n))) / n + np.eye(n))):
        for _ in range(2):
            t = time.time()
            np.linalg.solve(M, B)
            print(name, "solve n x n", time.time() - t, flush=True)
