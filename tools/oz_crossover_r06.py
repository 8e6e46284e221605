"""Where the int8 products start paying (dev tool, round 6): one LLH + gradient's phases and wall
time with GPEMU_OZAKI=1 / 0 at several n (two contexts per n), and the diagonal posterior's time
at m = 50000 points (precision 64 and 32).  usage: python tools/oz_crossover_r06.py"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def ctx_with(native, oz):
    os.environ["GPEMU_OZAKI"] = oz
    try:
        return native.Context(0)
    finally:
        os.environ.pop("GPEMU_OZAKI", None)


def main():
    from gp_emu_uqsa_amd import native, synthetic
    for n in (2048, 3072, 4096, 6144, 8192, 12288):
        X, f, H = synthetic.problem(n, 10, seed=0)
        hp = np.concatenate([np.ones(10), [1e-3, 1.0]])
        xs = synthetic.design(50000, 10, seed=3)
        hs = synthetic.linear_basis(xs)
        rec = {"n": n}
        for oz in ("1", "0"):
            c = ctx_with(native, oz)
            c.set_data(X, f, H)
            c.objective(0, 0, hp)
            ts = []
            for _ in range(5):
                t = time.perf_counter()
                c.objective(0, 0, hp)
                ts.append(time.perf_counter() - t)
            c.set_profiling(True)
            c.objective(0, 0, hp)
            ph = c.phase_times()
            c.set_profiling(False)
            rec["oz" + oz] = {"eval_ms": 1e3 * min(ts), "trtri": ph["trtri"], "inverse": ph["inverse"]}
            c.factor(native.KERNEL_STD, np.ones(10), 1e-3, 1.0, 0.0)
            beta = c.beta()
            for prec in (64, 32):
                c.posterior(xs[:1000], hs[:1000], beta, 1.0, full_var=False, precision=prec)
                t = time.perf_counter()
                c.posterior(xs, hs, beta, 1.0, full_var=False, precision=prec)
                rec["oz" + oz]["post%d_ms" % prec] = 1e3 * (time.perf_counter() - t)
            c.close()
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
