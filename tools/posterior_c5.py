"""BASELINE configs[4]: posterior mean + diagonal variance at m
prediction points (default 1e6) for an n=16384, d=10 emulator -- dev tool.
Prints one JSON line: seconds for gpe_factor + gpe_posterior(full_var=0) and
points/s.  usage: python tools/posterior_c5.py [--points 16384] [--m 1000000]"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--points", type=int, default=16384)
    ap.add_argument("--dims", type=int, default=10)
    ap.add_argument("--m", type=int, default=1000000)
    ap.add_argument("--precision", type=int, default=32)
    args = ap.parse_args()
    from gp_emu_uqsa_amd import native, synthetic
    X, f, H = synthetic.problem(args.points, args.dims, seed=0)
    xs = synthetic.design(args.m, args.dims, seed=7)
    hs = synthetic.linear_basis(xs)
    ctx = native.Context(int(os.environ.get("LOCAL_RANK", "0")))
    ctx.set_data(X, f, H)
    delta, nu, sigma = np.ones(args.dims), 1e-3, 1.0
    t0 = time.perf_counter()
    ctx.factor(native.KERNEL_STD, delta, nu, 1.0, 0.0)
    beta = ctx.beta()
    t1 = time.perf_counter()
    mean, var = ctx.posterior(xs, hs, beta, sigma, full_var=False, precision=args.precision)
    t2 = time.perf_counter()
    print(json.dumps({"config": f"C5 posterior: n={args.points} d={args.dims} m={args.m} fp{args.precision} diag var",
                      "factor_s": t1 - t0, "posterior_s": t2 - t1, "points_per_s": args.m / (t2 - t1),
                      "mean_checksum": float(np.sum(mean)), "var_min": float(np.min(var)),
                      "var_max": float(np.max(var))}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
