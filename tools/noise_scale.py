"""noise_fit's estimation step at scale -- dev/measurement tool.

For n training points in d=2 (alt-nugget kernel with a per-point r, as noise_fit
trains it) and m = n prediction points (noise_fit estimates at the training inputs),
times one estimation step: the full m x m posterior covariance, its Cholesky and the
`samples` draws L u_j (gpe_noise_sample), and the same through the separate entries
(gpe_posterior full, host copy, gpe_cholesky, host GEMM) for comparison.
The reference does this with three scipy LU solves of the n x n A, np.linalg.cholesky
and a Python loop of `samples` matrix-vector products.
usage: python tools/noise_scale.py [--points 4096 8192] [--samples 200]
"""
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
    ap.add_argument("--points", type=int, nargs="+", default=[4096, 8192, 16384])
    ap.add_argument("--samples", type=int, default=200)
    args = ap.parse_args()
    from gp_emu_uqsa_amd import native
    ctx = native.Context(0)
    for n in args.points:
        rs = np.random.RandomState(1)
        x = rs.uniform(size=(n, 2))
        f = 3 * x[:, 0] ** 3 + np.exp(np.cos(10 * x[:, 1]) * np.cos(5 * x[:, 0]) ** 2)
        r = (0.5 * x[:, 1] * (np.cos(6 * x[:, 0]) ** 2 + 0.1)) ** 2
        f = f + np.sqrt(r) * rs.randn(n)
        ctx.set_data(x, f, np.ones((n, 1)), r)
        delta, nu, sig, beta = np.array([0.3, 0.25]), 1e-5, 1.2, np.array([2.0])
        ctx.factor(native.KERNEL_ALT_NUG, delta, nu, 1.0, 1.0)
        U = rs.randn(args.samples, n)
        H = np.ones((n, 1))
        ctx.noise_sample(x, H, beta, sig, f, U, r_new=r, r_scale=1 / sig ** 2)   # warm-up
        t0 = time.perf_counter()
        mean, z = ctx.noise_sample(x, H, beta, sig, f, U, r_new=r, r_scale=1 / sig ** 2)
        t_fused = time.perf_counter() - t0
        out = {"n": n, "m": n, "samples": args.samples, "noise_sample_s": round(t_fused, 4)}
        if n <= 8192:
            t0 = time.perf_counter()
            m2, V = ctx.posterior(x, H, beta, sig, full_var=True)
            V[np.diag_indices(n)] += r
            L = ctx.cholesky(V, want=("L",))["L"]
            z2 = np.sum(0.5 * ((f - m2)[:, None] - L.dot(U.T)) ** 2, axis=1)
            out["separate_entries_s"] = round(time.perf_counter() - t0, 4)
            out["max_rel_diff"] = float(np.max(np.abs(z2 - z) / z2))
        print(json.dumps(out), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
