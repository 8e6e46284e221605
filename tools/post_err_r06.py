"""Diagonal posterior variance error of precision 32 against precision 64 (dev tool, round 6):
the fp32 GEMM (GPEMU_OZAKI=0) and the int8 product at several operand widths
(GPEMU_OZAKI_POST32_BITS), same data as tests/test_gpu_posterior.py."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(env, n, d, m, seed):
    from gp_emu_uqsa_amd import native, synthetic
    for k, v in env.items():
        os.environ[k] = v
    c = native.Context(0)
    X, f, H = synthetic.problem(n, d, seed=seed)
    c.set_data(X, f, H)
    c.factor(native.KERNEL_STD, np.full(d, 0.7), 1e-3, 1.0, 0.0)
    beta = c.beta()
    xs = synthetic.design(m, d, seed=seed + 1)
    hs = synthetic.linear_basis(xs)
    _, v64 = c.posterior(xs, hs, beta, 0.9, full_var=False, precision=64)
    _, v32 = c.posterior(xs, hs, beta, 0.9, full_var=False, precision=32)
    c.close()
    return v64, v32


def main():
    for (n, d) in ((2200, 5), (16384, 10)):
        ref, _ = run({"GPEMU_OZAKI": "0"}, n, d, 9000, 5)
        rec = {"n": n, "d": d}
        _, v = run({"GPEMU_OZAKI": "0"}, n, d, 9000, 5)
        rec["fp32_gemm"] = float(np.max(np.abs(v - ref)))
        for bits in ("24", "26", "28"):
            v64, v = run({"GPEMU_OZAKI": "1", "GPEMU_OZAKI_POST32_BITS": bits}, n, d, 9000, 5)
            rec["int8_%s" % bits] = float(np.max(np.abs(v - ref)))
            rec["int8_64_vs_fp64"] = float(np.max(np.abs(v64 - ref)))
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
