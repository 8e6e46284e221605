"""Accuracy of the int8-emulated A^-1 / top-TRTRI products (gpemu_ozaki.hpp) against the fp64
path of the same library (GPEMU_OZAKI=0) and, at n <= 4096, the oracle's LAPACK evaluation
(dev tool; prints one JSON line per (n, moduli)).  usage: python tools/ozaki_accuracy.py"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def ctx_with(native, **env):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update({k: str(v) for k, v in env.items()})
    try:
        return native.Context(0)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def main():
    from gp_emu_uqsa_amd import native, synthetic
    from oracle import gp_oracle as orc
    for n in (4096, 16384):
        X, f, H = synthetic.problem(n, 10, seed=0)
        hp = np.concatenate([np.ones(10), [1e-3, 1.0]])
        ref = fp = None
        c64 = ctx_with(native, GPEMU_OZAKI=0)
        c64.set_data(X, f, H)
        l64, g64, _ = c64.objective(native.GP4ML, native.KERNEL_STD, hp)
        c64.close()
        if n <= 4096:
            ref = orc.objective_fast(X, f, H, hp, orc.GP4ML, orc.STD, True)
        for nmod in (16, 14, 12):
            c = ctx_with(native, GPEMU_OZAKI=1, GPEMU_OZAKI_MODULI=nmod)
            c.set_data(X, f, H)
            l, g, _ = c.objective(native.GP4ML, native.KERNEL_STD, hp)
            c.set_profiling(True)
            c.objective(native.GP4ML, native.KERNEL_STD, hp)
            ph = c.phase_times()
            oz = c.ozaki_stats()
            c.set_profiling(False)
            c.close()
            scale = np.abs(g64) + np.max(np.abs(g64))
            rec = {"n": n, "moduli": nmod, "llh_rel_vs_fp64": abs(l - l64) / abs(l64),
                   "grad_max_rel_vs_fp64": float(np.max(np.abs(g - g64) / scale)),
                   "trtri_ms": ph["trtri"], "inverse_ms": ph["inverse"], "total_ms": ph["total"],
                   "int8_tops": oz["int8_ops"] / (oz["ms"] * 1e-3) / 1e12 if oz["ms"] else None}
            if ref is not None:
                sr = np.abs(ref[1]) + np.max(np.abs(ref[1]))
                rec["llh_rel_vs_oracle"] = abs(l - ref[0]) / abs(ref[0])
                rec["grad_max_rel_vs_oracle"] = float(np.max(np.abs(g - ref[1]) / sr))
                rec["fp64_path_grad_max_rel_vs_oracle"] = float(np.max(np.abs(g64 - ref[1]) / sr))
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
