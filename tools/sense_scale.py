"""Sensitivity / UQ at scale -- dev/measurement tool.

Builds an untrained linear-mean emulator on synthetic oLHC data (files as the
reference reads them; hyperparameters from the beliefs file), then runs the
reference example's sequence (uncertainty, sensitivity, main_effect(100),
interaction_effect(0, 1), totaleffectvariance) and prints one JSON line with
the wall time of each call.  The reference forms Rtt and every Pw with per-pair
Python loops and n x n x d arrays, so it cannot run at this size.
usage: python tools/sense_scale.py [--points 16384] [--dims 10]
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--points", type=int, default=16384)
    ap.add_argument("--dims", type=int, default=10)
    args = ap.parse_args()
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    plt.show = lambda *a, **k: None
    import gp_emu_uqsa_amd as g
    from gp_emu_uqsa_amd import synthetic
    from gp_emu_uqsa_amd import sensitivity as sa
    n, d = args.points, args.dims
    X, f, _ = synthetic.problem(n, d, seed=0)
    times = {}
    with tempfile.TemporaryDirectory() as tmp:
        cwd = os.getcwd()
        os.chdir(tmp)
        try:
            np.savetxt("s_input", X, fmt="%.10f")
            np.savetxt("s_output", f.reshape(-1, 1), fmt="%.10f")
            with open("s_config", "w") as fh:
                fh.write("beliefs s_beliefs\ninputs s_input\noutputs s_output\ntv_config 10 0 0\n"
                         "delta_bounds [ ]\nnugget_bounds [ ]\nsigma_bounds [ ]\ntries 1\nconstraints bounds\n")
            with open("s_beliefs", "w") as fh:
                fh.write("active all\noutput 0\nbasis_str 1.0" + " x" * d + "\n"
                         "basis_inf NA" + "".join(f" {k}" for k in range(d)) + "\n"
                         "beta" + " 0.5" * (d + 1) + "\ndelta" + " 0.8" * d + "\n"
                         "sigma 1.0\nnugget 0.001\nfix_nugget T\nmucm F\n")
            t = time.perf_counter()
            E = g.setup("s_config", datashuffle=False, scaleinputs=False)
            times["setup_s"] = time.perf_counter() - t
            calls = [("init_s", lambda: sa.setup(E, [0.5] * d, [0.02] * d))]
            t = time.perf_counter()
            s = calls[0][1]()
            times["init_s"] = time.perf_counter() - t
            for name, fn in (("uncertainty_s", s.uncertainty), ("sensitivity_s", s.sensitivity),
                             ("main_effect_s", lambda: s.main_effect(plot=False, points=100)),
                             ("interaction_effect_s", lambda: s.interaction_effect(0, 1)),
                             ("totaleffectvariance_s", s.totaleffectvariance)):
                t = time.perf_counter()
                fn()
                times[name] = time.perf_counter() - t
        finally:
            os.chdir(cwd)
    out = {"workload": f"case2 sensitivity, n={n} d={d}", **times,
           "uE": float(s.uE), "uEV": float(s.uEV), "senseindex_sum": float(np.sum(s.senseindex / s.uEV))}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
