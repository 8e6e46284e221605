"""g.setup() + g.train() at the reference's own example sizes, on the GPU and with the
reference's CPU objective (dev timing tool).

The examples' data files (tests/golden/examples/, copied from the reference's
examples/ directories: data, not source):
  toy-sim      examples/toy-sim (toy-sim_config: 60 points, d = 2, MUCM, tries 10)
  toysim3D     examples/sensitivity_multi_outputs (toysim3D_config0: 100 points, d = 3,
               gp4ml, tries 20, bounds)
  noisefit2D   examples/noisefit2D (config-data: 500 points, d = 2, alt nugget fitted,
               gp4ml, tries 3) -- the data emulator of its noisefit loop
Each is run in a scratch copy of its files, with np.random.seed(0) before setup, three
ways: the GPU path cold (first call: context and schedules), the GPU path again (warm),
and the same train() with every objective evaluation replaced by the CPU oracle's
objective_ref (the op-for-op restatement of loglikelihood_gp4ml / _mucm,
_emulatoroptimise.py:305-493, on this host's BLAS; the oracle is the measured CPU
baseline here, never the product path).  Reported: wall time of setup and train, the
objective evaluations and the time inside them, and the trained hyperparameters of the
GPU and CPU runs (the same L-BFGS-B chains up to rounding).
usage: python tools/example_train_time.py [> json]"""
import contextlib
import io
import json
import os
import shutil
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import gp_emu_uqsa_amd as g  # noqa: E402
from gp_emu_uqsa_amd import native, optimize  # noqa: E402
from oracle import gp_oracle as orc  # noqa: E402

EXAMPLES = [("toy-sim", "toy-sim", "toy-sim_config"),
            ("toysim3D", "toysim3D", "toysim3D_config0"),
            ("noisefit2D", "noisefit2D", "config-data")]


def run(sub, config, cpu):
    src = os.path.join(ROOT, "tests", "golden", "examples", sub)
    tmp = tempfile.mkdtemp(prefix="gpemu-ex-")
    for f in os.listdir(src):
        if os.path.isfile(os.path.join(src, f)):
            shutil.copy(os.path.join(src, f), tmp)
    stats = {"calls": 0, "s": 0.0}
    orig = optimize.Optimize._call

    def timed(self, variant, x, want_grad=True):
        t = time.perf_counter()
        try:
            if not cpu:
                return orig(self, variant, x, want_grad)
            r = None if np.isscalar(self.data.r) else self.data.r
            out = orc.objective_ref(self.data.inputs, self.data.outputs, self.data.H, np.asarray(x, float),
                                    variant, self.data.K.kind, self.beliefs.fix_nugget == "F", r=r,
                                    want_grad=want_grad, nu_fixed=float(self.data.K.n))
            if out is None:
                raise native.NotPositiveDefinite("objective_ref: not positive definite")
            return out
        finally:
            stats["calls"] += 1
            stats["s"] += time.perf_counter() - t

    cwd = os.getcwd()
    optimize.Optimize._call = timed
    try:
        os.chdir(tmp)
        np.random.seed(0)
        with contextlib.redirect_stdout(io.StringIO()):
            t0 = time.perf_counter()
            E = g.setup(config)
            t1 = time.perf_counter()
            g.train(E)
            t2 = time.perf_counter()
        n = int(E.training.inputs.shape[0])
        hp = [float(v) for v in np.concatenate([np.atleast_1d(E.par.delta), [E.par.nugget, E.par.sigma]])]
    finally:
        optimize.Optimize._call = orig
        os.chdir(cwd)
        shutil.rmtree(tmp, ignore_errors=True)
    return {"setup_s": t1 - t0, "train_s": t2 - t1, "objective_calls": stats["calls"],
            "objective_s": stats["s"], "objective_ms_per_call": 1e3 * stats["s"] / max(stats["calls"], 1),
            "n_train_final": n, "trained_hp": hp}


def main():
    out = {"host_cpus": os.cpu_count(), "examples": {}}
    for name, sub, cfg in EXAMPLES:
        rec = {"gpu_cold": run(sub, cfg, False), "gpu": run(sub, cfg, False), "cpu_objective_ref": run(sub, cfg, True)}
        rec["train_speedup"] = rec["cpu_objective_ref"]["train_s"] / rec["gpu"]["train_s"]
        rec["objective_speedup"] = (rec["cpu_objective_ref"]["objective_ms_per_call"] /
                                    max(rec["gpu"]["objective_ms_per_call"], 1e-9))
        rec["hp_max_rel_diff_gpu_cpu"] = float(np.max(np.abs(np.array(rec["gpu"]["trained_hp"]) -
                                                             np.array(rec["cpu_objective_ref"]["trained_hp"])) /
                                                      np.maximum(np.abs(rec["cpu_objective_ref"]["trained_hp"]), 1e-300)))
        out["examples"][name] = rec
        print(json.dumps({name: {k: (round(v, 4) if isinstance(v, float) else v) for k, v in rec.items()
                                 if not isinstance(v, dict)} | {
            "gpu_train_s": round(rec["gpu"]["train_s"], 4), "cpu_train_s": round(rec["cpu_objective_ref"]["train_s"], 4),
            "gpu_ms_per_eval": round(rec["gpu"]["objective_ms_per_call"], 4),
            "cpu_ms_per_eval": round(rec["cpu_objective_ref"]["objective_ms_per_call"], 4),
            "evals": rec["gpu"]["objective_calls"]}}), file=sys.stderr, flush=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
