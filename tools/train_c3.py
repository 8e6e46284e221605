"""BASELINE configs[2]: the full g.setup()/g.train() loop at
n=16384, d=10 through the reference's API and file surface, scipy L-BFGS-B
driving the GPU objective (LLH + gradient) -- dev/measurement tool.

configs[3] (C4, n=65536, d=20 on 8 GPUs): run under torchrun, one process per
GPU; the objective is then the row-block distributed one (distributed.
enable_objective over RCCL) and every rank steps the same L-BFGS-B chain.
--loopback P runs that path with P logical ranks on one GPU.

Writes config/beliefs/inputs/outputs for synthetic oLHC data into a scratch
directory (tv_config 10 0 0: every point in training; gp4ml, nugget fitted,
linear mean in all inputs, tries 1, constraints bounds), then times setup and
train and prints one JSON line: wall seconds, objective evaluations, seconds per
evaluation, trained delta / nugget / sigma, final LLH.
usage: python tools/train_c3.py [--points 16384] [--dims 10] [--tries 1] [--loopback P]
       python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
           tools/train_c3.py --points 65536 --dims 20
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


def write_files(root, n, d, tries):
    from gp_emu_uqsa_amd import synthetic
    X, f, _ = synthetic.problem(n, d, seed=0)
    np.savetxt(os.path.join(root, "c3_input"), X, fmt="%.10f")
    np.savetxt(os.path.join(root, "c3_output"), f.reshape(-1, 1), fmt="%.10f")
    with open(os.path.join(root, "c3_config"), "w") as fh:
        fh.write("beliefs c3_beliefs\ninputs c3_input\noutputs c3_output\ntv_config 10 0 0\n"
                 "delta_bounds [ ]\nnugget_bounds [ ]\nsigma_bounds [ ]\n"
                 f"tries {tries}\nconstraints bounds\n")
    with open(os.path.join(root, "c3_beliefs"), "w") as fh:
        fh.write("active all\noutput 0\n"
                 "basis_str 1.0" + " x" * d + "\n"
                 "basis_inf NA" + "".join(f" {k}" for k in range(d)) + "\n"
                 "beta" + " 1.0" * (d + 1) + "\n"
                 "delta" + " 1.0" * d + "\n"
                 "sigma 1.0\nnugget 0.001\nfix_nugget F\nmucm F\n")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--points", type=int, default=16384)
    ap.add_argument("--dims", type=int, default=10)
    ap.add_argument("--tries", type=int, default=1)
    ap.add_argument("--loopback", type=int, default=0, help="row-block objective, P logical ranks on one GPU")
    args = ap.parse_args()
    import gp_emu_uqsa_amd as g
    from gp_emu_uqsa_amd import distributed, native
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    mode = "single"
    group = None
    if world > 1:
        from gp_emu_uqsa_amd import rendezvous
        group = rendezvous.init_from_env()
        distributed.enable_objective()
        mode = f"rowblock-rccl-{world}"
    elif args.loopback:
        distributed.enable_objective(loopback=args.loopback)
        mode = f"rowblock-loopback-{args.loopback}"
    calls = {"n": 0, "s": 0.0}
    cls = native.Context if mode == "single" else distributed.RowBlockObjective
    orig = cls.objective

    def counted(self, *a, **k):
        t = time.perf_counter()
        try:
            return orig(self, *a, **k)
        finally:
            calls["n"] += 1
            calls["s"] += time.perf_counter() - t
    cls.objective = counted
    with tempfile.TemporaryDirectory() as tmp:
        write_files(tmp, args.points, args.dims, args.tries)
        cwd = os.getcwd()
        os.chdir(tmp)
        try:
            np.random.seed(0)
            t0 = time.perf_counter()
            E = g.setup("c3_config", datashuffle=True)
            t1 = time.perf_counter()
            g.train(E, auto=True)
            t2 = time.perf_counter()
        finally:
            os.chdir(cwd)
    out = {"config": f"g.train(): n={args.points} d={args.dims} gp4ml nugget fitted, tries {args.tries}",
           "objective": mode,
           "setup_s": t1 - t0, "train_s": t2 - t1, "objective_evals": calls["n"],
           "objective_s": calls["s"], "s_per_eval": calls["s"] / max(calls["n"], 1),
           "evals_per_s_of_train": calls["n"] / (t2 - t1),
           "concurrent_tries": os.environ.get("GPEMU_CONCURRENT_TRIES", "default"),
           "delta": np.asarray(E.par.delta).tolist(), "nugget": float(E.par.nugget),
           "sigma": float(E.par.sigma)}
    if rank == 0:
        print(json.dumps(out), flush=True)
    distributed.disable_objective()
    if group is not None:
        group.close()


if __name__ == "__main__":
    main()
