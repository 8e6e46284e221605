"""Distributed objective / gradient (BASELINE configs[3]) -- runner.

  one GPU, P logical ranks (loopback):   python tools/dist_objective.py --loopback P --points N --dims D
  P GPUs over RCCL (one process each):    python -m torch.distributed.run --nproc-per-node P \\
                                              --master-addr 127.0.0.1 tools/dist_objective.py --points N --dims D
Prints one JSON line (rank 0): llh, ms per eval (max over ranks), comm ms, and
with --check the single-GPU value (and gradient with --grad) for the same inputs.
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
    ap.add_argument("--points", type=int, default=4096)
    ap.add_argument("--dims", type=int, default=10)
    ap.add_argument("--loopback", type=int, default=0)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--grad", action="store_true", help="LLH + gradient instead of the value only")
    args = ap.parse_args()
    from gp_emu_uqsa_amd import native
    from gp_emu_uqsa_amd import synthetic
    X, f, H = synthetic.problem(args.points, args.dims, seed=0)
    hp = np.concatenate([np.ones(args.dims), [1e-3, 1.0]])
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    group = None
    if args.loopback:
        ctx = native.DistContext(int(os.environ.get("LOCAL_RANK", "0")), args.loopback)
        nranks = args.loopback
    else:
        from gp_emu_uqsa_amd import distributed, rendezvous
        group = rendezvous.init_from_env()
        ctx = distributed.dist_context()
        nranks = world
    ctx.set_data(X, f, H)
    def ev():
        r = ctx.objective(native.GP4ML, native.KERNEL_STD, hp, want_grad=args.grad)
        return r[0], (r[1] if args.grad else None)
    llh, g = ev()   # warm-up (allocates the gradient buffers)
    ts = []
    for _ in range(args.reps):
        if group is not None:
            group.barrier()
        t = time.perf_counter()
        llh, g = ev()
        ts.append(time.perf_counter() - t)
    el = min(ts)
    if group is not None:
        el = group.all_reduce_max(el)
    out = {"n": args.points, "d": args.dims, "ranks": nranks, "transport": "loopback" if args.loopback else "rccl",
           "grad": args.grad, "llh": llh, "ms_per_eval": 1e3 * el, **ctx.times()}
    if args.check and rank == 0:
        c1 = native.Context(int(os.environ.get("LOCAL_RANK", "0")))
        c1.set_data(X, f, H)
        ref, gref, _ = c1.objective(native.GP4ML, native.KERNEL_STD, hp, want_grad=args.grad)
        t1 = []
        for _ in range(args.reps):
            t = time.perf_counter()
            c1.objective(native.GP4ML, native.KERNEL_STD, hp, want_grad=args.grad)
            t1.append(time.perf_counter() - t)
        out["single_gpu_ms"] = 1e3 * min(t1)
        out["single_gpu_llh"] = ref
        out["rel_diff"] = abs(llh - ref) / abs(ref)
        if args.grad:
            out["grad_max_rel_diff"] = float(np.max(np.abs(g - gref)) / np.max(np.abs(gref)))
        c1.close()
    if rank == 0:
        print(json.dumps(out), flush=True)
    ctx.close()
    if group is not None:
        group.close()


if __name__ == "__main__":
    main()
