"""One rank of a multi-process RCCL run of the row-block distributed objective
(helper of tests/test_gpu_rccl_multirank.py; not collected by pytest).

Every rank runs the same cases through distributed.dist_context (RCCL communicator,
the id shared by the native file rendezvous).  Rank 0 also evaluates each case on
the single-GPU Context and prints one JSON line with both results; the test
compares them.  All ranks may sit on one GPU: the test gives every rank its own
NCCL_HOSTID, so RCCL treats them as separate hosts (socket transport over the
loopback interface) instead of refusing a second rank on the same device.

usage: RANK=r WORLD_SIZE=P GPEMU_RDZV_DIR=... python tests/rccl_worker.py n d [one]
("one": only the gp4ml std case, value + gradient once, and no non-PD case: the
full-size C4 run)
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from gp_emu_uqsa_amd import distributed, native, rendezvous, synthetic  # noqa: E402


def cases(d, n):
    rs = np.random.RandomState(7)
    r = 1e-3 * (1.0 + rs.uniform(size=n))
    base = np.concatenate([np.full(d, 0.7), [0.05, 1.3]])
    mucm = np.concatenate([np.full(d, 0.9), [0.02]])
    alt = np.concatenate([np.full(d, 0.6), [0.1, 1.1]])
    return [
        ("gp4ml_std", native.GP4ML, native.KERNEL_STD, base, 0.0, None),
        ("mucm_std", native.MUCM, native.KERNEL_STD, mucm, 0.0, None),
        ("gp4ml_alt_r", native.GP4ML, native.KERNEL_ALT_NUG, alt, 0.0, r),
        ("gp4ml_std_fixed_nugget", native.GP4ML, native.KERNEL_STD, base[[*range(d), d + 1]], 1e-3, None),
    ]


def main():
    n, d = int(sys.argv[1]), int(sys.argv[2])
    one = len(sys.argv) > 3 and sys.argv[3] == "one"
    group = rendezvous.init_from_env(timeout=600.0)
    rank, world = group.rank, group.world_size
    X, f, H = synthetic.problem(n, d, seed=3)
    dc = distributed.dist_context(0, group)
    out = {"ranks": world, "n": n, "d": d, "cases": {}}
    for name, variant, kernel, hp, nu, r in cases(d, n)[:1 if one else None]:
        dc.set_data(X, f, H, r)
        llh_v, s2_v = dc.objective(variant, kernel, hp, nu)
        llh, g, s2 = dc.objective(variant, kernel, hp, nu, want_grad=True)
        rec = {"llh_value_only": llh_v, "llh": llh, "grad": list(map(float, g)), "sigma2": s2}
        rec["rank_gb"] = group.all_gather(dc.rank_bytes() / 1e9)
        if one:   # free this rank's rows before rank 0 holds the single-GPU n x n buffers
            out["comm_ms"] = dc.times()["comm_ms"]
            dc.close()
            group.barrier()
        if rank == 0:
            c = native.Context(0)
            c.set_data(X, f, H, r)
            ref, gref, s2ref = c.objective(variant, kernel, hp, nu)
            c.close()
            rec.update(ref_llh=ref, ref_grad=list(map(float, gref)), ref_sigma2=s2ref)
        out["cases"][name] = rec
    if not one:
        # a matrix that is not positive definite (a duplicated point, no nugget): every
        # rank must report it, through the all-reduced failure flag
        Xd = X.copy()
        Xd[1] = Xd[0]
        dc.set_data(Xd, f, H)
        try:
            dc.objective(native.GP4ML, native.KERNEL_STD, np.concatenate([np.full(d, 0.5), [1.0]]),
                         nu_fixed=0.0, want_grad=True)
            out["not_pd"] = False
        except native.NotPositiveDefinite:
            out["not_pd"] = True
        out["comm_ms"] = dc.times()["comm_ms"]
        out["not_pd_all"] = group.all_gather(out["not_pd"])
        dc.close()
    group.barrier()
    if rank == 0:
        print("RESULT " + json.dumps(out), flush=True)
    group.close()


if __name__ == "__main__":
    main()
