"""CPU baseline at the metric's size, as BASELINE.md section 3 asks (dev tool, run on
the GPU box's host; writes profiles/cpu_ref_<tag>.json):

* ref mode: the oracle's op-for-op restatement of loglikelihood_gp4ml
  (oracle/gp_oracle.py objective_ref, _emulatoroptimise.py:412-493) ONCE at n=16384,
  d=10, with the BLAS on every CPU of the process's quota;
* fast mode: the GPU's formulation on LAPACK (objective_fast), 3 reps, median.

The oracle is test infrastructure; this tool only times it as the reference's CPU
path.  A progress line goes to stderr every 30 s (ref mode runs for minutes).

usage: python tools/cpu_ref_c3.py [tag] [n] [d]"""
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402  (host info, eval point)
from oracle import gp_oracle as orc  # noqa: E402


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r03"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
    d = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    host = bench._host_info()
    threads = host.get("affinity_cpus") or os.cpu_count() or 1
    if host.get("cgroup_cpu_quota"):
        threads = max(1, min(threads, int(host["cgroup_cpu_quota"])))
    from threadpoolctl import threadpool_limits
    limiter = threadpool_limits(limits=threads, user_api="blas")
    stop = threading.Event()
    t_start = time.perf_counter()
    phase = ["setup"]

    def beat():
        while not stop.wait(30.0):
            print(f"[cpu_ref] {phase[0]}: {time.perf_counter() - t_start:.0f} s", file=sys.stderr, flush=True)
    threading.Thread(target=beat, daemon=True).start()
    X, f, H = orc.synthetic_problem(n, d, seed=0)
    hp = bench.eval_point(d, 0)
    out = {"n": n, "d": d, "hp": hp.tolist(), "threads": threads, "host": host,
           "what": "oracle objective_ref (op-for-op loglikelihood_gp4ml, LLH + gradient) once; "
                   "objective_fast (Cholesky + inverse + contraction on LAPACK) 3 reps"}
    phase[0] = "fast mode"
    fast = []
    for _ in range(3):
        t = time.perf_counter()
        r = orc.objective_fast(X, f, H, hp, orc.GP4ML, orc.STD, True)
        fast.append(time.perf_counter() - t)
        print(f"[cpu_ref] objective_fast: {fast[-1]:.1f} s llh {r[0]!r}", file=sys.stderr, flush=True)
    out["fast_mode_s"] = fast
    out["fast_mode_median_s"] = float(np.median(fast))
    out["fast_llh"] = float(r[0])
    phase[0] = "ref mode"
    t = time.perf_counter()
    r = orc.objective_ref(X, f, H, hp, orc.GP4ML, orc.STD, True)
    out["ref_mode_s"] = time.perf_counter() - t
    out["ref_llh"] = float(r[0])
    out["ref_grad"] = [float(v) for v in r[1]]
    print(f"[cpu_ref] objective_ref: {out['ref_mode_s']:.1f} s llh {r[0]!r}", file=sys.stderr, flush=True)
    stop.set()
    limiter.unregister()
    path = os.path.join(ROOT, "gpurun_out", f"cpu_ref_{tag}.json")
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps({k: out[k] for k in ("n", "threads", "fast_mode_median_s", "ref_mode_s")}), flush=True)


if __name__ == "__main__":
    main()
