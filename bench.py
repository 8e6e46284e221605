"""Headline benchmark: log-marginal-likelihood evals/s at n=16384, d=10, fp64.

The unit is one evaluation of the reference objective (loglikelihood_gp4ml,
_emulatoroptimise.py:412-493) returning (LLH, gradient) -- what L-BFGS-B
consumes with jac=True -- on synthetic oLHC data: std Gaussian
kernel, nugget fitted, gp4ml, 12 hyperparameters, at delta near 1, nu=1e-3,
sigma=1.  Each GPU keeps --concurrent (default 2) multistart tries in flight, as
g.train() does at this size: one context (HIP stream, workspaces) and one host
thread per try, each at its own point.  One step = one evaluation of every try.

Processes: one per GPU.  `python bench.py --gpus N` starts its N ranks itself
(before anything touches a GPU); under `python -m torch.distributed.run
--nproc-per-node N bench.py --gpus N` the launcher has set RANK / WORLD_SIZE /
LOCAL_RANK and --gpus must equal WORLD_SIZE.  No PyTorch in any rank: barriers
and the max over ranks go through gp_emu_uqsa_amd/rendezvous.py, device
synchronisation through libgpemu.so.  The headline runs one replica per GPU
(independent multistart evaluations, no data-path collective; value =
evaluations by all ranks / the slowest rank's time).  With N > 1 the line also
carries two row-block legs, each ONE LLH + gradient spread over the N GPUs by the
row-block distributed objective over RCCL (include/gpemu_dist.h), with its
collective time and a rank-0 parity check against the single-GPU objective:
`extra.rowblock_metric` at the metric's own configuration (n=16384, d=10: the
strong-scaling latency of one evaluation against N) and `extra.rowblock` at
BASELINE configs[3] (n=65536, d=20).

Also reported: the roofline of the dominant kernel (the MFMA GEMM: algorithmic
flops per launch / mean launch time from HIP events on its own stream, recorded
live on the last timed step), its HBM traffic per launch from the committed
rocprofv3 PMC pass (profiles/, labelled), and a CPU baseline (the op-for-op
NumPy restatement of the reference, oracle/gp_oracle.py, on this host's cores;
rank 0, N=1 only).
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import subprocess
import sys
import tempfile
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "log-marginal-likelihood evals/sec at n=16384 d=10 fp64; 1/2/4/8 GPU"
FP64_MFMA_PEAK_TFLOPS = 78.6       # MI355X dense fp64 matrix peak (spec)
INT8_MFMA_PEAK_TOPS = 5033.0       # dense i8 matrix peak (spec: 2 x the 2.5 PF dense bf16)
INT8_RANDOM_CEILING_TOPS = 2449.0  # MFMA-only i8 loop on random operands, 4 waves/SIMD (tools/hip/i8_probe.hip)
C4 = (65536, 20)                   # BASELINE.json configs[3]


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--n", type=int, default=16384)
    ap.add_argument("--d", type=int, default=10)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-full", action="store_true",
                    help="CPU baseline: 3 op-for-op reps at n=4096 instead of 1 (~2 min more)")
    ap.add_argument("--no-cpu-fast", dest="cpu_fast", action="store_false",
                    help="CPU baseline: skip the measured fast-formulation evaluation at the metric "
                         "size (~40 s)")
    ap.add_argument("--no-profile", action="store_true",
                    help="time without per-launch HIP events (roofline omitted)")
    ap.add_argument("--no-other-configs", dest="other_configs", action="store_false",
                    help="skip the informational configs[1] / configs[4] timings")
    ap.add_argument("--concurrent", type=int, default=2,
                    help="multistart tries in flight per GPU (own context and HIP stream each), "
                         "as g.train() runs them at this size (optimize.Optimize._concurrency)")
    ap.add_argument("--no-rowblock", dest="rowblock", action="store_false",
                    help="N > 1: skip the row-block distributed configs[3] leg")
    ap.add_argument("--rowblock-n", type=int, default=C4[0])
    ap.add_argument("--rowblock-d", type=int, default=C4[1])
    ap.add_argument("--rowblock-steps", type=int, default=2)
    ap.add_argument("--rowblock-metric-steps", type=int, default=5,
                    help="N > 1: timed evaluations of the metric-config row-block leg (strong scaling)")
    ap.add_argument("--no-rowblock-metric", dest="rowblock_metric", action="store_false",
                    help="N > 1: skip the metric-config row-block leg")
    ap.add_argument("--rowblock-timeout", type=float, default=300.0)
    ap.add_argument("--rendezvous-check", action="store_true",
                    help="(test hook) spawn / rendezvous only: no GPU, rank 0 prints the ranks it saw")
    return ap.parse_args(argv)


# ---------------------------------------------------------------------------
# launcher: N rank processes, started before anything touches a GPU
# ---------------------------------------------------------------------------
def spawn_ranks(nprocs: int, argv: list[str]) -> int:
    """Run this script as `nprocs` rank processes on this node (RANK = LOCAL_RANK =
    0..N-1, WORLD_SIZE = N, a fresh rendezvous directory) and return the first
    non-zero exit status, or 0.  If a rank fails the others are stopped."""
    rdzv = tempfile.mkdtemp(prefix="gpemu-bench-")
    procs = []
    try:
        for r in range(nprocs):
            env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nprocs),
                       LOCAL_WORLD_SIZE=str(nprocs), MASTER_ADDR="127.0.0.1",
                       GPEMU_RDZV_DIR=rdzv)
            env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
            if os.environ.get("GPEMU_BENCH_ONE_DEVICE") == "1":
                # rehearsal with every rank on GPU 0: RCCL refuses two ranks on one device
                # of one host, so each rank names its own host and RCCL connects them
                # with its socket transport over the loopback interface
                env.update(NCCL_HOSTID=f"gpemu-bench-rank-{r}", NCCL_SOCKET_IFNAME="lo",
                           NCCL_IB_DISABLE="1")
            procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env))
        rc = 0
        pending = list(procs)
        while pending:
            for p in list(pending):
                code = p.poll()
                if code is None:
                    continue
                pending.remove(p)
                if code != 0 and rc == 0:
                    rc = code
                    for q in pending:      # the exact PIDs this launcher started
                        q.terminate()
            time.sleep(0.05)
        return rc
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
        import shutil
        shutil.rmtree(rdzv, ignore_errors=True)


def eval_point(d, rank):
    """Untransformed hp: delta(d), nu, sigma; one multistart point per rank."""
    delta = np.ones(d) * (1.0 + 0.02 * rank)
    return np.concatenate([delta, [1e-3, 1.0]])


# ---------------------------------------------------------------------------
# CPU baseline (rank 0, N=1 only)
# ---------------------------------------------------------------------------
def _host_info():
    """The CPU the baseline ran on: model, logical and physical CPUs,
    this process's affinity, the cgroup CPU quota, BLAS build."""
    info = {"cpu_model": None, "logical_cpus": os.cpu_count()}
    try:
        cores = set()
        phys = core = None
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name") and info["cpu_model"] is None:
                    info["cpu_model"] = line.split(":", 1)[1].strip()
                elif line.startswith("physical id"):
                    phys = line.split(":", 1)[1].strip()
                elif line.startswith("core id"):
                    core = line.split(":", 1)[1].strip()
                    cores.add((phys, core))
        info["physical_cores"] = len(cores) or None
    except OSError:
        pass
    try:
        info["affinity_cpus"] = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        info["affinity_cpus"] = None
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, per = fh.read().split()[:2]
            if q != "max":
                quota = float(q) / float(per)
    except (OSError, ValueError):
        pass
    info["cgroup_cpu_quota"] = quota
    try:
        from threadpoolctl import threadpool_info
        libs = [i for i in threadpool_info() if i.get("user_api") == "blas"]
        if libs:
            info["blas"] = f"{libs[0].get('internal_api')} {libs[0].get('version')} ({libs[0].get('architecture')})"
    except Exception:
        pass
    return info


def cpu_baseline(d, n_full, full=False, fast=True):
    """CPU baseline on this host, with the BLAS on every CPU this process may use (the
    affinity mask, capped by the cgroup quota), at the metric's size n_full:

    * value (kind "port"): the reference's evaluation (_emulatoroptimise.py:412-493)
      spends 90-94% of its time in np.linalg.solve with the n x n factor L (SURVEY.md
      6): 24 calls with n right-hand sides (two per hyperparameter, :452-479) and 5
      with at most q (:426-430), each an LU of L (dgesv).  One call of each kind is
      timed at n_full and the evaluation is taken as 24 t_n + 5 t_q; it omits the
      Cholesky, the 12 dense dA builds and the products, so the value is an UPPER bound
      on the reference's evals/s.
    * ref_mode_c2_measured: the op-for-op restatement of the reference's evaluation
      (oracle objective_ref, _emulatoroptimise.py:412-493: pdist/squareform/exp, the
      Cholesky, every np.linalg.solve with n right-hand sides, the 12 dense dA) run ONCE
      at configs[1]'s size (n=4096, d=10), ~60 s on the GPU box's host: the measured
      op-for-op CPU time of the same run.
    * fast_mode_measured (fast=True, the default): the oracle's objective_fast (the
      GPU's algorithm on LAPACK: Cholesky, explicit inverse, contraction) run ONCE at
      n_full (~40 s on the GPU box's 16-CPU quota): the measured CPU evaluation at the
      metric's own size in the same run.
    * full=True adds two more op-for-op repetitions at n=4096 (median of 3)."""
    from oracle import gp_oracle as orc

    def note(msg):   # progress on stderr: the CPU legs run for minutes
        print(f"[cpu_baseline] {msg}", file=sys.stderr, flush=True)
    host = _host_info()
    threads = host.get("affinity_cpus") or os.cpu_count() or 1
    if host.get("cgroup_cpu_quota"):
        threads = max(1, min(threads, int(host["cgroup_cpu_quota"])))
    try:
        from threadpoolctl import threadpool_limits
        limiter = threadpool_limits(limits=threads, user_api="blas")
    except Exception:
        limiter = None
    out = {}
    try:
        n, q = n_full, d + 1
        rs = np.random.RandomState(0)
        w = np.eye(512) + np.tril(rs.uniform(size=(512, 512))) / 512
        np.linalg.solve(w, w)   # start the BLAS thread pool outside the timed calls
        L = np.tril(rs.uniform(-1.0, 1.0, size=(n, n))) / n + np.eye(n)   # a lower-triangular factor
        B = rs.uniform(-1.0, 1.0, size=(n, n))
        t = time.perf_counter()
        np.linalg.solve(L, B)
        t_n = time.perf_counter() - t
        note(f"np.linalg.solve(L, {n} x {n}): {t_n:.1f} s")
        del B
        Bq = rs.uniform(-1.0, 1.0, size=(n, q))
        t = time.perf_counter()
        np.linalg.solve(L, Bq)
        t_q = time.perf_counter() - t
        note(f"np.linalg.solve(L, {n} x {q}): {t_q:.1f} s")
        del L, Bq
        t_ref = 24 * t_n + 5 * t_q
        out.update({"value": 1.0 / t_ref, "unit": "evals/s", "cores": int(threads), "kind": "port",
                    "host": host,
                    "sample": (f"reference op order at n={n}: np.linalg.solve(L, n x n) {t_n:.1f} s and "
                               f"np.linalg.solve(L, n x {q}) {t_q:.1f} s measured once each on {threads} BLAS "
                               f"threads; evaluation = 24 x + 5 x those = {t_ref:.0f} s (upper bound on "
                               f"evals/s: Cholesky, dA builds and products omitted)")})
        hp = eval_point(d, 0)
        X2, f2, H2 = orc.synthetic_problem(4096, d, seed=0)
        reps = []
        llh_ref = None
        for _ in range(3 if full else 1):
            t = time.perf_counter()
            llh_ref = orc.objective_ref(X2, f2, H2, hp, orc.GP4ML, orc.STD, True)[0]
            reps.append(time.perf_counter() - t)
            note(f"objective_ref n=4096: {reps[-1]:.1f} s")
        med = float(np.median(reps))
        out["ref_mode_c2_measured"] = {
            "s_per_eval": med, "evals_per_s": 1.0 / med, "reps_s": reps, "n": 4096, "d": d,
            "threads": int(threads), "llh": llh_ref,
            "sample": (f"the reference's op order (oracle objective_ref: pdist/squareform/exp, Cholesky, "
                       f"np.linalg.solve with n right-hand sides, 12 dense dA) at n=4096, d={d}, "
                       f"{len(reps)} evaluation(s) measured in this run on {threads} BLAS threads")}
        if fast:
            X, f, H = orc.synthetic_problem(n, d, seed=0)
            t = time.perf_counter()
            llh_fast = orc.objective_fast(X, f, H, hp, orc.GP4ML, orc.STD, True)[0]
            tf = time.perf_counter() - t
            del X, f, H
            note(f"objective_fast n={n}: {tf:.1f} s")
            out["fast_mode_measured"] = {
                "value": 1.0 / tf, "unit": "evals/s", "s_per_eval": tf, "n": n, "d": d,
                "threads": int(threads), "llh": llh_fast,
                "sample": (f"oracle objective_fast (the GPU's algorithm on LAPACK: Cholesky, explicit "
                           f"inverse, contraction; the best CPU formulation, not the reference's op "
                           f"order) measured ONCE in this run at n={n}, d={d} on {threads} BLAS "
                           f"threads: {tf:.1f} s/eval")}
    finally:
        if limiter is not None:
            limiter.unregister()
    ref = _ref_mode_measured(n_full, d)
    if ref is not None:
        out["ref_mode_measured"] = ref
    return out


def _ref_mode_measured(n, d):
    """The op-for-op reference path run once at this size on a GPU box's host
    (tools/cpu_ref_c3.py, committed under profiles/): too long (~8 min) to repeat in
    every bench run, so it is cited, not re-measured."""
    best = None
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "cpu_ref_*.json"))):
        try:
            rec = json.load(open(path))
        except Exception:
            continue
        if rec.get("n") == n and rec.get("d") == d and rec.get("ref_mode_s"):
            best = {"s_per_eval": rec["ref_mode_s"], "evals_per_s": 1.0 / rec["ref_mode_s"],
                    "fast_mode_median_s": rec.get("fast_mode_median_s"), "threads": rec.get("threads"),
                    "cpu_model": (rec.get("host") or {}).get("cpu_model"),
                    "source": os.path.relpath(path, ROOT) + " (committed; not measured in this run)"}
    return best


# ---------------------------------------------------------------------------
# informational legs (rank 0, after the timed region)
# ---------------------------------------------------------------------------
def other_configs(native, synthetic, ctx, args):
    """BASELINE.json configs[1] (n=4096, d=10: one LLH+grad and one value-only
    evaluation, single stream) and configs[4] (n=16384, d=10 emulator, posterior
    mean + diagonal variance at m=1e6 points, precision 32: 24-bit int8 products).  The headline metric
    stays configs[2]."""
    out = {}
    X, f, H = synthetic.problem(4096, 10, seed=0)
    c = native.Context(ctx.device)
    c.set_data(X, f, H)
    hp = eval_point(10, 0)
    c.objective(native.GP4ML, native.KERNEL_STD, hp)
    t = time.perf_counter()
    c.objective(native.GP4ML, native.KERNEL_STD, hp)
    out["c2_n4096_llh_grad_ms"] = 1000.0 * (time.perf_counter() - t)
    t = time.perf_counter()
    c.objective(native.GP4ML, native.KERNEL_STD, hp, want_grad=False)
    out["c2_n4096_value_only_ms"] = 1000.0 * (time.perf_counter() - t)
    c.close()
    if args.n == 16384 and args.d == 10:
        m = 1000000
        xs = synthetic.design(m, 10, seed=7)
        hs = synthetic.linear_basis(xs)
        ctx.factor(native.KERNEL_STD, np.ones(10), 1e-3, 1.0, 0.0)
        beta = ctx.beta()
        t = time.perf_counter()
        ctx.posterior(xs, hs, beta, 1.0, full_var=False, precision=32)
        dt = time.perf_counter() - t
        out["c5_posterior_fp32_points_per_s"] = m / dt
        out["c5_posterior_fp32_s"] = dt
        out["c5_product"] = ("precision 32: L^-1 K* as exact int8 products of 24-bit operands (8 moduli, "
                             "at least an fp32 GEMM's accuracy); GPEMU_OZAKI=0 runs it on fp32 MFMA")
    return out


def rowblock_leg(native, synthetic, group, rank, world, local, args, sync_all, n, d, steps, what):
    """One LLH+gradient (and one value-only evaluation) of n x n spread over the
    `world` GPUs by the row-block distributed objective over RCCL; time = max over
    ranks; rank 0 then checks value and gradient against the single-GPU objective
    (tolerances as tests/test_gpu_fullsize.py).  Run for configs[3] (n=65536, d=20)
    and for the metric's own configuration (n=16384, d=10: single-evaluation latency
    against N)."""
    from gp_emu_uqsa_amd import distributed
    X, f, H = synthetic.problem(n, d, seed=0)
    hp = eval_point(d, 0)
    dc = distributed.dist_context(local, group)
    dc.set_data(X, f, H)
    llh, g, _ = dc.objective(native.GP4ML, native.KERNEL_STD, hp, want_grad=True)   # allocates
    sync_all()
    t0 = time.perf_counter()
    comm = []
    for _ in range(steps):
        llh, g, _ = dc.objective(native.GP4ML, native.KERNEL_STD, hp, want_grad=True)
        comm.append(dc.times()["comm_ms"])
    sync_all()
    t_grad = group.all_reduce_max((time.perf_counter() - t0) / steps)
    t0 = time.perf_counter()
    dc.objective(native.GP4ML, native.KERNEL_STD, hp, want_grad=False)
    sync_all()
    t_val = group.all_reduce_max(time.perf_counter() - t0)
    comm_val = dc.times()["comm_ms"]
    rank_gb = group.all_gather(dc.rank_bytes() / 1e9)
    dc.close()
    out = None
    if rank == 0:
        c = native.Context(local)
        c.set_data(X, f, H)
        ref, gref, _ = c.objective(native.GP4ML, native.KERNEL_STD, hp)
        c.close()
        rel_llh = abs(llh - ref) / abs(ref)
        rel_g = float(np.max(np.abs(np.asarray(g) - gref)) / np.max(np.abs(gref)))
        flops = float(n) ** 3   # algorithmic: n^3/3 each for POTRF, TRTRI and the A^-1 partials
        out = {"config": f"{what}: gp4ml LLH+grad n={n} d={d}, one evaluation over {world} GPUs "
                         f"(row-block cyclic tile rows, RCCL)",
               "n": n, "d": d, "ranks": world,
               "llh_grad_ms": 1000.0 * t_grad, "llh_grad_evals_per_s": 1.0 / t_grad,
               "value_only_ms": 1000.0 * t_val,
               "comm_ms_llh_grad": float(np.mean(comm)), "comm_ms_value_only": comm_val,
               "algorithmic_tflops": flops / t_grad / 1e12,
               "per_rank_device_gb": rank_gb,
               "parity_vs_single_gpu": {"llh_rel": rel_llh, "grad_max_rel": rel_g,
                                        "ok": bool(rel_llh <= 1e-10 and rel_g <= 1e-8)}}
    return out


_EMIT = threading.Lock()
_EMITTED = [False]


def emit(out):
    """Rank 0's one JSON line, at most once (the row-block watchdog may print it)."""
    with _EMIT:
        if not _EMITTED[0]:
            _EMITTED[0] = True
            print(json.dumps(out), flush=True)


def guarded_rowblock(native, synthetic, group, rank, world, local, args, sync_all, out, key, n, d, steps, what):
    """rowblock_leg behind a pre-flight check and a watchdog, so that the headline
    line survives a row-block failure: every rank first reports whether its GPU is
    visible; a failure on any rank makes all skip; an exception is recorded; and if
    the leg outlives --rowblock-timeout (a rank stuck in a collective), rank 0
    prints the line with the error and every rank exits."""
    if os.environ.get("GPEMU_BENCH_ONE_DEVICE") == "1" and not os.environ.get("NCCL_HOSTID"):
        return {"skipped": "one-device rehearsal without per-rank NCCL_HOSTID: RCCL refuses two ranks "
                           "on one GPU of one host"}
    ok = native.load_library().gpe_device_count() > local
    if not all(group.all_gather(bool(ok))):
        return {"skipped": "a rank does not see its GPU"}
    done = threading.Event()

    def watchdog():
        if done.wait(args.rowblock_timeout):
            return
        if rank == 0:
            out.setdefault("extra", {})[key] = {"error": f"timed out after {args.rowblock_timeout:.0f} s"}
            emit(out)
        sys.stdout.flush()
        os._exit(0 if rank == 0 else 3)

    threading.Thread(target=watchdog, daemon=True).start()
    from gp_emu_uqsa_amd import rendezvous
    try:
        res = rowblock_leg(native, synthetic, group, rank, world, local, args, sync_all, n, d, steps, what)
        err = None
    except rendezvous.RendezvousAborted as e:   # a peer failed: its message
        res, err = None, str(e)
    except Exception as e:   # recorded in the line; the headline stands
        res, err = None, f"{type(e).__name__}: {e}"
        group.abort(err)     # peers waiting in a file collective raise with this message
    try:
        errs = [e for e in group.all_gather(err) if e] if group.aborted is None else [group.aborted]
    except rendezvous.RendezvousAborted as e:
        errs = [str(e)]
    done.set()
    if errs:
        return {"error": errs[0]}
    return res


def pmc_traffic(n, d, which="gemm"):
    """HBM bytes per launch of k_gemm (which="gemm") or k_oz_gemm ("ozaki") from the committed
    rocprofv3 PMC summary (tools/pmc_gemm.py)."""
    best = None
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_gemm_*.json"))):
        try:
            rec = json.load(open(path))
        except Exception:
            continue
        if rec.get("n") == n and rec.get("d") == d:
            best = (os.path.relpath(path, ROOT), rec)
    if best is None:
        return None, None
    key = "bytes_per_gemm_launch" if which == "gemm" else "bytes_per_ozaki_launch"
    return best[1].get(key), best[0]


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus, argv))
    world = int(world_env or 1)
    if args.gpus != world:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    if os.environ.get("GPEMU_BENCH_ONE_DEVICE") == "1":
        local = 0   # rehearsal of the N-rank path with every rank on GPU 0 (one-GPU box)
        if world > 1:   # under a launcher too: each rank names its own host for RCCL (see spawn_ranks)
            os.environ.setdefault("NCCL_HOSTID", f"gpemu-bench-rank-{rank}")
            os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
            os.environ.setdefault("NCCL_IB_DISABLE", "1")

    from gp_emu_uqsa_amd import rendezvous
    group = rendezvous.init_from_env() if world > 1 else None

    if args.rendezvous_check:   # spawn / rendezvous test hook: no GPU
        seen = group.all_gather([rank, local, world]) if group else [[rank, local, world]]
        mx = group.all_reduce_max(float(rank)) if group else 0.0
        if group:
            group.barrier()
        if rank == 0:
            print(json.dumps({"ranks": seen, "max_rank": mx}), flush=True)
        if group:
            group.close()
        return

    from gp_emu_uqsa_amd import native, synthetic

    def sync_all():
        native.device_synchronize(local)
        if group is not None:
            group.barrier()

    K = max(1, args.concurrent)
    X, f, H = synthetic.problem(args.n, args.d, seed=0)
    ctxs = []
    for k in range(K):
        c = native.Context(local)
        c.set_data(X, f, H)
        ctxs.append(c)
    ctx = ctxs[0]
    hps = [eval_point(args.d, rank * K + k) for k in range(K)]   # one multistart point per try
    prof = not args.no_profile
    last = [None] * K

    def run_tries(count):
        """Each of the K contexts evaluates `count` times, all K in flight at once
        (one host thread per context; ctypes releases the GIL during the call)."""
        def work(k):
            for _ in range(count):
                last[k] = ctxs[k].objective(native.GP4ML, native.KERNEL_STD, hps[k])
        if K == 1:
            work(0)
            return
        th = [threading.Thread(target=work, args=(k,)) for k in range(K)]
        for t in th:
            t.start()
        for t in th:
            t.join()

    run_tries(args.warmup)
    gemm_ms = gemm_fl = gemm_n = 0.0
    oz_ms = oz_ops = oz_fl = oz_n = 0.0
    phase_acc = {}
    prof_steps = 0
    sync_all()
    t0 = time.perf_counter()
    # steps 1..K-1: the K tries concurrently.  The last step evaluates the K tries
    # one after another with HIP events around every GEMM launch (~1.5 ms per eval),
    # so the roofline's per-launch times are those of a launch that has the GPU to
    # itself; that step is inside the timed region, at single-stream speed.
    run_tries(args.steps - 1 if prof else args.steps)
    if prof:
        for k in range(K):
            ctxs[k].set_profiling(True)
            last[k] = ctxs[k].objective(native.GP4ML, native.KERNEL_STD, hps[k])
            gs = ctxs[k].gemm_stats()
            gemm_ms += gs["ms"]
            gemm_fl += gs["flops"]
            gemm_n += gs["launches"]
            oz = ctxs[k].ozaki_stats()
            oz_ms += oz["ms"]
            oz_ops += oz["int8_ops"]
            oz_fl += oz["fp64_flops"]
            oz_n += oz["launches"]
            for key, v in ctxs[k].phase_times().items():
                phase_acc[key] = phase_acc.get(key, 0.0) + v
            prof_steps += 1
            ctxs[k].set_profiling(False)
    sync_all()
    elapsed = time.perf_counter() - t0
    llh = last[0][0]
    if group is not None:
        elapsed = group.all_reduce_max(elapsed)
    # informational, outside the timed region: one eval alone (latency) and value-only
    t1 = time.perf_counter()
    ctx.objective(native.GP4ML, native.KERNEL_STD, hps[0])
    single_s = time.perf_counter() - t1
    t1 = time.perf_counter()
    ctx.objective(native.GP4ML, native.KERNEL_STD, hps[0], want_grad=False)
    value_only_s = time.perf_counter() - t1
    other = other_configs(native, synthetic, ctx, args) if (rank == 0 and args.other_configs) else None
    if group is not None:
        group.barrier()
    out = None
    if rank == 0:
        n_units = world * args.steps * K
        out = {
            "metric": METRIC,
            "value": n_units / elapsed,
            "unit": "evals/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1000.0 * elapsed / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "dtype_note": "fp64 throughout; the A^-1 and top-TRTRI products are computed exactly (53-bit operands, "
                          "integer products reconstructed by CRT) on the int8 matrix cores",
            "data": "synthetic (oLHC design, toysim3D-style outputs + 0.01 N(0,1) noise)",
            "config": {"workload": f"gp4ml LLH+grad, n={args.n} d={args.d}, std Gaussian kernel, "
                                   f"nugget fitted ({args.d + 2} hp); a step = one eval of each of "
                                   f"{K} multistart tries in flight per GPU",
                       "n": args.n, "d": args.d, "q": args.d + 1, "tries_in_flight_per_gpu": K,
                       "parallelism": f"replicas{world}"},
        }
        if prof and gemm_ms > 0:
            achieved = gemm_fl / (gemm_ms * 1e-3) / 1e12
            traffic, tsrc = pmc_traffic(args.n, args.d)
            whole = K * 4398e9 * (args.n / 16384) ** 3 / 1e12   # ~n^3 algorithmic flops per eval
            step_tflops = whole / (elapsed / args.steps)
            out["roofline"] = {"bound": "mfma", "achieved": achieved,
                               "peak": FP64_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                               "frac": achieved / FP64_MFMA_PEAK_TFLOPS,
                               "frac_basis": "per launch: algorithmic flops of every k_gemm launch of one "
                                             "evaluation / their HIP-event durations, each launch with the "
                                             "GPU to itself (the tries run one after the other in that step)",
                               "achieved_step_level": step_tflops,
                               "frac_step_level": step_tflops / FP64_MFMA_PEAK_TFLOPS,
                               "step_level_basis": f"whole-job: n^3 algorithmic fp64 flops per evaluation x "
                                                   f"{K} tries in flight / ms_per_step (the headline regime; the "
                                                   f"A^-1 and top TRTRI products among them run as exact int8 "
                                                   f"products, see int8_emulation)",
                               "traffic": traffic,
                               "traffic_source": (f"{tsrc}: rocprofv3 --pmc passes of this bench command "
                                                  f"(committed, not measured in this run)") if tsrc else None,
                               "kernel": "k_gemm (fp64 v_mfma_f64_16x16x4_f64)",
                               "flops_per_launch": gemm_fl / gemm_n,
                               "ms_per_launch": gemm_ms / gemm_n}
            if oz_n > 0:
                ach = oz_ops / (oz_ms * 1e-3) / 1e12
                out["roofline"]["int8_emulation"] = {
                    "kernel": "k_oz_gemm (v_mfma_i32_32x32x32_i8): A^-1 = L^-T L^-1 and the top TRTRI level's two "
                              "products as exact integer products of 53-bit operands, 16 moduli, CRT back to fp64 "
                              "(gpemu_ozaki.hpp)",
                    "bound": "mfma", "unit": "TOPS (int8)", "achieved": ach, "peak": INT8_MFMA_PEAK_TOPS,
                    "frac": ach / INT8_MFMA_PEAK_TOPS,
                    "random_operand_ceiling": INT8_RANDOM_CEILING_TOPS,
                    "frac_of_random_operand_ceiling": ach / INT8_RANDOM_CEILING_TOPS,
                    "fp64_equivalent_tflops": oz_fl / (oz_ms * 1e-3) / 1e12,
                    "ms_per_eval": oz_ms / max(prof_steps, 1), "launches_per_eval": oz_n / max(prof_steps, 1),
                    "fp64_flops_share": oz_fl / (oz_fl + gemm_fl),
                    "traffic": pmc_traffic(args.n, args.d, "ozaki")[0]}
            phase_ms = {k: v / max(prof_steps, 1) for k, v in phase_acc.items()}
            third = float(args.n) ** 3 / 3.0   # algorithmic flops of POTRF, TRTRI and LAUUM each
            out["extra"] = {"phase_ms": phase_ms,
                            "phase_tflops": {k: third / (phase_ms[k] * 1e-3) / 1e12
                                             for k in ("cholesky", "trtri", "inverse") if phase_ms.get(k)},
                            "roofline_sample": f"HIP events around every GEMM launch of timed step "
                                               f"{args.steps} (its {K} evals run one at a time)",
                            "eval_tflops_algorithmic": step_tflops,
                            "step_level_frac": step_tflops / FP64_MFMA_PEAK_TFLOPS,
                            "single_eval_ms": 1000.0 * single_s,
                            "value_only_ms": 1000.0 * value_only_s,
                            "other_configs": other,
                            "llh": llh}
        if world == 1 and not args.no_cpu_baseline:
            cb = cpu_baseline(args.d, args.n, full=args.cpu_full, fast=args.cpu_fast)
            # the headline against each CPU figure (value = the reference's op-order bound)
            ratios = {"vs_ref_op_order_bound": out["value"] / cb["value"]}
            if cb.get("fast_mode_measured"):
                ratios["vs_fast_mode_measured"] = out["value"] / cb["fast_mode_measured"]["value"]
                fm = cb["fast_mode_measured"]
                fm["llh_rel_diff_vs_gpu"] = abs(fm["llh"] - llh) / abs(llh)   # (same data and point as try 0)
            if cb.get("ref_mode_measured"):
                ratios["vs_ref_mode_measured_cited"] = out["value"] * cb["ref_mode_measured"]["s_per_eval"]
            cb["gpu_evals_per_s_over_cpu"] = ratios
            out["cpu_baseline"] = cb
    if world > 1 and args.rowblock:
        for c in ctxs:          # the replica workspaces are not needed by the row-block leg
            c.close()
        ctxs = []
        # strong scaling of the metric's own unit first (one n=16384 evaluation over N
        # GPUs), then configs[3]; each leg guarded on its own
        legs = [("rowblock_metric", args.n, args.d, args.rowblock_metric_steps,
                 "metric configuration (strong scaling of one evaluation)"),
                ("rowblock", args.rowblock_n, args.rowblock_d, args.rowblock_steps, "BASELINE configs[3]")]
        for key, n_, d_, steps_, what in legs:
            if not args.rowblock_metric and key == "rowblock_metric":
                continue
            rb = guarded_rowblock(native, synthetic, group, rank, world, local, args, sync_all, out,
                                  key, n_, d_, steps_, what)
            if rank == 0:
                out.setdefault("extra", {})[key] = rb
                if key == "rowblock_metric" and isinstance(rb, dict) and rb.get("llh_grad_ms"):
                    rb["single_gpu_single_eval_ms"] = 1000.0 * single_s
                    rb["speedup_vs_single_gpu"] = 1000.0 * single_s / rb["llh_grad_ms"]
            if group.aborted is not None:
                break
    if rank == 0:
        emit(out)
    for c in ctxs:
        c.close()
    if group is not None:
        group.close()


if __name__ == "__main__":
    main()
