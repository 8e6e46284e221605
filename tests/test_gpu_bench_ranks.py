"""bench.py's multi-GPU path end to end on the one-GPU box: `--gpus 3` spawns three rank
processes (every rank on GPU 0 under GPEMU_BENCH_ONE_DEVICE=1, each with its own
NCCL_HOSTID so RCCL connects them over its socket transport), runs the replica legs,
then the guarded row-block leg over RCCL, whose rank-0 parity check against the
single-GPU objective must pass.  Small sizes: this checks the plumbing the driver's
N = 2, 4, 8 runs go through (spawner, rendezvous, max-over-ranks timing, RCCL id,
row-block collectives), not the timing."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(300)
def test_bench_three_ranks_rowblock_over_rccl():
    env = dict(os.environ, GPEMU_BENCH_ONE_DEVICE="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "GPEMU_RDZV_DIR"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "3", "--steps", "2", "--warmup", "1",
           "--n", "2048", "--d", "6", "--no-other-configs", "--rowblock-n", "3000", "--rowblock-d", "8",
           "--rowblock-timeout", "200"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=280, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-4000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 3 and line["config"]["parallelism"] == "replicas3"
    assert line["value"] > 0.0
    rb = line["extra"]["rowblock"]
    assert "error" not in rb and "skipped" not in rb, rb
    assert rb["ranks"] == 3 and rb["n"] == 3000
    assert rb["parity_vs_single_gpu"]["ok"], rb["parity_vs_single_gpu"]
    assert len(rb["per_rank_device_gb"]) == 3
    # the metric configuration's strong-scaling leg (here at the bench's --n / --d)
    rm = line["extra"]["rowblock_metric"]
    assert "error" not in rm and "skipped" not in rm, rm
    assert rm["ranks"] == 3 and rm["n"] == 2048 and rm["d"] == 6
    assert rm["parity_vs_single_gpu"]["ok"], rm["parity_vs_single_gpu"]
    assert rm["llh_grad_ms"] > 0.0 and rm["comm_ms_llh_grad"] > 0.0
    assert rm["speedup_vs_single_gpu"] > 0.0
