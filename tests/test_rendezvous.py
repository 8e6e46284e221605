"""The torch-free process group (gp_emu_uqsa_amd/rendezvous.py) on CPU, 2 and 3
ranks: barrier, broadcast of the RCCL id, all-gather, max over ranks, cleanup; the
replica gather and the RCCL-id hand-off through it; and bench.py's own rank
spawner (`--gpus N` without a launcher), which must start N ranks before anything
touches a GPU and refuse a --gpus that disagrees with WORLD_SIZE."""
import json
import multiprocessing as mp
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _group_worker(rank, world, path, q):
    sys.path.insert(0, ROOT)
    from gp_emu_uqsa_amd import distributed, rendezvous, replicas
    g = rendezvous.FileGroup(rank, world, path, timeout=60)
    rendezvous.set_default(g)
    try:
        g.barrier()
        blob = g.broadcast_bytes(b"\x01" * 128 if rank == 0 else None)
        gathered = g.all_gather({"rank": rank, "sq": rank * rank})
        mx = g.all_reduce_max(10.0 - rank)
        calls = []

        def make():
            calls.append(1)
            return bytes(range(128))
        uid = distributed.share_unique_id(make_id=make)
        mine = replicas.my_items(7)
        local = {i: (float(np.sin(i)), np.array([i, 0.1 * i]), None) if i != 3 else None for i in mine}
        merged = replicas.gather_results(local, 7)
        q.put((rank, blob, gathered, mx, uid, len(calls), mine,
               {k: (None if v is None else (v[0], v[1].tolist())) for k, v in merged.items()}))
    finally:
        rendezvous.set_default(None)
        g.close()


@pytest.mark.parametrize("world", [2, 3])
def test_file_group(tmp_path, world):
    path = str(tmp_path / "rdzv")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_group_worker, args=(r, world, path, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = {}
    for _ in range(world):
        item = q.get(timeout=120)
        res[item[0]] = item
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    seq = {i: (None if i == 3 else (float(np.sin(i)), [float(i), 0.1 * i])) for i in range(7)}
    for r in range(world):
        _, blob, gathered, mx, uid, ncalls, mine, merged = res[r]
        assert blob == b"\x01" * 128
        assert gathered == [{"rank": k, "sq": k * k} for k in range(world)]
        assert mx == 10.0
        assert uid == bytes(range(128)) and ncalls == (1 if r == 0 else 0)
        assert mine == list(range(r, 7, world))
        assert merged == seq                       # exact: floats travel as shortest repr
    assert not os.path.exists(path)                # rank 0 removed the directory


def test_single_process_defaults():
    sys.path.insert(0, ROOT)
    from gp_emu_uqsa_amd import rendezvous, replicas
    env = dict(os.environ)
    try:
        os.environ.pop("WORLD_SIZE", None)
        assert rendezvous.init_from_env() is None
        assert replicas.rank_world() == (0, 1)
    finally:
        os.environ.clear()
        os.environ.update(env)


def _bench(args, env=None):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "GPEMU_RDZV_DIR"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=e,
                          capture_output=True, text=True, timeout=120)


@pytest.mark.parametrize("n", [2, 4])
def test_bench_spawns_its_ranks(n):
    r = _bench(["--gpus", str(n), "--rendezvous-check"])
    assert r.returncode == 0, r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1                      # rank 0 prints the one line
    out = json.loads(lines[0])
    assert out["ranks"] == [[k, k, n] for k in range(n)]
    assert out["max_rank"] == n - 1


def test_bench_refuses_mismatched_world():
    r = _bench(["--gpus", "3", "--rendezvous-check"], {"WORLD_SIZE": "2", "RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr


def test_bench_single_rank_needs_no_group():
    r = _bench(["--gpus", "1", "--rendezvous-check"])
    assert r.returncode == 0, r.stderr
    assert json.loads(r.stdout.strip().splitlines()[-1])["ranks"] == [[0, 0, 1]]


def test_bench_under_torchrun():
    """The driver's N > 1 launch: `python -m torch.distributed.run ... bench.py --gpus N`;
    the ranks find each other through MASTER_PORT and their common parent."""
    import socket
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "GPEMU_RDZV_DIR"):
        e.pop(k, None)
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port),
                        os.path.join(ROOT, "bench.py"), "--gpus", "2", "--rendezvous-check"],
                       env=e, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1 and json.loads(lines[0])["ranks"] == [[0, 0, 2], [1, 1, 2]]
