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


def _stale_worker(rank, world, path, q):
    """A first attempt that dies after sharing its RCCL id: rank 1 exits without
    close(), rank 0 too, so every file of that attempt stays behind."""
    sys.path.insert(0, ROOT)
    from gp_emu_uqsa_amd import rendezvous
    g = rendezvous.FileGroup(rank, world, path, timeout=60)
    g.barrier()
    g.broadcast_bytes(b"\xee" * 128 if rank == 0 else None)
    g.barrier()
    g.all_gather("stale")
    q.put(rank)


def _run(target, world, path, extra=()):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=target, args=(r, world, path, q) + tuple(extra)) for r in range(world)]
    for p in ps:
        p.start()
    res = {}
    for _ in range(world):
        item = q.get(timeout=120)
        res[item[0] if isinstance(item, tuple) else item] = item
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


@pytest.mark.parametrize("world", [2, 3])
def test_group_over_leftover_directory(tmp_path, world):
    """a restarted job (same directory name: same port / parent / run id)
    must not read the files of the attempt before it: not its sequence files (the old
    RCCL id, old barrier marks), not its session, not stale hellos."""
    path = str(tmp_path / "rdzv")
    _run(_stale_worker, world, path)
    assert os.listdir(path)                      # the dead attempt's files are there
    res = _run(_group_worker, world, path)
    for r in range(world):
        _, blob, gathered, mx, *_ = res[r]
        assert blob == b"\x01" * 128               # not the stale id
        assert gathered == [{"rank": k, "sq": k * k} for k in range(world)]
        assert mx == 10.0


def _abort_worker(rank, world, path, q, mode):
    sys.path.insert(0, ROOT)
    import time
    from gp_emu_uqsa_amd import rendezvous
    g = rendezvous.FileGroup(rank, world, path, timeout=60)
    t0 = time.monotonic()
    try:
        g.barrier()   # the abort may already be visible here: any pending operation raises
        if rank == world - 1:
            if mode == "abort":
                g.abort("set_data failed: out of memory")
                raise rendezvous.RendezvousAborted("self")
            g.all_gather("err")          # the others are in a barrier
        else:
            g.barrier()
        q.put((rank, "none", time.monotonic() - t0))
    except (rendezvous.RendezvousAborted, rendezvous.RendezvousMismatch) as e:
        q.put((rank, f"{type(e).__name__}: {e}", time.monotonic() - t0))
    finally:
        g.close()


@pytest.mark.parametrize("mode", ["abort", "mismatch"])
def test_group_fails_fast(tmp_path, mode):
    """a rank that fails before a collective, or enters another one, makes
    its peers raise at once with its message (not a hang until the timeout)."""
    path = str(tmp_path / "rdzv")
    res = _run(_abort_worker, 3, path, (mode,))
    for r in range(2):
        _, err, dt = res[r]
        assert dt < 20.0
        if mode == "abort":
            assert err.startswith("RendezvousAborted") and "out of memory" in err and "rank 2" in err
        else:
            assert err.startswith("RendezvousMismatch") and "'ag'" in err


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
