"""Replica sharding of multistart units over 2 gloo ranks on CPU (the N>1 path:
one GPU per rank, no data-path collective, only (fun, x) gathered)."""
import os
import socket

import numpy as np
import torch.distributed as dist
import torch.multiprocessing as mp

from gp_emu_uqsa_amd import replicas


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _unit(i):
    x = np.array([np.sin(i), np.cos(i)])
    return float((x ** 2).sum() + 0.1 * i), x


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mine = replicas.my_items(7)
        assert mine == list(range(rank, 7, world))
        local = {i: (*_unit(i), None) if i != 3 else None for i in mine}
        merged = replicas.gather_results(local, 7)
        out[rank] = {k: (None if v is None else (v[0], v[1].tolist())) for k, v in merged.items()}
    finally:
        dist.destroy_process_group()


def test_two_rank_gather_equals_sequential():
    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_worker, args=(2, port, out), nprocs=2, join=True)
        res = dict(out)
    seq = {i: (None if i == 3 else (_unit(i)[0], _unit(i)[1].tolist())) for i in range(7)}
    assert res[0] == seq and res[1] == seq


def test_single_process_is_local():
    assert replicas.rank_world() == (0, 1)
    assert replicas.my_items(3) == [0, 1, 2]
