"""Replica scheduling of independent work units over ranks (one GPU per rank).

The reference has no parallelism; its multistart loop (_emulatoroptimise.py:227-278)
runs `tries` independent L-BFGS-B chains and keeps the best.  Here the chains are
dealt round-robin over the ranks of the job's group and the (fun, x) results are
gathered on every rank.  The group is the native rendezvous group
(rendezvous.init_from_env(), no PyTorch), or else a torch.distributed group the
caller initialised itself (any backend; only a few floats per chain travel).
Without a group, with world size 1, or while the row-block distributed objective
is enabled (distributed.enable_objective: each evaluation is itself collective),
everything runs locally in order.
"""
from __future__ import annotations

import sys

import numpy as np

from . import rendezvous


class _TorchGroup:
    """Adapter over an initialised torch.distributed default group."""

    def __init__(self, dist):
        self.dist = dist
        self.rank, self.world_size = dist.get_rank(), dist.get_world_size()

    def all_gather(self, value):
        out = [None] * self.world_size
        self.dist.all_gather_object(out, value)
        return out


def _group():
    from . import distributed
    if distributed.active_objective() is not None:
        return None   # collective objective: every rank runs every unit in lockstep
    g = rendezvous.default_group()
    if g is not None and g.world_size > 1:
        return g
    # a torch process group exists only if the caller imported torch.distributed and
    # initialised it; importing torch here would cost seconds per train()
    dist = sys.modules.get("torch.distributed")
    if dist is not None and dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        return _TorchGroup(dist)
    return None


def rank_world():
    g = _group()
    if g is None:
        return 0, 1
    return g.rank, g.world_size


def my_items(count: int, rank: int | None = None, world: int | None = None):
    """Indices of the units this rank evaluates (round-robin)."""
    if rank is None or world is None:
        rank, world = rank_world()
    return list(range(rank, count, world))


def gather_results(local: dict, count: int) -> dict:
    """Merge {index: (fun, x, res) or None} from every rank.  Remote entries keep
    only (fun, x); the scipy result object stays on the rank that produced it.
    fun and x travel as JSON numbers (Python's shortest round-trip repr: exact)."""
    g = _group()
    if g is None:
        return local
    payload = [[int(k), None if v is None else [float(v[0]), np.asarray(v[1], dtype=float).tolist()]]
               for k, v in local.items()]
    merged = {}
    for part in g.all_gather(payload):
        for k, v in part:
            merged[int(k)] = None if v is None else (v[0], np.asarray(v[1], dtype=float), None)
    for k, v in local.items():
        merged[k] = v
    missing = [i for i in range(count) if i not in merged]
    if missing:
        raise RuntimeError(f"replica gather lost units {missing}")
    return merged
