"""Replica scheduling of independent work units over ranks (one GPU per rank).

The reference has no parallelism; its multistart loop (_emulatoroptimise.py:227-278)
runs `tries` independent L-BFGS-B chains and keeps the best.  Here the chains are
dealt round-robin over the ranks of an initialised torch.distributed group (any
backend; gloo is enough since only a few floats per chain are exchanged) and the
(fun, x) results are gathered on every rank.  Without a process group, with
world_size 1, or while the row-block distributed objective is enabled
(distributed.enable_objective: each evaluation is itself collective), everything
runs locally in order.
"""
from __future__ import annotations

import sys


def _group():
    from . import distributed
    if distributed.active_objective() is not None:
        return None   # collective objective: every rank runs every unit in lockstep
    # a process group exists only if the caller imported torch.distributed and
    # initialised it; importing torch here would cost seconds per train()
    dist = sys.modules.get("torch.distributed")
    if dist is None:
        return None
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        return dist
    return None


def rank_world():
    dist = _group()
    if dist is None:
        return 0, 1
    return dist.get_rank(), dist.get_world_size()


def my_items(count: int, rank: int | None = None, world: int | None = None):
    """Indices of the units this rank evaluates (round-robin)."""
    if rank is None or world is None:
        rank, world = rank_world()
    return list(range(rank, count, world))


def gather_results(local: dict, count: int) -> dict:
    """Merge {index: (fun, x, res) or None} from every rank.  Remote entries keep
    only (fun, x); the scipy result object stays on the rank that produced it."""
    dist = _group()
    if dist is None:
        return local
    payload = {k: (None if v is None else (v[0], v[1])) for k, v in local.items()}
    gathered = [None] * dist.get_world_size()
    dist.all_gather_object(gathered, payload)
    merged = {}
    for part in gathered:
        for k, v in part.items():
            merged[k] = None if v is None else (v[0], v[1], None)
    for k, v in local.items():
        merged[k] = v
    missing = [i for i in range(count) if i not in merged]
    if missing:
        raise RuntimeError(f"replica gather lost units {missing}")
    return merged
