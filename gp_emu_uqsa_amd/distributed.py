"""Row-block distributed objective across the GPUs of one node.

One process per GPU (bench.py's spawner or torch.distributed.run sets RANK,
WORLD_SIZE, LOCAL_RANK).  The native rendezvous group (rendezvous.py: files on the
node, no PyTorch; or a torch.distributed group the caller initialised) carries
the 128-byte RCCL unique id from rank 0 to the others; every data-path
collective after that is RCCL on the GPU, issued by libgpemu.so itself
(include/gpemu_dist.h):
a 128 KB broadcast of the diagonal-block inverse and an all-gather of the panel
column per 128-column step; for the gradient a broadcast of one row of L^-1 per
step, an all-reduce of [sqrt(c) alpha, W] (n x (q+1)) and of d+2 sums.

This replaces, for one evaluation spread over P GPUs, Optimize.loglikelihood_gp4ml
/ _mucm and their gradients (_emulatoroptimise.py:412-493, :305-378).
``enable_objective()`` routes train()'s objective calls through it: every rank
then runs the same L-BFGS-B chains in lockstep (the objective is collective and
returns identical values on every rank), so multistart tries are not sharded
over ranks in that mode (replicas.py does that when the objective is local).
"""
from __future__ import annotations

import os
import sys

from . import native, rendezvous


def _resolve(group):
    """(rank, world, broadcast(bytes or None) -> bytes) of `group`: a rendezvous
    FileGroup, a torch.distributed group (or None = its default group when torch
    initialised one), or None = the native default group."""
    if group is None:
        group = rendezvous.default_group()
    if isinstance(group, rendezvous.FileGroup):
        return group.rank, group.world_size, lambda b: group.broadcast_bytes(b, 0)
    dist = sys.modules.get("torch.distributed")
    if dist is not None and dist.is_available() and dist.is_initialized():
        def bcast(b):
            box = [b]
            dist.broadcast_object_list(box, src=0, group=group)
            return box[0]
        return dist.get_rank(group), dist.get_world_size(group), bcast
    raise RuntimeError("no process group: call rendezvous.init_from_env() in every rank first")


def share_unique_id(make_id=None, group=None) -> bytes:
    """Rank 0 creates the communicator id, every rank returns the same 128 bytes.

    `make_id` (default: native.dist_unique_id) is only called on rank 0."""
    rank, _, bcast = _resolve(group)
    make_id = make_id or native.dist_unique_id
    uid = bcast(make_id() if rank == 0 else None)
    if not isinstance(uid, (bytes, bytearray)) or len(uid) != native.UNIQUE_ID_BYTES:
        raise RuntimeError("bad communicator id")
    return bytes(uid)


def dist_context(device: int | None = None, group=None) -> native.DistContext:
    """DistContext for this process's rank of the job's group."""
    rank, world, _ = _resolve(group)
    if device is None:
        device = int(os.environ.get("LOCAL_RANK", rank))
    uid = share_unique_id(group=group)
    return native.DistContext(device, world, rank, uid)


def partition(n: int, nranks: int, q: int = 0):
    """Tile rows per rank: {rank: [global tile rows]} including the ceil((q+1)/128)
    augmented [f H]^T rows (indices ceil(n/128) ...), dealt cyclically -- the map
    libgpemu.so uses."""
    nb = (n + 127) // 128
    na = (q + 1 + 127) // 128
    rows = {r: [] for r in range(nranks)}
    for t in range(nb + na):
        rows[native.dist_owner(nranks, t)].append(t)
    return rows


class RowBlockObjective:
    """Collective objective for Optimize: the DistContext plus resident-data tracking."""

    def __init__(self, ctx: native.DistContext):
        self.ctx = ctx
        self._key = None

    def ensure_data(self, X, f, H, r=None):
        key = native.Context._digest(X, f, H, r)
        if key != self._key:
            self.ctx.set_data(X, f, H, r)
            self._key = key

    def objective(self, variant, kernel, hp, nu_fixed=0.0, want_grad=True):
        """(llh, grad or None, sigma2), as native.Context.objective."""
        if want_grad:
            return self.ctx.objective(variant, kernel, hp, nu_fixed, want_grad=True)
        llh, s2 = self.ctx.objective(variant, kernel, hp, nu_fixed)
        return llh, None, s2

    def close(self):
        self.ctx.close()


_OBJECTIVE: RowBlockObjective | None = None


def enable_objective(device: int | None = None, group=None, loopback: int = 0) -> RowBlockObjective:
    """Route Optimize's objective through the row-block distributed path.

    With an initialised process group this is collective (every rank calls it);
    ``loopback=P`` instead runs P logical ranks in this process on one GPU."""
    global _OBJECTIVE
    disable_objective()
    if loopback:
        dev = int(os.environ.get("LOCAL_RANK", "0")) if device is None else device
        ctx = native.DistContext(dev, int(loopback))
    else:
        ctx = dist_context(device, group)
    _OBJECTIVE = RowBlockObjective(ctx)
    return _OBJECTIVE


def disable_objective():
    global _OBJECTIVE
    if _OBJECTIVE is not None:
        _OBJECTIVE.close()
        _OBJECTIVE = None


def active_objective() -> RowBlockObjective | None:
    return _OBJECTIVE
