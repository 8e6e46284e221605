"""Row-block distributed objective across the GPUs of one node.

One process per GPU (torchrun / torch.distributed.run sets RANK, WORLD_SIZE,
LOCAL_RANK).  torch.distributed (gloo is enough: only 128 bytes travel) carries
the RCCL unique id from rank 0 to the others; every data-path collective after
that is RCCL on the GPU, issued by libgpemu.so itself (include/gpemu_dist.h):
a 128 KB broadcast of the diagonal-block inverse and an all-gather of the panel
column per 128-column step, plus three tiny reductions at the end.

This replaces, for one evaluation spread over P GPUs, the value part of
Optimize.loglikelihood_gp4ml / _mucm (_emulatoroptimise.py:412-493, :305-378).
The gradient stays on the single-GPU path (distributed TRTRI/LAUUM is SURVEY.md
8f item 2); multistart tries are spread as replicas by replicas.py.
"""
from __future__ import annotations

import os

from . import native


def share_unique_id(make_id=None, group=None) -> bytes:
    """Rank 0 creates the communicator id, every rank returns the same 128 bytes.

    `make_id` (default: native.dist_unique_id) is only called on rank 0."""
    import torch.distributed as dist
    if not dist.is_initialized():
        raise RuntimeError("torch.distributed is not initialised")
    make_id = make_id or native.dist_unique_id
    box = [make_id() if dist.get_rank(group) == 0 else None]
    dist.broadcast_object_list(box, src=0, group=group)
    uid = box[0]
    if not isinstance(uid, (bytes, bytearray)) or len(uid) != native.UNIQUE_ID_BYTES:
        raise RuntimeError("bad communicator id")
    return bytes(uid)


def dist_context(device: int | None = None, group=None) -> native.DistContext:
    """DistContext for this process's rank of the initialised process group."""
    import torch.distributed as dist
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    if device is None:
        device = int(os.environ.get("LOCAL_RANK", rank))
    uid = share_unique_id(group=group)
    return native.DistContext(device, world, rank, uid)


def partition(n: int, nranks: int):
    """Tile rows per rank: {rank: [global tile rows]} including the augmented row
    (index ceil(n/128)), dealt cyclically -- the map libgpemu.so uses."""
    nb = (n + 127) // 128
    rows = {r: [] for r in range(nranks)}
    for t in range(nb + 1):
        rows[native.dist_owner(nranks, t)].append(t)
    return rows
