"""Process-group rendezvous for one node, without PyTorch.

The reference has no parallelism; here one process drives one GPU,
and the processes of a job need to agree on very little: the 128-byte RCCL
communicator id (distributed.py), barriers and a max over ranks around timed
regions (bench.py), and the (fun, x) of each multistart try (replicas.py).
Every data-path collective is RCCL, issued by libgpemu.so itself.

``FileGroup`` carries those few bytes through files in a directory that all
ranks of the node see (written to a temporary name, then renamed, so a reader
never sees a partial file).  Each operation has a sequence number, so the
files of one call never match another's.  The directory comes from
``GPEMU_RDZV_DIR`` (bench.py sets it when it spawns its ranks), or else from
the launcher's ``MASTER_PORT`` and parent process id (torch.distributed.run
starts all local workers from one agent process), under ``$TMPDIR``.
"""
from __future__ import annotations

import json
import os
import shutil
import tempfile
import time

_DEFAULT: "FileGroup | None" = None


class RendezvousTimeout(RuntimeError):
    """A rank did not arrive within the group's timeout."""


def _env_int(name, default):
    v = os.environ.get(name)
    return default if v in (None, "") else int(v)


def default_dir() -> str:
    d = os.environ.get("GPEMU_RDZV_DIR")
    if d:
        return d
    port = os.environ.get("MASTER_PORT", "0")
    return os.path.join(tempfile.gettempdir(), f"gpemu-rdzv-{port}-{os.getppid()}")


class FileGroup:
    """rank / world_size / barrier / broadcast_bytes / all_gather (JSON values)."""

    def __init__(self, rank: int, world_size: int, path: str | None = None, timeout: float = 900.0):
        if not (0 <= rank < world_size):
            raise ValueError(f"rank {rank} outside world of {world_size}")
        self.rank, self.world_size = int(rank), int(world_size)
        self.path = path or default_dir()
        self.timeout = float(timeout)
        self._seq = 0
        os.makedirs(self.path, exist_ok=True)

    # -- files ---------------------------------------------------------------
    def _name(self, seq, kind, rank):
        return os.path.join(self.path, f"{seq:08d}-{kind}-{rank}")

    def _put(self, seq, kind, payload: bytes):
        final = self._name(seq, kind, self.rank)
        tmp = final + f".tmp{os.getpid()}"
        with open(tmp, "wb") as fh:
            fh.write(payload)
        os.replace(tmp, final)

    def _get(self, seq, kind, rank) -> bytes:
        name = self._name(seq, kind, rank)
        t0 = time.monotonic()
        delay = 2e-4
        while True:
            try:
                with open(name, "rb") as fh:
                    return fh.read()
            except FileNotFoundError:
                pass
            if time.monotonic() - t0 > self.timeout:
                raise RendezvousTimeout(f"rank {rank} did not reach step {seq} ({kind}) within "
                                        f"{self.timeout:.0f} s ({self.path})")
            time.sleep(delay)
            delay = min(delay * 2, 0.01)

    def _next(self):
        self._seq += 1
        return self._seq

    # -- operations ----------------------------------------------------------
    def barrier(self):
        seq = self._next()
        self._put(seq, "bar", b"")
        for r in range(self.world_size):
            self._get(seq, "bar", r)

    def broadcast_bytes(self, data: bytes | None, root: int = 0) -> bytes:
        seq = self._next()
        if self.rank == root:
            if data is None:
                raise ValueError("the root rank must pass the data")
            self._put(seq, "bc", bytes(data))
            return bytes(data)
        return self._get(seq, "bc", root)

    def all_gather(self, value) -> list:
        """Every rank's JSON-serialisable value, in rank order."""
        seq = self._next()
        self._put(seq, "ag", json.dumps(value).encode())
        return [json.loads(self._get(seq, "ag", r).decode()) for r in range(self.world_size)]

    def all_reduce_max(self, x: float) -> float:
        return max(float(v) for v in self.all_gather(float(x)))

    def close(self):
        """Collective: every rank marks that it reads nothing more; rank 0 waits for
        all the marks, then removes the directory."""
        seq = self._next()
        self._put(seq, "done", b"")
        if self.rank == 0:
            for r in range(self.world_size):
                self._get(seq, "done", r)
            shutil.rmtree(self.path, ignore_errors=True)


def init_from_env(path: str | None = None, timeout: float = 900.0) -> "FileGroup | None":
    """The job's group from RANK / WORLD_SIZE (None for a single process); it also
    becomes the default group that replicas.py and distributed.py use."""
    global _DEFAULT
    world = _env_int("WORLD_SIZE", 1)
    if world <= 1:
        return None
    _DEFAULT = FileGroup(_env_int("RANK", 0), world, path, timeout)
    return _DEFAULT


def set_default(group: "FileGroup | None"):
    global _DEFAULT
    _DEFAULT = group


def default_group() -> "FileGroup | None":
    return _DEFAULT
