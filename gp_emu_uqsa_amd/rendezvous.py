"""Process-group rendezvous for one node, without PyTorch.

The reference has no parallelism; here one process drives one GPU,
and the processes of a job need to agree on very little: the 128-byte RCCL
communicator id (distributed.py), barriers and a max over ranks around timed
regions (bench.py), and the (fun, x) of each multistart try (replicas.py).
Every data-path collective is RCCL, issued by libgpemu.so itself.

``FileGroup`` carries those few bytes through files in a directory that all
ranks of the node see (written to a temporary name, then renamed, so a reader
never sees a partial file).  The directory comes from ``GPEMU_RDZV_DIR``
(bench.py sets it when it spawns its ranks), or else from the launcher's
``MASTER_PORT``, ``TORCHELASTIC_RUN_ID``, ``TORCHELASTIC_RESTART_COUNT`` and
parent process id (torch.distributed.run starts all local workers of an attempt
from one agent process), under ``$TMPDIR``.

Files a crashed earlier job (or an earlier elastic attempt) left in the same
directory are never read: the group first agrees on a fresh session.  Every rank
posts a hello with a random nonce; rank 0 answers with a session file naming a
fresh token and the nonce it saw from each rank; a rank joins only a session
that names its own nonce (a stale hello is re-read until it is fresh), and uses
the session only once rank 0 has sealed it.  Every operation then lives in the
session's own subdirectory, tagged with a sequence number and its kind; a rank
that finds a peer at the same step with another kind raises at once (the ranks
have diverged), and ``abort(msg)`` makes every peer's pending operation raise
``RendezvousAborted`` with the failing rank's message instead of timing out.
"""
from __future__ import annotations

import glob
import json
import os
import secrets
import shutil
import tempfile
import time

_DEFAULT: "FileGroup | None" = None


class RendezvousTimeout(RuntimeError):
    """A rank did not arrive within the group's timeout."""


class RendezvousAborted(RuntimeError):
    """A peer called abort(): its message, instead of a hang or a timeout."""


class RendezvousMismatch(RuntimeError):
    """A peer reached the same step with a different operation."""


def _env_int(name, default):
    v = os.environ.get(name)
    return default if v in (None, "") else int(v)


def default_dir() -> str:
    d = os.environ.get("GPEMU_RDZV_DIR")
    if d:
        return d
    port = os.environ.get("MASTER_PORT", "0")
    run = os.environ.get("TORCHELASTIC_RUN_ID", "none")
    attempt = os.environ.get("TORCHELASTIC_RESTART_COUNT", "0")
    safe = "".join(ch if ch.isalnum() or ch in "-_." else "_" for ch in f"{port}-{run}-{attempt}")
    return os.path.join(tempfile.gettempdir(), f"gpemu-rdzv-{safe}-{os.getppid()}")


class FileGroup:
    """rank / world_size / barrier / broadcast_bytes / all_gather (JSON values)."""

    def __init__(self, rank: int, world_size: int, path: str | None = None, timeout: float = 900.0):
        if not (0 <= rank < world_size):
            raise ValueError(f"rank {rank} outside world of {world_size}")
        self.rank, self.world_size = int(rank), int(world_size)
        self.base = path or default_dir()
        self.timeout = float(timeout)
        self._seq = 0
        self.aborted: str | None = None
        os.makedirs(self.base, exist_ok=True)
        self.token = self._join_session()
        self.path = os.path.join(self.base, "s-" + self.token)
        os.makedirs(self.path, exist_ok=True)

    # -- session agreement (stale files of earlier jobs are never read) --------
    def _write(self, name, payload: bytes):
        tmp = name + f".tmp{os.getpid()}-{secrets.token_hex(4)}"
        with open(tmp, "wb") as fh:
            fh.write(payload)
        os.replace(tmp, name)

    @staticmethod
    def _read(name):
        try:
            with open(name, "rb") as fh:
                return fh.read()
        except FileNotFoundError:
            return None

    def _join_session(self) -> str:
        nonce = secrets.token_hex(16)
        self._write(os.path.join(self.base, f"hello-{self.rank}"), nonce.encode())
        t0 = time.monotonic()
        delay = 2e-4

        def wait():
            nonlocal delay
            if time.monotonic() - t0 > self.timeout:
                raise RendezvousTimeout(f"no session agreed within {self.timeout:.0f} s ({self.base})")
            time.sleep(delay)
            delay = min(delay * 2, 0.01)

        if self.rank == 0:
            while True:
                hellos = [self._read(os.path.join(self.base, f"hello-{r}")) for r in range(self.world_size)]
                if any(h is None for h in hellos):
                    wait()
                    continue
                nonces = [h.decode() for h in hellos]
                nonces[0] = nonce
                token = secrets.token_hex(16)
                self._write(os.path.join(self.base, "session"),
                            json.dumps({"token": token, "nonces": nonces}).encode())
                # every rank joins it, or some hello was stale: re-read and re-issue
                t1 = time.monotonic()
                while time.monotonic() - t1 < 0.5:
                    joined = [r == 0 or self._read(os.path.join(self.base, f"join-{r}-{token}")) is not None
                              for r in range(self.world_size)]
                    if all(joined):
                        self._write(os.path.join(self.base, f"sealed-{token}"), b"")
                        return token
                    wait()
                fresh = [self._read(os.path.join(self.base, f"hello-{r}")) for r in range(self.world_size)]
                if fresh[1:] == hellos[1:]:
                    continue   # same hellos: a slow rank, issue the same nonces again
        joined = None
        while True:
            raw = self._read(os.path.join(self.base, "session"))
            if raw is not None:
                try:
                    sess = json.loads(raw.decode())
                except ValueError:
                    sess = None
                if sess and len(sess.get("nonces", [])) == self.world_size and sess["nonces"][self.rank] == nonce:
                    tok = sess["token"]
                    if tok != joined:
                        self._write(os.path.join(self.base, f"join-{self.rank}-{tok}"), b"")
                        joined = tok
                    if os.path.exists(os.path.join(self.base, f"sealed-{tok}")):
                        return tok
            wait()

    # -- files ---------------------------------------------------------------
    def _name(self, seq, kind, rank):
        return os.path.join(self.path, f"{seq:08d}-{kind}-{rank}")

    def _put(self, seq, kind, payload: bytes):
        self._write(self._name(seq, kind, self.rank), payload)

    def _check_abort(self):
        if self.aborted is not None:
            raise RendezvousAborted(self.aborted)
        for name in glob.glob(os.path.join(self.path, "abort-*")):
            msg = self._read(name)
            if msg is not None:
                self.aborted = msg.decode(errors="replace")
                raise RendezvousAborted(self.aborted)

    def _get(self, seq, kind, rank) -> bytes:
        name = self._name(seq, kind, rank)
        t0 = time.monotonic()
        delay = 2e-4
        polls = 0
        while True:
            data = self._read(name)
            if data is not None:
                return data
            polls += 1
            if polls % 8 == 1:
                self._check_abort()
                other = [os.path.basename(p).split("-")[1] for p in glob.glob(self._name(seq, "*", rank))
                         if ".tmp" not in p]
                other = [k for k in other if k != kind]
                if other:
                    got = other[0]
                    raise RendezvousMismatch(f"rank {rank} reached step {seq} with '{got}' while rank "
                                             f"{self.rank} is in '{kind}' ({self.path})")
            if time.monotonic() - t0 > self.timeout:
                raise RendezvousTimeout(f"rank {rank} did not reach step {seq} ({kind}) within "
                                        f"{self.timeout:.0f} s ({self.path})")
            time.sleep(delay)
            delay = min(delay * 2, 0.01)

    def _next(self):
        self._check_abort()
        self._seq += 1
        return self._seq

    # -- operations ----------------------------------------------------------
    def abort(self, message: str):
        """Fail the group: every peer's pending or next operation raises
        RendezvousAborted(message) instead of waiting for this rank."""
        if self.aborted is None:
            self.aborted = f"rank {self.rank}: {message}"
            self._write(os.path.join(self.path, f"abort-{self.rank}"), self.aborted.encode())

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

    def _gather(self, value, kind) -> list:
        seq = self._next()
        self._put(seq, kind, json.dumps(value).encode())
        return [json.loads(self._get(seq, kind, r).decode()) for r in range(self.world_size)]

    def all_gather(self, value) -> list:
        """Every rank's JSON-serialisable value, in rank order."""
        return self._gather(value, "ag")

    def all_reduce_max(self, x: float) -> float:
        return max(float(v) for v in self._gather(float(x), "max"))

    def close(self):
        """Collective: every rank marks that it reads nothing more; rank 0 waits for
        all the marks, then removes the session.  After an abort nobody waits and
        nothing is removed."""
        if self.aborted is None:
            try:
                seq = self._next()
                self._put(seq, "done", b"")
                if self.rank == 0:
                    for r in range(self.world_size):
                        self._get(seq, "done", r)
            except (RendezvousAborted, RendezvousMismatch, OSError):
                pass
        # after an abort the session stays (its abort mark is what the peers still
        # waiting must find; a unique subdirectory, never read by a later session)
        if self.rank == 0 and self.aborted is None:
            shutil.rmtree(self.path, ignore_errors=True)
            for name in ["session"] + [f"hello-{r}" for r in range(self.world_size)]:
                try:
                    os.remove(os.path.join(self.base, name))
                except OSError:
                    pass
            for name in glob.glob(os.path.join(self.base, f"*-{self.token}")):
                try:
                    os.remove(name)
                except OSError:
                    pass
            try:
                os.rmdir(self.base)   # only when empty (another job may share the base)
            except OSError:
                pass


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
