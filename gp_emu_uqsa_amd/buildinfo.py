"""Provenance of libgpemu.so: a SHA-256 over the HIP/C++ sources and public headers
it is built from.  build() (__graft_entry__.py) compiles it in as gpe_build_id(), and
native.load_library() refuses a library whose id differs from the sources beside it,
so the library a process loads is the one these sources make."""
from __future__ import annotations

import hashlib
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def source_files(root: str = ROOT) -> list[str]:
    csrc = os.path.join(root, "gp_emu_uqsa_amd", "csrc")
    inc = os.path.join(root, "include")
    files = [os.path.join(csrc, f) for f in os.listdir(csrc) if f.endswith((".hip", ".hpp", ".h"))]
    files += [os.path.join(inc, f) for f in os.listdir(inc) if f.endswith(".h")]
    return sorted(files, key=lambda p: os.path.relpath(p, root))


def source_hash(root: str = ROOT) -> str | None:
    """Hex digest over (relative path, contents) of every source; None when the sources
    are not present (an installed library without its tree)."""
    try:
        files = source_files(root)
    except OSError:
        return None
    if not files:
        return None
    h = hashlib.sha256()
    for p in files:
        h.update(os.path.relpath(p, root).encode())
        h.update(b"\0")
        with open(p, "rb") as fh:
            h.update(fh.read())
        h.update(b"\0")
    return h.hexdigest()
