"""CPU checks of the C-ABI library and the host logic (no GPU compute)."""
import ctypes
import os
import re

import numpy as np
import pytest

from gp_emu_uqsa_amd import native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_symbols():
    names = set()
    for h in sorted(os.listdir(os.path.join(ROOT, "include"))):
        if not h.endswith(".h"):
            continue
        text = open(os.path.join(ROOT, "include", h)).read()
        names |= set(re.findall(r"^\s*(?:int|int32_t|void|gpe_ctx\*|gpe_dist\*|const char\*)\s+\*?(gpe_\w+)\s*\(",
                                text, flags=re.M))
    return sorted(names)


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(native.LIB_PATH)
    names = _declared_symbols()
    assert len(names) >= 15
    for name in names:
        assert hasattr(lib, name), name
    assert set(names) == set(native.SIGNATURES), set(names) ^ set(native.SIGNATURES)


def test_abi_version_and_no_device_fails_loudly():
    lib = native.load_library()
    assert lib.gpe_abi_version() == 10
    if lib.gpe_device_count() == 0:
        with pytest.raises(native.NativeUnavailable):
            native.Context(0)
        assert lib.gpe_create(0) is None
        assert b"device" in lib.gpe_last_error(None)


def test_literal_parser_accepts_numpy2_reprs():
    from gp_emu_uqsa_amd.files import literal
    assert literal("[[np.float64(0.0157), np.float64(0.9854)], [0.1, 2]]") == [[0.0157, 0.9854], [0.1, 2]]
    assert literal("[ ]") == []
    assert literal("[[0.05,1.0],[0.05,10.00]]") == [[0.05, 1.0], [0.05, 10.0]]


def test_library_built_from_these_sources():
    """Provenance: the in-tree library carries the SHA-256 of the sources it was built
    from (gpe_build_id), equal to the sources present; a different one is refused."""
    from gp_emu_uqsa_amd import buildinfo
    assert native.build_id() == buildinfo.source_hash()
    assert len(native.build_id()) == 64


def test_source_hash_tracks_contents(tmp_path):
    from gp_emu_uqsa_amd import buildinfo
    root = tmp_path / "tree"
    (root / "gp_emu_uqsa_amd" / "csrc").mkdir(parents=True)
    (root / "include").mkdir()
    (root / "gp_emu_uqsa_amd" / "csrc" / "a.hip").write_text("x")
    (root / "include" / "b.h").write_text("y")
    h1 = buildinfo.source_hash(str(root))
    (root / "include" / "b.h").write_text("z")
    assert buildinfo.source_hash(str(root)) != h1
