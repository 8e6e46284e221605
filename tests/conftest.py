import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a visible gfx950 GPU and libgpemu.so")


@pytest.fixture(scope="session")
def ctx():
    from gp_emu_uqsa_amd import native
    c = native.Context(0)
    yield c
    c.close()
