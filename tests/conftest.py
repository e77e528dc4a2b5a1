import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through librpgpu.so)")


@pytest.fixture(scope="session")
def built():
    import __graft_entry__

    __graft_entry__.build()
    return True


@pytest.fixture(scope="session")
def eng(built):
    from redpanda_amd import engine

    e = engine.Engine(0)
    yield e
    e.close()
