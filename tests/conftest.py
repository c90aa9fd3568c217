import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libzenith_raster's HIP kernels)")


@pytest.fixture(scope="session")
def device():
    """One RenderDevice for the whole GPU session (one process on the card)."""
    from zenith_amd import rhi
    dev = rhi.RenderDevice(0)
    yield dev
    dev.close()
