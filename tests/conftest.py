"""Shared test configuration.

Markers:
  gpu -- needs a HIP device (MI355X); run with `pytest -m gpu` on the GPU box.
Everything unmarked runs on CPU (oracle pinning, host logic, ABI exports).
"""
import os
import sys

import pytest

TESTS = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(TESTS)
for p in (ROOT, TESTS):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP GPU (MI355X); parity tests through the C ABI")


@pytest.fixture(scope="session")
def vds_lib():
    """The built in-tree libvds_ec.so (built on demand)."""
    from vds_amd import build
    build.build()
    from vds_amd import _lib
    return _lib.lib()


@pytest.fixture(scope="session")
def gpu(vds_lib):
    """Skip-free GPU guard: on a GPU test run a missing device is a failure."""
    import torch
    assert torch.cuda.is_available(), "GPU test selected but no HIP device is visible"
    from vds_amd import _lib
    assert _lib.device_count() > 0
    return torch.device("cuda:0")
