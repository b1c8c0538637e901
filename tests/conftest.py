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

# the tests exercise the run-time compiler itself, not the on-disk cache of
# its outputs (tests/test_jit_gpu.py covers the cache in its own processes)
os.environ["VDS_EC_JIT_CACHE"] = "0"


def _dump_runtime_libs():
    """At exit, record which ROCm shared objects are mapped (one HIP runtime expected)."""
    out = os.environ.get("VDS_EC_MAPS_DUMP")
    if not out:
        return
    libs = set()
    with open("/proc/self/maps") as f:
        for line in f:
            parts = line.split()
            if len(parts) >= 6 and any(x in parts[5] for x in ("amdhip", "comgr", "hiprtc", "hsa-runtime",
                                                               "drm", "vds_ec", "oracle")):
                libs.add(parts[5])
    with open(out, "w") as f:
        f.write("\n".join(sorted(libs)) + "\n")


def pytest_configure(config):
    import atexit
    atexit.register(_dump_runtime_libs)
    config.addinivalue_line("markers", "gpu: needs a HIP GPU (MI355X); parity tests through the C ABI")


@pytest.fixture(scope="session")
def vds_lib():
    """The built in-tree libvds_ec.so (built on demand)."""
    from vds_amd import build
    build.build()
    from vds_amd import _lib
    lib = _lib.lib()
    # run-time compiled restore kernels off, so every test sees the path it
    # asserts; tests/test_jit_gpu.py switches them on
    lib.vds_ec_jit_set_mode(0)
    return lib


@pytest.fixture(scope="session")
def gpu(vds_lib):
    """Skip-free GPU guard: on a GPU test run a missing device is a failure."""
    import torch
    assert torch.cuda.is_available(), "GPU test selected but no HIP device is visible"
    from vds_amd import _lib
    assert _lib.device_count() > 0
    return torch.device("cuda:0")
