"""The C++ drop-in (vds_amd/include/vds_data/{gf.h,chunk.h,chunk_storage.h})
compiles against the reference's API and runs the reference's own tests
(tests/test_vds_data/gf_tests.cpp, chunk_tests.cpp), re-hosted in
tests/cpp/test_dropin.cpp.

CPU: build + gf_tests (gf<m>, gf_math<> -- host-side field helpers) + the
     no-GPU contract (data-path calls fail loudly).
GPU: chunk_tests (cell arrays uint8/uint16, 800-of-1000 chunk_storage
     round trip) and chunk_output_async == one-shot write.
"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def dropin_bin(vds_lib, tmp_path_factory):
    out = tmp_path_factory.mktemp("dropin") / "test_dropin"
    cmd = ["g++", "-O2", "-std=c++20", "-fcoroutines",
           "-I", os.path.join(ROOT, "include"),
           "-I", os.path.join(ROOT, "vds_amd", "include", "vds_data"),
           "-I", os.path.join(ROOT, "vds_amd", "include", "vds_core_compat"),
           os.path.join(ROOT, "tests", "cpp", "test_dropin.cpp"),
           os.path.join(ROOT, "vds_amd", "dropin", "chunk_storage.cpp"),
           "-L", os.path.join(ROOT, "vds_amd"), "-lvds_ec",
           "-Wl,-rpath," + os.path.join(ROOT, "vds_amd"), "-o", str(out)]
    subprocess.run(cmd, check=True)
    return str(out)


def test_dropin_gf_tests_cpu(dropin_bin):
    r = subprocess.run([dropin_bin, "gf"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "gf OK" in r.stdout


def _has_gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.mark.skipif(_has_gpu(), reason="checks the no-GPU contract")
def test_dropin_fails_loudly_without_gpu(dropin_bin):
    r = subprocess.run([dropin_bin, "chunk"], capture_output=True, text=True)
    assert r.returncode != 0
    assert "no CPU fallback" in (r.stdout + r.stderr)


@pytest.mark.gpu
def test_dropin_chunk_tests_gpu(dropin_bin):
    for seed in ("1", "2", "3"):
        r = subprocess.run([dropin_bin, "chunk", seed], capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stdout + r.stderr
        assert "chunk OK" in r.stdout
