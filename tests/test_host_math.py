"""Host build of tests/cpp/test_bitslice.cpp: the bit-sliced plane arithmetic,
transposes and field helpers the kernels share (vds_amd/csrc/bitslice.hpp,
gf_common.hpp), compiled with g++ and run on the CPU -- including the
Itoh-Tsujii inverse of the RT coefficient kernel against gf16_pow on every
element, and the survey's GF KATs."""
import os
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bitslice_host():
    with tempfile.TemporaryDirectory() as d:
        exe = os.path.join(d, "t")
        subprocess.run(["g++", "-O2", "-std=c++20", "-I", os.path.join(ROOT, "vds_amd", "csrc"),
                        os.path.join(ROOT, "tests", "cpp", "test_bitslice.cpp"), "-o", exe], check=True)
        r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stdout + r.stderr
