"""Host SHA-256 (vds_ec_sha256_host, sha256_host.cpp): upload_data's body hash
(server_api.cpp:16 -> hash::signature(sha256), kernel/vds_crypto/hash.cpp:
91-101, OpenSSL EVP_sha256), computed on the caller's thread by
vds_ec_save_temp16_host.  No GPU needed.  Checked against FIPS 180-4's
examples and hashlib (OpenSSL) at every length around the block and padding
boundaries, for the SHA-extension code and the portable code (the file
compiled on its own with and without -DVDS_HOST_SHA_PORTABLE=1)."""
import ctypes as C
import hashlib
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SRC = os.path.join(ROOT, "vds_amd", "csrc", "sha256_host.cpp")


def _host_lib(tmp_path, portable):
    """sha256_host.cpp alone as a host shared library (g++), the portable
    code forced by -DVDS_HOST_SHA_PORTABLE=1 or the default selection."""
    so = tmp_path / ("sha_portable.so" if portable else "sha_default.so")
    cmd = ["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-I", os.path.join(ROOT, "include"), SRC, "-o", str(so)]
    if portable:
        cmd.insert(1, "-DVDS_HOST_SHA_PORTABLE=1")
    subprocess.run(cmd, check=True, timeout=300)
    return C.CDLL(str(so))


def _check(lib):
    rng = np.random.default_rng(3)
    msgs = [b"", b"abc", b"abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq", b"a" * 1000000]
    msgs += [rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in list(range(0, 300)) + [65536, 65536 + 55, 2050]]
    bad = 0
    for m in msgs:
        out = (C.c_uint8 * 32)()
        buf = C.create_string_buffer(m, len(m) or 1)
        assert lib.vds_ec_sha256_host(buf, C.c_uint64(len(m)), out) == 0
        bad += bytes(out) != hashlib.sha256(m).digest()
    assert bad == 0, f"{bad} of {len(msgs)} digests differ"


def test_host_sha256_default_vs_hashlib(tmp_path):
    _check(_host_lib(tmp_path, False))


def test_host_sha256_portable_vs_hashlib(tmp_path):
    _check(_host_lib(tmp_path, True))


def test_host_sha256_fips_and_errors():
    from vds_amd import _lib
    lib = _lib.lib()
    out = (C.c_uint8 * 32)()
    assert lib.vds_ec_sha256_host(b"abc", 3, out) == 0
    assert bytes(out).hex() == "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad"
    assert lib.vds_ec_sha256_host(None, 3, out) != 0  # EINVAL: bytes but no pointer
    assert lib.vds_ec_sha256_host(None, 0, out) == 0
    assert bytes(out) == hashlib.sha256(b"").digest()
    assert lib.vds_ec_sha256_host(b"abc", 3, None) != 0
