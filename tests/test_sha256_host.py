"""Host SHA-256 (vds_ec_sha256_host, sha256_host.cpp): upload_data's body hash
(server_api.cpp:16 -> hash::signature(sha256), kernel/vds_crypto/hash.cpp:
91-101, OpenSSL EVP_sha256), computed on the caller's thread by
vds_ec_save_temp16_host.  No GPU needed.  Checked against FIPS 180-4's
examples and hashlib (OpenSSL) at every length around the block and padding
boundaries, for the SHA-extension code and the portable code
(VDS_EC_HOST_SHA=portable, in a child process)."""
import ctypes as C
import hashlib
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHECK = r"""
import ctypes as C, hashlib, sys
import numpy as np
sys.path.insert(0, %(root)r)
from vds_amd import _lib
lib = _lib.lib()
rng = np.random.default_rng(3)
msgs = [b"", b"abc", b"abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq", b"a" * 1000000]
msgs += [rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in list(range(0, 300)) + [65536, 65536 + 55, 2050]]
bad = 0
for m in msgs:
    out = (C.c_uint8 * 32)()
    buf = C.create_string_buffer(m, len(m) or 1)
    assert lib.vds_ec_sha256_host(buf, len(m), out) == 0
    bad += bytes(out) != hashlib.sha256(m).digest()
print("bad", bad, "of", len(msgs))
sys.exit(1 if bad else 0)
"""


def _run(env_extra):
    env = dict(os.environ, **env_extra)
    r = subprocess.run([sys.executable, "-c", CHECK % {"root": ROOT}], env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr[-3000:]
    assert "bad 0 of" in r.stdout


def test_host_sha256_default_vs_hashlib():
    _run({})


def test_host_sha256_portable_vs_hashlib():
    _run({"VDS_EC_HOST_SHA": "portable"})


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
