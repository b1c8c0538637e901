"""Content-addressed replica paths (on-disk layout).

The reference stores a replica at <storage>/<b64[0:10]>/<b64[10:20]>/<b64[20:]>
with b64 = base64(sha256(replica)) ('+' -> '#', '/' -> '_'):
dht_network_client.cpp:483-505 (save_data(file)) and :632-653 (save_data),
base64::from_bytes = encoding.cpp:136-174 (standard alphabet, '=' padding).
The checker restates that with Python's base64 module.  Host only (no GPU).
"""
import base64
import hashlib

import numpy as np


def reference_path(digest: bytes) -> str:
    p = base64.b64encode(digest).decode().replace("+", "#").replace("/", "_")
    return p[0:10] + "/" + p[10:20] + "/" + p[20:]


def test_paths_match_reference_layout(vds_lib):
    from vds_amd import chunk
    rng = np.random.default_rng(7)
    digests = [hashlib.sha256(rng.integers(0, 256, n, dtype=np.uint8).tobytes()).digest() for n in range(200)]
    digests += [b"\xff" * 32, b"\x00" * 32, bytes(range(32)), b"\xfb\xef\xbe" * 10 + b"\xfb\xef"]
    got = chunk.replica_storage_paths(digests)
    assert got == [reference_path(d) for d in digests]
    assert all(len(p) == 46 and "+" not in p and p.count("/") == 2 for p in got)
    assert any("#" in p for p in got) and any("_" in p for p in got)
