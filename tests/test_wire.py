"""Wire formats of the live upload path.

CPU: base64::to_bytes / from_bytes (encoding.cpp:138-247) against Python's
base64 on valid input and against a line-by-line Python restatement of the
reference's decode loop on malformed input (its quirks: the trailing-'=' count
decides the length, the first '=' ends the decode); save_temp's tmp-file
names (dht_network_client.cpp:91-95); the websocket "upload" answer
(websocket_api.cpp:120-121, 472-482, json_writer.cpp) parsed back with json.
GPU: vds_ec_save_temp16_host against the oracle's encode and hashlib.
"""
import base64
import hashlib
import json
import os
import random

import numpy as np
import pytest

import oracle_ctypes as O

ALPHA = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/"


def ref_to_bytes(data: bytes):
    """Restatement of base64::to_bytes (encoding.cpp:181-247): returns bytes,
    or the reference's error text.  Output bytes the reference leaves
    unwritten (malloc'd, never set on an early '=') are 0 here, as in the
    product."""
    if len(data) % 4:
        return "Non-Valid base64!"
    padding = 0
    if len(data) > 0 and data[-1:] == b"=":
        padding += 1
        if len(data) > 1 and data[-2:-1] == b"=":
            padding += 1
    out = bytearray((len(data) // 4) * 3 - padding)
    temp = 0
    offset = 0
    qp = 0
    for ch in data:
        temp = (temp << 6) & 0xFFFFFFFF
        if 0x41 <= ch <= 0x5A:
            temp |= ch - 0x41
        elif 0x61 <= ch <= 0x7A:
            temp |= ch - 0x47
        elif 0x30 <= ch <= 0x39:
            temp |= ch + 0x04
        elif ch == 0x2B:
            temp |= 0x3E
        elif ch == 0x2F:
            temp |= 0x3F
        elif ch == 0x3D:
            if padding == 1:
                out[offset] = (temp >> 16) & 0xFF
                offset += 1
                out[offset] = (temp >> 8) & 0xFF
                return bytes(out)
            if padding == 2:
                out[offset] = (temp >> 10) & 0xFF
                return bytes(out)
            return "Invalid Padding in Base 64!"
        else:
            return "Non-Valid Character in Base 64!"
        qp += 1
        if qp == 4:
            out[offset:offset + 3] = bytes([(temp >> 16) & 0xFF, (temp >> 8) & 0xFF, temp & 0xFF])
            offset += 3
            qp = 0
    return bytes(out)


def _decode(text: bytes):
    from vds_amd import chunk
    from vds_amd._lib import VdsEcError
    try:
        return chunk.base64_decode(text)
    except VdsEcError as e:
        return str(e).split(": ", 1)[-1]


def test_base64_roundtrip_matches_python(vds_lib):
    from vds_amd import chunk
    rng = random.Random(7)
    for n in list(range(0, 70)) + [1000, 65536, 65537, 65538]:
        data = bytes(rng.getrandbits(8) for _ in range(n))
        enc = chunk.base64_encode(data)
        assert enc == base64.b64encode(data).decode()
        assert chunk.base64_decode(enc) == data


def test_base64_malformed_follows_reference(vds_lib):
    rng = random.Random(11)
    cases = [b"", b"=", b"==", b"===", b"====", b"A===", b"AA==", b"AAA=", b"A=AA", b"AB=C", b"QQ==QQ==",
             b"AAAA====", b"ABC=AB==", b"=AA=", b"AAAAAAA=", b"AA*A", b"AA\x80A", b"QUE=", b"QUJD", b"Q", b"QUJDRA"]
    for _ in range(400):  # random strings over the alphabet, '=' and a few strays
        n = 4 * rng.randint(0, 4) + (rng.random() < 0.2) * rng.randint(1, 3)
        cases.append(bytes(rng.choice(ALPHA.encode() + b"====*-\x00\xff") for _ in range(n)))
    for c in cases:
        assert _decode(c) == ref_to_bytes(c), c


def test_tmp_names(vds_lib):
    from vds_amd import chunk
    digests = [hashlib.sha256(bytes([i]) * i).digest() for i in range(40)]
    names = chunk.tmp_names(digests)
    for d, name in zip(digests, names):
        assert name == base64.b64encode(d).decode().replace("+", "#").replace("/", "_")
        assert len(name) == 44
    # the storage path of save_data is the same name split 10/10/rest
    paths = chunk.replica_storage_paths(digests)
    assert [p.replace("/", "") for p in paths] == names


def test_upload_response_json(vds_lib):
    from vds_amd import chunk
    reps = [hashlib.sha256(b"r%d" % i).digest() for i in range(64)]
    data_hash = hashlib.sha256(b"body").digest()
    for rid in (0, 7, 123456, -1):
        text = chunk.upload_response_json(rid, reps, data_hash, 2050)
        assert " " not in text and "\n" not in text
        doc = json.loads(text)
        # json_writer: every primitive is a string, properties in insertion order
        assert list(doc) == ["id", "result"] and list(doc["result"]) == ["replicas", "hash", "replica_size"]
        assert doc["id"] == str(rid % (1 << 64))
        assert doc["result"]["replicas"] == [base64.b64encode(r).decode() for r in reps]
        assert doc["result"]["hash"] == base64.b64encode(data_hash).decode()
        assert doc["result"]["replica_size"] == "2050"
    assert chunk.upload_response_json(3, [], data_hash, 2) == \
        '{"id":"3","result":{"replicas":[],"hash":"%s","replica_size":"2"}}' % base64.b64encode(data_hash).decode()


@pytest.mark.gpu
def test_save_temp_and_upload_live_shape(gpu):
    """The live upload at the production constants (k = 32, n = 64,
    dht_network.h:22-25) on a ~64 KiB body (web/src/store/vds_api.jsx:76,
    deflated and encrypted by the client, so any length)."""
    from vds_amd import chunk
    rng = np.random.default_rng(5)
    for size in (0, 1, 65, 4096, 58113, 65536, 65552):
        body = rng.integers(0, 256, size, dtype=np.uint8)
        b64 = base64.b64encode(body.tobytes()).decode()
        res = chunk.upload(42, b64)
        want_hash = hashlib.sha256(body.tobytes()).digest()
        assert res["data_hash"] == want_hash
        for r in (0, 1, 31, 32, 63):
            ref = O.encode(32, r, body)
            assert np.array_equal(res["replicas"][r], ref), (size, r)
            assert res["replica_digests"][r] == hashlib.sha256(ref.tobytes()).digest()
        assert res["tmp_names"] == chunk.tmp_names([hashlib.sha256(O.encode(32, r, body).tobytes()).digest()
                                                   for r in range(64)])
        doc = json.loads(res["json"])
        assert doc["result"]["hash"] == base64.b64encode(want_hash).decode()
        assert doc["result"]["replica_size"] == str(O.replica_size(2, 32, size))
