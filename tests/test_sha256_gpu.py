"""GPU SHA-256 of replicas.

The reference names each replica by hash::signature(hash::sha256(), replica)
(dht_network_client.cpp:79, :593; kernel/vds_crypto/hash.cpp:91-101, OpenSSL
EVP_sha256).  The checker is FIPS 180-4 itself: the standard's example
digests, and Python's hashlib (OpenSSL) for everything else.  Bit-exact.
"""
import hashlib

import numpy as np
import pytest

import oracle_ctypes as O

pytestmark = pytest.mark.gpu

FIPS = {  # FIPS 180-4 / NIST example messages
    b"": "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855",
    b"abc": "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad",
    b"abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq":
        "248d6a61d20638b8e5c026930c3e6039a33ce45964ff2167f6ecedd419db06c1",
}


@pytest.fixture(scope="module")
def chunk(gpu):
    from vds_amd import chunk as c
    return c


def gpu_digests(chunk, torch, buf: np.ndarray, length: int, stride: int, count: int, offset: int = 0):
    dev = torch.from_numpy(np.ascontiguousarray(buf)).cuda()
    dig = torch.zeros((max(count, 1), 32), dtype=torch.uint8, device="cuda")
    chunk.sha256_device(dev.data_ptr() + offset, length, stride, count, dig)
    torch.cuda.synchronize()
    return [bytes(d) for d in dig.cpu().numpy()[:count]]


def test_fips_examples(chunk):
    import torch
    for msg, want in FIPS.items():
        buf = np.frombuffer(msg + b"\0", dtype=np.uint8)
        assert gpu_digests(chunk, torch, buf, len(msg), 0, 1)[0].hex() == want


@pytest.mark.parametrize("offset", [0, 1, 2, 3])
def test_lengths_and_alignments_vs_hashlib(chunk, offset):
    """Every length 0..200 (all padding cases: 55/56/63/64/119/120 ...) at
    every start alignment, many messages per launch."""
    import torch
    rng = np.random.default_rng(offset)
    for length in list(range(0, 201)) + [1000, 4099, 65536 + 7]:
        stride = length + 5
        count = 7
        buf = rng.integers(0, 256, size=offset + stride * count + 8, dtype=np.uint8)
        got = gpu_digests(chunk, torch, buf, length, stride, count, offset)
        for j in range(count):
            s = offset + j * stride
            assert got[j] == hashlib.sha256(buf[s:s + length].tobytes()).digest(), (length, offset, j)


def test_replica_names_of_a_batch(chunk):
    """The device form over bench.py's replica layout [n][objects][L]: every
    replica's name equals hashlib over the oracle's replica bytes."""
    import torch
    k, n, size, objects = 16, 20, 2 * 65536 + 321, 3
    L = chunk.replica_size(k, size)
    reps = np.stack([np.stack([O.encode(k, r, O.splitmix(0x7664730000000000 + o, size)) for o in range(objects)])
                     for r in range(n)])  # (n, objects, L)
    got = gpu_digests(chunk, torch, reps.reshape(-1), L, L, n * objects)
    for r in range(n):
        for o in range(objects):
            assert got[r * objects + o] == hashlib.sha256(reps[r, o].tobytes()).digest()


@pytest.mark.parametrize("size", [0, 1, 31, 1 << 20, 3 * 65536 + 77])
def test_encode_hash_host(chunk, size):
    """save_temp / save_data: replica bytes and their SHA-256 names in one call."""
    k, n = 16, 20
    data = O.splitmix(0x7664730000000000 + size, size)
    reps, names = chunk.encode_hash_host(k, list(range(n)), data)
    for r in range(n):
        want = O.encode(k, r, data)
        assert np.array_equal(reps[r], want)
        assert names[r] == hashlib.sha256(want.tobytes()).digest()
