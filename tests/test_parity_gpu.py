"""GPU parity tests: the HIP path (through the C ABI) against the oracle.

Bit-exact for every byte (integer/byte arithmetic: no tolerance).  Covers
the bit-sliced fast kernels (k=16/n=20, k=32/n=40, k=4/n=6 with contiguous
replica ids and >= one 2048-stripe tile) and the generic kernels (every other
shape, the tails, the trailers), both cell widths, the cell-array test paths,
the reference's own round-trip tests re-hosted, and full BASELINE sizes via
frozen oracle SHA-256s and round-trip properties.
"""
import hashlib
import json
import os

import numpy as np
import pytest

import oracle_ctypes as O

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
with open(os.path.join(GOLDEN, "golden_vectors.json")) as _f:
    G = json.load(_f)
SEED = G["seed_base"]


def sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.fixture(scope="module")
def ec(gpu):
    import vds_amd
    return vds_amd


# ------------------------------------------------------------------ helpers

def dev_object(torch, size, index):
    from vds_amd import chunk
    t = torch.empty(max(size, 1), dtype=torch.uint8, device="cuda")
    chunk.fill_splitmix_device(t, size, SEED + index)
    return t


def dev_encode(torch, k, n, t, size, count=1, stride=None, replicas=None):
    """Encode `count` objects laid out at `stride` in t; returns [count][n] uint8 tensors."""
    from vds_amd import chunk
    replicas = list(range(n)) if replicas is None else replicas
    L = chunk.replica_size(k, size)
    stride = size if stride is None else stride
    out = torch.zeros((len(replicas), count, max(L, 1)), dtype=torch.uint8, device="cuda")
    ptrs = [out[i].data_ptr() for i in range(len(replicas))]
    chunk.encode_device(k, replicas, t, size, stride, count, ptrs, out.shape[2])
    torch.cuda.synchronize()
    return out[:, :, :L]


# ------------------------------------------------------------------- inputs

def test_fill_splitmix_matches_oracle(ec):
    import torch
    for size, idx in ((0, 0), (1, 1), (7, 2), (8, 3), (1000, 4), (1 << 20, 5)):
        t = dev_object(torch, size, idx)
        assert t[:size].cpu().numpy().tobytes() == O.splitmix(SEED + idx, size).tobytes()


# ------------------------------------------------------------------- encode

def test_encode_small_golden_host_api(ec):
    for e in G["encode16_small"]:
        d = O.splitmix(SEED + e["object_index"], e["size"])
        outs = ec.chunk.encode_host(e["k"], list(range(6)), d)
        for r, hexs in e["replicas"].items():
            assert outs[int(r)].tobytes().hex() == hexs
        for r in range(6):  # per-replica drop-in call (chunk_generator::write)
            assert ec.ChunkGenerator(e["k"], r).write(d).tobytes().hex() == e["replicas"][str(r)]


def test_per_replica_loop_window(ec):
    """The drop-in per-replica loop (save_temp, dht_network_client.cpp:74-79):
    calls for replicas 0..n-1 of one buffer are served from an encoded window
    (vds_ec_api.cpp encode_host).  Every call must still give the encode of
    the buffer's CURRENT bytes: in-place edits, skipped / repeated / backward
    ids, other shapes in between, and the 8-bit generator."""
    k, n, size = 32, 64, 65536 - 77
    d = O.splitmix(SEED + 901, size).copy()
    gens = [ec.ChunkGenerator(k, r) for r in range(n)]
    want = {r: O.encode(k, r, d) for r in range(n)}
    for r in range(n):
        assert gens[r].write(d).tobytes() == want[r].tobytes(), f"replica {r}"
    for r in (63, 5, 5, 6, 7, 2, 64, 65):  # out of order, repeated, past the window
        assert ec.ChunkGenerator(k, r).write(d).tobytes() == O.encode(k, r, d).tobytes(), f"replica {r}"
    # same buffer edited in place mid-loop: the calls after the edit see it
    for r in range(10):
        if r == 4:
            d[1000] ^= 0x5A
            want = {q: O.encode(k, q, d) for q in range(4, 10)}
        got = gens[r].write(d)
        if r >= 4:
            assert got.tobytes() == want[r].tobytes(), f"replica {r} after edit"
    # a different shape / width / trailer flag between calls of the same loop
    e = O.splitmix(SEED + 902, 4099)
    assert gens[10].write(d).tobytes() == O.encode(k, 10, d).tobytes()
    assert ec.ChunkGenerator(16, 11).write(d).tobytes() == O.encode(16, 11, d).tobytes()
    assert gens[11].write(d, write_padding=False).tobytes() == O.encode(k, 11, d, write_padding=False).tobytes()
    assert gens[12].write(e).tobytes() == O.encode(k, 12, e).tobytes()
    assert ec.ChunkGenerator(8, 13, cell_bytes=1).write(e).tobytes() == O.encode(8, 13, e, 1).tobytes()
    assert ec.ChunkGenerator(8, 14, cell_bytes=1).write(e).tobytes() == O.encode(8, 14, e, 1).tobytes()
    assert gens[13].write(d).tobytes() == O.encode(k, 13, d).tobytes()
    # the 8-bit ids stop at 255
    for r in (253, 254, 255):
        assert ec.ChunkGenerator(8, r, cell_bytes=1).write(e).tobytes() == O.encode(8, r, e, 1).tobytes()
    assert ec.chunk.encode_host(k, [3], np.zeros(0, np.uint8))[0].tobytes() == O.encode(k, 3, np.zeros(0, np.uint8)).tobytes()


@pytest.mark.parametrize("entry", G["encode16_sha"], ids=lambda e: f"k{e['k']}n{e['n']}s{e['size']}")
def test_encode_golden_sha(ec, entry):
    import torch
    k, n, size = entry["k"], entry["n"], entry["size"]
    t = dev_object(torch, size, entry["object_index"])
    out = dev_encode(torch, k, n, t, size)
    for r in range(n):
        assert sha(out[r, 0].cpu().numpy()) == entry["sha256"][str(r)], f"replica {r}"
    if "head64" in entry:
        for r in range(n):
            assert out[r, 0, :64].cpu().numpy().tobytes().hex() == entry["head64"][str(r)]


def test_encode_special_inputs(ec):
    for e in G["encode16_special"]:
        d = np.full(e["size"], e["fill"], dtype=np.uint8)
        outs = ec.chunk.encode_host(e["k"], list(range(e["n"])), d)
        for r in range(e["n"]):
            assert sha(outs[r]) == e["sha256"][str(r)]


def test_encode_random_shapes_vs_oracle(ec):
    rng = np.random.default_rng(11)
    for trial in range(40):
        k = int(rng.integers(1, 41))
        size = int(rng.choice([0, 1, 2, 3, int(rng.integers(1, 5000)), int(rng.integers(5000, 300000))]))
        n = int(rng.integers(1, 9))
        ids = [int(x) for x in rng.choice(70000 if trial % 2 else 64, n, replace=False) % 65536]
        d = rng.integers(0, 256, size, dtype=np.uint8)
        outs = ec.chunk.encode_host(k, ids, d)
        for i, r in enumerate(ids):
            assert np.array_equal(outs[i], O.encode(k, r, d)), (k, size, r)
        nopad = ec.chunk.encode_host(k, ids[:1], d, write_padding=False)[0]
        assert np.array_equal(nopad, O.encode(k, ids[0], d, write_padding=False))


@pytest.mark.parametrize("k,n", [(16, 20), (32, 40), (4, 6)])
def test_fast_encode_tiles_and_tail_vs_oracle(ec, k, n):
    """>= 1 bit-sliced tile plus a ragged tail and a partial last stripe."""
    import torch
    from vds_amd import _lib
    tile_bytes = 2048 * 2 * k
    for size in (tile_bytes, tile_bytes + 1, 3 * tile_bytes + 2 * k * 5 + 3):
        assert _lib.lib().vds_ec_encode16_path(k, (np.arange(n, dtype=np.uint16)).ctypes.data_as(_lib.u16p),
                                               n, size) == 2
        t = dev_object(torch, size, 1000 + size % 97)
        d = t[:size].cpu().numpy()
        out = dev_encode(torch, k, n, t, size)
        for r in range(n):
            assert np.array_equal(out[r, 0].cpu().numpy(), O.encode(k, r, d)), (k, size, r)


def test_fast_equals_generic_path(ec):
    import torch
    k, n, size = 16, 20, 5 * 65536 + 123
    t = dev_object(torch, size, 77)
    fast = dev_encode(torch, k, n, t, size)
    perm = list(range(n))[::-1]  # non-contiguous ids -> generic kernel
    gen = dev_encode(torch, k, n, t, size, replicas=perm)
    for i, r in enumerate(perm):
        assert torch.equal(fast[r], gen[i])


@pytest.mark.parametrize("k,align", [(16, 256), (32, 4096)])
def test_bench_layout_aligned_replica_stride(ec, k, align):
    """bench.py's layout: replica buffers [n][objects][Ls] with the replica
    stride Ls = L rounded up to `align` (every replica starts aligned, as the
    reference's own heap buffers do).  Every replica equals the oracle's,
    the gaps stay untouched, and the syndrome restore from the survivors at
    chunk stride Ls gives back the objects."""
    import torch
    from vds_amd import chunk
    n, size, count = k + k // 4, 1 << 20, 3
    L = chunk.replica_size(k, size)
    Ls = -(-L // align) * align
    t = torch.empty(size * count, dtype=torch.uint8, device="cuda")
    for o in range(count):
        chunk.fill_splitmix_device(t[o * size:], size, SEED + 1300 + o)
    reps = torch.zeros((n, count * Ls), dtype=torch.uint8, device="cuda")
    chunk.encode_device(k, list(range(n)), t, size, size, count, [reps[i].data_ptr() for i in range(n)], Ls)
    erased = list(range(0, n, 5))[: n - k]
    nodes = [r for r in range(n) if r not in erased]
    out = torch.empty(size * count, dtype=torch.uint8, device="cuda")
    chunk.restore_device(k, nodes, [reps[r].data_ptr() for r in nodes], L, Ls, size % (2 * k), count, out, size)
    torch.cuda.synchronize()
    host = reps.view(n, count, Ls).cpu().numpy()
    for o in range(count):
        d = O.splitmix(SEED + 1300 + o, size)
        for r in range(n):
            assert np.array_equal(host[r, o, :L], O.encode(k, r, d)), f"object {o} replica {r}"
            assert not host[r, o, L:].any()
        assert np.array_equal(out[o * size:(o + 1) * size].cpu().numpy(), d)


def test_batched_objects_with_strides(ec):
    import torch
    k, n, size, count = 16, 20, 2 * 65536 + 1000, 5
    stride = size + 4096
    t = torch.empty(stride * count, dtype=torch.uint8, device="cuda")
    from vds_amd import chunk
    for o in range(count):
        chunk.fill_splitmix_device(t[o * stride:], size, SEED + 500 + o)
    out = dev_encode(torch, k, n, t, size, count=count, stride=stride)
    for o in range(count):
        d = O.splitmix(SEED + 500 + o, size)
        for r in (0, 1, 7, 19):
            assert np.array_equal(out[r, o].cpu().numpy(), O.encode(k, r, d))


@pytest.mark.parametrize("k,n,size,count,pad", [
    (32, 64, 65536, 5, 0),       # the live shape (dht_network.h:22-25): tiles straddle objects
    (32, 64, 65536, 3, 2),       # 4-byte-aligned replica stride
    (16, 20, 12288, 11, 0),      # 3 groups per object, stream tail in the middle of object 10
    (16, 20, 12288 + 7, 6, 0),   # + a partial last stripe per object
    (32, 40, 4 * 8192, 9, 6),
    (16, 20, 2 * 65536 + 1000, 3, 0),  # F % 128 != 0: whole tiles per object, generic rest
])
def test_fast_encode_object_stream(ec, k, n, size, count, pad):
    """Batches of small objects ride the bit-sliced kernel as one stripe
    stream (tiles cross object boundaries); every replica byte, trailer
    included, equals the oracle's, and nothing is written past a replica."""
    import torch
    from vds_amd import chunk
    L = chunk.replica_size(k, size)
    stride = size + 16
    t = torch.empty(stride * count, dtype=torch.uint8, device="cuda")
    for o in range(count):
        chunk.fill_splitmix_device(t[o * stride:], size, SEED + 900 + o)
    out = torch.zeros((n, count, L + pad), dtype=torch.uint8, device="cuda")
    chunk.encode_device(k, list(range(n)), t, size, stride, count, [out[i].data_ptr() for i in range(n)], L + pad)
    torch.cuda.synchronize()
    host = out.cpu().numpy()
    assert chunk._lib.lib().vds_ec_encode16_path(k, np.arange(n, dtype=np.uint16).ctypes.data_as(chunk._lib.u16p),
                                                  n, size) == 2
    for o in range(count):
        d = O.splitmix(SEED + 900 + o, size)
        for r in range(n):
            assert np.array_equal(host[r, o, :L], O.encode(k, r, d)), f"object {o} replica {r}"
            assert not host[r, o, L:].any()


# ------------------------------------------------------------------ restore

@pytest.mark.parametrize("k,nodes,size,count", [
    (32, list(range(1, 64, 2)), 65536, 5),                 # live shape: 2 groups per object, tiles straddle
    (16, list(range(20, 36)), 16384, 7),                   # runtime-coefficient kernel, 1 group per object
    (16, list(range(20, 36)), 3 * 16384 + 9, 4),          # + a partial stripe (generic tail per object)
    (32, list(range(8, 40)), 2 * 131072 + 64 * 512, 3),   # whole tiles + a stream of groups
    (32, [r for r in range(40) if r % 5], 65536, 5),      # syndrome-kernel survivors, objects under one tile
    (16, list(range(4, 20)), 16384, 7),                    # the same at k = 16
])
def test_fast_restore_object_stream(ec, k, nodes, size, count):
    """Batches of small objects on the bit-sliced runtime-coefficient restore
    (512-stripe groups, tiles across object boundaries) plus the generic
    remainder: every object comes back bit-exact, nothing written past it."""
    import torch
    from vds_amd import chunk
    L = chunk.replica_size(k, size)
    objs = [O.splitmix(SEED + 1300 + o, size) for o in range(count)]
    reps = np.stack([np.stack([O.encode(k, r, d) for d in objs]) for r in nodes])  # (k, count, L)
    dev = torch.from_numpy(reps).cuda()
    out = torch.zeros((count, size + 64), dtype=torch.uint8, device="cuda")
    chunk.restore_device(k, nodes, [dev[j].data_ptr() for j in range(k)], L, L, size % (2 * k), count, out, size + 64)
    torch.cuda.synchronize()
    host = out.cpu().numpy()
    for o in range(count):
        assert np.array_equal(host[o, :size], objs[o]), f"object {o}"
        assert not host[o, size:].any()


@pytest.mark.parametrize("entry", G["restore16"], ids=lambda e: f"k{e['k']}s{e['size']}")
def test_restore_golden(ec, entry):
    k, size = entry["k"], entry["size"]
    d = O.splitmix(SEED + entry["object_index"], size)
    chunks = [O.encode(k, r, d) for r in entry["nodes"]]
    out = ec.ChunkRestore(k, entry["nodes"]).restore(chunks)
    assert sha(out) == entry["sha256"]
    assert out.tobytes() == d.tobytes()


def test_restore_random_vs_oracle(ec):
    rng = np.random.default_rng(5)
    for trial in range(30):
        k = int(rng.integers(1, 35))
        size = int(rng.choice([0, 1, 2, int(rng.integers(1, 3000)), int(rng.integers(3000, 200000))]))
        d = rng.integers(0, 256, size, dtype=np.uint8)
        nodes = [int(x) for x in rng.choice(65536 if trial % 3 == 0 else 80, k, replace=False)]
        chunks = [O.encode(k, r, d) for r in nodes]
        out = ec.ChunkRestore(k, nodes).restore(chunks)
        ref = O.restore(k, nodes, chunks)
        assert ref is not None and np.array_equal(out, ref), (k, size)


@pytest.mark.parametrize("k,n", [(16, 20), (32, 40)])
def test_fast_restore_tiles_and_tail(ec, k, n):
    import torch
    from vds_amd import chunk, _lib
    tile_bytes = 2048 * 2 * k
    for size in (tile_bytes, 2 * tile_bytes + 2 * k * 3 + 1):
        t = dev_object(torch, size, 2000 + size % 89)
        enc = dev_encode(torch, k, n, t, size)
        for erased in ([0, 1, 2, 3][: n - k], list(range(n - (n - k), n)), list(range(0, n, n // (n - k)))[: n - k]):
            nodes = [r for r in range(n) if r not in erased][:k]
            L = enc.shape[2]
            assert _lib.lib().vds_ec_restore16_path(k, None, L, size % (2 * k), 1) == 2
            out = torch.zeros(size + 64, dtype=torch.uint8, device="cuda")
            chunk.restore_device(k, nodes, [enc[r, 0].data_ptr() for r in nodes], L, 0, size % (2 * k), 1, out, 0)
            torch.cuda.synchronize()
            assert torch.equal(out[:size], t[:size]), (size, erased)
            assert int(out[size:].sum().item()) == 0  # trimmed to E bytes


def _path(k, nodes, L, padding=0, count=1):
    from vds_amd import _lib
    arr = np.asarray(nodes, dtype=np.uint16)
    return _lib.lib().vds_ec_restore16_path(k, arr.ctypes.data_as(_lib.u16p), L, padding, count)


@pytest.mark.parametrize("k,n", [(16, 20), (32, 40)])
def test_syndrome_restore_erasure_patterns(ec, k, n):
    """k_restore_syn<16,20> / <32,40>: any k of the n replicas, in any order."""
    import itertools
    import torch
    from vds_amd import chunk
    m = n - k
    size = 2 * 2048 * 2 * k + 2 * k * 5 + 3  # two full tiles + generic tail
    t = dev_object(torch, size, 2100 + k)
    enc = dev_encode(torch, k, n, t, size)
    L = enc.shape[2]
    rng = np.random.default_rng(21)
    picks = [tuple(range(m)), tuple(range(k, n)), tuple(range(0, n, n // m))[:m], tuple(range(k - m // 2, k + m // 2))]
    if k == 16:
        combos = list(itertools.combinations(range(n), m))
        picks += [combos[i] for i in rng.choice(len(combos), 300, replace=False)]
    else:  # C(40, 8) patterns: a random sample
        picks += [tuple(sorted(int(x) for x in rng.choice(n, m, replace=False))) for _ in range(120)]
    out = torch.zeros(size + 64, dtype=torch.uint8, device="cuda")
    for erased in picks:
        nodes = [r for r in range(n) if r not in erased]
        rng.shuffle(nodes)
        assert _path(k, nodes, L) == 3
        out.zero_()
        chunk.restore_device(k, nodes, [enc[r, 0].data_ptr() for r in nodes], L, 0, size % (2 * k), 1, out, 0)
        torch.cuda.synchronize()
        assert torch.equal(out[:size], t[:size]), erased
        assert int(out[size:].sum().item()) == 0


@pytest.mark.parametrize("k,n", [(16, 20), (32, 40)])
def test_syndrome_restore_arbitrary_chunks_vs_oracle(ec, k, n):
    """Chunks that are NOT codewords: the result must still be V_S^{-1} applied
    to the survivors, exactly as the reference's chunk_restore computes it."""
    import torch
    from vds_amd import chunk
    rng = np.random.default_rng(22 + k)
    for trial in range(6 if k == 16 else 3):
        tiles = int(rng.integers(1, 4))
        size = tiles * 2048 * 2 * k + int(rng.integers(0, 2 * k * 7))
        L = chunk.replica_size(k, size)
        nodes = [int(x) for x in rng.choice(n, k, replace=False)]
        host = [rng.integers(0, 256, L, dtype=np.uint8) for _ in nodes]
        pad = size % (2 * k)
        for c in host:  # a valid trailer, as every replica of one object carries
            c[-2], c[-1] = pad >> 8, pad & 0xFF
        ref = O.restore(k, nodes, host)
        assert ref is not None
        dev = torch.from_numpy(np.stack(host)).cuda()
        out = torch.zeros(len(ref) + 64, dtype=torch.uint8, device="cuda")
        assert _path(k, nodes, L) == 3
        chunk.restore_device(k, nodes, [dev[j].data_ptr() for j in range(k)], L, 0, pad, 1, out, 0)
        torch.cuda.synchronize()
        assert np.array_equal(out[:len(ref)].cpu().numpy(), ref), (trial, nodes)


def test_restore_path_selection(ec):
    L = 2 * 2048 * 2 + 2
    assert _path(16, list(range(4, 20)), 2 * 2048 * 16 + 2) == 3
    assert _path(16, list(range(5, 21)), 2 * 2048 * 16 + 2) == 2   # point 20 is outside 0..19
    assert _path(16, list(range(4, 20)), 2 * 100 + 2) == 1         # no full tile
    assert _path(32, list(range(8, 40)), 2 * 2048 * 32 + 2) in (2, 3)
    assert _path(5, list(range(5)), L) == 1
    assert _path(32, list(range(32, 64)), 2 * 1024 + 2, 0, 2) == 2  # live shape: 64 KiB objects, stream mode
    assert _path(32, list(range(32, 64)), 2 * 1024 + 2, 0, 1) == 1  # ... needs two objects for one tile
    assert _path(32, [r for r in range(40) if r % 5], 2 * 1024 + 2, 0, 4) == 2  # (32, 40) survivors under one tile
    # a non-zero trailer padding leaves one stripe fewer whose cells all land
    # in the output (F = T - 1): the query follows restore_device
    assert _path(16, list(range(4, 20)), 2 * 2048 + 2, 0) == 3
    assert _path(16, list(range(4, 20)), 2 * 2048 + 2, 7) == 1
    assert _path(32, list(range(32, 64)), 2 * 1024 + 2, 5, 64) == 1
    assert _path(32, list(range(32, 64)), 2 * 1536 + 2, 0, 64) == 2
    assert _path(32, list(range(32, 64)), 2 * 1536 + 2, 3, 64) == 1


def test_restore_device_batched(ec):
    import torch
    from vds_amd import chunk
    k, n, size, count = 16, 20, 65536 * 3 + 17, 3
    t = torch.empty(size * count, dtype=torch.uint8, device="cuda")
    for o in range(count):
        chunk.fill_splitmix_device(t[o * size:], size, SEED + 900 + o)
    enc = dev_encode(torch, k, n, t, size, count=count)
    nodes = [r for r in range(n) if r not in (0, 5, 10, 15)]
    L = enc.shape[2]
    out = torch.zeros(size * count, dtype=torch.uint8, device="cuda")
    # chunk j of object o at enc[nodes[j], o]: stride between objects = L
    chunk.restore_device(k, nodes, [enc[r, 0].data_ptr() for r in nodes], L, enc.stride(1), size % (2 * k),
                         count, out, size)
    torch.cuda.synchronize()
    assert torch.equal(out, t)


def test_restore_error_paths(ec):
    from vds_amd import VdsEcError
    d = O.splitmix(SEED + 3, 100)
    chunks = [O.encode(4, r, d) for r in (1, 2, 3, 4)]
    with pytest.raises(VdsEcError):  # duplicate replica ids
        ec.ChunkRestore(4, [1, 2, 2, 4]).restore(chunks)
    bad = [c.copy() for c in chunks]
    for c in bad:  # trailer claims more bytes than the chunks can produce
        c[-2:] = [0xFF, 0xFF]
    assert O.restore(4, [1, 2, 3, 4], bad) is None
    with pytest.raises(VdsEcError):
        ec.ChunkRestore(4, [1, 2, 3, 4]).restore(bad)
    # a trailer that is wrong but within range decodes the trailer row like the reference
    odd = [c.copy() for c in chunks]
    for c in odd:
        c[-2:] = [0, 7]
    ref = O.restore(4, [1, 2, 3, 4], odd)
    assert ref is not None
    assert np.array_equal(ec.ChunkRestore(4, [1, 2, 3, 4]).restore(odd), ref)
    # trailer in (2k, 4k]: the reference returns MORE than (size-2)*k bytes,
    # decoding the trailer row as data
    long = [c.copy() for c in chunks]
    for c in long:
        c[-2:] = [0, 11]
    ref = O.restore(4, [1, 2, 3, 4], long)
    assert ref is not None and ref.size == (chunks[0].size - 2) * 4 + 3
    assert np.array_equal(ec.ChunkRestore(4, [1, 2, 3, 4]).restore(long), ref)


# ----------------------------------------------------------- uint8_t / cells

def test_uint8_instantiation(ec):
    e = G["encode8"]
    d = O.splitmix(SEED + e["object_index"], e["size"])
    for r, h in e["replicas"].items():
        assert sha(ec.ChunkGenerator(e["k"], int(r), cell_bytes=1).write(d)) == h
    rng = np.random.default_rng(9)
    for trial in range(20):
        k = int(rng.integers(1, 30))
        size = int(rng.integers(0, 20000))
        d = rng.integers(0, 256, size, dtype=np.uint8)
        nodes = [int(x) for x in rng.choice(256, k, replace=False)]
        chunks = ec.chunk.encode_host(k, nodes, d, cell_bytes=1)
        for i, r in enumerate(nodes):
            assert np.array_equal(chunks[i], O.encode(k, r, d, cell_bytes=1))
        out = ec.ChunkRestore(k, nodes, cell_bytes=1).restore(chunks)
        assert np.array_equal(out, O.restore(k, nodes, chunks, cell_bytes=1))
        assert out.tobytes() == d.tobytes()


def test_cell_array_paths(ec):
    c = G["chunk_cells16"]
    cells = O.splitmix(SEED + c["object_index"], 2 * c["cells"]).view(np.uint16)
    ids = [5, 9, 200]
    got = {}
    for r in ids:
        got[r] = ec.chunk_cells(ec.ChunkGenerator(3, r), cells)
        assert got[r].tolist() == c["chunks"][str(r)]
    rest = ec.ChunkRestore(3, ids).restore_cells([got[r] for r in ids])
    assert rest.tolist() == c["restore"]


# ------------------------------------------- reference tests, re-hosted on GPU

def test_chunk_tests_test_chunks_uint8(ec):
    """chunk_tests.cpp:10-59 (seeded instead of time-seeded)."""
    rng = np.random.default_rng(10)
    for _ in range(10):
        size = int(rng.integers(1, 1001))
        size -= size % 3
        data = rng.integers(0, 256, size, dtype=np.uint8)
        ids = [int(x) for x in rng.choice(256, 3, replace=False)]
        chunks = [ec.chunk_cells(ec.ChunkGenerator(3, r, cell_bytes=1), data) for r in ids]
        res = ec.ChunkRestore(3, ids, cell_bytes=1).restore_cells(chunks)
        assert res.size == size and np.array_equal(res, data)


def test_chunk_tests_test_chunks16(ec):
    """chunk_tests.cpp:61-110."""
    rng = np.random.default_rng(11)
    for _ in range(10):
        size = int(rng.integers(1, 1001))
        size -= size % 3
        data = rng.integers(0, 65536, size).astype(np.uint16)
        ids = [int(x) for x in rng.choice(256, 3, replace=False)]
        chunks = [ec.chunk_cells(ec.ChunkGenerator(3, r), data) for r in ids]
        res = ec.ChunkRestore(3, ids).restore_cells(chunks)
        assert res.size == size and np.array_equal(res, data)


def test_chunk_tests_test_chunks_storage(ec):
    """chunk_tests.cpp:112-162: 800 distinct replicas < 1000, 2000-6000 bytes."""
    rng = np.random.default_rng(12)
    size = int(rng.integers(2000, 6001))
    data = rng.integers(0, 256, size, dtype=np.uint8)
    storage = ec.ChunkStorage(800)
    ids = [int(x) for x in rng.choice(1000, 800, replace=False)]
    horcruxes = {r: storage.generate_replica(r, data) for r in ids[:40]}
    batch = storage.generate_replicas(ids[40:], data)
    horcruxes.update({r: b for r, b in zip(ids[40:], batch)})
    for r in ids[:3]:
        assert np.array_equal(horcruxes[r], O.encode(800, r, data))
    result = storage.restore_data(horcruxes)
    assert result.size == size and result.tobytes() == data.tobytes()
    from vds_amd import VdsEcError
    with pytest.raises(VdsEcError):
        storage.restore_data(dict(list(horcruxes.items())[:799]))  # "Error at restoring data"


# ------------------------------------------------ full BASELINE-size properties

@pytest.mark.parametrize("k,n", [(16, 20), (32, 40)])
def test_full_size_roundtrip_64MiB(ec, k, n):
    import torch
    from vds_amd import chunk
    size = 64 << 20
    t = dev_object(torch, size, 0)
    enc = dev_encode(torch, k, n, t, size)
    L = enc.shape[2]
    m = n - k
    for erased in (list(range(m)), list(range(0, n, n // m))[:m], list(range(n - m, n))):
        nodes = [r for r in range(n) if r not in erased]
        out = torch.empty(size, dtype=torch.uint8, device="cuda")
        chunk.restore_device(k, nodes, [enc[r, 0].data_ptr() for r in nodes], L, 0, size % (2 * k), 1, out, 0)
        torch.cuda.synchronize()
        assert torch.equal(out, t), erased
    # linearity: enc(a ^ b) == enc(a) ^ enc(b) on the data cells
    t2 = dev_object(torch, size, 1)
    enc2 = dev_encode(torch, k, n, t2, size)
    enc3 = dev_encode(torch, k, n, t ^ t2, size)
    assert torch.equal(enc3[:, :, : L - 2], enc[:, :, : L - 2] ^ enc2[:, :, : L - 2])


def test_host_batch_multi_device(ec):
    rng = np.random.default_rng(13)
    objs = [rng.integers(0, 256, int(s), dtype=np.uint8) for s in (0, 17, 65536 * 2 + 5, 300000, 4096)]
    outs = ec.encode_host_batch(16, list(range(20)), objs)
    for o, d in zip(outs, objs):
        for r in (0, 3, 19):
            assert np.array_equal(o[r], O.encode(16, r, d))


@pytest.mark.parametrize("k,n", [(16, 20), (32, 40), (4, 6)])
def test_restore_host_batch(ec, k, n):
    """vds_ec_restore16_host_batch: per-object survivor sets and sizes, bit-exact
    against the oracle's restore (chunk.h:402-444) of the same chunks."""
    from vds_amd._lib import VdsEcError
    rng = np.random.default_rng(31 + k)
    sizes = [1, 2 * k * 2048 * 2 + 7, 65536 * 3 + 1, 2 * k, 300001]
    objs = [rng.integers(0, 256, s, dtype=np.uint8) for s in sizes]
    nodes, chunks = [], []
    for d in objs:
        ids = [int(x) for x in rng.choice(n, k, replace=False)]
        nodes.append(ids)
        chunks.append([O.encode(k, r, d) for r in ids])
    got = ec.restore_host_batch(k, nodes, chunks)
    for d, g, ids, ch in zip(objs, got, nodes, chunks):
        assert np.array_equal(g, d), (k, d.size, ids)
        assert np.array_equal(g, O.restore(k, ids, ch))
    # one id list for every object
    ids = list(range(n - k, n))
    same = ec.restore_host_batch(k, ids, [[O.encode(k, r, d) for r in ids] for d in objs[:3]])
    assert all(np.array_equal(g, d) for g, d in zip(same, objs[:3]))
    with pytest.raises(VdsEcError):  # chunks of one object differ in size (chunk_storage.cpp:73-76)
        ec.restore_host_batch(k, [nodes[0]], [[c[:-1] if j == 0 else c for j, c in enumerate(chunks[1])]])
    bad = [c.copy() for c in chunks[1]]
    for c in bad:  # a trailer claiming more bytes than the chunks hold: the reference's fatal error
        c[-2], c[-1] = 0xFF, 0xFF
    with pytest.raises(VdsEcError):
        ec.restore_host_batch(k, [nodes[1]], [bad])


def test_large_k_parameters_are_stream_ordered(ec):
    """k > 32 (the inverse does not fit the kernel arguments) and k > 64 (nor
    does the chunk table): restore_device and regenerate_device stage them
    through the stream-ordered parameter ring.  Several calls with different
    survivor sets are enqueued back to back on one stream with no host sync in
    between; each must see its own parameters (oracle-checked)."""
    import torch
    from vds_amd import chunk
    rng = np.random.default_rng(77)
    stream = torch.cuda.Stream()
    for k, n, size in ((40, 48, 40 * 2 * 37 + 11), (80, 90, 80 * 2 * 9 + 3)):
        host = O.splitmix(SEED + k, size)
        t = torch.from_numpy(host.copy()).cuda()
        reps = dev_encode(torch, k, n, t, size, replicas=list(range(n)))
        L = reps.shape[2]
        trials = [sorted(rng.choice(n, k, replace=False).tolist()) for _ in range(6)]
        outs = [torch.zeros(size + 2 * k, dtype=torch.uint8, device="cuda") for _ in trials]
        regen_targets = [[r for r in range(n) if r not in nodes][:8] for nodes in trials]
        regen_outs = [torch.zeros((8, L), dtype=torch.uint8, device="cuda") for _ in trials]
        torch.cuda.synchronize()
        with torch.cuda.stream(stream):
            for nodes, out, tg, ro in zip(trials, outs, regen_targets, regen_outs):
                chunk.restore_device(k, nodes, [reps[r, 0].data_ptr() for r in nodes], L, 0, size % (2 * k), 1,
                                     out, 0, stream=stream)
                chunk.regenerate_device(k, nodes, [reps[r, 0].data_ptr() for r in nodes], L, 0, 1, tg,
                                        [ro[i].data_ptr() for i in range(len(tg))], L, stream=stream)
        stream.synchronize()
        for nodes, out, tg, ro in zip(trials, outs, regen_targets, regen_outs):
            assert np.array_equal(out[:size].cpu().numpy(), host), (k, nodes)
            for i, r in enumerate(tg):
                assert np.array_equal(ro[i].cpu().numpy(), O.encode(k, r, host)), (k, nodes, r)


@pytest.mark.parametrize("k,n", [(16, 20), (32, 64)])
def test_host_batches_pack_groups(ec, k, n):
    """The host batches pack runs of equal-size objects into groups of up to
    64 MiB (several groups per run, the three-slot ring reused, size changes
    between runs, empty objects); every replica equals the one-object host
    encode (itself oracle-checked above; two objects re-checked here against
    the oracle), and the batched restore from a survivor set per object gives
    every object back."""
    from vds_amd import chunk
    rng = np.random.default_rng(90 + k)
    sizes = [65536] * 400 + [3 << 20] * 3 + [0, 17] + [65536] * 7 + [2 * k * 2048 + 5] * 2
    objs = [rng.integers(0, 256, s, dtype=np.uint8) for s in sizes]
    ids = list(range(n))
    reps = ec.encode_host_batch(k, ids, objs)
    for i, d in enumerate(objs):
        if i % 37 == 0 or i >= 400:
            want = chunk.encode_host(k, ids, d)
            assert all(np.array_equal(a, b) for a, b in zip(reps[i], want)), (i, d.size)
    for i in (5, 401):
        assert np.array_equal(reps[i][n - 1], O.encode(k, n - 1, objs[i]))
    nodes = []
    for _ in objs:  # restore_async: the first k replicas found per object
        gone = set(rng.choice(n, n - k, replace=False).tolist()) if rng.random() < 0.7 else set()
        nodes.append([r for r in range(n) if r not in gone][:k])
    got = ec.restore_host_batch(k, nodes, [[reps[o][r] for r in nd] for o, nd in enumerate(nodes)])
    for g, d in zip(got, objs):
        assert np.array_equal(g, d), d.size


@pytest.mark.parametrize("jit", [0, 2], ids=["aot", "jit"])
def test_c4_full_size_golden(ec, jit):
    """BASELINE configs[3] at full size (k = 32, n = 40, one 64 MiB object):
    every replica of the device encode against the oracle's SHA-256s, and the
    device repair from the C4 survivors {r : r mod 5 != 0} -- the syndrome
    kernel k_restore_syn<32,40> (jit 0) and the survivor set's run-time
    compiled kernel (jit 2, compiled synchronously) -- against the oracle's
    restore (chunk.h:245-281, 402-444; tests/golden/make_golden.py)."""
    import torch
    from vds_amd import chunk
    enc = next(e for e in G["encode16_sha"] if (e["k"], e["n"], e["size"]) == (32, 40, 64 << 20))
    rest = next(e for e in G["restore16"] if (e["k"], e["size"]) == (32, 64 << 20))
    k, n, size = 32, 40, 64 << 20
    assert rest["nodes"] == [r for r in range(n) if r % 5][:k]
    t = dev_object(torch, size, enc["object_index"])
    out = dev_encode(torch, k, n, t, size)
    for r in range(n):
        assert sha(out[r, 0].cpu().numpy()) == enc["sha256"][str(r)], f"replica {r}"
    L = out.shape[2]
    chunk.jit_set_mode(jit)
    try:
        res = torch.full((size,), 0xA5, dtype=torch.uint8, device="cuda")
        chunk.restore_device(k, rest["nodes"], [out[r, 0].data_ptr() for r in rest["nodes"]], L, L, 0, 1, res, size)
        torch.cuda.synchronize()
        assert _path(k, rest["nodes"], L) == (4 if jit else 3)  # (sync mode: compiled at that first use)
        assert sha(res.cpu().numpy()) == rest["sha256"]
    finally:
        chunk.jit_set_mode(0)


_ORACLE_CACHE = {}


@pytest.mark.parametrize("jit", [0, 2], ids=["aot", "jit"])
def test_headline_full_size_non_codeword_vs_oracle(ec, jit):
    """The headline configuration (k = 16, n = 20, erased {0, 5, 10, 15}) at
    full size with survivors that are not one codeword (random bytes): the
    syndrome kernel k_restore_syn<16,20> (jit 0) and the survivor set's
    run-time kernel (jit 2: its fill reads the stage-1 registers) against the
    oracle's restore (chunk.h:402-444).  1024 tiles, so every workgroup walks
    several of them."""
    import torch
    from vds_amd import chunk
    k, n, size = 16, 20, 64 << 20
    L = chunk.replica_size(k, size)
    nodes = [r for r in range(n) if r % 5]
    if "headline" not in _ORACLE_CACHE:  # (one oracle restore, ~4 s, for both kernels)
        rng = np.random.default_rng(SEED + 1616)
        host = [rng.integers(0, 256, L, dtype=np.uint8) for _ in nodes]
        for c in host:
            c[-2], c[-1] = 0, 0  # (size % 2k == 0)
        _ORACLE_CACHE["headline"] = (host, O.restore(k, nodes, host))
    host, ref = _ORACLE_CACHE["headline"]
    dev = torch.from_numpy(np.stack(host)).cuda()
    chunk.jit_set_mode(jit)
    try:
        out = torch.zeros(len(ref) + 64, dtype=torch.uint8, device="cuda")
        chunk.restore_device(k, nodes, [dev[j].data_ptr() for j in range(k)], L, 0, 0, 1, out, 0)
        torch.cuda.synchronize()
        assert _path(k, nodes, L) == (4 if jit else 3)
        assert np.array_equal(out[:len(ref)].cpu().numpy(), ref)
        assert int(out[len(ref):].sum().item()) == 0
    finally:
        chunk.jit_set_mode(0)
