"""GPU parity of the fused regenerate path.

The reference repairs a replica by restoring the object and re-encoding it
(sync_process.cpp:313-335 -> restore_async, then save_data at
dht_network_client.cpp:582-658).  The checker here is exactly that route on
the oracle: oracle restore from the survivors, then oracle encode of each
target replica.  Bit-exact, no tolerance.
"""
import numpy as np
import pytest

import oracle_ctypes as O

pytestmark = pytest.mark.gpu

SEED = 0x7664730000000000


@pytest.fixture(scope="module")
def chunk(gpu):
    from vds_amd import chunk as c
    return c


def reference_route(k, nodes, chunks, targets):
    """restore (chunk.h:402-444) then chunk_generator(k, t).write (chunk.h:245-281)."""
    obj = O.restore(k, nodes, chunks)
    return [O.encode(k, t, obj) for t in targets]


def replicas_of(k, n, data):
    return [O.encode(k, r, data) for r in range(n)]


@pytest.mark.parametrize("size", [3 * 65536 + 77, 2 * 65536, 65536 - 6, 1000, 1])
def test_regenerate_host_k16_erased_targets(chunk, size):
    k, n = 16, 20
    data = O.splitmix(SEED + size, size)
    reps = replicas_of(k, n, data)
    erased = [0, 5, 10, 15]
    nodes = [r for r in range(n) if r not in erased]
    for targets in (erased, [5], [15, 0], [19 if 19 in erased else 10]):
        got = chunk.regenerate_host(k, nodes, [reps[r] for r in nodes], targets)
        want = reference_route(k, nodes, [reps[r] for r in nodes], targets)
        for t, g, w in zip(targets, got, want):
            assert np.array_equal(g, w), f"replica {t} differs (size {size})"
            assert np.array_equal(g, reps[t])


def test_regenerate_fast_path_selected(chunk):
    from vds_amd import _lib
    k = 16
    nodes = np.array([r for r in range(20) if r not in (0, 5, 10, 15)], dtype=np.uint16)
    L = chunk.replica_size(k, 64 << 20)
    p = _lib.lib().vds_ec_regenerate16_path
    t_in = np.array([5, 0], dtype=np.uint16)
    t_out = np.array([5, 21], dtype=np.uint16)
    assert p(k, nodes.ctypes.data_as(_lib.u16p), t_in.ctypes.data_as(_lib.u16p), 2, L) == 3
    assert p(k, nodes.ctypes.data_as(_lib.u16p), t_out.ctypes.data_as(_lib.u16p), 2, L) == 2  # runtime-coefficient kernel
    assert p(k, nodes.ctypes.data_as(_lib.u16p), t_in.ctypes.data_as(_lib.u16p), 2, 1000) == 1


@pytest.mark.parametrize("k,n,erased,targets,size", [
    (16, 20, [16, 17, 18, 19], [16, 19], 2 * 65536 + 33),   # parity-only erasures, fast path
    (16, 20, [1, 2, 3, 4], [1, 2, 3, 4, 30], 65536 * 2),    # a target beyond n: generic path
    (4, 6, [0, 1], [0, 1], 1 << 20),                         # BASELINE config 1 shape
    (32, 40, [0, 7, 8, 9, 20, 21, 38, 39], [0, 38], 3 * 131072 + 5),
    (3, 5, [4, 1], [1, 4, 0], 17),
])
def test_regenerate_host_shapes(chunk, k, n, erased, targets, size):
    data = O.splitmix(SEED + 7 * size + k, size)
    reps = replicas_of(k, n, data)
    nodes = [r for r in range(n) if r not in erased][:k]
    got = chunk.regenerate_host(k, nodes, [reps[r] for r in nodes], targets)
    want = reference_route(k, nodes, [reps[r] for r in nodes], targets)
    for t, g, w in zip(targets, got, want):
        assert np.array_equal(g, w), f"replica {t} differs (k={k} size={size})"


def test_regenerate_device_batched_strided(chunk):
    import torch
    k, n, size, count = 16, 20, 2 * 65536 + 100, 3
    L = chunk.replica_size(k, size)
    objs = [O.splitmix(SEED + 100 + o, size) for o in range(count)]
    reps = np.zeros((n, count, L + 6), dtype=np.uint8)  # padded stride
    for o, d in enumerate(objs):
        for r in range(n):
            reps[r, o, :L] = O.encode(k, r, d)
    dev = torch.from_numpy(reps).cuda()
    erased = [2, 9, 12, 17]
    nodes = [r for r in range(n) if r not in erased]
    out = torch.zeros((len(erased), count, L + 10), dtype=torch.uint8, device="cuda")
    chunk.regenerate_device(k, nodes, [dev[r].data_ptr() for r in nodes], L, L + 6, count, erased,
                            [out[i].data_ptr() for i in range(len(erased))], L + 10)
    torch.cuda.synchronize()
    host = out.cpu().numpy()
    for i, t in enumerate(erased):
        for o in range(count):
            assert np.array_equal(host[i, o, :L], reps[t, o, :L]), f"replica {t} object {o}"
            assert not host[i, o, L:].any(), "wrote past the replica"


@pytest.mark.parametrize("k,n,size,count,erased,targets,path", [
    # the live shape (dht_network.h:22-25): 64 KiB objects, tiles straddle objects, last object generic
    (32, 64, 65536, 5, list(range(1, 64, 2)), [1, 3, 63, 33, 0], 2),
    (32, 64, 2 * 65536 + 3000, 3, list(range(32, 64)), list(range(32, 64)), 2),  # whole tiles + generic rest
    (16, 20, 3 * 65536 + 77, 2, [1, 2, 3, 4], [1, 2, 3, 4, 30], 2),           # a target beyond n
    (16, 20, 4 * 65536, 3, [16, 17, 18, 19], [0, 19, 16], 2),                 # a surviving point as target
    (16, 20, 4 * 65536, 3, [0, 5, 10, 15], [15, 0], 3),                       # syndrome kernel
])
def test_regenerate_device_fast_paths(chunk, k, n, size, count, erased, targets, path):
    """Every fast regenerate path against the reference route (restore, then
    encode of the target) on batches of objects: bit-exact, trailers included,
    nothing written past a replica."""
    import torch
    from vds_amd import _lib
    L = chunk.replica_size(k, size)
    objs = [O.splitmix(SEED + 300 + 7 * o + k, size) for o in range(count)]
    nodes = [r for r in range(n) if r not in erased][:k]
    stride = L + 4
    reps = np.zeros((k, count, stride), dtype=np.uint8)
    want = np.zeros((len(targets), count, L), dtype=np.uint8)
    for o, d in enumerate(objs):
        for j, r in enumerate(nodes):
            reps[j, o, :L] = O.encode(k, r, d)
        for i, t in enumerate(targets):
            want[i, o] = O.encode(k, t, d)
    nd = np.array(nodes, dtype=np.uint16)
    tg = np.array(targets, dtype=np.uint16)
    assert _lib.lib().vds_ec_regenerate16_path(k, nd.ctypes.data_as(_lib.u16p), tg.ctypes.data_as(_lib.u16p),
                                               len(targets), L) == path
    dev = torch.from_numpy(reps).cuda()
    out = torch.zeros((len(targets), count, L + 8), dtype=torch.uint8, device="cuda")
    chunk.regenerate_device(k, nodes, [dev[j].data_ptr() for j in range(k)], L, stride, count, targets,
                            [out[i].data_ptr() for i in range(len(targets))], L + 8)
    torch.cuda.synchronize()
    host = out.cpu().numpy()
    for i, t in enumerate(targets):
        for o in range(count):
            assert np.array_equal(host[i, o, :L], want[i, o]), f"replica {t} object {o}"
            assert not host[i, o, L:].any(), "wrote past the replica"


def test_regenerate_storage_facade_and_errors(chunk):
    from vds_amd._lib import VdsEcError
    k, n, size = 16, 20, 70000
    data = O.splitmix(SEED + 5, size)
    reps = replicas_of(k, n, data)
    st = chunk.ChunkStorage(k)
    have = {r: reps[r] for r in range(4, 20)}
    got = st.regenerate_replicas(have, [0, 3])
    assert np.array_equal(got[0], reps[0]) and np.array_equal(got[1], reps[3])
    with pytest.raises(VdsEcError):  # not exactly min_horcrux horcruxes (chunk_storage.cpp:65-67)
        st.regenerate_replicas({r: reps[r] for r in range(5, 20)}, [0])
    with pytest.raises(VdsEcError):  # duplicate survivor ids: singular
        chunk.regenerate_host(k, [4] * 16, [reps[4]] * 16, [0])
    with pytest.raises(VdsEcError):  # a replica shorter than its trailer
        chunk.regenerate_host(k, list(range(4, 20)), [np.zeros(1, np.uint8)] * 16, [0])
