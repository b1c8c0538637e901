"""Caller-pinned host slabs (vds_ec_host_alloc / vds_ec_host_register): the
host batches read the caller's pinned objects / survivors by DMA and write
replicas / restored objects straight into the caller's pinned pages (no
staging copies).  Bytes against the oracle (chunk.h:245-281, :402-444) and
against the staged path on the same inputs."""
import numpy as np
import pytest

import oracle_ctypes as O

SEED = 0x7664730000000000
pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("k,n,size,count", [(16, 20, 1 << 20, 5), (32, 64, 65536, 40), (4, 6, 1000, 9)])
def test_pinned_slab_encode_and_restore(gpu, k, n, size, count):
    from vds_amd import chunk
    L = chunk.replica_size(k, size)
    src = chunk.PinnedBuffer(count * size)
    reps = chunk.PinnedBuffer(count * n * L)
    objs = [O.splitmix(SEED + 1000 * k + o, size) for o in range(count)]
    for o in range(count):
        src.array[o * size:(o + 1) * size] = objs[o]
    reps.array[:] = 0x5A
    views = [src.array[o * size:(o + 1) * size] for o in range(count)]
    outs = [[reps.array[(o * n + i) * L:(o * n + i + 1) * L] for i in range(n)] for o in range(count)]
    chunk.encode_host_batch(k, range(n), views, outs=outs)
    for o in (0, count - 1):
        for i in (0, n - 1):
            assert np.array_equal(outs[o][i], O.encode(k, i, objs[o])), (o, i)
    staged = chunk.encode_host_batch(k, range(n), objs)  # the staged path: same bytes
    assert all(np.array_equal(outs[o][i], staged[o][i]) for o in range(count) for i in range(n))
    # restore from a pinned survivor slab [count][k][L] into a pinned output slab
    nodes = [r for r in range(n) if r % 5 != 1][:k]
    surv = chunk.PinnedBuffer(count * k * L)
    for o in range(count):
        for j, r in enumerate(nodes):
            surv.array[(o * k + j) * L:(o * k + j + 1) * L] = outs[o][r]
    dst = chunk.PinnedBuffer(count * size)
    dst.array[:] = 0xA5
    got = chunk.restore_host_batch(k, nodes, [[surv.array[(o * k + j) * L:(o * k + j + 1) * L] for j in range(k)]
                                              for o in range(count)],
                                   outs=[dst.array[o * size:(o + 1) * size] for o in range(count)])
    assert all(np.array_equal(g, d) for g, d in zip(got, objs))
    for b in (src, reps, surv, dst):
        b.close()


def test_registered_buffer_and_errors(gpu):
    from vds_amd import chunk
    from vds_amd._lib import VdsEcError
    k, n, size, count = 16, 20, 131072, 3
    L = chunk.replica_size(k, size)
    objs = np.concatenate([O.splitmix(SEED + 5 + o, size) for o in range(count)])
    reps = np.zeros(count * n * L, dtype=np.uint8)
    chunk.host_register(objs)
    chunk.host_register(reps)
    try:
        outs = [[reps[(o * n + i) * L:(o * n + i + 1) * L] for i in range(n)] for o in range(count)]
        chunk.encode_host_batch(k, range(n), [objs[o * size:(o + 1) * size] for o in range(count)], outs=outs)
        assert np.array_equal(outs[2][19], O.encode(k, 19, objs[2 * size:]))
        with pytest.raises(VdsEcError):  # registered memory is not the allocator's to free
            chunk._lib.check(chunk._lib.lib().vds_ec_host_free(objs.ctypes.data), "free")
    finally:
        chunk.host_unregister(objs)
        chunk.host_unregister(reps)
    with pytest.raises(VdsEcError):
        chunk.host_unregister(objs)  # no longer registered


def test_registered_slabs_on_every_device(gpu):
    """A registered range's device address is resolved per device (ADVICE r4:
    the host batches send group g to device g mod ndev, and a mapped host
    range need not have one address on all of them).  Many small groups over
    every visible device (max_devices = 8), registered input and output slabs,
    against the oracle; on a one-GPU box this still runs the lookup path."""
    from vds_amd import chunk
    k, n, size, count = 32, 64, 65536, 4096  # 4096 x 64 KiB: several 64 MiB groups
    L = chunk.replica_size(k, size)
    objs = np.concatenate([O.splitmix(SEED + 77 + o, size) for o in range(16)] * (count // 16))
    reps = np.zeros(count * n * L, dtype=np.uint8)
    chunk.host_register(objs)
    chunk.host_register(reps)
    try:
        outs = [[reps[(o * n + i) * L:(o * n + i + 1) * L] for i in range(n)] for o in range(count)]
        chunk.encode_host_batch(k, range(n), [objs[o * size:(o + 1) * size] for o in range(count)], outs=outs,
                                max_devices=8)
        for o in (0, 1, count // 2 + 3, count - 1):
            for i in (0, 33, n - 1):
                assert np.array_equal(outs[o][i], O.encode(k, i, objs[o * size:(o + 1) * size])), (o, i)
    finally:
        chunk.host_unregister(objs)
        chunk.host_unregister(reps)
