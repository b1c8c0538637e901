"""C5: host-resident objects, PCIe-inclusive rates.

Encode: vds_ec_encode16_host_batch (pinned ring, H2D -> encode -> D2H of all n
replicas, objects round-robin over the visible GPUs).  Repair:
vds_ec_restore16_host_batch (the same ring: H2D of k replicas -> restore ->
D2H), and beside it vds_ec_restore16_host per object (ChunkStorage.restore_data).
Prints one JSON line.  This rate is never bench.py's `value`.

  python tools/bench_host.py [--objects 16] [--object-mib 64] [--k 16] [--m 4] [--live 16384]

--live N adds the production shape: N host objects of 64 KiB at k = 32, n = 64
(dht_network.h:22-25, web/src/store/vds_api.jsx:76), encoded with one
vds_ec_encode16_host_batch call and restored with one
vds_ec_restore16_host_batch call from the first 32 replicas found per object
(replica loss p = 0.02, restore_async, dht_network_client.cpp:851-901).
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402

from vds_amd import chunk  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--objects", type=int, default=16)
p.add_argument("--object-mib", type=int, default=64)
p.add_argument("--k", type=int, default=16)
p.add_argument("--m", type=int, default=4)
p.add_argument("--reps", type=int, default=2)
p.add_argument("--live", type=int, default=0)
p.add_argument("--split-mib", type=int, default=0, help="one object of this size over every GPU by stripe ranges")
a = p.parse_args()
k, n, size = a.k, a.k + a.m, a.object_mib << 20
rng = np.random.default_rng(1)
objs = [rng.integers(0, 256, size, dtype=np.uint8) for _ in range(a.objects)]
ids = list(range(n))
L = chunk.replica_size(k, size)
# caller-owned, pre-faulted replica buffers (a storage node writes into its own)
outs = [[np.ones(L, dtype=np.uint8) for _ in ids] for _ in objs]
chunk.encode_host_batch(k, ids, objs[:1], outs=outs[:1])  # warm-up: contexts, pinned rings
best_enc = None
for _ in range(a.reps):
    t0 = time.perf_counter()
    reps = chunk.encode_host_batch(k, ids, objs, outs=outs)
    dt = time.perf_counter() - t0
    best_enc = dt if best_enc is None else min(best_enc, dt)
erased = list(range(0, n, max(1, n // a.m)))[: a.m]
nodes = [r for r in range(n) if r not in erased][:k]
store = chunk.ChunkStorage(k)
best_rep = None
for _ in range(a.reps):
    t0 = time.perf_counter()
    for o in range(a.objects):
        out = store.restore_data({r: reps[o][r] for r in nodes})
    dt = time.perf_counter() - t0
    best_rep = dt if best_rep is None else min(best_rep, dt)
assert out.tobytes() == objs[-1].tobytes()
routs = [np.ones(size, dtype=np.uint8) for _ in objs]  # caller-owned, pre-faulted
chunk.restore_host_batch(k, nodes, [[reps[0][r] for r in nodes]], outs=routs[:1])  # warm-up
best_rb = None
for _ in range(a.reps):
    t0 = time.perf_counter()
    got = chunk.restore_host_batch(k, nodes, [[reps[o][r] for r in nodes] for o in range(a.objects)], outs=routs)
    dt = time.perf_counter() - t0
    best_rb = dt if best_rb is None else min(best_rb, dt)
assert all(g.tobytes() == d.tobytes() for g, d in zip(got, objs))
gib = a.objects * size / 2**30


def live(count, reps, pinned=False):
    """The live shape through the C ABI with flat numpy buffers (one pointer
    per object / replica, no per-object Python arrays).  pinned: the caller's
    slabs come from vds_ec_host_alloc (objects, replicas, a survivor slab
    [count][k][L] the download loop would receive into, restored objects), so
    no staging copies are made."""
    import ctypes as C
    from vds_amd import _lib
    lib = _lib.lib()
    k, n, size = 32, 64, 65536
    L = chunk.replica_size(k, size)
    keep = []

    def buf(nbytes, fill):
        if not pinned:
            return np.full(nbytes, fill, dtype=np.uint8)  # caller-owned, pre-faulted
        b = chunk.PinnedBuffer(nbytes)
        keep.append(b)
        b.array[:] = fill
        return b.array
    objs = buf(count * size, 0)
    objs[:] = rng.integers(0, 256, count * size, dtype=np.uint8)
    reps_buf = buf(count * n * L, 1)
    out = buf(count * size, 1)
    obj_ptrs = (np.uint64(objs.ctypes.data) + np.arange(count, dtype=np.uint64) * np.uint64(size))
    rep_ptrs = (np.uint64(reps_buf.ctypes.data) + np.arange(count * n, dtype=np.uint64) * np.uint64(L))
    sizes = np.full(count, size, dtype=np.uint64)
    ids = np.arange(n, dtype=np.uint16)

    def enc():
        _lib.check(lib.vds_ec_encode16_host_batch(k, ids.ctypes.data_as(_lib.u16p), n,
                                                  obj_ptrs.ctypes.data_as(_lib.vpp), sizes.ctypes.data_as(_lib.u64p),
                                                  count, rep_ptrs.ctypes.data_as(_lib.vpp), 0, 0))
    lost = np.random.default_rng(2).random((count, n)) < 0.02
    nodes = np.stack([np.flatnonzero(~lost[o])[:k] for o in range(count)]).astype(np.uint16)
    chunk_ptrs = (np.uint64(reps_buf.ctypes.data) +
                  (np.arange(count, dtype=np.uint64)[:, None] * np.uint64(n) + nodes.astype(np.uint64)) * np.uint64(L))
    chunk_ptrs = np.ascontiguousarray(chunk_ptrs)
    if pinned:  # the survivors as the download loop would lay them out: one slab [count][k][L]
        surv = buf(count * k * L, 0)
        enc()
        rv = reps_buf.reshape(count, n, L)
        surv.reshape(count, k, L)[:] = rv[np.arange(count)[:, None], nodes.astype(np.int64)]
        chunk_ptrs = np.ascontiguousarray(np.uint64(surv.ctypes.data) + np.arange(count * k, dtype=np.uint64).reshape(
            count, k) * np.uint64(L))
    csz = np.full(count, L, dtype=np.uint64)
    out_ptrs = (np.uint64(out.ctypes.data) + np.arange(count, dtype=np.uint64) * np.uint64(size))
    caps = np.full(count, size, dtype=np.uint64)

    def rest():
        caps[:] = size
        _lib.check(lib.vds_ec_restore16_host_batch(k, nodes.ctypes.data_as(_lib.u16p), chunk_ptrs.ctypes.data_as(_lib.vpp),
                                                   csz.ctypes.data_as(_lib.u64p), count,
                                                   out_ptrs.ctypes.data_as(_lib.vpp), caps.ctypes.data_as(_lib.u64p),
                                                   0, 0))

    def best(fn):
        fn()
        b = None
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            dt = time.perf_counter() - t0
            b = dt if b is None else min(b, dt)
        return b
    te = best(enc)
    tr = best(rest)
    assert np.array_equal(out, objs), "live host restore differs"
    g = count * size / 2**30
    del keep
    return {"shape": f"k=32, n=64, {count} x 64 KiB host objects, loss p=0.02" + (", caller-pinned slabs" if pinned else ""),
            "encode_GiBps": round(g / te, 3),
            "repair_GiBps": round(g / tr, 3), "encode_s": round(te, 4), "repair_s": round(tr, 4),
            "pcie_bytes_per_object_encode": size + n * L, "pcie_bytes_per_object_repair": k * L + size}


def split(mib, reps):
    size = mib << 20
    obj = rng.integers(0, 256, size, dtype=np.uint8)
    chunk.encode_host_split(k, ids, obj[: 1 << 20])  # warm-up
    b = None
    for _ in range(reps):
        t0 = time.perf_counter()
        out = chunk.encode_host_split(k, ids, obj)
        dt = time.perf_counter() - t0
        b = dt if b is None else min(b, dt)
    import torch
    return {"object_bytes": size, "devices": torch.cuda.device_count(), "encode_GiBps": round(size / b / 2**30, 3),
            "check": bool(np.array_equal(out[0][:1024], chunk.encode_host(k, [0], obj[:2 * k * 512])[0][:1024]))}


print(json.dumps({"metric": "host-resident (PCIe-inclusive) encode / repair GiB/s", "objects": a.objects,
                  "object_bytes": size, "k": k, "n": n, "erased": erased,
                  "encode_GiBps": round(gib / best_enc, 3), "repair_GiBps": round(gib / best_rb, 3),
                  "repair_per_object_GiBps": round(gib / best_rep, 3),
                  "encode_s": round(best_enc, 4), "repair_s": round(best_rb, 4),
                  "live": live(a.live, a.reps) if a.live else None,
                  "live_pinned": live(a.live, a.reps, pinned=True) if a.live else None,
                  "split": split(a.split_mib, a.reps) if a.split_mib else None}), flush=True)
