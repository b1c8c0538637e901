"""Batched restore / regenerate with a survivor set, size and output per
object (vds_ec_restore16_batch_device / vds_ec_regenerate16_batch_device):
the download and repair loops' shape (restore_async takes the first k
replicas found per object, dht_network_client.cpp:851-901; sync_process
repairs object by object, sync_process.cpp:313-335).  Every object is checked
against the oracle (chunk.h:402-444 / chunk.h:245-281)."""
import numpy as np
import pytest

import oracle_ctypes as O

SEED = 0x7664730000000000
pytestmark = pytest.mark.gpu


def _objects(torch, k, n, sizes, seed):
    """Encode objects of the given sizes (all n replicas, oracle-checked
    encode path) into separate device buffers: [(host bytes, [n tensors])]."""
    from vds_amd import chunk
    out = []
    for i, size in enumerate(sizes):
        host = O.splitmix(SEED + seed + i, size)
        t = torch.from_numpy(host.copy()).cuda() if size else torch.zeros(1, dtype=torch.uint8, device="cuda")
        L = chunk.replica_size(k, size)
        reps = [torch.zeros(L, dtype=torch.uint8, device="cuda") for _ in range(n)]
        chunk.encode_device(k, list(range(n)), t, size, size, 1, [r.data_ptr() for r in reps], L)
        out.append((host, reps))
    return out


def _first_k_found(rng, k, n_total, lost):
    """restore_async's choice: the first k replica ids not lost, in order."""
    gone = set(rng.choice(n_total, lost, replace=False).tolist()) if lost else set()
    return [r for r in range(n_total) if r not in gone][:k]


@pytest.mark.parametrize("k,n_total", [(16, 20), (16, 40), (32, 40), (32, 64), (16, 18), (32, 34)])
def test_restore_batch_per_object_survivors(gpu, k, n_total):
    import torch
    from vds_amd import chunk
    rng = np.random.default_rng(k * 100 + n_total)
    tile = 2048 * 2 * k
    sizes = [0, 1, 2 * k, 2 * k * 7 + 3, tile // 2 - 1, tile // 2, tile // 2 + 1, tile - 1, tile, tile + 5,
             2 * tile + 2 * k * 3 + 1, 65536, 58113, 3 * tile + 11] + [int(x) for x in rng.integers(1, 3 * tile, 9)]
    objs = _objects(torch, k, n_total, sizes, seed=k)
    nodes, chunks, csz, pads, outs = [], [], [], [], []
    for (host, reps), size in zip(objs, sizes):
        lost = int(rng.integers(0, n_total - k + 1))
        nd = _first_k_found(rng, k, n_total, lost)
        if rng.random() < 0.3:  # any order of the survivors
            nd = list(rng.permutation(nd))
        nodes.append(nd)
        chunks.append([reps[r].data_ptr() for r in nd])
        csz.append(reps[0].numel())
        pads.append(size % (2 * k))
        outs.append(torch.full((size + 4 * k,), 0xA5, dtype=torch.uint8, device="cuda"))
    chunk.restore_batch_device(k, nodes, chunks, csz, pads, [o.data_ptr() for o in outs])
    torch.cuda.synchronize()
    for (host, reps), size, out, nd in zip(objs, sizes, outs, nodes):
        got = out.cpu().numpy()
        ref = O.restore(k, nd, [reps[r].cpu().numpy() for r in nd])
        assert np.array_equal(got[:size], ref), (size, nd)
        assert np.array_equal(got[:size], host)
        assert (got[size:] == 0xA5).all(), size  # nothing written past the object


@pytest.mark.parametrize("k,n_total", [(16, 20), (16, 40), (32, 40), (32, 64), (16, 18), (32, 34)])
def test_regenerate_batch_per_object(gpu, k, n_total):
    import torch
    from vds_amd import chunk
    rng = np.random.default_rng(7 + k + n_total)
    tile = 2048 * 2 * k
    sizes = [1, 2 * k * 9 + 1, tile // 2 - 2 * k, tile // 2, tile // 2 + 1, tile, tile + 2 * k, 2 * tile + 7, 65536] + [int(x) for x in rng.integers(1, 2 * tile, 6)]
    objs = _objects(torch, k, n_total, sizes, seed=500 + k)
    nt = 2
    nodes, chunks, csz, targets, outs = [], [], [], [], []
    for host, reps in objs:
        nd = _first_k_found(rng, k, n_total, int(rng.integers(nt, n_total - k + 1)))
        missing = [r for r in range(n_total) if r not in nd]
        tg = sorted(rng.choice(missing, nt, replace=False).tolist())
        nodes.append(nd)
        chunks.append([reps[r].data_ptr() for r in nd])
        csz.append(reps[0].numel())
        targets.append(tg)
        outs.append([torch.full((reps[0].numel() + 16,), 0x5A, dtype=torch.uint8, device="cuda") for _ in tg])
    chunk.regenerate_batch_device(k, nodes, chunks, csz, targets, [[o.data_ptr() for o in os_] for os_ in outs])
    torch.cuda.synchronize()
    for (host, reps), tg, os_ in zip(objs, targets, outs):
        L = reps[0].numel()
        for t, o in zip(tg, os_):
            got = o.cpu().numpy()
            assert np.array_equal(got[:L], O.encode(k, t, host)), (host.size, t)
            assert (got[L:] == 0x5A).all()


def test_restore_batch_rejects_bad_objects(gpu):
    import torch
    from vds_amd import chunk
    from vds_amd._lib import VdsEcError, ERESTORE
    k, n = 16, 20
    (host, reps), = _objects(torch, k, n, [1000], seed=900)
    out = torch.zeros(4096, dtype=torch.uint8, device="cuda")
    nd = list(range(k))
    # a trailer claiming more bytes than the replicas hold: "Fatal error" (chunk.h:443), nothing enqueued
    with pytest.raises(VdsEcError) as e:
        chunk.restore_batch_device(k, [nd, nd], [[reps[r].data_ptr() for r in nd]] * 2, [reps[0].numel()] * 2,
                                   [1000 % 32, 65535], [out.data_ptr()] * 2)
    assert e.value.status == ERESTORE


@pytest.mark.parametrize("k,n_total", [(16, 20), (32, 64)])
def test_batch_pairs_halves_of_small_objects(gpu, k, n_total):
    """Many objects of half a tile or less sharing a few survivor sets: their
    halves are paired into tiles across objects (odd counts leave an empty
    half); restore and regenerate both checked object by object."""
    import torch
    from vds_amd import chunk
    rng = np.random.default_rng(31 + k)
    half = 1024 * 2 * k
    sizes = [half] * 9 + [half - 2 * k * 5 - 3] * 4 + [int(x) for x in rng.integers(1, 3 * half, 12)]
    objs = _objects(torch, k, n_total, sizes, seed=700 + k)
    sets = [_first_k_found(rng, k, n_total, int(rng.integers(1, n_total - k + 1))) for _ in range(3)]
    nodes = [sets[i % 3] if i % 5 else list(rng.permutation(sets[i % 3])) for i in range(len(sizes))]
    chunks = [[reps[r].data_ptr() for r in nd] for (_, reps), nd in zip(objs, nodes)]
    csz = [reps[0].numel() for _, reps in objs]
    outs = [torch.full((size + 2 * k,), 0xA5, dtype=torch.uint8, device="cuda") for size in sizes]
    chunk.restore_batch_device(k, nodes, chunks, csz, [sz % (2 * k) for sz in sizes], [o.data_ptr() for o in outs])
    targets = [[min(r for r in range(n_total) if r not in nd)] for nd in nodes]
    rg = [torch.full((c + 8,), 0x5A, dtype=torch.uint8, device="cuda") for c in csz]
    chunk.regenerate_batch_device(k, nodes, chunks, csz, targets, [[o.data_ptr()] for o in rg])
    torch.cuda.synchronize()
    for (host, reps), size, out, tg, r, c in zip(objs, sizes, outs, targets, rg, csz):
        got = out.cpu().numpy()
        assert np.array_equal(got[:size], host), size
        assert (got[size:] == 0xA5).all(), size
        g = r.cpu().numpy()
        assert np.array_equal(g[:c], O.encode(k, tg[0], host)), (size, tg)
        assert (g[c:] == 0x5A).all()


@pytest.mark.parametrize("k", [16, 32])
def test_batch_routes_mixed(gpu, k):
    """One call whose objects take every route: the syndrome batch (survivors
    within 0..k+k/4-1), the RT batch (any other ids < 256, rows = erased
    points below k; regenerate: more targets than n - k split into several
    descriptors), and the per-object path (an id >= 256).  Every object
    against the oracle."""
    import torch
    from vds_amd import chunk
    rng = np.random.default_rng(900 + k)
    n = k + k // 4
    tile = 2048 * 2 * k
    sizes = [tile // 2, tile + 3 * k, 1000, tile // 2 - 2 * k, 2 * tile + 1, 77, tile // 2, tile]
    ids_of = [
        list(range(k)),                                           # syn, nothing erased below k
        [r for r in range(n) if r not in (1, 2)][:k],             # syn
        list(range(3, 3 + k)),                                    # RT: survivors up to k + 2 < n? (syn when < n)
        [0, 300] + list(range(2, k)),                             # per object: id >= 256
        list(range(k // 2)) + list(range(n, n + k // 2)),         # RT: half the points below k erased
        list(range(200, 200 + k)),                                # RT: every point below k erased
        list(rng.permutation(list(range(1, k)) + [n + 5])),       # RT, any order
        list(range(k - 1)) + [255],                               # RT: id 255
    ]
    hosts, reps_of, nodes, chunks, csz, pads, outs = [], [], [], [], [], [], []
    for size, nd in zip(sizes, ids_of):
        host = O.splitmix(SEED + 31 * size + k, size)
        L = chunk.replica_size(k, size)
        reps = {r: torch.from_numpy(O.encode(k, r, host)).cuda() for r in nd}
        hosts.append(host)
        reps_of.append(reps)
        nodes.append(nd)
        chunks.append([reps[r].data_ptr() for r in nd])
        csz.append(L)
        pads.append(size % (2 * k))
        outs.append(torch.full((size + 64,), 0xA5, dtype=torch.uint8, device="cuda"))
    chunk.restore_batch_device(k, nodes, chunks, csz, pads, [o.data_ptr() for o in outs])
    # regenerate: n - k + 3 targets each (more than one RT descriptor holds)
    nt = n - k + 3
    targets = [sorted(rng.choice([r for r in range(260) if r not in nd], nt, replace=False).tolist()) for nd in nodes]
    rg = [[torch.full((c + 8,), 0x5A, dtype=torch.uint8, device="cuda") for _ in range(nt)] for c in csz]
    chunk.regenerate_batch_device(k, nodes, chunks, csz, targets, [[x.data_ptr() for x in r] for r in rg])
    torch.cuda.synchronize()
    for i, (host, size) in enumerate(zip(hosts, sizes)):
        got = outs[i].cpu().numpy()
        assert np.array_equal(got[:size], host), (i, nodes[i])
        assert (got[size:] == 0xA5).all()
        for t, x in zip(targets[i], rg[i]):
            g = x.cpu().numpy()
            assert np.array_equal(g[:csz[i]], O.encode(k, t, host)), (i, t)
            assert (g[csz[i]:] == 0x5A).all()


def test_batch_many_threads_mixed_routes(gpu):
    """More threads than the parameter ring has slots (16), each making
    batched calls whose objects take both the syndrome and the RT route (two
    slots per call), on streams of their own.  The two slots of a call are
    reserved together, so no thread holds one while waiting for another (the
    hold-and-wait deadlock of round 3).  Every output checked."""
    import threading
    import torch
    from vds_amd import chunk
    k, n = 16, 20
    size = 2048 * 2 * k + 300
    host = O.splitmix(SEED + 4242, size)
    L = chunk.replica_size(k, size)
    reps = {r: torch.from_numpy(O.encode(k, r, host)).cuda() for r in list(range(n)) + [40, 41, 42]}
    sets = [list(range(k)), [r for r in range(n) if r not in (2, 9)][:k],  # syndrome route
            list(range(2, k)) + [40, 41], list(range(1, k)) + [42]]        # RT route
    nthreads, calls = 24, 6
    outs = [[torch.zeros(size + 16, dtype=torch.uint8, device="cuda") for _ in sets] for _ in range(nthreads)]
    errors = []
    barrier = threading.Barrier(nthreads)

    def worker(t):
        try:
            s = torch.cuda.Stream()
            barrier.wait()
            for _ in range(calls):
                chunk.restore_batch_device(k, sets, [[reps[r].data_ptr() for r in nd] for nd in sets], [L] * len(sets),
                                           [size % (2 * k)] * len(sets), [o.data_ptr() for o in outs[t]], stream=s)
            s.synchronize()
        except Exception as e:  # noqa: BLE001 (reported below)
            errors.append(repr(e))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(nthreads)]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=90)
    assert not any(x.is_alive() for x in th), "batched calls deadlocked"
    assert not errors, errors
    torch.cuda.synchronize()
    for t in range(nthreads):
        for o in outs[t]:
            got = o.cpu().numpy()
            assert np.array_equal(got[:size], host)
            assert (got[size:] == 0).all()


def test_host_contexts_reused_across_threads(gpu):
    """Each calling thread gets a host staging context (pinned and device
    buffers and a stream); a thread that exits returns its context to a pool,
    so short-lived threads reuse them instead of leaking one set each."""
    import ctypes
    import threading
    from vds_amd import _lib, chunk
    k = 16
    data = O.splitmix(SEED + 77, 5000)
    want = [O.encode(k, r, data) for r in range(4)]
    created, pooled = ctypes.c_uint64(), ctypes.c_uint64()

    def one():
        got = chunk.encode_host(k, range(4), data)
        assert all(np.array_equal(g, w) for g, w in zip(got, want))

    one()  # this thread's own context
    _lib.lib().vds_ec_host_ctx_stats(ctypes.byref(created), ctypes.byref(pooled))
    before = created.value
    for _ in range(12):  # sequential short-lived threads: one pooled context serves them all
        t = threading.Thread(target=one)
        t.start()
        t.join()
    _lib.lib().vds_ec_host_ctx_stats(ctypes.byref(created), ctypes.byref(pooled))
    assert created.value <= before + 1, (before, created.value)
    assert pooled.value >= 1


@pytest.mark.parametrize("k", [16, 32])
def test_batch_small_perm_many_tiles(gpu, k):
    """More tiles than the launch has workgroups (each workgroup walks several
    tiles, so the next tile's survivors must be prefetched on every route):
    the SMALL ms = 1 / 2 restore and regenerate and the PERM regenerate over
    one tile per object, 700 objects, codewords checked against the encode."""
    import torch
    from vds_amd import chunk
    n = 2 * k
    size = 2048 * 2 * k  # one tile per object
    count = 700
    L = chunk.replica_size(k, size)
    inp = torch.empty(count * size, dtype=torch.uint8, device="cuda")
    chunk.fill_splitmix_device(inp, count * size, SEED + 31 * k)
    reps = torch.empty((n, count * L), dtype=torch.uint8, device="cuda")
    chunk.encode_device(k, list(range(n)), inp, size, size, count, [reps[i].data_ptr() for i in range(n)], L)
    rng = np.random.default_rng(k)
    nodes, targets = [], []
    for o in range(count):
        kind = o % 4
        if kind == 0:    # survivors 0..k-1: restore skips phase 2, regenerate is PERM
            nd, t = list(range(k)), int(rng.integers(k, n))
        elif kind == 1:  # SMALL ms = 1
            e = int(rng.integers(0, k))
            nd, t = [r for r in range(k + 1) if r != e], e
        else:            # SMALL ms = 2
            e = sorted(rng.choice(k + 2, 2, replace=False).tolist())
            nd, t = [r for r in range(k + 2) if r not in e], e[0]
        if o % 3 == 0:
            nd = list(rng.permutation(nd))
        nodes.append(nd)
        targets.append([t])
    chunks = [[reps[r].data_ptr() + o * L for r in nd] for o, nd in enumerate(nodes)]
    out = torch.zeros(count * size, dtype=torch.uint8, device="cuda")
    chunk.restore_batch_device(k, nodes, chunks, [L] * count, [0] * count,
                               [out.data_ptr() + o * size for o in range(count)])
    rg = torch.zeros(count * L, dtype=torch.uint8, device="cuda")
    chunk.regenerate_batch_device(k, nodes, chunks, [L] * count, targets, [[rg.data_ptr() + o * L] for o in range(count)])
    torch.cuda.synchronize()
    assert torch.equal(out, inp)
    want = torch.stack([reps[targets[o][0], o * L:(o + 1) * L] for o in range(count)])
    assert torch.equal(rg.view(count, L), want)


@pytest.mark.parametrize("k", [16, 32])
def test_regenerate_same_set_two_small_sizes(gpu, k):
    """One survivor set, two objects whose targets route it to SMALL ms = 1
    (target an erased point below k) and ms = 2 (target k + 1): the plans are
    per (set, size), not per set."""
    import torch
    from vds_amd import chunk
    n = k + 2
    size = 1024 * 2 * k
    nd = [r for r in range(k + 1) if r != 3]  # erased 3 and k + 1 within 0..k+1
    objs = _objects(torch, k, n, [size, size], seed=4400 + k)
    targets = [[3], [k + 1]]
    chunks = [[reps[r].data_ptr() for r in nd] for _, reps in objs]
    L = objs[0][1][0].numel()
    outs = [torch.zeros(L + 8, dtype=torch.uint8, device="cuda") for _ in range(2)]
    chunk.regenerate_batch_device(k, [nd, nd], chunks, [L, L], targets, [[o.data_ptr()] for o in outs])
    torch.cuda.synchronize()
    for (host, reps), t, o in zip(objs, targets, outs):
        assert np.array_equal(o.cpu().numpy()[:L], O.encode(k, t[0], host)), t


@pytest.mark.parametrize("k", [16, 32])
def test_batch_planner_many_parts(gpu, k):
    """A call large enough for the planner's sixteen parallel parts (>= 16384
    objects), whose survivor sets repeat across parts and cover every route:
    survivors exactly 0..k-1 (SMALL / PERM), the first k found at a low loss
    rate (SMALL, the N = k + k/4 syndrome kernel; sets shared by many
    objects), at a high loss rate (RT / RT2; sets nearly all distinct), and
    permuted orders.  Every restored object equals its input and every
    regenerated replica (the first lost one) equals the encoded replica, both
    compared on the device."""
    import torch
    from vds_amd import _lib, chunk
    n = 64 if k == 32 else 40
    count, size = 17000, 2 * k * 37 + 5  # (odd: a non-zero trailer; one half tile per object)
    L = chunk.replica_size(k, size)
    Ls = -(-L // 256) * 256
    inp = torch.empty(count * size, dtype=torch.uint8, device="cuda")
    chunk.fill_splitmix_device(inp, count * size, SEED + 4242 + k)
    reps = torch.zeros((n, count * Ls), dtype=torch.uint8, device="cuda")
    chunk.encode_device(k, list(range(n)), inp, size, size, count, [reps[i].data_ptr() for i in range(n)], Ls)
    rng = np.random.default_rng(77 + k)
    kind = rng.choice(4, count, p=[0.2, 0.4, 0.3, 0.1])
    loss = np.where(kind == 2, 0.25, 0.03)
    lost = rng.random((count, n)) < loss[:, None]
    lost[kind == 0, :k] = False  # survivors exactly 0..k-1 (the first k found)
    lost[kind == 0, k] = True    # (and replica k lost: the first target is k)
    lost[:, :k + 4][(~lost).sum(axis=1) < k] = False  # (every object restorable)
    nodes = np.stack([np.flatnonzero(~lost[o])[:k] for o in range(count)]).astype(np.uint16)
    perm = kind == 3
    nodes[perm] = np.stack([rng.permutation(r) for r in nodes[perm]])
    base = np.asarray([reps[i].data_ptr() for i in range(n)], dtype=np.uint64)
    cp = (base[nodes] + (np.arange(count, dtype=np.uint64) * Ls)[:, None]).astype(np.uint64)
    sizes = np.full(count, L, dtype=np.uint64)
    pads = np.full(count, size % (2 * k), dtype=np.uint16)
    out = torch.zeros(count * size, dtype=torch.uint8, device="cuda")
    outs = (np.uint64(out.data_ptr()) + np.arange(count, dtype=np.uint64) * size).astype(np.uint64)
    lib = _lib.lib()
    s = torch.cuda.current_stream().cuda_stream
    _lib.check(lib.vds_ec_restore16_batch_device(k, count, nodes.ctypes.data_as(_lib.u16p), cp.ctypes.data_as(_lib.vpp),
                                                 sizes.ctypes.data_as(_lib.u64p), pads.ctypes.data_as(_lib.u16p),
                                                 outs.ctypes.data_as(_lib.vpp), 0, s))
    rg = np.flatnonzero(lost.any(axis=1))
    tg = np.argmax(lost[rg], axis=1).astype(np.uint16)
    rgo = torch.zeros(len(rg) * Ls, dtype=torch.uint8, device="cuda")
    rgp = (np.uint64(rgo.data_ptr()) + np.arange(len(rg), dtype=np.uint64) * Ls).astype(np.uint64)
    rn, rc = np.ascontiguousarray(nodes[rg]), np.ascontiguousarray(cp[rg])
    rs = np.full(len(rg), L, dtype=np.uint64)
    _lib.check(lib.vds_ec_regenerate16_batch_device(k, len(rg), rn.ctypes.data_as(_lib.u16p), rc.ctypes.data_as(_lib.vpp),
                                                    rs.ctypes.data_as(_lib.u64p), 1, tg.ctypes.data_as(_lib.u16p),
                                                    rgp.ctypes.data_as(_lib.vpp), s))
    torch.cuda.synchronize()
    bad = (out.view(count, size) != inp.view(count, size)).any(dim=1).nonzero().flatten().tolist()
    assert not bad, f"{len(bad)} restored objects differ, first {bad[:5]}"
    want = reps.view(n, count, Ls)[torch.from_numpy(tg.astype(np.int64)).cuda(), torch.from_numpy(rg).cuda(), :L]
    badr = (rgo.view(-1, Ls)[:, :L] != want).any(dim=1).nonzero().flatten().tolist()
    assert not badr, f"{len(badr)} regenerated replicas differ, first {badr[:5]}"
    # the routes the call took (the test is meant to cover them all)
    assert (nodes < k + k // 4).all(axis=1).sum() > count // 2 and (~(nodes < k + k // 4).all(axis=1)).sum() > 100


def test_restore_batch_dual_tiles(gpu):
    """k = 32, n = 40: objects whose erased sets are all different (the live
    shape at a high loss rate) -- restore and regenerate: each plan's odd half goes into a dual tile
    with another plan's (kTileDual: two survivor layouts and two coefficient
    walks in one tile).  Codeword and non-codeword survivors, objects of one
    to three halves and ragged sizes, a few sets shared; every object against
    the oracle's restore of the same chunks."""
    import torch
    from vds_amd import chunk
    k, n = 32, 40
    rng = np.random.default_rng(4242)
    half = 1024 * 2 * k
    sizes = ([half] * 23 + [half - 2 * k * 3 - 1, 2 * half, 3 * half + 5, 1, 2 * k * 11 + 7] +
             [int(x) for x in rng.integers(1, 3 * half, 10)])
    objs = _objects(torch, k, n, sizes, seed=1300)
    sets = []
    while len(sets) < len(sizes):
        er = set(rng.choice(n, n - k, replace=False).tolist())
        nd = [r for r in range(n) if r not in er]
        if max(nd) >= k + 2 and min(er) < k:  # the N-point syndrome class (not SMALL)
            sets.append(nd)
    sets[5] = sets[4]  # two objects of one plan beside the singles
    nodes, chunks, csz, pads, outs, data = [], [], [], [], [], []
    for i, ((host, reps), size) in enumerate(zip(objs, sizes)):
        nd = sets[i] if i % 3 else list(rng.permutation(sets[i]))
        if i % 2:  # non-codeword survivors: random cells in every chunk (trailers kept)
            for r in nd:
                reps[r][:-2].copy_(torch.from_numpy(rng.integers(0, 256, reps[r].numel() - 2, dtype=np.uint8)).cuda())
        nodes.append(nd)
        chunks.append([reps[r].data_ptr() for r in nd])
        csz.append(reps[0].numel())
        pads.append(size % (2 * k))
        outs.append(torch.full((size + 4 * k,), 0xA5, dtype=torch.uint8, device="cuda"))
        data.append([reps[r].cpu().numpy() for r in nd])
    chunk.restore_batch_device(k, nodes, chunks, csz, pads, [o.data_ptr() for o in outs])
    # regenerate: two erased points below n of each object (the repair
    # route's result: restore, then re-encode the E bytes)
    targets = [sorted(rng.choice([r for r in range(n) if r not in nd], 2, replace=False).tolist()) for nd in nodes]
    rg = [[torch.full((c + 8,), 0x5A, dtype=torch.uint8, device="cuda") for _ in tg] for c, tg in zip(csz, targets)]
    chunk.regenerate_batch_device(k, nodes, chunks, csz, targets, [[x.data_ptr() for x in r] for r in rg])
    torch.cuda.synchronize()
    for i, ((host, reps), size, out, nd) in enumerate(zip(objs, sizes, outs, nodes)):
        got = out.cpu().numpy()
        ref = O.restore(k, nd, data[i])
        assert ref is not None and ref.size == size
        assert np.array_equal(got[:size], ref), (i, size, nd)
        if i % 2 == 0:
            assert np.array_equal(got[:size], host), (i, size)
        assert (got[size:] == 0xA5).all(), (i, size)
        for t, x in zip(targets[i], rg[i]):
            g = x.cpu().numpy()
            assert np.array_equal(g[:csz[i]], O.encode(k, t, ref)), (i, t)
            assert (g[csz[i]:] == 0x5A).all()
