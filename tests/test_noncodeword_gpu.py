"""Survivors that are NOT one codeword, on every restore and regenerate path.

A stored replica can be corrupt, so the survivors handed to restore or repair
need not be evaluations of one polynomial.  The reference still produces
well-defined bytes for them:
  - restore (chunk.h:402-444) applies V_S^{-1} to the survivors' cells and
    returns the first E bytes, E from the trailer p of chunks[0]
    (chunk.h:408, 415-419);
  - repair (sync_process.cpp:313-335) is that restore followed by a re-encode
    of the E bytes (dht_network_client.cpp:582-658 -> chunk.h:245-281): the
    last stripe zero-padded past E, the trailer E mod 2k.
For a codeword the decode is already zero past E; for random survivors it is
not, so the trim shows.  Every device path here (syndrome kernel, its batch
mode, the runtime-coefficient kernel in whole-tile and stream mode, the
generic kernel, the batch fallback) is compared byte for byte with the oracle
on random survivors, with p = 0, odd and even p, p = 2k, and survivors whose
trailers disagree (restore and repair read chunks[0]'s).
"""
import numpy as np
import pytest

import oracle_ctypes as O

pytestmark = pytest.mark.gpu


def _survivors(rng, k, T, p, vary=False):
    """k random replicas of 2T+2 bytes with trailer p (vary: only the
    first carries p, the others random trailers)."""
    out = []
    for j in range(k):
        b = rng.integers(0, 256, 2 * T + 2, dtype=np.uint8)
        q = p if (j == 0 or not vary) else int(rng.integers(0, 65536))
        b[-2], b[-1] = q >> 8, q & 0xFF
        out.append(b)
    return out


def _ref_regen(k, nodes, chunks, targets):
    obj = O.restore(k, nodes, chunks)
    assert obj is not None
    return [O.encode(k, t, obj) for t in targets]


def _path_restore(k, nodes, L, p, count):
    from vds_amd import _lib
    nd = np.array(nodes, dtype=np.uint16)
    return _lib.lib().vds_ec_restore16_path(k, nd.ctypes.data_as(_lib.u16p), L, p, count)


def _path_regen(k, nodes, targets, L):
    from vds_amd import _lib
    nd = np.array(nodes, dtype=np.uint16)
    tg = np.array(targets, dtype=np.uint16)
    return _lib.lib().vds_ec_regenerate16_path(k, nd.ctypes.data_as(_lib.u16p), tg.ctypes.data_as(_lib.u16p),
                                               len(targets), L)


def _stage(torch, objs, stride):
    """objs[o][j] (host arrays) -> k device buffers of count objects at `stride`."""
    k = len(objs[0])
    count = len(objs)
    host = np.zeros((k, count, stride), dtype=np.uint8)
    for o, sv in enumerate(objs):
        for j, b in enumerate(sv):
            host[j, o, :b.size] = b
    return torch.from_numpy(host).cuda()


# (k, nodes, T, path): the restore paths vds_ec_restore16_path reports
RESTORE_CASES = [
    (16, [r for r in range(20) if r not in (0, 5, 10, 15)], 2 * 2048 + 3, 3),   # syndrome kernel, whole tiles
    (16, list(range(4, 20)), 2048 * 2 + 1, 3),                                   # last stripe right after the tiles
    (16, list(range(8, 24)), 4096 + 1, 2),                                       # runtime-coefficient, whole tiles
    (16, [25] + list(range(1, 16)), 1025, 2),                                    # runtime-coefficient stream mode
    (32, [40] + list(range(1, 32)), 1025, 2),                                    # ... at k = 32
    (16, [3, 30, 7, 1, 9, 11, 2, 4, 6, 8, 10, 12, 13, 14, 15, 0], 200, 1),      # generic
    (32, [r for r in range(40) if r % 5 != 2], 2048 + 9, 3),                     # syndrome k = 32
]


@pytest.mark.parametrize("k,nodes,T,path", RESTORE_CASES)
@pytest.mark.parametrize("pmode", ["zero", "odd", "even", "one"])
def test_restore_noncodeword_paths(gpu, k, nodes, T, path, pmode):
    import torch
    from vds_amd import chunk
    p = {"zero": 0, "odd": 2 * k - 3, "even": 2 * k - 2, "one": 1}[pmode]
    # the paths are chosen by full output stripes: keep F = T (p = 0) or T - 1
    T_ = T if p else T - 1
    rng = np.random.default_rng(1000 * k + T_ + p)
    count = 3
    objs = [_survivors(rng, k, T_, p) for _ in range(count)]
    L = 2 * T_ + 2
    assert _path_restore(k, nodes, L, p, count) == path
    stride = L + 6
    dev = _stage(torch, objs, stride)
    want = [O.restore(k, nodes, sv) for sv in objs]
    E = want[0].size
    ostride = E + 40
    out = torch.full((count, ostride), 0xA5, dtype=torch.uint8, device="cuda")
    chunk.restore_device(k, nodes, [dev[j].data_ptr() for j in range(k)], L, stride, p, count, out, ostride)
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    for o in range(count):
        assert np.array_equal(got[o, :E], want[o]), (o, E)
        assert (got[o, E:] == 0xA5).all(), "wrote past E"


@pytest.mark.parametrize("k,n_total", [(16, 20), (16, 48), (32, 40), (32, 64), (16, 17), (16, 18), (32, 33), (32, 34)])
def test_restore_batch_noncodeword(gpu, k, n_total):
    """Batch mode (k_restore_syn BATCH for survivors within its points -- the
    SMALL ms = 1, 2 kernels for survivors within 0..k, 0..k+1 -- the RT mode
    and the per-object fallback for the rest) on random survivors and trailers."""
    import torch
    from vds_amd import chunk
    rng = np.random.default_rng(77 + k + n_total)
    Ts = [1, 7, 1023, 1024, 1025, 2048, 2049, 3000, 4096 + 513]
    pvals = [0, 1, 2 * k - 1, 2 * k - 2, 2 * k, 5]
    nodes, chunks, csz, pads, outs, want, keep = [], [], [], [], [], [], []
    for i, T in enumerate(Ts * 2):
        p = pvals[i % len(pvals)]
        if p == 2 * k and T == 1:
            p = 0
        sv = _survivors(rng, k, T, p)
        gone = set(rng.choice(n_total, n_total - k, replace=False).tolist())
        nd = [r for r in range(n_total) if r not in gone]
        if i % 3 == 0:
            nd = list(rng.permutation(nd))
        bufs = [torch.from_numpy(b).cuda() for b in sv]
        keep.append(bufs)
        nodes.append(nd)
        chunks.append([b.data_ptr() for b in bufs])
        csz.append(2 * T + 2)
        pads.append(p)
        w = O.restore(k, nd, sv)
        want.append(w)
        outs.append(torch.full((w.size + 64,), 0xA5, dtype=torch.uint8, device="cuda"))
    chunk.restore_batch_device(k, nodes, chunks, csz, pads, [o.data_ptr() for o in outs])
    torch.cuda.synchronize()
    for i, (w, o) in enumerate(zip(want, outs)):
        g = o.cpu().numpy()
        assert np.array_equal(g[:w.size], w), (i, csz[i], pads[i], nodes[i])
        assert (g[w.size:] == 0xA5).all()


# (k, nodes, targets, T, path): the regenerate paths vds_ec_regenerate16_path reports
REGEN_CASES = [
    (16, [r for r in range(20) if r not in (0, 5, 10, 15)], [15, 0], 2 * 2048 + 3, 3),
    (16, [r for r in range(20) if r not in (1, 2, 3, 4)], [1, 4], 2 * 2048, 3),    # last stripe in a tile
    (16, list(range(4, 20)), [0, 3, 30], 2048 + 2, 2),                            # a target outside the code
    (32, [40] + list(range(1, 32)), [0, 63], 1024, 2),                             # stream mode (T % 512 == 0)
    (16, [r for r in range(20) if r not in (0, 5, 10, 15)], [5, 10], 300, 1),      # generic
    (32, [r for r in range(40) if r % 5 != 2], [2, 37], 2048 * 2 + 1, 3),
    (3, [4, 1, 2], [0, 3, 7], 50, 1),
]


@pytest.mark.parametrize("k,nodes,targets,T,path", REGEN_CASES)
@pytest.mark.parametrize("pmode", ["zero", "odd", "even", "full"])
def test_regenerate_noncodeword_paths(gpu, k, nodes, targets, T, path, pmode):
    """restore -> re-encode on the oracle vs the fused regenerate: every byte,
    the trimmed last cell and the trailer E mod 2k included; only the first
    survivor carries the trailer the route reads."""
    import torch
    from vds_amd import chunk
    p = {"zero": 0, "odd": 2 * k - 3, "even": 2 * k - 4 if k > 2 else 2, "full": 2 * k}[pmode]
    rng = np.random.default_rng(3 * T + 11 * k + p)
    count = 2
    objs = [_survivors(rng, k, T, p, vary=True) for _ in range(count)]
    L = 2 * T + 2
    assert _path_regen(k, nodes, targets, L) == path
    stride = L + 4
    dev = _stage(torch, objs, stride)
    ostride = L + 8
    outs = torch.full((len(targets), count, ostride), 0x5A, dtype=torch.uint8, device="cuda")
    chunk.regenerate_device(k, nodes, [dev[j].data_ptr() for j in range(k)], L, stride, count, targets,
                            [outs[i].data_ptr() for i in range(len(targets))], ostride)
    torch.cuda.synchronize()
    got = outs.cpu().numpy()
    for o in range(count):
        want = _ref_regen(k, nodes, objs[o], targets)
        for i, t in enumerate(targets):
            assert want[i].size == L
            assert np.array_equal(got[i, o, :L], want[i]), (o, t, p)
            assert (got[i, o, L:] == 0x5A).all()


@pytest.mark.parametrize("k,n_total", [(16, 20), (16, 48), (32, 40), (32, 64), (16, 18), (32, 34)])
def test_regenerate_batch_noncodeword(gpu, k, n_total):
    """Batch regenerate (syndrome batch kernel + its device-side tail, and the
    per-object fallback) on random survivors with disagreeing trailers."""
    import torch
    from vds_amd import chunk
    rng = np.random.default_rng(500 + k + n_total)
    Ts = [0, 1, 5, 1023, 1024, 1025, 2048, 2051, 4096]
    pvals = [0, 1, 2 * k - 1, 2 * k - 2, 2 * k, 7]
    nt = 2
    nodes, chunks, csz, targets, outs, want, keep = [], [], [], [], [], [], []
    for i, T in enumerate(Ts * 2):
        p = pvals[i % len(pvals)]
        if T == 0:
            p = 0 if i % 2 else 2 * k  # (E must be restorable: 0 or 2k when there are no cells)
        sv = _survivors(rng, k, T, p, vary=True)
        gone = set(rng.choice(n_total, n_total - k, replace=False).tolist())
        nd = [r for r in range(n_total) if r not in gone]
        if i % 2 == 0:
            nd = list(rng.permutation(nd))
        missing = [r for r in range(n_total) if r not in nd]
        tg = sorted(rng.choice(missing, nt, replace=False).tolist())
        bufs = [torch.from_numpy(b).cuda() for b in sv]
        keep.append(bufs)
        nodes.append(nd)
        chunks.append([b.data_ptr() for b in bufs])
        csz.append(2 * T + 2)
        targets.append(tg)
        want.append(_ref_regen(k, nd, sv, tg))
        outs.append([torch.full((2 * T + 2 + 16,), 0x5A, dtype=torch.uint8, device="cuda") for _ in tg])
    chunk.regenerate_batch_device(k, nodes, chunks, csz, targets, [[o.data_ptr() for o in os_] for os_ in outs])
    torch.cuda.synchronize()
    for i, (ws, os_) in enumerate(zip(want, outs)):
        L = csz[i]
        for t, w, o in zip(targets[i], ws, os_):
            g = o.cpu().numpy()
            assert w.size == L
            assert np.array_equal(g[:L], w), (i, L, t, nodes[i])
            assert (g[L:] == 0x5A).all()


def test_regenerate_host_noncodeword_and_trailer_errors(gpu):
    from vds_amd import chunk
    from vds_amd._lib import VdsEcError, ERESTORE
    k, T = 16, 700
    rng = np.random.default_rng(5)
    nodes = [r for r in range(20) if r not in (2, 3, 11, 19)]
    for p in (0, 1, 13, 31, 32):
        sv = _survivors(rng, k, T, p, vary=True)
        got = chunk.regenerate_host(k, nodes, sv, [2, 19, 40])
        for g, w in zip(got, _ref_regen(k, nodes, sv, [2, 19, 40])):
            assert np.array_equal(g, w), p
    # p > 2k: the route re-encodes to a longer replica (p <= 4k) or fails
    # (p > 4k, "Fatal error at chunk_restore::restore"); both refused
    for p in (33, 64, 65, 4000):
        sv = _survivors(rng, k, T, p)
        with pytest.raises(VdsEcError) as e:
            chunk.regenerate_host(k, nodes, sv, [2])
        assert e.value.status == ERESTORE, p


def test_batch_rejects_duplicate_ids_before_enqueue(gpu):
    """an object with a repeated replica id fails the whole call
    with ESINGULAR before anything is written (restore and regenerate)."""
    import torch
    from vds_amd import chunk
    from vds_amd._lib import VdsEcError, ESINGULAR
    k, T = 16, 1024
    rng = np.random.default_rng(9)
    good = list(range(16))
    dup = list(range(15)) + [3]
    sv = [torch.from_numpy(b).cuda() for b in _survivors(rng, k, T, 0)]
    ptrs = [b.data_ptr() for b in sv]
    out = torch.full((2, 2 * k * T + 64), 0xA5, dtype=torch.uint8, device="cuda")
    with pytest.raises(VdsEcError) as e:
        chunk.restore_batch_device(k, [good, dup], [ptrs, ptrs], [2 * T + 2] * 2, [0, 0],
                                   [out[0].data_ptr(), out[1].data_ptr()])
    assert e.value.status == ESINGULAR
    rg = torch.full((2, 2 * T + 2), 0x5A, dtype=torch.uint8, device="cuda")
    with pytest.raises(VdsEcError) as e:
        chunk.regenerate_batch_device(k, [good, dup], [ptrs, ptrs], [2 * T + 2] * 2, [[16], [17]],
                                      [[rg[0].data_ptr()], [rg[1].data_ptr()]])
    assert e.value.status == ESINGULAR
    torch.cuda.synchronize()
    assert (out.cpu().numpy() == 0xA5).all() and (rg.cpu().numpy() == 0x5A).all(), "partial output"


@pytest.mark.parametrize("k", [16, 32])
def test_regenerate_batch_perm_noncodeword(gpu, k):
    """The PERM batch regenerate (survivors exactly 0..k-1 in any order, one
    target t in k..2k-1: P(t) = sum_c l_c(k) y_(c ^ (t - k)), one fixed program
    read through a permuted address): random survivors and trailers, every
    target of k..2k-1, sizes across the half-tile boundaries, against the
    oracle's restore -> re-encode route."""
    import torch
    from vds_amd import chunk
    rng = np.random.default_rng(4100 + k)
    Ts = [0, 1, 5, 1023, 1024, 1025, 2048, 3000]
    pvals = [0, 1, 2 * k - 1, 2 * k - 2, 2 * k, 7]
    nodes, chunks, csz, targets, outs, want, keep = [], [], [], [], [], [], []
    for i in range(2 * k + 5):
        T = Ts[i % len(Ts)]
        p = pvals[i % len(pvals)]
        if T == 0:
            p = 0 if i % 2 else 2 * k
        sv = _survivors(rng, k, T, p, vary=True)
        nd = list(range(k)) if i % 3 else list(rng.permutation(k))
        t = k + (i % k) if i < 2 * k else int(rng.integers(k, 2 * k))
        bufs = [torch.from_numpy(b).cuda() for b in sv]
        keep.append(bufs)
        nodes.append(nd)
        chunks.append([b.data_ptr() for b in bufs])
        csz.append(2 * T + 2)
        targets.append([t])
        want.append(_ref_regen(k, nd, sv, [t]))
        outs.append([torch.full((2 * T + 2 + 16,), 0x5A, dtype=torch.uint8, device="cuda")])
    chunk.regenerate_batch_device(k, nodes, chunks, csz, targets, [[o.data_ptr() for o in os_] for os_ in outs])
    torch.cuda.synchronize()
    for i, (ws, os_) in enumerate(zip(want, outs)):
        L = csz[i]
        g = os_[0].cpu().numpy()
        assert np.array_equal(g[:L], ws[0]), (i, L, targets[i])
        assert (g[L:] == 0x5A).all()


def test_restore_batch_rt2_rows_noncodeword(gpu):
    """RT2 (k = 32, every survivor below 2k, at most kRt2MaxRows = 12 erased
    points below k: the PERM evaluations of P0 and the |E| x |E| products in
    groups of eight, ec_internal.hpp; rows 9..12 spread over all waves) in one
    batch call: random survivors, every trailer kind, 1..12 rows, objects of
    one to three tiles and tiles whose halves have different row counts,
    borrowed ids in any order."""
    import torch
    from vds_amd import chunk
    k = 32
    rng = np.random.default_rng(4242)
    Ts = [1, 7, 1023, 1024, 1025, 2048, 3000, 5000]
    pvals = [0, 1, 2 * k - 1, 2 * k - 2, 2 * k, 5]
    nodes, keep, chunks, csz, pads, outs, want = [], [], [], [], [], [], []
    for i in range(72):
        T = Ts[i % len(Ts)]
        p = pvals[i % len(pvals)]
        if p == 2 * k and T == 1:
            p = 0
        rows = 1 + (i * 7) % 12
        erased = set(rng.choice(k, rows, replace=False).tolist())
        nd = [a for a in range(k) if a not in erased] + sorted(rng.choice(np.arange(k, 2 * k), rows, replace=False).tolist())
        if i % 3 == 1:
            nd = list(rng.permutation(nd))
        sv = _survivors(rng, k, T, p, vary=(i % 5 == 0))
        bufs = [torch.from_numpy(b).cuda() for b in sv]
        keep.append(bufs)
        nodes.append(nd)
        chunks.append([b.data_ptr() for b in bufs])
        csz.append(2 * T + 2)
        pads.append(p)
        w = O.restore(k, nd, sv)
        want.append(w)
        outs.append(torch.full((w.size + 64,), 0xA5, dtype=torch.uint8, device="cuda"))
    chunk.restore_batch_device(k, nodes, chunks, csz, pads, [o.data_ptr() for o in outs])
    torch.cuda.synchronize()
    for i, (w, o) in enumerate(zip(want, outs)):
        g = o.cpu().numpy()
        assert np.array_equal(g[:w.size], w), (i, csz[i], pads[i], nodes[i])
        assert (g[w.size:] == 0xA5).all()
