"""Run-time compiled restore kernels (vds_amd/csrc/vds_ec_jit.cpp): for a
survivor set of the syndrome kernel's points, the library generates that set's
fill programs (the erased points below k as Lagrange combinations of the
survivors) and compiles k_restore_syn's body with them (hiprtc).  The bytes
must equal the reference's V_S^{-1} route (chunk.h:290-444, the oracle) for
codewords and non-codewords alike.

CPU: the compile itself (no device needed) and the argument checks.
GPU: every kind of erased set (all below k, none below k, mixed, one), the
     object / tail / batch layouts, non-codeword survivors vs the oracle.
"""
import numpy as np
import pytest

import oracle_ctypes as O

SEED = 0x7664730000000000


def _nodes(n, erased):
    return [r for r in range(n) if r not in erased]


def test_jit_build_compiles_without_gpu(vds_lib):
    from vds_amd import chunk
    # erased points all below k, and all beyond it (no fill program at all)
    assert chunk.jit_build(16, _nodes(20, (0, 5, 10, 15))) > 10000
    assert chunk.jit_build(16, _nodes(20, (16, 17, 18, 19))) > 10000
    assert chunk.jit_build(32, _nodes(40, (1, 2, 3, 4, 33, 34, 38, 39))) > 10000


def test_jit_build_rejects_sets_outside_the_syndrome_points(vds_lib):
    from vds_amd import chunk
    from vds_amd._lib import VdsEcError
    for k, nodes in ((16, list(range(1, 17)) [:15] + [20]),   # id beyond k + k/4 - 1
                     (16, [0] * 16),                          # repeated id
                     (24, list(range(24))),                   # no compiled (k, n)
                     (16, list(range(15)) + [14])):
        with pytest.raises(VdsEcError):
            chunk.jit_build(k, nodes)


def test_jit_disk_cache_across_processes(vds_lib, tmp_path):
    """VDS_EC_JIT_CACHE: the first process compiles and stores the code
    object; a second process loads the same bytes without the compiler."""
    import os
    import subprocess
    import sys
    script = ("from vds_amd import chunk, _lib; _lib.lib();"
              "print(chunk.jit_build(16, [r for r in range(20) if r not in (2, 7, 12, 17)]))")
    env = dict(os.environ, VDS_EC_JIT_CACHE=str(tmp_path))
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sizes = [int(subprocess.run([sys.executable, "-c", script], env=env, cwd=root, check=True,
                                capture_output=True, text=True, timeout=300).stdout.split()[-1])
             for _ in range(2)]
    files = list(tmp_path.glob("*.co"))
    # the file: a 32-byte header (magic, key, length, checksum), then the code object
    assert len(files) == 1 and sizes[0] == sizes[1] == files[0].stat().st_size - 32 > 10000
    head = files[0].read_bytes()[:32]
    assert head[:8] == b"VDSECJ1\0" and int.from_bytes(head[16:24], "little") == sizes[0]
    assert not list(tmp_path.glob("*.co.*"))  # (mkstemp temporaries renamed or removed)


def test_jit_disk_cache_rejects_damaged_files(vds_lib, tmp_path):
    """A cache file whose checksum, length or key does not match is a miss:
    it is removed and the kernel recompiled (the directory may be shared)."""
    import os
    import subprocess
    import sys
    script = ("from vds_amd import chunk, _lib; _lib.lib();"
              "print(chunk.jit_build(16, [r for r in range(20) if r not in (1, 6, 11, 16)]))")
    env = dict(os.environ, VDS_EC_JIT_CACHE=str(tmp_path))
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

    def run():
        return int(subprocess.run([sys.executable, "-c", script], env=env, cwd=root, check=True,
                                  capture_output=True, text=True, timeout=300).stdout.split()[-1])
    size = run()
    f, = tmp_path.glob("*.co")
    good = f.read_bytes()
    for bad in (good[:-100],                                   # short
                good[:5000] + bytes([good[5000] ^ 1]) + good[5001:],  # one flipped bit
                b"\0" * len(good)):                            # foreign
        f.write_bytes(bad)
        assert run() == size
        assert f.read_bytes() == good  # recompiled and rewritten


@pytest.fixture
def jit_sync(gpu):
    from vds_amd import chunk
    chunk.jit_set_mode(2)
    yield
    chunk.jit_set_mode(0)


def _path(k, nodes, L, padding=0, count=1):
    from vds_amd import _lib
    arr = np.asarray(nodes, dtype=np.uint16)
    return _lib.lib().vds_ec_restore16_path(k, arr.ctypes.data_as(_lib.u16p), L, padding, count)


def _sets(k, n, rng, extra):
    m = n - k
    sets = [tuple(range(0, n, n // m))[:m],          # every erased point below k
            tuple(range(k, n)),                       # none below k: no fill at all
            tuple(range(m)),
            tuple(range(k - m // 2, k + m // 2)),     # mixed
            (3,) + tuple(range(k + 1, n))]            # one below k
    sets += [tuple(sorted(int(x) for x in rng.choice(n, m, replace=False))) for _ in range(extra)]
    return sets


@pytest.mark.gpu
@pytest.mark.parametrize("k,n,extra", [(16, 20, 6), (32, 40, 1)])
def test_jit_restore_erased_sets(jit_sync, k, n, extra):
    """Objects of two whole tiles plus a generic tail, three at a stride: the
    compiled kernel runs (path 4) and restores every byte, nothing past."""
    import torch
    from vds_amd import chunk
    size = 2 * 2048 * 2 * k + 2 * k * 5 + 3
    count, stride = 3, size + 40
    L = chunk.replica_size(k, size)
    t = torch.zeros(stride * count, dtype=torch.uint8, device="cuda")
    for o in range(count):
        chunk.fill_splitmix_device(t[o * stride:], size, SEED + 3100 + o)
    reps = torch.zeros((n, count, L), dtype=torch.uint8, device="cuda")
    chunk.encode_device(k, list(range(n)), t, size, stride, count, [reps[i].data_ptr() for i in range(n)], L)
    rng = np.random.default_rng(31 + k)
    out = torch.zeros((count, stride), dtype=torch.uint8, device="cuda")
    for erased in _sets(k, n, rng, extra):
        nodes = _nodes(n, erased)
        rng.shuffle(nodes)
        out.zero_()
        chunk.restore_device(k, nodes, [reps[r].data_ptr() for r in nodes], L, L, size % (2 * k), count, out, stride)
        torch.cuda.synchronize()
        assert _path(k, nodes, L, size % (2 * k), count) == 4, erased
        for o in range(count):
            assert torch.equal(out[o, :size], t[o * stride:o * stride + size]), (erased, o)
        assert int(out[:, size:].sum().item()) == 0


@pytest.mark.gpu
@pytest.mark.parametrize("k,n", [(16, 20), (32, 40)])
def test_jit_restore_non_codewords_vs_oracle(jit_sync, k, n):
    """Survivors that are not one codeword: the compiled kernel must give
    V_S^{-1} applied to them, as the reference's chunk_restore does."""
    import torch
    from vds_amd import chunk
    rng = np.random.default_rng(77 + k)
    for erased in _sets(k, n, rng, 1)[:4 if k == 16 else 2]:
        tiles = int(rng.integers(1, 3))
        size = tiles * 2048 * 2 * k + int(rng.integers(1, 2 * k * 7))
        L = chunk.replica_size(k, size)
        nodes = _nodes(n, erased)
        rng.shuffle(nodes)
        pad = size % (2 * k)
        host = [rng.integers(0, 256, L, dtype=np.uint8) for _ in nodes]
        for c in host:
            c[-2], c[-1] = pad >> 8, pad & 0xFF
        ref = O.restore(k, nodes, host)
        dev = torch.from_numpy(np.stack(host)).cuda()
        out = torch.zeros(len(ref) + 64, dtype=torch.uint8, device="cuda")
        chunk.restore_device(k, nodes, [dev[j].data_ptr() for j in range(k)], L, 0, pad, 1, out, 0)
        torch.cuda.synchronize()
        assert _path(k, nodes, L, pad) == 4
        assert np.array_equal(out[:len(ref)].cpu().numpy(), ref), erased
        assert int(out[len(ref):].sum().item()) == 0


@pytest.mark.gpu
def test_jit_background_mode_switches_after_second_use(gpu):
    """Default mode: a set's first use runs k_restore_syn; its second queues
    the compile; after vds_ec_jit_wait the set runs its own kernel."""
    import torch
    from vds_amd import chunk
    k, n = 16, 20
    size = 2048 * 2 * k
    L = chunk.replica_size(k, size)
    t = torch.empty(size, dtype=torch.uint8, device="cuda")
    chunk.fill_splitmix_device(t, size, SEED + 3200)
    reps = torch.zeros((n, 1, L), dtype=torch.uint8, device="cuda")
    chunk.encode_device(k, list(range(n)), t, size, size, 1, [reps[i].data_ptr() for i in range(n)], L)
    nodes = _nodes(n, (1, 6, 11, 19))
    out = torch.zeros(size, dtype=torch.uint8, device="cuda")
    chunk.jit_set_mode(1)
    try:
        for use in range(3):
            out.zero_()
            chunk.restore_device(k, nodes, [reps[r].data_ptr() for r in nodes], L, L, 0, 1, out, size)
            torch.cuda.synchronize()
            assert torch.equal(out, t), use
            if use == 1:
                chunk.jit_wait()
                assert chunk.jit_ready(k, nodes)
        assert _path(k, nodes, L) == 4
    finally:
        chunk.jit_set_mode(0)


def _path_regen(k, nodes, targets, L):
    from vds_amd import _lib
    nd = np.array(nodes, dtype=np.uint16)
    tg = np.array(targets, dtype=np.uint16)
    return _lib.lib().vds_ec_regenerate16_path(k, nd.ctypes.data_as(_lib.u16p), tg.ctypes.data_as(_lib.u16p),
                                               len(targets), L)


@pytest.mark.gpu
@pytest.mark.parametrize("k,erased,targets,T", [
    (16, (0, 5, 10, 15), [15, 0], 2 * 2048 + 3),
    (16, (1, 2, 17, 19), [2, 17, 19], 2048),          # targets beyond k (no interpolation point)
    (32, (0, 5, 10, 15, 20, 25, 30, 35), [35, 0, 20], 2048 * 2 + 1),
])
@pytest.mark.parametrize("codeword", [True, False])
def test_jit_regenerate_vs_oracle(jit_sync, k, erased, targets, T, codeword):
    """The regenerate kernel compiled for the survivor set (targets: every
    erased point) against the oracle's restore -> re-encode route, codewords
    and random survivors (trailer only on the first), two objects at a stride."""
    import torch
    from vds_amd import chunk
    n = k + k // 4
    nodes = _nodes(n, erased)
    rng = np.random.default_rng(T + k + codeword)
    L = 2 * T + 2
    p = (2 * k - 3) if not codeword else 0
    objs = []
    for o in range(2):
        if codeword:
            d = O.splitmix(SEED + 3300 + o, 2 * k * T)
            objs.append([O.encode(k, r, d) for r in nodes])
        else:
            sv = [rng.integers(0, 256, L, dtype=np.uint8) for _ in nodes]
            sv[0][-2], sv[0][-1] = p >> 8, p & 0xFF
            objs.append(sv)
    stride = L + 4
    host = np.zeros((k, 2, stride), dtype=np.uint8)
    for o, sv in enumerate(objs):
        for j, b in enumerate(sv):
            host[j, o, :L] = b
    dev = torch.from_numpy(host).cuda()
    ostride = L + 8
    outs = torch.full((len(targets), 2, ostride), 0x5A, dtype=torch.uint8, device="cuda")
    chunk.regenerate_device(k, nodes, [dev[j].data_ptr() for j in range(k)], L, stride, 2, targets,
                            [outs[i].data_ptr() for i in range(len(targets))], ostride)
    torch.cuda.synchronize()
    assert _path_regen(k, nodes, targets, L) == 4
    got = outs.cpu().numpy()
    for o in range(2):
        rest = O.restore(k, nodes, objs[o])
        for i, t in enumerate(targets):
            want = O.encode(k, t, rest)
            assert np.array_equal(got[i, o, :L], want), (o, t)
            assert (got[i, o, L:] == 0x5A).all()
