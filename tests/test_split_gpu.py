"""One object split by stripe range (SURVEY.md 8(e) bullet 2): ranges encoded
or restored separately equal the whole-object result and the oracle
(chunk.h:245-281 encode, chunk.h:402-444 restore); the multi-GPU host split
run with several ranges on the one GPU of the test box."""
import numpy as np
import pytest

import oracle_ctypes as O

pytestmark = pytest.mark.gpu
SEED = 0x5350_4C49_5400


def _ranges(T, cuts):
    edges = sorted({0, T, *[c for c in cuts if 0 < c < T]})
    return list(zip(edges[:-1], edges[1:])) or [(0, 0)]


@pytest.mark.parametrize("k,n,size,cuts", [
    (16, 20, 0, []),
    (16, 20, 1, []),
    (16, 20, 32 * 4096 + 17, [1, 2048, 3000]),
    (16, 20, 32 * 8192, [2048, 4096, 6144]),
    (32, 64, 65536, [512, 1000]),
    (4, 6, 1000, [7, 100]),
])
def test_encode_ranges_equal_whole(gpu, k, n, size, cuts):
    import torch
    from vds_amd import chunk
    host = O.splitmix(SEED + size, size)
    inp = torch.from_numpy(host.copy()).cuda() if size else torch.zeros(1, dtype=torch.uint8, device="cuda")
    L = chunk.replica_size(k, size)
    T = (size + 2 * k - 1) // (2 * k)
    outs = [torch.full((L + 4,), 0x33, dtype=torch.uint8, device="cuda") for _ in range(n)]
    for t0, t1 in _ranges(T, cuts):
        chunk.encode_range_device(k, list(range(n)), inp, size, t0, t1, [o.data_ptr() for o in outs])
    torch.cuda.synchronize()
    for r in (0, 1, k - 1, k, n - 1):
        got = outs[r].cpu().numpy()
        assert np.array_equal(got[:L], O.encode(k, r, host)), (r, size)
        assert (got[L:] == 0x33).all()


@pytest.mark.parametrize("k,n,size,cuts", [
    (16, 20, 32 * 4096 + 17, [2048, 3000]),
    (16, 20, 32 * 2048 * 3, [2048, 4096]),
    (32, 40, 64 * 4096 + 64 * 3 + 5, [1, 2048]),
    (32, 64, 65536, [300]),
])
def test_restore_ranges_equal_whole(gpu, k, n, size, cuts):
    import torch
    from vds_amd import chunk
    host = O.splitmix(SEED + 7 + size, size)
    rng = np.random.default_rng(size)
    nodes = sorted(rng.choice(n, k, replace=False).tolist())
    reps = {r: torch.from_numpy(O.encode(k, r, host)).cuda() for r in nodes}
    L = reps[nodes[0]].numel()
    out = torch.full((size + 64,), 0x77, dtype=torch.uint8, device="cuda")
    nst = (size + 2 * k - 1) // (2 * k)
    for t0, t1 in _ranges(nst, cuts):
        chunk.restore_range_device(k, nodes, [reps[r].data_ptr() for r in nodes], L, size % (2 * k), t0, t1, out)
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    assert np.array_equal(got[:size], host)
    assert (got[size:] == 0x77).all()


@pytest.mark.parametrize("k,n,size,parts", [(16, 20, 32 * 2048 * 5 + 3, 3), (16, 20, 100, 4), (32, 64, 65536, 2),
                                            (16, 20, 0, 2)])
def test_host_split_several_ranges_on_one_gpu(gpu, k, n, size, parts):
    from vds_amd import chunk
    host = O.splitmix(SEED + 99 + size, size)
    reps = chunk.encode_host_split(k, list(range(n)), host, parts=parts)
    for r in (0, k - 1, n - 1):
        assert np.array_equal(reps[r], O.encode(k, r, host)), r
    nodes = list(range(n - k, n))
    got = chunk.restore_host_split(k, nodes, [reps[r] for r in nodes], parts=parts)
    assert np.array_equal(got, host)


def test_range_arguments_rejected(gpu):
    import torch
    from vds_amd import chunk
    from vds_amd._lib import VdsEcError, EINVAL
    k, size = 16, 32 * 100
    inp = torch.zeros(size, dtype=torch.uint8, device="cuda")
    outs = [torch.zeros(chunk.replica_size(k, size), dtype=torch.uint8, device="cuda") for _ in range(20)]
    for t0, t1 in ((5, 4), (0, 101), (3, 3)):
        with pytest.raises(VdsEcError) as e:
            chunk.encode_range_device(k, list(range(20)), inp, size, t0, t1, [o.data_ptr() for o in outs])
        assert e.value.status == EINVAL
