"""Randomised batched restore / regenerate against the oracle (a soak of the
batch planner's routes: SMALL, PERM, the N-point syndrome class with shared
and distinct erased sets -- dual tiles at k = 32 --, RT / RT2 with borrowed
ids, the per-object fallback for ids >= 256).  Every object's survivors are
random bytes (not one codeword) with a chosen trailer, so every restored byte
and every regenerated replica is checked against the reference route
(chunk.h:402-444, then chunk.h:245-281 for a repair).  Time-bounded:
VDS_FUZZ_SECONDS (default 20) of calls; the seed is printed on failure."""
import os
import time

import numpy as np
import pytest

import oracle_ctypes as O

pytestmark = pytest.mark.gpu


def _survivors(rng, k, T, p):
    out = []
    for _ in range(k):
        b = rng.integers(0, 256, 2 * T + 2, dtype=np.uint8)
        b[-2], b[-1] = p >> 8, p & 0xFF
        out.append(b)
    return out


def _ids(rng, k, n_total, shared):
    kind = rng.integers(0, 6)
    if kind == 0 and shared:
        return list(shared[rng.integers(0, len(shared))])
    if kind == 1:  # restore_async's first k found among n_total with losses
        lost = set(rng.choice(n_total, int(rng.integers(0, n_total - k + 1)), replace=False).tolist())
        return [r for r in range(n_total) if r not in lost][:k]
    if kind == 2:  # survivors within 0..k+1 (SMALL) or exactly 0..k-1
        m = int(rng.integers(0, 3))
        return sorted(rng.choice(k + m, k, replace=False).tolist())
    if kind == 3:  # borrowed ids below 2k (RT2 at k = 32)
        e = int(rng.integers(1, min(13, k)))
        keep = sorted(rng.choice(k, k - e, replace=False).tolist())
        return keep + sorted(rng.choice(np.arange(k, 2 * k), e, replace=False).tolist())
    if kind == 4:  # any ids below 256 (RT mode 0), rarely one >= 256 (per-object path)
        hi = 300 if rng.random() < 0.1 else 256
        return sorted(rng.choice(hi, k, replace=False).tolist())
    return sorted(rng.choice(k + k // 4, k, replace=False).tolist())  # the N-point class


def test_batch_fuzz_vs_oracle(gpu):
    import torch
    from vds_amd import chunk
    seconds = float(os.environ.get("VDS_FUZZ_SECONDS", "20"))
    seed0 = int(os.environ.get("VDS_FUZZ_SEED", "20261018"))
    t_end = time.monotonic() + seconds
    t_note = time.monotonic() + 30
    it = 0
    while time.monotonic() < t_end:
        if time.monotonic() > t_note:  # (a progress line: long soaks must not look hung)
            print(f"batch fuzz: {it} calls", flush=True)
            t_note += 30
        seed = seed0 + it
        it += 1
        rng = np.random.default_rng(seed)
        k = int(rng.choice([16, 32]))
        n_total = int(rng.choice([k + k // 4, 2 * k]))
        count = int(rng.integers(1, 90))
        shared = [_ids(rng, k, n_total, None) for _ in range(3)]
        nodes, keep, chunks, csz, pads, data = [], [], [], [], [], []
        for _ in range(count):
            T = int(rng.choice([1, 7, 1023, 1024, 1025, 2048, int(rng.integers(1, 5000))]))
            p = int(rng.integers(0, 2 * k + 1))
            if p == 2 * k and T == 1:
                p = 0
            nd = _ids(rng, k, n_total, shared)
            if rng.random() < 0.3:
                nd = list(rng.permutation(nd))
            sv = _survivors(rng, k, T, p)
            bufs = [torch.from_numpy(b).cuda() for b in sv]
            keep.append(bufs)
            nodes.append([int(x) for x in nd])
            chunks.append([b.data_ptr() for b in bufs])
            csz.append(2 * T + 2)
            pads.append(p)
            data.append(sv)
        want = [O.restore(k, nd, sv) for nd, sv in zip(nodes, data)]
        outs = [torch.full((w.size + 64,), 0xA5, dtype=torch.uint8, device="cuda") for w in want]
        chunk.restore_batch_device(k, nodes, chunks, csz, pads, [o.data_ptr() for o in outs])
        nt = int(rng.integers(1, 3))
        targets = [sorted(rng.choice([r for r in range(260) if r not in nd], nt, replace=False).tolist()) for nd in nodes]
        rg = [[torch.full((c + 8,), 0x5A, dtype=torch.uint8, device="cuda") for _ in range(nt)] for c in csz]
        chunk.regenerate_batch_device(k, nodes, chunks, csz, targets, [[x.data_ptr() for x in r] for r in rg])
        torch.cuda.synchronize()
        for i in range(count):
            got = outs[i].cpu().numpy()
            w = want[i]
            assert np.array_equal(got[:w.size], w), (seed, i, k, nodes[i], csz[i], pads[i])
            assert (got[w.size:] == 0xA5).all(), (seed, i)
            for t, x in zip(targets[i], rg[i]):
                g = x.cpu().numpy()
                assert np.array_equal(g[:csz[i]], O.encode(k, t, w)), (seed, i, t, nodes[i], csz[i], pads[i])
                assert (g[csz[i]:] == 0x5A).all(), (seed, i, t)
    print(f"batch fuzz: {it} restore + regenerate calls in {seconds:.0f} s (seeds {seed0}..{seed0 + it - 1})")
    assert it > 0
