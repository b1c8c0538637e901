"""Study: encode and repair of different object batches on two streams at
once (batch b's repair waits for batch b's encode) against the sequential
step, at the bench shape (k=16, m=4, 64 MiB objects).

  python tools/ubench/overlap.py [--objects 512] [--batches 4 8 16]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))))
import torch  # noqa: E402

from vds_amd import chunk  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--objects", type=int, default=512)
p.add_argument("--batches", type=int, nargs="*", default=[4, 8, 16])
p.add_argument("--reps", type=int, default=3)
a = p.parse_args()
k, m, n, size = 16, 4, 20, 64 << 20
dev = torch.device("cuda:0")
L = chunk.replica_size(k, size)
O = a.objects
inp = torch.empty(O * size, dtype=torch.uint8, device=dev)
reps = torch.empty((n, O * L), dtype=torch.uint8, device=dev)
out = torch.empty(O * size, dtype=torch.uint8, device=dev)
for i in range(O):
    chunk.fill_splitmix_device(inp[i * size:], size, 0x7664730000000000 + i)
erased = [0, 5, 10, 15]
nodes = [r for r in range(n) if r not in erased][:k]
padding = size % (2 * k)
sA, sB = torch.cuda.Stream(dev), torch.cuda.Stream(dev)


def enc(o0, cnt, s):
    chunk.encode_device(k, list(range(n)), inp[o0 * size:], size, size, cnt,
                        [reps[i].data_ptr() + o0 * L for i in range(n)], L, stream=s)


def rep(o0, cnt, s):
    chunk.restore_device(k, nodes, [reps[r].data_ptr() + o0 * L for r in nodes], L, L, padding, cnt,
                         out[o0 * size:], size, stream=s)


def sequential():
    enc(0, O, sA)
    rep(0, O, sA)


def pipelined(B):
    bs = O // B
    evs = [torch.cuda.Event() for _ in range(B)]
    for b in range(B):
        enc(b * bs, bs, sA)
        evs[b].record(sA)
        sB.wait_event(evs[b])
        rep(b * bs, bs, sB)
    sA.wait_stream(sB)


def timeit(f):
    torch.cuda.synchronize()
    f()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(a.reps):
        t = time.perf_counter()
        f()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t)
    return best


gib = O * size / 2**30
t = timeit(sequential)
print(f"sequential: {t*1e3:.2f} ms  {gib/t:.1f} GiB/s", flush=True)
for B in a.batches:
    out.zero_()
    t = timeit(lambda: pipelined(B))
    ok = torch.equal(out, inp)
    print(f"pipelined B={B}: {t*1e3:.2f} ms  {gib/t:.1f} GiB/s  ok={ok}", flush=True)
