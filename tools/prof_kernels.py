"""Run the fast encode and restore kernels on a resident batch (for rocprofv3).

  python tools/prof_kernels.py [--k 16] [--m 4] [--objects 64] [--iters 3] [--only encode|restore]
"""
import argparse
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from vds_amd import chunk  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--k", type=int, default=16)
p.add_argument("--m", type=int, default=4)
p.add_argument("--objects", type=int, default=64)
p.add_argument("--iters", type=int, default=3)
p.add_argument("--only", default="")
p.add_argument("--replica-align", type=int, default=256, help="replica stride alignment (bench.py's default)")
p.add_argument("--no-jit", action="store_true", help="repair on k_restore_syn (no survivor-set kernel)")
a = p.parse_args()
if a.no_jit:
    chunk.jit_set_mode(0)
k, n = a.k, a.k + a.m
size = 64 << 20
L = chunk.replica_size(k, size)
Ls = -(-L // a.replica_align) * a.replica_align
inp = torch.empty(a.objects * size, dtype=torch.uint8, device="cuda")
reps = torch.empty((n, a.objects * Ls), dtype=torch.uint8, device="cuda")
out = torch.empty(a.objects * size, dtype=torch.uint8, device="cuda")
for i in range(a.objects):
    chunk.fill_splitmix_device(inp[i * size:], size, 0x7664730000000000 + i)
erased = list(range(0, n, n // a.m))[: a.m]
nodes = [r for r in range(n) if r not in erased]
rp = [reps[i].data_ptr() for i in range(n)]
chunk.encode_device(k, list(range(n)), inp, size, size, a.objects, rp, Ls)
if a.only != "encode" and not a.no_jit:  # the survivor set's own kernel, as bench.py measures it
    for _ in range(2):
        chunk.restore_device(k, nodes, [reps[r].data_ptr() for r in nodes], L, Ls, size % (2 * k), a.objects, out, size)
    chunk.jit_wait()
for _ in range(a.iters):
    if a.only != "restore":
        chunk.encode_device(k, list(range(n)), inp, size, size, a.objects, rp, Ls)
    if a.only != "encode":
        chunk.restore_device(k, nodes, [reps[r].data_ptr() for r in nodes], L, Ls, size % (2 * k), a.objects, out, size)
torch.cuda.synchronize()
assert torch.equal(out[:size], inp[:size]) or a.only == "encode"
print("ok", k, n, a.objects)
