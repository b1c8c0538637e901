"""Study: does the placement of the replica buffers relative to each other
change the encode / repair rate?  One process, one allocation; the n replica
buffers start `skew` bytes beyond the packed spacing (objects x stride), for
several skews, interleaved, at the bench shape (k=16, m=4, 64 MiB objects,
the bench's 256-byte-padded replica stride).  Run it in several processes:
the bench's encode moves between ~13.1 and ~14.9 ms (512 objects) from one
process to the next on some boxes.

  python tools/ubench/skew.py [--objects 512] [--skews 0 4096 ...] [--rounds 2]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))))
import torch  # noqa: E402

import bench  # noqa: E402
from vds_amd import chunk  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--objects", type=int, default=512)
p.add_argument("--skews", type=int, nargs="*", default=[0, 4096, 65536, 1 << 20, (1 << 20) + 4096 * 5, 2 << 20])
p.add_argument("--rounds", type=int, default=2)
p.add_argument("--iters", type=int, default=5)
a = p.parse_args()
k, m, size = 16, 4, 64 << 20
n = k + m
L = chunk.replica_size(k, size)
Ls = bench.replica_stride(L, 256)
span = a.objects * Ls
inp = torch.empty(a.objects * size, dtype=torch.uint8, device="cuda")
for i in range(a.objects):
    chunk.fill_splitmix_device(inp[i * size:], size, 0x7664730000000000 + i)
area = torch.empty(n * (span + max(a.skews)) + 4096, dtype=torch.uint8, device="cuda")
out = torch.empty(a.objects * size, dtype=torch.uint8, device="cuda")
base = area.data_ptr()
nodes = [r for r in range(n) if r % 5]
res = {s: {"encode": [], "repair": []} for s in a.skews}
for rnd in range(a.rounds):
    for s in (a.skews if rnd % 2 == 0 else a.skews[::-1]):
        rp = [base + r * (span + s) for r in range(n)]
        enc = lambda: chunk.encode_device(k, list(range(n)), inp, size, size, a.objects, rp, Ls)  # noqa: E731
        cp = [rp[r] for r in nodes]
        rep = lambda: chunk.restore_device(k, nodes, cp, L, Ls, size % (2 * k), a.objects, out, size)  # noqa: E731
        enc(); rep(); rep()  # noqa: E702
        chunk.jit_wait()
        rep()
        torch.cuda.synchronize()
        for name, f in (("encode", enc), ("repair", rep)):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                f()
            e1.record()
            torch.cuda.synchronize()
            res[s][name].append(round(e0.elapsed_time(e1) / a.iters, 3))
print(json.dumps({"objects": a.objects, "span": span, "ms": {str(s): v for s, v in res.items()}}))
