"""Live-shape encode alone (k=32, n=64, 16384 x 64 KiB, replica stride 2304),
HIP-event time per call: python tools/ab_live_encode.py [--iters 20]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from vds_amd import chunk  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--iters", type=int, default=20)
p.add_argument("--objects", type=int, default=16384)
a = p.parse_args()
k, n, size = 32, 64, 65536
L = chunk.replica_size(k, size)
Ls = -(-L // 256) * 256
inp = torch.empty(a.objects * size, dtype=torch.uint8, device="cuda")
chunk.fill_splitmix_device(inp, a.objects * size, 99)
reps = torch.empty((n, a.objects * Ls), dtype=torch.uint8, device="cuda")
rp = [reps[i].data_ptr() for i in range(n)]
enc = lambda: chunk.encode_device(k, list(range(n)), inp, size, size, a.objects, rp, Ls)  # noqa: E731
for _ in range(3):
    enc()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(a.iters):
    enc()
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / a.iters
ok = bool(torch.equal(reps[5].view(a.objects, Ls)[7, L - 2:L].cpu(), torch.zeros(2, dtype=torch.uint8)))
print(json.dumps({"tag": os.environ.get("VDS_EC_ENC_TRAILER", "1"), "ms": round(ms, 4),
                  "GiBps": round(a.objects * size / (ms * 1e-3) / 2**30, 2), "trailer_zero": ok}))
