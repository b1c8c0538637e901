"""The live-shape legs of bench.py alone (for rocprofv3 / quick A/B):
  python tools/live_prof.py [--objects 16384] [--loss 0.25] [--steps 10]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import bench  # noqa: E402
from vds_amd import chunk  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--objects", type=int, default=16384)
p.add_argument("--loss", type=float, nargs="+", default=[0.25])
p.add_argument("--steps", type=int, default=10)
a = p.parse_args()
dev = torch.device("cuda", 0)
r = bench.live_shape(torch, chunk, dev, torch.cuda.Stream(dev), a.objects, a.steps, 3, losses=tuple(a.loss))
print(json.dumps(r))

# host-side enqueue cost of the batched calls (planning + staging), p = last loss rate
import time  # noqa: E402
import numpy as np  # noqa: E402
from vds_amd import _lib  # noqa: E402

k, n, size, objects = 32, 64, 65536, a.objects
L = chunk.replica_size(k, size)
Ls = bench.replica_stride(L, 256)
reps = torch.zeros((n, objects * Ls), dtype=torch.uint8, device=dev)
out = torch.empty(objects * size, dtype=torch.uint8, device=dev)
rng = np.random.default_rng(1)
lost = rng.random((objects, n)) < a.loss[-1]
objs = np.flatnonzero((~lost).sum(axis=1) >= k)
nodes = np.stack([np.flatnonzero(~lost[o])[:k] for o in objs]).astype(np.uint16)
base = np.asarray([reps[i].data_ptr() for i in range(n)], dtype=np.uint64)
cp = (base[nodes] + (objs.astype(np.uint64) * Ls)[:, None]).astype(np.uint64)
sizes = np.full(len(objs), L, dtype=np.uint64)
pads = np.zeros(len(objs), dtype=np.uint16)
outs = (np.uint64(out.data_ptr()) + objs.astype(np.uint64) * size).astype(np.uint64)
lib = _lib.lib()
s = torch.cuda.current_stream().cuda_stream
def call():
    _lib.check(lib.vds_ec_restore16_batch_device(k, len(objs), nodes.ctypes.data_as(_lib.u16p), cp.ctypes.data_as(_lib.vpp),
               sizes.ctypes.data_as(_lib.u64p), pads.ctypes.data_as(_lib.u16p), outs.ctypes.data_as(_lib.vpp), 0, s))
for _ in range(3):
    call()
torch.cuda.synchronize()
ts = []
for _ in range(10):
    t0 = time.perf_counter(); call(); ts.append(time.perf_counter() - t0)
    torch.cuda.synchronize()
print(json.dumps({"host_enqueue_ms": [round(t * 1e3, 3) for t in ts], "objects": int(len(objs))}))
