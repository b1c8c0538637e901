"""Host planning cost of the live shape's batched restore / regenerate
(a library built with -DVDS_HOST_TRACE=1 prints each call's phases to stderr).
  python -c "from vds_amd import build as b; b.build(out='ab/trace/libvds_ec.so', defines=('-DVDS_HOST_TRACE=1',))"
  VDS_EC_LIB=ab/trace/libvds_ec.so python tools/host_trace.py [--loss 0.02] [--objects 16384]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from vds_amd import _lib, chunk  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--objects", type=int, default=16384)
p.add_argument("--loss", type=float, default=0.02)
a = p.parse_args()
k, n, size = 32, 64, 65536
L = chunk.replica_size(k, size)
Ls = -(-L // 256) * 256
dev = torch.device("cuda", 0)
reps = torch.zeros((n, a.objects * Ls), dtype=torch.uint8, device=dev)
out = torch.empty(a.objects * size, dtype=torch.uint8, device=dev)
rng = np.random.default_rng(1)
lost = rng.random((a.objects, n)) < a.loss
objs = np.flatnonzero((~lost).sum(axis=1) >= k)
nodes = np.stack([np.flatnonzero(~lost[o])[:k] for o in objs]).astype(np.uint16)
base = np.asarray([reps[i].data_ptr() for i in range(n)], dtype=np.uint64)
cp = (base[nodes] + (objs.astype(np.uint64) * Ls)[:, None]).astype(np.uint64)
sizes = np.full(len(objs), L, dtype=np.uint64)
pads = np.zeros(len(objs), dtype=np.uint16)
outs = (np.uint64(out.data_ptr()) + objs.astype(np.uint64) * size).astype(np.uint64)
rg = np.flatnonzero(lost[objs].any(axis=1))
tg = np.argmax(lost[objs[rg]], axis=1).astype(np.uint16)
rgo = torch.empty(max(1, len(rg)) * Ls, dtype=torch.uint8, device=dev)
rgp = (np.uint64(rgo.data_ptr()) + np.arange(len(rg), dtype=np.uint64) * Ls).astype(np.uint64)
rn, rc = np.ascontiguousarray(nodes[rg]), np.ascontiguousarray(cp[rg])
rs = np.full(len(rg), L, dtype=np.uint64)
lib = _lib.lib()
s = torch.cuda.current_stream().cuda_stream


def restore():
    _lib.check(lib.vds_ec_restore16_batch_device(k, len(objs), nodes.ctypes.data_as(_lib.u16p), cp.ctypes.data_as(_lib.vpp),
                                                 sizes.ctypes.data_as(_lib.u64p), pads.ctypes.data_as(_lib.u16p),
                                                 outs.ctypes.data_as(_lib.vpp), 0, s))


def regen():
    _lib.check(lib.vds_ec_regenerate16_batch_device(k, len(rg), rn.ctypes.data_as(_lib.u16p), rc.ctypes.data_as(_lib.vpp),
                                                    rs.ctypes.data_as(_lib.u64p), 1, tg.ctypes.data_as(_lib.u16p),
                                                    rgp.ctypes.data_as(_lib.vpp), s))


for name, fn in (("restore", restore), ("regenerate", regen)):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(6):
        t0 = time.perf_counter()
        fn()
        ts.append((time.perf_counter() - t0) * 1e3)
        torch.cuda.synchronize()
    print(name, "host ms", [round(t, 3) for t in ts], flush=True)
