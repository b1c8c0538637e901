"""RT batch restore at the live shape with a fixed number of erased points
below k per object (every object on the RT route): GPU time per call and a
check of every restored object against the encoded input.  Run with the
default library and with a -DVDS_BATCH_RT2=0 build (VDS_EC_LIB=...) for the
RT2 rows A/B.
  python tools/rt2_bench.py [--objects 16384] [--rows 8] [--steps 10]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from vds_amd import _lib, chunk  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--objects", type=int, default=16384)
p.add_argument("--rows", type=int, default=8)
p.add_argument("--steps", type=int, default=10)
a = p.parse_args()
dev = torch.device("cuda", 0)
k, n, size, objects = 32, 64, 65536, a.objects
L = chunk.replica_size(k, size)
Ls = bench.replica_stride(L, 256)
inp = torch.empty(objects * size, dtype=torch.uint8, device=dev)
chunk.fill_splitmix_device(inp, objects * size, 0x7664730000000000 ^ 0x5254)
reps = torch.empty((n, objects * Ls), dtype=torch.uint8, device=dev)
chunk.encode_device(k, list(range(n)), inp, size, size, objects, [reps[i].data_ptr() for i in range(n)], Ls)
out = torch.empty(objects * size, dtype=torch.uint8, device=dev)
rng = np.random.default_rng(7)
nodes = np.empty((objects, k), dtype=np.uint16)
for o in range(objects):
    er = set(rng.choice(k, a.rows, replace=False).tolist())
    extra = sorted(rng.choice(np.arange(k + 8, 2 * k), a.rows, replace=False).tolist())  # beyond the syndrome points
    nodes[o] = [x for x in range(k) if x not in er] + extra
base = np.asarray([reps[i].data_ptr() for i in range(n)], dtype=np.uint64)
cp = (base[nodes] + (np.arange(objects, dtype=np.uint64) * Ls)[:, None]).astype(np.uint64)
sizes = np.full(objects, L, dtype=np.uint64)
pads = np.zeros(objects, dtype=np.uint16)
outs = (np.uint64(out.data_ptr()) + np.arange(objects, dtype=np.uint64) * size).astype(np.uint64)
lib = _lib.lib()
st = torch.cuda.current_stream().cuda_stream


def call():
    _lib.check(lib.vds_ec_restore16_batch_device(k, objects, nodes.ctypes.data_as(_lib.u16p), cp.ctypes.data_as(_lib.vpp),
                                                 sizes.ctypes.data_as(_lib.u64p), pads.ctypes.data_as(_lib.u16p),
                                                 outs.ctypes.data_as(_lib.vpp), 0, st))


out.fill_(0)
call()
torch.cuda.synchronize()
assert torch.equal(out, inp), "RT restore differs from the encoded objects"
for _ in range(3):
    call()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
torch.cuda.synchronize()
e0.record()
for _ in range(a.steps):
    call()
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / a.steps
print(json.dumps({"lib": os.environ.get("VDS_EC_LIB", "default"), "rows": a.rows, "objects": objects, "ms_per_call": round(ms, 4),
                  "GiBps": round(objects * size / (ms * 1e-3) / 2**30, 2)}))

# VDS_EC_LIB = a -DVDS_DIAG_STAMPS=1 build: the per-phase ticks of the last call
if hasattr(lib, "vds_ec_diag_stamps"):
    import ctypes as C
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    NPH, WV, grid = 24, 8, 256
    buf = np.zeros(4096 * 4 * NPH, dtype=np.uint64)
    torch.cuda.synchronize()
    assert lib.vds_ec_diag_stamps(buf.ctypes.data_as(C.POINTER(C.c_ulonglong)), C.c_size_t(buf.size)) == 0
    per_block = (objects // 2) / grid
    stp = buf[: grid * WV * NPH].reshape(grid, WV, NPH).astype(np.float64) / per_block
    names = ["stage1", "B1", "phase2a", "phase2b", "B2", "phase2c", "B3", "S1", "B(S1)", "S2", "B(S2)", "S2 puts",
             "B", "stage C", "B(stage C)", "staging", "B(staging)", "copy-out", "B(tile end)"]
    tot = stp[:, :, :19].sum(axis=2).mean()
    print(f"ticks per tile {tot:.0f}")
    for ph in range(19):
        col = stp[:, :, ph].mean(axis=0)
        print(f"{names[ph]:14s} " + " ".join(f"{c:7.0f}" for c in col) + f" {col.mean():8.0f} {100 * col.mean() / tot:5.1f}%")
