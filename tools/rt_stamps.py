"""Per-phase stamps of the RT batch kernel (k = 32, n = 64 live shape) from a
VDS_DIAG_STAMPS build: only the objects the RT route takes (some survivor
beyond point 39), so no other stamping kernel runs.

  python -c "from vds_amd import build as b; b.build(out='ab/stamps/libvds_ec.so', defines=('-DVDS_DIAG_STAMPS=1',))"
  VDS_EC_LIB=ab/stamps/libvds_ec.so python tools/rt_stamps.py [--loss 0.25] [--objects 16384]

Phases (restore_syn.hpp marks): stage 1, its barrier, RT2 (a) borrowed
survivors into slots K.., (b) PERM evaluations of P0, (b)'s barrier,
(c) runtime products, (d) + the phase-2 barrier, the interpolation stages,
staging, copy-out."""
import argparse
import ctypes as C
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from vds_amd import _lib, chunk  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--objects", type=int, default=16384)
p.add_argument("--loss", type=float, default=0.25)
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
rt = nodes.max(axis=1) >= k + k // 4
objs, nodes = objs[rt], np.ascontiguousarray(nodes[rt])
base = np.asarray([reps[i].data_ptr() for i in range(n)], dtype=np.uint64)
cp = (base[nodes] + (objs.astype(np.uint64) * Ls)[:, None]).astype(np.uint64)
sizes = np.full(len(objs), L, dtype=np.uint64)
pads = np.zeros(len(objs), dtype=np.uint16)
outs = (np.uint64(out.data_ptr()) + objs.astype(np.uint64) * size).astype(np.uint64)
erased_below_k = np.array([k - np.count_nonzero(nd < k) for nd in nodes])
lib = _lib.lib()
s = torch.cuda.current_stream().cuda_stream
for _ in range(3):
    _lib.check(lib.vds_ec_restore16_batch_device(k, len(objs), nodes.ctypes.data_as(_lib.u16p), cp.ctypes.data_as(_lib.vpp),
                                                 sizes.ctypes.data_as(_lib.u64p), pads.ctypes.data_as(_lib.u16p),
                                                 outs.ctypes.data_as(_lib.vpp), 0, s))
torch.cuda.synchronize()
NPH = 24
buf = np.zeros(4096 * 4 * NPH, dtype=np.uint64)
rc = lib.vds_ec_diag_stamps(buf.ctypes.data_as(C.POINTER(C.c_ulonglong)), C.c_size_t(buf.size))
assert rc == 0, rc
st = buf.reshape(-1, NPH)[: 256 * 8].reshape(256, 8, NPH).astype(np.float64)
tiles = (len(objs) + 1) // 2 / 256  # tiles per workgroup (two objects per tile)
names = {0: "stage 1", 1: "B(stage 1)", 2: "RT2 (a) borrowed -> slots", 3: "RT2 (b) PERM evaluations", 4: "B(b)",
         19: "RT2 (c) runtime products", 5: "(d) + scatter", 6: "B(phase 2)", 7: "S1", 8: "B(S1)", 9: "S2", 10: "B(S2)",
         11: "S3", 12: "B(S3)", 13: "stage C", 14: "B(stage C) + late loads", 15: "staging", 16: "B(staging)",
         17: "copy-out", 18: "B(tile end)"}
tot = st[:, :, :20].sum(axis=2).mean() / tiles
print(f"RT objects {len(objs)} (erased below k: mean {erased_below_k.mean():.2f}, max {erased_below_k.max()}); "
      f"~{tiles:.1f} tiles per workgroup; mean ticks per tile {tot:.0f}")
print(f"{'phase':32s}" + "".join(f"{'w' + str(w):>8s}" for w in range(8)) + f"{'mean':>9s}{'%':>7s}")
for ph in (0, 1, 2, 3, 4, 19, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18):
    per_w = st[:, :, ph].mean(axis=0) / tiles
    print(f"{names[ph]:32s}" + "".join(f"{x:8.0f}" for x in per_w) + f"{per_w.mean():9.0f}{100 * per_w.mean() / tot:7.1f}")
