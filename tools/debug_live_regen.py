"""Debug: the live shape's batched regenerate (k=32, n=64, 64 KiB objects,
first 32 found at loss p) against the encoded replicas; prints the failing
objects' survivor sets and targets by route class."""
import os
import sys
import numpy as np
import torch

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
from vds_amd import chunk, _lib  # noqa: E402

objects = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
loss = float(sys.argv[2]) if len(sys.argv) > 2 else 0.02
k, n, size = 32, 64, 65536
L = chunk.replica_size(k, size)
Ls = -(-L // 256) * 256
dev = torch.device("cuda", 0)
inp = torch.empty(objects * size, dtype=torch.uint8, device=dev)
chunk.fill_splitmix_device(inp, objects * size, 12345)
reps = torch.empty((n, objects * Ls), dtype=torch.uint8, device=dev)
rep_ptrs = [reps[i].data_ptr() for i in range(n)]
chunk.encode_device(k, list(range(n)), inp, size, size, objects, rep_ptrs, Ls)
rng = np.random.default_rng(1)
lost = rng.random((objects, n)) < loss
objs = np.flatnonzero((~lost).sum(axis=1) >= k)
nodes = np.stack([np.flatnonzero(~lost[o])[:k] for o in objs]).astype(np.uint16)
base = np.asarray(rep_ptrs, dtype=np.uint64)
chunk_ptrs = (base[nodes] + (objs.astype(np.uint64) * Ls)[:, None]).astype(np.uint64)
rg = np.flatnonzero(lost[objs].any(axis=1))
tg = np.argmax(lost[objs[rg]], axis=1).astype(np.uint16)
out = torch.zeros(max(1, len(rg)) * Ls, dtype=torch.uint8, device=dev)
outs = (np.uint64(out.data_ptr()) + np.arange(len(rg), dtype=np.uint64) * Ls).astype(np.uint64)
rn = np.ascontiguousarray(nodes[rg])
rc = np.ascontiguousarray(chunk_ptrs[rg])
sz = np.full(len(rg), L, dtype=np.uint64)
lib = _lib.lib()
_lib.check(lib.vds_ec_regenerate16_batch_device(k, len(rg), rn.ctypes.data_as(_lib.u16p), rc.ctypes.data_as(_lib.vpp),
                                                sz.ctypes.data_as(_lib.u64p), 1, tg.ctypes.data_as(_lib.u16p),
                                                outs.ctypes.data_as(_lib.vpp), None))
torch.cuda.synchronize()
reps2d = reps.view(n, objects, Ls)
want = reps2d[torch.from_numpy(tg.astype(np.int64)).to(dev), torch.from_numpy(objs[rg]).to(dev), :L]
got = out.view(-1, Ls)[:len(rg), :L]
bad = (got != want).any(dim=1).cpu().numpy()
print("objects", len(rg), "bad", int(bad.sum()))


def cls(nd, t):
    mx = int(nd.max())
    if mx < k and t >= k:
        return "perm"
    if max(mx, t) < k + 1:
        return "small1"
    if max(mx, t) < k + 2:
        return "small2"
    if max(mx, t) < 40:
        return "syn40"
    return "rt"


from collections import Counter  # noqa: E402
print("classes all", Counter(cls(rn[i], int(tg[i])) for i in range(len(rg))))
print("classes bad", Counter(cls(rn[i], int(tg[i])) for i in np.flatnonzero(bad)))
for i in np.flatnonzero(bad)[:8]:
    g = got[i].cpu().numpy()
    w = want[i].cpu().numpy()
    d = np.flatnonzero(g != w)
    print("obj", int(objs[rg[i]]), "target", int(tg[i]), "maxid", int(rn[i].max()),
          "erased<32", [int(x) for x in range(32) if x not in set(rn[i].tolist())],
          "ndiff", len(d), "first", int(d[0]), "last", int(d[-1]))
