"""Per-phase cycle breakdown of k_restore_syn from the VDS_DIAG_STAMPS build.

  python -c "from vds_amd import build as b; b.build(out='ab/stamps/libvds_ec.so', defines=('-DVDS_DIAG_STAMPS=1',))"
  VDS_EC_LIB=ab/stamps/libvds_ec.so python tools/syn_stamps.py [--objects 128] [--k 32] [--jit]

--jit: the survivor set's run-time compiled kernel (compiled synchronously,
stamps read from its own module) instead of the syndrome kernel.

Each wave sums s_memtime deltas per phase over its tiles; this prints the
mean per tile of every phase, per wave and overall (barrier phases are the
time a wave waits for the slowest one).
"""
import argparse
import ctypes as C
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from vds_amd import _lib, chunk  # noqa: E402

PHASES = ["stage1 transposes+puts", "B1", "syndrome+load issue", "recovery walk", "B2", "ds_xor scatter", "B3",
          "stage A", "B(stage A)", "stage B programs", "B(Q read)", "P0/P1 puts", "B(P put)", "stage C",
          "B(stage C read)", "staging transposes+writes", "B(staging)", "copy-out stores", "B(tile end)", "-"]
NPH = 24

p = argparse.ArgumentParser()
p.add_argument("--objects", type=int, default=128)
p.add_argument("--k", type=int, default=16, choices=(16, 32))
p.add_argument("--jit", action="store_true")
a = p.parse_args()
if a.jit:  # phases of the fill + two-level interpolation kernel (restore_syn.hpp marks)
    PHASES = ["stage1 transposes+puts", "B1", "-", "-", "-", "scatter fill", "B(fill)", "S1 (levels 1-2)", "B(S1)",
              "S2 (families)", "B(S2)", "S3 + puts", "B(S3)", "stage C", "B(stage C read) + late loads",
              "staging transposes+writes", "B(staging)", "copy-out stores", "B(tile end)", "-"]
k, n, size = a.k, a.k + a.k // 4, 64 << 20
WV = 4 if k == 16 else 8
L = chunk.replica_size(k, size)
inp = torch.empty(a.objects * size, dtype=torch.uint8, device="cuda")
reps = torch.empty((n, a.objects * L), dtype=torch.uint8, device="cuda")
out = torch.empty(a.objects * size, dtype=torch.uint8, device="cuda")
for i in range(a.objects):
    chunk.fill_splitmix_device(inp[i * size:], size, 0x7664730000000000 + i)
nodes = [r for r in range(n) if r % 5 != 0 or r >= 5 * (n - k)][:k]
chunk.encode_device(k, list(range(n)), inp, size, size, a.objects, [reps[i].data_ptr() for i in range(n)], L)
cp = [reps[r].data_ptr() for r in nodes]
chunk.jit_set_mode(2 if a.jit else 0)
for _ in range(2):
    chunk.restore_device(k, nodes, cp, L, L, size % (2 * k), a.objects, out, size)
torch.cuda.synchronize()
lib = _lib.lib()
buf = np.zeros(4096 * 4 * NPH, dtype=np.uint64)
if a.jit:
    nd = np.asarray(nodes, dtype=np.uint16)
    rc = lib.vds_ec_diag_jit_stamps(C.c_uint16(k), nd.ctypes.data_as(C.POINTER(C.c_uint16)),
                                    buf.ctypes.data_as(C.POINTER(C.c_ulonglong)), C.c_size_t(buf.size))
else:
    rc = lib.vds_ec_diag_stamps(buf.ctypes.data_as(C.POINTER(C.c_ulonglong)), C.c_size_t(buf.size))
assert rc == 0, rc
grid = 512 if k == 16 else 256
total_tiles = a.objects * size // (2048 * 2 * k)
per_block = total_tiles / grid
st = buf[: grid * WV * NPH].reshape(grid, WV, NPH).astype(np.float64) / per_block
tot = st[:, :, :19].sum(axis=2).mean()
print(f"{total_tiles} tiles, {per_block:.1f} per block; mean s_memtime ticks per tile: {tot:.0f}")
print(f"{'phase':28s} " + " ".join(f"{'w%d' % w:>8s}" for w in range(WV)) + f" {'mean':>8s} {'%':>6s}")
for ph in range(19):
    col = st[:, :, ph].mean(axis=0)
    print(f"{PHASES[ph]:28s} " + " ".join(f"{c:8.0f}" for c in col) + f" {col.mean():8.0f} {100 * col.mean() / tot:6.1f}")

# Phase coherence across CUs (slots 20..23: s_memrealtime, the chip-global
# 100 MHz clock, at wave 0's survivor-load issue of its tiles 4, 64, 160, 240).
# Each workgroup's phase is its issue time modulo the median tile period; R is
# the length of the mean phase vector (1: every CU issues its loads in the
# same instant of the period, ~0: spread evenly over the period).
ITERS = [4, 64, 160, 240]
rt = buf[: grid * WV * NPH].reshape(grid, WV, NPH)[:, 0, 20:24].astype(np.int64)
ok = [j for j in range(4) if ITERS[j] < per_block and (rt[:, j] > 0).all()]
if len(ok) >= 2:
    j0, j1 = ok[0], ok[-1]
    period = np.median((rt[:, j1] - rt[:, j0]) / (ITERS[j1] - ITERS[j0]))
    print(f"\nload-issue phase across {grid} workgroups (tile period {period * 10:.0f} ns, median):")
    odd = ((np.arange(grid) >> 3) & 1).astype(bool)
    for j in ok:
        ph = ((rt[:, j] - np.median(rt[:, j])) / period) % 1.0
        vec = np.exp(2j * np.pi * ph)
        hist = np.histogram(ph, bins=8, range=(0, 1))[0]
        print(f"  tile {ITERS[j]:4d}: R = {abs(vec.mean()):.3f}  (even half {abs(vec[~odd].mean()):.3f}, odd half "
              f"{abs(vec[odd].mean()):.3f}, odd-even offset {np.angle(vec[odd].mean() / vec[~odd].mean()) / (2 * np.pi):+.2f}"
              f" period)  phase histogram (8 bins) {hist.tolist()}")
