"""Time the encode and repair launches on a resident batch (no correctness
check: used for A/B of diagnostic variant builds via VDS_EC_LIB).

  python tools/time_kernels.py [--objects 128] [--iters 5] [--k 16|32] [--check]
"""
import argparse
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from vds_amd import chunk  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--objects", type=int, default=128)
p.add_argument("--iters", type=int, default=5)
p.add_argument("--tag", default=os.path.basename(os.environ.get("VDS_EC_LIB", "default")))
p.add_argument("--k", type=int, default=16, choices=(16, 32))
p.add_argument("--n", type=int, default=0, help="replicas (default k + k/4; 64 = the live shape)")
p.add_argument("--check", action="store_true", help="compare the restored objects with the input")
p.add_argument("--align", type=int, default=1, help="replica stride rounded up to this many bytes")
p.add_argument("--skew", type=int, default=0, help="extra bytes between consecutive replica buffers")
a = p.parse_args()
k, size = a.k, 64 << 20
n = a.n or k + k // 4
L = chunk.replica_size(k, size)
Ls = -(-L // a.align) * a.align  # replica stride
inp = torch.empty(a.objects * size, dtype=torch.uint8, device="cuda")
RB = a.objects * Ls + a.skew  # replica buffer i at i * RB
reps = torch.empty(n * RB, dtype=torch.uint8, device="cuda").as_strided((n, a.objects * Ls), (RB, 1))
out = torch.empty(a.objects * size, dtype=torch.uint8, device="cuda")
for i in range(a.objects):
    chunk.fill_splitmix_device(inp[i * size:], size, 0x7664730000000000 + i)
nodes = [r for r in range(n) if r % 5 != 0 or r >= 5 * (n - k)][:k]  # erase 0, 5, 10, ..
rp = [reps[i].data_ptr() for i in range(n)]
cp = [reps[r].data_ptr() for r in nodes]
enc = lambda: chunk.encode_device(k, list(range(n)), inp, size, size, a.objects, rp, Ls)  # noqa: E731
rep = lambda: chunk.restore_device(k, nodes, cp, L, Ls, size % (2 * k), a.objects, out, size)  # noqa: E731
enc()
rep()
rep()  # (a survivor set's second use queues its own kernel's compile, vds_ec_jit.cpp)
chunk.jit_wait()
rep()
torch.cuda.synchronize()
res = {}
for name, f in (("encode", enc), ("repair", rep)):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        f()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.iters
    res[name] = (ms, a.objects * size / (ms * 1e-3) / 2**30)
ok = ""
if a.check:
    ok = " check " + ("ok" if torch.equal(out, inp) else "MISMATCH")
print(f"{a.tag} k={k} n={n} align={a.align} skew={a.skew}: encode {res['encode'][0]:.3f} ms ({res['encode'][1]:.1f} GiB/s)  "
      f"repair {res['repair'][0]:.3f} ms ({res['repair'][1]:.1f} GiB/s){ok}", flush=True)
