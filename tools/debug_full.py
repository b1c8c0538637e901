import sys, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import torch
from vds_amd import chunk, _lib
_lib.lib()
k, n = int(sys.argv[1]), int(sys.argv[2])
step = sys.argv[3] if len(sys.argv) > 3 else "all"
def p(*a): print(*a, flush=True)
maps = sorted({l.split()[5] for l in open('/proc/self/maps') if len(l.split()) >= 6 and 'amdhip' in l})
p("maps", maps)
size = 64 << 20
t = torch.empty(size, dtype=torch.uint8, device="cuda")
chunk.fill_splitmix_device(t, size, 0x7664730000000000)
torch.cuda.synchronize(); p("filled")
L = chunk.replica_size(k, size)
out = torch.zeros((n, 1, L), dtype=torch.uint8, device="cuda")
chunk.encode_device(k, list(range(n)), t, size, size, 1, [out[i].data_ptr() for i in range(n)], L)
torch.cuda.synchronize(); p("encoded")
m = n - k
for erased in (list(range(m)), list(range(0, n, n // m))[:m], list(range(n - m, n))):
    nodes = [r for r in range(n) if r not in erased]
    r = torch.empty(size, dtype=torch.uint8, device="cuda")
    chunk.restore_device(k, nodes, [out[j, 0].data_ptr() for j in nodes], L, 0, size % (2 * k), 1, r, 0)
    torch.cuda.synchronize(); p("restored", erased, torch.equal(r, t))
t2 = torch.empty(size, dtype=torch.uint8, device="cuda")
chunk.fill_splitmix_device(t2, size, 0x7664730000000001)
x = t ^ t2
torch.cuda.synchronize(); p("xor done")
p("done")
