"""PCIe / host-copy ceilings for the host-resident path (C5).

Measures on the current GPU: pinned H2D and D2H alone and concurrently
(two streams), pageable H2D / D2H (the runtime's own staging), a host memcpy
into pinned memory with 1..16 threads, and the cost of registering a caller
buffer (hipHostRegister through torch's cudaHostRegister binding).
Prints one JSON line.

  python tools/ubench/pcie.py [--mib 256]
"""
import argparse
import ctypes
import json
import threading
import time

import numpy as np
import torch

p = argparse.ArgumentParser()
p.add_argument("--mib", type=int, default=256)
a = p.parse_args()
N = a.mib << 20
dev = torch.device("cuda:0")
d = torch.empty(N, dtype=torch.uint8, device=dev)
d2 = torch.empty(N, dtype=torch.uint8, device=dev)
hp = torch.empty(N, dtype=torch.uint8).pin_memory()
hp2 = torch.empty(N, dtype=torch.uint8).pin_memory()
hq = torch.ones(N, dtype=torch.uint8)  # pageable, pre-faulted
res = {"bytes": N}


def rate(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    best = None
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    return round(N / best / 1e9, 2)


res["h2d_pinned_GBps"] = rate(lambda: d.copy_(hp, non_blocking=True))
res["d2h_pinned_GBps"] = rate(lambda: hp.copy_(d, non_blocking=True))
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()


def both():
    with torch.cuda.stream(s1):
        d.copy_(hp, non_blocking=True)
    with torch.cuda.stream(s2):
        hp2.copy_(d2, non_blocking=True)


res["h2d_plus_d2h_each_GBps"] = rate(both)
res["h2d_pageable_GBps"] = rate(lambda: d.copy_(hq))
res["d2h_pageable_GBps"] = rate(lambda: hq.copy_(d))
src = hq.numpy()
dst = hp.numpy()
for nt in (1, 4, 8, 16):
    def mc(nt=nt):
        step = N // nt
        th = [threading.Thread(target=lambda i=i: np.copyto(dst[i * step:(i + 1) * step], src[i * step:(i + 1) * step]))
              for i in range(nt)]
        for t in th:
            t.start()
        for t in th:
            t.join()
    res[f"memcpy_to_pinned_{nt}t_GBps"] = rate(mc, reps=3)
# registering a pageable caller buffer (what a zero-copy path would pay per buffer)
buf = np.ones(N, dtype=np.uint8)
cudart = torch.cuda.cudart()
t0 = time.perf_counter()
rc = cudart.cudaHostRegister(buf.ctypes.data, N, 0)
t1 = time.perf_counter()
rc2 = cudart.cudaHostUnregister(buf.ctypes.data)
t2 = time.perf_counter()
res["host_register_ms"] = round((t1 - t0) * 1e3, 3) if rc == 0 else f"error {rc}"
res["host_unregister_ms"] = round((t2 - t1) * 1e3, 3) if rc2 == 0 else f"error {rc2}"
print(json.dumps(res), flush=True)
