"""bench.py -- device-resident encode+repair throughput of the MI355X codec.

One "step" = encode every object of the batch into all n = k+m replicas
(chunk_generator<uint16_t>::write for replicas 0..n-1, chunk.h:245-281) and
then repair every object from the k replicas left after erasing m of them
(chunk_restore<uint16_t>::restore, chunk.h:290-444).  Inputs are synthetic
(splitmix64) and already resident in HBM when timing starts.

Default workload (BASELINE.json configs[1]/[2]): k=16, m=4, 1024 objects of
64 MiB per GPU, erasures {0,5,10,15}.  Multi-GPU: one process per GPU
(torchrun), objects round-robin by rank, no data-path collective ("weak"
scaling: per-GPU work is fixed).  rank 0 prints ONE JSON line.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--k 16] [--m 4]
                  [--objects 1024] [--object-mib 64] [--no-cpu-baseline]
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

SEED = 0x7664730000000000
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--k", type=int, default=16)
    p.add_argument("--m", type=int, default=4)
    p.add_argument("--objects", type=int, default=1024, help="objects per GPU")
    p.add_argument("--object-mib", type=float, default=64.0)
    p.add_argument("--erase", type=str, default="", help="comma list of erased replica ids")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-live", action="store_true", help="skip the live-shape line (k=32, n=64, 64 KiB objects)")
    p.add_argument("--no-align16", action="store_true", help="skip the 16-byte replica stride line")
    p.add_argument("--no-jit", action="store_true",
                   help="no run-time compiled survivor-set kernel: the repair runs k_restore_syn")
    p.add_argument("--live-objects", type=int, default=16384)
    p.add_argument("--no-c4", action="store_true", help="skip the k=32, m=8 leg (BASELINE.json configs[3])")
    p.add_argument("--c4-objects", type=int, default=1024, help="objects per GPU of the k=32, m=8 leg")
    p.add_argument("--replica-align", type=int, default=256,
                   help="replica buffers start on multiples of this many bytes (1: packed at the odd stride L)")
    p.add_argument("--cpu-objects", type=int, default=8, help="objects in the CPU baseline sample")
    p.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"),
                   help="per-object HBM bytes per kernel from rocprofv3 PMC passes (tools/pmc_traffic.py)")
    p.add_argument("--traffic-json-k32", default=os.path.join(ROOT, "profiles", "traffic_k32.json"),
                   help="the same for the k=32, n=40 kernels (the C4 leg)")
    return p.parse_args()


def relaunch_with_torchrun(args) -> int:
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", "--master-port=29533", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


CPU_THREAD_CAP = 16


def cpu_threads() -> int:
    """Host threads for the object-parallel leg: the CPUs this process may run
    on, capped at 16.  SURVEY.md 8(d) asks for nproc threads; on the GPU box
    nproc and os.cpu_count() show the whole 256-CPU machine, but one GPU's
    share of it is 16 CPUs (the box's process rules), so 16 is the host a
    one-GPU deployment of this codec has."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(n, CPU_THREAD_CAP))


def cpu_baseline(k, n, size, nodes, count):
    """The oracle (CPU restatement of kernel/vds_data) timed on a bounded
    sample of the same workload: one thread, as the reference runs (its codec
    runs on the single DB apartment thread), and the
    object-parallel rate over the box's host threads.  Test
    infrastructure: never part of the GPU measurement."""
    import concurrent.futures as cf

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ctypes as O

    O.lib()

    def one(o):  # encode all n replicas of object o, then repair from `nodes`
        d = O.splitmix(SEED + o, size)
        chunks = [O.encode(k, r, d) for r in range(n)]
        out = O.restore(k, nodes, [chunks[r] for r in nodes])
        assert out is not None and out.size == size

    t0 = time.perf_counter()
    for o in range(count):
        one(o)
    dt = time.perf_counter() - t0
    nt = cpu_threads()
    pcount = 2 * nt
    t1 = time.perf_counter()
    with cf.ThreadPoolExecutor(nt) as ex:  # ctypes releases the GIL around the oracle calls
        list(ex.map(one, range(pcount)))
    pdt = time.perf_counter() - t1
    return {"value": round(count * size / dt / 2**30, 6), "unit": "GiB/s", "cores": 1, "kind": "port",
            "sample": f"{count} x {size >> 20} MiB objects, encode all {n} replicas + repair from {len(nodes)} "
                      f"(oracle/vds_oracle.c, 1 thread, {dt:.2f} s; input generation included)",
            "seconds": round(dt, 3),
            "parallel": {"value": round(pcount * size / pdt / 2**30, 6), "unit": "GiB/s", "cores": nt,
                         "sample": f"{pcount} x {size >> 20} MiB objects over {nt} threads ({pdt:.2f} s)",
                         "thread_cap": f"{CPU_THREAD_CAP}: one GPU's CPU share of the box (nproc shows "
                                       f"{os.cpu_count()})"},
            "cpu_model": cpu_model(), "host_cpus": os.cpu_count()}


def replica_stride(L, align):
    """Distance between consecutive objects' replicas in one replica buffer.
    256 bytes is this benchmark's device layout (each replica starts on a
    256-byte boundary, as the device allocator hands out buffers), not a
    property of the reference: its replicas live in separate malloc'd
    const_data_buffers, which guarantee 16-byte alignment only.  Packing them
    at the odd length L = 2T + 2 would start every odd object 2 bytes off a
    dword and make every 1 KiB wave access straddle an extra 128-byte line
    (one box, 512 x 64 MiB at k=16: encode 2290 -> 2405, repair 1632 -> 1738
    GiB/s with the 256-byte stride).  The bytes moved are the same; the rate
    at a 16-byte stride is reported beside the metric (align16)."""
    return -(-L // align) * align


def kernel_names(k, n, nodes, size, L, objects):
    """Names of the kernels the C ABI dispatches for this workload."""
    import ctypes as C
    import numpy as np
    from vds_amd import _lib
    ids = np.arange(n, dtype=np.uint16)
    nd = np.asarray(nodes, dtype=np.uint16)
    ep = _lib.lib().vds_ec_encode16_path(k, ids.ctypes.data_as(_lib.u16p), n, C.c_uint64(size))
    rp = _lib.lib().vds_ec_restore16_path(k, nd.ctypes.data_as(_lib.u16p), C.c_uint64(L), size % (2 * k), objects)
    enc = {2: f"k_encode_bs<{k},{n}>"}.get(ep, "k_encode_generic")
    # the run-time compiled kernel's symbol carries (k, n) and the survivor
    # mask (vds_ec_jit.cpp kernel_name), as rocprofv3 lists it
    mask = sum(1 << int(r) for r in nodes)
    rep = {4: f"vds_ec_jit_restore_{k}_{n}_{mask:x}", 3: f"k_restore_syn<{k},{n}>", 2: f"k_restore_bs<{k}>"}.get(
        rp, "k_restore_generic")
    return enc, rep


def pmc_traffic(path, kernel, objects, k, n):
    """roofline.traffic: HBM bytes per launch of `kernel` from the committed
    rocprofv3 FETCH_SIZE/WRITE_SIZE passes (bytes per object x objects), only
    when they were measured on the same code shape (k, n)."""
    try:
        with open(path) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return None, None
    e = t.get(kernel.split("<")[0])
    if e is None and kernel.startswith("vds_ec_jit_restore"):
        e = t.get("vds_ec_jit_restore")  # (profiles taken before the kernels carried their survivor set)
    if not e or (e.get("k", 16), e.get("n", 20)) != (k, n):
        return None, None
    return round(e["bytes_per_object"] * objects), f"{os.path.relpath(path, ROOT)}: {e['source']}"


def owned_objects(rank: int, world: int, per_rank: int) -> list[int]:
    """Global ids of the objects rank `rank` encodes and repairs: round-robin
    ownership, object o -> rank o % world; every rank has
    the same count, so per-GPU work is fixed as the world grows (weak scaling)."""
    return [rank + world * i for i in range(per_rank)]


def max_over_ranks(values, dist, device):
    """Element-wise MAX of per-rank timings (the job finishes with its slowest
    rank).  The only collective in the benchmark; none is on the data path."""
    import torch
    t = torch.tensor(list(values), dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(x) for x in t.tolist()]


def save_temp_leg(torch, chunk, dev, stream, inp, objects, size, k, n, L, Ls, timed, gib, batches=8):
    """save_temp (dht_network_client.cpp:74-104): encode replicas 0..n-1 of an
    object and name each by its SHA-256.  The encode is memory-bound and the
    hash VALU-bound, so batch b's hashes run on a second stream beside batch
    b+1's encode (replicas object-major here, [objects][n][Ls], so a batch's
    n x objects/batches messages are one strided launch).  Reported: the
    pipelined rate, the same work serial on one stream, and the digests
    checked against hashlib."""
    import hashlib
    rep = torch.empty(objects * n * Ls, dtype=torch.uint8, device=dev)
    dig = torch.empty(objects * n * 32, dtype=torch.uint8, device=dev)
    per = objects // batches
    s2 = torch.cuda.Stream(dev)
    evs = [torch.cuda.Event() for _ in range(batches)]
    done = torch.cuda.Event()
    b0 = rep.data_ptr()

    def enc(o0, cnt, st):
        chunk.encode_device(k, list(range(n)), inp[o0 * size:], size, size, cnt,
                            [b0 + (o0 * n + i) * Ls for i in range(n)], n * Ls, stream=st)

    def sha(o0, cnt, st):
        chunk.sha256_device(rep[o0 * n * Ls:], L, Ls, cnt * n, dig[o0 * n * 32:], st)

    def serial():
        enc(0, objects, stream)
        sha(0, objects, stream)

    def pipelined():
        s2.wait_stream(stream)
        for b in range(batches):
            o0 = b * per
            cnt = per if b + 1 < batches else objects - o0
            enc(o0, cnt, stream)
            evs[b].record(stream)
            s2.wait_event(evs[b])
            sha(o0, cnt, s2)
        done.record(s2)
        stream.wait_event(done)  # (the timed region ends on `stream` after the last hash)

    with torch.cuda.stream(stream):
        ser_wall, ser_gpu = timed(serial)
        pip_wall, pip_gpu = timed(pipelined)
    torch.cuda.synchronize(dev)
    hb = rep[:(2 * n) * Ls].cpu().numpy().tobytes()
    dg = dig[:(2 * n) * 32].cpu().numpy().tobytes()
    assert all(hashlib.sha256(hb[i * Ls:i * Ls + L]).digest() == dg[32 * i:32 * (i + 1)] for i in range(2 * n)), \
        "save_temp sha"
    del rep, dig
    pip, ser = gib(objects * size, pip_gpu), gib(objects * size, ser_gpu)
    # headline: the schedule the library's own save_temp16_host uses (serial,
    # one stream), not the better of two per run; the two-stream pipeline is
    # reported beside it (it has measured slower: both kernels are VALU-heavy)
    return {"save_temp_GiBps": ser, "save_temp_schedule": "serial",
            "pipelined_GiBps": pip, "serial_GiBps": ser,
            "batches": batches, "layout": "replicas object-major [objects][n][Ls]",
            "what": "encode of replicas 0..n-1 + SHA-256 of each; pipelined: batch b's hashes on a second stream "
                    "beside batch b+1's encode; serial: one stream"}


def live_shape(torch, chunk, dev, stream, objects, steps, warmup=3, losses=(0.02, 0.25), seed=1, align=256):
    """The production shape beside the metric (never in it): MIN_HORCRUX 32,
    GENERATE_HORCRUX 64 (dht_network.h:22-25) on the web client's 64 KiB
    blocks (web/src/store/vds_api.jsx:76).  Encode all 64 replicas of every
    object (save_temp) and name each by its SHA-256; then, per replica-loss
    rate p, every replica is lost independently with probability p, each
    object is restored from the first 32 replicas found (restore_async,
    dht_network_client.cpp:851-901) with ONE batched call over all objects
    (vds_ec_restore16_batch_device), and the first lost replica of every
    object that lost one is regenerated (sync_process's repair) with
    vds_ec_regenerate16_batch_device.  At p = 0.02 almost every survivor set
    lies within replicas 0..39 (the syndrome kernel's points); at p = 0.25
    most do not (the runtime-coefficient batch mode).  Host times include the
    per-object planning and table staging of the batched calls; max(steps, 10)
    timed calls follow max(5, warmup) untimed ones (by then the process-wide
    erased-set plans are solved and the pinned staging slots allocated, as in
    a running node).  Every restored object and every regenerated replica is
    checked against the encoded bytes."""
    import numpy as np
    from vds_amd import _lib
    k, n, size = 32, 64, 65536
    L = chunk.replica_size(k, size)
    Ls = replica_stride(L, align)
    inp = torch.empty(objects * size, dtype=torch.uint8, device=dev)
    chunk.fill_splitmix_device(inp, objects * size, SEED ^ 0x6C697665)
    reps = torch.empty((n, objects * Ls), dtype=torch.uint8, device=dev)
    out = torch.empty(objects * size, dtype=torch.uint8, device=dev)
    rep_ptrs = [reps[i].data_ptr() for i in range(n)]
    lib = _lib.lib()
    sp = stream.cuda_stream
    reps_timed = max(steps, 10)  # (beside the metric: enough calls for a stable rate)

    spreads = {}

    def timed(fn, name=None):
        """Back-to-back calls (the rate: what a caller looping on the call
        sees) with an event before every call, so each call's stream span is
        a sample; and, with `name`, the same call alone behind a spin kernel
        long enough to cover its host planning, so its span is device time
        only.  A leg whose stream span exceeds its device time is host-bound:
        its rate then follows the host CPU, not the kernels."""
        for _ in range(max(5, warmup)):  # steady state: staging slots allocated, erased-set plans solved
            fn()
        torch.cuda.synchronize(dev)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(reps_timed + 1)]
        host = []
        t0 = time.perf_counter()
        ev[0].record(stream)
        for i in range(reps_timed):
            h0 = time.perf_counter()
            fn()
            host.append(time.perf_counter() - h0)
            ev[i + 1].record(stream)
        torch.cuda.synchronize(dev)
        wall = (time.perf_counter() - t0) / reps_timed
        gpu = ev[0].elapsed_time(ev[-1]) / reps_timed * 1e-3
        if name:
            spans = [ev[i].elapsed_time(ev[i + 1]) for i in range(reps_timed)]
            dev_ms = []
            for _ in range(reps_timed):  # the device alone: the call is enqueued while the stream spins
                torch.cuda._sleep(spin_cycles(2 * max(host) * 1e3 + 2.0))
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(stream)
                fn()
                b.record(stream)
                torch.cuda.synchronize(dev)
                dev_ms.append(a.elapsed_time(b))

            def mm(x):
                return {"median": round(float(np.median(x)), 4), "min": round(float(min(x)), 4),
                        "max": round(float(max(x)), 4)}
            spreads[name] = {"stream_ms_per_call": mm(spans), "device_ms_per_call": mm(dev_ms),
                             "host_enqueue_ms_per_call": mm([h * 1e3 for h in host]), "calls": reps_timed,
                             "bound": "host" if np.median(spans) > 1.1 * np.median(dev_ms) else "device"}
        return wall, gpu

    spin = {}

    def spin_cycles(ms):
        """torch.cuda._sleep cycles for about `ms` milliseconds (calibrated once)."""
        if "per_ms" not in spin:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            with torch.cuda.stream(stream):
                a.record(stream)
                torch.cuda._sleep(10 ** 7)
                b.record(stream)
            torch.cuda.synchronize(dev)
            spin["per_ms"] = 10 ** 7 / max(a.elapsed_time(b), 1e-3)
        return int(spin["per_ms"] * ms)

    def enc():
        chunk.encode_device(k, list(range(n)), inp, size, size, objects, rep_ptrs, Ls)

    # save_temp names every replica by its SHA-256 (dht_network_client.cpp:77-79):
    # one launch over all n x objects replicas (n * objects messages of L bytes)
    digests = torch.empty(n * objects * 32, dtype=torch.uint8, device=dev)

    def sha():
        chunk.sha256_device(reps, L, Ls, n * objects, digests, stream)

    gib = lambda nbytes, t: round(nbytes / t / 2**30, 3) if t else None

    def roof(nbytes, t, what):
        """Per-leg roofline: algorithmic HBM bytes of one call (SURVEY.md 8(d):
        encode S + n L, restore k L + S, regenerate k L + L per object; SHA-256
        L read + 32 written per message) over the call's device time (HIP
        events around the call on its stream: every kernel and copy of it)."""
        if not t:
            return None
        return {"algorithmic_bytes_per_call": int(nbytes), "gpu_ms_per_call": round(t * 1e3, 4),
                "achieved_GBps": round(nbytes / t / 1e9, 1), "peak_GBps": HBM_PEAK_GBPS,
                "frac": round(nbytes / t / 1e9 / HBM_PEAK_GBPS, 4), "bytes": what}

    with torch.cuda.stream(stream):
        enc_wall, enc_gpu = timed(enc, "encode")
        sha_wall, sha_gpu = timed(sha, "sha256")
    torch.cuda.synchronize(dev)
    enc_bytes, sha_bytes = objects * (size + n * L), n * objects * (L + 32)
    res = {"shape": f"k={k}, n={n}, {objects} x 64 KiB objects, replica stride {Ls} B",
           "encode_GiBps": gib(objects * size, enc_gpu),
           "sha256_replicas_GiBps": gib(n * objects * L, sha_gpu),
           "sha256_object_GiBps": gib(objects * size, sha_gpu),
           "roofline": {"encode": roof(enc_bytes, enc_gpu, "objects x (S + n L)"),
                        "sha256": roof(sha_bytes, sha_gpu, "n objects x (L + 32)")}}
    # spot-check the digests against hashlib
    import hashlib
    hb = reps.view(-1)[: 4 * Ls].cpu().numpy().tobytes()
    dg = digests[: 4 * 32].cpu().numpy().tobytes()
    assert all(hashlib.sha256(hb[i * Ls:i * Ls + L]).digest() == dg[32 * i:32 * (i + 1)] for i in range(4)), "sha"
    del digests
    res["save_temp"] = save_temp_leg(torch, chunk, dev, stream, inp, objects, size, k, n, L, Ls, timed, gib)
    base = np.asarray(rep_ptrs, dtype=np.uint64)
    reps2d = reps.view(n, objects, Ls)

    for loss in losses:
        rng = np.random.default_rng(seed)
        lost = rng.random((objects, n)) < loss
        objs = np.flatnonzero((~lost).sum(axis=1) >= k)
        nodes = np.stack([np.flatnonzero(~lost[o])[:k] for o in objs]).astype(np.uint16)
        chunk_ptrs = (base[nodes] + (objs.astype(np.uint64) * Ls)[:, None]).astype(np.uint64)
        sizes = np.full(len(objs), L, dtype=np.uint64)
        pads = np.zeros(len(objs), dtype=np.uint16)
        outs = (np.uint64(out.data_ptr()) + objs.astype(np.uint64) * size).astype(np.uint64)

        def restore():
            _lib.check(lib.vds_ec_restore16_batch_device(
                k, len(objs), nodes.ctypes.data_as(_lib.u16p), chunk_ptrs.ctypes.data_as(_lib.vpp),
                sizes.ctypes.data_as(_lib.u64p), pads.ctypes.data_as(_lib.u16p), outs.ctypes.data_as(_lib.vpp), 0, sp))

        # regenerate: the first lost replica of every object that lost one
        rg = np.flatnonzero(lost[objs].any(axis=1))
        rg_targets = np.argmax(lost[objs[rg]], axis=1).astype(np.uint16)
        rg_out = torch.empty(max(1, len(rg)) * Ls, dtype=torch.uint8, device=dev)
        rg_outs = (np.uint64(rg_out.data_ptr()) + np.arange(len(rg), dtype=np.uint64) * Ls).astype(np.uint64)
        rg_nodes = np.ascontiguousarray(nodes[rg])
        rg_chunks = np.ascontiguousarray(chunk_ptrs[rg])
        rg_sizes = np.full(len(rg), L, dtype=np.uint64)

        def regen():
            _lib.check(lib.vds_ec_regenerate16_batch_device(
                k, len(rg), rg_nodes.ctypes.data_as(_lib.u16p), rg_chunks.ctypes.data_as(_lib.vpp),
                rg_sizes.ctypes.data_as(_lib.u64p), 1, rg_targets.ctypes.data_as(_lib.u16p),
                rg_outs.ctypes.data_as(_lib.vpp), sp))

        out.zero_()
        rg_out.zero_()
        with torch.cuda.stream(stream):
            rest_wall, rest_gpu = timed(restore, f"repair_{loss}")
            regen_wall, regen_gpu = timed(regen, f"regenerate_{loss}") if len(rg) else (None, None)
        torch.cuda.synchronize(dev)
        idx = torch.from_numpy(objs).to(dev)
        assert torch.equal(out.view(objects, size)[idx], inp.view(objects, size)[idx]), f"live restore differs (p={loss})"
        if len(rg):  # every regenerated replica equals the encoded one
            want = reps2d[torch.from_numpy(rg_targets.astype(np.int64)).to(dev), torch.from_numpy(objs[rg]).to(dev), :L]
            assert torch.equal(rg_out.view(-1, Ls)[:len(rg), :L], want), f"live regenerate differs (p={loss})"
        syn_pts = int(((nodes < 40).all(axis=1)).sum())
        leg = {"loss": loss, "restorable": int(len(objs)), "regenerated": int(len(rg)),
               "roofline": {"repair": roof(len(objs) * (k * L + size), rest_gpu, "restorable x (k L + S)"),
                            "regenerate": roof(len(rg) * (k * L + L), regen_gpu, "regenerated x (k L + L)")},
               "repair_GiBps": gib(len(objs) * size, rest_gpu),
               "repair_host_GiBps": gib(len(objs) * size, rest_wall),
               "regenerate_GiBps": gib(len(rg) * size, regen_gpu),
               "regenerate_host_GiBps": gib(len(rg) * size, regen_wall),
               "distinct_survivor_sets": int(len({tuple(r) for r in nodes.tolist()})),
               "survivors_within_0_39": syn_pts,
               "spread": {"repair": spreads.get(f"repair_{loss}"), "regenerate": spreads.get(f"regenerate_{loss}")}}
        if loss == losses[0]:  # (the round-2 keys: the first loss rate)
            res.update({kk: v for kk, v in leg.items() if kk not in ("loss", "roofline", "spread")})
            res["roofline"].update(leg["roofline"])
            res["shape"] += f"; replica loss p={loss}; {len(objs)} restorable, {len(rg)} regenerated"
        res[f"loss_{loss}"] = leg
        del rg_out
    res["spread"] = {"encode": spreads.get("encode"), "sha256": spreads.get("sha256")}
    del inp, reps, out
    return res


def c4_jit_prebuild(k, nodes):
    """Compile the C4 survivor set's kernel into the on-disk JIT cache on a
    host thread while the headline runs (a k=32 compile takes ~12 s of host
    CPU; no device is touched).  The leg's own warm-up then loads it from the
    cache instead of waiting for a compile."""
    import threading
    import numpy as np
    from vds_amd import _lib
    nd = np.asarray(nodes, dtype=np.uint16)
    th = threading.Thread(target=lambda: _lib.lib().vds_ec_jit_build16(k, nd.ctypes.data_as(_lib.u16p), None),
                          daemon=True)
    th.start()
    return th


def c4_leg(torch, chunk, dev, stream, args, rank, world, dist, prebuild=None):
    """BASELINE.json configs[3]: k=32, m=8 encode of all 40 replicas and repair
    from 32 (erased every fifth replica, {0, 5, .., 35}), objects round-robin
    over the GPUs as the headline (weak scaling), 64 MiB objects, `--c4-objects`
    per GPU (1024: 208 GiB of inputs, replicas and outputs).  Reported beside
    the metric, never in it, with its own roofline block per kernel: algorithmic
    bytes per launch (S + n L encode, k L + S repair) over the
    HIP-event launch time, against 8 TB/s."""
    k, m = 32, 8
    n = k + m
    size = 64 << 20
    L = chunk.replica_size(k, size)
    Ls = replica_stride(L, args.replica_align)
    erased = list(range(0, n, n // m))[:m]
    nodes = [r for r in range(n) if r not in erased][:k]
    free, _total = torch.cuda.mem_get_info(dev)
    per_obj = size + n * Ls + size
    objects = min(args.c4_objects, max(1, int(0.92 * free // per_obj)))
    if world > 1:
        objects = int(-max_over_ranks([-objects], dist, dev)[0])
    inp = torch.empty(objects * size, dtype=torch.uint8, device=dev)
    reps = torch.empty((n, objects * Ls), dtype=torch.uint8, device=dev)
    restored = torch.empty(objects * size, dtype=torch.uint8, device=dev)
    for i, oid in enumerate(owned_objects(rank, world, objects)):
        chunk.fill_splitmix_device(inp[i * size:], size, SEED ^ 0xC4 ^ (oid << 8))
    rep_ptrs = [reps[i].data_ptr() for i in range(n)]
    chunk_ptrs = [reps[r].data_ptr() for r in nodes]
    padding = size % (2 * k)

    def encode():
        chunk.encode_device(k, list(range(n)), inp, size, size, objects, rep_ptrs, Ls)

    def repair():
        chunk.restore_device(k, nodes, chunk_ptrs, L, Ls, padding, objects, restored, size)

    def timed(fn, steps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(dev)
        e0.record(stream)
        for _ in range(steps):
            fn()
        e1.record(stream)
        torch.cuda.synchronize(dev)
        return e0.elapsed_time(e1) / steps

    for _ in range(max(1, args.warmup)):
        encode()
    # the pattern-independent syndrome kernel first (it serves every set until
    # the set's own kernel is loaded), then the survivor set's kernel
    chunk.jit_set_mode(0)
    repair()
    aot_ms = timed(repair, args.steps)
    aot_kernel = kernel_names(k, n, nodes, size, L, objects)[1]
    jit_s = None
    if not args.no_jit:
        chunk.jit_set_mode(1)
        t0 = time.perf_counter()
        if prebuild is not None:
            prebuild.join()
        repair()
        repair()
        chunk.jit_wait()
        repair()
        jit_s = time.perf_counter() - t0
    torch.cuda.synchronize(dev)
    assert torch.equal(restored[:size], inp[:size]) and \
        torch.equal(restored[(objects - 1) * size:], inp[(objects - 1) * size:]), "c4 repair differs"
    enc_ms = timed(encode, args.steps)
    rep_ms = timed(repair, args.steps)
    if world > 1:
        enc_ms, rep_ms, aot_ms = max_over_ranks([enc_ms, rep_ms, aot_ms], dist, dev)
    sl = 1 << 30
    assert all(torch.equal(restored[i:i + sl], inp[i:i + sl]) for i in range(0, objects * size, sl)), "c4 repair"
    enc_name, rep_name = kernel_names(k, n, nodes, size, L, objects)
    enc_bytes = objects * (size + n * L)
    rep_bytes = objects * (k * L + size)
    gb = world * objects * size / 2**30

    def roof(name, nbytes, ms):
        ach = nbytes / (ms * 1e-3) / 1e9
        tr, src = pmc_traffic(args.traffic_json_k32, name, objects, k, n)
        return {"kernel": name, "algorithmic_bytes_per_launch": nbytes, "avg_launch_ms": round(ms, 4),
                "achieved": round(ach, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBPS, 4), "traffic": tr, "traffic_source": src}

    res = {"workload": f"k={k},m={m} encode of all {n} replicas + repair from {k} (erased {erased}), "
                       f"{objects} x 64 MiB objects per GPU",
           "k": k, "m": m, "objects_per_gpu": objects, "n_gpus": world, "erased": erased,
           "value": round(gb / ((enc_ms + rep_ms) * 1e-3), 3), "unit": "GiB/s",
           "encode_GiBps": round(gb / (enc_ms * 1e-3), 3), "repair_GiBps": round(gb / (rep_ms * 1e-3), 3),
           "encode_ms": round(enc_ms, 3), "repair_ms": round(rep_ms, 3),
           "restore_aot_ms": round(aot_ms, 3), "restore_aot_kernel": aot_kernel,
           "restore_kernel": rep_name, "jit_wait_s": round(jit_s, 3) if jit_s is not None else None,
           "roofline": {"encode": roof(enc_name, enc_bytes, enc_ms), "repair": roof(rep_name, rep_bytes, rep_ms),
                        "repair_aot": roof(aot_kernel, rep_bytes, aot_ms)}}
    del inp, reps, restored
    torch.cuda.empty_cache()
    return res


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    from vds_amd import build as vbuild
    if args.gpus > 1 and world == 1:
        vbuild.build()  # once, in the parent (no GPU touched), before the ranks start
        sys.exit(relaunch_with_torchrun(args))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    import torch
    import torch.distributed as dist

    vbuild.build()  # a no-op when fresh; build.py serialises concurrent callers
    from vds_amd import chunk
    if args.no_jit:
        chunk.jit_set_mode(0)

    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    k, m = args.k, args.m
    n = k + m
    size = int(args.object_mib * (1 << 20))
    L = chunk.replica_size(k, size)
    Ls = replica_stride(L, args.replica_align)
    if args.erase:
        erased = [int(x) for x in args.erase.split(",")]
    else:
        step = max(1, n // m)
        erased = list(range(0, n, step))[:m]
    nodes = [r for r in range(n) if r not in erased][:k]

    # ---- memory plan: inputs + all replicas + restored objects, resident in HBM
    objects = args.objects
    free, _total = torch.cuda.mem_get_info(dev)
    per_obj = size + n * Ls + size
    if objects * per_obj > 0.92 * free:
        objects = max(1, int(0.92 * free // per_obj))
    if world > 1:  # every rank runs the same count (weak scaling, value = world * objects)
        objects = int(-max_over_ranks([-objects], dist, dev)[0])
    inp = torch.empty(objects * size, dtype=torch.uint8, device=dev)
    reps = torch.empty((n, objects * Ls), dtype=torch.uint8, device=dev)
    restored = torch.empty(objects * size, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    for i, oid in enumerate(owned_objects(rank, world, objects)):
        chunk.fill_splitmix_device(inp[i * size:], size, SEED + oid)
    torch.cuda.synchronize(dev)

    rep_ptrs = [reps[i].data_ptr() for i in range(n)]
    chunk_ptrs = [reps[r].data_ptr() for r in nodes]
    padding = size % (2 * k)

    def encode():
        chunk.encode_device(k, list(range(n)), inp, size, size, objects, rep_ptrs, Ls)

    def repair():
        chunk.restore_device(k, nodes, chunk_ptrs, L, Ls, padding, objects, restored, size)

    c4_pre = None
    if not args.no_c4 and not args.no_jit:
        c4_pre = c4_jit_prebuild(32, [r for r in range(40) if r % 5][:32])
    if not args.no_jit:
        chunk.jit_set_mode(0)  # (the AOT timing below first)
    for _ in range(args.warmup):
        encode()
        repair()
    # The pattern-independent syndrome kernel k_restore_syn serves a survivor
    # set until the set's own kernel is loaded (every first-seen set, every
    # deployment without the JIT helper): its repair time, beside the metric.
    aot_ms = None
    if not args.no_jit:
        torch.cuda.synchronize(dev)
        a0, a1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a0.record(stream)
        for _ in range(args.steps):
            repair()
        a1.record(stream)
        torch.cuda.synchronize(dev)
        aot_ms = a0.elapsed_time(a1) / args.steps
        aot_name = kernel_names(k, n, nodes, size, L, objects)[1]
        chunk.jit_set_mode(1)
    # The survivor set's own restore kernel (vds_amd/csrc/vds_ec_jit.cpp) is
    # compiled in the background from the set's second use; a repair pass
    # keeps using it for the rest of the set's objects, so the steady state is
    # measured with it loaded (untimed here: two uses, the wait, one launch).
    jit_s = None  # host seconds of those untimed calls (the compile overlaps the warmup's GPU work)
    if not args.no_jit:
        t_jit = time.perf_counter()
        repair()
        repair()
        chunk.jit_wait()
        repair()
        jit_s = time.perf_counter() - t_jit
    torch.cuda.synchronize(dev)
    restore_kernel = {4: "jit", 3: "syndrome", 2: "bitsliced", 1: "generic"}[chunk.restore_path(k, nodes, L, padding,
                                                                                             objects)]
    # correctness guard on the measured buffers (outside the timed region):
    # every restored object equals its input (a device-side compare of the
    # whole batch); the parity suite checks the bytes against the oracle
    # (in 1 GiB slices: torch.equal materialises an element-wise result)
    sl = 1 << 30
    assert all(torch.equal(restored[i:i + sl], inp[i:i + sl]) for i in range(0, objects * size, sl)), \
        "repair output differs from the input"

    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True),
           torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for s in range(args.steps):
        ev[s][0].record(stream)
        encode()
        ev[s][1].record(stream)
        repair()
        ev[s][2].record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    enc_ms = sum(a.elapsed_time(b) for a, b, _ in ev) / args.steps
    rep_ms = sum(b.elapsed_time(c) for _, b, c in ev) / args.steps

    # Fused repair, reported beside the metric, not in
    # it: regenerate the m erased replicas of every object straight from the
    # k survivors (the reference's repair restores and re-encodes instead).
    regen_out = reps[erased[0]] if erased and erased[0] < n else None
    regen_ms = None
    if regen_out is not None and len(erased) == m:
        # written over the erased replicas' own buffers: same bytes, same place
        def regenerate():
            chunk.regenerate_device(k, nodes, chunk_ptrs, L, Ls, objects, erased,
                                    [reps[e].data_ptr() for e in erased], Ls)
        regenerate()
        torch.cuda.synchronize(dev)
        r0, r1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        r0.record(stream)
        for _ in range(args.steps):
            regenerate()
        r1.record(stream)
        torch.cuda.synchronize(dev)
        regen_ms = r0.elapsed_time(r1) / args.steps
        if world > 1:
            regen_ms = max_over_ranks([regen_ms], dist, dev)[0]

    if world > 1:
        elapsed, enc_ms, rep_ms = max_over_ranks([elapsed, enc_ms, rep_ms], dist, dev)
        if aot_ms is not None:
            aot_ms = max_over_ranks([aot_ms], dist, dev)[0]

    # Replica names, also beside the metric: SHA-256 of
    # every replica of the batch, one lane per replica (reps is [n][objects][L]).
    digests = torch.empty((n * objects, 32), dtype=torch.uint8, device=dev)
    chunk.sha256_device(reps, L, Ls, n * objects, digests)
    torch.cuda.synchronize(dev)
    h0, h1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    h0.record(stream)
    chunk.sha256_device(reps, L, Ls, n * objects, digests)
    h1.record(stream)
    torch.cuda.synchronize(dev)
    sha_ms = h0.elapsed_time(h1)
    if world > 1:
        sha_ms = max_over_ranks([sha_ms], dist, dev)[0]

    ms_per_step = elapsed / args.steps * 1e3
    total_bytes = world * objects * size
    value = total_bytes / (elapsed / args.steps) / 2**30

    enc_bytes = objects * (size + n * L)      # S + n*(2*ceil(S/2k)+2)
    rep_bytes = objects * (k * L + size)      # k*L + S
    enc_name, rep_name = kernel_names(k, n, nodes, size, L, objects)
    if enc_ms >= rep_ms:
        dom, dom_bytes, dom_ms = enc_name, enc_bytes, enc_ms
    else:
        dom, dom_bytes, dom_ms = rep_name, rep_bytes, rep_ms
    achieved = dom_bytes / (dom_ms * 1e-3) / 1e9
    traffic, traffic_src = pmc_traffic(args.traffic_json, dom, objects, k, n)

    # The same encode + repair at a 16-byte replica stride (the
    # reference's malloc'd replica buffers guarantee 16-byte alignment only),
    # beside the metric: min(256, objects) of the same objects.
    align16 = None
    if args.replica_align != 16 and not args.no_align16:
        del reps, digests, regen_out
        torch.cuda.empty_cache()
        o16 = min(256, objects)
        L16 = replica_stride(L, 16)
        reps16 = torch.empty((n, o16 * L16), dtype=torch.uint8, device=dev)
        p16 = [reps16[i].data_ptr() for i in range(n)]
        c16 = [reps16[r].data_ptr() for r in nodes]

        def enc16():
            chunk.encode_device(k, list(range(n)), inp, size, size, o16, p16, L16)

        def rep16():
            chunk.restore_device(k, nodes, c16, L, L16, padding, o16, restored, size)

        enc16()
        rep16()
        torch.cuda.synchronize(dev)
        assert torch.equal(restored[:size], inp[:size]) and \
            torch.equal(restored[(o16 - 1) * size:o16 * size], inp[(o16 - 1) * size:o16 * size]), "align16 repair"
        a0, a1, a2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        e16 = r16 = 0.0
        for _ in range(args.steps):
            a0.record(stream)
            enc16()
            a1.record(stream)
            rep16()
            a2.record(stream)
            torch.cuda.synchronize(dev)
            e16 += a0.elapsed_time(a1)
            r16 += a1.elapsed_time(a2)
        e16, r16 = e16 / args.steps, r16 / args.steps
        if world > 1:
            e16, r16 = max_over_ranks([e16, r16], dist, dev)
        gb = world * o16 * size / 2**30
        align16 = {"replica_stride": L16, "objects_per_gpu": o16, "encode_GiBps": round(gb / (e16 * 1e-3), 3),
                   "repair_GiBps": round(gb / (r16 * 1e-3), 3), "value": round(gb / ((e16 + r16) * 1e-3), 3),
                   "encode_ms": round(e16, 3), "repair_ms": round(r16, 3)}
        del reps16

    if align16 is None:
        del reps, digests, regen_out
    del inp, restored
    torch.cuda.empty_cache()
    c4 = None
    if not args.no_c4:
        c4 = c4_leg(torch, chunk, dev, stream, args, rank, world, dist if world > 1 else None, c4_pre)
    live = None
    if not args.no_live:
        live = live_shape(torch, chunk, dev, torch.cuda.Stream(dev), args.live_objects, args.steps, args.warmup,
                          align=args.replica_align)

    result = {
        "metric": "device-resident encode+repair GiB/s, k=16 m=4 64 MiB stripes, 1/2/4/8 GPU",
        "value": round(value, 3),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u16",
        "data": "synthetic (splitmix64 objects generated on device)",
        "config": {"workload": f"k={k},m={m} encode of all {n} replicas + repair from {len(nodes)} "
                               f"(erased {erased}), {objects} x {size >> 20} MiB objects per GPU",
                   "k": k, "m": m, "objects_per_gpu": objects, "object_bytes": size,
                   "erased": erased, "replica_bytes": L, "replica_stride": Ls, "parallelism": f"objects round-robin over {world} GPU(s), no collective"},
        "encode_GiBps": round(world * objects * size / (enc_ms * 1e-3) / 2**30, 3),
        "repair_GiBps": round(world * objects * size / (rep_ms * 1e-3) / 2**30, 3),
        "encode_ms": round(enc_ms, 3),
        "repair_ms": round(rep_ms, 3),
        "regenerate_GiBps": round(world * objects * size / (regen_ms * 1e-3) / 2**30, 3) if regen_ms else None,
        "regenerate_ms": round(regen_ms, 3) if regen_ms else None,
        "sha256_replicas_GiBps": round(world * objects * n * L / (sha_ms * 1e-3) / 2**30, 3),
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic,
                     "traffic_source": traffic_src, "algorithmic_bytes_per_launch": dom_bytes,
                     "avg_launch_ms": round(dom_ms, 4), "kernels": {"encode": enc_name, "repair": rep_name}},
        "restore_kernel": restore_kernel,
        "restore_aot_ms": round(aot_ms, 3) if aot_ms is not None else None,
        "restore_aot": ({"kernel": aot_name, "repair_GiBps": round(world * objects * size / (aot_ms * 1e-3) / 2**30, 3),
                         "frac": round(rep_bytes / (aot_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)}
                        if aot_ms is not None else None),
        "c4": c4,
        "jit_wait_s": round(jit_s, 3) if jit_s is not None else None,
        "align16": align16,
        "live_shape": live,
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(k, n, size, nodes, args.cpu_objects)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
