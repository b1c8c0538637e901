"""Python mirror of lboss75/vds kernel/vds_data's chunk-transform API.

Same names, argument meaning and error behaviour as the reference's C++
templates (chunk.h:59-114, chunk_storage.h:13-34), backed by the HIP kernels
through the C ABI.  `cell_bytes` selects the uint16_t (2, production) or
uint8_t (1) instantiation.

  ChunkGenerator(k, n).write(data, write_padding=True)   chunk.h:245-281
  ChunkGenerator.write_padding(size)                     chunk.h:283-287
  chunk_cells(generator, cells)                          chunk.h:206-224
  ChunkRestore(k, nodes).restore(chunks)                 chunk.h:290-444
  ChunkRestore.restore_cells(chunks)                     chunk.h:383-400
  ChunkStorage(min_horcrux).generate_replica / restore_data
                                                         chunk_storage.cpp:41-86
  encode_device / restore_device                          batched device-memory
                                                         forms for torch tensors
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Dict, Iterable, Mapping, Sequence

import numpy as np

from . import _lib
from ._lib import F_CELLS, F_NO_TRAILER, VdsEcError, check

__all__ = [
    "ChunkGenerator", "ChunkRestore", "ChunkStorage", "chunk_cells", "replica_size",
    "encode_device", "restore_device", "fill_splitmix_device", "encode_host_batch", "restore_host_batch",
    "regenerate_host",
    "regenerate_device", "sha256_device", "encode_hash_host", "replica_storage_paths",
    "VdsEcError", "multipliers", "inverse", "encode_range_device", "restore_range_device", "encode_host_split",
    "restore_host_split",
]


def _u8(data) -> np.ndarray:
    if isinstance(data, (bytes, bytearray, memoryview)):
        return np.frombuffer(bytes(data), dtype=np.uint8)
    return np.ascontiguousarray(data).view(np.uint8).reshape(-1)


def _ids(values: Iterable[int], cell_bytes: int) -> np.ndarray:
    dt = np.uint16 if cell_bytes == 2 else np.uint8
    return np.ascontiguousarray(np.asarray(list(values), dtype=np.int64).astype(dt))


def _idp(a: np.ndarray, cell_bytes: int):
    return a.ctypes.data_as(_lib.u16p if cell_bytes == 2 else _lib.u8p)


def replica_size(k: int, size: int, cell_bytes: int = 2, write_padding: bool = True) -> int:
    return int(_lib.lib().vds_ec_replica_size(cell_bytes, k, size, 0 if write_padding else F_NO_TRAILER))


def multipliers(k: int, node: int, cell_bytes: int = 2) -> np.ndarray:
    """chunk<cell>::generate_multipliers (chunk.h:183-194)."""
    dt = np.uint16 if cell_bytes == 2 else np.uint8
    out = np.zeros(k, dtype=dt)
    f = _lib.lib().vds_ec_multipliers16 if cell_bytes == 2 else _lib.lib().vds_ec_multipliers8
    check(f(k, node, _idp(out, cell_bytes)))
    return out


def inverse(k: int, nodes: Sequence[int], cell_bytes: int = 2) -> np.ndarray:
    """The chunk_restore<cell>(k, n) multipliers matrix (chunk.h:290-375)."""
    ids = _ids(nodes, cell_bytes)
    dt = np.uint16 if cell_bytes == 2 else np.uint8
    out = np.zeros(k * k, dtype=dt)
    f = _lib.lib().vds_ec_inverse16 if cell_bytes == 2 else _lib.lib().vds_ec_inverse8
    check(f(k, _idp(ids, cell_bytes), _idp(out, cell_bytes)), "chunk_restore")
    return out.reshape(k, k)


class ChunkGenerator:
    """chunk_generator<cell>(k, n) (chunk.h:59-88, 232-243)."""

    def __init__(self, k: int, n: int, cell_bytes: int = 2):
        if cell_bytes not in (1, 2):
            raise ValueError("cell_bytes must be 1 (uint8_t) or 2 (uint16_t)")
        limit = 0xFFFF if cell_bytes == 2 else 0xFF
        self._k = int(k) & limit  # cell_type arithmetic
        self._n = int(n) & limit
        self.cell_bytes = cell_bytes
        self._mult = multipliers(self._k, self._n, cell_bytes)

    def k(self) -> int:
        return self._k

    def n(self) -> int:
        return self._n

    def multipliers(self) -> np.ndarray:
        return self._mult

    def write(self, data, write_padding: bool = True) -> np.ndarray:
        """Bytes chunk_generator::write appends to the serializer."""
        return encode_host(self._k, [self._n], data, self.cell_bytes, write_padding)[0]

    def write_padding(self, size: int) -> np.ndarray:
        pad = size % (self.cell_bytes * self._k)  # chunk.h:286
        return np.array([(pad >> 8) & 0xFF, pad & 0xFF], dtype=np.uint8)


def encode_host(k: int, replicas: Sequence[int], data, cell_bytes: int = 2,
                write_padding: bool = True, cells: bool = False) -> list:
    """All requested replicas of one host object in one device pass."""
    buf = _u8(data)
    ids = _ids(replicas, cell_bytes)
    flags = (0 if write_padding else F_NO_TRAILER) | (F_CELLS if cells else 0)
    L = int(_lib.lib().vds_ec_replica_size(cell_bytes, k, buf.size, flags))
    outs = [np.empty(max(L, 1), dtype=np.uint8) for _ in range(ids.size)]
    ptrs = (C.c_void_p * max(1, ids.size))(*[o.ctypes.data for o in outs])
    f = _lib.lib().vds_ec_encode16_host if cell_bytes == 2 else _lib.lib().vds_ec_encode8_host
    check(f(k, _idp(ids, cell_bytes), ids.size, buf.ctypes.data if buf.size else None, buf.size, ptrs, flags),
          "chunk_generator::write")
    return [o[:L] for o in outs]


def chunk_cells(generator: ChunkGenerator, cells) -> np.ndarray:
    """chunk<cell>(generator, data, len).data() (chunk.h:206-224)."""
    dt = np.uint16 if generator.cell_bytes == 2 else np.uint8
    arr = np.ascontiguousarray(cells, dtype=dt)
    out = encode_host(generator.k(), [generator.n()], arr.view(np.uint8), generator.cell_bytes, cells=True)[0]
    return out.view(dt).copy()


class ChunkRestore:
    """chunk_restore<cell>(k, n) (chunk.h:90-114, 290-444)."""

    def __init__(self, k: int, nodes: Sequence[int], cell_bytes: int = 2):
        self._k = int(k)
        self.cell_bytes = cell_bytes
        self._nodes = _ids(nodes, cell_bytes)
        if self._nodes.size < self._k:
            raise ValueError("chunk_restore needs k replica ids")
        self._nodes = self._nodes[: self._k]
        self._error = None
        try:
            self._mult = inverse(self._k, self._nodes, cell_bytes)
        except VdsEcError as e:  # duplicate ids: the reference yields garbage here
            self._mult = None
            self._error = e

    def multipliers(self) -> np.ndarray:
        if self._error is not None:
            raise self._error
        return self._mult

    def restore(self, chunks: Sequence) -> np.ndarray:
        """chunk_restore::restore(const std::vector<const_data_buffer>&)."""
        if self._error is not None:
            raise self._error
        bufs = [_u8(c) for c in chunks[: self._k]]
        if len(bufs) < self._k:
            raise VdsEcError(_lib.EINVAL, "chunk_restore::restore")
        size = bufs[0].size
        if any(b.size != size for b in bufs):
            raise VdsEcError(_lib.EINVAL, "chunk_restore::restore")
        # a corrupt trailer can make the reference return up to size*k bytes (chunk.h:415-441)
        out = np.empty(max(1, size * self._k), dtype=np.uint8)
        out_size = C.c_uint64(0)
        ptrs = (C.c_void_p * self._k)(*[b.ctypes.data for b in bufs])
        f = _lib.lib().vds_ec_restore16_host if self.cell_bytes == 2 else _lib.lib().vds_ec_restore8_host
        check(f(self._k, _idp(self._nodes, self.cell_bytes), ptrs, size, out.ctypes.data, C.byref(out_size), 0),
              "chunk_restore::restore")
        return out[: out_size.value]

    def restore_cells(self, chunks: Sequence) -> np.ndarray:
        """chunk_restore::restore(std::vector<cell>&, const chunk<cell>**)."""
        if self._error is not None:
            raise self._error
        dt = np.uint16 if self.cell_bytes == 2 else np.uint8
        arrs = [np.ascontiguousarray(c, dtype=dt) for c in chunks[: self._k]]
        n_cells = arrs[0].size
        out = np.empty(max(1, n_cells * self._k), dtype=dt)
        out_size = C.c_uint64(0)
        ptrs = (C.c_void_p * self._k)(*[a.ctypes.data for a in arrs])
        f = _lib.lib().vds_ec_restore16_host if self.cell_bytes == 2 else _lib.lib().vds_ec_restore8_host
        check(f(self._k, _idp(self._nodes, self.cell_bytes), ptrs, n_cells * self.cell_bytes, out.ctypes.data,
                C.byref(out_size), F_CELLS), "chunk_restore::restore")
        return out[: n_cells * self._k]


class ChunkStorage:
    """chunk_storage (chunk_storage.h:13-34, chunk_storage.cpp:10-86)."""

    def __init__(self, min_horcrux: int):
        self.min_horcrux = int(min_horcrux) & 0xFFFF
        self._generators: Dict[int, ChunkGenerator] = {}

    def generate_replica(self, replica: int, data) -> np.ndarray:
        g = self._generators.get(replica)
        if g is None:
            g = self._generators[replica] = ChunkGenerator(self.min_horcrux, replica)
        return g.write(data)

    def generate_replicas(self, replicas: Sequence[int], data) -> list:
        """Batched form of generate_replica for the save_temp / save_data loops."""
        return encode_host(self.min_horcrux, replicas, data)

    def regenerate_replicas(self, horcruxes: Mapping[int, object], targets: Sequence[int]) -> list:
        """Replicas `targets` from exactly min_horcrux equal-size horcruxes, in
        one pass (the repair's restore_data + generate_replica, fused)."""
        if self.min_horcrux != len(horcruxes):
            raise VdsEcError(_lib.EINVAL, "Error at restoring data")
        items = list(horcruxes.items())
        return regenerate_host(self.min_horcrux, [r for r, _ in items], [v for _, v in items], targets)

    def restore_data(self, horcruxes: Mapping[int, object]) -> np.ndarray:
        if self.min_horcrux != len(horcruxes):
            raise VdsEcError(_lib.EINVAL, "Error at restoring data")  # chunk_storage.cpp:65-67
        items = list(horcruxes.items())
        size = _u8(items[0][1]).size
        for _, v in items:
            if _u8(v).size != size:
                raise VdsEcError(_lib.EINVAL, "Error at restoring data")  # chunk_storage.cpp:76-78
        return ChunkRestore(self.min_horcrux, [r for r, _ in items]).restore([v for _, v in items])


# --------------------------------------------------------------- device forms

def _stream_ptr(stream) -> int | None:
    """A hipStream_t for the C ABI: None = torch's current stream; a
    torch.cuda.Stream or a raw handle otherwise."""
    if stream is None:
        import torch
        return torch.cuda.current_stream().cuda_stream
    if hasattr(stream, "cuda_stream"):
        return stream.cuda_stream
    return int(stream)


def encode_device(k: int, replicas: Sequence[int], inp, size: int, in_stride: int, count: int,
                  outs: Sequence[int], out_stride: int, write_padding: bool = True, stream=None) -> None:
    """vds_ec_encode16_device on raw device pointers (ints) / torch tensors."""
    ids = _ids(replicas, 2)
    ptrs = (C.c_void_p * ids.size)(*[int(o) for o in outs])
    in_ptr = inp.data_ptr() if hasattr(inp, "data_ptr") else int(inp)
    check(_lib.lib().vds_ec_encode16_device(k, _idp(ids, 2), ids.size, in_ptr, size, in_stride, count, ptrs,
                                            out_stride, 0 if write_padding else F_NO_TRAILER,
                                            _stream_ptr(stream)), "encode16_device")


def restore_device(k: int, nodes: Sequence[int], chunks: Sequence[int], chunk_size: int, chunk_stride: int,
                   padding: int, count: int, out, out_stride: int, stream=None) -> None:
    ids = _ids(nodes, 2)
    ptrs = (C.c_void_p * ids.size)(*[int(c) for c in chunks])
    out_ptr = out.data_ptr() if hasattr(out, "data_ptr") else int(out)
    check(_lib.lib().vds_ec_restore16_device(k, _idp(ids, 2), ptrs, chunk_size, chunk_stride, padding, count,
                                             out_ptr, out_stride, 0, _stream_ptr(stream)), "restore16_device")


def encode_range_device(k: int, replicas: Sequence[int], inp, size: int, t0: int, t1: int, outs: Sequence[int],
                        write_padding: bool = True, stream=None) -> None:
    """vds_ec_encode16_range_device: stripes [t0, t1) of one device object
    into replica bytes [2 t0, 2 t1) of the whole replica buffers `outs`
    (SURVEY.md 8(e) stripe-range split)."""
    ids = _ids(replicas, 2)
    ptrs = (C.c_void_p * max(1, ids.size))(*[int(o) for o in outs])
    in_ptr = inp.data_ptr() if hasattr(inp, "data_ptr") else int(inp)
    check(_lib.lib().vds_ec_encode16_range_device(k, _idp(ids, 2), ids.size, in_ptr, size, t0, t1, ptrs,
                                                  0 if write_padding else F_NO_TRAILER, _stream_ptr(stream)),
          "encode16_range_device")


def restore_range_device(k: int, nodes: Sequence[int], chunks: Sequence[int], chunk_size: int, padding: int,
                         t0: int, t1: int, out, stream=None) -> None:
    """vds_ec_restore16_range_device: object bytes [2k t0, min(2k t1, E)) of
    `out` from stripes [t0, t1) of the whole survivor buffers."""
    ids = _ids(nodes, 2)
    ptrs = (C.c_void_p * ids.size)(*[int(c) for c in chunks])
    out_ptr = out.data_ptr() if hasattr(out, "data_ptr") else int(out)
    check(_lib.lib().vds_ec_restore16_range_device(k, _idp(ids, 2), ptrs, chunk_size, padding, t0, t1, out_ptr, 0,
                                                   _stream_ptr(stream)), "restore16_range_device")


def encode_host_split(k: int, replicas: Sequence[int], data, parts: int = 0, max_devices: int = 0) -> list:
    """One host object over the GPUs by stripe ranges (vds_ec_encode16_host_split);
    returns the n replicas."""
    ids = _ids(replicas, 2)
    buf = _u8(data)
    L = replica_size(k, buf.size)
    outs = [np.empty(max(L, 1), dtype=np.uint8) for _ in range(ids.size)]
    ptrs = (C.c_void_p * max(1, ids.size))(*[o.ctypes.data for o in outs])
    check(_lib.lib().vds_ec_encode16_host_split(k, _idp(ids, 2), ids.size, buf.ctypes.data, buf.size, ptrs, 0,
                                                max_devices, parts), "encode16_host_split")
    return [o[:L] for o in outs]


def restore_host_split(k: int, nodes: Sequence[int], chunks: Sequence, parts: int = 0, max_devices: int = 0):
    """One object restored over the GPUs by stripe ranges from k host
    replicas (vds_ec_restore16_host_split); returns the restored bytes."""
    ids = _ids(nodes, 2)
    bufs = [_u8(c) for c in chunks]
    cs = bufs[0].size
    out = np.empty(max(cs * k, 1), dtype=np.uint8)
    n_out = C.c_uint64(out.size)
    ptrs = (C.c_void_p * ids.size)(*[b.ctypes.data for b in bufs])
    check(_lib.lib().vds_ec_restore16_host_split(k, _idp(ids, 2), ptrs, cs, out.ctypes.data, C.byref(n_out), 0,
                                                 max_devices, parts), "restore16_host_split")
    return out[: n_out.value]


def restore_batch_device(k: int, nodes: Sequence[Sequence[int]], chunks: Sequence[Sequence[int]],
                         chunk_sizes: Sequence[int], paddings: Sequence[int], outs: Sequence[int],
                         stream=None) -> None:
    """vds_ec_restore16_batch_device: object o restored from its own survivors
    nodes[o] at device pointers chunks[o] (chunk_sizes[o] bytes, trailer
    value paddings[o]) into the device pointer outs[o]."""
    count = len(nodes)
    ids = _ids([r for nd in nodes for r in nd], 2)
    cp = (C.c_void_p * max(1, count * k))(*[int(c) for ch in chunks for c in ch])
    cs = np.asarray(chunk_sizes, dtype=np.uint64)
    pd = np.asarray(paddings, dtype=np.uint16)
    op = (C.c_void_p * max(1, count))(*[int(o) for o in outs])
    check(_lib.lib().vds_ec_restore16_batch_device(k, count, _idp(ids, 2), cp, cs.ctypes.data_as(_lib.u64p),
                                                   pd.ctypes.data_as(_lib.u16p), op, 0, _stream_ptr(stream)),
          "restore16_batch_device")


def regenerate_batch_device(k: int, nodes: Sequence[Sequence[int]], chunks: Sequence[Sequence[int]],
                            chunk_sizes: Sequence[int], targets: Sequence[Sequence[int]],
                            outs: Sequence[Sequence[int]], stream=None) -> None:
    """vds_ec_regenerate16_batch_device: replicas targets[o] of object o from
    its own survivors, into the device pointers outs[o]."""
    count = len(nodes)
    nt = len(targets[0]) if count else 0
    ids = _ids([r for nd in nodes for r in nd], 2)
    tg = _ids([t for ts in targets for t in ts], 2)
    cp = (C.c_void_p * max(1, count * k))(*[int(c) for ch in chunks for c in ch])
    cs = np.asarray(chunk_sizes, dtype=np.uint64)
    op = (C.c_void_p * max(1, count * nt))(*[int(x) for os_ in outs for x in os_])
    check(_lib.lib().vds_ec_regenerate16_batch_device(k, count, _idp(ids, 2), cp, cs.ctypes.data_as(_lib.u64p), nt,
                                                      _idp(tg, 2), op, _stream_ptr(stream)),
          "regenerate16_batch_device")


def regenerate_host(k: int, nodes: Sequence[int], chunks: Sequence, targets: Sequence[int]) -> list:
    """vds_ec_regenerate16_host: replicas `targets` of one object from k
    survivor replicas (host buffers), bytes as restore + re-encode."""
    ids = _ids(nodes, 2)[:k]
    tg = _ids(targets, 2)
    bufs = [_u8(c) for c in chunks[:k]]
    if len(bufs) < k or any(b.size != bufs[0].size for b in bufs):
        raise VdsEcError(_lib.EINVAL, "regenerate")
    size = bufs[0].size
    outs = [np.empty(max(size, 1), dtype=np.uint8) for _ in range(tg.size)]
    cp = (C.c_void_p * k)(*[b.ctypes.data for b in bufs])
    op = (C.c_void_p * max(1, tg.size))(*[o.ctypes.data for o in outs])
    check(_lib.lib().vds_ec_regenerate16_host(k, _idp(ids, 2), cp, size, _idp(tg, 2), tg.size, op), "regenerate")
    return [o[:size] for o in outs]


def regenerate_device(k: int, nodes: Sequence[int], chunks: Sequence[int], chunk_size: int, chunk_stride: int,
                      count: int, targets: Sequence[int], outs: Sequence[int], out_stride: int, stream=None) -> None:
    ids = _ids(nodes, 2)
    tg = _ids(targets, 2)
    cp = (C.c_void_p * ids.size)(*[int(c) for c in chunks])
    op = (C.c_void_p * max(1, tg.size))(*[int(o) for o in outs])
    check(_lib.lib().vds_ec_regenerate16_device(k, _idp(ids, 2), cp, chunk_size, chunk_stride, count, _idp(tg, 2),
                                                tg.size, op, out_stride, _stream_ptr(stream)), "regenerate16_device")


def sha256_device(base, length: int, stride: int, count: int, digests, stream=None) -> None:
    """SHA-256 of `count` device messages of `length` bytes at base + j*stride
    into digests (device, 32*count bytes): the replica names of
    dht_network_client.cpp:79 / :593."""
    bp = base.data_ptr() if hasattr(base, "data_ptr") else int(base)
    dp = digests.data_ptr() if hasattr(digests, "data_ptr") else int(digests)
    check(_lib.lib().vds_ec_sha256_device(bp, length, stride, count, dp, _stream_ptr(stream)), "sha256_device")


def encode_hash_host(k: int, replicas: Sequence[int], data, write_padding: bool = True):
    """All requested replicas of one host object plus their SHA-256 names
    (save_temp / save_data: write, then hash::signature(sha256, replica))."""
    buf = _u8(data)
    ids = _ids(replicas, 2)
    flags = 0 if write_padding else F_NO_TRAILER
    L = replica_size(k, buf.size, 2, write_padding)
    outs = [np.empty(max(L, 1), dtype=np.uint8) for _ in range(ids.size)]
    digests = np.empty((max(1, ids.size), 32), dtype=np.uint8)
    ptrs = (C.c_void_p * max(1, ids.size))(*[o.ctypes.data for o in outs])
    check(_lib.lib().vds_ec_encode16_hash_host(k, _idp(ids, 2), ids.size, buf.ctypes.data if buf.size else None,
                                               buf.size, ptrs, digests.ctypes.data, flags), "encode16_hash_host")
    return [o[:L] for o in outs], [bytes(d) for d in digests[: ids.size]]


def replica_storage_paths(digests) -> list:
    """Storage paths <b64[0:10]>/<b64[10:20]>/<b64[20:]> of replicas from their
    SHA-256 names (dht_network_client.cpp:483-505; base64 with '+' -> '#',
    '/' -> '_').  Host-only."""
    d = np.ascontiguousarray(np.frombuffer(b"".join(bytes(x) for x in digests), dtype=np.uint8))
    count = d.size // 32
    out = np.zeros(48 * max(count, 1), dtype=np.uint8)
    check(_lib.lib().vds_ec_replica_paths(d.ctypes.data if count else None, count, out.ctypes.data), "replica_paths")
    return [bytes(out[48 * i:48 * i + 46]).decode() for i in range(count)]


# ------------------------------------------------- upload path (wire formats)

def base64_decode(text) -> bytes:
    """base64::to_bytes (encoding.cpp:181-247), reference quirks included;
    raises VdsEcError with the reference's message on malformed input."""
    raw = text.encode() if isinstance(text, str) else bytes(text)
    size = _lib.lib().vds_ec_base64_decoded_size(raw, len(raw))
    out = np.empty(max(1, size), dtype=np.uint8)
    n = C.c_size_t(0)
    check(_lib.lib().vds_ec_base64_decode(raw, len(raw), out.ctypes.data, C.byref(n)), "base64_decode")
    return bytes(out[: n.value])


def base64_encode(data) -> str:
    """base64::from_bytes (encoding.cpp:138-174)."""
    buf = _u8(data)
    n = C.c_size_t(0)
    lib = _lib.lib()
    check(lib.vds_ec_base64_encode(buf.ctypes.data if buf.size else None, buf.size, None, 0, C.byref(n)))
    out = C.create_string_buffer(n.value + 1)
    check(lib.vds_ec_base64_encode(buf.ctypes.data if buf.size else None, buf.size, out, n.value + 1, C.byref(n)))
    return out.value.decode()


def tmp_names(digests) -> list:
    """save_temp's tmp-file names of replicas (dht_network_client.cpp:91-95)."""
    d = np.ascontiguousarray(np.frombuffer(b"".join(bytes(x) for x in digests), dtype=np.uint8))
    count = d.size // 32
    out = np.zeros(45 * max(count, 1), dtype=np.uint8)
    check(_lib.lib().vds_ec_tmp_names(d.ctypes.data if count else None, count, out.ctypes.data), "tmp_names")
    return [bytes(out[45 * i:45 * i + 44]).decode() for i in range(count)]


def upload_response_json(req_id: int, replica_digests, data_digest, replica_size: int) -> str:
    """The websocket answer to "upload" (websocket_api.cpp:120-121, 472-482)."""
    d = np.ascontiguousarray(np.frombuffer(b"".join(bytes(x) for x in replica_digests), dtype=np.uint8))
    n = d.size // 32
    h = np.frombuffer(bytes(data_digest), dtype=np.uint8).copy()
    ln = C.c_size_t(0)
    lib = _lib.lib()
    args = (req_id, d.ctypes.data if n else None, n, h.ctypes.data, replica_size)
    check(lib.vds_ec_upload_response_json(*args, None, 0, C.byref(ln)))
    out = C.create_string_buffer(ln.value + 1)
    check(lib.vds_ec_upload_response_json(*args, out, ln.value + 1, C.byref(ln)))
    return out.value.decode()


def save_temp(k: int, n: int, body):
    """upload_data + save_temp on the device (server_api.cpp:12-30,
    dht_network_client.cpp:62-107): replicas 0..n-1 of `body`, their SHA-256
    names, the body's SHA-256 and the replica size."""
    buf = _u8(body)
    L = replica_size(k, buf.size)
    outs = [np.empty(max(L, 1), dtype=np.uint8) for _ in range(n)]
    rd = np.empty((max(1, n), 32), dtype=np.uint8)
    dd = np.empty(32, dtype=np.uint8)
    rs = C.c_uint32(0)
    ptrs = (C.c_void_p * max(1, n))(*[o.ctypes.data for o in outs])
    check(_lib.lib().vds_ec_save_temp16_host(k, n, buf.ctypes.data if buf.size else None, buf.size, ptrs,
                                             rd.ctypes.data, dd.ctypes.data, C.byref(rs)), "save_temp16_host")
    return [o[:L] for o in outs], [bytes(x) for x in rd[:n]], bytes(dd), rs.value


def upload(req_id: int, body_b64, k: int = 32, n: int = 64):
    """The live upload end to end: websocket "upload" body (base64) ->
    replicas, tmp-file names and the JSON answer (MIN_HORCRUX = 32,
    GENERATE_HORCRUX = 64 by default, dht_network.h:22-25)."""
    body = base64_decode(body_b64)
    reps, names, data_hash, rsize = save_temp(k, n, body)
    return {"replicas": reps, "tmp_names": tmp_names(names), "replica_digests": names, "data_hash": data_hash,
            "json": upload_response_json(req_id, names, data_hash, rsize)}


def restore_path(k: int, nodes: Sequence[int], chunk_size: int, padding: int = 0, count: int = 1) -> int:
    """vds_ec_restore16_path: 4 = the survivor set's run-time compiled kernel,
    3 = k_restore_syn, 2 = k_restore_bs, 1 = generic only."""
    a = _ids(nodes, 2)
    return int(_lib.lib().vds_ec_restore16_path(k, _idp(a, 2), chunk_size, padding, count))


def jit_set_mode(mode: int) -> None:
    """0 = off, 1 = background compiles from a survivor set's second use
    (default), 2 = compile at the first use (vds_ec_jit_set_mode)."""
    check(_lib.lib().vds_ec_jit_set_mode(mode))


def jit_wait() -> None:
    """Block until the library's run-time compiles of survivor-set-specific
    restore kernels (vds_ec_jit_*) are done."""
    check(_lib.lib().vds_ec_jit_wait())


def jit_build(k: int, nodes: Sequence[int]) -> int:
    """Compile (no device needed) the restore kernel of survivor set `nodes`;
    returns its code object size."""
    a = _ids(nodes, 2)
    out = C.c_uint64(0)
    check(_lib.lib().vds_ec_jit_build16(k, _idp(a, 2), C.byref(out)))
    return out.value


def jit_ready(k: int, nodes: Sequence[int]) -> bool:
    a = _ids(nodes, 2)
    return bool(_lib.lib().vds_ec_jit_ready16(k, _idp(a, 2)))


def jit_dump(k: int, nodes: Sequence[int], directory: str, regen: bool = False) -> None:
    """Compile (no device needed) the kernel of survivor set `nodes` and write
    its source and code object into `directory` (vds_ec_jit_dump16)."""
    a = _ids(nodes, 2)
    check(_lib.lib().vds_ec_jit_dump16(k, _idp(a, 2), 1 if regen else 0, os.fsencode(directory)))


def fill_splitmix_device(dst, size: int, seed: int, stream=None) -> None:
    ptr = dst.data_ptr() if hasattr(dst, "data_ptr") else int(dst)
    check(_lib.lib().vds_ec_fill_splitmix_device(ptr, size, seed, _stream_ptr(stream)), "fill_splitmix")


def restore_host_batch(k: int, nodes: Sequence, chunks: Sequence[Sequence], max_devices: int = 0,
                       outs: list | None = None) -> list:
    """Multi-GPU host-memory restore of many objects (chunk_storage::restore_data
    per object, chunk_storage.cpp:62-85).  `chunks[o]` are the k replicas of
    object o, holding replica ids `nodes[o]` (or one id list for every object).
    `outs[o]` (optional) are caller-owned uint8 buffers; each must hold the
    restored object.  Returns the restored objects (trailer-trimmed, as
    restore16_host), as views of `outs` when given."""
    count = len(chunks)
    per = [list(nodes)] * count if count and np.ndim(nodes) == 1 else [list(n) for n in nodes]
    if len(per) != count or any(len(n) != k or len(c) != k for n, c in zip(per, chunks)):
        raise VdsEcError(_lib.EINVAL, "restore_host_batch: need k ids and k chunks per object")
    bufs = [[_u8(c) for c in row] for row in chunks]
    if any(c.size != row[0].size for row in bufs for c in row):  # chunk_storage.cpp:73-76
        raise VdsEcError(_lib.EINVAL, "restore_host_batch: chunks of one object differ in size")
    sizes = np.array([row[0].size for row in bufs], dtype=np.uint64)
    ids = np.ascontiguousarray(np.array(per, dtype=np.uint16).reshape(-1))
    if outs is None:
        outs = [np.empty(max(int(s) * k, 1), dtype=np.uint8) for s in sizes]
    outs = [_u8(o) for o in outs]
    if len(outs) != count:
        raise VdsEcError(_lib.EINVAL, "restore_host_batch: one output buffer per object")
    caps = np.array([o.size for o in outs], dtype=np.uint64)
    cptrs = (C.c_void_p * max(1, count * k))(*[c.ctypes.data for row in bufs for c in row])
    optrs = (C.c_void_p * max(1, count))(*[o.ctypes.data for o in outs])
    check(_lib.lib().vds_ec_restore16_host_batch(k, ids.ctypes.data_as(_lib.u16p), cptrs,
                                                 sizes.ctypes.data_as(_lib.u64p), count, optrs,
                                                 caps.ctypes.data_as(_lib.u64p), 0, max_devices),
          "restore16_host_batch")
    return [o[: int(n)] for o, n in zip(outs, caps)]


def encode_host_batch(k: int, replicas: Sequence[int], objects: Sequence, max_devices: int = 0,
                      outs: list | None = None) -> list:
    """Multi-GPU host-memory encode (one thread + pinned ring per device).
    `outs[o][i]` (optional) are caller-owned uint8 buffers of at least
    replica_size(k, len(objects[o])) bytes that receive replica i of object o."""
    ids = _ids(replicas, 2)
    bufs = [_u8(o) for o in objects]
    sizes = np.array([b.size for b in bufs], dtype=np.uint64)
    if outs is None:
        outs = [[np.empty(max(replica_size(k, b.size), 1), dtype=np.uint8) for _ in range(ids.size)] for b in bufs]
    for row, b in zip(outs, bufs):
        if len(row) != ids.size or any(_u8(o).size < replica_size(k, b.size) for o in row):
            raise VdsEcError(_lib.EINVAL, "encode_host_batch: output buffer too small")
    optrs = (C.c_void_p * (len(bufs) * ids.size))(*[o.ctypes.data for row in outs for o in row])
    iptrs = (C.c_void_p * max(1, len(bufs)))(*[b.ctypes.data for b in bufs])
    check(_lib.lib().vds_ec_encode16_host_batch(k, _idp(ids, 2), ids.size, iptrs,
                                                sizes.ctypes.data_as(_lib.u64p), len(bufs), optrs, 0,
                                                max_devices), "encode16_host_batch")
    return [[o[: replica_size(k, b.size)] for o in row] for row, b in zip(outs, bufs)]


class PinnedBuffer:
    """Caller-owned pinned host memory (vds_ec_host_alloc): page-locked,
    device-mapped.  Host batches whose objects, replicas, survivors or outputs
    lie back to back in such a buffer read and write it directly (no staging
    copies).  `.array` is a uint8 numpy view; close() (or del) frees it."""

    def __init__(self, nbytes: int):
        p = C.c_void_p()
        check(_lib.lib().vds_ec_host_alloc(int(nbytes), C.byref(p)), "host_alloc")
        self.ptr, self.nbytes = p.value, int(nbytes)
        self.array = np.ctypeslib.as_array((C.c_uint8 * self.nbytes).from_address(self.ptr))

    def close(self) -> None:
        if self.ptr:
            self.array = None
            check(_lib.lib().vds_ec_host_free(self.ptr), "host_free")
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 (interpreter teardown)
            pass


def host_register(arr) -> None:
    """Pin (and map) a caller's contiguous numpy buffer for the host batches
    (vds_ec_host_register); host_unregister before it is freed."""
    a = _u8(arr)
    check(_lib.lib().vds_ec_host_register(a.ctypes.data, a.size), "host_register")


def host_unregister(arr) -> None:
    check(_lib.lib().vds_ec_host_unregister(_u8(arr).ctypes.data), "host_unregister")
