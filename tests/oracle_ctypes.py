"""ctypes binding of the CPU oracle (oracle/liboracle.so) -- TEST INFRASTRUCTURE.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module.  The oracle restates lboss75/vds kernel/vds_data (gf.h, chunk.h);
see oracle/vds_oracle.h for the per-function reference citations.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB_PATH = os.path.join(ORACLE_DIR, "liboracle.so")
REF_GF = os.path.join(ORACLE_DIR, "_ref", "gf_ref")

_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", ORACLE_DIR, "liboracle.so"], check=True)


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = C.CDLL(LIB_PATH)
        u8p = C.POINTER(C.c_uint8)
        u16p = C.POINTER(C.c_uint16)
        _lib.vds_oracle_gf_mul_bitserial.restype = C.c_uint32
        _lib.vds_oracle_gf_mul_bitserial.argtypes = [C.c_uint, C.c_uint32, C.c_uint32, C.c_uint32]
        for n, t in (("gf16", C.c_uint16), ("gf8", C.c_uint8)):
            for op in ("mul", "div"):
                f = getattr(_lib, f"vds_oracle_{n}_{op}")
                f.restype = t
                f.argtypes = [t, t]
        _lib.vds_oracle_replica_size.restype = C.c_size_t
        _lib.vds_oracle_replica_size.argtypes = [C.c_uint, C.c_uint, C.c_size_t, C.c_int]
        _lib.vds_oracle_encode16.restype = C.c_size_t
        _lib.vds_oracle_encode16.argtypes = [C.c_uint16, C.c_uint16, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p]
        _lib.vds_oracle_encode8.restype = C.c_size_t
        _lib.vds_oracle_encode8.argtypes = [C.c_uint8, C.c_uint8, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p]
        _lib.vds_oracle_inverse16.restype = C.c_int
        _lib.vds_oracle_inverse16.argtypes = [C.c_uint16, u16p, u16p]
        _lib.vds_oracle_inverse8.restype = C.c_int
        _lib.vds_oracle_inverse8.argtypes = [C.c_uint8, u8p, u8p]
        _lib.vds_oracle_restore16.restype = C.c_size_t
        _lib.vds_oracle_restore16.argtypes = [C.c_uint16, u16p, C.POINTER(C.c_void_p), C.c_size_t, C.c_void_p]
        _lib.vds_oracle_restore8.restype = C.c_size_t
        _lib.vds_oracle_restore8.argtypes = [C.c_uint8, u8p, C.POINTER(C.c_void_p), C.c_size_t, C.c_void_p]
        _lib.vds_oracle_chunk_cells16.restype = C.c_size_t
        _lib.vds_oracle_chunk_cells16.argtypes = [C.c_uint16, C.c_uint16, C.c_void_p, C.c_size_t, C.c_void_p]
        _lib.vds_oracle_chunk_cells8.restype = C.c_size_t
        _lib.vds_oracle_chunk_cells8.argtypes = [C.c_uint8, C.c_uint8, C.c_void_p, C.c_size_t, C.c_void_p]
        _lib.vds_oracle_restore_cells16.restype = None
        _lib.vds_oracle_restore_cells16.argtypes = [C.c_uint16, u16p, C.POINTER(C.c_void_p), C.c_size_t, C.c_void_p]
        _lib.vds_oracle_restore_cells8.restype = None
        _lib.vds_oracle_restore_cells8.argtypes = [C.c_uint8, u8p, C.POINTER(C.c_void_p), C.c_size_t, C.c_void_p]
        _lib.vds_oracle_splitmix_fill.restype = None
        _lib.vds_oracle_splitmix_fill.argtypes = [C.c_uint64, C.c_void_p, C.c_size_t]
        for n in ("gf16_mul_n", "gf16_div_n", "gf8_mul_n", "gf8_div_n"):
            f = getattr(_lib, f"vds_oracle_{n}")
            f.restype = None
            f.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t]
    return _lib


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


def splitmix(seed: int, size: int) -> np.ndarray:
    out = np.empty(size, dtype=np.uint8)
    lib().vds_oracle_splitmix_fill(seed, _ptr(out), size)
    return out


def gf_mul_bitserial(m: int, poly_low: int, a: int, b: int) -> int:
    return lib().vds_oracle_gf_mul_bitserial(m, poly_low, a, b)


def gf16_mul(a: int, b: int) -> int:
    return lib().vds_oracle_gf16_mul(a, b)


def gf16_div(a: int, b: int) -> int:
    return lib().vds_oracle_gf16_div(a, b)


def gf8_mul(a: int, b: int) -> int:
    return lib().vds_oracle_gf8_mul(a, b)


def gf8_div(a: int, b: int) -> int:
    return lib().vds_oracle_gf8_div(a, b)


def bulk(op: str, a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """op in gf16_mul/gf16_div/gf8_mul/gf8_div (element-wise)."""
    a = np.ascontiguousarray(a)
    b = np.ascontiguousarray(b)
    out = np.empty_like(a)
    getattr(lib(), f"vds_oracle_{op}_n")(_ptr(a), _ptr(b), _ptr(out), a.size)
    return out


def replica_size(cell_bytes: int, k: int, size: int, write_padding: bool = True) -> int:
    return lib().vds_oracle_replica_size(cell_bytes, k, size, int(write_padding))


def encode(k: int, replica: int, data: np.ndarray, cell_bytes: int = 2, write_padding: bool = True) -> np.ndarray:
    """chunk_generator<cell>::write for ONE replica (chunk.h:245-281)."""
    data = np.ascontiguousarray(data, dtype=np.uint8)
    out = np.empty(max(1, replica_size(cell_bytes, k, data.size, write_padding)), dtype=np.uint8)
    fn = lib().vds_oracle_encode16 if cell_bytes == 2 else lib().vds_oracle_encode8
    n = fn(k, replica, _ptr(data), data.size, int(write_padding), _ptr(out))
    return out[:n]


def inverse(k: int, nodes, cell_bytes: int = 2) -> tuple[np.ndarray, int]:
    """chunk_restore<cell>(k, n) multipliers (chunk.h:290-375)."""
    dt = np.uint16 if cell_bytes == 2 else np.uint8
    ct = C.c_uint16 if cell_bytes == 2 else C.c_uint8
    nodes = np.ascontiguousarray(nodes, dtype=dt)
    out = np.empty(k * k, dtype=dt)
    fn = lib().vds_oracle_inverse16 if cell_bytes == 2 else lib().vds_oracle_inverse8
    rc = fn(k, nodes.ctypes.data_as(C.POINTER(ct)), out.ctypes.data_as(C.POINTER(ct)))
    return out.reshape(k, k), rc


def restore(k: int, nodes, chunks, cell_bytes: int = 2):
    """chunk_restore<cell>::restore(vector<const_data_buffer>) (chunk.h:402-444).
    Returns the restored bytes or None for the reference's error path."""
    dt = np.uint16 if cell_bytes == 2 else np.uint8
    ct = C.c_uint16 if cell_bytes == 2 else C.c_uint8
    nodes = np.ascontiguousarray(nodes, dtype=dt)
    chunks = [np.ascontiguousarray(c, dtype=np.uint8) for c in chunks]
    size = chunks[0].size
    ptrs = (C.c_void_p * k)(*[_ptr(c) for c in chunks])
    out = np.empty(max(1, size * k), dtype=np.uint8)  # the most the reference loop can produce
    fn = lib().vds_oracle_restore16 if cell_bytes == 2 else lib().vds_oracle_restore8
    n = fn(k, nodes.ctypes.data_as(C.POINTER(ct)), ptrs, size, _ptr(out))
    if n == C.c_size_t(-1).value:
        return None
    return out[:n]


def chunk_cells(k: int, n: int, data: np.ndarray, cell_bytes: int = 2) -> np.ndarray:
    """chunk<cell>(generator, data, len) (chunk.h:206-224)."""
    dt = np.uint16 if cell_bytes == 2 else np.uint8
    data = np.ascontiguousarray(data, dtype=dt)
    out = np.empty(max(1, -(-data.size // k)), dtype=dt)
    fn = lib().vds_oracle_chunk_cells16 if cell_bytes == 2 else lib().vds_oracle_chunk_cells8
    cnt = fn(k, n, _ptr(data), data.size, _ptr(out))
    return out[:cnt]


def restore_cells(k: int, nodes, chunks, cell_bytes: int = 2) -> np.ndarray:
    """chunk_restore<cell>::restore(vector<cell>&, const chunk**) (chunk.h:383-400)."""
    dt = np.uint16 if cell_bytes == 2 else np.uint8
    ct = C.c_uint16 if cell_bytes == 2 else C.c_uint8
    nodes = np.ascontiguousarray(nodes, dtype=dt)
    chunks = [np.ascontiguousarray(c, dtype=dt) for c in chunks]
    cells = chunks[0].size
    ptrs = (C.c_void_p * k)(*[_ptr(c) for c in chunks])
    out = np.empty(max(1, cells * k), dtype=dt)
    fn = lib().vds_oracle_restore_cells16 if cell_bytes == 2 else lib().vds_oracle_restore_cells8
    fn(k, nodes.ctypes.data_as(C.POINTER(ct)), ptrs, cells, _ptr(out))
    return out[: cells * k]
