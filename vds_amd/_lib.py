"""ctypes loader for libvds_ec.so (the C ABI in include/vds_ec.h).

The library is built in-tree by vds_amd/build.py.  There is no CPU fallback:
if the shared object is missing or no GPU is visible, calls raise.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("VDS_EC_LIB") or os.path.join(HERE, "libvds_ec.so")

OK = 0
EINVAL = -1
ENODEV = -2
ENOMEM = -3
ESINGULAR = -4
ERESTORE = -5
EHIP = -6
EB64_LENGTH = -7
EB64_PADDING = -8
EB64_CHAR = -9

F_NO_TRAILER = 0x1
F_CELLS = 0x2

# Every entry point include/vds_ec.h declares, with its ctypes signature.
u8p = C.POINTER(C.c_uint8)
u16p = C.POINTER(C.c_uint16)
u64p = C.POINTER(C.c_uint64)
vpp = C.POINTER(C.c_void_p)
SIGNATURES = {
    "vds_ec_strerror": (C.c_char_p, [C.c_int]),
    "vds_ec_version": (C.c_int, []),
    "vds_ec_host_ctx_stats": (C.c_int, [C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    "vds_ec_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "vds_ec_replica_size": (C.c_uint64, [C.c_uint, C.c_uint, C.c_uint64, C.c_uint]),
    "vds_ec_restored_size": (C.c_uint64, [C.c_uint, C.c_uint, C.c_uint64, C.c_uint16]),
    "vds_ec_gf16_tables": (C.c_int, [u16p, u16p]),
    "vds_ec_gf8_tables": (C.c_int, [u8p, u8p]),
    "vds_ec_multipliers16": (C.c_int, [C.c_uint16, C.c_uint16, u16p]),
    "vds_ec_multipliers8": (C.c_int, [C.c_uint8, C.c_uint8, u8p]),
    "vds_ec_inverse16": (C.c_int, [C.c_uint16, u16p, u16p]),
    "vds_ec_inverse8": (C.c_int, [C.c_uint8, u8p, u8p]),
    "vds_ec_encode16_device": (C.c_int, [C.c_uint16, u16p, C.c_uint32, C.c_void_p, C.c_uint64, C.c_uint64,
                                         C.c_uint32, vpp, C.c_uint64, C.c_uint, C.c_void_p]),
    "vds_ec_encode8_device": (C.c_int, [C.c_uint8, u8p, C.c_uint32, C.c_void_p, C.c_uint64, C.c_uint64,
                                        C.c_uint32, vpp, C.c_uint64, C.c_uint, C.c_void_p]),
    "vds_ec_restore16_device": (C.c_int, [C.c_uint16, u16p, vpp, C.c_uint64, C.c_uint64, C.c_uint16,
                                          C.c_uint32, C.c_void_p, C.c_uint64, C.c_uint, C.c_void_p]),
    "vds_ec_restore8_device": (C.c_int, [C.c_uint8, u8p, vpp, C.c_uint64, C.c_uint64, C.c_uint16,
                                         C.c_uint32, C.c_void_p, C.c_uint64, C.c_uint, C.c_void_p]),
    "vds_ec_encode16_host": (C.c_int, [C.c_uint16, u16p, C.c_uint32, C.c_void_p, C.c_uint64, vpp, C.c_uint]),
    "vds_ec_encode8_host": (C.c_int, [C.c_uint8, u8p, C.c_uint32, C.c_void_p, C.c_uint64, vpp, C.c_uint]),
    "vds_ec_restore16_host": (C.c_int, [C.c_uint16, u16p, vpp, C.c_uint64, C.c_void_p, u64p, C.c_uint]),
    "vds_ec_restore8_host": (C.c_int, [C.c_uint8, u8p, vpp, C.c_uint64, C.c_void_p, u64p, C.c_uint]),
    "vds_ec_host_alloc": (C.c_int, [C.c_uint64, C.POINTER(C.c_void_p)]),
    "vds_ec_host_free": (C.c_int, [C.c_void_p]),
    "vds_ec_host_register": (C.c_int, [C.c_void_p, C.c_uint64]),
    "vds_ec_host_unregister": (C.c_int, [C.c_void_p]),
    "vds_ec_encode16_host_batch": (C.c_int, [C.c_uint16, u16p, C.c_uint32, vpp, u64p, C.c_uint32, vpp,
                                             C.c_uint, C.c_int]),
    "vds_ec_restore16_host_batch": (C.c_int, [C.c_uint16, u16p, vpp, u64p, C.c_uint32, vpp, u64p, C.c_uint, C.c_int]),
    "vds_ec_regenerate16_device": (C.c_int, [C.c_uint16, u16p, vpp, C.c_uint64, C.c_uint64, C.c_uint32, u16p,
                                             C.c_uint32, vpp, C.c_uint64, C.c_void_p]),
    "vds_ec_regenerate16_host": (C.c_int, [C.c_uint16, u16p, vpp, C.c_uint64, u16p, C.c_uint32, vpp]),
    "vds_ec_regenerate16_path": (C.c_int, [C.c_uint16, u16p, u16p, C.c_uint32, C.c_uint64]),
    "vds_ec_sha256_device": (C.c_int, [C.c_void_p, C.c_uint64, C.c_uint64, C.c_uint32, C.c_void_p, C.c_void_p]),
    "vds_ec_sha256_host": (C.c_int, [C.c_void_p, C.c_uint64, C.c_void_p]),
    "vds_ec_encode16_hash_host": (C.c_int, [C.c_uint16, u16p, C.c_uint32, C.c_void_p, C.c_uint64, vpp, C.c_void_p,
                                            C.c_uint]),
    "vds_ec_replica_paths": (C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p]),
    "vds_ec_fill_splitmix_device": (C.c_int, [C.c_void_p, C.c_uint64, C.c_uint64, C.c_void_p]),
    "vds_ec_encode16_path": (C.c_int, [C.c_uint16, u16p, C.c_uint32, C.c_uint64]),
    "vds_ec_restore16_path": (C.c_int, [C.c_uint16, u16p, C.c_uint64, C.c_uint16, C.c_uint32]),
    "vds_ec_jit_set_mode": (C.c_int, [C.c_int]),
    "vds_ec_jit_wait": (C.c_int, []),
    "vds_ec_jit_build16": (C.c_int, [C.c_uint16, u16p, u64p]),
    "vds_ec_jit_ready16": (C.c_int, [C.c_uint16, u16p]),
    "vds_ec_jit_dump16": (C.c_int, [C.c_uint16, u16p, C.c_int, C.c_char_p]),
    "vds_ec_restore16_batch_device": (C.c_int, [C.c_uint16, C.c_uint32, u16p, vpp, u64p, u16p, vpp, C.c_uint,
                                                C.c_void_p]),
    "vds_ec_regenerate16_batch_device": (C.c_int, [C.c_uint16, C.c_uint32, u16p, vpp, u64p, C.c_uint32, u16p, vpp,
                                                   C.c_void_p]),
    "vds_ec_base64_decoded_size": (C.c_size_t, [C.c_char_p, C.c_size_t]),
    "vds_ec_base64_decode": (C.c_int, [C.c_char_p, C.c_size_t, C.c_void_p, C.POINTER(C.c_size_t)]),
    "vds_ec_base64_encode": (C.c_int, [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t)]),
    "vds_ec_tmp_names": (C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p]),
    "vds_ec_upload_response_json": (C.c_int, [C.c_int, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32, C.c_void_p,
                                              C.c_size_t, C.POINTER(C.c_size_t)]),
    "vds_ec_save_temp16_host": (C.c_int, [C.c_uint16, C.c_uint32, C.c_void_p, C.c_uint64, vpp, C.c_void_p,
                                          C.c_void_p, C.POINTER(C.c_uint32)]),
    "vds_ec_encode16_range_device": (C.c_int, [C.c_uint16, u16p, C.c_uint32, C.c_void_p, C.c_uint64, C.c_uint64,
                                               C.c_uint64, vpp, C.c_uint, C.c_void_p]),
    "vds_ec_restore16_range_device": (C.c_int, [C.c_uint16, u16p, vpp, C.c_uint64, C.c_uint16, C.c_uint64,
                                                C.c_uint64, C.c_void_p, C.c_uint, C.c_void_p]),
    "vds_ec_encode16_host_split": (C.c_int, [C.c_uint16, u16p, C.c_uint32, C.c_void_p, C.c_uint64, vpp, C.c_uint,
                                             C.c_int, C.c_uint32]),
    "vds_ec_restore16_host_split": (C.c_int, [C.c_uint16, u16p, vpp, C.c_uint64, C.c_void_p, u64p, C.c_uint, C.c_int,
                                              C.c_uint32]),
}

_lib = None
_lock = threading.Lock()


class VdsEcError(RuntimeError):
    """A non-zero vds_ec status (the C++ drop-in maps these to
    make_unexpected<std::runtime_error>, expected.h:46-49)."""

    def __init__(self, status: int, what: str = ""):
        self.status = status
        msg = strerror(status)
        super().__init__(f"{what}: {msg}" if what else msg)


def _bind_runtime_first() -> None:
    """Load torch's HIP runtime before ours when torch is installed.

    torch ships its own libamdhip64.so (soname libamdhip64.so.7) and links it
    under the unversioned name; if libvds_ec.so (NEEDED libamdhip64.so.7 from
    /opt/rocm) were loaded first, importing torch afterwards would map a second
    HIP runtime into the process.  Loading torch first makes our NEEDED entry
    resolve to the runtime already present, so there is exactly one.
    """
    try:
        import torch  # noqa: F401
    except ImportError:
        pass


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        with _lock:
            if _lib is None:
                _bind_runtime_first()
                if not os.path.exists(LIB_PATH):
                    raise RuntimeError(f"{LIB_PATH} is missing: run vds_amd/build.py (no CPU fallback)")
                h = C.CDLL(LIB_PATH)
                for name, (res, args) in SIGNATURES.items():
                    f = getattr(h, name)
                    f.restype = res
                    f.argtypes = args
                _lib = h
    return _lib


def strerror(status: int) -> str:
    try:
        return lib().vds_ec_strerror(status).decode()
    except Exception:  # pragma: no cover - library unavailable
        return f"vds_ec status {status}"


def check(status: int, what: str = "") -> None:
    if status != OK:
        raise VdsEcError(status, what)


def device_count() -> int:
    n = C.c_int(0)
    check(lib().vds_ec_device_count(C.byref(n)))
    return n.value
