"""C-ABI boundary checks that need no GPU.

* libvds_ec.so builds for gfx950, loads, and exports every entry point that
  include/vds_ec.h declares (and vds_amd/_lib.py binds).
* Host-side pieces of the boundary (no kernels): gf tables, multipliers,
  the Vandermonde inverse (chunk_restore ctor) and size arithmetic, against
  the oracle.
* Without a GPU every data-path entry point fails loudly (VDS_EC_ENODEV):
  there is no CPU fallback.
"""
import ctypes as C
import json
import os
import re

import numpy as np
import pytest

import oracle_ctypes as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "vds_ec.h")


def _declared():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(vds_ec_\w+)\s*\(", text)))


def test_header_and_binding_agree():
    from vds_amd import _lib
    assert set(_declared()) == set(_lib.SIGNATURES)


def test_library_exports_every_declared_symbol(vds_lib):
    for name in _declared():
        assert hasattr(vds_lib, name), name
    # and the exported dynamic symbols really are the C names (no mangling)
    import subprocess
    nm = subprocess.run(["nm", "-D", "--defined-only", os.path.join(ROOT, "vds_amd", "libvds_ec.so")],
                        capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\b(vds_ec_\w+)\b", nm))
    assert set(_declared()) <= exported


def test_version_and_strerror(vds_lib):
    assert vds_lib.vds_ec_version() >= 100
    assert b"no CPU fallback" in vds_lib.vds_ec_strerror(-2)


def test_sizes_match_oracle(vds_lib):
    for cb in (1, 2):
        for k in (1, 3, 4, 16, 32, 800):
            for size in (0, 1, 2, 31, 32, 33, 1 << 20, (64 << 20) + 5):
                if cb == 1 and k > 255:
                    continue
                for pad in (True, False):
                    assert vds_lib.vds_ec_replica_size(cb, k, size, 0 if pad else 1) == \
                        O.replica_size(cb, k, size, pad)
    # restored size = object size for a well-formed trailer (chunk.h:415-419)
    for k, size in ((4, 19), (16, 65541), (16, 64 << 20), (3, 1000)):
        L = O.replica_size(2, k, size)
        assert vds_lib.vds_ec_restored_size(2, k, L, size % (2 * k)) == size


def test_gf_tables_match_oracle(vds_lib):
    from vds_amd import _lib
    v2l = np.zeros(65536, np.uint16)
    l2v = np.zeros(65536, np.uint16)
    assert vds_lib.vds_ec_gf16_tables(v2l.ctypes.data_as(_lib.u16p), l2v.ctypes.data_as(_lib.u16p)) == 0
    a = np.arange(65536, dtype=np.uint16)
    for b in (1, 2, 3, 19, 0x8000, 0xFFFF):
        bb = np.full_like(a, b)
        ours = np.where((a == 0) | (bb == 0), 0, l2v[(v2l[a].astype(np.int64) + v2l[bb]) % 65535])
        assert np.array_equal(ours.astype(np.uint16), O.bulk("gf16_mul", a, bb))
    v8 = np.zeros(256, np.uint8)
    l8 = np.zeros(256, np.uint8)
    assert vds_lib.vds_ec_gf8_tables(v8.ctypes.data_as(_lib.u8p), l8.ctypes.data_as(_lib.u8p)) == 0
    a8 = np.repeat(np.arange(256, dtype=np.uint8), 256)
    b8 = np.tile(np.arange(256, dtype=np.uint8), 256)
    ours8 = np.where((a8 == 0) | (b8 == 0), 0, l8[(v8[a8].astype(np.int64) + v8[b8]) % 255]).astype(np.uint8)
    assert np.array_equal(ours8, O.bulk("gf8_mul", a8, b8))


def test_multipliers_and_inverse_match_oracle(vds_lib):
    from vds_amd import chunk
    for k, node in ((4, 0), (4, 5), (16, 19), (32, 39), (800, 999), (3, 65535)):
        m = chunk.multipliers(k, node)
        ref = np.array([O.gf16_mul(1, 1)] * 0 + [1] * 0, dtype=np.uint16)
        acc, ref = 1, []
        for _ in range(k):
            ref.append(acc)
            acc = O.gf16_mul(acc, node)
        assert m.tolist() == ref
    with open(os.path.join(ROOT, "tests", "golden", "golden_vectors.json")) as f:
        g = json.load(f)
    for inv in g["inverse16"]:
        M = chunk.inverse(inv["k"], inv["nodes"])
        assert M.tolist() == inv["rows"]
    M8 = chunk.inverse(g["inverse8"]["k"], g["inverse8"]["nodes"], cell_bytes=1)
    assert M8.tolist() == g["inverse8"]["rows"]
    # larger random node sets against the reference's Gauss-Jordan (oracle)
    rng = np.random.default_rng(3)
    for k in (5, 17, 64):
        nodes = [int(x) for x in rng.choice(65536, k, replace=False)]
        M, rc = O.inverse(k, nodes)
        assert rc == 0
        assert np.array_equal(chunk.inverse(k, nodes), M)


def test_duplicate_nodes_are_an_error(vds_lib):
    from vds_amd import chunk, VdsEcError
    with pytest.raises(VdsEcError):
        chunk.inverse(3, [1, 2, 1])


def _has_gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.mark.skipif(_has_gpu(), reason="checks the no-GPU behaviour")
def test_no_cpu_fallback_without_gpu(vds_lib):
    from vds_amd import chunk, VdsEcError
    with pytest.raises(VdsEcError) as e:
        chunk.ChunkGenerator(4, 1).write(b"hello world")
    assert e.value.status == -2
    with pytest.raises(VdsEcError) as e:
        chunk.ChunkRestore(2, [0, 1]).restore([b"\x00\x00\x00\x00", b"\x00\x00\x00\x00"])
    assert e.value.status == -2
