"""Pin the CPU oracle (oracle/vds_oracle.c) to the reference before trusting it.

1. The reference's own kernel/vds_data/gf.h, compiled unmodified into
   oracle/_ref/gf_ref (oracle/Makefile), against the oracle's GF arithmetic:
   every 8-bit pair and a structured + random set of 16-bit pairs.
2. The known-answer vectors recorded from the reference in SURVEY.md 8(a)/(c)
   (tests/golden/survey_kats.json) and the GF(2^3) table of
   tests/test_vds_data/gf_tests.cpp:9-38.
3. The frozen oracle fixtures (tests/golden/golden_vectors.json).
4. The reference's round-trip tests re-hosted on the oracle
   (chunk_tests.cpp:10-162), seeded.
"""
import json
import os
import subprocess

import numpy as np
import pytest

import oracle_ctypes as O

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _kats():
    with open(os.path.join(GOLDEN, "survey_kats.json")) as f:
        return json.load(f)


def _golden():
    with open(os.path.join(GOLDEN, "golden_vectors.json")) as f:
        return json.load(f)


def _read_dump(path, dtype, arrays):
    raw = open(path, "rb").read()
    out, pos = [], 0
    for _ in range(arrays):
        n = int(np.frombuffer(raw[pos:pos + 4], dtype=np.uint32)[0])
        pos += 4
        nbytes = n * np.dtype(dtype).itemsize
        out.append(np.frombuffer(raw[pos:pos + nbytes], dtype=dtype))
        pos += nbytes
    return out


def test_gf3_table_matches_gf_tests():
    tbl = _kats()["gf3_table_gf_tests_cpp_9_38"]
    for i in range(8):
        for j in range(8):
            assert O.gf_mul_bitserial(3, 0x0B, i, j) == tbl[i][j]


def test_survey_kats():
    k = _kats()
    e = k["encode16_k4_s19"]
    data = np.array([(37 * i + 11) % 256 for i in range(e["size"])], dtype=np.uint8)
    for r, hexs in e["replicas"].items():
        assert O.encode(e["k"], int(r), data).tobytes().hex() == hexs
    M, rc = O.inverse(4, [2, 3, 4, 5])
    assert rc == 0
    assert ["%04x" % x for x in M[0]] == k["inverse16_k4_nodes_2345_row0"]
    for a, b, p in k["gf8_mul"]:
        assert O.gf8_mul(a, b) == p
    for a, b, p in k["gf16_mul"]:
        assert O.gf16_mul(a, b) == p
    for a, b, p in k["gf16_div"]:
        assert O.gf16_div(a, b) == p


REF_GF = O.REF_GF


@pytest.mark.skipif(not os.path.exists(REF_GF), reason="oracle/_ref/gf_ref not built (reference tree absent)")
@pytest.mark.parametrize("mode", ["gf3", "gf8", "gf16"])
def test_oracle_matches_compiled_reference_gf(mode, tmp_path):
    out = tmp_path / f"{mode}.bin"
    subprocess.run([REF_GF, mode, str(out)], check=True)
    if mode == "gf3":
        a, b, p = _read_dump(out, np.uint8, 3)
        ours = np.array([O.gf_mul_bitserial(3, 0x0B, x, y) for x, y in zip(a, b)], dtype=np.uint8)
        assert np.array_equal(ours, p)
        return
    dt = np.uint8 if mode == "gf8" else np.uint16
    a, b, mul, div, bits = _read_dump(out, dt, 5)
    assert a.size == b.size == mul.size == div.size == bits.size > 0
    assert np.array_equal(O.bulk(f"{mode}_mul", a, b), mul)
    assert np.array_equal(O.bulk(f"{mode}_div", a, b), div)
    # table multiply == bit-serial gf<m> multiply (x primitive) on every pair
    assert np.array_equal(mul, bits)
    if mode == "gf8":
        sample = slice(None)
    else:
        sample = slice(0, None, 97)
    m = 8 if mode == "gf8" else 16
    poly = 0x1D if mode == "gf8" else 0x100B
    ours = np.array([O.gf_mul_bitserial(m, poly, int(x), int(y)) for x, y in zip(a[sample], b[sample])], dtype=dt)
    assert np.array_equal(ours, bits[sample])


def test_golden_fixtures_regress():
    g = _golden()
    base = g["seed_base"]
    for e in g["encode16_small"]:
        d = O.splitmix(base + e["object_index"], e["size"])
        for r, hexs in e["replicas"].items():
            assert O.encode(e["k"], int(r), d).tobytes().hex() == hexs
    for inv in g["inverse16"]:
        M, rc = O.inverse(inv["k"], inv["nodes"])
        assert rc == inv["rc"] == 0
        assert M.tolist() == inv["rows"]


def test_oracle_restore_roundtrip_edges():
    rng = np.random.default_rng(1)
    for k, size in ((4, 0), (4, 1), (4, 7), (4, 8), (4, 9), (3, 1000), (16, 65541), (5, 12345)):
        d = rng.integers(0, 256, size, dtype=np.uint8)
        nodes = list(rng.choice(np.arange(1, 300), size=k, replace=False))
        chunks = [O.encode(k, int(r), d) for r in nodes]
        out = O.restore(k, nodes, chunks)
        assert out is not None and out.tobytes() == d.tobytes()


def test_rehost_chunk_tests_on_oracle():
    """chunk_tests.cpp:10-110 (cell arrays, uint8/uint16, k=3) and
    :112-162 (byte API, min_horcrux replicas of < 1000), seeded."""
    rng = np.random.default_rng(7)
    for cb in (1, 2):
        size = 999
        data = rng.integers(0, 256 if cb == 1 else 65536, size).astype(np.uint8 if cb == 1 else np.uint16)
        ids = [int(x) for x in rng.choice(256, 3, replace=False)]
        chunks = [O.chunk_cells(3, r, data, cell_bytes=cb) for r in ids]
        out = O.restore_cells(3, ids, chunks, cell_bytes=cb)
        assert np.array_equal(out[:size], data)
    k = 120  # the reference uses 800; the full size runs on the GPU path
    size = 4321
    data = rng.integers(0, 256, size, dtype=np.uint8)
    ids = [int(x) for x in rng.choice(1000, k, replace=False)]
    chunks = [O.encode(k, r, data) for r in ids]
    out = O.restore(k, ids, chunks)
    assert out.tobytes() == data.tobytes()
