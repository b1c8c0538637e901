"""The in-tree build (vds_amd/build.py) on CPU: concurrent builds of a stale
tree (what bench.py's torchrun ranks or parallel test runners do) and a
compile check of the one diagnostic build switch the kernels keep
(VDS_DIAG_STAMPS, tools/syn_stamps.py).  No GPU is touched."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from vds_amd import build as vbuild  # noqa: E402


def test_concurrent_builds_of_a_stale_tree(tmp_path):
    # make the library stale, then let two processes build at once: the lock
    # serialises them, the second re-checks and returns the first's library
    hdr = os.path.join(vbuild.CSRC, "ec_internal.hpp")
    os.utime(hdr, None)
    assert vbuild._stale(vbuild.LIB)
    code = ("import sys; sys.path.insert(0, %r); from vds_amd import build; "
            "import ctypes; p = build.build(); ctypes.CDLL(p).vds_ec_version; print(p)" % ROOT)
    procs = [subprocess.Popen([sys.executable, "-c", code], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                              text=True) for _ in range(2)]
    outs = [p.communicate(timeout=600) for p in procs]
    for p, (out, err) in zip(procs, outs):
        assert p.returncode == 0, err[-2000:]
        assert out.strip().endswith("libvds_ec.so")
    assert not vbuild._stale(vbuild.LIB)
    leftovers = [d for d in os.listdir(vbuild.HERE) if d.startswith("vds_build_")]
    assert leftovers == [], leftovers


def test_diag_stamps_build_compiles(tmp_path):
    obj = str(tmp_path / "syn_stamps.o")
    cmd = vbuild.compile_cmd("ec_restore_syn.hip", obj, ("-DVDS_DIAG_STAMPS=1",))
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    syms = subprocess.run(["nm", obj], capture_output=True, text=True).stdout
    assert "vds_ec_diag_stamps" in syms
