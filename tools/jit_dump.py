"""Compile one survivor set's run-time kernel on the CPU (no GPU needed) and
print its resource usage from the code object's metadata: VGPRs, SGPRs,
spills, scratch, LDS.  Used to check a restore_syn.hpp change for spills
before spending a GPU run on it.

  python tools/jit_dump.py [--k 32] [--nodes 1,2,3,...] [--lib path.so] [--keep DIR]

Default set: the C4 survivors (k = 32, erased r mod 5 == 0 of 0..39), or at
k = 16 the headline survivors (erased 0, 5, 10, 15).
"""
from __future__ import annotations

import argparse
import ctypes as C
import glob
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"


def resources(co: str) -> dict:
    out = subprocess.run([READELF, "--notes", co], capture_output=True, text=True, check=True).stdout
    keys = [".vgpr_count", ".sgpr_count", ".vgpr_spill_count", ".sgpr_spill_count", ".private_segment_fixed_size",
            ".group_segment_fixed_size", ".agpr_count"]
    res = {}
    for k in keys:
        m = re.search(re.escape(k) + r":\s+(\d+)", out)
        if m:
            res[k.lstrip(".")] = int(m.group(1))
    m = re.search(r"\.name:\s+(\S+)", out)
    if m:
        res["name"] = m.group(1)
    return res


def main() -> int:
    p = argparse.ArgumentParser()
    p.add_argument("--k", type=int, default=32)
    p.add_argument("--nodes", default="")
    p.add_argument("--lib", default=os.path.join(ROOT, "vds_amd", "libvds_ec.so"))
    p.add_argument("--keep", default="")
    a = p.parse_args()
    k = a.k
    n = k + k // 4
    if a.nodes:
        nodes = [int(x) for x in a.nodes.split(",")]
    else:
        step = n // (n - k)
        nodes = [r for r in range(n) if r % step][:k]
    d = a.keep or tempfile.mkdtemp(prefix="jit_dump_")
    os.makedirs(d, exist_ok=True)
    os.environ["VDS_EC_JIT_CACHE"] = "0"
    lib = C.CDLL(a.lib)
    arr = (C.c_uint16 * k)(*nodes)
    rc = lib.vds_ec_jit_dump16(C.c_uint16(k), arr, C.c_int(0), os.fsencode(d))
    if rc != 0:
        print("build failed", rc, file=sys.stderr)
        return 1
    for co in sorted(glob.glob(os.path.join(d, "*.co"))):
        print(os.path.basename(co), os.path.getsize(co), "bytes", resources(co))
    return 0


if __name__ == "__main__":
    sys.exit(main())
