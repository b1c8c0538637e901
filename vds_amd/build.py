"""Build libvds_ec.so (HIP kernels + C ABI) in-tree for gfx950.

Used by __graft_entry__.build() and the tests.  The .so lands next to this
file so it travels to the GPU box with the repository snapshot.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libvds_ec.so")
SOURCES = ["ec_kernels.hip", "sha256.hip", "vds_ec_api.cpp"]
HEADERS = ["bitslice.hpp", "gf_common.hpp", "ec_internal.hpp"]
ARCH = os.environ.get("VDS_EC_ARCH", "gfx950")


def _hipcc() -> str:
    for c in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found: cannot build libvds_ec.so")


def _stale() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS] + [os.path.join(ROOT, "include", "vds_ec.h")]
    gen = os.path.join(CSRC, "generated")
    if os.path.isdir(gen):
        deps += [os.path.join(gen, f) for f in os.listdir(gen)]
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = False, out: str | None = None,
          defines: tuple[str, ...] = ()) -> str:
    """Build the library (default: in-tree libvds_ec.so, rebuilt when stale).
    `out` + `defines` build a variant (e.g. -DVDS_SYN_PREFETCH=0) for A/B
    measurements; the variant is loaded with VDS_EC_LIB=<path>."""
    lib = out or LIB
    if out is None and not force and not _stale():
        return LIB
    objs = []
    for src in SOURCES:
        obj = os.path.join(CSRC, src.rsplit(".", 1)[0] + (".variant.o" if out else ".o"))
        cmd = [_hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++20", "-fPIC", "-c", *defines,
               "-I", os.path.join(ROOT, "include"), os.path.join(CSRC, src), "-o", obj]
        if src.endswith(".cpp"):
            cmd[1:1] = ["-x", "hip"]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
        objs.append(obj)
    tmp = lib + ".tmp"
    subprocess.run([_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs +
                   ["-lpthread"], check=True)
    os.replace(tmp, lib)
    for o in objs:
        os.remove(o)
    return lib


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
