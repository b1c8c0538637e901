"""The run-time compiled survivor-set kernels include restore_syn.hpp under
hiprtc, with no standard library (vds_ec_jitc.cpp embeds the device headers
at build time).  Compile a kernel of that header through the helper here,
without a GPU, so a host-only construct in the shared kernel body (a std::
index sequence broke every JIT kernel once) fails on the CPU suite instead of
as silent AOT fallbacks on the GPU box."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HELPER = os.path.join(ROOT, "vds_amd", "vds_ec_jitc")

SRC = """#define VDS_GM2 1
#define VDS_GM2_PRIO 1
#define VDS_SCHED_FENCE() __builtin_amdgcn_sched_barrier(0)
#include "restore_syn.hpp"
namespace vds_ec {
#include "generated/restore_%(k)d_%(n)d_w%(wv)d.inc"
}
extern "C" __global__ void f(vds_ec::SynRestoreArgs a) {
  vds_ec::restore_syn_body<%(k)d, %(n)d, %(wv)d, %(regen)s, false>(a);
}
"""


@pytest.mark.skipif(not os.access(HELPER, os.X_OK), reason="vds_ec_jitc not built (run __graft_entry__.build())")
@pytest.mark.parametrize("regen", ["false", "true"])
def test_restore_body_compiles_under_hiprtc(tmp_path, regen):
    src = tmp_path / "k.hip"
    out = tmp_path / "k.co"
    src.write_text(SRC % {"k": 16, "n": 20, "wv": 4, "regen": regen})
    r = subprocess.run([HELPER, str(src), str(out)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    assert out.stat().st_size > 0


@pytest.mark.skipif(not os.access(HELPER, os.X_OK), reason="vds_ec_jitc not built (run __graft_entry__.build())")
def test_jit_kernel_symbol_names_its_set(tmp_path):
    """The run-time kernels are named by kind, (k, n) and survivor mask
    (vds_ec_jit.cpp kernel_name), so rocprofv3 summaries separate the
    headline set's kernel from every other instantiation."""
    code = ("import sys\nfrom vds_amd import chunk\n"
            "chunk.jit_dump(16, [r for r in range(20) if r not in (0, 5, 10, 15)], sys.argv[1])\n")
    env = dict(os.environ, VDS_EC_JIT_CACHE="0")
    r = subprocess.run([sys.executable, "-c", code, str(tmp_path)], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    cos = list(tmp_path.glob("*.co"))
    assert len(cos) == 1
    notes = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "--notes", str(cos[0])], capture_output=True,
                           text=True, check=True).stdout
    mask = sum(1 << r for r in range(20) if r not in (0, 5, 10, 15))
    assert f".name:           vds_ec_jit_restore_16_20_{mask:x}" in notes or \
        f"vds_ec_jit_restore_16_20_{mask:x}" in notes
