"""Build libvds_ec.so (HIP kernels + C ABI) in-tree for gfx950.

Used by __graft_entry__.build(), bench.py and the tests.  The .so lands next
to this file so it travels to the GPU box with the repository snapshot.

Safe to call from several processes at once (bench.py's torchrun ranks, the
test runner): builds are serialised by an fcntl lock, each build compiles
into a private temporary directory, and the library is swapped in with one
atomic rename; a process that waited for the lock re-checks staleness and
returns the library the other process built.
"""
from __future__ import annotations

import concurrent.futures as cf
import fcntl
import hashlib
import os
import re
import shutil
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libvds_ec.so")
JITC = os.path.join(HERE, "vds_ec_jitc")  # the run-time kernel compiler (vds_ec_jitc.cpp), next to the library
LOCK = os.path.join(HERE, ".build.lock")
# one translation unit per kernel family, compiled in parallel
SOURCES = ["ec_encode_16_20.hip", "ec_encode_32_40.hip", "ec_encode_32_64.hip", "ec_restore_syn_32a.hip",
           "ec_restore_syn_32b.hip", "ec_restore_syn_16.hip", "ec_encode.hip", "ec_restore_syn.hip", "ec_generic.hip",
           "ec_restore_bs.hip", "sha256.hip", "vds_ec_api.cpp", "api_batch.cpp", "api_host_batch.cpp", "api_param_ring.cpp",
           "vds_ec_wire.cpp", "vds_ec_jit.cpp", "sha256_host.cpp"]
HOST_ONLY = {"sha256_host.cpp"}
HEADERS = ["bitslice.hpp", "gf_common.hpp", "ec_internal.hpp", "ec_device.hpp", "restore_syn.hpp", "xorprog.hpp",
           "ec_encode.hpp", "ec_restore_syn.hpp", "api_internal.hpp", "vds_ec_jitc.cpp"]
# The device sources the run-time kernels are compiled from (vds_ec_jit.cpp,
# hiprtc in the helper vds_ec_jitc), embedded in the helper as jit_embed.inc
# (written into the build directory).
JIT_FILES = ["gf_common.hpp", "bitslice.hpp", "ec_internal.hpp", "ec_device.hpp", "restore_syn.hpp",
             "generated/restore_16_20_w4.inc", "generated/restore_32_40_w8.inc"]
ARCH = os.environ.get("VDS_EC_ARCH", "gfx950")


def _arch_define() -> str:
    """The target architecture, for the JIT helper (its --offload-arch) and the
    library (the JIT cache key): both must agree with the library's own."""
    return f'-DVDS_EC_ARCH_STR="{ARCH}"'


def _hipcc() -> str:
    for c in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found: cannot build libvds_ec.so")


def _deps() -> list[str]:
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS] + [os.path.join(ROOT, "include", "vds_ec.h")]
    gen = os.path.join(CSRC, "generated")
    if os.path.isdir(gen):
        deps += [os.path.join(gen, f) for f in sorted(os.listdir(gen))]
    return deps


def _stale(lib: str) -> bool:
    if not os.path.exists(lib) or (lib == LIB and not os.path.exists(JITC)):
        return True
    t = os.path.getmtime(lib)
    return any(os.path.getmtime(d) > t for d in _deps())


def write_jit_embed(out_dir: str) -> None:
    """jit_embed.inc: kJitFiles[] = {include name, text} of JIT_FILES."""
    delim = "vdsjit"
    parts = ["static const EmbeddedFile kJitFiles[] = {\n"]
    for name in JIT_FILES:
        with open(os.path.join(CSRC, name)) as f:
            text = f.read()
        if ")" + delim + '"' in text:
            raise RuntimeError(f"{name} contains the raw-string delimiter")
        parts.append(f'    {{"{name}", R"{delim}({text}){delim}"}},\n')
    parts.append("};\n")
    with open(os.path.join(out_dir, "jit_embed.inc"), "w") as f:
        f.write("".join(parts))


def compile_cmd(src: str, obj: str, defines: tuple[str, ...] = (), includes: tuple[str, ...] = ()) -> list[str]:
    cmd = [_hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++20", "-fPIC", "-c", *defines, _arch_define(),
           "-I", os.path.join(ROOT, "include"), *[a for d in includes for a in ("-I", d)],
           os.path.join(CSRC, src), "-o", obj]
    if src in HOST_ONLY:  # plain C++ (x86 intrinsics): no device pass
        cmd = [a for a in cmd if not a.startswith("--offload-arch")]
        cmd[1:1] = ["-x", "c++"]
    elif src.endswith(".cpp"):
        cmd[1:1] = ["-x", "hip"]
    return cmd


OBJCACHE = os.path.join(HERE, ".objcache")  # compiled objects by content hash (git- and gpurun-ignored)
_INC = re.compile(r'^\s*#\s*include\s+"([^"]+)"', re.M)


def _local_includes(path: str, seen: set[str]) -> None:
    """`path` and every quoted include it reaches under csrc/ or include/."""
    if path in seen or not os.path.exists(path):
        return
    seen.add(path)
    with open(path, errors="replace") as f:
        text = f.read()
    for name in _INC.findall(text):
        for d in (os.path.dirname(path), CSRC, os.path.join(ROOT, "include")):
            c = os.path.join(d, name)
            if os.path.exists(c):
                _local_includes(c, seen)
                break


_TOOLCHAIN: str | None = None


def _toolchain_id() -> str:
    """Identity of the compiler (hipcc --version and the clang binary's path,
    size and mtime), computed once per process: an in-place ROCm upgrade
    behind the same hipcc path must not reuse objects built by the old one."""
    global _TOOLCHAIN
    if _TOOLCHAIN is None:
        hipcc = _hipcc()
        try:
            ver = subprocess.run([hipcc, "--version"], capture_output=True, text=True, timeout=60).stdout
        except (OSError, subprocess.SubprocessError):
            ver = "?"
        rocm = os.path.dirname(os.path.dirname(os.path.realpath(hipcc)))
        clang = os.path.realpath(os.path.join(rocm, "lib", "llvm", "bin", "clang"))
        st = os.stat(clang) if os.path.exists(clang) else None
        _TOOLCHAIN = f"{ver}|{clang}|{st.st_size if st else 0}|{st.st_mtime_ns if st else 0}"
    return _TOOLCHAIN


def _obj_key(cmd: list[str], src: str) -> str:
    """Hash of the toolchain identity, the compile command (minus the output
    path) and the bytes of the source and every local header it includes.  A
    project switch (-DVDS_...) that the unit never names cannot change its
    object and is left out, so a variant build recompiles only the units its
    switches reach; every other -D is kept (it may act through a system
    header, e.g. NDEBUG)."""
    files: set[str] = set()
    _local_includes(os.path.join(CSRC, src), files)
    texts = []
    for f in sorted(files):
        with open(f, "rb") as fh:
            texts.append((f, fh.read()))
    blob = b"".join(t for _, t in texts)

    def unused_switch(a: str) -> bool:
        name = a[2:].split("=")[0]
        return a.startswith("-DVDS_") and name.encode() not in blob

    args = [a for a in cmd[:-2] if not unused_switch(a)]
    h = hashlib.sha256()
    h.update(_toolchain_id().encode())
    h.update("\0".join(args).encode())
    for f, t in texts:
        h.update(f.encode())
        h.update(t)
    return h.hexdigest()[:32]


def _cached_compile(cmd: list[str], obj: str, key: str | None) -> None:
    """Compile unless an object with the same key is cached; keep the result.
    key None: compile, bypassing the cache (forced builds, VDS_EC_OBJCACHE=0)."""
    if key is None:
        subprocess.run(cmd, check=True)
        return
    hit = os.path.join(OBJCACHE, key + ".o")
    if os.path.exists(hit):
        shutil.copyfile(hit, obj)
        return
    subprocess.run(cmd, check=True)
    os.makedirs(OBJCACHE, exist_ok=True)
    tmp = hit + f".{os.getpid()}.tmp"
    shutil.copyfile(obj, tmp)
    os.replace(tmp, hit)
    # bounded: the oldest objects go first
    ents = sorted((os.path.getmtime(os.path.join(OBJCACHE, e)), e) for e in os.listdir(OBJCACHE) if e.endswith(".o"))
    for _, e in ents[:-96]:
        try:
            os.remove(os.path.join(OBJCACHE, e))
        except OSError:
            pass


def _compile_all(tmp: str, defines: tuple[str, ...], verbose: bool, use_cache: bool = True) -> list[str]:
    jobs = []
    write_jit_embed(tmp)
    use_cache = use_cache and os.environ.get("VDS_EC_OBJCACHE", "1") != "0"
    for src in SOURCES:
        obj = os.path.join(tmp, src.rsplit(".", 1)[0] + ".o")
        cmd = compile_cmd(src, obj, defines)
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        jobs.append((cmd, obj, _obj_key(cmd, src) if use_cache else None))
    workers = max(1, min(len(jobs), int(os.environ.get("MAX_JOBS", "0")) or (os.cpu_count() or 1), 8))
    rocm = os.path.dirname(os.path.dirname(os.path.realpath(_hipcc())))
    jitc = [_hipcc(), "-O2", "-std=c++20", _arch_define(), "-I", tmp, os.path.join(CSRC, "vds_ec_jitc.cpp"), "-o",
            os.path.join(tmp, "vds_ec_jitc"), f"-L{rocm}/lib", "-lhiprtc", f"-Wl,-rpath,{rocm}/lib",
            "-Wl,--disable-new-dtags"]
    with cf.ThreadPoolExecutor(workers) as ex:
        # (SOURCES lists the longest translation units first)
        futs = [ex.submit(_cached_compile, cmd, obj, key) for cmd, obj, key in jobs]
        futs.append(ex.submit(subprocess.run, jitc, check=True))
        for f in futs:
            f.result()
    return [obj for _, obj, _ in jobs]


def build(force: bool = False, verbose: bool = False, out: str | None = None,
          defines: tuple[str, ...] = ()) -> str:
    """Build the library (default: in-tree libvds_ec.so, rebuilt when stale).
    `out` + `defines` build a variant (e.g. -DVDS_DIAG_STAMPS=1) for A/B
    measurements; the variant is loaded with VDS_EC_LIB=<path>.  force=True
    recompiles every unit (the object cache is bypassed; VDS_EC_OBJCACHE=0
    turns the cache off for any build)."""
    lib = out or LIB
    if out is None and not force and not _stale(lib):
        return LIB
    os.makedirs(os.path.dirname(os.path.abspath(lib)), exist_ok=True)
    with open(LOCK, "a+") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        try:
            if out is None and not force and not _stale(lib):
                return LIB  # built by another process while this one waited
            with tempfile.TemporaryDirectory(prefix="vds_build_", dir=HERE) as tmp:
                objs = _compile_all(tmp, defines, verbose, use_cache=not force)
                tmp_lib = os.path.join(tmp, "lib.so")
                subprocess.run([_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp_lib] + objs +
                               ["-lpthread", "-ldl"], check=True)
                os.replace(os.path.join(tmp, "vds_ec_jitc"), os.path.join(os.path.dirname(os.path.abspath(lib)),
                                                                        "vds_ec_jitc"))
                os.replace(tmp_lib, lib)
        finally:
            fcntl.flock(lk, fcntl.LOCK_UN)
    return lib


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
