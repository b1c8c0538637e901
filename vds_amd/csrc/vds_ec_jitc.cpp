// vds_ec_jitc.cpp -- the run-time kernel compiler of vds_ec_jit.cpp, as a
// helper executable (vds_amd/vds_ec_jitc, built next to libvds_ec.so).
//
// Why a separate process: a process that imports torch before libvds_ec.so
// has torch's own libhiprtc / libamd_comgr mapped (same sonames as ROCm's),
// so an in-process hiprtc call would compile with torch's older LLVM.  For
// k_restore_syn<16,20> that compiler spilled 51 VGPRs where the ROCm one the
// static kernels are built with spills none (repair 17.5 vs 15.0 ms, 512 x 64
// MiB).  This executable links the image's hiprtc only.
//
//   vds_ec_jitc SOURCE.hip OUT.co     exit 0: OUT.co written; else the log on stderr
//
// The kernel source includes the device headers embedded here at build time
// (jit_embed.inc, vds_amd/build.py), the same set the library was built from,
// and compiles for the architecture the library was built for (VDS_EC_ARCH_STR,
// passed by build.py to both).
#include <hip/hiprtc.h>

#include <cstdio>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#ifndef VDS_EC_ARCH_STR
#define VDS_EC_ARCH_STR "gfx950"
#endif

namespace {
struct EmbeddedFile {
  const char *name;
  const char *text;
};
#include "jit_embed.inc"
}  // namespace

int main(int argc, char **argv) {
  if (argc != 3) {
    std::fprintf(stderr, "usage: %s SOURCE.hip OUT.co\n", argv[0]);
    return 2;
  }
  std::ifstream in(argv[1]);
  if (!in) {
    std::fprintf(stderr, "vds_ec_jitc: cannot read %s\n", argv[1]);
    return 2;
  }
  std::stringstream ss;
  ss << in.rdbuf();
  const std::string src = ss.str();
  std::vector<const char *> hdr, names;
  for (const EmbeddedFile &f : kJitFiles) {
    names.push_back(f.name);
    hdr.push_back(f.text);
  }
  hiprtcProgram prog;
  if (hiprtcCreateProgram(&prog, src.c_str(), "vds_ec_jit_restore.hip", (int)hdr.size(), hdr.data(), names.data()) !=
      HIPRTC_SUCCESS) {
    std::fprintf(stderr, "vds_ec_jitc: hiprtcCreateProgram failed\n");
    return 1;
  }
  const char *opts[] = {"--offload-arch=" VDS_EC_ARCH_STR, "-O3", "-std=c++20"};
  const hiprtcResult r = hiprtcCompileProgram(prog, 3, opts);
  size_t ls = 0;
  hiprtcGetProgramLogSize(prog, &ls);
  if (ls > 1) {
    std::string log(ls, '\0');
    hiprtcGetProgramLog(prog, &log[0]);
    std::fputs(log.c_str(), stderr);
  }
  size_t cs = 0;
  std::vector<char> code;
  bool ok = r == HIPRTC_SUCCESS && hiprtcGetCodeSize(prog, &cs) == HIPRTC_SUCCESS && cs > 0;
  if (ok) {
    code.resize(cs);
    ok = hiprtcGetCode(prog, code.data()) == HIPRTC_SUCCESS;
  }
  hiprtcDestroyProgram(&prog);
  if (!ok) {
    std::fprintf(stderr, "vds_ec_jitc: compile failed (%d)\n", (int)r);
    return 1;
  }
  std::ofstream out(argv[2], std::ios::binary);
  out.write(code.data(), (std::streamsize)code.size());
  return out.good() ? 0 : 1;
}
