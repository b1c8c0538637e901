// ec_restore_syn_32a.hip -- k_restore_syn<32,40> instantiations:
// the plain (C4), batch and RT kernels at k = 32.
// (One translation unit per group so the builds compile them in parallel.)
#include "ec_restore_syn.hpp"

namespace vds_ec {

hipError_t syn_launch_32a(SynKind kind, const SynRestoreArgs &a, hipStream_t s, bool regen) {
  switch (kind) {
    case SynKind::kPlain:
      return syn_launch_kind<32, 40, 8, SynKind::kPlain>(a, s, regen);
    case SynKind::kBatch:
      return syn_launch_kind<32, 40, 8, SynKind::kBatch>(a, s, regen);
    case SynKind::kRt:
      return syn_launch_kind<32, 40, 8, SynKind::kRt>(a, s, regen);
    default:
      return hipErrorNotSupported;
  }
}

#if VDS_DIAG_STAMPS
hipError_t syn_stamps_32a(unsigned long long *host, size_t n) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_syn_stamps), n * sizeof(unsigned long long));
}
#endif

}  // namespace vds_ec
