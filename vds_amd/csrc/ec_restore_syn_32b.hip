// ec_restore_syn_32b.hip -- k_restore_syn<32,40> instantiations:
// the SMALL, PERM and MULTI batch kernels at k = 32.
// (One translation unit per group so the builds compile them in parallel.)
#include "ec_restore_syn.hpp"

namespace vds_ec {

hipError_t syn_launch_32b(SynKind kind, const SynRestoreArgs &a, hipStream_t s, bool regen) {
  switch (kind) {
    case SynKind::kSmall1:
      return syn_launch_kind<32, 40, 8, SynKind::kSmall1>(a, s, regen);
    case SynKind::kSmall2:
      return syn_launch_kind<32, 40, 8, SynKind::kSmall2>(a, s, regen);
    case SynKind::kPerm:
      return syn_launch_kind<32, 40, 8, SynKind::kPerm>(a, s, regen);
    case SynKind::kMulti:
      return syn_launch_kind<32, 40, 8, SynKind::kMulti>(a, s, regen);
    default:
      return hipErrorNotSupported;
  }
}

#if VDS_DIAG_STAMPS
hipError_t syn_stamps_32b(unsigned long long *host, size_t n) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_syn_stamps), n * sizeof(unsigned long long));
}
#endif

}  // namespace vds_ec
