// ec_restore_syn_16.hip -- k_restore_syn<16,20> instantiations:
// every kernel family at k = 16.
// (One translation unit per group so the builds compile them in parallel.)
#include "ec_restore_syn.hpp"

namespace vds_ec {

hipError_t syn_launch_16(SynKind kind, const SynRestoreArgs &a, hipStream_t s, bool regen) {
  switch (kind) {
    case SynKind::kPlain:
      return syn_launch_kind<16, 20, 4, SynKind::kPlain>(a, s, regen);
    case SynKind::kBatch:
      return syn_launch_kind<16, 20, 4, SynKind::kBatch>(a, s, regen);
    case SynKind::kRt:
      return syn_launch_kind<16, 20, 4, SynKind::kRt>(a, s, regen);
    case SynKind::kSmall1:
      return syn_launch_kind<16, 20, 4, SynKind::kSmall1>(a, s, regen);
    case SynKind::kSmall2:
      return syn_launch_kind<16, 20, 4, SynKind::kSmall2>(a, s, regen);
    case SynKind::kPerm:
      return syn_launch_kind<16, 20, 4, SynKind::kPerm>(a, s, regen);
    case SynKind::kMulti:
      return syn_launch_kind<16, 20, 4, SynKind::kMulti>(a, s, regen);
    default:
      return hipErrorNotSupported;
  }
}

#if VDS_DIAG_STAMPS
hipError_t syn_stamps_16(unsigned long long *host, size_t n) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_syn_stamps), n * sizeof(unsigned long long));
}
#endif

}  // namespace vds_ec
