// ec_restore_syn.hip -- dispatch of k_restore_syn<K,N> (ec_restore_syn.hpp,
// restore_syn.hpp) to its instantiation units, the run-time compiled
// survivor-set kernels' launch, and the diagnostic stamp readout.
#include "ec_restore_syn.hpp"

#include <vector>

namespace vds_ec {

#if VDS_DIAG_STAMPS
// Each instantiation unit is its own code object with its own g_syn_stamps;
// a run stamps through the kernels of one of them, so the sum is that one.
extern "C" int vds_ec_diag_stamps(unsigned long long *host, size_t n) {
  if (n > (size_t)kStampSlots) n = kStampSlots;
  std::vector<unsigned long long> part(n);
  for (size_t i = 0; i < n; ++i) host[i] = 0;
  for (auto rd : {syn_stamps_16, syn_stamps_32a, syn_stamps_32b}) {
    const hipError_t e = rd(part.data(), n);
    if (e != hipSuccess) return (int)e;
    for (size_t i = 0; i < n; ++i) host[i] += part[i];
  }
  return 0;
}
#endif

bool has_restore_syn(uint32_t k, uint32_t n) { return (k == 16 && n == 20) || (k == 32 && n == 40); }

const uint16_t *restore_syn_weights(uint32_t k, uint32_t n) {
  if (k == 16 && n == 20) return &RestorePrograms<16, 20, 4>::kSyndromeW[0][0];
  if (k == 32 && n == 40) return &RestorePrograms<32, 40, 8>::kSyndromeW[0][0];
  return nullptr;
}

hipError_t launch_restore_syn(uint32_t k, uint32_t n, const SynRestoreArgs &a, hipStream_t s, bool regen) {
  if (k == 16 && n == 20)
    return syn_launch_16(SynKind::kPlain, a, s, regen);
  if (k == 32 && n == 40)
    return syn_launch_32a(SynKind::kPlain, a, s, regen);
  return hipErrorNotSupported;
}

// A run-time compiled instantiation of the same body (vds_ec_jit.cpp: the
// survivor set's fill programs instead of syndromes + recovery), launched as
// its static twin would be.
hipError_t launch_restore_syn_jit(hipFunction_t fn, uint32_t k, uint32_t n, const SynRestoreArgs &a, hipStream_t s) {
  int lds = 0, threads = 0, blocks_per_cu = 0;
  if (k == 16 && n == 20) {
    using S = SynShape<16, 20, 4>;
    lds = S::kLdsBytes, threads = S::kThreads;
  } else if (k == 32 && n == 40) {
    using S = SynShape<32, 40, 8>;
    lds = S::kLdsBytes, threads = S::kThreads;
  } else {
    return hipErrorNotSupported;
  }
  blocks_per_cu = (160 * 1024) / lds;
  uint32_t grid = 256u * (blocks_per_cu > 0 ? blocks_per_cu : 1);
  if (VDS_SYN_GRID > 0) grid = VDS_SYN_GRID;
  if (grid > a.total_tiles) grid = a.total_tiles;
  if (grid == 0) return hipSuccess;
  // survivors in point order: the scatter fill programs of wave w take the
  // survivors of rank 4w..4w+3 (vds_ec_jit.cpp)
  SynRestoreArgs b = a;
  uint32_t ord[kMaxFastK];
  for (uint32_t j = 0; j < k; ++j) ord[j] = j;
  std::sort(ord, ord + k, [&](uint32_t x, uint32_t y) { return a.point[x] < a.point[y]; });
  for (uint32_t j = 0; j < k; ++j) {
    b.chunks[j] = a.chunks[ord[j]];
    b.point[j] = a.point[ord[j]];
  }
  void *args[] = {&b};
  return hipModuleLaunchKernel(fn, grid, 1, 1, threads, 1, 1, lds, s, args, nullptr);
}

hipError_t launch_restore_syn_batch(uint32_t k, uint32_t n, const SynRestoreArgs &a, hipStream_t s, bool regen) {
  if (k == 16 && n == 20)
    return syn_launch_16(SynKind::kBatch, a, s, regen);
  if (k == 32 && n == 40)
    return syn_launch_32a(SynKind::kBatch, a, s, regen);
  return hipErrorNotSupported;
}

bool has_restore_small(uint32_t k, uint32_t ms) { return (k == 16 || k == 32) && (ms == 1 || ms == 2); }

const uint16_t *restore_small_weights(uint32_t k, uint32_t ms) {
  if (k == 16 && ms == 1) return &SmallSyn<16, 1>::kW[0][0];
  if (k == 16 && ms == 2) return &SmallSyn<16, 2>::kW[0][0];
  if (k == 32 && ms == 1) return &SmallSyn<32, 1>::kW[0][0];
  if (k == 32 && ms == 2) return &SmallSyn<32, 2>::kW[0][0];
  return nullptr;
}

hipError_t launch_restore_small_batch(uint32_t k, uint32_t ms, const SynRestoreArgs &a, hipStream_t s, bool regen) {
  static_assert(SmallSyn<16, 2>::kSynSlot + 2 <= 20 && SmallSyn<32, 2>::kSynSlot + 2 <= 40,
                "syndrome slots inside the LDS points");
  const SynKind kind = ms == 1 ? SynKind::kSmall1 : SynKind::kSmall2;
  if (k == 16 && (ms == 1 || ms == 2)) return syn_launch_16(kind, a, s, regen);
  if (k == 32 && (ms == 1 || ms == 2)) return syn_launch_32b(kind, a, s, regen);
  return hipErrorNotSupported;
}

hipError_t launch_regen_perm_batch(uint32_t k, const SynRestoreArgs &a, hipStream_t s) {
  if (k == 16) return syn_launch_16(SynKind::kPerm, a, s, true);
  if (k == 32) return syn_launch_32b(SynKind::kPerm, a, s, true);
  return hipErrorNotSupported;
}

hipError_t launch_restore_multi_batch(uint32_t k, const SynRestoreArgs &a, hipStream_t s, bool regen) {
  if (k == 16) return syn_launch_16(SynKind::kMulti, a, s, regen);
  if (k == 32) return syn_launch_32b(SynKind::kMulti, a, s, regen);
  return hipErrorNotSupported;
}

hipError_t launch_restore_rt_batch(uint32_t k, uint32_t n, const SynRestoreArgs &a, hipStream_t s, bool regen) {
  if (k == 16 && n == 20) return syn_launch_16(SynKind::kRt, a, s, regen);
  if (k == 32 && n == 40) return syn_launch_32a(SynKind::kRt, a, s, regen);
  return hipErrorNotSupported;
}

}  // namespace vds_ec
