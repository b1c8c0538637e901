// ec_restore_syn.hip -- k_restore_syn<K,N>: restore of an object from any K
// of its N replicas without a per-pattern K x K inverse
// (chunk_restore<uint16_t>::restore, chunk.h:290-444; instantiated for
// (16, 20) and (32, 40), the BASELINE configs).
//
// With M = N - K erased points E, per 2048-stripe tile:
//   1. syndromes S_j = sum_a v_a a^j c_a over all N points (erased = 0): a
//      fixed map, generated XOR programs (tools/xorgen/gen_restore.cpp);
//   2. recovery c_E = W_E^{-1} S -- the only runtime arithmetic, M x M;
//   3. interpolation from the fixed points 0..K-1 (one additive-FFT level +
//      generated half-size programs + an XOR-only expansion);
//   4. big-endian stores through an LDS staging of the tile.
// REGEN stops after step 2 and writes the recovered points as replica bytes:
// the fused repair of sync_process.cpp:313-335 (decode + re-encode).
#include <algorithm>

#include "restore_syn.hpp"

namespace vds_ec {

#define VDS_SCHED_FENCE() __builtin_amdgcn_sched_barrier(0)
#include "generated/restore_16_20_w4.inc"
#include "generated/restore_32_40_w8.inc"
#include "generated/smallsyn_16_1.inc"
#include "generated/smallsyn_16_2.inc"
#include "generated/smallsyn_32_1.inc"
#include "generated/smallsyn_32_2.inc"
#include "generated/permsyn_16.inc"
#include "generated/permsyn_32.inc"
#undef VDS_SCHED_FENCE

template <int K, int N, int WV, bool REGEN, bool BATCH, bool RT = false, class FillP = NoFill>
__global__ __launch_bounds__((SynShape<K, N, WV>::kThreads), (SynShape<K, N, WV>::kWavesPerSimd))
void k_restore_syn(SynRestoreArgs a) {
  restore_syn_body<K, N, WV, REGEN, BATCH, RT, FillP>(a);
}

#if VDS_DIAG_STAMPS
extern "C" int vds_ec_diag_stamps(unsigned long long *host, size_t n) {
  if (n > (size_t)kStampSlots) n = kStampSlots;
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_syn_stamps), n * sizeof(unsigned long long));
}
#endif

// =================================================================== launchers

bool has_restore_syn(uint32_t k, uint32_t n) { return (k == 16 && n == 20) || (k == 32 && n == 40); }

const uint16_t *restore_syn_weights(uint32_t k, uint32_t n) {
  if (k == 16 && n == 20) return &RestorePrograms<16, 20, 4>::kSyndromeW[0][0];
  if (k == 32 && n == 40) return &RestorePrograms<32, 40, 8>::kSyndromeW[0][0];
  return nullptr;
}

template <int K, int N, int WV, bool REGEN, bool BATCH = false, bool RT = false, class FILL = NoFill>
static hipError_t launch_restore_syn_kn(const SynRestoreArgs &a, hipStream_t s) {
  using S = SynShape<K, N, WV>;
  hipError_t e = ensure_lds_attr(&k_restore_syn<K, N, WV, REGEN, BATCH, RT, FILL>, S::kLdsBytes);
  if (e != hipSuccess) return e;
  const int blocks_per_cu = (160 * 1024) / S::kLdsBytes;
  uint32_t grid = 256u * (blocks_per_cu > 0 ? blocks_per_cu : 1);
  static const uint32_t over = grid_override("VDS_EC_SYN_GRID");
  if (over) grid = over;
  if (grid > a.total_tiles) grid = a.total_tiles;
  if (grid == 0) return hipSuccess;
  hipLaunchKernelGGL((k_restore_syn<K, N, WV, REGEN, BATCH, RT, FILL>), dim3(grid), dim3(S::kThreads), S::kLdsBytes, s, a);
  return hipGetLastError();
}

hipError_t launch_restore_syn(uint32_t k, uint32_t n, const SynRestoreArgs &a, hipStream_t s, bool regen) {
  if (k == 16 && n == 20)
    return regen ? launch_restore_syn_kn<16, 20, 4, true>(a, s) : launch_restore_syn_kn<16, 20, 4, false>(a, s);
  if (k == 32 && n == 40)
    return regen ? launch_restore_syn_kn<32, 40, 8, true>(a, s) : launch_restore_syn_kn<32, 40, 8, false>(a, s);
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
  static const uint32_t over = grid_override("VDS_EC_SYN_GRID");
  if (over) grid = over;
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
    return regen ? launch_restore_syn_kn<16, 20, 4, true, true>(a, s) : launch_restore_syn_kn<16, 20, 4, false, true>(a, s);
  if (k == 32 && n == 40)
    return regen ? launch_restore_syn_kn<32, 40, 8, true, true>(a, s) : launch_restore_syn_kn<32, 40, 8, false, true>(a, s);
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

template <int K, int N, int WV, int MS>
static hipError_t launch_small_kn(const SynRestoreArgs &a, hipStream_t s, bool regen) {
  static_assert(SmallSyn<K, MS>::kSynSlot + MS <= N, "syndrome slots inside the LDS points");
  return regen ? launch_restore_syn_kn<K, N, WV, true, true, false, SmallSyn<K, MS>>(a, s)
               : launch_restore_syn_kn<K, N, WV, false, true, false, SmallSyn<K, MS>>(a, s);
}

hipError_t launch_restore_small_batch(uint32_t k, uint32_t ms, const SynRestoreArgs &a, hipStream_t s, bool regen) {
  if (k == 16 && ms == 1) return launch_small_kn<16, 20, 4, 1>(a, s, regen);
  if (k == 16 && ms == 2) return launch_small_kn<16, 20, 4, 2>(a, s, regen);
  if (k == 32 && ms == 1) return launch_small_kn<32, 40, 8, 1>(a, s, regen);
  if (k == 32 && ms == 2) return launch_small_kn<32, 40, 8, 2>(a, s, regen);
  return hipErrorNotSupported;
}

hipError_t launch_regen_perm_batch(uint32_t k, const SynRestoreArgs &a, hipStream_t s) {
  if (k == 16) return launch_restore_syn_kn<16, 20, 4, true, true, false, PermSyn<16>>(a, s);
  if (k == 32) return launch_restore_syn_kn<32, 40, 8, true, true, false, PermSyn<32>>(a, s);
  return hipErrorNotSupported;
}

hipError_t launch_restore_multi_batch(uint32_t k, const SynRestoreArgs &a, hipStream_t s, bool regen) {
  if (k == 16)
    return regen ? launch_restore_syn_kn<16, 20, 4, true, true, false, MultiP<16>>(a, s)
                 : launch_restore_syn_kn<16, 20, 4, false, true, false, MultiP<16>>(a, s);
  if (k == 32)
    return regen ? launch_restore_syn_kn<32, 40, 8, true, true, false, MultiP<32>>(a, s)
                 : launch_restore_syn_kn<32, 40, 8, false, true, false, MultiP<32>>(a, s);
  return hipErrorNotSupported;
}

hipError_t launch_restore_rt_batch(uint32_t k, uint32_t n, const SynRestoreArgs &a, hipStream_t s, bool regen) {
  if (k == 16 && n == 20)
    return regen ? launch_restore_syn_kn<16, 20, 4, true, true, true>(a, s)
                 : launch_restore_syn_kn<16, 20, 4, false, true, true>(a, s);
  if (k == 32 && n == 40)
    return regen ? launch_restore_syn_kn<32, 40, 8, true, true, true>(a, s)
                 : launch_restore_syn_kn<32, 40, 8, false, true, true>(a, s);
  return hipErrorNotSupported;
}

}  // namespace vds_ec
