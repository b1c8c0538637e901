// ec_restore_syn.hpp -- k_restore_syn<K,N>: restore of an object from any K
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
//
// The instantiations are compiled in parallel, one translation unit per
// group (ec_restore_syn_16.hip, _32a.hip, _32b.hip), behind syn_launch<K>()
// with one SynKind per kernel family; ec_restore_syn.hip dispatches.
#pragma once

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



// =================================================================== launchers

template <int K, int N, int WV, bool REGEN, bool BATCH = false, bool RT = false, class FILL = NoFill>
static hipError_t launch_restore_syn_kn(const SynRestoreArgs &a, hipStream_t s) {
  using S = SynShape<K, N, WV>;
  hipError_t e = ensure_lds_attr(&k_restore_syn<K, N, WV, REGEN, BATCH, RT, FILL>, S::kLdsBytes);
  if (e != hipSuccess) return e;
  const int blocks_per_cu = (160 * 1024) / S::kLdsBytes;
  uint32_t grid = 256u * (blocks_per_cu > 0 ? blocks_per_cu : 1);
  if (VDS_SYN_GRID > 0) grid = VDS_SYN_GRID;
  if (grid > a.total_tiles) grid = a.total_tiles;
  if (grid == 0) return hipSuccess;
  hipLaunchKernelGGL((k_restore_syn<K, N, WV, REGEN, BATCH, RT, FILL>), dim3(grid), dim3(S::kThreads), S::kLdsBytes, s, a);
  return hipGetLastError();
}

enum class SynKind { kPlain, kBatch, kRt, kSmall1, kSmall2, kPerm, kMulti };

// One kernel family at K (N = K + K / 4, WV = K / 4): defined by the
// instantiation units (ec_restore_syn_16.hip: every kind at K = 16;
// _32a.hip: plain, batch, RT at K = 32; _32b.hip: SMALL, PERM, MULTI).
hipError_t syn_launch_16(SynKind kind, const SynRestoreArgs &a, hipStream_t s, bool regen);
hipError_t syn_launch_32a(SynKind kind, const SynRestoreArgs &a, hipStream_t s, bool regen);
hipError_t syn_launch_32b(SynKind kind, const SynRestoreArgs &a, hipStream_t s, bool regen);
#if VDS_DIAG_STAMPS
hipError_t syn_stamps_16(unsigned long long *host, size_t n);  // (this unit's g_syn_stamps)
hipError_t syn_stamps_32a(unsigned long long *host, size_t n);
hipError_t syn_stamps_32b(unsigned long long *host, size_t n);
#endif

template <int K, int N, int WV, SynKind KIND>
hipError_t syn_launch_kind(const SynRestoreArgs &a, hipStream_t s, bool regen) {
  if constexpr (KIND == SynKind::kPlain)
    return regen ? launch_restore_syn_kn<K, N, WV, true>(a, s) : launch_restore_syn_kn<K, N, WV, false>(a, s);
  if constexpr (KIND == SynKind::kBatch)
    return regen ? launch_restore_syn_kn<K, N, WV, true, true>(a, s) : launch_restore_syn_kn<K, N, WV, false, true>(a, s);
  if constexpr (KIND == SynKind::kRt)
    return regen ? launch_restore_syn_kn<K, N, WV, true, true, true>(a, s)
                 : launch_restore_syn_kn<K, N, WV, false, true, true>(a, s);
  if constexpr (KIND == SynKind::kSmall1)
    return regen ? launch_restore_syn_kn<K, N, WV, true, true, false, SmallSyn<K, 1>>(a, s)
                 : launch_restore_syn_kn<K, N, WV, false, true, false, SmallSyn<K, 1>>(a, s);
  if constexpr (KIND == SynKind::kSmall2)
    return regen ? launch_restore_syn_kn<K, N, WV, true, true, false, SmallSyn<K, 2>>(a, s)
                 : launch_restore_syn_kn<K, N, WV, false, true, false, SmallSyn<K, 2>>(a, s);
  if constexpr (KIND == SynKind::kPerm)
    return regen ? launch_restore_syn_kn<K, N, WV, true, true, false, PermSyn<K>>(a, s) : hipErrorNotSupported;
  if constexpr (KIND == SynKind::kMulti)
    return regen ? launch_restore_syn_kn<K, N, WV, true, true, false, MultiP<K>>(a, s)
                 : launch_restore_syn_kn<K, N, WV, false, true, false, MultiP<K>>(a, s);
  return hipErrorNotSupported;
}

}  // namespace vds_ec
