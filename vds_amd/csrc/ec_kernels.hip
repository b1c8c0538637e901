// ec_kernels.hip -- CDNA4 (gfx950) kernels of the object-chunk erasure codec.
//
//  * k_encode_generic / k_restore_generic: any k, any replica ids, 8- or
//    16-bit cells.  One lane per output cell, carry-less field multiply.
//    These handle the tails of the fast kernels and every shape the fast
//    kernels are not instantiated for.
//  * k_encode_bs<K,N>: bit-sliced encode of replicas 0..N-1 for full tiles of
//    2048 stripes (lane = set of 32 stripes, one bit per stripe in each
//    32-bit plane).  The workgroup's waves split the input transposes, share
//    the bit planes through LDS, and each wave evaluates a compile-time group
//    of replicas by Horner with constant multipliers (chunk.h:245-281 is a
//    polynomial evaluation at the replica id).
//  * k_restore_bs<K>: bit-sliced restore with the k x k inverse as
//    wave-uniform runtime constants (chunk.h:402-444).
//  * k_fill_splitmix: synthetic objects on the device.
#include <hip/hip_runtime.h>

#include <array>
#include <utility>

#include "bitslice.hpp"
#include "ec_internal.hpp"

namespace vds_ec {

// ============================================================ generic kernels

template <int CB>
__device__ __forceinline__ uint32_t gf_mul_cell(uint32_t a, uint32_t b) {
  if constexpr (CB == 2)
    return gf16_mul(a, b);
  else
    return gf8_mul(a, b);
}

// Cell j of stripe t of an object, zero beyond `size` (chunk.h:254-260).
template <int CB>
__device__ __forceinline__ uint32_t read_cell(const uint8_t *obj, uint64_t size, uint64_t t, uint32_t j,
                                              uint32_t k, bool native) {
  const uint64_t pos = (t * k + j) * CB;
  if constexpr (CB == 1) {
    return pos < size ? obj[pos] : 0u;
  } else {
    if (native) {  // cell arrays: whole native uint16 cells (chunk.h:213-221)
      return pos + 1 < size ? (uint32_t)(obj[pos] | (obj[pos + 1] << 8)) : 0u;
    }
    uint32_t hi = pos < size ? obj[pos] : 0u;
    uint32_t lo = pos + 1 < size ? obj[pos + 1] : 0u;
    return (hi << 8) | lo;
  }
}

template <int CB>
__global__ void k_encode_generic(GenericEncodeArgs a) {
  const uint64_t per_rep = a.t_count + (a.write_trailer ? 1 : 0);
  const uint64_t total = per_rep * a.nrep * (uint64_t)a.count;
  const bool native = (a.flags & 0x2u) != 0;
  for (uint64_t idx = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; idx < total;
       idx += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t ti = idx % per_rep;
    const uint64_t rest = idx / per_rep;
    const uint32_t i = (uint32_t)(rest % a.nrep);
    const uint32_t o = (uint32_t)(rest / a.nrep);
    uint8_t *out = a.outs[i] + (uint64_t)o * a.out_stride;
    if (ti == a.t_count) {
      // trailer BE16(size % (k*cell)) after the T cells (chunk.h:273-275)
      const uint64_t pad = a.size % ((uint64_t)a.k * CB);
      out[a.stripes * CB] = (uint8_t)(pad >> 8);
      out[a.stripes * CB + 1] = (uint8_t)(pad & 0xFF);
      continue;
    }
    const uint64_t t = a.t_begin + ti;
    const uint8_t *obj = a.in + (uint64_t)o * a.in_stride;
    const uint32_t node = a.nodes[i];
    uint32_t acc = 0;
    for (int32_t j = (int32_t)a.k - 1; j >= 0; --j)  // Horner: sum_j node^j x_j
      acc = gf_mul_cell<CB>(acc, node) ^ read_cell<CB>(obj, a.size, t, (uint32_t)j, a.k, native);
    if constexpr (CB == 2) {
      if (native) {
        out[2 * t] = (uint8_t)(acc & 0xFF);
        out[2 * t + 1] = (uint8_t)(acc >> 8);
      } else {
        out[2 * t] = (uint8_t)(acc >> 8);  // binary_serialize.cpp:18-22
        out[2 * t + 1] = (uint8_t)(acc & 0xFF);
      }
    } else {
      out[t] = (uint8_t)acc;
    }
  }
}

template <int CB>
__global__ void k_restore_generic(GenericRestoreArgs a) {
  const uint64_t per_obj = a.t_count * a.k;
  const uint64_t total = per_obj * a.count;
  const bool native = (a.flags & 0x2u) != 0;
  for (uint64_t idx = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; idx < total;
       idx += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t o = (uint32_t)(idx / per_obj);
    const uint64_t r = idx % per_obj;
    const uint64_t t = a.t_begin + r / a.k;
    const uint32_t m = (uint32_t)(r % a.k);
    const uint64_t pos = (t * a.k + m) * CB;
    if (pos >= a.out_len) continue;
    uint32_t acc = 0;
    const uint64_t row = (uint64_t)m * a.k;
    for (uint32_t j = 0; j < a.k; ++j) {
      const uint8_t *base = a.chunk_pitch ? a.chunk_base + (uint64_t)j * a.chunk_pitch
                                          : (a.chunk_table ? a.chunk_table[j] : a.chunk_ptr[j]);
      const uint8_t *c = base + (uint64_t)o * a.chunk_stride + t * CB;
      const uint64_t e = row + j;
      const uint32_t coef = a.matrix_dev ? a.matrix_dev[e] : (a.matrix_inline[e >> 1] >> (16 * (e & 1))) & 0xFFFFu;
      uint32_t cell;
      if constexpr (CB == 2)
        cell = native ? (uint32_t)(c[0] | (c[1] << 8)) : (uint32_t)((c[0] << 8) | c[1]);
      else
        cell = c[0];
      acc ^= gf_mul_cell<CB>(coef, cell);
    }
    uint8_t *out = a.out + (uint64_t)o * a.out_stride;
    if constexpr (CB == 2) {
      const uint8_t b0 = native ? (uint8_t)(acc & 0xFF) : (uint8_t)(acc >> 8);
      const uint8_t b1 = native ? (uint8_t)(acc >> 8) : (uint8_t)(acc & 0xFF);
      out[pos] = b0;
      if (pos + 1 < a.out_len) out[pos + 1] = b1;  // trimmed to E bytes (chunk.h:437-439)
    } else {
      out[pos] = (uint8_t)acc;
    }
  }
}

// ========================================================== bit-sliced encode

constexpr int popcount32(uint32_t v) {
  int c = 0;
  for (int i = 0; i < 32; ++i) c += (v >> i) & 1u;
  return c;
}


// VALU cost of one row-form Horner step for replica r (bitslice.hpp): used
// to balance replicas across waves.
constexpr int horner_cost(int r) { return r == 0 ? 1 : row_horner_cost((uint32_t)r); }

template <int N, int WAVES, int RPW>
struct ReplicaPlan {
  int rep[WAVES][RPW];
};

// Longest-processing-time assignment of replicas 0..N-1 to waves.
template <int N, int WAVES, int RPW>
constexpr ReplicaPlan<N, WAVES, RPW> plan_replicas() {
  ReplicaPlan<N, WAVES, RPW> p{};
  int load[WAVES] = {};
  int cnt[WAVES] = {};
  bool used[N] = {};
  int cost[N] = {};
  for (int r = 0; r < N; ++r) cost[r] = horner_cost(r);
  for (int w = 0; w < WAVES; ++w)
    for (int s = 0; s < RPW; ++s) p.rep[w][s] = -1;
  for (int it = 0; it < N; ++it) {
    int best = -1;
    for (int r = 0; r < N; ++r)
      if (!used[r] && (best < 0 || cost[r] > cost[best])) best = r;
    used[best] = true;
    int bw = -1;
    for (int w = 0; w < WAVES; ++w)
      if (cnt[w] < RPW && (bw < 0 || load[w] < load[bw])) bw = w;
    p.rep[bw][cnt[bw]++] = best;
    load[bw] += cost[best];
  }
  return p;
}

template <int K, int N, int RPW, int WV>
struct EncodeShape {
  // Loads: every lane takes two dwords (4 cells) of each of its set's 32
  // stripes, so K/4 lanes cover a stripe and one wave covers 256/K sets: a
  // wave-load instruction reads 256/K whole consecutive stripes = 512 B
  // contiguous.  The WV = K/4 waves then split the replicas.
  static constexpr int kWaves = WV;
  static constexpr int kThreads = kWaves * 64;
  static constexpr int kLanesPerSet = K / 4;
  static constexpr int kSetsPerWave = 64 / kLanesPerSet;
  // LDS: set s (= the Horner lane) holds cell c's 16 planes at dword
  // 16 c + kGroupPad (c / 4); the set stride is 4 mod 32 dwords.  Both the
  // transposes' ds_write_b128 (lanes = cell groups of a few sets) and the
  // Horner's ds_read_b128 (lanes = sets) are then bank-conflict free.
  static constexpr int kGroupPad = (K % 32 == 0) ? 4 : 8;
  static constexpr int kSetData = 16 * K + kGroupPad * (K / 4);
  static constexpr int kSetWords = kSetData + ((4 - kSetData % 32) + 32) % 32;
  static constexpr int kPlaneBytes = 64 * kSetWords * 4;
  static constexpr int kLdsBytes = kPlaneBytes;
  static constexpr int kWavesPerSimd = 2;  // 256 VGPRs: accumulators ping-pong + the prefetched tile
  static constexpr int kMap = kLanesPerSet >= 2 ? 3 : 0;  // slot map (store_replica_groups); k = 4: 0
  static constexpr ReplicaPlan<N, kWaves, RPW> kPlan = plan_replicas<N, kWaves, RPW>();
  static_assert(K % 4 == 0 && WV == K / 4, "fast encode: k % 4 == 0 and k/4 waves");
  static_assert(RPW * WV >= N, "every replica needs a wave");
  __device__ __forceinline__ static constexpr int cell_off(int c) { return 16 * c + kGroupPad * (c >> 2); }
};

// Four ds_read_b128 per cell.  A volatile 128-bit load through an LDS
// (address_space(3)) pointer keeps the compiler from splitting the reads into
// ds_read2_b32 / ds_read_b64, which bank-conflict at this padding.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) const volatile u32x4 lds_u32x4;

__device__ __forceinline__ Plane16 lds_planes(const uint32_t *p) {
  Plane16 x;
  lds_u32x4 *q = (lds_u32x4 *)(p);
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const u32x4 v = q[m];
    x.p[4 * m + 0] = v.x;
    x.p[4 * m + 1] = v.y;
    x.p[4 * m + 2] = v.z;
    x.p[4 * m + 3] = v.w;
  }
  return x;
}

#ifndef VDS_DIAG_ENC  // diagnostic builds (timing only, wrong results): 1 = no stores and no output
#define VDS_DIAG_ENC 0  // transposes, 2 = no Horner, 3 = no stores, 5 = 16-byte stores
#endif                  // (same bytes, wrong layout)

// Transpose one replica's planes back to big-endian cells and store them.
// After the transpose, word q of lane l holds the cells of stripes l + 64 q
// (low half) and l + 1024 + 64 q (high half); each half goes out as a 2-byte
// store (global_store_short / _d16_hi), so one wave-instruction writes 128
// contiguous bytes and no cross-lane shuffle is needed.
__device__ __forceinline__ void store_replica(const Plane16 &acc, uint8_t *base, const BitMasks &bm) {
  uint32_t rows[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) rows[j] = acc.p[j ^ 8];  // word bit j <-> cell bit j^8 (BE)
  transpose16x2(rows, bm);
#if VDS_DIAG_ENC == 3
  if (((uintptr_t)base & 1) == 0) return;  // transposes kept, stores never run for real tiles
#endif
#if VDS_DIAG_ENC == 5  // dwordx4 stores, 1 KiB per instruction (wrong layout: timing only)
  base -= 2 * (threadIdx.x & 63);
#pragma unroll
  for (int q = 0; q < 4; ++q)
    *reinterpret_cast<uint4 *>(base + 1024 * q + 16 * (threadIdx.x & 63)) =
        make_uint4(rows[4 * q], rows[4 * q + 1], rows[4 * q + 2], rows[4 * q + 3]);
  return;
#endif
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    *reinterpret_cast<uint16_t *>(base + 128 * q) = (uint16_t)rows[q];
    *reinterpret_cast<uint16_t *>(base + 2048 + 128 * q) = (uint16_t)(rows[q] >> 16);
  }
}

// acc[s] <- acc[s] * r_s + x for this wave's replicas (replica 0 is skipped:
// it is cell 0 itself and is taken from the last x).
typedef __attribute__((address_space(3))) char lds_stage;

// acc[i] <- acc[i] * r + x for replicas r = plan slots S0 .. S0+PR-1 of wave
// W (replica 0, and empty slots, are skipped: replica 0 is cell 0 itself).
template <int K, int N, int RPW, int WV, int W, int S0, int PR>
__device__ __forceinline__ void rows_step(Plane16 (&dst)[PR], const Plane16 (&src)[PR], const Plane16 &x) {
  using S = EncodeShape<K, N, RPW, WV>;
  [&]<size_t... I>(std::index_sequence<I...>) {
    constexpr auto rep = [](int i) { return S0 + i < RPW ? S::kPlan.rep[W][S0 + i] : -1; };
    ((rep(I) > 0 ? (void)(dst[I] = plane_horner_rows<(uint32_t)(rep(I) > 0 ? rep(I) : 0)>(src[I], x)) : (void)0), ...);
  }(std::make_index_sequence<PR>{});
}

// Where a tile's cells live.  The batch is one stream of count x F full
// stripes (F = 128 groups_per_obj): group j (128 stripes) of tile t is global
// group 16 t + j, i.e. group q of object o = (16 t + j) / groups_per_obj.  A
// group never straddles two objects, but a tile may (the live production
// shape: k = 32, 64 KiB objects = 8 groups).
struct TilePos {
  uint32_t o, q;  // object and group-in-object of the tile's first group (wave-uniform)
};

__device__ __forceinline__ TilePos tile_pos(const FastEncodeArgs &a, uint32_t tile) {
  const uint32_t g = 16u * tile;
  const uint32_t o = g / a.groups_per_obj;
  return TilePos{o, g - o * a.groups_per_obj};
}

// Map 3 (k >= 8): slots j and 16 + j of set s hold stripes 2s + 128j and
// 2s + 128j + 1, so output word j (low half = slot j, high half = slot 16 + j,
// transpose16x2) is the 4 bytes of stripes 2s, 2s+1 of group j: one dword
// store per word, 256 contiguous bytes per wave-instruction.
// Streaming (non-temporal) global accesses for the data path, A/B switch:
// VDS_NT bit 1 = encode replica stores, 2 = encode object loads, 4 = restore
// survivor loads, 8 = restore / regenerate stores.  Every byte is read or
// written exactly once, so nothing is lost by not keeping it in L2.  Only for
// whole-line wave accesses: k_restore_bs with non-temporal 4-byte strided
// stores and loads measured 3.4x slower (live shape repair 212 -> 79 GiB/s),
// so it keeps plain accesses.
#ifndef VDS_NT
#define VDS_NT 13  // A/B (512 x 64 MiB, 3 rounds): 0 -> 840, 13 -> 859, 15 -> 856 GiB/s encode+repair
#endif
template <int BIT, class T>
__device__ __forceinline__ T g_ld(const void *p) {
  if constexpr ((VDS_NT & BIT) != 0) return __builtin_nontemporal_load(reinterpret_cast<const T *>(p));
  else return *reinterpret_cast<const T *>(p);
}
template <int BIT, class T>
__device__ __forceinline__ void g_st(void *p, T v) {
  if constexpr ((VDS_NT & BIT) != 0) __builtin_nontemporal_store(v, reinterpret_cast<T *>(p));
  else *reinterpret_cast<T *>(p) = v;
}

template <bool STREAM>
__device__ __forceinline__ void store_replica_groups(const Plane16 &acc, uint8_t *rep, const FastEncodeArgs &a,
                                                     TilePos tp, int lane, const BitMasks &bm) {
  uint32_t rows[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) rows[j] = acc.p[j ^ 8];  // word bit j <-> cell bit j^8 (BE)
  transpose16x2(rows, bm);
#if VDS_DIAG_ENC == 3
  if (tp.o != 0xFFFFFFFFu) return;  // transposes kept, stores never run
#endif
  // (replica strides L = 2T + 2 leave odd objects 2-byte aligned: gfx950
  // global stores need no natural alignment, tested by the strided batches)
  if constexpr (!STREAM) {  // whole tiles per object: one base, immediate offsets
    uint32_t *b = reinterpret_cast<uint32_t *>(rep + (uint64_t)tp.o * a.out_stride + 256u * tp.q + 4 * lane);
#pragma unroll
    for (int j = 0; j < 16; ++j) g_st<1>(b + 64 * j, rows[j]);
  } else {
    uint32_t o = tp.o, q = tp.q;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      g_st<1>(rep + (uint64_t)o * a.out_stride + 256u * q + 4 * lane, rows[j]);
      if (++q == a.groups_per_obj) {
        q = 0;
        ++o;
      }
    }
  }
}

template <int MAP, bool STREAM>
__device__ __forceinline__ void store_rep(const Plane16 &acc, uint8_t *rep, const FastEncodeArgs &a, TilePos tp,
                                          int lane, const BitMasks &bm) {
#if VDS_DIAG_ENC == 1
  if (tp.o != 0xFFFFFFFFu) return;  // never stores
#endif
  if constexpr (MAP == 0)  // k = 4: whole tiles of one object
    store_replica(acc, rep + (uint64_t)tp.o * a.out_stride + 256u * tp.q + 2 * lane, bm);
  else
    store_replica_groups<STREAM>(acc, rep, a, tp, lane, bm);
}

#ifndef VDS_ENC_CONTIG
#define VDS_ENC_CONTIG 0  // A/B: contiguous ranges measured slower (encode 1923 -> 1814 GiB/s)
#endif

#ifndef VDS_ENC_PRIO  // wave priority while a pass issues its stores (A/B; 0 = off)
#define VDS_ENC_PRIO 2  // A/B (512 objects, 2 rounds): encode 1881-1895 -> 1917-1918 GiB/s
#endif

#ifndef VDS_ENC_PASS  // replicas evaluated per pass over the tile's cells (k = 4, 32)
#define VDS_ENC_PASS 3
#endif
#ifndef VDS_ENC_PASS32  // k = 32, n = 40, whole tiles (C4)
#define VDS_ENC_PASS32 5  // A/B (256 objects, 2 rounds): 2 -> 1266, 3 -> 1335, 4 -> 1311, 5 -> 1396 GiB/s; no spills at 256 VGPRs
#endif
#ifndef VDS_ENC_PASS64  // k = 32, n = 64 (the live production shape)
#define VDS_ENC_PASS64 3
#endif
#ifndef VDS_ENC_PASS16  // the same for k = 16 (A/B with the non-temporal, prioritised stores, 512
#define VDS_ENC_PASS16 5  // objects, 2 rounds: 1 -> 1740, 2 -> 1825, 3 -> 1867, 5 -> 1914 GiB/s encode;
#endif                    // 5 at k = 32 spills)

// One pass: Horner for plan slots S0 .. S0+PR-1 over cells K-1 .. 0, then the
// stores.  Two Horner steps per iteration, so the accumulators alternate
// between A and B and the loop carries no register copies.  Splitting a
// wave's replicas into passes spreads its stores over the tile instead of
// one burst at the end (the kernel is write-bound when they bunch up).
template <int K, int N, int RPW, int WV, int W, int S0, int PR, bool ST>
__device__ __forceinline__ void encode_pass(const uint32_t *set_planes, const FastEncodeArgs &a, TilePos tp, int lane,
                                            const BitMasks &bm) {
  using S = EncodeShape<K, N, RPW, WV>;
  constexpr bool kAnyHorner = [] {
    for (int s = S0; s < S0 + PR && s < RPW; ++s)
      if (S::kPlan.rep[W][s] > 0) return true;
    return false;
  }();
  if constexpr (!kAnyHorner) {  // only replica 0 (= cell 0) or empty slots
#pragma unroll
    for (int s = S0; s < S0 + PR && s < RPW; ++s)
      if (S::kPlan.rep[W][s] == 0)
        store_rep<S::kMap, ST>(lds_planes(set_planes + S::cell_off(0)), a.outs[0], a, tp, lane, bm);
    return;
  }
  Plane16 A[PR], B[PR];
  {
    const Plane16 x = lds_planes(set_planes + S::cell_off(K - 1));
#pragma unroll
    for (int s = 0; s < PR; ++s) A[s] = x;
  }
  Plane16 xa = lds_planes(set_planes + S::cell_off(K - 2));
#pragma clang loop unroll(disable)
  for (int c = K - 2; c >= 1 && VDS_DIAG_ENC != 2; c -= 2) {
    const Plane16 xb = lds_planes(set_planes + S::cell_off(c - 1));
    rows_step<K, N, RPW, WV, W, S0, PR>(B, A, xa);
    xa = lds_planes(set_planes + S::cell_off(c - 2));
    rows_step<K, N, RPW, WV, W, S0, PR>(A, B, xb);
  }
  rows_step<K, N, RPW, WV, W, S0, PR>(A, A, xa);  // cell 0 (each step returns a fresh value)
  if constexpr (VDS_ENC_PRIO > 0) __builtin_amdgcn_s_setprio(VDS_ENC_PRIO);
#pragma unroll
  for (int s = 0; s < PR; ++s) {
    const int r = S0 + s < RPW ? S::kPlan.rep[W][S0 + s] : -1;
    if (r == 0) store_rep<S::kMap, ST>(xa, a.outs[0], a, tp, lane, bm);
    if (r > 0) store_rep<S::kMap, ST>(A[s], a.outs[r], a, tp, lane, bm);
  }
  if constexpr (VDS_ENC_PRIO > 0) __builtin_amdgcn_s_setprio(0);
}

template <int K, int N, int RPW, int WV, int W, bool ST, int S0 = 0>
__device__ __forceinline__ void encode_wave_group(const uint32_t *set_planes, const FastEncodeArgs &a, TilePos tp,
                                                  int lane, const BitMasks &bm) {
  constexpr int kPass = K == 16                     ? VDS_ENC_PASS16
                        : (K == 32 && N == 40 && !ST) ? VDS_ENC_PASS32
                        : (K == 32 && N == 64)        ? VDS_ENC_PASS64
                                                      : VDS_ENC_PASS;
  constexpr int PR = kPass < RPW ? kPass : RPW;
  if constexpr (S0 < RPW) {
    encode_pass<K, N, RPW, WV, W, S0, PR, ST>(set_planes, a, tp, lane, bm);
    encode_wave_group<K, N, RPW, WV, W, ST, S0 + PR>(set_planes, a, tp, lane, bm);
  }
}

template <int K, int N, int RPW, int WV, bool ST, int W>
__device__ __forceinline__ void encode_dispatch(int wave, const uint32_t *set_planes, const FastEncodeArgs &a, TilePos tp,
                                                int lane, const BitMasks &bm) {
  using S = EncodeShape<K, N, RPW, WV>;
  if constexpr (W < S::kWaves) {
    if (wave == W)
      encode_wave_group<K, N, RPW, WV, W, ST>(set_planes, a, tp, lane, bm);
    else
      encode_dispatch<K, N, RPW, WV, ST, W + 1>(wave, set_planes, a, tp, lane, bm);
  }
}

// k = 4: load dwords 2p, 2p+1 of the 32 stripes of set `set`; slot i <->
// stripe stripe0 + s + 64 i (whole tiles of one object).  The data stays in
// the loaded vector registers until the next iteration unpacks it, so no copy
// forces an early s_waitcnt.
template <int K>
__device__ __forceinline__ void encode_load(u32x2 (&P)[32], const FastEncodeArgs &a, uint32_t tile, int set, int p) {
  const TilePos tp = tile_pos(a, tile);
  const uint8_t *src = a.in + (uint64_t)tp.o * a.in_stride + ((uint64_t)128 * tp.q + set) * (2 * K) + 8 * p;
#pragma unroll
  for (int i = 0; i < 32; ++i) P[i] = *reinterpret_cast<const u32x2 *>(src + (uint64_t)i * 64 * (2 * K));
}

// k >= 8: 16-byte pair loads.  The lanes of an adjacent pair (same set, p =
// 2u + par) each load one whole 16-byte chunk u -- par 0 of stripe 2s + 128j
// (slot j), par 1 of stripe 2s + 128j + 1 (slot 16 + j) -- and swap halves
// with one DPP quad_perm, so every lane ends with dwords 2p, 2p+1 of both.  A
// wave-load reads 256/k * 2 whole stripes = 1 KiB contiguous, 16 B per lane.
template <int K, bool STREAM>
__device__ __forceinline__ void encode_load16(u32x4 (&V)[16], const FastEncodeArgs &a, uint32_t tile, int set, int p) {
  const TilePos tp = tile_pos(a, tile);
  const uint64_t lane_off = (uint64_t)(2 * set + (p & 1)) * (2 * K) + 16 * (p >> 1);
  uint32_t o = tp.o, q = tp.q;
  if constexpr (!STREAM) {  // whole tiles per object
    const uint8_t *src = a.in + (uint64_t)o * a.in_stride + (uint64_t)q * 128 * (2 * K) + lane_off;
#pragma unroll
    for (int j = 0; j < 16; ++j) V[j] = g_ld<2, u32x4>(src + (uint64_t)j * 128 * (2 * K));
    return;
  }
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    V[j] = g_ld<2, u32x4>(a.in + (uint64_t)o * a.in_stride + (uint64_t)q * 128 * (2 * K) + lane_off);
    if (++q == a.groups_per_obj) {
      q = 0;
      ++o;
    }
  }
}

// R[g][i] = dword 2p + g of slot i's stripe, from the loaded chunks (pair j
// holds slots j and 16 + j).
__device__ __forceinline__ void encode_unpack16(const u32x4 (&V)[16], uint32_t (&R)[2][32], bool par) {
#pragma unroll
  for (int m = 0; m < 16; ++m) {
    const u32x4 v = V[m];
    const uint32_t s0 = par ? v.x : v.z, s1 = par ? v.y : v.w;   // the partner's half
    const uint32_t r0 = __builtin_amdgcn_mov_dpp(s0, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
    const uint32_t r1 = __builtin_amdgcn_mov_dpp(s1, 0xB1, 0xF, 0xF, false);
    R[0][m] = par ? r0 : v.x;
    R[1][m] = par ? r1 : v.y;
    R[0][16 + m] = par ? v.z : r0;
    R[1][16 + m] = par ? v.w : r1;
  }
}

// STREAM: tiles may straddle objects (groups_per_obj % 16 != 0, k >= 8); the
// non-stream instantiation keeps one base address per tile.
template <int K, int N, int RPW, int WV, bool STREAM>
__global__ __launch_bounds__((EncodeShape<K, N, RPW, WV>::kThreads), (EncodeShape<K, N, RPW, WV>::kWavesPerSimd))
void k_encode_bs(FastEncodeArgs a) {
  using S = EncodeShape<K, N, RPW, WV>;
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // transposes: this lane's set and 4-cell group; Horner: lane = set
  const int tset = wave * S::kSetsPerWave + lane / S::kLanesPerSet;
  const int tp = lane % S::kLanesPerSet;
  uint32_t *t_planes = lds + tset * S::kSetWords + S::cell_off(4 * tp);
  const uint32_t *my_set = lds + lane * S::kSetWords;
  const BitMasks bm = bit_masks();

  constexpr bool kLoad16 = S::kMap != 0;
  u32x2 P[kLoad16 ? 1 : 32];
  u32x4 V[kLoad16 ? 16 : 1];
  const bool par = (lane & 1) != 0;
  auto load = [&](uint32_t t) {
    if constexpr (kLoad16)
      encode_load16<K, STREAM>(V, a, t, tset, tp);
    else
      encode_load<K>(P, a, t, tset, tp);
  };
#if VDS_ENC_CONTIG  // A/B: one contiguous range of tiles per workgroup
  const uint32_t t_per = (a.total_tiles + gridDim.x - 1) / gridDim.x;
  uint32_t tile = blockIdx.x * t_per;
  const uint32_t t_end = tile + t_per < a.total_tiles ? tile + t_per : a.total_tiles;
  const uint32_t t_step = 1;
#else
  uint32_t tile = blockIdx.x;
  const uint32_t t_end = a.total_tiles, t_step = gridDim.x;
#endif
  if (tile < t_end) load(tile);
  for (; tile < t_end; tile += t_step) {
    // ---- transpose to planes and publish in LDS: cell 4p+2g+h, bit b = R[g][16h + (b^8)]
    uint32_t R[2][32];
    if constexpr (kLoad16) {
      encode_unpack16(V, R, par);
    } else {
#pragma unroll
      for (int i = 0; i < 32; ++i) {
        R[0][i] = P[i].x;
        R[1][i] = P[i].y;
      }
    }
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      transpose32(R[g], bm);
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          const int b0 = 16 * h + 4 * (m ^ 2);
          *reinterpret_cast<uint4 *>(t_planes + (2 * g + h) * 16 + 4 * m) =
              make_uint4(R[g][b0], R[g][b0 + 1], R[g][b0 + 2], R[g][b0 + 3]);
        }
    }
    __syncthreads();
    // ---- prefetch the next tile while this one is evaluated (software pipeline)
    const uint32_t next = tile + t_step;
    if (next < t_end) load(next);
    // ---- evaluate this wave's replicas and store
    encode_dispatch<K, N, RPW, WV, STREAM, 0>(wave, my_set, a, tile_pos(a, tile), lane, bm);
    __syncthreads();
  }
}

// ========================================================= bit-sliced restore

template <int K>
struct RestoreShape {
  static constexpr int kPerWave = 4;           // survivors loaded / outputs computed per wave
  static constexpr int kWaves = K / kPerWave;
  static constexpr int kThreads = 64 * kWaves;
  static constexpr int kSetWords = K * 16 + 4;
  static constexpr int kLdsBytes = 64 * kSetWords * 4;
  static_assert(K % 8 == 0, "restore fast path needs k % 8 == 0");
};

// slot i (0..31) of lane l <-> stripe stripe0 + 8 l + 512 (i / 8) + (i % 8);
// bit position pi of a plane <-> slot (pi < 16 ? 2 pi : 2 (pi - 16) + 1).
__device__ __forceinline__ uint64_t restore_slot_stripe(int lane, int slot) {
  return 8u * lane + 512u * (slot >> 3) + (slot & 7);
}

// Tiles in 512-stripe groups (1 KiB of every survivor): group q of tile t is
// global group 4 t + q = group r of object o (groups_per_obj per object).
// STREAM: tiles may straddle objects (small objects, groups_per_obj % 4 != 0).
__device__ __forceinline__ void restore_group(const FastRestoreArgs &a, uint32_t tile, uint32_t q, uint32_t &o,
                                              uint32_t &r) {
  const uint32_t g = 4u * tile + q;
  o = g / a.groups_per_obj;
  r = g - o * a.groups_per_obj;
}

template <int K, bool STREAM>
__device__ __forceinline__ void restore_load(u32x4 (&Q)[RestoreShape<K>::kPerWave][4], const FastRestoreArgs &a,
                                             uint32_t tile, int lane, int wave) {
  using S = RestoreShape<K>;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    uint32_t o, r;
    restore_group(a, tile, STREAM ? q : 0, o, r);
    const uint64_t off = (uint64_t)o * a.chunk_stride + 1024ull * (STREAM ? r : r + q) + 16 * lane;
#pragma unroll
    for (int s = 0; s < S::kPerWave; ++s) Q[s][q] = *reinterpret_cast<const u32x4 *>(a.chunks[wave * S::kPerWave + s] + off);
  }
}

template <int K, bool STREAM, bool REGEN>
__global__ __launch_bounds__((RestoreShape<K>::kThreads), 2) void k_restore_bs(FastRestoreArgs a) {
  using S = RestoreShape<K>;
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint32_t *my_set = lds + lane * S::kSetWords;

  u32x4 Q[S::kPerWave][4];
  uint32_t tile = blockIdx.x;
  if (tile < a.total_tiles) restore_load<K, STREAM>(Q, a, tile, lane, wave);
  for (; tile < a.total_tiles; tile += gridDim.x) {
    uint32_t W[S::kPerWave][16];
#pragma unroll
    for (int s = 0; s < S::kPerWave; ++s)
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int d = 0; d < 4; ++d) W[s][4 * q + d] = Q[s][q][d];
    // ---- transpose this wave's survivors to planes: W[x] = plane of cell bit x^8
#pragma unroll
    for (int s = 0; s < S::kPerWave; ++s) {
      const int j = wave * S::kPerWave + s;
      transpose16x2(W[s]);
#pragma unroll
      for (int m = 0; m < 4; ++m)
        *reinterpret_cast<uint4 *>(my_set + j * 16 + 4 * m) =
            make_uint4(W[s][4 * (m ^ 2)], W[s][4 * (m ^ 2) + 1], W[s][4 * (m ^ 2) + 2], W[s][4 * (m ^ 2) + 3]);
    }
    __syncthreads();
    const uint32_t next = tile + gridDim.x;
    if (next < a.total_tiles) restore_load<K, STREAM>(Q, a, next, lane, wave);
    // ---- outputs m = wave*kPerWave + s : sum_j M[m][j] * Y_j
    Plane16 acc[S::kPerWave];
#pragma unroll
    for (int s = 0; s < S::kPerWave; ++s) acc[s] = plane_zero();
    Plane16 yn = lds_planes(my_set);  // one survivor ahead
#pragma clang loop unroll(disable)
    for (int j = 0; j < K; ++j) {
      const Plane16 y = yn;
      if (j + 1 < K) yn = lds_planes(my_set + (j + 1) * 16);
      uint32_t c[S::kPerWave];
#pragma unroll
      for (int s = 0; s < S::kPerWave; ++s) {
        const uint32_t idx = (wave * S::kPerWave + s) * K + j;
        c[s] = (a.matrix2[idx >> 1] >> (16 * (idx & 1))) & 0xFFFFu;
      }
      plane_mac_rt<S::kPerWave>(acc, y, c);
    }
    if constexpr (REGEN) {
      // ---- regenerate: output m is replica regen[m]'s cells for the same
      // stripes the survivors were loaded from; undo the load transpose and
      // store with the load's addressing (1 KiB per wave-instruction)
#pragma unroll
      for (int s = 0; s < S::kPerWave; ++s) {
        const uint32_t m = wave * S::kPerWave + s;
        if (m >= a.nt) continue;
        uint32_t W[16];
#pragma unroll
        for (int b = 0; b < 16; ++b) W[b ^ 8] = acc[s].p[b];
        transpose16x2(W);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          uint32_t o, r;
          restore_group(a, tile, STREAM ? q : 0, o, r);
          uint8_t *dst = a.regen[m] + (uint64_t)o * a.out_stride + 1024ull * (STREAM ? r : r + q) + 16 * lane;
          *reinterpret_cast<u32x4 *>(dst) = u32x4{W[4 * q], W[4 * q + 1], W[4 * q + 2], W[4 * q + 3]};
        }
      }
      __syncthreads();
      continue;
    }
    // ---- back to big-endian cells: word group w' = cells (2w', 2w'+1)
#pragma unroll
    for (int g = 0; g < S::kPerWave / 2; ++g) {
      uint32_t rows[32];
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int jb = 0; jb < 16; ++jb) rows[16 * h + jb] = acc[2 * g + h].p[jb ^ 8];
      transpose32(rows);
      const int wg = (wave * S::kPerWave) / 2 + g;
      // slot 8q+e <-> stripe 8 lane + 512 q + e of the tile (group q); plane bit
      // pi <-> slot (pi < 16 ? 2 pi : 2 (pi-16) + 1)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        uint32_t o, r;
        restore_group(a, tile, STREAM ? q : 0, o, r);
        uint8_t *base = a.out + (uint64_t)o * a.out_stride + ((uint64_t)512 * (STREAM ? r : r + q) + 8u * lane) * (2 * K) +
                        4 * wg;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int slot = 8 * q + e;
          const int pi = (slot & 1) ? 16 + (slot >> 1) : (slot >> 1);
          *reinterpret_cast<uint32_t *>(base + e * (2 * K)) = rows[pi];
        }
      }
    }
    __syncthreads();
  }
}

// ============================================ erasure-pattern-independent restore

template <int K, int N, int WV> struct RestorePrograms;
// Waves per k_restore_syn<16,20> workgroup (two workgroups per CU either way).
// 8 waves (128 VGPRs, 4 waves per SIMD) measured 984 against 1375 GiB/s for 4:
// the doubled barrier fan-in and spills outweigh the occupancy.
#ifndef VDS_SYN_WAVES
#define VDS_SYN_WAVES 4
#endif
#define VDS_SCHED_FENCE() __builtin_amdgcn_sched_barrier(0)
#ifdef VDS_SYN_INC  // A/B builds of alternative generated programs
#include VDS_SYN_INC
#else
#if VDS_SYN_WAVES == 8
#include "generated/restore_16_20_w8.inc"
#else
#include "generated/restore_16_20_w4.inc"
#endif
#endif
#include "generated/restore_32_40_w8.inc"
#undef VDS_SCHED_FENCE

// k_restore_syn<K, N, WV>: one 2048-stripe tile per workgroup of WV waves.
template <int K, int N, int WV>
struct SynShape {
  static constexpr int kWaves = WV;
  static constexpr int kThreads = 64 * WV;
  static constexpr int kM = N - K;
  static constexpr int kLoadPer = K / WV;          // survivors loaded per wave
  using P = RestorePrograms<K, N, WV>;
  static constexpr int kSynRows = P::kSynRows;     // syndrome bit-rows per wave
  static constexpr int kCells = P::kIntRows / 16;  // object cells per wave
  // group-major LDS: plane p = 16 point + bit lives in group p / 4; the four
  // planes of a group are one 16-byte word per lane, so every access is a
  // conflict-free ds_{read,write}_b128 (byte (p/4)*1024 + lane*16 + 4*(p%4))
  static constexpr int kLdsBytes = N * 16 * 64 * 4;
  static constexpr int kWavesPerSimd = (160 * 1024 / kLdsBytes) * WV / 4;
  static_assert(K % WV == 0 && kM <= WV, "survivor loads and erased slots must map onto waves");
  static_assert(kSynRows % 4 == 0 && (kCells == 2 || kCells == 4), "row split must be b128 / word-group aligned");
};

typedef __attribute__((address_space(3))) volatile u32x4 lds_v4;
typedef __attribute__((address_space(3))) char lds_char;

// Diagnostic builds (wrong results; timing only): VDS_DIAG_RES = 1 skips the
// interpolation, 2 the stores, 3 the syndrome programs.
#ifndef VDS_DIAG_RES
#define VDS_DIAG_RES 0
#endif
// Diagnostic build switch (wrong results; timing only): every wave runs wave
// 1's programs, to measure what the per-wave code footprint costs.
#ifndef VDS_SYN_SAME_CODE
#define VDS_SYN_SAME_CODE 0
#endif
constexpr bool kSynSameCode = VDS_SYN_SAME_CODE;

// Diagnostic build (VDS_DIAG_STAMPS=1, timing only): every wave of
// k_restore_syn accumulates s_memtime deltas per phase of its tiles into
// g_syn_stamps[block][wave][phase] (read with vds_ec_diag_stamps; phases in
// tools/syn_stamps.py).  The marks wait for outstanding scalar and LDS
// operations and the compiler may move VALU work across them: read the
// barrier waits, not the exact split of neighbouring phases.  Off: the marks
// compile to nothing.
#ifndef VDS_DIAG_STAMPS
#define VDS_DIAG_STAMPS 0
#endif
#if VDS_DIAG_STAMPS
constexpr int kStampPhases = 20;
constexpr int kStampSlots = 4096 * 4 * kStampPhases;
__device__ unsigned long long g_syn_stamps[kStampSlots];
struct Stamps {
  uint64_t prev, acc[kStampPhases];
  __device__ __forceinline__ void init() {
    prev = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < kStampPhases; ++i) acc[i] = 0;
  }
  __device__ __forceinline__ void mark(int i) {
    const uint64_t now = __builtin_amdgcn_s_memtime();
    acc[i] += now - prev;
    prev = now;
  }
  __device__ __forceinline__ void flush(int slot, int lane) {
    if (lane == 0 && slot < 4096 * 4)
      for (int i = 0; i < kStampPhases; ++i) g_syn_stamps[slot * kStampPhases + i] = acc[i];
  }
};
#else
struct Stamps {
  __device__ __forceinline__ void init() {}
  __device__ __forceinline__ void mark(int) {}
  __device__ __forceinline__ void flush(int, int) {}
};
#endif

// Group g of the plane-major LDS as seen by one lane.  ds_read_b128 carries a
// 16-bit immediate offset, so groups past 64 KiB (points >= 16) are addressed
// from a second base register; the base is laundered through an empty asm so
// the compiler does not fold it back into one address register per group.
struct SynLds {
  lds_char *base;
  uint32_t lo;   // 16 * lane
  uint32_t hi;   // 16 * lane + 64 KiB (opaque)
  uint32_t hi2;  // 16 * lane + 128 KiB (opaque; points 32.. of k = 32)
  // A compile-time group is an immediate offset (< 64 KiB) from one of the
  // three bases, so no per-group address register stays live; a runtime
  // group costs one address add.
  __device__ __forceinline__ lds_char *at(int g) const {
    if (__builtin_constant_p(g)) {
      if (g < 64) return base + lo + g * 1024;
      if (g < 128) return base + hi + (g - 64) * 1024;
      return base + hi2 + (g - 128) * 1024;
    }
    return base + lo + g * 1024;
  }
  __device__ __forceinline__ u32x4 operator()(int g) const { return *(lds_v4 *)at(g); }
  __device__ __forceinline__ void put(int g, u32x4 v) const { *(lds_v4 *)at(g) = v; }
};

__device__ __forceinline__ void syn_put_point(const SynLds &L, int pt, const uint32_t (&v)[16]) {
#pragma unroll
  for (int g = 0; g < 4; ++g) L.put(4 * pt + g, u32x4{v[4 * g], v[4 * g + 1], v[4 * g + 2], v[4 * g + 3]});
}

__device__ __forceinline__ void syn_get_point(const SynLds &L, int pt, uint32_t (&v)[16]) {
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const u32x4 x = L(4 * pt + g);
    v[4 * g] = x[0];
    v[4 * g + 1] = x[1];
    v[4 * g + 2] = x[2];
    v[4 * g + 3] = x[3];
  }
}

#ifndef VDS_SYN_LATE  // k = 32: 1 issues the next tile's survivor loads after the interpolation, 0 after the syndromes
#define VDS_SYN_LATE 1
#endif

#ifndef VDS_SYN_CONTIG  // 1: each workgroup restores one contiguous range of tiles (A/B)
#define VDS_SYN_CONTIG 0  // A/B: contiguous ranges measured slower (repair 1572 -> 1460 GiB/s)
#endif

#ifndef VDS_SYN_PRIO  // wave priority while issuing the survivor loads and the copy-out stores (A/B; 0 = off)
#define VDS_SYN_PRIO 0  // A/B: 2 measured the same as 0 (repair 1598-1602 vs 1604-1606)
#endif

#ifndef VDS_SYN_LATE16  // 1: k = 16 also issues the next tile's loads after the interpolation (A/B)
#define VDS_SYN_LATE16 0
#endif

#ifndef VDS_SYN_REC  // 2: scatter recovery with LDS XOR atomics; 1: gather (parks the syndromes)
#define VDS_SYN_REC 2
#endif

#ifndef VDS_SYN_CFENCE  // 1: one scheduling fence per stage-C term
#define VDS_SYN_CFENCE 0
#endif

#ifndef VDS_SYN_GM  // 1: interpolation by one additive-FFT level + half-size programs; 0: one 16-point program
#define VDS_SYN_GM 1
#endif

// Interpolation from the fixed points F = {0..K-1} by one level of the
// additive FFT (Gao-Mateer).  F is the GF(2)-span of 1, x, x^2, x^3, so with
// G = {0, 2, .., K-2} (the span of x, x^2, x^3) and s(X) = X^2 + X (which maps
// g and g+1 to the same point):
//   P(X) = P0(s(X)) + X P1(s(X)),  deg P0, P1 < K/2,
//   P1(s(g)) = c_g + c_{g+1},  P0(s(g)) = c_g + g P1(s(g)).
// Stage A forms those K/2 value pairs in place (Q0 -> slot g, Q1 -> slot g+1),
// stage B interpolates P0 and P1 on D = s(G) with generated XOR programs
// (RestorePrograms::interpB), and stage C expands (X^2+X)^i = X^i (X+1)^i,
// whose coefficients are binomials mod 2, so it is XORs only.  About 60% of
// the XORs of the direct 16-point program (tools/xorgen/gen_restore.cpp).
template <int W, int NP, int Q = 0>
__device__ __forceinline__ void syn_gm_stage_a(const SynLds &L) {
  if constexpr (Q < NP) {
    constexpr int i = NP * W + Q;  // the pair (g, g + 1) = (2 i, 2 i + 1)
    Plane16 c0, c1;
    syn_get_point(L, 2 * i, c0.p);
    syn_get_point(L, 2 * i + 1, c1.p);
    const Plane16 q1 = plane_xor(c0, c1);
    const Plane16 q0 = plane_horner_rows<(uint32_t)(2 * i)>(q1, c0);
    syn_put_point(L, 2 * i, q0.p);
    syn_put_point(L, 2 * i + 1, q1.p);
    syn_gm_stage_a<W, NP, Q + 1>(L);
  }
}

// Output cell k = sum of P0_i with C(i, k - i) odd and of P1_i with
// C(i, k - 1 - i) odd (Lucas: C(i, m) is odd iff the bits of m are a subset of
// those of i).  P0_i sits in LDS slot i, P1_i in slot K/2 + i.
template <int K, int W, int NC>
__device__ __forceinline__ void syn_gm_stage_c(const SynLds &L, uint32_t (&cells)[16 * NC]) {
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int k = NC * W + c;
    uint32_t acc[16];
#pragma unroll
    for (int b = 0; b < 16; ++b) acc[b] = 0u;
#pragma unroll
    for (int t = 0; t < K; ++t) {
      const int i = t % (K / 2);
      const int m = t < K / 2 ? k - i : k - 1 - i;
      if (m >= 0 && m <= i && (m & ~i) == 0) {
        uint32_t v[16];
        syn_get_point(L, t, v);
#pragma unroll
        for (int b = 0; b < 16; ++b) acc[b] ^= v[b];
#if VDS_SYN_CFENCE
        __builtin_amdgcn_sched_barrier(0);  // keep the scheduler from hoisting every term's reads
#endif
      }
    }
#pragma unroll
    for (int b = 0; b < 16; ++b) cells[16 * c + b] = acc[b];
  }
}

template <int K, int N, int WV, int W>
__device__ __forceinline__ void syn_interp_gm(int wave, const SynLds &L, uint32_t (&cells)[16 * (K / WV)], Stamps &st) {
  static_assert((K == 16 && (WV == 4 || WV == 8)) || (K == 32 && WV == 8),
                "the one-level interpolation is laid out for k = 16 and k = 32");
  using P = RestorePrograms<K, N, WV>;
  constexpr int kPairs = (K / 2) / WV;           // stage-A pairs per wave
  constexpr int kHalfCells = P::kHalfRows / 16;  // stage-B cells per wave
  constexpr int kParts = WV / 2;                 // waves per half-size polynomial
  if constexpr (W < WV) {
    if (wave != W) return syn_interp_gm<K, N, WV, W + 1>(wave, L, cells, st);
    syn_gm_stage_a<W, kPairs>(L);
    st.mark(7);
    __syncthreads();
    st.mark(8);
    uint32_t half[P::kHalfRows];
    P::interpB(W, L, half);
    st.mark(9);
    __syncthreads();  // every wave has read its Q values
    st.mark(10);
    // P0 (W < kParts) or P1 cells kHalfCells (W % kParts) + c -> slot (K/2) (W / kParts) + ..
#pragma unroll
    for (int c = 0; c < kHalfCells; ++c) {
      uint32_t v[16];
#pragma unroll
      for (int b = 0; b < 16; ++b) v[b] = half[16 * c + b];
      syn_put_point(L, (K / 2) * (W / kParts) + kHalfCells * (W % kParts) + c, v);
    }
    st.mark(11);
    __syncthreads();
    st.mark(12);
    syn_gm_stage_c<K, W, K / WV>(L, cells);
    st.mark(13);
  }
}

// Restore of an object from any K of its N replicas without a per-pattern
// K x K inverse (tools/xorgen/gen_restore.cpp).  Per tile, wave w:
//  1. loads survivors kLoadPer*w.. into their points' planes (waves < M also
//     zero one erased point);
//  2. computes syndrome bit-rows kSynRows*w.. over all N points (erased
//     points read as zero) and parks them in the erased slots;
//  3. (waves < M) recovers erased point e_w = sum_j R[w][j] S_j by Horner
//     over the coefficient bits -- the only runtime-coefficient arithmetic;
//  4. interpolates cells kCells*w.. from the fixed points 0..K-1 and stores
//     them big-endian.
template <int K, int N, int WV, bool REGEN>
__global__ __launch_bounds__((SynShape<K, N, WV>::kThreads), (SynShape<K, N, WV>::kWavesPerSimd))
void k_restore_syn(SynRestoreArgs a) {
  using S = SynShape<K, N, WV>;
  using P = typename S::P;
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const BitMasks bm = bit_masks();
  SynLds L;
  L.base = (lds_char *)lds;
  L.lo = 16u * lane;
  L.hi = 16u * lane + 65536u;
  asm volatile("" : "+v"(L.hi));
  if constexpr (N * 16 > 128) {
    L.hi2 = 16u * lane + 131072u;
    asm volatile("" : "+v"(L.hi2));
  } else {
    L.hi2 = L.hi;
  }
  const int my_erased = wave < S::kM ? a.erased[wave] : 0;

  // survivor staging: the next tile's loads are issued after the syndrome
  // programs and land while the recovery and interpolation run
  u32x4 Q[S::kLoadPer][4];
  auto load = [&](uint32_t t) {
    const uint32_t ob = t / a.tiles_per_obj;
    const uint64_t st0 = (uint64_t)(t % a.tiles_per_obj) * kTileStripes;
#pragma unroll
    for (int s = 0; s < S::kLoadPer; ++s) {
      const uint8_t *src = a.chunks[wave * S::kLoadPer + s] + (uint64_t)ob * a.chunk_stride + 2 * st0 + 16 * lane;
#pragma unroll
      for (int q = 0; q < 4; ++q) Q[s][q] = g_ld<4, u32x4>(src + 1024 * q);
    }
  };
  // The next tile's survivors, or zeros past the last tile: both paths define
  // Q, so the values consumed by this tile's stage 1 die there instead of
  // staying live (as loop-carried state) through the programs until the load
  // tiles of this workgroup: strided over the grid, or (VDS_SYN_CONTIG) one
  // contiguous range per workgroup
#if VDS_SYN_CONTIG
  const uint32_t t_per = (a.total_tiles + gridDim.x - 1) / gridDim.x;
  const uint32_t t_begin = blockIdx.x * t_per;
  const uint32_t t_end = t_begin + t_per < a.total_tiles ? t_begin + t_per : a.total_tiles;
  const uint32_t t_step = 1;
#else
  const uint32_t t_begin = blockIdx.x, t_end = a.total_tiles, t_step = gridDim.x;
#endif
  auto prefetch = [&](uint32_t t) {
    if (t < t_end) {
      if constexpr (VDS_SYN_PRIO > 0) __builtin_amdgcn_s_setprio(VDS_SYN_PRIO);
      load(t);
      if constexpr (VDS_SYN_PRIO > 0) __builtin_amdgcn_s_setprio(0);
    } else {
#pragma unroll
      for (int s = 0; s < S::kLoadPer; ++s)
#pragma unroll
        for (int q = 0; q < 4; ++q) Q[s][q] = u32x4{0u, 0u, 0u, 0u};
    }
  };
  Stamps st;
  st.init();
  // k = 32 (one 160 KiB workgroup per CU): the prefetched survivors would be
  // live across the syndrome and stage-B programs, which then spill; they are
  // issued after the interpolation instead and land under the staging and
  // stores (REGEN has no interpolation and keeps the early issue)
  constexpr bool kLateLoad = VDS_SYN_LATE && (K == 32 || VDS_SYN_LATE16) && !REGEN && VDS_SYN_GM;
  // VDS_SYN_LATE 2: issued inside the output staging, once the first word
  // group's cells are dead (no spills of loop-carried state around them)
  constexpr bool kStageLoad = kLateLoad && VDS_SYN_LATE == 2;
  if (t_begin < t_end) load(t_begin);
  for (uint32_t tile = t_begin; tile < t_end; tile += t_step) {
    const uint32_t o = tile / a.tiles_per_obj;
    const uint64_t stripe0 = (uint64_t)(tile % a.tiles_per_obj) * kTileStripes;
    // ---- 1. survivors -> planes of their points; waves < M zero one erased point
    {
      if (wave < S::kM) {
        const u32x4 z = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int g = 0; g < 4; ++g) L.put(4 * my_erased + g, z);
      }
#pragma unroll
      for (int s = 0; s < S::kLoadPer; ++s) {
        uint32_t W[16];
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int d = 0; d < 4; ++d) W[4 * q + d] = Q[s][q][d];
        transpose16x2(W, bm);  // W[x] = plane of cell bit x^8
        uint32_t Pl[16];
#pragma unroll
        for (int b = 0; b < 16; ++b) Pl[b] = W[b ^ 8];
        syn_put_point(L, a.point[wave * S::kLoadPer + s], Pl);
      }
    }
    st.mark(0);
    __syncthreads();
    st.mark(1);
#if VDS_SYN_REC == 2
    // ---- 2+3. wave j holds syndrome S_j whole and scatters its share of every
    // recovered point, c_e[m] += R[m][j] S_j, into the erased slots (zero since
    // stage 1) with LDS XOR atomics: T = x^b S_j walks the coefficient bits
    // once for all M products, and no wave has to gather the syndromes (two
    // barriers and a park/reload of the syndromes fewer than VDS_SYN_REC 1)
    {
      static_assert(S::kSynRows == 16 && S::kM == WV, "scatter recovery needs one whole syndrome per wave");
      Plane16 t;
#if VDS_DIAG_RES == 3
      for (int r = 0; r < 16; ++r) t.p[r] = lane + r;
#else
      P::syndrome(kSynSameCode ? 1 : wave, L, t.p);
#endif
      if (!kLateLoad) prefetch(tile + t_step);
      st.mark(2);
      // M <= 4: all products before the barrier (their walk overlaps the
      // slower waves' syndromes); M = 8: four at a time after it (eight
      // accumulators would not fit beside the prefetched survivors)
      constexpr int kMC = S::kM <= 4 ? S::kM : 4;
      if constexpr (kMC < S::kM) __syncthreads();  // every wave is done reading the zeroed erased planes
#pragma unroll
      for (int m0 = 0; m0 < S::kM; m0 += kMC) {
        Plane16 ce[kMC];
#pragma unroll
        for (int m = 0; m < kMC; ++m) ce[m] = plane_zero();
        Plane16 t_copy;  // several chunks walk from the same syndrome
        Plane16 &tt = kMC < S::kM ? (t_copy = t, t_copy) : t;
#pragma unroll
        for (int b = 0; b < 16; b += 2) {
          const Plane16 t1 = plane_mulx(tt);
#pragma unroll
          for (int m = 0; m < kMC; ++m) {
            const uint32_t two = (a.solve_sel[m0 + m][b >> 2] >> (8 * (b & 3) + wave)) & 0x101u;
            if (two == 1u)
              ce[m] = plane_xor(ce[m], tt);
            else if (two == 0x100u)
              ce[m] = plane_xor(ce[m], t1);
            else if (two == 0x101u)
              ce[m] = plane_xor3(ce[m], tt, t1);
          }
          if (b < 14) tt = plane_mulx(t1);
        }
        st.mark(3);
        if constexpr (kMC == S::kM) __syncthreads();  // every wave is done reading the zeroed erased planes
        st.mark(4);
#pragma unroll
        for (int m = 0; m < kMC; ++m) {
          __attribute__((address_space(3))) uint64_t *dst =
              (__attribute__((address_space(3))) uint64_t *)(L.base + L.lo + 4096u * a.erased[m0 + m]);
#pragma unroll
          for (int h = 0; h < 8; ++h)
            __hip_atomic_fetch_xor(dst + 128 * (h >> 1) + (h & 1),
                                   (uint64_t)ce[m].p[2 * h] | ((uint64_t)ce[m].p[2 * h + 1] << 32), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_WORKGROUP);
        }
      }
    }
    st.mark(5);
    __syncthreads();
    st.mark(6);
#else
    // ---- 2. syndrome bit-rows of this wave, parked in the erased slots
    {
      uint32_t syn[S::kSynRows];
#if VDS_DIAG_RES == 3
      for (int r = 0; r < S::kSynRows; ++r) syn[r] = lane + r;
#else
      P::syndrome(kSynSameCode ? 1 : wave, L, syn);
#endif
      prefetch(tile + t_step);
      __syncthreads();  // every wave is done reading the zeroed erased planes
#pragma unroll
      for (int r = 0; r < S::kSynRows; r += 4) {
        const int q = S::kSynRows * wave + r;  // syndrome q / 16, planes q % 16 ..
        L.put(4 * a.erased[q >> 4] + ((q & 15) >> 2), u32x4{syn[r], syn[r + 1], syn[r + 2], syn[r + 3]});
      }
    }
    __syncthreads();
    // ---- 3. c_e = sum_j R[w][j] S_j for e = erased[w], w < M: Horner over the
    // 16 coefficient bits (ce = ce * x, then add the S_j whose coefficient has
    // that bit); the selections are wave-uniform bytes, the adds plain XORs
    if (wave < S::kM) {
      Plane16 sy[S::kM];
#pragma unroll
      for (int j = 0; j < S::kM; ++j) syn_get_point(L, a.erased[j], sy[j].p);
      Plane16 ce = plane_zero();
#pragma unroll
      for (int b = 15; b >= 0; --b) {
        if (b != 15) ce = plane_mulx(ce);
        const uint32_t sel = (a.solve_sel[wave][b >> 2] >> (8 * (b & 3))) & 0xFFu;
#pragma unroll
        for (int j = 0; j < S::kM; j += 2) {
          const uint32_t two = (sel >> j) & 3u;
          if (two == 1u)
            ce = plane_xor(ce, sy[j]);
          else if (two == 2u)
            ce = plane_xor(ce, sy[j + 1]);
          else if (two == 3u)
            ce = plane_xor3(ce, sy[j], sy[j + 1]);
        }
      }
      __syncthreads();  // every recovering wave has read all syndromes
      syn_put_point(L, my_erased, ce.p);
    } else {
      __syncthreads();
    }
    __syncthreads();
#endif
    if constexpr (REGEN) {
      // ---- 4'. regenerate: the recovered point e_w IS replica e_w's cells
      // (P(e_w) stripe by stripe).  Undo the stage-1 transpose and store it as
      // big-endian cells, one 1 KiB store per wave-instruction; no
      // interpolation (fused "decode + re-encode" of sync_process.cpp:313-335).
      if (wave < S::kM && a.regen[wave] != nullptr) {
        uint32_t Pl[16], W[16];
        syn_get_point(L, my_erased, Pl);
#pragma unroll
        for (int b = 0; b < 16; ++b) W[b ^ 8] = Pl[b];
        transpose16x2(W, bm);  // self-inverse: back to the loaded word layout
        uint8_t *dst = a.regen[wave] + (uint64_t)o * a.regen_stride + 2 * stripe0 + 16 * lane;
#pragma unroll
        for (int q = 0; q < 4; ++q)
          g_st<8>(dst + 1024 * q, u32x4{W[4 * q], W[4 * q + 1], W[4 * q + 2], W[4 * q + 3]});
      }
      __syncthreads();  // every wave is done with this tile's planes
      continue;
    }
    // ---- 4. fixed interpolation from points 0..K-1, then big-endian stores
    {
      uint32_t cells[16 * S::kCells];
#if VDS_DIAG_RES == 1
      for (int r = 0; r < 16 * S::kCells; ++r) cells[r] = lane * r;
#elif VDS_SYN_GM
      syn_interp_gm<K, N, WV, 0>(wave, L, cells, st);
      if (kLateLoad && !kStageLoad) prefetch(tile + t_step);
#else
      P::interp(kSynSameCode ? 1 : wave, L, cells);
#endif
      uint8_t *dst = a.out + (uint64_t)o * a.out_stride;
      constexpr int kGroups = S::kCells / 2;  // word groups (2 cells) per wave
      if constexpr (K == 16) {
        // Stage the tile's output in LDS (the planes are dead once every wave
        // has interpolated), stripe-major with 16 bytes of padding after every
        // 16 stripes: the writes of one instruction then hit distinct banks,
        // and the copy-out is 16 contiguous bytes per lane, so every HBM
        // write is a whole 1 KiB wave-instruction (no partial lines).  One
        // word group at a time keeps 32, not 64, transposed rows live.
        static_assert(2048 * 32 + 128 * 16 <= S::kLdsBytes, "staging layout is for 32-byte stripes");
        __syncthreads();
        st.mark(14);
#pragma unroll
        for (int g = 0; g < kGroups; ++g) {
          uint32_t rows[32];
#pragma unroll
          for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int jb = 0; jb < 16; ++jb) rows[16 * h + jb] = cells[16 * (2 * g + h) + (jb ^ 8)];
          transpose32(rows, bm);
          // slot 8q+e is stripe st = 8 lane + 512 q + e at byte st*32 + (st/16)*16,
          // i.e. a per-lane base plus a compile-time offset
          lds_char *w0 = L.base + 256u * lane + 16u * (lane >> 1) + 4u * (kGroups * wave + g);
#pragma unroll
          for (int slot = 0; slot < 32; ++slot) {
            const int pi = (slot & 1) ? 16 + (slot >> 1) : (slot >> 1);
            *(__attribute__((address_space(3))) uint32_t *)(w0 + (slot >> 3) * (16384 + 512) + (slot & 7) * 32) =
                rows[pi];
          }
        }
        st.mark(15);
        __syncthreads();
        st.mark(16);
        // 16-byte chunk c = 64 (kChunks wave + i) + lane of the tile: stripe c/2, half c%2
        constexpr int kChunks = 64 / WV;  // 1 KiB pieces of the tile each wave writes
        if constexpr (VDS_SYN_PRIO > 0) __builtin_amdgcn_s_setprio(VDS_SYN_PRIO);
        const lds_char *r0 =
            L.base + 1056u * kChunks * wave + 32u * (lane >> 1) + 16u * (lane >> 5) + 16u * (lane & 1);
        uint8_t *g0 = dst + stripe0 * (2 * K) + 1024u * kChunks * wave + 16u * lane;
#pragma unroll
        for (int i = 0; i < kChunks; ++i) {
          const u32x4 v = *(lds_v4 *)(r0 + 1056 * i);
#if VDS_DIAG_RES == 2
          if (a.out_stride == 1)
#endif
          g_st<8>(g0 + 1024 * i, v);
        }
        if constexpr (VDS_SYN_PRIO > 0) __builtin_amdgcn_s_setprio(0);
        st.mark(17);
      } else if constexpr (K == 32) {
        // Stage as for k = 16 with 64-byte stripes and 8 bytes of padding
        // after every 8 stripes: stripe st, word w at st*64 + (st/8)*8 + 4w;
        // the copy-out reads 16 bytes per lane as two 8-byte-aligned halves.
        static_assert(S::kCells == 4 && 2048 * 64 + 256 * 8 <= S::kLdsBytes, "staging layout is for 64-byte stripes");
        __syncthreads();
        st.mark(14);
#pragma unroll
        for (int g = 0; g < 2; ++g) {
          uint32_t rows[32];
#pragma unroll
          for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int jb = 0; jb < 16; ++jb) rows[16 * h + jb] = cells[16 * (2 * g + h) + (jb ^ 8)];
          transpose32(rows, bm);
          // slot 8q+e is stripe st = 8 lane + 512 q + e: byte 512 lane + 8 lane
          // + q (32768 + 512) + 64 e + 4 (2 wave + g); lanes l and l + 16 of a
          // 32-lane group share a bank (one word group at a time keeps 32,
          // not 64, transposed rows live)
          lds_char *w0 = L.base + 520u * lane + 4u * (2 * wave + g);
#pragma unroll
          for (int slot = 0; slot < 32; ++slot) {
            const int pi = (slot & 1) ? 16 + (slot >> 1) : (slot >> 1);
            *(__attribute__((address_space(3))) uint32_t *)(w0 + (slot >> 3) * (32768 + 512) + (slot & 7) * 64) =
                rows[pi];
          }
          if (kStageLoad && g == 0) prefetch(tile + t_step);
        }
        st.mark(15);
        __syncthreads();
        st.mark(16);
        // 16-byte chunk c = 64 (16 wave + i) + lane of the tile: stripe c/4,
        // quarter c%4, at 64 (c/4) + 8 (c/32) + 16 (c%4) = r0 + 1040 i (one
        // per-lane base, compile-time offsets: no hoisted address per i)
        uint8_t *g0 = dst + stripe0 * (2 * K) + 16384u * wave + 16u * lane;
        const lds_char *r0 = L.base + 16640u * wave + 64u * (lane >> 2) + 8u * (lane >> 5) + 16u * (lane & 3);
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const lds_char *r = r0 + 1040 * i;
          const u32x2 v0 = *(__attribute__((address_space(3))) const u32x2 *)r;
          const u32x2 v1 = *(__attribute__((address_space(3))) const u32x2 *)(r + 8);
#if VDS_DIAG_RES == 2
          if (a.out_stride == 1)
#endif
          g_st<8>(g0 + 1024 * i, u32x4{v0[0], v0[1], v1[0], v1[1]});
        }
        st.mark(17);
      } else {
        uint32_t rows[1][32];
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int jb = 0; jb < 16; ++jb) rows[0][16 * h + jb] = cells[16 * h + (jb ^ 8)];
        transpose32(rows[0], bm);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          uint8_t *base = dst + (stripe0 + 8u * lane + 512u * q) * (2 * K) + 4 * wave;
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const int slot = 8 * q + e;
            const int pi = (slot & 1) ? 16 + (slot >> 1) : (slot >> 1);
            *reinterpret_cast<uint32_t *>(base + e * (2 * K)) = rows[0][pi];
          }
        }
      }
    }
    __syncthreads();
    st.mark(18);
  }
  st.flush(blockIdx.x * WV + wave, lane);
}

#if VDS_DIAG_STAMPS
extern "C" int vds_ec_diag_stamps(unsigned long long *host, size_t n) {
  if (n > (size_t)kStampSlots) n = kStampSlots;
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_syn_stamps), n * sizeof(unsigned long long));
}
#endif

// ========================================================= generic regenerate

template <int CB>
__global__ void k_regen_generic(RegenArgs a) {
  const uint64_t per = a.t_count + 1;  // cells + the trailer
  const uint64_t total = per * a.nt * (uint64_t)a.count;
  for (uint64_t idx = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; idx < total;
       idx += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t ti = idx % per;
    const uint64_t rest = idx / per;
    const uint32_t i = (uint32_t)(rest % a.nt);
    const uint32_t o = (uint32_t)(rest / a.nt);
    uint8_t *out = a.outs[i] + (uint64_t)o * a.out_stride;
    auto chunk = [&](uint32_t j) {
      return (a.chunk_table ? a.chunk_table[j] : a.chunk_ptr[j]) + (uint64_t)o * a.chunk_stride;
    };
    if (ti == a.t_count) {  // trailer BE16(size % (k*cell)), identical in every replica (chunk.h:273-275)
      const uint8_t *c0 = chunk(0);
      out[a.T * CB] = c0[a.T * CB];
      out[a.T * CB + 1] = c0[a.T * CB + 1];
      continue;
    }
    const uint64_t t = a.t_begin + ti;
    uint32_t acc = 0;
    for (uint32_t j = 0; j < a.k; ++j) {
      const uint64_t e = (uint64_t)i * a.k + j;
      const uint32_t coef = a.coef_dev ? a.coef_dev[e] : (a.coef_inline[e >> 1] >> (16 * (e & 1))) & 0xFFFFu;
      const uint8_t *c = chunk(j) + t * CB;
      const uint32_t cell = CB == 2 ? (uint32_t)((c[0] << 8) | c[1]) : (uint32_t)c[0];
      acc ^= gf_mul_cell<CB>(coef, cell);
    }
    if constexpr (CB == 2) {
      out[2 * t] = (uint8_t)(acc >> 8);  // binary_serialize.cpp:18-22
      out[2 * t + 1] = (uint8_t)(acc & 0xFF);
    } else {
      out[t] = (uint8_t)acc;
    }
  }
}

// ============================================================== synthetic data

__global__ void k_fill_splitmix(uint8_t *dst, uint64_t size, uint64_t seed) {
  const uint64_t words = (size + 7) / 8;
  for (uint64_t w = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; w < words;
       w += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t z = seed + (w + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    if (8 * w + 8 <= size) {
      *reinterpret_cast<uint64_t *>(dst + 8 * w) = z;
    } else {
      for (uint64_t b = 0; 8 * w + b < size; ++b) dst[8 * w + b] = (uint8_t)(z >> (8 * b));
    }
  }
}

// =================================================================== launchers

static int grid_for(uint64_t work, int block) {
  uint64_t g = (work + block - 1) / block;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  return (int)g;
}

hipError_t launch_encode_generic(const GenericEncodeArgs &a, hipStream_t s) {
  const uint64_t work = (a.t_count + (a.write_trailer ? 1 : 0)) * a.nrep * (uint64_t)a.count;
  if (work == 0) return hipSuccess;
  const int grid = grid_for(work, 256);
  if (a.cell_bytes == 2)
    hipLaunchKernelGGL(k_encode_generic<2>, dim3(grid), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL(k_encode_generic<1>, dim3(grid), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_restore_generic(const GenericRestoreArgs &a, hipStream_t s) {
  const uint64_t work = a.t_count * a.k * (uint64_t)a.count;
  if (work == 0) return hipSuccess;
  const int grid = grid_for(work, 256);
  if (a.cell_bytes == 2)
    hipLaunchKernelGGL(k_restore_generic<2>, dim3(grid), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL(k_restore_generic<1>, dim3(grid), dim3(256), 0, s, a);
  return hipGetLastError();
}

template <int K, int N, int RPW, int WV, bool STREAM>
static hipError_t launch_encode_bs_st(const FastEncodeArgs &a, hipStream_t s) {
  using S = EncodeShape<K, N, RPW, WV>;
  static bool configured = false;
  if (!configured) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(&k_encode_bs<K, N, RPW, WV, STREAM>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, S::kLdsBytes);
    if (e != hipSuccess) return e;
    configured = true;
  }
  const int blocks_per_cu = (160 * 1024) / S::kLdsBytes;
  int grid = 256 * (blocks_per_cu > 0 ? blocks_per_cu : 1);
  if ((uint32_t)grid > a.total_tiles) grid = (int)a.total_tiles;
  if (grid == 0) return hipSuccess;
  hipLaunchKernelGGL((k_encode_bs<K, N, RPW, WV, STREAM>), dim3(grid), dim3(S::kThreads), S::kLdsBytes, s, a);
  return hipGetLastError();
}

template <int K, int N, int RPW, int WV>
static hipError_t launch_encode_bs(const FastEncodeArgs &a, hipStream_t s) {
  if (a.groups_per_obj % 16 == 0) return launch_encode_bs_st<K, N, RPW, WV, false>(a, s);
  if constexpr (K >= 8) return launch_encode_bs_st<K, N, RPW, WV, true>(a, s);
  return hipErrorNotSupported;
}

#ifndef VDS_ENC16_RPW  // replicas per wave / waves of the k=16, n=20 encode
#define VDS_ENC16_RPW 5
#define VDS_ENC16_WAVES 4
#endif

bool has_encode_fast(uint32_t k, uint32_t n) {
  return (k == 16 && n == 20) || (k == 32 && n == 40) || (k == 32 && n == 64) || (k == 4 && n == 6);
}

hipError_t launch_encode_fast(uint32_t k, uint32_t n, const FastEncodeArgs &a, hipStream_t s) {
  if (k == 16 && n == 20) return launch_encode_bs<16, 20, VDS_ENC16_RPW, VDS_ENC16_WAVES>(a, s);
  if (k == 32 && n == 40) return launch_encode_bs<32, 40, 5, 8>(a, s);
  if (k == 32 && n == 64) return launch_encode_bs<32, 64, 8, 8>(a, s);  // the live shape (dht_network.h:22-25)
  if (k == 4 && n == 6) return launch_encode_bs<4, 6, 6, 1>(a, s);
  return hipErrorNotSupported;
}

template <int K, bool STREAM, bool REGEN>
static hipError_t launch_restore_bs_k(const FastRestoreArgs &a, hipStream_t s) {
  using S = RestoreShape<K>;
  static bool configured = false;
  if (!configured) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(&k_restore_bs<K, STREAM, REGEN>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, S::kLdsBytes);
    if (e != hipSuccess) return e;
    configured = true;
  }
  const int blocks_per_cu = (160 * 1024) / S::kLdsBytes;
  int grid = 256 * (blocks_per_cu > 0 ? blocks_per_cu : 1);
  if ((uint32_t)grid > a.total_tiles) grid = (int)a.total_tiles;
  if (grid == 0) return hipSuccess;
  hipLaunchKernelGGL((k_restore_bs<K, STREAM, REGEN>), dim3(grid), dim3(S::kThreads), S::kLdsBytes, s, a);
  return hipGetLastError();
}

bool has_restore_fast(uint32_t k) { return k == 16 || k == 32; }

template <int K>
static hipError_t launch_restore_bs_kk(const FastRestoreArgs &a, hipStream_t s, bool regen) {
  const bool stream = a.groups_per_obj % 4 != 0;
  if (regen) return stream ? launch_restore_bs_k<K, true, true>(a, s) : launch_restore_bs_k<K, false, true>(a, s);
  return stream ? launch_restore_bs_k<K, true, false>(a, s) : launch_restore_bs_k<K, false, false>(a, s);
}

hipError_t launch_restore_fast(uint32_t k, const FastRestoreArgs &a, hipStream_t s, bool regen) {
  if (k == 16) return launch_restore_bs_kk<16>(a, s, regen);
  if (k == 32) return launch_restore_bs_kk<32>(a, s, regen);
  return hipErrorNotSupported;
}


bool has_restore_syn(uint32_t k, uint32_t n) { return (k == 16 && n == 20) || (k == 32 && n == 40); }

constexpr int kSynWaves16 = VDS_SYN_WAVES;

const uint16_t *restore_syn_weights(uint32_t k, uint32_t n) {
  if (k == 16 && n == 20) return &RestorePrograms<16, 20, kSynWaves16>::kSyndromeW[0][0];
  if (k == 32 && n == 40) return &RestorePrograms<32, 40, 8>::kSyndromeW[0][0];
  return nullptr;
}

template <int K, int N, int WV, bool REGEN>
static hipError_t launch_restore_syn_kn(const SynRestoreArgs &a, hipStream_t s) {
  using S = SynShape<K, N, WV>;
  static bool configured = false;
  if (!configured) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(&k_restore_syn<K, N, WV, REGEN>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, S::kLdsBytes);
    if (e != hipSuccess) return e;
    configured = true;
  }
  const int blocks_per_cu = (160 * 1024) / S::kLdsBytes;
  int grid = 256 * (blocks_per_cu > 0 ? blocks_per_cu : 1);
  if ((uint32_t)grid > a.total_tiles) grid = (int)a.total_tiles;
  if (grid == 0) return hipSuccess;
  hipLaunchKernelGGL((k_restore_syn<K, N, WV, REGEN>), dim3(grid), dim3(S::kThreads), S::kLdsBytes, s, a);
  return hipGetLastError();
}

hipError_t launch_restore_syn(uint32_t k, uint32_t n, const SynRestoreArgs &a, hipStream_t s, bool regen) {
  if (k == 16 && n == 20)
    return regen ? launch_restore_syn_kn<16, 20, kSynWaves16, true>(a, s)
                 : launch_restore_syn_kn<16, 20, kSynWaves16, false>(a, s);
  if (k == 32 && n == 40)
    return regen ? launch_restore_syn_kn<32, 40, 8, true>(a, s) : launch_restore_syn_kn<32, 40, 8, false>(a, s);
  return hipErrorNotSupported;
}

hipError_t launch_regen_generic(const RegenArgs &a, hipStream_t s) {
  const uint64_t work = (a.t_count + 1) * a.nt * (uint64_t)a.count;
  if (work == 0) return hipSuccess;
  const int grid = grid_for(work, 256);
  if (a.cell_bytes == 2)
    hipLaunchKernelGGL(k_regen_generic<2>, dim3(grid), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL(k_regen_generic<1>, dim3(grid), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_fill_splitmix(uint8_t *dst, uint64_t size, uint64_t seed, hipStream_t s) {
  if (size == 0) return hipSuccess;
  const int grid = grid_for((size + 7) / 8, 256);
  hipLaunchKernelGGL(k_fill_splitmix, dim3(grid), dim3(256), 0, s, dst, size, seed);
  return hipGetLastError();
}

}  // namespace vds_ec
