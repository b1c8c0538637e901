// ec_encode.hpp -- k_encode_bs<K,N>: bit-sliced encode of replicas 0..N-1
// (chunk_generator<uint16_t>::write, chunk.h:245-281, for every replica of a
// batch of objects in one pass over the input).
//
// A tile is 2048 stripes: lane = set of 32 stripes, one bit per stripe in
// each 32-bit plane.  The workgroup's waves split the input transposes, share
// the bit planes through LDS, and each wave evaluates a compile-time group of
// replicas by Horner with constant multipliers (replica r is the polynomial
// of the stripe's cells evaluated at r).  Tails, trailers and other shapes
// are ec_generic.hip's.  The instantiations are compiled in parallel, one
// translation unit per shape (ec_encode_K_N.hip); ec_encode.hip dispatches.
#pragma once

#include <array>
#include <utility>

#include "ec_device.hpp"

namespace vds_ec {

#ifndef VDS_ENC_PLAN_LS
#define VDS_ENC_PLAN_LS 1  // local search after the LPT pair plan (plan_pairs)
#endif

// Transposes on rotated words (bitslice.hpp transpose_round) except at k =
// 32, whose encode measured 2.8% slower with them (9.45-9.51 -> 9.72-9.78
// ms at 256 x 64 MiB; k = 16 unchanged, profiles/round5/ab_transpose.log).
constexpr bool enc_rot(int K) { return K != 32; }

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

// ---- one-level additive split of the stripe polynomial.  The Taylor
// expansion at z^2 + z (XORs only) gives P(z) = P0(y) + z P1(y), y = z^2 + z,
// deg P0, P1 < K/2; y is the same for z = r and r + 1 (r even: char 2), so
// P(r) = P0(y) + r P1(y) and P(r + 1) = P(r) + P1(y).  A pair of replicas
// costs two K/2-step Horners with the constant y, against two K-step Horners
// with r and r + 1: 64-70% of the row-form XORs for n = 20, 40, 64 (the first
// level of the additive FFT of tools/xorgen/gen_encode_gm.py, without its
// register-hungry deeper levels).
// Horner steps acc * C + x with the constants of the split modes as Paar XOR
// programs (tools/xorgen/gen_horner: shared pairs of acc planes between the
// output rows), where that beats the row form; VDS_ENC_PAAR=0: row form only.
#ifndef VDS_ENC_PAAR
#define VDS_ENC_PAAR 1
#endif
template <uint32_t C>
struct HornerPaar {
  static constexpr int kCost = 0;  // 0: no program, the row form is used
};
#include "generated/horner_paar.inc"

template <uint32_t C>
__device__ __forceinline__ Plane16 plane_horner_enc(const Plane16 &acc, const Plane16 &x) {
  if constexpr (VDS_ENC_PAAR && HornerPaar<C>::kCost > 0)
    return HornerPaar<C>::apply(acc, x);
  else
    return plane_horner_rows<C>(acc, x);
}
constexpr int enc_step_cost(uint32_t c) {
  return (VDS_ENC_PAAR && horner_paar_cost(c) > 0) ? horner_paar_cost(c) : horner_cost((int)c);
}


constexpr uint32_t pair_y(int r) { return gf16_mul((uint32_t)r, (uint32_t)r) ^ (uint32_t)r; }
constexpr int pair_cost(int r) { return 2 * enc_step_cost(pair_y(r)) + 1; }

template <int WAVES, int PPW>
struct PairPlan {
  int r[WAVES][PPW];  // even r of the pair (r, r + 1); -1: empty
};

template <int N, int WAVES, int PPW>
constexpr PairPlan<WAVES, PPW> plan_pairs() {
  PairPlan<WAVES, PPW> p{};
  int load[WAVES] = {};
  int cnt[WAVES] = {};
  bool used[N / 2 + 1] = {};
  int cost[N / 2 + 1] = {};
  // per cell step: the pair's two half-Horner steps, plus its two replica
  // stores (two 16x16 transposes and 16 dword stores each, ~100 VALU) spread
  // over the K / 2 = 2 WAVES steps
  constexpr int kStoreUnits = VDS_ENC_PLAN_LS ? (2 * 100 + WAVES) / (2 * WAVES) : 0;
  for (int q = 0; q < N / 2; ++q) cost[q] = pair_cost(2 * q) + kStoreUnits;  // (once each: constexpr step limit)
  for (int w = 0; w < WAVES; ++w)
    for (int s = 0; s < PPW; ++s) p.r[w][s] = -1;
  for (int it = 0; it < N / 2; ++it) {
    int best = -1;
    for (int q = 0; q < N / 2; ++q)
      if (!used[q] && (best < 0 || cost[q] > cost[best])) best = q;
    used[best] = true;
    int bw = -1;
    for (int w = 0; w < WAVES; ++w)
      if (cnt[w] < PPW && (bw < 0 || load[w] < load[bw])) bw = w;
    p.r[bw][cnt[bw]++] = 2 * best;
    load[bw] += cost[best];
  }
  // Then local search on the largest load (VDS_ENC_PLAN_LS): move one pair of
  // the most loaded wave to a wave with room, or swap it with a pair of
  // another wave, whenever that lowers the larger of the two loads.  LPT left
  // 20 pairs on 8 waves at loads 162..205 (k = 32, n = 40) and 10 on 4 at
  // 130..171 (k = 16): a wave that runs alone once its SIMD partner is done
  // issues at about half the rate, so the tile waits on the heaviest wave.
  if constexpr (VDS_ENC_PLAN_LS) {
    for (int round = 0; round < 64; ++round) {
      int a = 0;
      for (int w = 1; w < WAVES; ++w)
        if (load[w] > load[a]) a = w;
      int gain = 0, bi = -1, bw = -1, bj = -1;  // best: item bi of a -> wave bw (bj = -1) or swap with item bj of bw
      for (int i = 0; i < cnt[a]; ++i) {
        const int ci = cost[p.r[a][i] / 2];
        for (int w = 0; w < WAVES; ++w) {
          if (w == a) continue;
          if (cnt[w] < PPW) {  // move
            const int m = (load[a] - ci > load[w] + ci) ? load[a] - ci : load[w] + ci;
            if (load[a] - m > gain) gain = load[a] - m, bi = i, bw = w, bj = -1;
          }
          for (int j = 0; j < cnt[w]; ++j) {  // swap
            const int cj = cost[p.r[w][j] / 2];
            const int la = load[a] - ci + cj, lw = load[w] - cj + ci;
            const int m = la > lw ? la : lw;
            if (load[a] - m > gain) gain = load[a] - m, bi = i, bw = w, bj = j;
          }
        }
      }
      if (bi < 0) break;
      const int ri = p.r[a][bi], ci = cost[ri / 2];
      if (bj < 0) {
        p.r[a][bi] = p.r[a][--cnt[a]];
        p.r[a][cnt[a]] = -1;
        p.r[bw][cnt[bw]++] = ri;
        load[a] -= ci, load[bw] += ci;
      } else {
        const int rj = p.r[bw][bj], cj = cost[rj / 2];
        p.r[a][bi] = rj, p.r[bw][bj] = ri;
        load[a] += cj - ci, load[bw] += ci - cj;
      }
    }
  }
  return p;
}

// ---- two-level additive split (QUAD).  After the level-1 Taylor step, each
// half P_H (H = 0, 1; degree < K/2) is normalised by 6 = s(x) (Q_H(Z) =
// P_H(6Z): coefficient i times 6^i) and Taylor-expanded at Z^2 + Z again:
// Q_H(Z) = A_H(Z^2+Z) + Z B_H(Z^2+Z), degree < K/4.  For the quad of replicas
// 4j..4j+3, y0 = s(4j) and y1 = s(4j+2) = y0 + 6 share w = z0^2 + z0 with z0
// = y0 / 6 (z1 = z0 + 1), so
//   P_H(y0) = A_H(w) + z0 B_H(w),      P_H(y1) = P_H(y0) + B_H(w),
//   P(4j) = P0(y0) + 4j P1(y0),        P(4j+1) = P(4j) + P1(y0),
//   P(4j+2) = P0(y1) + (4j+2) P1(y1),  P(4j+3) = P(4j+2) + P1(y1):
// four K/4-step Horners with the one constant w per quad, against four
// K/2-step ones for the same four replicas as two level-1 pairs.
constexpr uint32_t kQuadD = 6u;  // s(x) = x^2 + x
constexpr uint32_t quad_z0(int j) { return gf16_mul(pair_y(4 * j), gf16_inv(kQuadD)); }
constexpr uint32_t quad_w(int j) { return gf16_mul(quad_z0(j), quad_z0(j)) ^ quad_z0(j); }
constexpr int quad_cost(int j) { return 4 * enc_step_cost(quad_w(j)) + 4; }

template <int WAVES, int QPW>
struct QuadPlan {
  int j[WAVES][QPW];  // quad index (replicas 4j..4j+3); -1: empty
};

template <int N, int WAVES, int QPW>
constexpr QuadPlan<WAVES, QPW> plan_quads() {
  QuadPlan<WAVES, QPW> p{};
  int load[WAVES] = {};
  int cnt[WAVES] = {};
  bool used[N / 4 + 1] = {};
  int cost[N / 4 + 1] = {};
  for (int q = 0; q < N / 4; ++q) cost[q] = quad_cost(q);
  for (int w = 0; w < WAVES; ++w)
    for (int s = 0; s < QPW; ++s) p.j[w][s] = -1;
  for (int it = 0; it < N / 4; ++it) {
    int best = -1;
    for (int q = 0; q < N / 4; ++q)
      if (!used[q] && (best < 0 || cost[q] > cost[best])) best = q;
    used[best] = true;
    int bw = -1;
    for (int w = 0; w < WAVES; ++w)
      if (cnt[w] < QPW && (bw < 0 || load[w] < load[bw])) bw = w;
    p.j[bw][cnt[bw]++] = best;
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
  static constexpr int kPPW = (N / 2 + kWaves - 1) / kWaves;  // replica pairs per wave (split mode)
  static constexpr PairPlan<kWaves, kPPW> kPairs = plan_pairs<N, kWaves, kPPW>();
  static constexpr int kQPW = (N / 4 + kWaves - 1) / kWaves;  // replica quads per wave (quad mode)
  static constexpr QuadPlan<kWaves, kQPW> kQuads = plan_quads<N, kWaves, kQPW>();
  static_assert(K % 4 == 0 && WV == K / 4, "fast encode: k % 4 == 0 and k/4 waves");
  static_assert(RPW * WV >= N, "every replica needs a wave");
  __device__ __forceinline__ static constexpr int cell_off(int c) { return 16 * c + kGroupPad * (c >> 2); }
};

// Replica r's output pointer, read from the kernel arguments where it is used.
// Left to itself the compiler hoists all N pointers out of the tile loop; at
// N = 40 or 64 they do not fit the SGPRs, spill to scratch, and every scratch
// reload's s_waitcnt vmcnt(0) then waits for all the stores in flight (28-41
// such drains per tile).  The opaque zero keeps the s_load at its use, and
// the pointer comes from the kernarg segment itself (the kernel's only
// explicit argument, at offset 0): indexing the by-value parameter at a
// runtime index makes the compiler copy the whole struct to scratch.
__device__ __forceinline__ uint8_t *rep_ptr(const FastEncodeArgs &, int r) {
  int z;
  asm volatile("s_mov_b32 %0, 0" : "=s"(z));
  const auto *k = (const __attribute__((address_space(4))) FastEncodeArgs *)__builtin_amdgcn_kernarg_segment_ptr();
  return k->outs[r + z];
}

// Transpose one replica's planes back to big-endian cells and store them.
// After the transpose, word q of lane l holds the cells of stripes l + 64 q
// (low half) and l + 1024 + 64 q (high half); each half goes out as a 2-byte
// store (global_store_short / _d16_hi), so one wave-instruction writes 128
// contiguous bytes and no cross-lane shuffle is needed.
template <bool ROT>
__device__ __forceinline__ void store_replica(const Plane16 &acc, uint8_t *base, const BitMasks &bm) {
  uint32_t rows[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) rows[j] = acc.p[j ^ 8];  // word bit j <-> cell bit j^8 (BE)
  transpose16x2<ROT>(rows, bm);
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    *reinterpret_cast<uint16_t *>(base + 128 * q) = (uint16_t)rows[q];
    *reinterpret_cast<uint16_t *>(base + 2048 + 128 * q) = (uint16_t)(rows[q] >> 16);
  }
}

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
template <bool STREAM, bool ROT>
__device__ __forceinline__ void store_replica_groups(const Plane16 &acc, uint8_t *rep, const FastEncodeArgs &a,
                                                     TilePos tp, int lane, const BitMasks &bm) {
  uint32_t rows[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) rows[j] = acc.p[j ^ 8];  // word bit j <-> cell bit j^8 (BE)
  transpose16x2<ROT>(rows, bm);
  // (replica strides L = 2T + 2 leave odd objects 2-byte aligned: gfx950
  // global stores need no natural alignment, tested by the strided batches)
  // The trailer (trailer0): when group j is its object's last, lane 0 also
  // writes the object's zero BE16 trailer right after it (cell T = 128
  // groups_per_obj), instead of a generic launch over every replica of every
  // object (live shape: 1M two-byte stores, 32 us a launch).
  if constexpr (!STREAM) {  // whole tiles per object: one base, immediate offsets
    uint32_t *b = reinterpret_cast<uint32_t *>(rep + (uint64_t)tp.o * a.out_stride + 256u * tp.q + 4 * lane);
#pragma unroll
    for (int j = 0; j < 16; ++j) g_st<1>(b + 64 * j, rows[j]);
    if (a.trailer0 && tp.q + 16 == a.groups_per_obj && lane == 0)
      *(gmem<uint16_t> *)(rep + (uint64_t)tp.o * a.out_stride + 256u * a.groups_per_obj) = (uint16_t)0;
  } else {
    uint32_t o = tp.o, q = tp.q;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      g_st<1>(rep + (uint64_t)o * a.out_stride + 256u * q + 4 * lane, rows[j]);
      if (++q == a.groups_per_obj) {
        if (a.trailer0 && lane == 0) *(gmem<uint16_t> *)(rep + (uint64_t)o * a.out_stride + 256u * q) = (uint16_t)0;
        q = 0;
        ++o;
      }
    }
  }
}

template <int MAP, bool STREAM, bool ROT>
__device__ __forceinline__ void store_rep(const Plane16 &acc, uint8_t *rep, const FastEncodeArgs &a, TilePos tp,
                                          int lane, const BitMasks &bm) {
  if constexpr (MAP == 0)  // k = 4: whole tiles of one object
    store_replica<ROT>(acc, rep + (uint64_t)tp.o * a.out_stride + 256u * tp.q + 2 * lane, bm);
  else
    store_replica_groups<STREAM, ROT>(acc, rep, a, tp, lane, bm);
}

// Wave priority while a pass issues its stores (same-box A/B, 512 objects:
// encode 1881-1895 -> 1917-1918 GiB/s), so one wave's store stream is not
// starved by the other workgroup's Horner.
constexpr int kEncStorePrio = 2;
// (k = 32, one workgroup per CU: the second-dispatched half of the waves at
// priority 1 for the whole kernel -- as the k = 32 restore does -- measured
// slower, C4 encode 9.48-9.53 -> 10.38-10.46 ms at 256 x 64 MiB, round 5.)


// Replicas evaluated per pass over the tile's cells.  A/B at k = 16 with the
// non-temporal, prioritised stores (512 objects, 2 rounds): 1 -> 1740, 2 ->
// 1825, 3 -> 1867, 5 -> 1914 GiB/s; k = 32, n = 40 (256 objects): 2 -> 1266,
// 3 -> 1335, 4 -> 1311, 5 -> 1396 (no spills at 256 VGPRs); n = 64 and the
// stream instantiation of n = 40 spill at 5 and keep 3.
template <int K, int N, bool ST>
constexpr int enc_pass() {
  return K == 16 ? 5 : (K == 32 && N == 40 && !ST) ? 5 : 3;
}

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
        store_rep<S::kMap, ST, enc_rot(K)>(lds_planes(set_planes + S::cell_off(0)), rep_ptr(a, 0), a, tp, lane, bm);
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
  for (int c = K - 2; c >= 1; c -= 2) {
    const Plane16 xb = lds_planes(set_planes + S::cell_off(c - 1));
    rows_step<K, N, RPW, WV, W, S0, PR>(B, A, xa);
    xa = lds_planes(set_planes + S::cell_off(c - 2));
    rows_step<K, N, RPW, WV, W, S0, PR>(A, B, xb);
  }
  rows_step<K, N, RPW, WV, W, S0, PR>(A, A, xa);  // cell 0 (each step returns a fresh value)
  __builtin_amdgcn_s_setprio(kEncStorePrio);
#pragma unroll
  for (int s = 0; s < PR; ++s) {
    const int r = S0 + s < RPW ? S::kPlan.rep[W][S0 + s] : -1;
    if (r == 0) store_rep<S::kMap, ST, enc_rot(K)>(xa, rep_ptr(a, 0), a, tp, lane, bm);
    if (r > 0) store_rep<S::kMap, ST, enc_rot(K)>(A[s], rep_ptr(a, r), a, tp, lane, bm);
  }
  __builtin_amdgcn_s_setprio(0);
}

template <int K, int N, int RPW, int WV, int W, bool ST, int S0 = 0>
__device__ __forceinline__ void encode_wave_group(const uint32_t *set_planes, const FastEncodeArgs &a, TilePos tp,
                                                  int lane, const BitMasks &bm) {
  constexpr int kPass = enc_pass<K, N, ST>();
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
  } else {
    // wave < kWaves: no path through the dispatch skips the stores (a
    // store-free path would make the vmcnt waits at the top of the tile loop
    // conservative, see the entry of k_encode_bs)
    __builtin_unreachable();
  }
}

// The stores encode_dispatch issues for one tile, with zero planes: see the
// entry of k_encode_bs for why.
template <int K, int N, int RPW, int WV, bool ST, int W>
__device__ __forceinline__ void encode_zero_dispatch(int wave, const FastEncodeArgs &a, TilePos tp, int lane,
                                                     const BitMasks &bm) {
  using S = EncodeShape<K, N, RPW, WV>;
  if constexpr (W < S::kWaves) {
    if (wave == W) {
#pragma unroll
      for (int s = 0; s < RPW; ++s)
        if (S::kPlan.rep[W][s] >= 0)
          store_rep<S::kMap, ST, enc_rot(K)>(plane_zero(), rep_ptr(a, S::kPlan.rep[W][s]), a, tp, lane, bm);
    } else {
      encode_zero_dispatch<K, N, RPW, WV, ST, W + 1>(wave, a, tp, lane, bm);
    }
  } else {
    __builtin_unreachable();
  }
}

// ---- split mode

// In-place Taylor expansion at z^2 + z of c[OFF .. OFF + NN) (NN a power of
// two): blocks C0..C3 of NN/4: C2 ^= C3, C1 ^= C2, then each half.  Cell 2i
// ends as the coefficient i of P0, cell 2i + 1 as that of P1.
template <int K, int OFF, int NN, class T>
__device__ __forceinline__ void taylor_inplace(T (&c)[K]) {
  if constexpr (NN > 2) {
    constexpr int t = NN / 4;
#pragma unroll
    for (int i = 0; i < t; ++i) c[OFF + 2 * t + i] ^= c[OFF + 3 * t + i];
#pragma unroll
    for (int i = 0; i < t; ++i) c[OFF + t + i] ^= c[OFF + 2 * t + i];
    taylor_inplace<K, OFF, 2 * t>(c);
    taylor_inplace<K, OFF + 2 * t, 2 * t>(c);
  }
}

// The tile's sets in LDS -> their Taylor coefficients, in place; plane-
// parallel (the XORs never mix planes): wave w < 4 takes planes 4w..4w+3 of
// every cell (one ds_read_b128 / ds_write_b128 per cell, conflict-free as
// the Horner reads).
#ifndef VDS_DIAG_ENC
#define VDS_DIAG_ENC 0
#endif
template <int K, int N, int RPW, int WV>
__device__ __forceinline__ void taylor_lds(int wave, uint32_t *set_planes) {
  using S = EncodeShape<K, N, RPW, WV>;
  if (wave < 4) {
    u32x4 c[K];
#pragma unroll
    for (int i = 0; i < K; ++i) c[i] = *(lds_u32x4 *)(set_planes + S::cell_off(i) + 4 * wave);
    taylor_inplace<K, 0, K>(c);
#pragma unroll
    for (int i = 0; i < K; ++i) *(lds_v4 *)(set_planes + S::cell_off(i) + 4 * wave) = c[i];
  }
}

// dst[p] = src[p] * y_p + x for the pairs S0 .. S0+PP-1 of wave W
template <int K, int N, int RPW, int WV, int W, int S0, int PP>
__device__ __forceinline__ void pair_step(Plane16 (&dst)[PP], const Plane16 (&src)[PP], const Plane16 &x) {
  using S = EncodeShape<K, N, RPW, WV>;
  [&]<size_t... I>(std::index_sequence<I...>) {
    constexpr auto r = [](int i) { return S0 + i < S::kPPW ? S::kPairs.r[W][S0 + i] : -1; };
    ((r(I) >= 0 ? (void)(dst[I] = plane_horner_enc<(r(I) >= 0 ? pair_y(r(I)) : 0u)>(src[I], x)) : (void)0), ...);
  }(std::make_index_sequence<PP>{});
}

// Horner of P_H (H = 0: even cells, 1: odd cells) for the pairs S0.. of wave
// W, two steps per iteration (A / B ping-pong, as encode_pass).
template <int K, int N, int RPW, int WV, int W, int S0, int PP, int H>
__device__ __forceinline__ void pair_half(const uint32_t *set_planes, Plane16 (&A)[PP]) {
  using S = EncodeShape<K, N, RPW, WV>;
  constexpr int HK = K / 2;
  auto X = [&](int c) { return lds_planes(set_planes + S::cell_off(2 * c + H)); };
  Plane16 B[PP];
  {
    const Plane16 x = X(HK - 1);
#pragma unroll
    for (int p = 0; p < PP; ++p) A[p] = x;
  }
  Plane16 xa = X(HK - 2);
#pragma clang loop unroll(disable)
  for (int c = HK - 2; c >= 1; c -= 2) {
    const Plane16 xb = X(c - 1);
    pair_step<K, N, RPW, WV, W, S0, PP>(B, A, xa);
    xa = X(c - 2);
    pair_step<K, N, RPW, WV, W, S0, PP>(A, B, xb);
  }
  pair_step<K, N, RPW, WV, W, S0, PP>(A, A, xa);
}

template <int K, int N, bool ST>
constexpr int pair_pass() {
  return (K == 32 && N == 64) ? 2 : 3;
}

template <int K, int N, int RPW, int WV, int W, bool ST, int S0 = 0>
__device__ __forceinline__ void encode_pair_group(const uint32_t *set_planes, const FastEncodeArgs &a, TilePos tp,
                                                  int lane, const BitMasks &bm) {
  using S = EncodeShape<K, N, RPW, WV>;
  constexpr int kP = pair_pass<K, N, ST>();
  constexpr int PP = kP < S::kPPW ? kP : S::kPPW;
  if constexpr (S0 < S::kPPW) {
    Plane16 R0[PP], R1[PP];
    pair_half<K, N, RPW, WV, W, S0, PP, 0>(set_planes, R0);
    pair_half<K, N, RPW, WV, W, S0, PP, 1>(set_planes, R1);
    __builtin_amdgcn_s_setprio(kEncStorePrio);
    [&]<size_t... I>(std::index_sequence<I...>) {
      constexpr auto r = [](int i) { return S0 + i < S::kPPW ? S::kPairs.r[W][S0 + i] : -1; };
      auto one = [&](auto ic) {
        constexpr int i = decltype(ic)::value;
        if constexpr (r(i) >= 0) {
          // P(r) = P0(y) + r P1(y) as one Horner step (its Paar program where
          // one beats the row form).  Against a multiply and an XOR, same box
          // (round 4, tools/runs/gpu_ab_trailer.sh): k = 16 encode 13.47 -> 13.31
          // ms (512 x 64 MiB), k = 32 / n = 40 9.50-9.53 ms either way.
          const Plane16 o0 = plane_horner_enc<(uint32_t)(r(i) >= 0 ? r(i) : 0)>(R1[i], R0[i]);  // R1 r + R0
          store_rep<S::kMap, ST, enc_rot(K)>(o0, rep_ptr(a, r(i)), a, tp, lane, bm);
          store_rep<S::kMap, ST, enc_rot(K)>(plane_xor(o0, R1[i]), rep_ptr(a, r(i) + 1), a, tp, lane, bm);
        }
      };
      (one(std::integral_constant<int, (int)I>{}), ...);
    }(std::make_index_sequence<PP>{});
    __builtin_amdgcn_s_setprio(0);
    encode_pair_group<K, N, RPW, WV, W, ST, S0 + PP>(set_planes, a, tp, lane, bm);
  }
}

template <int K, int N, int RPW, int WV, bool ST, int W>
__device__ __forceinline__ void pair_dispatch(int wave, const uint32_t *set_planes, const FastEncodeArgs &a, TilePos tp,
                                              int lane, const BitMasks &bm) {
  if constexpr (W < WV) {
    if (wave == W)
      encode_pair_group<K, N, RPW, WV, W, ST>(set_planes, a, tp, lane, bm);
    else
      pair_dispatch<K, N, RPW, WV, ST, W + 1>(wave, set_planes, a, tp, lane, bm);
  } else {
    __builtin_unreachable();
  }
}

template <int K, int N, int RPW, int WV, bool ST, int W>
__device__ __forceinline__ void pair_zero_dispatch(int wave, const FastEncodeArgs &a, TilePos tp, int lane,
                                                   const BitMasks &bm) {
  using S = EncodeShape<K, N, RPW, WV>;
  if constexpr (W < WV) {
    if (wave == W) {
#pragma unroll
      for (int s = 0; s < S::kPPW; ++s)
        if (S::kPairs.r[W][s] >= 0) {
          store_rep<S::kMap, ST, enc_rot(K)>(plane_zero(), rep_ptr(a, S::kPairs.r[W][s]), a, tp, lane, bm);
          store_rep<S::kMap, ST, enc_rot(K)>(plane_zero(), rep_ptr(a, S::kPairs.r[W][s] + 1), a, tp, lane, bm);
        }
    } else {
      pair_zero_dispatch<K, N, RPW, WV, ST, W + 1>(wave, a, tp, lane, bm);
    }
  } else {
    __builtin_unreachable();
  }
}

// ---- quad mode

// Level 2 in LDS, step 1 (cell-parallel: every cm mixes all 16 planes): cell
// 2i + H *= 6^i for i = 1..K/2-1, cells dealt round-robin over the waves.
template <int K, int N, int RPW, int WV, int C = 2>
__device__ __forceinline__ void quad_twist_lds(int wave, uint32_t *set_planes) {
  using S = EncodeShape<K, N, RPW, WV>;
  if constexpr (C < K) {
    if (wave == C % WV) {
      constexpr uint32_t tw = gf16_pow(kQuadD, (uint32_t)(C / 2));
      uint32_t *p = set_planes + S::cell_off(C);
      const Plane16 v = plane_horner_enc<tw>(lds_planes(p), plane_zero());
#pragma unroll
      for (int m = 0; m < 4; ++m)
        *(lds_v4 *)(p + 4 * m) = u32x4{v.p[4 * m], v.p[4 * m + 1], v.p[4 * m + 2], v.p[4 * m + 3]};
    }
    quad_twist_lds<K, N, RPW, WV, C + 1>(wave, set_planes);
  }
}

// Level 2 in LDS, step 2 (plane-parallel, XORs only): each half's twisted
// coefficients (cells 2i + H) Taylor-expanded at Z^2 + Z in place: A_H,u at
// cell 4u + H, B_H,u at cell 4u + 2 + H.
template <int K, int N, int RPW, int WV>
__device__ __forceinline__ void quad_taylor_lds(int wave, uint32_t *set_planes) {
  using S = EncodeShape<K, N, RPW, WV>;
  if (wave < 4) {
#pragma unroll
    for (int H = 0; H < 2; ++H) {
      u32x4 c[K / 2];
#pragma unroll
      for (int i = 0; i < K / 2; ++i) c[i] = *(lds_u32x4 *)(set_planes + S::cell_off(2 * i + H) + 4 * wave);
      taylor_inplace<K / 2, 0, K / 2>(c);
#pragma unroll
      for (int i = 0; i < K / 2; ++i) *(lds_v4 *)(set_planes + S::cell_off(2 * i + H) + 4 * wave) = c[i];
    }
  }
}

// acc = sum_u coef(cell 4u + OFF) w^u by Horner, two steps per iteration.
// (The two chains A_H, B_H interleaved in one loop spill 18-32 VGPRs at k = 32
// beside the prefetched tile.)
template <int K, int N, int RPW, int WV, uint32_t W, int OFF>
__device__ __forceinline__ Plane16 quad_horner(const uint32_t *set_planes) {
  using S = EncodeShape<K, N, RPW, WV>;
  constexpr int Q = K / 4;
  auto X = [&](int u) { return lds_planes(set_planes + S::cell_off(4 * u + OFF)); };
  Plane16 A = X(Q - 1), B;
  Plane16 xa = X(Q - 2);
#pragma clang loop unroll(disable)
  for (int u = Q - 2; u >= 1; u -= 2) {
    const Plane16 xb = X(u - 1);
    B = plane_horner_enc<W>(A, xa);
    xa = X(u - 2);
    A = plane_horner_enc<W>(B, xb);
  }
  return plane_horner_enc<W>(A, xa);
}

template <int K, int N, int RPW, int WV, int W, bool ST, int S0 = 0>
__device__ __forceinline__ void encode_quad_group(const uint32_t *set_planes, const FastEncodeArgs &a, TilePos tp,
                                                  int lane, const BitMasks &bm) {
  using S = EncodeShape<K, N, RPW, WV>;
  if constexpr (S0 < S::kQPW) {
    constexpr int j = S::kQuads.j[W][S0];
    if constexpr (j >= 0) {
      constexpr uint32_t w = quad_w(j), z0 = quad_z0(j);
      // P_H(y0), P_H(y1) for H = 0, 1 (H = 1 first: its values are scaled below)
      Plane16 p1y0, p1y1;
      {
        const Plane16 A1 = quad_horner<K, N, RPW, WV, w, 1>(set_planes);
        const Plane16 B1 = quad_horner<K, N, RPW, WV, w, 3>(set_planes);
        p1y0 = plane_horner_enc<z0>(B1, A1);
        p1y1 = plane_xor(p1y0, B1);
      }
      const Plane16 A0 = quad_horner<K, N, RPW, WV, w, 0>(set_planes);
      const Plane16 B0 = quad_horner<K, N, RPW, WV, w, 2>(set_planes);
      const Plane16 p0y0 = plane_horner_enc<z0>(B0, A0);
      const Plane16 p0y1 = plane_xor(p0y0, B0);
      __builtin_amdgcn_s_setprio(kEncStorePrio);
      const Plane16 r0 = plane_horner_enc<(uint32_t)(4 * j)>(p1y0, p0y0);
      store_rep<S::kMap, ST, enc_rot(K)>(r0, rep_ptr(a, 4 * j), a, tp, lane, bm);
      store_rep<S::kMap, ST, enc_rot(K)>(plane_xor(r0, p1y0), rep_ptr(a, 4 * j + 1), a, tp, lane, bm);
      const Plane16 r2 = plane_horner_enc<(uint32_t)(4 * j + 2)>(p1y1, p0y1);
      store_rep<S::kMap, ST, enc_rot(K)>(r2, rep_ptr(a, 4 * j + 2), a, tp, lane, bm);
      store_rep<S::kMap, ST, enc_rot(K)>(plane_xor(r2, p1y1), rep_ptr(a, 4 * j + 3), a, tp, lane, bm);
      __builtin_amdgcn_s_setprio(0);
    }
    encode_quad_group<K, N, RPW, WV, W, ST, S0 + 1>(set_planes, a, tp, lane, bm);
  }
}

template <int K, int N, int RPW, int WV, bool ST, int W>
__device__ __forceinline__ void quad_dispatch(int wave, const uint32_t *set_planes, const FastEncodeArgs &a, TilePos tp,
                                              int lane, const BitMasks &bm) {
  if constexpr (W < WV) {
    if (wave == W)
      encode_quad_group<K, N, RPW, WV, W, ST>(set_planes, a, tp, lane, bm);
    else
      quad_dispatch<K, N, RPW, WV, ST, W + 1>(wave, set_planes, a, tp, lane, bm);
  } else {
    __builtin_unreachable();
  }
}

template <int K, int N, int RPW, int WV, bool ST, int W>
__device__ __forceinline__ void quad_zero_dispatch(int wave, const FastEncodeArgs &a, TilePos tp, int lane,
                                                   const BitMasks &bm) {
  using S = EncodeShape<K, N, RPW, WV>;
  if constexpr (W < WV) {
    if (wave == W) {
#pragma unroll
      for (int s = 0; s < S::kQPW; ++s)
        if (S::kQuads.j[W][s] >= 0)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            store_rep<S::kMap, ST, enc_rot(K)>(plane_zero(), rep_ptr(a, 4 * S::kQuads.j[W][s] + r), a, tp, lane, bm);
    } else {
      quad_zero_dispatch<K, N, RPW, WV, ST, W + 1>(wave, a, tp, lane, bm);
    }
  } else {
    __builtin_unreachable();
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
// non-stream instantiation keeps one base address per tile.  SPLIT: replica
// pairs from the one-level split (Taylor coefficients in LDS); QUAD (with
// SPLIT): replica quads from the two-level split.
template <int K, int N, int RPW, int WV, bool STREAM, bool SPLIT, bool QUAD = false>
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
  uint32_t *my_set = lds + lane * S::kSetWords;
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
  // tiles strided over each XCD's workgroups (tile_range; one contiguous
  // range per workgroup measured slower: encode 1923 -> 1814 GiB/s)
  const TileRange tr = tile_range(a.total_tiles);
  uint32_t tile = tr.first;
  const uint32_t t_end = tr.end, t_step = tr.step;
  if (tile < t_end) {
    load(tile);
    // vmcnt counts loads and stores together and retires them in issue order.
    // In the loop a tile's replica stores are issued after the next tile's
    // loads, so the loads can be waited for while the stores drain.  The
    // compiler's wait insertion merges the loop's entry and back-edge states
    // by the youngest position of each pending register: at the entry the
    // loads ARE the youngest ops, so it would wait vmcnt(1) at the top of
    // every tile -- for all of the previous tile's stores to complete.
    // Issuing the same stores here (zeros into this wave's replica cells of
    // its first tile, which that tile overwrites, in order, from the same
    // wave) makes both states alike.
    if constexpr (QUAD)
      quad_zero_dispatch<K, N, RPW, WV, STREAM, 0>(wave, a, tile_pos(a, tile), lane, bm);
    else if constexpr (SPLIT)
      pair_zero_dispatch<K, N, RPW, WV, STREAM, 0>(wave, a, tile_pos(a, tile), lane, bm);
    else
      encode_zero_dispatch<K, N, RPW, WV, STREAM, 0>(wave, a, tile_pos(a, tile), lane, bm);
  }
  for (; tile < t_end; tile += t_step) {
    // ---- transpose to planes and publish in LDS: cell 4p+2g+h, bit b = R[g][16h + (b^8)]
    uint32_t R[2][32];
    // Two workgroups per CU (k = 16): the one transposing a tile into LDS
    // runs at priority 1, so it reaches the barrier while the other's Horner
    // waits a little (same-box A/B, 512 objects, three rounds: 13.94-13.96 ->
    // 13.72-13.75 ms; priority on the Taylor step as well: no further gain).
    constexpr bool kPrio = 2 * S::kLdsBytes <= 160 * 1024;
    if constexpr (kPrio) __builtin_amdgcn_s_setprio(1);
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
      transpose32<enc_rot(K)>(R[g], bm);
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          const int b0 = 16 * h + 4 * (m ^ 2);
          *reinterpret_cast<uint4 *>(t_planes + (2 * g + h) * 16 + 4 * m) =
              make_uint4(R[g][b0], R[g][b0 + 1], R[g][b0 + 2], R[g][b0 + 3]);
        }
    }
    if constexpr (kPrio) __builtin_amdgcn_s_setprio(0);
    __syncthreads();
    // ---- prefetch the next tile while this one is evaluated (software pipeline)
    const uint32_t next = tile + t_step;
    if (next < t_end) load(next);
    // ---- evaluate this wave's replicas and store
    if constexpr (QUAD) {
      taylor_lds<K, N, RPW, WV>(wave, my_set);
      __syncthreads();
      quad_twist_lds<K, N, RPW, WV>(wave, my_set);
      __syncthreads();
      quad_taylor_lds<K, N, RPW, WV>(wave, my_set);
      __syncthreads();
      quad_dispatch<K, N, RPW, WV, STREAM, 0>(wave, my_set, a, tile_pos(a, tile), lane, bm);
    } else if constexpr (SPLIT) {
#if VDS_DIAG_ENC != 1  // diagnostic builds (wrong bytes, timing only): 1 = no Taylor step, 2 = no evaluation
      taylor_lds<K, N, RPW, WV>(wave, my_set);
      __syncthreads();
#endif
#if VDS_DIAG_ENC != 2
      pair_dispatch<K, N, RPW, WV, STREAM, 0>(wave, my_set, a, tile_pos(a, tile), lane, bm);
#endif
    } else {
      encode_dispatch<K, N, RPW, WV, STREAM, 0>(wave, my_set, a, tile_pos(a, tile), lane, bm);
    }
    __syncthreads();
  }
}

template <int K, int N, int RPW, int WV, bool STREAM, bool SPLIT, bool QUAD>
static hipError_t launch_encode_bs_st(const FastEncodeArgs &a, hipStream_t s) {
  using S = EncodeShape<K, N, RPW, WV>;
  // VDS_ENC_LDS_EXTRA: extra (unused) LDS bytes per workgroup, to measure
  // the kernel at fewer workgroups per CU (diagnostic, ec_device.hpp)
  static_assert(VDS_ENC_LDS_EXTRA >= 0 && VDS_ENC_LDS_EXTRA < 64 * 1024, "VDS_ENC_LDS_EXTRA");
  const int lds = S::kLdsBytes + VDS_ENC_LDS_EXTRA;
  hipError_t e = ensure_lds_attr(&k_encode_bs<K, N, RPW, WV, STREAM, SPLIT, QUAD>, lds);
  if (e != hipSuccess) return e;
  const int blocks_per_cu = (160 * 1024) / lds;
  int grid = 256 * (blocks_per_cu > 0 ? blocks_per_cu : 1);
  if (VDS_ENC_GRID > 0) grid = VDS_ENC_GRID;
  if ((uint32_t)grid > a.total_tiles) grid = (int)a.total_tiles;
  if (grid == 0) return hipSuccess;
  hipLaunchKernelGGL((k_encode_bs<K, N, RPW, WV, STREAM, SPLIT, QUAD>), dim3(grid), dim3(S::kThreads), lds, s, a);
  return hipGetLastError();
}

// A/B builds: -DVDS_ENCODE_PATH=1 plain Horner where split mode is compiled,
// 2 the one-level split where the two-level one is the default, 3 the
// two-level split everywhere; 0 (default) the measured choice below.
#ifndef VDS_ENCODE_PATH
#define VDS_ENCODE_PATH 0
#endif
constexpr char encode_path() {
  return VDS_ENCODE_PATH == 1 ? 'h' : VDS_ENCODE_PATH == 2 ? 'p' : VDS_ENCODE_PATH == 3 ? 'q' : '\0';
}

template <int K, int N, int RPW, int WV, bool SPLIT, bool QUAD>
static hipError_t launch_encode_bs_sp(const FastEncodeArgs &a, hipStream_t s) {
  if (a.groups_per_obj % 16 == 0) return launch_encode_bs_st<K, N, RPW, WV, false, SPLIT, QUAD>(a, s);
  if constexpr (K >= 8) return launch_encode_bs_st<K, N, RPW, WV, true, SPLIT, QUAD>(a, s);
  return hipErrorNotSupported;
}

// Two-level split for N = 64 (the live shape: +5.5%, same box), one-level for
// K >= 16 otherwise (two-level measured slower at k = 32 / n = 40, 10.35-10.5
// vs 10.1-10.15 ms, and at k = 16: DESIGN.md section 3), plain Horner below.
template <int K, int N, int RPW, int WV>
static hipError_t launch_encode_bs(const FastEncodeArgs &a, hipStream_t s) {
  if constexpr (K >= 16 && N % 4 == 0) {
    if (encode_path() == 'q' || (N == 64 && encode_path() == '\0'))
      return launch_encode_bs_sp<K, N, RPW, WV, true, true>(a, s);
  }
  if constexpr (K >= 16) {
    if (encode_path() != 'h') return launch_encode_bs_sp<K, N, RPW, WV, true, false>(a, s);
  }
  return launch_encode_bs_sp<K, N, RPW, WV, false, false>(a, s);
}

}  // namespace vds_ec
