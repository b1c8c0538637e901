// restore_syn.hpp -- the k_restore_syn kernel body (ec_restore_syn.hip), in a
// header of its own so that vds_ec_jit.cpp can compile pattern-specific
// instantiations of it at run time (hiprtc) from the same source.
//
// Restore of an object from any K of its N replicas without a per-pattern
// K x K inverse (chunk_restore<uint16_t>::restore, chunk.h:290-444; the
// BASELINE configs (16, 20) and (32, 40)).  The generated RestorePrograms<K,
// N, WV> specialisations (generated/restore_K_N_wW.inc) must be included
// before the body is instantiated.
#pragma once

#include "ec_device.hpp"

namespace vds_ec {

constexpr int64_t kNoBound = 0x7FFFFFFFFFFFFFFFll;

template <int K, int N, int WV> struct RestorePrograms;

// k_restore_syn<K, N, WV>: one 2048-stripe tile per workgroup of WV waves.
// Two such workgroups share a CU (k = 16); their phases drift apart, so one
// workgroup's barrier waits and memory phases overlap the other's VALU.  (Two
// tiles per 8-wave workgroup, which keeps the two waves of a SIMD in the same
// phase, measured slower: repair 1597 -> 1478-1486 GiB/s at 512 objects.)
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
  static constexpr bool kPrio = 160 * 1024 / kLdsBytes >= 2;  // phase priorities (syn_prio)
  static_assert(K % WV == 0 && kM <= WV, "survivor loads and erased slots must map onto waves");
  static_assert(kSynRows == 16 && kM == WV, "scatter recovery needs one whole syndrome per wave");
  static_assert(kCells == 2 || kCells == 4, "row split must be b128 / word-group aligned");
  static_assert(kLdsBytes <= 160 * 1024, "LDS");
};

// Diagnostic build (VDS_DIAG_STAMPS=1, timing only): every wave of
// k_restore_syn accumulates s_memtime deltas per phase of its tiles into
// g_syn_stamps[block][wave][phase] (read with vds_ec_diag_stamps; phases in
// tools/syn_stamps.py).  The marks wait for outstanding scalar and LDS
// operations and the compiler may move VALU work across them: read the
// barrier waits, not the exact split of neighbouring phases.  Off: the marks
// compile to nothing.  tests/test_build.py compile-checks this build.
#ifndef VDS_DIAG_STAMPS
#define VDS_DIAG_STAMPS 0
#endif
// Load study (wrong results, timing only; with the stamps): 1 = every tile
// after the first reloads the first tile's survivors (L2 hits), 2 = no loads
// after the first tile (zero survivors).  Round 6, k = 32 (§3.7 of DESIGN.md).
#ifndef VDS_DIAG_LOADS
#define VDS_DIAG_LOADS 0
#endif

// Wave priority by phase when two workgroups share a CU (k = 16).  Their
// phases drift apart; the workgroup in stage 1 (survivors -> LDS planes) and
// stage A runs at priority 1, and the one transposing and staging its output
// at 2, so the other workgroup's long XOR programs fill the gaps instead of
// delaying the phases that end in a barrier of all four waves.  Same-box A/B,
// 512 x 64 MiB: repair 18.65 -> 16.54-16.59 ms (+12%), again on a second box
// 19.0-19.25 -> 16.9-17.0 ms.  Also measured: priority on the copy-out stores
// (neutral), on stage 1 alone (+1.6%), staging alone (+0.5%), the syndrome
// programs or stage B or C as well (less gain; every phase at 1 is the
// default again); stage C at 1 or every level one higher (1 -> 2, 2 -> 3):
// within 1%.  One workgroup per CU (k = 32): neutral, not used.
template <int PRIO, bool ON>
__device__ __forceinline__ void syn_prio() {
  if constexpr (ON) __builtin_amdgcn_s_setprio(PRIO);
}

#if VDS_DIAG_STAMPS
// phases 0..19 are s_memtime sums; 20..23 hold the s_memrealtime (chip-wide
// 100 MHz clock) at which the wave issued the survivor loads of its
// kStampRtIter[j]-th tile, so the host can compare the CUs' phases.
constexpr int kStampPhases = 24;
constexpr uint32_t kStampRtIter[4] = {4, 64, 160, 240};
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
  __device__ __forceinline__ void rt(uint32_t iter) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (iter == kStampRtIter[j]) acc[20 + j] = __builtin_amdgcn_s_memrealtime();
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
  __device__ __forceinline__ void rt(uint32_t) {}
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

// Interpolation from the fixed points F = {0..K-1} by one level of the
// additive FFT (Gao-Mateer).  F is the GF(2)-span of 1, x, x^2, x^3 (, x^4),
// so with G = {0, 2, .., K-2} and s(X) = X^2 + X (which maps g and g+1 to the
// same point):
//   P(X) = P0(s(X)) + X P1(s(X)),  deg P0, P1 < K/2,
//   P1(s(g)) = c_g + c_{g+1},  P0(s(g)) = c_g + g P1(s(g)).
// Stage A forms those K/2 value pairs in place (Q0 -> slot g, Q1 -> slot g+1),
// stage B interpolates P0 and P1 on D = s(G) with generated XOR programs
// (RestorePrograms::interpB), and stage C expands (X^2+X)^i = X^i (X+1)^i,
// whose coefficients are binomials mod 2, so it is XORs only.  About 60% of
// the XORs of the direct 16-point program (1375 vs 1280 GiB/s).
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
// k = 16: each slot the wave's cells use is read once and XORed into every
// cell that takes it (slot-major).  Cell-major (G = 1), the compiler re-read
// a slot for every cell that takes it: 54 slot reads per tile for 30 distinct
// ones (wave 3: 36 ds_read_b128 for 4 slots).  Same box, three interleaved
// rounds at 512 x 64 MiB (profiles/round5/ab_stagec.log): survivor-set repair
// 14.22-14.38 -> 14.15-14.26 ms, k_restore_syn<16,20> 16.78-16.86 -> 16.55-
// 16.60.  k = 32 keeps cell-major: all four cells at once spilled 96 VGPRs
// beside the late loads, two at a time (162 -> 122 slot reads) measured
// 10.13-10.19 -> 10.19-10.25 ms (256 x 64 MiB).
template <int K, int W, int NC, int G = (K == 16 ? NC : 1)>
__device__ __forceinline__ void syn_gm_stage_c(const SynLds &L, uint32_t (&cells)[16 * NC]) {
  constexpr auto takes = [](int c, int t) {
    const int k = NC * W + c, i = t % (K / 2);
    const int m = t < K / 2 ? k - i : k - 1 - i;
    return m >= 0 && m <= i && (m & ~i) == 0;
  };
#pragma unroll
  for (int c0 = 0; c0 < NC; c0 += G) {
    bool first[G];
#pragma unroll
    for (int c = 0; c < G; ++c) first[c] = true;
#pragma unroll
    for (int t = 0; t < K; ++t) {
      bool any = false;
#pragma unroll
      for (int c = 0; c < G; ++c) any |= takes(c0 + c, t);
      if (any) {
        uint32_t v[16];
        syn_get_point(L, t, v);
#pragma unroll
        for (int c = 0; c < G; ++c)
          if (takes(c0 + c, t)) {
#pragma unroll
            for (int b = 0; b < 16; ++b) cells[16 * (c0 + c) + b] = first[c] ? v[b] : cells[16 * (c0 + c) + b] ^ v[b];
            first[c] = false;
          }
      }
    }
#pragma unroll
    for (int c = 0; c < G; ++c)
      if (first[c])
#pragma unroll
        for (int b = 0; b < 16; ++b) cells[16 * (c0 + c) + b] = 0u;
  }
}

template <int K, int N, int WV, int W>
__device__ __forceinline__ void syn_interp_gm(int wave, const SynLds &L, uint32_t (&cells)[16 * (K / WV)], Stamps &st) {
  static_assert((K == 16 && WV == 4) || (K == 32 && WV == 8),
                "the one-level interpolation is laid out for k = 16 and k = 32");
  using P = RestorePrograms<K, N, WV>;
  constexpr int kPairs = (K / 2) / WV;           // stage-A pairs per wave
  constexpr int kHalfCells = P::kHalfRows / 16;  // stage-B cells per wave
  constexpr int kParts = WV / 2;                 // waves per half-size polynomial
  constexpr bool kPrio = SynShape<K, N, WV>::kPrio;
  if constexpr (W < WV) {
    if (wave != W) return syn_interp_gm<K, N, WV, W + 1>(wave, L, cells, st);
    syn_prio<1, kPrio>();
    syn_gm_stage_a<W, kPairs>(L);
    syn_prio<0, kPrio>();
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

// S1's input with point EP served from registers (the own-group fill below).
template <int EP>
struct S1In {
  const SynLds &L;
  const Plane16 &own;
  __device__ __forceinline__ u32x4 operator()(int g) const {
    if ((g >> 2) == EP) return u32x4{own.p[4 * (g & 3)], own.p[4 * (g & 3) + 1], own.p[4 * (g & 3) + 2], own.p[4 * (g & 3) + 3]};
    return L(g);
  }
};

// Two-level interpolation (VDS_GM2, default; generated gm_* programs,
// tools/xorgen/gen_restore.cpp emit_gm2): levels 1 and 2 of the additive FFT
// on each wave's own four slots (S1, in place), the K/4-point direct
// interpolation of the four level-2 families (S2), the level-2 expansion and
// twist (S3, into stage C's layout), then stage C.  Against one level + K/2-
// point direct programs: 3175 vs ~4700 XOR instructions per tile at k = 16,
// 12311 vs ~20000 at k = 32, for one (k = 16) or two more barriers.
#ifndef VDS_GM2
#define VDS_GM2 1
#endif
// Phases of the two-level interpolation run at wave priority 1 (bit 0: S1,
// bit 1: S2, bit 2: S3, bit 3: stage C; two workgroups per CU only, see
// syn_prio).  Same box, k = 16 repair at 512 x 64 MiB: S1 alone 14.19-14.30
// ms, S1 + stage C 14.05-14.10 (default); none 15.0-15.15; S2 or S3 added
// 14.67-14.88 (profiles/round3/ab/gm2_prio_ab.log, prio2_ab.log).
#ifndef VDS_GM2_PRIO
#define VDS_GM2_PRIO 9
#endif
// One workgroup per CU (k = 32): the second-dispatched half of the waves
// (wave >= WV / 2) loses VALU arbitration to the older half by age and lags
// in every phase (profiles/round4/ablog/l2_touch_k32_stamps.txt), so it runs
// at priority 1 for the whole kernel.  Same box, C4 at 256 x 64 MiB, three
// interleaved rounds (profiles/round5/ab_halfprio.log): survivor-set kernel
// 10.03-10.16 -> 9.83-9.89 ms, k_restore_syn<32,40> 12.33-12.40 -> 12.26-12.32.
// VDS_HALF_PRIO=0 is the A/B switch.
#ifndef VDS_HALF_PRIO
#define VDS_HALF_PRIO 1
#endif
// OwnP (not void): the own-group fill's policy; `own` is this wave's group's
// erased point, which S1 takes from registers.
template <int K, int N, int WV, int W, class Tail, class OwnP = void>
__device__ __forceinline__ void syn_interp_gm2(int wave, const SynLds &L, Stamps &st, Tail &&tail,
                                               const Plane16 *own = nullptr) {
  using P = RestorePrograms<K, N, WV>;
  constexpr bool kPrio = SynShape<K, N, WV>::kPrio;
  constexpr int H = K / 2, kWpf = WV / 4, kWpq = WV / 2;
  if constexpr (W < WV) {
    if (wave != W) return syn_interp_gm2<K, N, WV, W + 1, Tail &, OwnP>(wave, L, st, tail, own);
    uint32_t cells[16 * (K / WV)];
    uint32_t acc[64];
    auto cell = [&](int c) -> uint32_t(&)[16] { return *reinterpret_cast<uint32_t(*)[16]>(acc + 16 * c); };
    // S1: levels 1 and 2 on this wave's slots 4W..4W+3 (only this wave touches them)
    syn_prio<1, kPrio && (VDS_GM2_PRIO & 1)>();
    if constexpr (__is_same(OwnP, void))
      P::gm_s1_(W, L, acc);
    else
      P::gm_s1_(W, S1In<OwnP::kPoint[W]>{L, *own}, acc);
#pragma unroll
    for (int c = 0; c < 4; ++c) syn_put_point(L, 4 * W + c, cell(c));
    syn_prio<0, kPrio && (VDS_GM2_PRIO & 1)>();
    st.mark(7);
    __syncthreads();
    st.mark(8);
    // S2: family f = W / kWpf (slots 4j + f), coefficients c0.. -> slot 4c + f
    // (k = 32: the family's two waves each hold planes 8h..8h+7 of all eight
    // coefficients, acc[8c + ..], h = W % 2: gen_restore.cpp emit_gm2)
    syn_prio<1, kPrio && (VDS_GM2_PRIO & 2)>();
    P::gm_s2_(W, L, acc);
    constexpr int f = W / kWpf, c0 = 4 * (W % kWpf);
    if constexpr (kWpf > 1) {
      __syncthreads();  // (every wave of the family has read it)
      constexpr int h = W % kWpf;
      static_assert(kWpf == 2 && K / 4 == 8, "plane-split S2 is laid out for k = 32");
#pragma unroll
      for (int c = 0; c < 8; ++c)
#pragma unroll
        for (int g = 0; g < 2; ++g)
          L.put(4 * (4 * c + f) + 2 * h + g,
                u32x4{acc[8 * c + 4 * g], acc[8 * c + 4 * g + 1], acc[8 * c + 4 * g + 2], acc[8 * c + 4 * g + 3]});
    } else {
#pragma unroll
      for (int c = 0; c < 4; ++c) syn_put_point(L, 4 * (c0 + c) + f, cell(c));
    }
    syn_prio<0, kPrio && (VDS_GM2_PRIO & 2)>();
    st.mark(9);
    __syncthreads();
    st.mark(10);
    // S3: Q_par coefficients i0.. (expansion sums, then the twists) -> slot H par + i
    syn_prio<1, kPrio && (VDS_GM2_PRIO & 4)>();
    P::gm_s3sum_(W, L, acc);
    constexpr int par = W / kWpq, i0 = 4 * (W % kWpq);
#pragma unroll
    for (int c = 0; c < 4; ++c) P::gm_twist(i0 + c, cell(c));
    syn_prio<0, kPrio && (VDS_GM2_PRIO & 4)>();
    __syncthreads();  // every wave has read the R coefficients
#pragma unroll
    for (int c = 0; c < 4; ++c) syn_put_point(L, H * par + i0 + c, cell(c));
    st.mark(11);
    __syncthreads();
    st.mark(12);
    syn_prio<1, kPrio && (VDS_GM2_PRIO & 8)>();
    syn_gm_stage_c<K, W, K / WV>(L, cells);
    syn_prio<0, kPrio && (VDS_GM2_PRIO & 8)>();
    st.mark(13);
    tail(cells);  // (staging and copy-out, in this wave's branch: see the caller)
  }
}

// One coefficient-bit pair of the recovery walk: acc ^= T, T1 or T ^ T1 as
// the pair's two bits select (two = bit b | bit b+1 << 8), in one asm block
// with its own branches.  As plain C++ the three arms computed into
// different registers and every merge block copied the sixteen planes back
// (8 v_mov_b64 per product and bit pair: as many moves as XORs); here the
// planes are updated in place.  (The compares write SCC: declared clobbered,
// or a live SCC of the surrounding code is lost.)
#define VDS_RS_C(i) [c##i] "+v"(acc.p[i])
#define VDS_RS_A(i) [a##i] "v"(t.p[i])
#define VDS_RS_B(i) [b##i] "v"(t1.p[i])
#define VDS_RS_LIST(M) M(0), M(1), M(2), M(3), M(4), M(5), M(6), M(7), M(8), M(9), M(10), M(11), M(12), M(13), M(14), M(15)
#define VDS_RS_SEQ(M) M(0) M(1) M(2) M(3) M(4) M(5) M(6) M(7) M(8) M(9) M(10) M(11) M(12) M(13) M(14) M(15)
#define VDS_RS_XA(i) "v_xor_b32 %[c" #i "], %[c" #i "], %[a" #i "]\n"
#define VDS_RS_XB(i) "v_xor_b32 %[c" #i "], %[c" #i "], %[b" #i "]\n"
#define VDS_RS_X3(i) "v_bitop3_b32 %[c" #i "], %[c" #i "], %[a" #i "], %[b" #i "] bitop3:0x96\n"
__device__ __forceinline__ void rec_pair(Plane16 &acc, const Plane16 &t, const Plane16 &t1, uint32_t two) {
  asm volatile(
      "s_cmp_eq_u32 %[two], 1\n"
      "s_cbranch_scc0 1f\n" VDS_RS_SEQ(VDS_RS_XA)
      "s_branch 3f\n"
      "1:\n"
      "s_cmpk_eq_u32 %[two], 0x100\n"
      "s_cbranch_scc0 2f\n" VDS_RS_SEQ(VDS_RS_XB)
      "s_branch 3f\n"
      "2:\n"
      "s_cmpk_eq_u32 %[two], 0x101\n"
      "s_cbranch_scc0 3f\n" VDS_RS_SEQ(VDS_RS_X3)
      "3:\n"
      : VDS_RS_LIST(VDS_RS_C)
      : VDS_RS_LIST(VDS_RS_A), VDS_RS_LIST(VDS_RS_B), [two] "s"(two)
      : "scc");
}
// RT mode: the same walk with a different coefficient in each half of the
// tile.  After the stage-1 transpose, bits 0-7 and 16-23 of every plane word
// hold half 0's stripes and bits 8-15, 24-31 half 1's (kRtH0 / kRtH1), so a
// coefficient bit is a wave-uniform mask per bit -- 0, kRtH0, kRtH1 or all
// ones -- and acc ^= (T & ma) ^ (T1 & mb) is one masked v_bitop3 per plane
// and nonzero mask.  (Seven specialised arms per bit pair, as rec_pair's,
// made the unrolled walk ~128 KiB of code: it thrashed the instruction cache,
// 4x slower per tile; one arm per mask value, with the masks preloaded in
// VGPRs, measured no faster than this copy of the mask: 363 vs 377 GiB/s.)
// The mask is copied to a VGPR first: a v_bitop3 reading an SGPR issues at
// ~0.6 of the all-VGPR rate.
//
// x holds the two halves' coefficients of one (row, slot) as bits 0-7 = half
// 0's low byte, 8-15 = half 1's, 16-23 / 24-31 the high bytes
// (SynBatchRt::coef's spread words, half 1's shifted by 8).  Bit b's two bits
// are then 0x101 << pos(b), and ((x & that) >> pos) * 0x00FF00FF is the
// plane mask in three SALU, the s_and's SCC (mask nonzero) feeding the
// branch: against seven (two bit extracts, two selects, an or, a compare)
// when the mask was built from the two coefficients bit by bit.
constexpr uint32_t kRtH0 = 0x00FF00FFu, kRtH1 = 0xFF00FF00u;
// f(IntK<B>{}), .., f(IntK<E - 1>{}) (the run-time compiled kernels include
// this header under hiprtc, without the standard library's index sequences)
template <int V> struct IntK {
  static constexpr int value = V;
};
template <int B, int E, class F> __device__ __forceinline__ void static_for(F &&f) {
  if constexpr (B < E) {
    f(IntK<B>{});
    static_for<B + 1, E>(f);
  }
}
#define VDS_RD_MA(i) "v_bitop3_b32 %[c" #i "], %[c" #i "], %[a" #i "], %[tm] bitop3:0x78\n"
#define VDS_RD_MB(i) "v_bitop3_b32 %[c" #i "], %[c" #i "], %[b" #i "], %[tm] bitop3:0x78\n"
template <int BIT>
__device__ __forceinline__ void rec_dual_x(Plane16 &acc, const Plane16 &t, const Plane16 &t1, uint32_t x) {
  constexpr uint32_t pa = BIT < 8 ? BIT : BIT + 8, pb = BIT + 1 < 8 ? BIT + 1 : BIT + 9;
  uint32_t tm, sm;
  asm volatile(
      "s_and_b32 %[sm], %[x], %[ka]\n"
      "s_cbranch_scc0 1f\n"
      "s_lshr_b32 %[sm], %[sm], %[pa]\n"
      "s_mul_i32 %[sm], %[sm], 0xff00ff\n"
      "v_mov_b32 %[tm], %[sm]\n" VDS_RS_SEQ(VDS_RD_MA)
      "1:\n"
      "s_and_b32 %[sm], %[x], %[kb]\n"
      "s_cbranch_scc0 2f\n"
      "s_lshr_b32 %[sm], %[sm], %[pb]\n"
      "s_mul_i32 %[sm], %[sm], 0xff00ff\n"
      "v_mov_b32 %[tm], %[sm]\n" VDS_RS_SEQ(VDS_RD_MB)
      "2:\n"
      : VDS_RS_LIST(VDS_RS_C), [tm] "=&v"(tm), [sm] "=&s"(sm)
      : VDS_RS_LIST(VDS_RS_A), VDS_RS_LIST(VDS_RS_B), [x] "s"(x), [ka] "i"(0x101u << pa), [kb] "i"(0x101u << pb),
        [pa] "i"(pa), [pb] "i"(pb)
      : "scc");
}
// The same with the two masks given: acc ^= (T & ma) ^ (T1 & mb), ma / mb in
// {0, kRtH0, kRtH1, ~0} (a dual syndrome tile's bit pair of one row: each
// half's own coefficient bit).
__device__ __forceinline__ void rec_dual_m(Plane16 &acc, const Plane16 &t, const Plane16 &t1, uint32_t ma,
                                           uint32_t mb) {
  uint32_t tm;
  asm volatile(
      "s_cmp_eq_u32 %[ma], 0\n"
      "s_cbranch_scc1 1f\n"
      "v_mov_b32 %[tm], %[ma]\n" VDS_RS_SEQ(VDS_RD_MA)
      "1:\n"
      "s_cmp_eq_u32 %[mb], 0\n"
      "s_cbranch_scc1 2f\n"
      "v_mov_b32 %[tm], %[mb]\n" VDS_RS_SEQ(VDS_RD_MB)
      "2:\n"
      : VDS_RS_LIST(VDS_RS_C), [tm] "=&v"(tm)
      : VDS_RS_LIST(VDS_RS_A), VDS_RS_LIST(VDS_RS_B), [ma] "s"(ma), [mb] "s"(mb)
      : "scc");
}
#undef VDS_RD_MA
#undef VDS_RD_MB
#undef VDS_RS_C
#undef VDS_RS_A
#undef VDS_RS_B
#undef VDS_RS_LIST
#undef VDS_RS_SEQ
#undef VDS_RS_XA
#undef VDS_RS_XB
#undef VDS_RS_X3

// LDS XOR of a point's sixteen planes (this lane's 64 bytes) as eight
// ds_xor_b64: planes 4g..4g+3 of point pt at byte (4 pt + g) 1 KiB + 16 lane.
// With every lane on the same 8-byte half of its 16-byte slot, lanes 8 or 16
// apart hit the same banks (2-way).  A swizzle that gave lanes whose bits 3
// and 4 differ the other half first removed every conflict
// (SQ_LDS_BANK_CONFLICT 0) and was slower: same box, k = 16 repair 13.99-
// 14.04 -> 14.17-14.33 ms, k = 32 9.67 -> 10.41 ms
// (profiles/round3/ab/swz_ab.log; deleted in round 4).
__device__ __forceinline__ void lds_xor_point(const SynLds &L, int pt, const Plane16 &v) {
  __attribute__((address_space(3))) uint64_t *dst =
      (__attribute__((address_space(3))) uint64_t *)(L.base + L.lo + 4096u * pt);
#pragma unroll
  for (int h = 0; h < 8; ++h)
    __hip_atomic_fetch_xor(dst + 128 * (h >> 1) + (h & 1), (uint64_t)v.p[2 * h] | ((uint64_t)v.p[2 * h + 1] << 32),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Scatter fill (FillP::kScatter, vds_ec_jit.cpp): wave W's share of every
// erased point below K, XORed into the zeroed slots.  Dispatched on a
// compile-time wave so each arm stores its own results (a runtime switch
// merged the 64 result registers of all arms and spilled them).
// VDS_FILL_REGS (k = 16): the programs read the wave's four survivors from
// the stage-1 registers (FillRegIn) instead of reading back the slots it has
// just stored (16 of the tile's ~920 LDS instructions per wave).  Same box,
// six processes each in ABBA order at 512 x 64 MiB, with the staging in each
// wave's branch (below): survivor-set repair 14.05-14.18 -> 13.85-13.99 ms,
// mean -1.3% (profiles/round5/ab_fill_regs_abba.log).  Running the fill's XORs before stage
// 1's barrier as well (one barrier in each wave's arm, guarding only the
// atomics) measured no better than before: 14.04-14.16 ms.
#ifndef VDS_FILL_REGS
#define VDS_FILL_REGS 1
#endif
template <class FillP, int W>
struct FillRegIn {
  const Plane16 (&P)[4];
  static constexpr int slot(int pt) {
    for (int i = 0; i < 4; ++i)
      if (FillP::kSurv[4 * W + i] == pt) return i;
    return -1;
  }
  __device__ __forceinline__ u32x4 operator()(int idx) const {
    const int i = slot(idx >> 2), g = idx & 3;
    return u32x4{P[i].p[4 * g], P[i].p[4 * g + 1], P[i].p[4 * g + 2], P[i].p[4 * g + 3]};
  }
};
template <int WV, class FillP, bool REGS, int W>
__device__ __forceinline__ void syn_scatter_fill(int wave, const SynLds &L, const Plane16 (&Ps)[4]) {
  if constexpr (W < WV) {
    if (wave != W) return syn_scatter_fill<WV, FillP, REGS, W + 1>(wave, L, Ps);
#pragma unroll
    for (int q = 0; q < FillP::kParts; ++q) {
      uint32_t acc[16 * FillP::kPart];
      if constexpr (REGS)
        FillP::fill_part(q, W, FillRegIn<FillP, W>{Ps}, acc);
      else
        FillP::fill_part(q, W, L, acc);
#pragma unroll
      for (int m = 0; m < FillP::kPart; ++m)
        if (q * FillP::kPart + m < FillP::kFill)
          lds_xor_point(L, FillP::kPoint[q * FillP::kPart + m < FillP::kFill ? q * FillP::kPart + m : 0],
                        *reinterpret_cast<const Plane16 *>(acc + 16 * m));
    }
  }
}

// Own-group fill (FillP::kOwn, xorprog.hpp emit_fill_own; k = 16 survivor
// sets with one erased point in each wave's interpolation group 4w..4w+3):
// wave W computes its group's erased point from all survivors -- its own
// four from the stage-1 registers (OwnIn), the rest from LDS -- and S1 reads
// it from registers (S1In), so nothing is written, zeroed or XORed into LDS
// for it and no barrier separates the fill from S1.
template <class F, class = void>
struct FillOwn {
  static constexpr bool value = false;
};
template <class F>
struct FillOwn<F, decltype(void(F::kOwn))> {
  static constexpr bool value = F::kOwn;
};
template <class FillP, int W>
struct OwnIn {
  const SynLds &L;
  const Plane16 (&P)[4];
  __device__ __forceinline__ u32x4 operator()(int idx) const {
    const int i = FillRegIn<FillP, W>::slot(idx >> 2), g = idx & 3;
    if (i >= 0) return u32x4{P[i].p[4 * g], P[i].p[4 * g + 1], P[i].p[4 * g + 2], P[i].p[4 * g + 3]};
    return L(idx);
  }
};
template <int WV, class FillP, int W>
__device__ __forceinline__ void syn_own_fill(int wave, const SynLds &L, const Plane16 (&Ps)[4], Plane16 &own) {
  if constexpr (W < WV) {
    if (wave != W) return syn_own_fill<WV, FillP, W + 1>(wave, L, Ps, own);
    FillP::template own<W>(OwnIn<FillP, W>{L, Ps}, own.p);
  }
}

// Batch mode: the last tile of an object may run past its bytes.  Loads
// beyond `valid` bytes read zeros and stores beyond it write nothing (byte by
// byte for the one 16-byte piece that straddles the end).
__device__ __forceinline__ u32x4 ld16_guard(const uint8_t *p, int64_t valid) {
  if (valid >= 16) return g_ld<4, u32x4>(p);
  u32x4 v = {0u, 0u, 0u, 0u};
  if (valid > 0) {  // (chunk lengths are even: whole dwords, then a 2-byte cell)
#pragma unroll
    for (int i = 0; i < 3; ++i)
      if (4 * i + 4 <= valid) v[i] = *(const gmem<uint32_t> *)(p + 4 * i);
    if (valid & 2) v[valid >> 2] = *(const gmem<uint16_t> *)(p + (valid & ~3));
  }
  return v;
}
__device__ __forceinline__ void st16_guard(uint8_t *p, u32x4 v, int64_t valid) {
  if (valid >= 16) {
    g_st<8>(p, v);
  } else if (valid > 0) {
#pragma unroll
    for (int i = 0; i < 3; ++i)
      if (4 * i + 4 <= valid) *(gmem<uint32_t> *)(p + 4 * i) = v[i];
    const int w = (int)(valid >> 2);
    const uint32_t x = v[w];
    for (int b = 0; b < (int)(valid & 3); ++b) ((gmem<uint8_t> *)p)[4 * w + b] = uint8_t(x >> (8 * b));
  }
}

// Restore of an object from any K of its N replicas without a per-pattern
// K x K inverse (tools/xorgen/gen_restore.cpp).  Per tile, wave w:
//  1. loads survivors kLoadPer*w.. into their points' planes (waves < M also
//     zero one erased point);
//  2. computes syndrome S_w over all N points (erased points read as zero)
//     and scatters its share of every recovered point into the erased slots;
//  3. interpolates cells kCells*w.. from the fixed points 0..K-1 and stores
//     them big-endian.
// Tiles are strided over each XCD's workgroups (tile_range; one contiguous
// range of tiles per workgroup measured slower: repair 1572 -> 1460 GiB/s).
// BATCH: one launch over the tiles of many objects, each with its own
// survivors, erasure plan, size and output (SynBatchTile / SynBatchObj /
// SynBatchPlan, read with wave-uniform scalar loads).  Each half of a tile
// (q = 0, 1 and q = 2, 3 of the loads; waves 0..WV/2-1 and WV/2.. of the
// copy-out) is a stripe range of its own object; a half that runs past its
// object's bytes takes the guarded loads and stores.
// RT (batch only): phase 2 is the runtime-coefficient combination of the
// slots (SynBatchRt) instead of syndromes + recovery, so any k survivors of
// any ids serve, a different set in each half of a tile: restore writes the
// combinations into the borrowed slots' erased points and interpolates as
// usual; regenerate accumulates row m in LDS slot K + m and stores it as
// replica bytes.  Each wave combines the slots it loaded (registers) for
// every row and adds its share with LDS XOR atomics, so the waves split the
// work evenly whatever the rows.
// FILL: a pattern-specific program (FillP, generated for one erased set and
// compiled at run time, vds_ec_jit.cpp) computes the erased points below K
// straight from the survivors instead of syndromes + recovery.
struct NoFill {
  static constexpr int kFill = -1;
  static constexpr bool kScatter = false;
  static constexpr bool kSmall = false;
  static constexpr bool kPerm = false;
  static constexpr bool kMulti = false;
};
// MULTI (batch only): one launch over the tiles of every class of a batch --
// the N = K + K/4 syndromes (kClsSyn), SMALL ms = 1, 2 (kClsSmall1/2), PERM
// (kClsPerm, regenerate) -- each tile's phase 2 chosen by its plan's cls, so
// no class waits for another launch's last tiles.  (Side-by-side launches of
// the classes on their own streams and CU shares measured much slower: live
// repair 1283 -> 823 GiB/s.)
constexpr uint32_t kClsSyn = 0, kClsSmall1 = 1, kClsSmall2 = 2, kClsPerm = 3;
template <int K> struct MultiP {
  static constexpr int kFill = -1;
  static constexpr bool kScatter = false, kSmall = false, kPerm = false, kMulti = true;
};
template <class T> struct TypeTag {
  using type = T;
};
// PERM (batch regenerate only): FillP = PermSyn<K> (generated/permsyn_K.inc).
// Survivors exactly U = {0..K-1}, one target t = K + t' (t' in U): P(t) =
// sum_c l_c(K) y_(c ^ t') -- one fixed program for every such target, its
// LDS reads permuted by the plan's t' (gen_restore.cpp main_perm).  Wave w
// adds its four points' share into slot K; wave 0 stores it as replica t.
// The plan's erased[0] is t (the regenerate tail reads it there too).
template <int K> struct PermSyn;
// SMALL (batch only): FillP = SmallSyn<K, MS> (generated/smallsyn_K_MS.inc).
// The survivors lie in A = {0..K+MS-1}: the MS checks of the code restricted
// to A, S_j = sum_{a in A} v_a a^j y_a (erased points zero), determine A's
// erased points through the plan's MS x MS solve.  Wave w computes its share
// of every S_j from its fixed points (4w..4w+3, and K + w for w < MS) and adds
// it into the syndrome slots with LDS XOR atomics; after a barrier, wave w
// forms planes (16/WV) w.. of every recovered point with the plan's bit masks
// and writes them into the point's zeroed slot.  A plan with nothing to
// recover (restore: no erased point below K) skips the phase, barriers and
// all.  Against the N = K + K/4 syndrome kernel at MS = 2: 2.4K instead of
// 13.4K syndrome XORs per tile (k = 32), and no M x M runtime walk.
template <int K, int MS> struct SmallSyn;
#ifndef VDS_SYN_RT2
#define VDS_SYN_RT2 1  // (A/B: 0 compiles the RT kernels without the RT2 rows)
#endif
// Dual syndrome tiles (batched restore and regenerate, k = 32;
// SynBatchTile::mode kTileDual):
// the two halves are objects of different plans -- the N-point class's single
// halves, which at a high loss rate are nearly every object (distinct erased
// sets).  The syndrome programs serve both halves as they are; stage 1 places
// each half's survivors at its own points and phase 2 walks each half's
// coefficients under its half mask (regenerate: and stores each half's own
// erased points).  (A/B: 0 compiles the batch kernels
// without it; the host pairs only what the kernels support, api_batch.cpp.)
#ifndef VDS_BATCH_DUAL
#define VDS_BATCH_DUAL 1
#endif
// RT2 (c): the extra rows' columns spread over all eight waves (A/B: 0 = rows
// w and w + 8 whole on wave w).
#ifndef VDS_RT2_SPREAD
#define VDS_RT2_SPREAD 1
#endif
template <int K, int N, int WV, bool REGEN, bool BATCH, bool RT = false, class FillP = NoFill>
__device__ __forceinline__ void restore_syn_body(const SynRestoreArgs &a) {
  constexpr bool FILL = FillP::kFill >= 0;
  constexpr bool kScatter = FILL && FillP::kScatter;
  constexpr bool kOwn = FILL && FillOwn<FillP>::value;
  static_assert(!kOwn || (K == 16 && !REGEN && !BATCH && !RT), "the own-group fill is a k = 16 restore form");
  constexpr bool kSmall = FillP::kSmall;
  constexpr bool kPerm = FillP::kPerm;
  constexpr bool kMulti = FillP::kMulti;
  static_assert(!kMulti || (BATCH && !RT), "MULTI is a batch mode");
  static_assert(!kSmall || (BATCH && !RT && !FILL), "SMALL is a batch mode of its own");
  static_assert(!kPerm || (BATCH && REGEN && !RT && !FILL), "PERM is a batch regenerate mode of its own");
  using S = SynShape<K, N, WV>;
  using P = typename S::P;
  constexpr bool kPrio = S::kPrio;
  static_assert(!RT || BATCH, "RT is a batch mode");
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const BitMasks bm = bit_masks();
  if constexpr (!kPrio && VDS_HALF_PRIO)
    if (wave >= WV / 2) __builtin_amdgcn_s_setprio(1);
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
  // per-tile data: the launch's (uniform), or in batch mode the tile
  // record's (t and wave are uniform, so the s_ld reads are scalar loads)
  auto obj_of = [&](uint32_t t) -> uint32_t { return t / a.tiles_per_obj; };
  auto stripe0_of = [&](uint32_t t) -> uint64_t { return (uint64_t)(t % a.tiles_per_obj) * kTileStripes; };
  auto half_obj = [&](uint32_t t, int h) -> const SynBatchObj & { return a.objs[s_ld(&a.tiles[t].obj[h])]; };
  auto half_s0 = [&](uint32_t t, int h) -> uint64_t { return s_ld(&a.tiles[t].stripe0[h]); };

  // survivor staging: the next tile's loads are issued after the syndrome
  // programs (k = 32: after the interpolation, see kLateLoad) and land while
  // the rest of this tile runs
  u32x4 Q[S::kLoadPer][4];
  auto load = [&](uint32_t t) {
    if constexpr (BATCH) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const SynBatchObj &d = half_obj(t, h);
        const uint64_t st0 = half_s0(t, h);
        // bytes of each survivor from this half's first cell on
        const int64_t valid = (int64_t)s_ld(&d.chunk_len) - (int64_t)(2 * st0);
        const uint8_t *src[S::kLoadPer];
#pragma unroll
        for (int s = 0; s < S::kLoadPer; ++s) src[s] = s_ld(&d.chunks[wave * S::kLoadPer + s]) + 2 * st0 + 16 * lane;
        if (valid >= 2 * (int64_t)kHalfStripes) {
#pragma unroll
          for (int s = 0; s < S::kLoadPer; ++s)
#pragma unroll
            for (int q = 0; q < 2; ++q) Q[s][2 * h + q] = g_ld<4, u32x4>(src[s] + 1024 * q);
        } else {
#pragma unroll
          for (int s = 0; s < S::kLoadPer; ++s)
#pragma unroll
            for (int q = 0; q < 2; ++q) Q[s][2 * h + q] = ld16_guard(src[s] + 1024 * q, valid - 16 * lane - 1024 * q);
        }
      }
    } else {
      const uint32_t ob = obj_of(t);
      const uint64_t st0 = stripe0_of(t);
#pragma unroll
      for (int s = 0; s < S::kLoadPer; ++s) {
        const uint8_t *src = a.chunks[wave * S::kLoadPer + s] + (uint64_t)ob * a.chunk_stride + 2 * st0 + 16 * lane;
#pragma unroll
        for (int q = 0; q < 4; ++q) Q[s][q] = g_ld<4, u32x4>(src + 1024 * q);
      }
    }
  };
  // The next tile's survivors, or zeros past the last tile: both paths define
  // Q, so the values consumed by this tile's stage 1 die there instead of
  // staying live (as loop-carried state) through the programs until the load
  // (k = 32 spilled 203 VGPRs that way: 1.6x / 1.4x the algorithmic traffic).
  const TileRange tr = tile_range(a.total_tiles);
  Stamps st;
  st.init();
  auto prefetch = [&](uint32_t t) {
    if (t < tr.end && (VDS_DIAG_LOADS != 2 || t == tr.first)) {
      st.rt((t - tr.first) / tr.step);
      load(VDS_DIAG_LOADS == 1 ? tr.first : t);
    } else {
#pragma unroll
      for (int s = 0; s < S::kLoadPer; ++s)
#pragma unroll
        for (int q = 0; q < 4; ++q) Q[s][q] = u32x4{0u, 0u, 0u, 0u};
    }
  };
  // k = 32 (one 160 KiB workgroup per CU): the prefetched survivors would be
  // live across the syndrome and stage-B programs, which then spill; they are
  // issued after the interpolation instead and land under the staging and
  // stores (REGEN has no interpolation and keeps the early issue)
  // (batch: the guarded loads and descriptor addresses would not fit beside
  // the programs either)
  // (RT: this wave's slots stay in registers through phase 2; the regenerate
  // branch issues its prefetch there)
  // (the survivor-set kernel at k = 32 with the early issue, after the fill:
  // 90 VGPRs spilled, round 5 tools/jit_dump.py)
  constexpr bool kLateLoad = ((K == 32 || BATCH) && !REGEN) || RT;
  const uint32_t t_step = tr.step;
  prefetch(tr.first);
  // vmcnt counts loads and stores together and retires them in issue order.
  // In the loop, the 16 copy-out stores of a tile are issued after the next
  // tile's survivor loads, so the loads can be waited for with vmcnt(16 + ..)
  // while the stores drain.  The compiler's wait insertion merges the loop's
  // entry and back-edge states by the youngest position of each pending
  // register: at the entry the prefetched loads ARE the youngest ops, so it
  // would wait vmcnt(<16) at the top of every tile -- for the previous tile's
  // stores to complete.  Issuing the same 16 stores here (zeros into this
  // wave's copy-out chunk of its first tile, which that tile's copy-out
  // overwrites, in order, from the same wave) makes both states alike.
  if constexpr (!REGEN && !BATCH) {  // (batch: guarded stores; nothing to mirror)
    if (tr.first < tr.end) {
      const uint32_t t0 = tr.first;
      uint8_t *g0 = a.out + (uint64_t)(t0 / a.tiles_per_obj) * a.out_stride +
                    (uint64_t)(t0 % a.tiles_per_obj) * kTileStripes * (2 * K) + 16384u * wave + 16u * lane;
#pragma unroll
      for (int i = 0; i < 16; ++i) g_st<8>(g0 + 1024 * i, u32x4{0u, 0u, 0u, 0u});
    }
  }
  for (uint32_t tile = tr.first; tile < tr.end; tile += t_step) {
    const uint32_t o = BATCH ? 0u : obj_of(tile);  // (non-batch)
    const uint64_t stripe0 = BATCH ? 0u : stripe0_of(tile);
    const SynBatchPlan *pl = (BATCH && !RT) ? &a.plans[s_ld(&a.tiles[tile].plan)] : nullptr;
    auto erased_of = [&](int m) -> int { return (int)s_ld_u8(BATCH ? pl->erased : a.erased, m); };
    // the LDS point this wave zeroes and (regenerate) stores: an erased point,
    // or RT regenerate's row slot K + wave
    // MULTI: this tile's class (uniform); a PERM tile accumulates in slot K
    const uint32_t cls = kMulti ? s_ld(&pl->cls) : (kPerm ? kClsPerm : kClsSyn);
    const bool perm_tile = kPerm || (kMulti && REGEN && cls == kClsPerm);
    const int my_erased = RT ? K + wave : perm_tile ? K : (wave < S::kM ? erased_of(wave) : 0);
    // RT: this wave's slots, kept for phase 2; the scatter fill: its survivors (VDS_FILL_REGS)
    constexpr bool kFillRegs = kScatter && VDS_FILL_REGS && K == 16;
    constexpr bool kKeepPs = RT || kFillRegs || kOwn;
    Plane16 own;  // (own-group fill: this wave's group's erased point)
    static_assert(!kKeepPs || S::kLoadPer == 4, "four survivors per wave");
    Plane16 Ps[kKeepPs ? S::kLoadPer : 1];

    // RT2 tile (SynBatchRt, ec_internal.hpp): restore at k = 32 through the
    // PERM evaluations of P0 and |E| x |E| runtime products
    constexpr bool kRt2 = VDS_SYN_RT2 && RT && !REGEN && K == 32 && N >= K + 8;
    const bool rt2_tile = kRt2 && s_ld(&a.tiles[tile].mode) == 1u;
    // dual syndrome tile: half 1's plan (half 0's is the tile's)
    constexpr bool kDual = VDS_BATCH_DUAL && BATCH && !RT && !FILL && !kSmall && !kPerm && K == 32;
    const bool dual_tile = kDual && s_ld(&a.tiles[tile].mode) == kTileDual;
    const SynBatchPlan *pl1 = kDual && dual_tile ? &a.plans[s_ld(&half_obj(tile, 1).plan)] : pl;
    // ---- 1. survivors -> planes of their points; waves < M zero one erased point
    syn_prio<1, kPrio>();
    uint64_t bor[2] = {0, 0};  // RT restore: borrowed slots of each half
    {
      if constexpr (kDual) {
        if (dual_tile) {  // every slot zero first: a slot may take its halves from two waves
          static_assert(N % WV == 0, "dual tiles: whole slots per wave");
          const u32x4 z = {0u, 0u, 0u, 0u};
#pragma unroll
          for (int i = 0; i < N / WV; ++i)
#pragma unroll
            for (int g = 0; g < 4; ++g) L.put(4 * ((N / WV) * wave + i) + g, z);
          __syncthreads();
        }
      }
      if (wave < S::kM && (!RT || REGEN) && !FILL && (!perm_tile || wave == 0) && !(kDual && dual_tile)) {
        const u32x4 z = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int g = 0; g < 4; ++g) L.put(4 * my_erased + g, z);
      }
      if constexpr (kScatter) {  // the fill shares meet in these slots (LDS XOR atomics)
        if (wave < FillP::kFill) {
          // (this zero vector lives across the tile loop and is the run-time
          // kernels' 16-byte scratch spill, reloaded once per tile; made per
          // tile instead -- Scratch_Size 0 -- the k = 16 repair measured ~1%
          // slower: 14.40-14.65 vs 14.33-14.36 ms, 512 x 64 MiB, three
          // interleaved rounds, profiles/round4/ablog/zero_spill_ab.log)
          const u32x4 z = {0u, 0u, 0u, 0u};
#pragma unroll
          for (int g = 0; g < 4; ++g) L.put(4 * (int)FillP::kPoint[wave < FillP::kFill ? wave : 0] + g, z);
        }
      }
      if (rt2_tile) {  // RT2: slot K + wave collects r_j of rows j = wave (+ 8) in phase 2
        const u32x4 z = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int g = 0; g < 4; ++g) L.put(4 * (K + wave) + g, z);
      }
      if constexpr (RT && !REGEN) {
        bor[0] = s_ld(&half_obj(tile, 0).rt.borrowed);
        bor[1] = s_ld(&half_obj(tile, 1).rt.borrowed);
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
        if constexpr (RT) {
          const int j = wave * S::kLoadPer + s;
#pragma unroll
          for (int b = 0; b < 16; ++b) Ps[s].p[b] = Pl[b];
          if constexpr (!REGEN) {
            // slot j as point j: a borrowed half keeps zeros there (its
            // erased point's value is added in phase 2)
            const uint32_t keep = (((bor[0] >> j) & 1u) ? 0u : kRtH0) | (((bor[1] >> j) & 1u) ? 0u : kRtH1);
            if (keep != 0xFFFFFFFFu)
#pragma unroll
              for (int b = 0; b < 16; ++b) Pl[b] &= keep;
            syn_put_point(L, j, Pl);
          }
        } else {
          if constexpr (kKeepPs)
#pragma unroll
            for (int b = 0; b < 16; ++b) Ps[s].p[b] = Pl[b];
          const int p0 = (int)s_ld_u8(BATCH ? pl->point : a.point, wave * S::kLoadPer + s);
          const int p1 = kDual && dual_tile ? (int)s_ld_u8(pl1->point, wave * S::kLoadPer + s) : p0;
          if (p0 == p1) {
            syn_put_point(L, p0, Pl);
          } else {  // (dual: each half's bits at its own point)
            Plane16 v;
#pragma unroll
            for (int b = 0; b < 16; ++b) v.p[b] = Pl[b] & kRtH0;
            lds_xor_point(L, p0, v);
#pragma unroll
            for (int b = 0; b < 16; ++b) v.p[b] = Pl[b] & kRtH1;
            lds_xor_point(L, p1, v);
          }
        }
      }
    }
    syn_prio<0, kPrio>();
    st.mark(0);
    __syncthreads();
    st.mark(1);
    // phase-2 bodies, shared by the single-class kernels and MULTI
    auto phase_perm = [&](auto tag) {
      using PF = typename decltype(tag)::type;
      // ---- 2 (PERM). wave w's four points' share of P(K + t'), read through
      // the permutation c -> c ^ t', into slot K (zeroed in stage 1)
      const uint32_t tp = (uint32_t)erased_of(0) ^ (uint32_t)K;
      struct PermIn {
        const SynLds &L;
        uint32_t tp;
        __device__ __forceinline__ u32x4 operator()(int g) const { return L(4 * (int)((uint32_t)(g >> 2) ^ tp) + (g & 3)); }
      } in{L, tp};
      uint32_t acc[16];
      PF::part(wave, in, acc);
      lds_xor_point(L, K, *reinterpret_cast<const Plane16 *>(acc));
      if (!kLateLoad) prefetch(tile + t_step);  // (regenerate: the next tile's survivors now)
    };
    auto phase_small = [&](auto tag) {
      using PF = typename decltype(tag)::type;
      // ---- 2 (SMALL). the MS checks over A, then the MS x MS recovery
      const uint32_t nrec = s_ld(&pl->nrec);
      if (nrec != 0) {
        {
          uint32_t acc[16 * PF::kM];
          PF::part(wave, L, acc);
#pragma unroll
          for (int j = 0; j < PF::kM; ++j)
            lds_xor_point(L, PF::kSynSlot + j, *reinterpret_cast<const Plane16 *>(acc + 16 * j));
        }
        st.mark(2);
        __syncthreads();  // the syndromes are whole
        st.mark(3);
        constexpr int PW = 16 / WV;  // planes of each recovered point formed by this wave
        static_assert(PW == 2 || PW == 4, "plane split: 8 or 4 waves");
        uint32_t sy[PF::kM][16];
#pragma unroll
        for (int j = 0; j < PF::kM; ++j) syn_get_point(L, PF::kSynSlot + j, sy[j]);
#pragma unroll
        for (int m = 0; m < PF::kM; ++m) {
          if ((uint32_t)m >= nrec) break;
          uint32_t o[PW];
#pragma unroll
          for (int i = 0; i < PW; ++i) o[i] = 0u;
#pragma unroll
          for (int j = 0; j < PF::kM; ++j) {
            // this wave's PW masks of R[m][j] (16 bits each, one scalar load)
            uint64_t mk;
            if constexpr (PW == 2)
              mk = s_ld(reinterpret_cast<const uint32_t *>(&pl->small_mask[m][j][PW * wave]));
            else
              mk = s_ld(reinterpret_cast<const uint64_t *>(&pl->small_mask[m][j][PW * wave]));
#pragma unroll
            for (int i = 0; i < PW; ++i)
#pragma unroll
              for (int b = 0; b < 16; ++b) o[i] ^= sy[j][b] & (0u - (uint32_t)((mk >> (16 * i + b)) & 1u));
          }
          // planes PW w .. PW w + PW - 1 of point erased[m]: 4 PW bytes of
          // this lane's 16-byte word of group (PW w) / 4
          const int e = (int)s_ld_u8(pl->erased, m);
          lds_char *dst = L.at(4 * e + (PW * wave) / 4) + 4 * ((PW * wave) % 4);
          if constexpr (PW == 2)
            *(__attribute__((address_space(3))) u32x2 *)dst = u32x2{o[0], o[1]};
          else
            *(lds_v4 *)dst = u32x4{o[0], o[1], o[2], o[3]};
        }
      }
      if (!kLateLoad) prefetch(tile + t_step);  // (regenerate: the next tile's survivors now)
    };
    auto phase_syn = [&]() {
      // ---- 2. wave j holds syndrome S_j whole and scatters its share of every
      // recovered point, c_e[m] += R[m][j] S_j, into the erased slots (zero since
      // stage 1) with LDS XOR atomics: T = x^b S_j walks the coefficient bits
      // once for all M products, and no wave has to gather the syndromes (two
      // barriers and a park/reload of the syndromes fewer than a gather:
      // 1384 -> 1525 GiB/s).  The wave-uniform branches measured faster than
      // their alternatives (512 objects): two separate ifs 1562-1563, masked
      // v_bitop3 with VGPR masks 1520-1534, against 1573-1577 GiB/s.
      {
        Plane16 t;
        P::syndrome(wave, L, t.p);
        if (!kLateLoad) prefetch(tile + t_step);
        st.mark(2);
        // M <= 4: all products before the barrier (their walk overlaps the
        // slower waves' syndromes); M = 8: four at a time after it (eight
        // accumulators would not fit beside the prefetched survivors)
        constexpr int kMC = S::kM <= 4 ? S::kM : 4;
        if constexpr (kMC < S::kM) __syncthreads();  // every wave is done reading the zeroed erased planes
        if constexpr (kDual) {
          if (dual_tile) {
            // each half's bit pair of row m as a mask pair (rolled over the
            // pairs: the masks are run-time values, one body serves them all)
#pragma unroll
            for (int m0 = 0; m0 < S::kM; m0 += kMC) {
              Plane16 ce[kMC];
#pragma unroll
              for (int m = 0; m < kMC; ++m) ce[m] = plane_zero();
              Plane16 tt = t;
#pragma clang loop unroll(disable)
              for (int b = 0; b < 16; b += 2) {
                const Plane16 t1 = plane_mulx(tt);
#pragma unroll
                for (int m = 0; m < kMC; ++m) {
                  const uint32_t sh = 8u * (uint32_t)(b & 3) + (uint32_t)wave;
                  const uint32_t two0 = (s_ld(&pl->solve_sel[m0 + m][b >> 2]) >> sh) & 0x101u;
                  const uint32_t two1 = (s_ld(&pl1->solve_sel[m0 + m][b >> 2]) >> sh) & 0x101u;
                  const uint32_t ma = (two0 & 1u ? kRtH0 : 0u) | (two1 & 1u ? kRtH1 : 0u);
                  const uint32_t mb = (two0 & 0x100u ? kRtH0 : 0u) | (two1 & 0x100u ? kRtH1 : 0u);
                  rec_dual_m(ce[m], tt, t1, ma, mb);
                }
                tt = plane_mulx(t1);
              }
              st.mark(3);
              if constexpr (kMC == S::kM) __syncthreads();
              st.mark(4);
#pragma unroll
              for (int m = 0; m < kMC; ++m) {
                const int e0 = (int)s_ld_u8(pl->erased, m0 + m), e1 = (int)s_ld_u8(pl1->erased, m0 + m);
                if (e0 == e1) {
                  lds_xor_point(L, e0, ce[m]);
                } else {
                  Plane16 v;
#pragma unroll
                  for (int q = 0; q < 16; ++q) v.p[q] = ce[m].p[q] & kRtH0;
                  lds_xor_point(L, e0, v);
#pragma unroll
                  for (int q = 0; q < 16; ++q) v.p[q] = ce[m].p[q] & kRtH1;
                  lds_xor_point(L, e1, v);
                }
              }
            }
            return;
          }
        }
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
              const uint32_t sel = BATCH ? s_ld(&pl->solve_sel[m0 + m][b >> 2]) : a.solve_sel[m0 + m][b >> 2];
              const uint32_t two = (sel >> (8 * (b & 3) + wave)) & 0x101u;
              rec_pair(ce[m], tt, t1, two);
            }
            if (b < 14) tt = plane_mulx(t1);
          }
          st.mark(3);
          if constexpr (kMC == S::kM) __syncthreads();  // every wave is done reading the zeroed erased planes
          st.mark(4);
#pragma unroll
          for (int m = 0; m < kMC; ++m) lds_xor_point(L, erased_of(m0 + m), ce[m]);
        }
      }
    };
    uint32_t rt_rows = 0;  // RT: rows of this tile
    if constexpr (RT) {
      // ---- 2'. row m of each half = sum_j coef[m][j] * slot j: every wave
      // combines its own slots (Ps) for all rows, kMC rows per walk of each
      // slot's x^b chain, and adds its share into the row's LDS point
      // (restore: the half's erased point epoint[m], masked to the half when
      // the two halves' points differ; regenerate: slot K + m)
      const SynBatchObj &d0 = half_obj(tile, 0), &d1 = half_obj(tile, 1);
      rt_rows = s_ld(&a.tiles[tile].nm);
      const uint32_t ne0 = s_ld(&d0.rt.ne), ne1 = s_ld(&d1.rt.ne);
      const uint32_t *cf0 = s_ld(&d0.rt.coef), *cf1 = s_ld(&d1.rt.coef);
      uint32_t vh0, vh1;  // the half masks in VGPRs (for the scatter)
      asm("v_mov_b32 %0, %1" : "=v"(vh0) : "i"(kRtH0));
      asm("v_mov_b32 %0, %1" : "=v"(vh1) : "i"(kRtH1));
      // two rows per walk of each slot's chain, the pairs in a rolled loop
      // (code size: see rec_dual)
      constexpr int kMC = 2;
      if (rt2_tile) {
        if constexpr (kRt2) {
          // ---- 2 (RT2). Rows in groups of 8 (slots K..K+7 collect the
          // group's r_j): (a) this wave's borrowed survivors y_(b_j) into slot
          // K + j - g0 (their half's bits; the first group from the stage-1
          // registers, a second one reloaded from the survivors' bytes, so
          // the registers do not live across the first group), (b) the PERM
          // program's P0(b_j) of both halves (reads through c -> c ^ t'_h,
          // merged by half) into the same slots, barrier, (c) the wave's rows
          // accumulate sum_j c[m][j] r_j (two rows per walk of each r_j's x^b
          // chain; see row[] below); after the last group (d) P(e_m) into the erased
          // slots (zero in their halves until then: the P0 reads need that)
          const uint8_t *ep0 = d0.rt.epoint, *ep1 = d1.rt.epoint, *sp0 = d0.rt.spoint, *sp1 = d1.rt.spoint;
          Plane16 racc[2];
          racc[0] = plane_zero();
          racc[1] = plane_zero();
          // (c)'s rows of this wave: row w over every column and, with E =
          // rows - 8 > 0, extra row 8 + e (e = w E / 8) over the columns j with
          // j mod parts = part -- the extra rows' columns spread over all eight
          // waves, whose partial sums (d) adds into the erased slots.  (Rows w
          // and w + 8 over every column put two rows on waves 0..E-1 and one on
          // the rest: those waves set the barrier's pace, RT stamps r6o.)
          const uint32_t xE = rt_rows > 8u ? rt_rows - 8u : 0u;
          uint32_t xpart = 0, xparts = 1;
          const uint32_t row[2] = {(uint32_t)wave, VDS_RT2_SPREAD ? 8u + (uint32_t)wave * xE / 8u : (uint32_t)wave + 8u};
          const bool has_row[2] = {(uint32_t)wave < rt_rows, VDS_RT2_SPREAD ? xE != 0u : (uint32_t)wave + 8u < rt_rows};
          if (VDS_RT2_SPREAD && xE != 0u) {
            const uint32_t e = row[1] - 8u, w0 = (8u * e + xE - 1u) / xE, w1 = (8u * (e + 1u) + xE - 1u) / xE;
            xpart = (uint32_t)wave - w0;
            xparts = w1 - w0;
          }
          // (a), first group: from the stage-1 registers (dead after this)
#pragma unroll
          for (int sl = 0; sl < S::kLoadPer; ++sl) {
            const int slot = wave * S::kLoadPer + sl;
#pragma unroll
            for (int h = 0; h < 2; ++h)
              if ((bor[h] >> slot) & 1u) {
                const uint32_t j = (uint32_t)__builtin_popcountll(bor[h] & ((1ull << slot) - 1));
                if (j < 8u) {
                  Plane16 v;
#pragma unroll
                  for (int b = 0; b < 16; ++b) v.p[b] = Ps[sl].p[b] & (h ? vh1 : vh0);
                  lds_xor_point(L, K + (int)j, v);
                }
              }
          }
#pragma clang loop unroll(disable)
          for (uint32_t g0 = 0; g0 < rt_rows; g0 += 8) {
            const uint32_t g1 = rt_rows < g0 + 8 ? rt_rows : g0 + 8;
            // (a), a later group: reloaded
            if (g0 > 0) {
              __syncthreads();  // every wave has read the previous group's r_j, (c)
              const u32x4 z = {0u, 0u, 0u, 0u};
#pragma unroll
              for (int g = 0; g < 4; ++g) L.put(4 * (K + wave) + g, z);
              __syncthreads();
#pragma unroll
              for (int sl = 0; sl < S::kLoadPer; ++sl) {
                const int slot = wave * S::kLoadPer + sl;
#pragma unroll
                for (int h = 0; h < 2; ++h)
                  if ((bor[h] >> slot) & 1u) {
                    const uint32_t j = (uint32_t)__builtin_popcountll(bor[h] & ((1ull << slot) - 1));
                    if (j >= g0 && j < g1) {
                      const SynBatchObj &d = half_obj(tile, h);
                      const uint64_t st0 = half_s0(tile, h);
                      const int64_t valid = (int64_t)s_ld(&d.chunk_len) - (int64_t)(2 * st0) - 16 * lane;
                      const uint8_t *src = s_ld(&d.chunks[slot]) + 2 * st0 + 16 * lane;
                      uint32_t W[16];
#pragma unroll
                      for (int q = 0; q < 4; ++q) {
                        const u32x4 v = (q >> 1) == h ? ld16_guard(src + 1024 * (q & 1), valid - 1024 * (q & 1))
                                                      : u32x4{0u, 0u, 0u, 0u};
#pragma unroll
                        for (int d4 = 0; d4 < 4; ++d4) W[4 * q + d4] = v[d4];
                      }
                      transpose16x2(W, bm);
                      Plane16 v;
#pragma unroll
                      for (int b = 0; b < 16; ++b) v.p[b] = W[b ^ 8] & (h ? vh1 : vh0);
                      lds_xor_point(L, K + (int)(j - g0), v);
                    }
                  }
              }
            }
            st.mark(2);  // (RT2 stamps: 2 = (a), 3 = (b), 4 = its barrier, 19 = (c), 5 = (d))
            // (b)
#pragma clang loop unroll(disable)
            for (uint32_t j = g0; j < g1; ++j) {
              const bool h0 = j < ne0, h1 = j < ne1;
              const uint32_t t0 = h0 ? s_ld_u8(sp0, (int)s_ld_u8(ep0, (int)j)) - (uint32_t)K : 0u;
              const uint32_t t1 = h1 ? s_ld_u8(sp1, (int)s_ld_u8(ep1, (int)j)) - (uint32_t)K : 0u;
              // half 0's bits read through t0, half 1's through t1, one
              // v_bitop3 select per word; a half without row j reads the other
              // half's way (its bits are garbage that no coefficient uses)
              struct Rt2In {
                const SynLds &L;
                uint32_t t0, t1, sel;
                __device__ __forceinline__ u32x4 operator()(int g) const {
                  const u32x4 x0 = L(4 * (int)((uint32_t)(g >> 2) ^ t0) + (g & 3));
                  const u32x4 x1 = L(4 * (int)((uint32_t)(g >> 2) ^ t1) + (g & 3));
                  u32x4 v;
#pragma unroll
                  for (int w = 0; w < 4; ++w) v[w] = __builtin_amdgcn_bitop3_b32(sel, x0[w], x1[w], 0xCA);
                  return v;
                }
              } in{L, h0 ? t0 : t1, h1 ? t1 : t0, vh0};
              uint32_t pacc[16];
              PermSyn<K>::part(wave, in, pacc);
              lds_xor_point(L, K + (int)(j - g0), *reinterpret_cast<const Plane16 *>(pacc));
            }
            st.mark(3);
            __syncthreads();  // the group's r_j are whole
            st.mark(4);
            // (c)
            if (has_row[0]) {
#pragma clang loop unroll(disable)
              for (uint32_t j = g0; j < g1; ++j) {
                const bool two_rows = has_row[1] && j % xparts == xpart;
                uint32_t x[2];
#pragma unroll
                for (int mi = 0; mi < 2; ++mi) {
                  const uint32_t m = row[mi];
                  const uint32_t c0 = (m < ne0 && j < ne0) ? s_ld(cf0 + (m * K + j)) : 0u;
                  const uint32_t c1 = (m < ne1 && j < ne1) ? s_ld(cf1 + (m * K + j)) : 0u;
                  x[mi] = c0 | (c1 << 8);
                }
                Plane16 tt;
                syn_get_point(L, K + (int)(j - g0), tt.p);
                if (two_rows) {
                  static_for<0, 8>([&](auto bp) {
                    constexpr int b = 2 * decltype(bp)::value;
                    __builtin_amdgcn_sched_barrier(0);
                    const Plane16 t1 = plane_mulx(tt);
                    rec_dual_x<b>(racc[0], tt, t1, x[0]);
                    rec_dual_x<b>(racc[1], tt, t1, x[1]);
                    if constexpr (b < 14) tt = plane_mulx(t1);
                  });
                } else {
                  static_for<0, 8>([&](auto bp) {
                    constexpr int b = 2 * decltype(bp)::value;
                    __builtin_amdgcn_sched_barrier(0);
                    const Plane16 t1 = plane_mulx(tt);
                    rec_dual_x<b>(racc[0], tt, t1, x[0]);
                    if constexpr (b < 14) tt = plane_mulx(t1);
                  });
                }
              }
            }
            st.mark(19);
          }
          // (d)
#pragma unroll
          for (int mi = 0; mi < 2; ++mi) {
            const uint32_t m = row[mi];
            if (!has_row[mi]) continue;
            const int p0 = m < ne0 ? (int)s_ld_u8(ep0, (int)m) : -1;
            const int p1 = m < ne1 ? (int)s_ld_u8(ep1, (int)m) : -1;
            if (p0 >= 0 && p0 == p1) {
              lds_xor_point(L, p0, racc[mi]);
            } else {
              if (p0 >= 0) {
                Plane16 v;
#pragma unroll
                for (int b = 0; b < 16; ++b) v.p[b] = racc[mi].p[b] & vh0;
                lds_xor_point(L, p0, v);
              }
              if (p1 >= 0) {
                Plane16 v;
#pragma unroll
                for (int b = 0; b < 16; ++b) v.p[b] = racc[mi].p[b] & vh1;
                lds_xor_point(L, p1, v);
              }
            }
          }
        }
      } else
#pragma clang loop unroll(disable)
      for (uint32_t m0 = 0; m0 < rt_rows; m0 += kMC) {
        Plane16 ce[kMC];
#pragma unroll
        for (int m = 0; m < kMC; ++m) ce[m] = plane_zero();
        // this wave's kLoadPer = 4 slot coefficients of each row, both
        // halves: 16 contiguous bytes per (half, row), all issued at once
        static_assert(S::kLoadPer == 4, "one 16-byte scalar load per row and half");
        u32x4 q0[kMC], q1[kMC];
#pragma unroll
        for (int m = 0; m < kMC; ++m) {
          const uint32_t at = (m0 + m) * K + wave * S::kLoadPer;
          q0[m] = m0 + m < ne0 ? s_ld(reinterpret_cast<const u32x4 *>(cf0 + at)) : u32x4{0u, 0u, 0u, 0u};
          q1[m] = m0 + m < ne1 ? s_ld(reinterpret_cast<const u32x4 *>(cf1 + at)) : u32x4{0u, 0u, 0u, 0u};
        }
#pragma unroll
        for (int s = 0; s < S::kLoadPer; ++s) {
          uint32_t x[kMC];  // the (row, slot)'s two coefficients packed for rec_dual_x
#pragma unroll
          for (int m = 0; m < kMC; ++m) x[m] = q0[m][s] | (q1[m][s] << 8);
          // (one slot's chain at a time: interleaving the four independent
          // chains would not fit beside the accumulators)
          __builtin_amdgcn_sched_barrier(0);
          Plane16 tt = Ps[s];
          // (opaque per row pair: the chains do not depend on m0, and hoisted
          // out of the loop all 4 x 16 of them spilled)
#pragma unroll
          for (int i = 0; i < 16; ++i) asm volatile("" : "+v"(tt.p[i]));
          static_for<0, 8>([&](auto bp) {
            constexpr int b = 2 * decltype(bp)::value;
            __builtin_amdgcn_sched_barrier(0);
            const Plane16 t1 = plane_mulx(tt);
#pragma unroll
            for (int m = 0; m < kMC; ++m) rec_dual_x<b>(ce[m], tt, t1, x[m]);
            if constexpr (b < 14) tt = plane_mulx(t1);
          });
        }
#pragma unroll
        for (int m = 0; m < kMC; ++m) {
          const uint32_t r = m0 + m;
          if (r >= rt_rows) break;
          if constexpr (REGEN) {
            lds_xor_point(L, K + (int)r, ce[m]);
          } else {
            const int p0 = r < ne0 ? (int)s_ld_u8(d0.rt.epoint, (int)r) : -1;
            const int p1 = r < ne1 ? (int)s_ld_u8(d1.rt.epoint, (int)r) : -1;
            if (p0 >= 0 && p0 == p1) {
              lds_xor_point(L, p0, ce[m]);
            } else {
              if (p0 >= 0) {
                Plane16 v;
#pragma unroll
                for (int b = 0; b < 16; ++b) v.p[b] = ce[m].p[b] & vh0;
                lds_xor_point(L, p0, v);
              }
              if (p1 >= 0) {
                Plane16 v;
#pragma unroll
                for (int b = 0; b < 16; ++b) v.p[b] = ce[m].p[b] & vh1;
                lds_xor_point(L, p1, v);
              }
            }
          }
        }
      }
    } else if constexpr (kScatter) {
      // ---- 2''. this wave's survivors' share of every erased point below K
      // (its own stage-1 slots in, LDS XOR atomics out; survivors sorted by point)
      if constexpr (kFillRegs)
        syn_scatter_fill<WV, FillP, true, 0>(wave, L, Ps);
      else
        syn_scatter_fill<WV, FillP, false, 0>(wave, L, {});
      if (!kLateLoad) prefetch(tile + t_step);
    } else if constexpr (kOwn) {
      // ---- 2 (own). this wave's group's erased point, kept in registers for S1
      syn_own_fill<WV, FillP, 0>(wave, L, Ps, own);
      if (!kLateLoad) prefetch(tile + t_step);
    } else if constexpr (kPerm) {
      phase_perm(TypeTag<FillP>{});
    } else if constexpr (kSmall) {
      phase_small(TypeTag<FillP>{});
    } else if constexpr (kMulti) {
      if (cls == kClsSmall1) {
        phase_small(TypeTag<SmallSyn<K, 1>>{});
      } else if (cls == kClsSmall2) {
        phase_small(TypeTag<SmallSyn<K, 2>>{});
      } else if (REGEN && cls == kClsPerm) {
        if constexpr (REGEN) phase_perm(TypeTag<PermSyn<K>>{});
      } else {
        phase_syn();
      }
    } else if constexpr (FILL) {
      if (wave < FillP::kFill) {
        uint32_t acc[16];
        FillP::fill(wave, L, acc);
        syn_put_point(L, FillP::kPoint[wave], acc);
      }
      if (!kLateLoad) prefetch(tile + t_step);
    } else {
      phase_syn();
    }  // (phase 2)
    st.mark(5);
    if constexpr (!kOwn) __syncthreads();  // (own-group fill: S1 reads only what stage 1 published)
    st.mark(6);
    if constexpr (REGEN) {
      // ---- 3'. regenerate: the recovered point e_w IS replica e_w's cells
      // (P(e_w) stripe by stripe).  Undo the stage-1 transpose and store it as
      // big-endian cells, one 1 KiB store per wave-instruction; no
      // interpolation (fused "decode + re-encode" of sync_process.cpp:313-335).
      // (RT: row w's slot K + w, for w < the tile's rows)
      if constexpr (RT) prefetch(tile + t_step);
      if constexpr (BATCH) {
        if (RT ? (uint32_t)wave < rt_rows : perm_tile ? wave == 0 : wave < S::kM) {
          uint32_t Pl[16], W[16];
          syn_get_point(L, my_erased, Pl);
          if constexpr (kDual) {
            const int e1 = dual_tile ? (int)s_ld_u8(pl1->erased, wave) : my_erased;
            if (e1 != my_erased) {  // (dual: half 1's row w is its own erased point)
              uint32_t P1[16];
              syn_get_point(L, e1, P1);
#pragma unroll
              for (int b = 0; b < 16; ++b) Pl[b] = __builtin_amdgcn_bitop3_b32(kRtH0, Pl[b], P1[b], 0xCA);
            }
          }
#pragma unroll
          for (int b = 0; b < 16; ++b) W[b ^ 8] = Pl[b];
          transpose16x2(W, bm);  // self-inverse: back to the loaded word layout
          const uint32_t trailer = s_ld(&a.tiles[tile].trailer);
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const SynBatchObj &d = half_obj(tile, h);
            uint8_t *const rg = s_ld(&d.regen[wave]);
            if (rg == nullptr) continue;
            const uint64_t st0 = half_s0(tile, h);
            const uint64_t clen = s_ld(&d.chunk_len);
            // the T cells; the trailer cell is copied from survivor 0 by the
            // object's last half (as restore + re-encode writes it)
            const int64_t valid = (int64_t)clen - 2 - (int64_t)(2 * st0);
            uint8_t *dst = rg + 2 * st0 + 16 * lane;
            if (valid >= 2 * (int64_t)kHalfStripes) {
#pragma unroll
              for (int q = 0; q < 2; ++q)
                g_st<8>(dst + 1024 * q, u32x4{W[8 * h + 4 * q], W[8 * h + 4 * q + 1], W[8 * h + 4 * q + 2],
                                              W[8 * h + 4 * q + 3]});
            } else {
#pragma unroll
              for (int q = 0; q < 2; ++q)
                st16_guard(dst + 1024 * q,
                           u32x4{W[8 * h + 4 * q], W[8 * h + 4 * q + 1], W[8 * h + 4 * q + 2], W[8 * h + 4 * q + 3]},
                           valid - 16 * lane - 1024 * q);
            }
            if (((trailer >> h) & 1u) && lane == 0)
              *(gmem<uint16_t> *)(rg + clen - 2) = *(const gmem<uint16_t> *)(s_ld(&d.chunks[0]) + clen - 2);
          }
        }
        __syncthreads();  // every wave is done with this tile's planes
        continue;
      }
      uint8_t *const rg = wave < S::kM ? a.regen[wave] : nullptr;
      if (rg != nullptr) {
        uint32_t Pl[16], W[16];
        syn_get_point(L, my_erased, Pl);
#pragma unroll
        for (int b = 0; b < 16; ++b) W[b ^ 8] = Pl[b];
        transpose16x2(W, bm);  // self-inverse: back to the loaded word layout
        {
          uint8_t *dst = rg + (uint64_t)o * a.regen_stride + 2 * stripe0 + 16 * lane;
#pragma unroll
          for (int q = 0; q < 4; ++q)
            g_st<8>(dst + 1024 * q, u32x4{W[4 * q], W[4 * q + 1], W[4 * q + 2], W[4 * q + 3]});
        }
      }
      __syncthreads();  // every wave is done with this tile's planes
      continue;
    }
    // ---- 3. fixed interpolation from points 0..K-1, then big-endian stores
    {
      // The RT kernels and the k = 16 survivor-set kernels run the staging
      // and copy-out (the tail) inside each wave's interpolation branch:
      // after the join of the WV branches the cells are a merge of WV
      // definitions, and the k = 32 RT kernel (RT2 rows compiled in) spilled
      // 22 of them per wave to scratch at every tile (176 VGPRs; 24 with the
      // tail in the branches), the k = 16 survivor-set kernel with its fill
      // from registers 113 (0 in the branches, also without the 5-VGPR zero
      // vector spill of before).  The other kernels keep the join: with the
      // tail in the branches the plain k = 32 kernel spilled 1,844 (the late
      // loads beside the staging).
      constexpr bool kTailInWave = RT || kFillRegs || kOwn;
      auto tail = [&](uint32_t (&cells)[16 * S::kCells]) {
      if (kLateLoad && !BATCH) prefetch(tile + t_step);
      // this wave's copy-out: 1024 kChunks bytes at wofs of the tile's output
      // (batch: of its half's object's output, with out_valid bytes of the
      // object still to go from there)
      constexpr int kChunks = 4 * K / WV;  // 1 KiB pieces of the tile (2048 stripes x 2K bytes) each wave writes
      constexpr uint32_t kHalfBytes = kHalfStripes * 2 * K;
      static_assert(kHalfBytes % (1024u * kChunks) == 0, "a wave's copy-out lies in one half");
      // (computed where the stores start: live across the staging, the
      // addresses cost k = 32 SGPR spills)
      struct Target {
        uint8_t *g0;
        int64_t valid;
        bool guard;
      };
      auto target = [&]() -> Target {
        const uint32_t wofs = 1024u * kChunks * wave;
        if constexpr (BATCH) {
          const int h = (int)(wofs / kHalfBytes);
          const SynBatchObj &d = half_obj(tile, h);
          const uint64_t at = half_s0(tile, h) * (2 * K) + (wofs - h * kHalfBytes);
          const int64_t valid = (int64_t)s_ld(&d.out_len) - (int64_t)at;
          return {s_ld(&d.out) + at + 16u * lane, valid, valid < 1024 * kChunks};
        } else {
          return {a.out + (uint64_t)o * a.out_stride + stripe0 * (2 * K) + wofs + 16u * lane,
                  kNoBound, false};
        }
      };
      constexpr int kGroups = S::kCells / 2;  // word groups (2 cells) per wave
      if constexpr (K == 16) {
        // Stage the tile's output in LDS (the planes are dead once every wave
        // has interpolated), stripe-major with 8 bytes of padding after every
        // 8 stripes: stripe st at byte 32 st + 8 (st / 8).  Each lane writes
        // its wave's 8 bytes (cells 4w..4w+3) of a stripe with one
        // ds_write_b64; lane l's stripes 8 l + e are 264 bytes apart, so the
        // 16 lanes of a write group cover all 32 banks once (16-byte padding
        // after every 16 stripes put 4 lanes on each bank of a ds_write_b32:
        // 4-way conflicts).  The copy-out reads 16 contiguous bytes per lane
        // as two 8-byte halves, so every HBM write is a whole 1 KiB
        // wave-instruction (no partial lines).
        static_assert(S::kCells == 4, "one ds_write_b64 = the wave's 4 cells of a stripe");
        static_assert(2048 * 32 + 256 * 8 <= S::kLdsBytes, "staging layout is for 32-byte stripes");
        syn_prio<2, kPrio>();
        uint32_t rows[2][32];
#pragma unroll
        for (int g = 0; g < kGroups; ++g) {
#pragma unroll
          for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int jb = 0; jb < 16; ++jb) rows[g][16 * h + jb] = cells[16 * (2 * g + h) + (jb ^ 8)];
          transpose32(rows[g], bm);
        }
        __syncthreads();
        st.mark(14);
        // slot 8q+e is stripe 8 lane + 512 q + e at byte 264 lane + 16896 q +
        // 32 e: a per-lane base plus a compile-time offset
        lds_char *w0 = L.base + 264u * lane + 8u * wave;
#pragma unroll
        for (int slot = 0; slot < 32; ++slot) {
          const int pi = (slot & 1) ? 16 + (slot >> 1) : (slot >> 1);
          *(__attribute__((address_space(3))) u32x2 *)(w0 + (slot >> 3) * 16896 + (slot & 7) * 32) =
              u32x2{rows[0][pi], rows[1][pi]};
        }
        syn_prio<0, kPrio>();
        st.mark(15);
        if (BATCH) prefetch(tile + t_step);  // (batch: the staged rows are dead; room for the survivors)
        __syncthreads();
        st.mark(16);
        // 16-byte chunk c = 64 (kChunks wave + i) + lane of the tile: stripe c/2,
        // half c%2, at 16 c + 8 (c / 16) = r0 + 1056 i
        const lds_char *r0 = L.base + 1056u * kChunks * wave + 16u * lane + 8u * (lane >> 4);
        const auto [g0, out_valid, guard] = target();
        // (the compiler merges the two halves into one ds_read2_b64: 8 LDS
        // cycles, banks (a/4) mod 32 over 16 lanes, 2-way at lanes l, l + 8;
        // as two volatile ds_read_b64 -- 2 + 2 cycles, conflict-free thanks to
        // the padding -- they measured slower, swz_ab.log)
        auto piece = [&](int i) {
          const lds_char *r = r0 + 1056 * i;
          const u32x2 v0 = *(__attribute__((address_space(3))) const u32x2 *)r;
          const u32x2 v1 = *(__attribute__((address_space(3))) const u32x2 *)(r + 8);
          return u32x4{v0[0], v0[1], v1[0], v1[1]};
        };
        if (!guard) {
#pragma unroll
          for (int i = 0; i < kChunks; ++i) g_st<8>(g0 + 1024 * i, piece(i));
        } else {
#pragma unroll
          for (int i = 0; i < kChunks; ++i) st16_guard(g0 + 1024 * i, piece(i), out_valid - 16 * lane - 1024 * i);
        }
        st.mark(17);
      } else {
        // k = 32: stage as for k = 16 with 64-byte stripes and 8 bytes of
        // padding after every 8 stripes: stripe st, word w at st*64 + (st/8)*8
        // + 4w; the copy-out reads 16 bytes per lane as two 8-byte halves.
        static_assert(K == 32 && S::kCells == 4 && 2048 * 64 + 256 * 8 <= S::kLdsBytes,
                      "staging layout is for 64-byte stripes");
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
        }
        st.mark(15);
        if (BATCH) prefetch(tile + t_step);  // (batch: the staged rows are dead; room for the survivors)
        __syncthreads();
        st.mark(16);
        // 16-byte chunk c = 64 (16 wave + i) + lane of the tile: stripe c/4,
        // quarter c%4, at 64 (c/4) + 8 (c/32) + 16 (c%4) = r0 + 1040 i (one
        // per-lane base, compile-time offsets: no hoisted address per i)
        static_assert(kChunks == 16, "16 KiB of copy-out per wave");
        const lds_char *r0 = L.base + 16640u * wave + 64u * (lane >> 2) + 8u * (lane >> 5) + 16u * (lane & 3);
        const auto [g0, out_valid, guard] = target();
        auto piece = [&](int i) {
          const lds_char *r = r0 + 1040 * i;
          const u32x2 v0 = *(__attribute__((address_space(3))) const u32x2 *)r;
          const u32x2 v1 = *(__attribute__((address_space(3))) const u32x2 *)(r + 8);
          return u32x4{v0[0], v0[1], v1[0], v1[1]};
        };
        if (!guard) {
#pragma unroll
          for (int i = 0; i < 16; ++i) g_st<8>(g0 + 1024 * i, piece(i));
        } else {
#pragma unroll
          for (int i = 0; i < 16; ++i) st16_guard(g0 + 1024 * i, piece(i), out_valid - 16 * lane - 1024 * i);
        }
        st.mark(17);
      }
      };
      if constexpr (VDS_GM2 != 0 && kOwn) {
        syn_interp_gm2<K, N, WV, 0, decltype(tail) &, FillP>(wave, L, st, tail, &own);
      } else if constexpr (VDS_GM2 != 0 && kTailInWave) {
        syn_interp_gm2<K, N, WV, 0>(wave, L, st, tail);
      } else if constexpr (VDS_GM2 != 0) {
        uint32_t cells[16 * S::kCells];
        syn_interp_gm2<K, N, WV, 0>(wave, L, st, [&](uint32_t (&c)[16 * S::kCells]) {
#pragma unroll
          for (int i = 0; i < 16 * S::kCells; ++i) cells[i] = c[i];
        });
        tail(cells);
      } else {
        uint32_t cells[16 * S::kCells];
        syn_interp_gm<K, N, WV, 0>(wave, L, cells, st);
        tail(cells);
      }
    }
    __syncthreads();
    st.mark(18);
  }
  st.flush(blockIdx.x * WV + wave, lane);
}

}  // namespace vds_ec
