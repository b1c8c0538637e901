// bitslice.hpp -- bit-sliced GF(2^16) arithmetic on 32-stripe "planes".
//
// A Plane16 holds one GF(2^16) value for each of 32 independent stripes:
// word p[b] carries bit b of the 32 values (bit position = stripe slot).
// Field addition is a per-word XOR; multiplication by x is a rotation of the
// word indices plus three XORs (x^16 = x^12 + x^3 + x + 1, gf.h:114-119);
// multiplication by a compile-time constant C is Horner over the bits of C.
// Because every index is a compile-time constant after unrolling, the
// "rotation" is register renaming and costs nothing.
//
// The transposes convert between this layout and the byte layout of the
// reference (big-endian 16-bit cells, binary_serialize.cpp:18-22).
#pragma once

#include "gf_common.hpp"

#if defined(__HIPCC__) || defined(__HIP__)
#define VDS_INLINE __host__ __device__ __forceinline__
#else
#define VDS_INLINE inline
#endif

namespace vds_ec {

struct Plane16 {
  uint32_t p[16];
};

VDS_INLINE Plane16 plane_xor(const Plane16 &a, const Plane16 &b) {
  Plane16 r;
#pragma unroll
  for (int i = 0; i < 16; ++i) r.p[i] = a.p[i] ^ b.p[i];
  return r;
}

VDS_INLINE uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);  // v_bitop3_b32 (gfx950)
#else
  return a ^ b ^ c;
#endif
}

VDS_INLINE Plane16 plane_xor3(const Plane16 &a, const Plane16 &b, const Plane16 &c) {
  Plane16 r;
#pragma unroll
  for (int i = 0; i < 16; ++i) r.p[i] = xor3(a.p[i], b.p[i], c.p[i]);
  return r;
}

// acc ^= a & m  (m all-ones or zero; one v_bitop3_b32 per plane on gfx950)
VDS_INLINE void plane_xor_masked(Plane16 &acc, const Plane16 &a, uint32_t m) {
#pragma unroll
  for (int i = 0; i < 16; ++i) {
#if defined(__HIP_DEVICE_COMPILE__)
    // truth table over S0=0xF0, S1=0xCC, S2=0xAA: S0 ^ (S1 & S2) = 0x78
    acc.p[i] = __builtin_amdgcn_bitop3_b32(acc.p[i], a.p[i], m, 0x78);
#else
    acc.p[i] ^= a.p[i] & m;
#endif
  }
}

VDS_INLINE Plane16 plane_zero() {
  Plane16 r;
#pragma unroll
  for (int i = 0; i < 16; ++i) r.p[i] = 0;
  return r;
}

// a * x  (mod x^16 + x^12 + x^3 + x + 1)
VDS_INLINE Plane16 plane_mulx(const Plane16 &a) {
  Plane16 r;
  const uint32_t t = a.p[15];
  r.p[0] = t;
  r.p[1] = a.p[0] ^ t;
  r.p[2] = a.p[1];
  r.p[3] = a.p[2] ^ t;
#pragma unroll
  for (int i = 4; i < 12; ++i) r.p[i] = a.p[i - 1];
  r.p[12] = a.p[11] ^ t;
  r.p[13] = a.p[12];
  r.p[14] = a.p[13];
  r.p[15] = a.p[14];
  return r;
}

// Horner over the bits of C below bit B+1: u <- u*x (+ a if bit set).
template <uint32_t C, int B>
struct PlaneMulC {
  VDS_INLINE static Plane16 run(const Plane16 &u, const Plane16 &a) {
    Plane16 v = plane_mulx(u);
    if constexpr (((C >> B) & 1u) != 0) v = plane_xor(v, a);
    return PlaneMulC<C, B - 1>::run(v, a);
  }
};
template <uint32_t C>
struct PlaneMulC<C, -1> {
  VDS_INLINE static Plane16 run(const Plane16 &u, const Plane16 &) { return u; }
};

// a * C for a compile-time field constant C (< 2^16).
template <uint32_t C>
VDS_INLINE Plane16 plane_mulc(const Plane16 &a) {
  if constexpr (C == 0) {
    return plane_zero();
  } else {
    constexpr int top = poly_degree(C);
    return PlaneMulC<C, top - 1>::run(a, a);
  }
}

// Horner step of the encode: acc * C + x.
template <uint32_t C>
VDS_INLINE Plane16 plane_horner(const Plane16 &acc, const Plane16 &x) {
  if constexpr (C == 0) {
    return x;
  } else {
    constexpr int top = poly_degree(C);
    if constexpr (top == 0) {
      return plane_xor(acc, x);
    } else {
      // Bits top-1 .. 1 of C (== bits top-2 .. 0 of C>>1), then fuse the last
      // "+acc" with "+x" so the compiler can form v_xor3_b32.
      const Plane16 v = PlaneMulC<(C >> 1), top - 2>::run(acc, acc);
      const Plane16 w = plane_mulx(v);
      if constexpr ((C & 1u) != 0)
        return plane_xor3(w, acc, x);
      else
        return plane_xor(w, x);
    }
  }
}

// Multiplication by a constant C as a 16x16 bit matrix, stored as operand
// lists: output plane i of (acc * C) is the XOR of acc planes j[i][0..n[i]),
// i.e. of the planes j with bit i of C * x^j set.
struct MulRowLists {
  int8_t j[16][16];
  int8_t n[16];
};

constexpr MulRowLists mul_row_lists(uint32_t C) {
  MulRowLists L{};
  for (int i = 0; i < 16; ++i) L.n[i] = 0;
  for (int jj = 0; jj < 16; ++jj) {
    const uint32_t v = gf16_mul(C, 1u << jj);
    for (int i = 0; i < 16; ++i)
      if ((v >> i) & 1u) L.j[i][L.n[i]++] = (int8_t)jj;
  }
  return L;
}

// VALU instructions of one row-form Horner step acc * C + x: every output
// plane folds its n[i] acc planes and the x plane two at a time (xor3).
constexpr int row_horner_cost(uint32_t C) {
  if (C == 0) return 0;
  const MulRowLists L = mul_row_lists(C);
  int c = 0;
  for (int i = 0; i < 16; ++i) c += (L.n[i] + 1) / 2;
  return c;
}

template <uint32_t C>
struct RowHorner {
  static constexpr MulRowLists L = mul_row_lists(C);
};

template <uint32_t C, int I, int Q>
VDS_INLINE uint32_t fold_row(uint32_t v, const Plane16 &acc) {
  constexpr MulRowLists L = RowHorner<C>::L;
  if constexpr (Q + 1 < L.n[I])
    return fold_row<C, I, Q + 2>(xor3(v, acc.p[L.j[I][Q]], acc.p[L.j[I][Q + 1]]), acc);
  else if constexpr (Q < L.n[I])
    return v ^ acc.p[L.j[I][Q]];
  else
    return v;
}

// (an integer sequence of our own: the kernels also compile under hiprtc,
// which has no standard library headers)
template <class T, T... I>
struct IntSeq {};
#if defined(__clang__)
template <int N>
using IntSeqN = __make_integer_seq<IntSeq, int, N>;
#else  // (g++: the host build of tests/cpp/test_bitslice.cpp)
template <int N>
using IntSeqN = IntSeq<int, __integer_pack(N)...>;
#endif

template <uint32_t C, int... I>
VDS_INLINE Plane16 row_horner_impl(const Plane16 &acc, const Plane16 &x, IntSeq<int, I...>) {
  Plane16 out;
  ((out.p[I] = fold_row<C, (int)I, 0>(x.p[I], acc)), ...);
  return out;
}

// Horner step acc * C + x in row form: each output plane is one XOR of its
// matrix row's acc planes and the x plane, folded into v_bitop3_b32 xor3s.
// Unlike the x-shift chain (plane_horner) there is no plane renaming, so a
// rolled loop needs no register copies, and the feedback XORs of the
// reduction merge into the row sums (~27% fewer VALU ops
// summed over replicas 0..19).
template <uint32_t C>
VDS_INLINE Plane16 plane_horner_rows(const Plane16 &acc, const Plane16 &x) {
  if constexpr (C == 0)
    return x;
  else
    return row_horner_impl<C>(acc, x, IntSeqN<16>{});
}

// Multiply by a wave-uniform runtime constant c (< 2^16): Horner over all 16
// bit positions, branch-free (the add is masked by the bit of c).
VDS_INLINE Plane16 plane_mul_rt(const Plane16 &a, uint32_t c) {
  Plane16 u = plane_zero();
#pragma unroll
  for (int b = 15; b >= 0; --b) {
    u = plane_mulx(u);
    plane_xor_masked(u, a, 0u - ((c >> b) & 1u));
  }
  return u;
}

// acc[s] ^= c[s] * y for NS runtime constants, sharing the y * x^b chain:
// y*c = sum_b c_b (y x^b).  Cost: 45 XOR + 16*16*NS masked XOR.  The
// coefficients are wave-uniform (SGPRs); each bit's all-ones/zero mask is
// moved to a VGPR first: a v_bitop3_b32 reading an SGPR issues at ~0.6 of
// the all-VGPR rate (profiles/round1/valu_op_rates.txt), one v_mov per mask
// buys sixteen full-rate bitop3s.
template <int NS>
VDS_INLINE void plane_mac_rt(Plane16 (&acc)[NS], Plane16 y, const uint32_t (&c)[NS]) {
#pragma unroll
  for (int b = 0; b < 16; ++b) {
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      uint32_t m = 0u - ((c[s] >> b) & 1u);
#if defined(__HIP_DEVICE_COMPILE__) && !defined(VDS_MAC_SGPR_MASK)
      asm("v_mov_b32 %0, %1" : "=v"(m) : "s"(m));
#endif
      plane_xor_masked(acc[s], y, m);
    }
    if (b < 15) y = plane_mulx(y);
  }
}

// ---------------------------------------------------------------- transposes

// One butterfly round of the bit transpose for a power-of-two shift J < 8:
// swaps (row k, bits with J set) <-> (row k+J, bits with J clear).
// Masks of the j = 4, 2, 1 transpose rounds.  On the device they live in
// VGPRs: a v_bitop3_b32 whose operands are all VGPRs issues at the rate of a
// 2-input XOR, while one reading an SGPR (or v_bfi_b32) issues at ~0.6 of it
// (tools/ubench/valu_latency.hip).  The asm is not volatile, so the movs are
// CSE'd and hoisted out of the tile loops.
struct BitMasks {
  uint32_t m4, m2, m1;
};

VDS_INLINE BitMasks bit_masks() {
  BitMasks m;
#if defined(__HIP_DEVICE_COMPILE__)
  asm("v_mov_b32 %0, %1" : "=v"(m.m4) : "i"(0x0F0F0F0F));
  asm("v_mov_b32 %0, %1" : "=v"(m.m2) : "i"(0x33333333));
  asm("v_mov_b32 %0, %1" : "=v"(m.m1) : "i"(0x55555555));
#else
  m.m4 = 0x0F0F0F0Fu;
  m.m2 = 0x33333333u;
  m.m1 = 0x55555555u;
#endif
  return m;
}

// (m & a) | (~m & b): truth table over S0=0xF0 (m), S1=0xCC (a), S2=0xAA (b)
VDS_INLINE uint32_t bit_select(uint32_t m, uint32_t a, uint32_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_bitop3_b32(m, a, b, 0xCA);
#else
  return (m & a) | (~m & b);
#endif
}

VDS_INLINE uint32_t rotl32(uint32_t x, int s) {  // s in 1..31
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_alignbit(x, x, 32 - s);
#else
  return (x << s) | (x >> (32 - s));
#endif
}

// The sub-byte rounds J = 4, 2, 1 of a bit transpose, on words kept
// rotated: each pair (k, k + J) costs one rotate and two selects instead of
// two shifts and two selects.  Before round J both words of a pair are
// rotated left by the same r (a multiple of 2J, so the masks, of period 2J,
// are unchanged); with bs = rotl(b, J),
//   new_k   = (a & m) | ((b << J) & ~m)  kept rotated by r:     sel(m, a, bs)
//   new_k+J = ((a >> J) & m) | (b & ~m)  kept rotated by r + J: sel(m, bs, a)
// (the bits a rotate brings in where a shift brings zeros fall under the
// other operand's mask).  After rounds 4, 2, 1 word q is rotated by q & 7;
// rotate_back undoes that.  A transpose16x2 takes 102 instructions instead
// of 112, a transpose32 236 instead of 256.
// (ROT = false: the plain shift form, two shifts and two selects per pair;
// the k = 32 encode keeps it -- 9.45-9.51 vs 9.72-9.78 ms with the rotated
// one, while the k = 16 repair gained 4%: profiles/round5/ab_transpose.log)
template <int J, int ROWS, bool ROT, typename Arr>
VDS_INLINE void transpose_round(Arr &A, const BitMasks &bm) {
  const uint32_t m = (J == 4) ? bm.m4 : (J == 2) ? bm.m2 : bm.m1;
#pragma unroll
  for (int k0 = 0; k0 < ROWS; k0 += 2 * J)
#pragma unroll
    for (int k = k0; k < k0 + J; ++k) {
      if constexpr (ROT) {
        const uint32_t a = A[k], bs = rotl32(A[k + J], J);
        A[k] = bit_select(m, a, bs);
        A[k + J] = bit_select(m, bs, a);
      } else {
        const uint32_t a = A[k], b = A[k + J];
        A[k] = bit_select(m, a, b << J);
        A[k + J] = bit_select(m, a >> J, b);
      }
    }
}
template <int ROWS, bool ROT, typename Arr>
VDS_INLINE void rotate_back(Arr &A) {
  if constexpr (ROT)
#pragma unroll
    for (int q = 0; q < ROWS; ++q)
      if (q & 7) A[q] = rotl32(A[q], 32 - (q & 7));
}

// 32x32 bit transpose in place: afterwards A[p] bit i == before A[i] bit p.
template <bool ROT = true>
VDS_INLINE void transpose32(uint32_t (&A)[32], const BitMasks &bm = bit_masks()) {
  // j = 16: swap (row k, bits 16..31) <-> (row k+16, bits 0..15)
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const uint32_t a = A[k], b = A[k + 16];
#if defined(__HIP_DEVICE_COMPILE__)
    A[k] = __builtin_amdgcn_perm(b, a, 0x05040100u);
    A[k + 16] = __builtin_amdgcn_perm(b, a, 0x07060302u);
#else
    A[k] = (a & 0x0000FFFFu) | (b << 16);
    A[k + 16] = (a >> 16) | (b & 0xFFFF0000u);
#endif
  }
  // j = 8
#pragma unroll
  for (int k0 = 0; k0 < 32; k0 += 16)
#pragma unroll
    for (int k = k0; k < k0 + 8; ++k) {
      const uint32_t a = A[k], b = A[k + 8];
#if defined(__HIP_DEVICE_COMPILE__)
      A[k] = __builtin_amdgcn_perm(b, a, 0x06020400u);
      A[k + 8] = __builtin_amdgcn_perm(b, a, 0x07030501u);
#else
      A[k] = (a & 0x00FF00FFu) | ((b << 8) & 0xFF00FF00u);
      A[k + 8] = ((a >> 8) & 0x00FF00FFu) | (b & 0xFF00FF00u);
#endif
    }
  // j = 4, 2, 1 : bitfield inserts
  transpose_round<4, 32, ROT>(A, bm);
  transpose_round<2, 32, ROT>(A, bm);
  transpose_round<1, 32, ROT>(A, bm);
  rotate_back<32, ROT>(A);
}

// Two independent 16x16 bit transposes held in the low / high halves of 16
// words: afterwards A[q] bit (16h + j) == before A[j] bit (16h + q).
template <bool ROT = true>
VDS_INLINE void transpose16x2(uint32_t (&A)[16], const BitMasks &bm = bit_masks()) {
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const uint32_t a = A[k], b = A[k + 8];
#if defined(__HIP_DEVICE_COMPILE__)
    A[k] = __builtin_amdgcn_perm(b, a, 0x06020400u);
    A[k + 8] = __builtin_amdgcn_perm(b, a, 0x07030501u);
#else
    A[k] = (a & 0x00FF00FFu) | ((b << 8) & 0xFF00FF00u);
    A[k + 8] = ((a >> 8) & 0x00FF00FFu) | (b & 0xFF00FF00u);
#endif
  }
  transpose_round<4, 16, ROT>(A, bm);
  transpose_round<2, 16, ROT>(A, bm);
  transpose_round<1, 16, ROT>(A, bm);
  rotate_back<16, ROT>(A);
}

}  // namespace vds_ec
