// sha256.hip -- SHA-256 (FIPS 180-4) of replica buffers on the device.
//
// The reference names every replica by the SHA-256 of its bytes:
// save_temp and save_data (dht_network_client.cpp:79, :593) call
// hash::signature(hash::sha256(), replica), i.e. OpenSSL EVP_sha256
// (kernel/vds_crypto/hash.cpp:21-29, 91-101).  After a GPU encode the replica
// bytes are already in HBM, so hashing them there replaces n CPU passes over
// the replicas.
//
// SHA-256 is a sequential chain over 64-byte blocks, so one lane hashes one
// message; a launch hashes many messages (every replica of every object of a
// batch) side by side.  Replicas are 2 T + 2 bytes long, so a message may
// start at any byte: each lane reads aligned dwords and assembles the
// big-endian message words with one v_perm_b32 each.
#include <hip/hip_runtime.h>

#include "ec_internal.hpp"

namespace vds_ec {

namespace {

constexpr uint32_t kSha256K[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};

constexpr uint32_t kSha256H0[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                                   0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};

__device__ __forceinline__ uint32_t rotr(uint32_t x, uint32_t n) { return __builtin_amdgcn_alignbit(x, x, n); }
// three-input XOR as one v_bitop3_b32 (truth table 0x96)
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
// Ch(e, f, g) = e ? f : g and Maj(a, b, c) as one v_bitop3_b32 each (0xCA, 0xE8);
// left to the compiler they came out as two to three ops per round.
__device__ __forceinline__ uint32_t ch(uint32_t e, uint32_t f, uint32_t g) {
  return __builtin_amdgcn_bitop3_b32(e, f, g, 0xCA);
}
__device__ __forceinline__ uint32_t maj(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);
}

// One compression of the 16 big-endian message words w (w is the schedule ring).
__device__ __forceinline__ void sha256_compress(uint32_t (&h)[8], uint32_t (&w)[16]) {
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
#pragma unroll
  for (int i = 0; i < 64; ++i) {
    if (i >= 16) {  // W_i = s1(W_{i-2}) + W_{i-7} + s0(W_{i-15}) + W_{i-16}
      const uint32_t w15 = w[(i + 1) & 15], w2 = w[(i + 14) & 15];
      const uint32_t s0 = xor3(rotr(w15, 7), rotr(w15, 18), w15 >> 3);
      const uint32_t s1 = xor3(rotr(w2, 17), rotr(w2, 19), w2 >> 10);
      w[i & 15] += s0 + w[(i + 9) & 15] + s1;
    }
    const uint32_t t1 = hh + xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25)) + ch(e, f, g) + kSha256K[i] + w[i & 15];
    const uint32_t t2 = xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22)) + maj(a, b, c);
    hh = g;
    g = f;
    f = e;
    e = d + t1;
    d = c;
    c = b;
    b = a;
    a = t1 + t2;
  }
  h[0] += a;
  h[1] += b;
  h[2] += c;
  h[3] += d;
  h[4] += e;
  h[5] += f;
  h[6] += g;
  h[7] += hh;
}

// Message j = base + j * stride (len bytes) -> digest at digests + 32 j.
// ALIGNED (base and stride multiples of 16, e.g. the replica layouts of the
// batched encodes): whole blocks as four 16-byte loads per lane, the next
// block's loads issued before this block's 64 rounds (each lane walks its
// own message: without the prefetch every block waited out a full memory
// latency).  Otherwise aligned dwords and one v_perm_b32 per word.
template <bool ALIGNED>
__global__ __launch_bounds__(64) void k_sha256(const uint8_t *base, uint64_t len, uint64_t stride, uint32_t count,
                                               uint8_t *digests) {
  const uint32_t j = blockIdx.x * 64u + threadIdx.x;
  if (j >= count) return;
  const uint8_t *m = base + (uint64_t)j * stride;
  uint32_t h[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) h[i] = kSha256H0[i];

  // Whole blocks from aligned dwords: block b needs dwords 16 b .. 16 b + 16
  // of p (17 with the misalignment), all inside the message while
  // 64 b + 68 <= len + sh.  (ALIGNED: sh = 0 and 64 b + 64 <= len.)
  const uint32_t sh = ALIGNED ? 0u : (uint32_t)((uintptr_t)m & 3u);
  const uint32_t *p = reinterpret_cast<const uint32_t *>(m - sh);
  // big-endian word of message bytes 4i..4i+3 = bytes sh+3, sh+2, sh+1, sh of (p[i+1]:p[i])
  const uint32_t sel = (sh + 3u) | ((sh + 2u) << 8) | ((sh + 1u) << 16) | (sh << 24);
  uint64_t nfast;
  if constexpr (ALIGNED) {
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 *q = reinterpret_cast<const u32x4 *>(m);
    nfast = len / 64;
    u32x4 nx[4];
    if (nfast) {
#pragma unroll
      for (int i = 0; i < 4; ++i) nx[i] = q[i];
    }
    for (uint64_t blk = 0; blk < nfast; ++blk) {
      uint32_t w[16];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int t = 0; t < 4; ++t) w[4 * i + t] = __builtin_amdgcn_perm(0u, nx[i][t], 0x00010203u);
      if (blk + 1 < nfast) {
#pragma unroll
        for (int i = 0; i < 4; ++i) nx[i] = q[4 * (blk + 1) + i];
      }
      sha256_compress(h, w);
    }
  } else {
    nfast = len + sh >= 68 ? (len + sh - 68) / 64 + 1 : 0;
    uint32_t carry = nfast ? p[0] : 0u;
    for (uint64_t blk = 0; blk < nfast; ++blk) {
      const uint32_t *q = p + 16 * blk;
      uint32_t raw[17];
      raw[0] = carry;
#pragma unroll
      for (int i = 1; i <= 16; ++i) raw[i] = q[i];
      carry = raw[16];
      uint32_t w[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) w[i] = __builtin_amdgcn_perm(raw[i + 1], raw[i], sel);
      sha256_compress(h, w);
    }
  }

  // The rest (< 132 bytes) the same way, from the aligned dwords that hold at
  // least one message byte (never past the dword of the last byte), then
  // bytes >= rem masked off, 0x80 after them, and the 64-bit big-endian bit
  // length in the last block.
  const uint64_t rem = len - 64 * nfast;
  const uint32_t nb = (uint32_t)((rem + 9 + 63) / 64);
  const uint64_t bits = len * 8;
  const uint64_t lim = len + sh;  // aligned byte offsets < lim hold message bytes
  for (uint32_t blk = 0; blk < nb; ++blk) {
    const uint64_t q0 = 16 * (nfast + blk);
    uint32_t raw[17];
#pragma unroll
    for (int i = 0; i <= 16; ++i) raw[i] = 4 * (q0 + i) < lim ? p[q0 + i] : 0u;
    uint32_t w[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int64_t c = (int64_t)rem - (int64_t)(64 * blk + 4 * i);  // message bytes left at this word
      uint32_t v = __builtin_amdgcn_perm(raw[i + 1], raw[i], sel);
      if (c < 4) v = c <= 0 ? 0u : v & ~(0xFFFFFFFFu >> (8 * c));
      if (c >= 0 && c < 4) v |= 0x80u << (24 - 8 * c);
      w[i] = v;
    }
    if (blk + 1 == nb) {
      w[14] = (uint32_t)(bits >> 32);
      w[15] = (uint32_t)bits;
    }
    sha256_compress(h, w);
  }
  uint8_t *dg = digests + 32ull * j;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int t = 0; t < 4; ++t) dg[4 * i + t] = (uint8_t)(h[i] >> (24 - 8 * t));
}

}  // namespace

hipError_t launch_sha256(const uint8_t *base, uint64_t len, uint64_t stride, uint32_t count, uint8_t *digests,
                         hipStream_t s) {
  if (count == 0) return hipSuccess;
  if ((((uintptr_t)base | stride) & 15u) == 0)
    hipLaunchKernelGGL(k_sha256<true>, dim3((count + 63) / 64), dim3(64), 0, s, base, len, stride, count, digests);
  else
    hipLaunchKernelGGL(k_sha256<false>, dim3((count + 63) / 64), dim3(64), 0, s, base, len, stride, count, digests);
  return hipGetLastError();
}

}  // namespace vds_ec
