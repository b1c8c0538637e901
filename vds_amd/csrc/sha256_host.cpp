// sha256_host.cpp -- SHA-256 of one message on the calling CPU thread.
//
// upload_data hashes the whole body once per 64 KiB upload
// (server_api.cpp:16, hash::signature(sha256, ...), kernel/vds_crypto/
// hash.cpp:84-100).  That is ONE Merkle-Damgard chain of 1024 dependent
// compressions: on the GPU it runs in a single lane, latency-bound at ~3 us a
// block (3.2 ms per call, round 5 tools/dropin_loop), while the replica names
// (64 independent chains per upload) stay on the device (sha256.hip).  So
// vds_ec_save_temp16_host hashes the body here, on the caller's thread, while
// the device encodes and hashes the replicas.
//
// Two implementations, picked once: the x86 SHA extensions (sha256rnds2 /
// sha256msg1 / sha256msg2, present on the GPU box's EPYC and on this
// container's Xeon) and a portable one (FIPS 180-4 section 6.2), the only
// one on other hosts.  A -DVDS_HOST_SHA_PORTABLE=1 build forces the latter
// (tests/test_sha256_host.py compiles this file both ways and compares each
// with hashlib).
#ifndef VDS_HOST_SHA_PORTABLE
#define VDS_HOST_SHA_PORTABLE 0
#endif
#if defined(__x86_64__) || defined(__i386__)
#define VDS_HOST_SHA_X86 1
#include <cpuid.h>
#include <immintrin.h>
#else
#define VDS_HOST_SHA_X86 0
#endif

#include <cstdint>
#include <cstring>

#include "vds_ec.h"

namespace vds_ec {
namespace {

constexpr uint32_t kK[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
constexpr uint32_t kH0[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                             0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};

inline uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

// Portable compression of `nblocks` 64-byte blocks.
void blocks_portable(uint32_t h[8], const uint8_t *p, size_t nblocks) {
  for (size_t blk = 0; blk < nblocks; ++blk, p += 64) {
    uint32_t w[64];
    for (int t = 0; t < 16; ++t)
      w[t] = (uint32_t)p[4 * t] << 24 | (uint32_t)p[4 * t + 1] << 16 | (uint32_t)p[4 * t + 2] << 8 | p[4 * t + 3];
    for (int t = 16; t < 64; ++t) {
      const uint32_t s0 = rotr(w[t - 15], 7) ^ rotr(w[t - 15], 18) ^ (w[t - 15] >> 3);
      const uint32_t s1 = rotr(w[t - 2], 17) ^ rotr(w[t - 2], 19) ^ (w[t - 2] >> 10);
      w[t] = w[t - 16] + s0 + w[t - 7] + s1;
    }
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
    for (int t = 0; t < 64; ++t) {
      const uint32_t t1 = hh + (rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25)) + ((e & f) ^ (~e & g)) + kK[t] + w[t];
      const uint32_t t2 = (rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
      hh = g;
      g = f;
      f = e;
      e = d + t1;
      d = c;
      c = b;
      b = a;
      a = t1 + t2;
    }
    h[0] += a, h[1] += b, h[2] += c, h[3] += d, h[4] += e, h[5] += f, h[6] += g, h[7] += hh;
  }
}

#if VDS_HOST_SHA_X86
// The SHA extensions: the state lives as ABEF / CDGH in two xmm registers,
// four rounds per pair of sha256rnds2, the schedule by sha256msg1/msg2.
__attribute__((target("sha,sse4.1,ssse3"))) void blocks_shani(uint32_t h[8], const uint8_t *p, size_t nblocks) {
  const __m128i bswap = _mm_set_epi64x(0x0c0d0e0f08090a0bll, 0x0405060700010203ll);
  __m128i tmp = _mm_loadu_si128((const __m128i *)&h[0]);     // DCBA
  __m128i st1 = _mm_loadu_si128((const __m128i *)&h[4]);     // HGFE
  tmp = _mm_shuffle_epi32(tmp, 0xB1);                        // CDAB
  st1 = _mm_shuffle_epi32(st1, 0x1B);                        // EFGH
  __m128i st0 = _mm_alignr_epi8(tmp, st1, 8);                // ABEF
  st1 = _mm_blend_epi16(st1, tmp, 0xF0);                     // CDGH
  for (size_t blk = 0; blk < nblocks; ++blk, p += 64) {
    const __m128i a0 = st0, c0 = st1;
    __m128i m[4];
    for (int i = 0; i < 4; ++i) m[i] = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i *)(p + 16 * i)), bswap);
    for (int r = 0; r < 16; ++r) {  // rounds 4r .. 4r + 3
      __m128i msg = _mm_add_epi32(m[r & 3], _mm_loadu_si128((const __m128i *)&kK[4 * r]));
      st1 = _mm_sha256rnds2_epu32(st1, st0, msg);
      msg = _mm_shuffle_epi32(msg, 0x0E);
      st0 = _mm_sha256rnds2_epu32(st0, st1, msg);
      if (r < 12) {
        // W[4(r+4) ..] = msg2(msg1(W[4r..], W[4r+4..]) + W[4r+9 .. 4r+12], W[4r+12..])
        __m128i x = _mm_sha256msg1_epu32(m[r & 3], m[(r + 1) & 3]);
        x = _mm_add_epi32(x, _mm_alignr_epi8(m[(r + 3) & 3], m[(r + 2) & 3], 4));
        m[r & 3] = _mm_sha256msg2_epu32(x, m[(r + 3) & 3]);
      }
    }
    st0 = _mm_add_epi32(st0, a0);
    st1 = _mm_add_epi32(st1, c0);
  }
  tmp = _mm_shuffle_epi32(st0, 0x1B);                        // FEBA
  st1 = _mm_shuffle_epi32(st1, 0xB1);                        // DCHG
  st0 = _mm_blend_epi16(tmp, st1, 0xF0);                     // DCBA
  st1 = _mm_alignr_epi8(st1, tmp, 8);                        // HGFE
  _mm_storeu_si128((__m128i *)&h[0], st0);
  _mm_storeu_si128((__m128i *)&h[4], st1);
}

bool have_shani() {
  unsigned a, b, c, d;
  if (!__get_cpuid_count(7, 0, &a, &b, &c, &d)) return false;
  const bool sha = (b >> 29) & 1u;
  if (!__get_cpuid(1, &a, &b, &c, &d)) return false;
  const bool sse41 = (c >> 19) & 1u, ssse3 = (c >> 9) & 1u;
  return sha && sse41 && ssse3;
}
#endif  // VDS_HOST_SHA_X86

using BlocksFn = void (*)(uint32_t *, const uint8_t *, size_t);
BlocksFn blocks_fn() {
  static const BlocksFn f = [] {
#if VDS_HOST_SHA_X86 && !VDS_HOST_SHA_PORTABLE
    if (have_shani()) return (BlocksFn)blocks_shani;
#endif
    return (BlocksFn)blocks_portable;
  }();
  return f;
}

}  // namespace

void sha256_host(const uint8_t *data, uint64_t len, uint8_t out[32]) {
  uint32_t h[8];
  std::memcpy(h, kH0, sizeof h);
  const BlocksFn f = blocks_fn();
  const uint64_t full = len / 64;
  if (full) f(h, data, full);
  uint8_t tail[128] = {};
  const size_t rem = (size_t)(len - 64 * full);
  if (rem) std::memcpy(tail, data + 64 * full, rem);
  tail[rem] = 0x80;
  const size_t tb = rem + 9 <= 64 ? 64 : 128;
  const uint64_t bits = len * 8;
  for (int i = 0; i < 8; ++i) tail[tb - 1 - i] = (uint8_t)(bits >> (8 * i));
  f(h, tail, tb / 64);
  for (int i = 0; i < 8; ++i) {
    out[4 * i] = (uint8_t)(h[i] >> 24);
    out[4 * i + 1] = (uint8_t)(h[i] >> 16);
    out[4 * i + 2] = (uint8_t)(h[i] >> 8);
    out[4 * i + 3] = (uint8_t)h[i];
  }
}

}  // namespace vds_ec

extern "C" int vds_ec_sha256_host(const uint8_t *data, uint64_t len, uint8_t *digest) {
  if (!digest || (len && !data)) return VDS_EC_EINVAL;
  vds_ec::sha256_host(data, len, digest);
  return VDS_EC_OK;
}
