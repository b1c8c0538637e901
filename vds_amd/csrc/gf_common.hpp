// gf_common.hpp -- GF(2^16) / GF(2^8) arithmetic of lboss75/vds kernel/vds_data,
// re-derived as carry-less polynomial arithmetic (no log tables) so that the
// same constexpr code runs on the host, on the device and at compile time.
//
// Field definitions (reference gf.h):
//   GF(2^16): p(x) = x^16 + x^12 + x^3 + x + 1  (gf.h:114-119, {0x0B,0x10})
//   GF(2^8) : p(x) = x^8 + x^4 + x^3 + x^2 + 1  (gf.h:107-112, 0x1D)
// x (=2) is primitive in both (order 65535 / 255), so the reference's
// log/antilog multiply (gf.h:156-165, 218-227) IS polynomial multiplication
// mod p(x); every kernel here relies on that identity and the tests pin it
// against the compiled reference gf.h.
#pragma once

#ifndef __HIPCC_RTC__  // (hiprtc: the restore kernels compiled at run time, vds_ec_jit.cpp)
#include <cstddef>
#endif
#include <cstdint>

#if defined(__HIPCC__) || defined(__HIP__)
#define VDS_HD __host__ __device__
#else
#define VDS_HD
#endif

namespace vds_ec {

constexpr uint32_t kPoly16 = 0x1100Bu;
constexpr uint32_t kPoly8 = 0x11Du;

// Carry-less product of two polynomials of degree < 16.
VDS_HD constexpr uint32_t clmul16(uint32_t a, uint32_t b) {
  uint32_t p = 0;
  for (int i = 0; i < 16; ++i)
    if ((b >> i) & 1u) p ^= a << i;
  return p;
}

// Reduce a polynomial of degree <= 30 modulo kPoly16 (x^16 = x^12+x^3+x+1).
VDS_HD constexpr uint32_t reduce16(uint32_t p) {
  for (int r = 0; r < 4; ++r) {
    const uint32_t h = p >> 16;
    p = (p & 0xFFFFu) ^ h ^ (h << 1) ^ (h << 3) ^ (h << 12);
  }
  return p;
}

VDS_HD constexpr uint16_t gf16_mul(uint32_t a, uint32_t b) { return (uint16_t)reduce16(clmul16(a, b)); }

VDS_HD constexpr uint8_t gf8_mul(uint32_t a, uint32_t b) {
  uint32_t p = 0;
  for (int i = 0; i < 8; ++i)
    if ((b >> i) & 1u) p ^= a << i;
  for (int r = 0; r < 3; ++r) {
    const uint32_t h = p >> 8;
    p = (p & 0xFFu) ^ h ^ (h << 2) ^ (h << 3) ^ (h << 4);
  }
  return (uint8_t)p;
}

VDS_HD constexpr uint16_t gf16_pow(uint32_t a, uint32_t e) {
  uint32_t r = 1;
  uint32_t b = a;
  while (e) {
    if (e & 1u) r = gf16_mul(r, b);
    b = gf16_mul(b, b);
    e >>= 1;
  }
  return (uint16_t)r;
}

VDS_HD constexpr uint8_t gf8_pow(uint32_t a, uint32_t e) {
  uint32_t r = 1;
  uint32_t b = a;
  while (e) {
    if (e & 1u) r = gf8_mul(r, b);
    b = gf8_mul(b, b);
    e >>= 1;
  }
  return (uint8_t)r;
}

// Multiplicative inverse; inv(0) = 0 (matches the reference's div(x,0)=0).
VDS_HD constexpr uint16_t gf16_inv(uint32_t a) { return a ? gf16_pow(a, 65534u) : 0; }

// a^2: squaring is GF(2)-linear -- spread bit i to bit 2i, then reduce.
VDS_HD constexpr uint16_t gf16_sqr(uint32_t a) {
  uint32_t x = a & 0xFFFFu;
  x = (x | (x << 8)) & 0x00FF00FFu;
  x = (x | (x << 4)) & 0x0F0F0F0Fu;
  x = (x | (x << 2)) & 0x33333333u;
  x = (x | (x << 1)) & 0x55555555u;
  return (uint16_t)reduce16(x);
}

// a^(2^n): n squarings.
VDS_HD constexpr uint16_t gf16_sqr_n(uint32_t a, int n) {
  for (int i = 0; i < n; ++i) a = gf16_sqr(a);
  return (uint16_t)a;
}

// Inverse by Itoh-Tsujii: a^-1 = (a^(2^15 - 1))^2, with b_m = a^(2^m - 1)
// built along the chain 1, 2, 3, 6, 12, 15 (b_{m+n} = b_m^(2^n) b_n): five
// multiplies and fifteen (linear, cheap) squarings instead of the 30
// multiplies of gf16_pow.  inv(0) = 0.
VDS_HD constexpr uint16_t gf16_inv_it(uint32_t a) {
  const uint32_t b1 = a;
  const uint32_t b2 = gf16_mul(gf16_sqr(b1), b1);
  const uint32_t b3 = gf16_mul(gf16_sqr(b2), b1);
  const uint32_t b6 = gf16_mul(gf16_sqr_n(b3, 3), b3);
  const uint32_t b12 = gf16_mul(gf16_sqr_n(b6, 6), b6);
  const uint32_t b15 = gf16_mul(gf16_sqr_n(b12, 3), b3);
  return gf16_sqr(b15);
}
VDS_HD constexpr uint8_t gf8_inv(uint32_t a) { return a ? gf8_pow(a, 254u) : 0; }

// chunk.h:183-194: multipliers[j] = n^j, with n^0 = 1 even for n = 0.
VDS_HD constexpr uint16_t gf16_vandermonde(uint32_t node, uint32_t j) {
  return j == 0 ? (uint16_t)1 : gf16_pow(node, j);
}

// Degree of a nonzero polynomial (index of the top set bit).
VDS_HD constexpr int poly_degree(uint32_t c) {
  int d = -1;
  for (int i = 0; i < 32; ++i)
    if ((c >> i) & 1u) d = i;
  return d;
}

}  // namespace vds_ec
