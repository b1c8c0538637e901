// gf.h -- drop-in for lboss75/vds kernel/vds_data/gf.h (gf.h:15-297).
//
// Same public API (gf<m>, gf_math<uint8_t>, gf_math<uint16_t>) so tests and
// callers compile unchanged.  gf<m> multiplies bit-serially over a 64-bit
// accumulator; the gf_math log/antilog tables are produced by the MI355X
// codec library (vds_ec_gf8_tables / vds_ec_gf16_tables, include/vds_ec.h),
// which owns the field definition used by the GPU kernels.
#ifndef __VDS_DATA_GF_H_
#define __VDS_DATA_GF_H_

#include <cassert>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>

#include "vds_ec.h"

namespace vds {

namespace gf_detail {
// Low bits of the reduction polynomials (gf.h:100-126): the bytes are
// little-endian, the x^m term is implicit except for m = 3, where the
// reference's mask keeps it inside the byte.
template <unsigned m> struct poly;
template <> struct poly<3> { static constexpr uint64_t low = 0x0B; };
template <> struct poly<8> { static constexpr uint64_t low = 0x1D; };
template <> struct poly<16> { static constexpr uint64_t low = 0x100B; };
template <> struct poly<32> { static constexpr uint64_t low = 0x00400007; };
}  // namespace gf_detail

template <unsigned int m>
class gf {
 public:
  static constexpr size_t ArraySize = (m + 7) / 8;
  typedef uint8_t DataType[(m + 7) / 8];

  gf(const gf &left, const gf &right) {
    for (size_t i = 0; i < ArraySize; ++i) data_[i] = left.data_[i] ^ right.data_[i];
  }
  gf(const DataType &data) { std::memcpy(data_, data, ArraySize); }

  gf operator+(const gf &right) const { return gf(*this, right); }

  gf operator*(const gf &right) const {
    const uint64_t width = ArraySize >= 8 ? ~0ull : ((1ull << (8 * ArraySize)) - 1);
    const uint64_t top = 1ull << (m - 1);
    uint64_t a = pack(data_), b = pack(right.data_), p = 0;
    for (unsigned i = 0; i < m; ++i, b >>= 1) {
      if (b & 1) p ^= a;
      const bool carry = (a & top) != 0;
      a = (a << 1) & width;
      if (carry) a ^= gf_detail::poly<m>::low;
    }
    DataType out;
    for (size_t i = 0; i < ArraySize; ++i) out[i] = uint8_t(p >> (8 * i));
    return gf(out);
  }

  bool operator==(const gf &right) const { return 0 == std::memcmp(data_, right.data_, ArraySize); }
  const DataType &data() const { return data_; }

  std::string toString() const {
    std::string r;
    char b[4];
    for (size_t i = 0; i < ArraySize; ++i) {
      std::snprintf(b, sizeof(b), "%02x", data_[i]);
      r += b;
    }
    return r;
  }

 private:
  DataType data_;
  static uint64_t pack(const DataType &d) {
    uint64_t v = 0;
    for (size_t i = 0; i < ArraySize; ++i) v |= uint64_t(d[i]) << (8 * i);
    return v;
  }
};

template <typename value_type>
class gf_math;

// gf.h:131-191: log/antilog over x^8+x^4+x^3+x^2+1, generator 2.
template <>
class gf_math<uint8_t> {
 public:
  gf_math() { vds_ec_gf8_tables(value2log_, log2value_); }
  uint8_t mul(uint8_t a, uint8_t b) const {
    return (a == 0 || b == 0) ? 0 : log2value_[(value2log_[a] + value2log_[b]) % 255];
  }
  uint8_t div(uint8_t a, uint8_t b) const {
    if (a == 0 || b == 0) return 0;  // div(x, 0) = 0 as in the reference
    return log2value_[(value2log_[a] + 255 - value2log_[b]) % 255];
  }
  uint8_t add(uint8_t a, uint8_t b) const { return a ^ b; }
  uint8_t sub(uint8_t a, uint8_t b) const { return a ^ b; }

 private:
  uint8_t value2log_[0x100];
  uint8_t log2value_[0x100];
};

// gf.h:193-253: the production field, x^16+x^12+x^3+x+1, generator 2.
template <>
class gf_math<uint16_t> {
 public:
  gf_math() { vds_ec_gf16_tables(value2log_, log2value_); }
  uint16_t mul(uint16_t a, uint16_t b) const {
    return (a == 0 || b == 0) ? 0 : log2value_[(uint32_t(value2log_[a]) + value2log_[b]) % 0xFFFF];
  }
  uint16_t div(uint16_t a, uint16_t b) const {
    if (a == 0 || b == 0) return 0;
    return log2value_[(uint32_t(value2log_[a]) + 0xFFFF - value2log_[b]) % 0xFFFF];
  }
  uint16_t add(uint16_t a, uint16_t b) const { return a ^ b; }
  uint16_t sub(uint16_t a, uint16_t b) const { return a ^ b; }

 private:
  uint16_t value2log_[0x10000];
  uint16_t log2value_[0x10000];
};

}  // namespace vds

#endif  // __VDS_DATA_GF_H_
