// ref_gf_harness.cpp -- TEST INFRASTRUCTURE ONLY.
//
// Driver that exercises the REFERENCE's own kernel/vds_data/gf.h, compiled
// unmodified from /root/reference (include path set by oracle/Makefile; the
// header is never copied into this repository).  gf.h is self-contained
// (<unordered_map>, <string>, <assert.h>, <cstring>), so no stand-in header
// is needed.  chunk.h is NOT built: it includes vds_core/stream.h ->
// async_task.h -> <experimental/coroutine>, which this image lacks.
//
// Output: a binary dump that tests/test_oracle_pin.py compares against the
// CPU restatement in oracle/vds_oracle.c.
//
//   gf_ref gf3  <file>   8x8 gf<3> products               (gf_tests.cpp:9-38)
//   gf_ref gf8  <file>   all 256x256 pairs: gf_math<uint8_t>::mul/div, gf<8> *
//   gf_ref gf16 <file>   structured + 2^20 random pairs:  gf_math<uint16_t>
//                        mul/div and gf<16> bit-serial *
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "gf.h"

namespace {

uint64_t splitmix(uint64_t &state) {
  uint64_t z = (state += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

template <typename T>
void put(FILE *f, const std::vector<T> &v) {
  uint32_t n = (uint32_t)v.size();
  fwrite(&n, sizeof(n), 1, f);
  fwrite(v.data(), sizeof(T), v.size(), f);
}

}  // namespace

int main(int argc, char **argv) {
  if (argc != 3) {
    fprintf(stderr, "usage: %s gf3|gf8|gf16 <out>\n", argv[0]);
    return 2;
  }
  FILE *f = fopen(argv[2], "wb");
  if (!f) return 1;
  const std::string mode = argv[1];

  if (mode == "gf3") {
    std::vector<uint8_t> a, b, p;
    for (uint8_t i = 0; i < 8; ++i)
      for (uint8_t j = 0; j < 8; ++j) {
        uint8_t l[1] = {i}, r[1] = {j};
        a.push_back(i);
        b.push_back(j);
        p.push_back((vds::gf<3>(l) * vds::gf<3>(r)).data()[0]);
      }
    put(f, a); put(f, b); put(f, p);
  } else if (mode == "gf8") {
    static vds::gf_math<uint8_t> math;
    std::vector<uint8_t> a, b, mul, div, bits;
    for (unsigned i = 0; i < 256; ++i)
      for (unsigned j = 0; j < 256; ++j) {
        uint8_t l[1] = {(uint8_t)i}, r[1] = {(uint8_t)j};
        a.push_back((uint8_t)i);
        b.push_back((uint8_t)j);
        mul.push_back(math.mul((uint8_t)i, (uint8_t)j));
        div.push_back(math.div((uint8_t)i, (uint8_t)j));
        bits.push_back((vds::gf<8>(l) * vds::gf<8>(r)).data()[0]);
      }
    put(f, a); put(f, b); put(f, mul); put(f, div); put(f, bits);
  } else if (mode == "gf16") {
    // gf_math<uint16_t> holds 2 x 128 KiB; keep it off the stack.
    static vds::gf_math<uint16_t> math;
    std::vector<uint16_t> a, b, mul, div, bits;
    const uint16_t fixed[] = {0, 1, 2, 3, 5, 19, 39, 63, 0x100B, 0x8000, 0x1234, 0xFFFF};
    auto add = [&](uint16_t x, uint16_t y) {
      uint8_t l[2] = {(uint8_t)(x & 0xFF), (uint8_t)(x >> 8)};
      uint8_t r[2] = {(uint8_t)(y & 0xFF), (uint8_t)(y >> 8)};
      auto g = vds::gf<16>(l) * vds::gf<16>(r);
      a.push_back(x);
      b.push_back(y);
      mul.push_back(math.mul(x, y));
      div.push_back(math.div(x, y));
      bits.push_back((uint16_t)(g.data()[0] | (g.data()[1] << 8)));
    };
    for (unsigned x = 0; x < 65536; ++x)
      for (uint16_t y : fixed) {
        add((uint16_t)x, y);
        add(y, (uint16_t)x);
      }
    uint64_t st = 0x7664730000000000ull;
    for (unsigned i = 0; i < (1u << 20); ++i) {
      uint64_t z = splitmix(st);
      add((uint16_t)z, (uint16_t)(z >> 16));
    }
    put(f, a); put(f, b); put(f, mul); put(f, div); put(f, bits);
  } else {
    fclose(f);
    return 2;
  }
  fclose(f);
  return 0;
}
