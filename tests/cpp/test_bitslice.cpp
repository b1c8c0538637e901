// Host unit test of the bit-slicing primitives in vds_amd/csrc/bitslice.hpp.
// Built and run by tests/test_host_primitives.py (g++, no GPU).
#include <cstdio>
#include <cstdlib>
#include "../../vds_amd/csrc/bitslice.hpp"

using namespace vds_ec;
static uint64_t st = 0x1234567ull;
static uint32_t rnd() { st ^= st << 13; st ^= st >> 7; st ^= st << 17; return (uint32_t)st; }
static int fails = 0;
#define CHECK(c) do { if (!(c)) { if (fails++ < 10) printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c); } } while (0)

static Plane16 to_planes(const uint16_t v[32]) {
  Plane16 r = plane_zero();
  for (int b = 0; b < 16; ++b) for (int i = 0; i < 32; ++i) r.p[b] |= ((v[i] >> b) & 1u) << i;
  return r;
}
static void from_planes(const Plane16 &a, uint16_t v[32]) {
  for (int i = 0; i < 32; ++i) { v[i] = 0; for (int b = 0; b < 16; ++b) v[i] |= ((a.p[b] >> i) & 1u) << b; }
}
template <uint32_t C> static void check_const() {
  uint16_t v[32], w[32], acc[32];
  for (int i = 0; i < 32; ++i) { v[i] = rnd(); acc[i] = rnd(); }
  from_planes(plane_mulc<C>(to_planes(v)), w);
  for (int i = 0; i < 32; ++i) CHECK(w[i] == gf16_mul(v[i], C));
  from_planes(plane_horner<C>(to_planes(acc), to_planes(v)), w);
  for (int i = 0; i < 32; ++i) CHECK(w[i] == (uint16_t)(gf16_mul(acc[i], C) ^ v[i]));
  from_planes(plane_mul_rt(to_planes(v), C), w);
  for (int i = 0; i < 32; ++i) CHECK(w[i] == gf16_mul(v[i], C));
}
int main() {
  // field identities against the survey KATs
  CHECK(gf16_mul(2, 0x8000) == 0x100B);
  CHECK(gf16_mul(0x1234, 0x5678) == 0x6324);
  CHECK(gf16_mul(1, gf16_inv(3)) == 0xF006);
  CHECK(gf8_mul(0x53, 0xCA) == 0x8F);
  CHECK(gf8_mul(2, 0x80) == 0x1D);
  for (int t = 0; t < 1000; ++t) { uint32_t a = rnd() & 0xFFFF; if (a) CHECK(gf16_mul(a, gf16_inv(a)) == 1); }
  // the RT coefficient kernel's Itoh-Tsujii inverse and linear squaring, every element
  for (uint32_t a = 0; a < 65536; ++a) {
    CHECK(gf16_inv_it(a) == gf16_inv(a));
    CHECK(gf16_sqr(a) == gf16_mul(a, a));
  }
  // transpose32
  uint32_t A[32], B[32];
  for (int i = 0; i < 32; ++i) A[i] = B[i] = rnd();
  transpose32(A);
  for (int p = 0; p < 32; ++p) for (int i = 0; i < 32; ++i) CHECK(((A[p] >> i) & 1u) == ((B[i] >> p) & 1u));
  // transpose16x2
  uint32_t C16[16], D16[16];
  for (int i = 0; i < 16; ++i) C16[i] = D16[i] = rnd();
  transpose16x2(C16);
  for (int q = 0; q < 16; ++q) for (int h = 0; h < 2; ++h) for (int j = 0; j < 16; ++j)
    CHECK(((C16[q] >> (16 * h + j)) & 1u) == ((D16[j] >> (16 * h + q)) & 1u));
  check_const<0>(); check_const<1>(); check_const<2>(); check_const<3>(); check_const<7>();
  check_const<19>(); check_const<39>(); check_const<63>(); check_const<0x105>(); check_const<0x8000>();
  check_const<0xFFFF>(); check_const<0x1234>();
  printf("%s (%d failures)\n", fails ? "FAILED" : "OK", fails);
  return fails ? 1 : 0;
}
