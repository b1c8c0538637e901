// gen_restore.cpp -- offline generator of the compile-time XOR programs used by
// the erasure-pattern-independent restore kernel k_restore_syn<K,N>.
//
// For the code of vds kernel/vds_data (replica r = P(r), deg P < K, points
// 0..N-1, chunk.h:245-281) the restore of an object from any K of the N
// replicas is split into two FIXED GF(2^16)-linear maps plus an M x M runtime
// solve (M = N - K):
//
//   1. syndromes  S_j = sum_a v_a a^j c_a,  j < M, over all N points, with the
//      erased c_a = 0 (v_a = 1 / prod_{b != a} (a - b): the dual of the
//      evaluation code, so the sum over a full codeword vanishes);
//   2. runtime:   c_E = W_E^{-1} S  (W_E[j][e] = v_e e^j, inverted on the host);
//   3. interpolation from the fixed points F = {0..K-1}:  x = V_F^{-1} c_F.
//
// Maps 1 and 3 are compile-time constant bit-matrices; this tool turns each
// wave's share of them into a short straight-line XOR program with Paar's
// greedy common-subexpression elimination and prints it as C++ for
// vds_amd/csrc/generated/restore_K_N.inc.  Points are processed in blocks so
// the live temps of one block fit the register file.
//
//   gen_restore K N WAVES syndrome_block interp_block [half_block [half_split]] > restore_K_N_wW.inc
//   gen_restore small K MS block > smallsyn_K_MS.inc   (see main_small)
//   gen_restore perm K block > permsyn_K.inc            (see main_perm)
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "../../include/vds_ec.h"
#include "../../vds_amd/csrc/gf_common.hpp"
#include "../../vds_amd/csrc/xorprog.hpp"

using namespace vds_ec;

using xorgen::all_bitrows;
using xorgen::row_range;

// The generator prints what xorprog.hpp emits (the same code the library's
// run-time compiler uses).
static xorgen::InputMap g_im;
static size_t emit_program(const char *name, const std::vector<std::vector<int>> &rows, int C,
                           const std::vector<int> &rowsel, int pb) {
  std::string s;
  const size_t ops = xorgen::emit_program(s, name, rows, C, rowsel, pb, g_im);
  std::fputs(s.c_str(), stdout);
  std::fprintf(stderr, "  %s: %zu ops\n", name, ops);
  return ops;
}

// ------------------------------------------------------------------
// Two-level additive-FFT interpolation from the points 0..K-1 (K = 2^m; wave
// W owns slots 4W..4W+3), k_restore_syn's gm2 stages:
//   S1 (local to wave W's four slots): level 1, the pairs (2i, 2i+1) of U =
//      span{1, x, ..}: q1_i = v_2i + v_2i+1 -> slot 2i+1, q0_i = v_2i + 2i q1_i
//      -> slot 2i; P(X) = P0(X^2+X) + X P1(X^2+X), P0 / P1 take q0 / q1 on D =
//      s(2i) (index i <-> sum_t bit_t(i) d_t, d_t = s(x^(t+1)), s = X^2+X).
//      Level 2 on Q_par (par 0: P0, 1: P1), normalised by delta = d_0 (R(Y) =
//      Q(delta Y) on the points ptR(h) = sum_t bit_t(h) d_t / delta, which
//      contain 1): the pairs (2j, 2j+1): r1_j = v + v', r0_j = v + ptR(2j) r1_j
//      -> slots 4j + par (r0) and 4j + 2 + par (r1).  Both levels touch only
//      slots 4W..4W+3 (j = W, i = 2W, 2W+1).
//   S2: family f (slots 4j + f: f = par for R0 of Q_par, par + 2 for R1) is
//      interpolated directly on its K/4 points s(ptR(2j)); coefficient c ->
//      slot 4c + f.  K = 16: one wave per family, in place; K = 32: two, each
//      computing half the bit planes of every coefficient.
//   S3: Q_par coefficient i = delta^-i (sum_c [C(c, i-c) odd] R0_c + [C(c,
//      i-1-c) odd] R1_c) (the expansion R(Y) = R0(Y^2+Y) + Y R1(Y^2+Y), then
//      the twist) -> slot (K/2) par + i: the layout stage C reads.
static bool binom_odd(int n, int r) { return r >= 0 && r <= n && (r & ~n) == 0; }

// acc[0..16) *= c in place (a Paar program on the 16 x 16 bit matrix of c)
static size_t emit_twist(const char *name, uint32_t c) {
  std::vector<uint32_t> M = {c};
  const auto rows = all_bitrows(M, 1, 1);
  const xorgen::Block B = xorgen::make_block(xorgen::paar(16, rows), 0);
  std::string s;
  xorgen::appendf(s, "  __device__ __forceinline__ static void %s(uint32_t (&acc)[16]) {\n", name);
  for (int g = 0; g < 4; ++g)
    xorgen::appendf(s, "    const u32x4 g0_%d = {acc[%d], acc[%d], acc[%d], acc[%d]};\n", g, 4 * g, 4 * g + 1, 4 * g + 2,
                    4 * g + 3);
  const size_t ops = xorgen::emit_compute(s, B, 0, true);
  xorgen::appendf(s, "  }\n");
  std::fputs(s.c_str(), stdout);
  return ops;
}

static size_t emit_gm2(int K, int waves) {
  const int H = K / 2, F = K / 4;  // Q size, family size
  int m = 0;
  while ((1 << m) < K) ++m;
  std::vector<uint32_t> d(m - 1), nb(m - 1);
  for (int t = 0; t < m - 1; ++t) d[t] = gf16_mul(1u << (t + 1), 1u << (t + 1)) ^ (1u << (t + 1));
  const uint32_t delta = d[0], dinv = gf16_inv(delta);
  for (int t = 0; t < m - 1; ++t) nb[t] = gf16_mul(d[t], dinv);
  auto ptR = [&](int h) {
    uint32_t p = 0;
    for (int t = 0; t < m - 1; ++t)
      if ((h >> t) & 1) p ^= nb[t];
    return p;
  };
  size_t total = 0;
  std::printf("  // two-level interpolation (gm2; see tools/xorgen/gen_restore.cpp emit_gm2)\n");
  std::printf("  static constexpr bool kGm2 = true;\n");
  // S1: wave W, slots 4W..4W+3 -> the same slots
  for (int w = 0; w < waves; ++w) {
    std::vector<uint32_t> M(16, 0);  // 4 x 4: out slot 4W+o from in slot 4W+i
    // level 1 on pairs (4W, 4W+1), (4W+2, 4W+3): q0 -> even, q1 -> odd slot
    uint32_t L1[4][4] = {};
    for (int q = 0; q < 2; ++q) {
      const uint32_t g = 2 * (2 * w + q);
      L1[2 * q][2 * q] = 1u ^ g, L1[2 * q][2 * q + 1] = g;  // q0 = (1 + g) v0 + g v1
      L1[2 * q + 1][2 * q] = 1u, L1[2 * q + 1][2 * q + 1] = 1u;
    }
    // level 2: for par, v = slot 4W + par (index 2W of Q_par), v' = slot 4W + 2 + par
    uint32_t L2[4][4] = {};
    const uint32_t g2 = ptR(2 * w);
    for (int par = 0; par < 2; ++par) {
      L2[par][par] = 1u ^ g2, L2[par][par + 2] = g2;
      L2[par + 2][par] = 1u, L2[par + 2][par + 2] = 1u;
    }
    for (int o = 0; o < 4; ++o)
      for (int i = 0; i < 4; ++i) {
        uint32_t acc = 0;
        for (int k = 0; k < 4; ++k) acc ^= gf16_mul(L2[o][k], L1[k][i]);
        M[o * 4 + i] = acc;
      }
    const auto rows = all_bitrows(M, 4, 4);
    xorgen::InputMap im;
    for (int i = 0; i < 4; ++i) im.map.push_back(4 * w + i);
    char name[32];
    std::snprintf(name, sizeof name, "gm_s1_%d", w);
    std::string s;
    total += xorgen::emit_program(s, name, rows, 4, row_range(0, 64), 2, im);
    std::fputs(s.c_str(), stdout);
  }
  // S2: family interpolation on the points s(ptR(2j))
  std::vector<uint16_t> dp(F), dinvm((size_t)F * F);
  for (int j = 0; j < F; ++j) {
    const uint32_t p = ptR(2 * j);
    dp[j] = (uint16_t)(gf16_mul(p, p) ^ p);
  }
  if (vds_ec_inverse16(F, dp.data(), dinvm.data()) != VDS_EC_OK) std::exit(1);
  const std::vector<uint32_t> M2(dinvm.begin(), dinvm.end());
  const auto rows2 = all_bitrows(M2, F, F);
  const int wpf = waves / 4;  // waves per family
  for (int w = 0; w < waves; ++w) {
    const int f = w / wpf, c0 = 4 * (w % wpf);
    xorgen::InputMap im;
    for (int j = 0; j < F; ++j) im.map.push_back(4 * j + f);
    std::vector<int> rowsel;
    if (wpf == 1) {  // K = 16: the wave's family whole
      for (int c = c0; c < c0 + 4; ++c)
        for (int b = 0; b < 16; ++b) rowsel.push_back(16 * c + b);
    } else {
      // K = 32: the two waves of a family split the planes (h = w % 2: planes
      // 8h..8h+7 of all 8 coefficients, acc[8c + b - 8h]); split by
      // coefficients instead, the halves' programs cost 889 and 1069 XORs
      // (every 4 + 4 split: at least 1060), split by planes 999 and 994
      const int h = w % wpf;
      for (int c = 0; c < F; ++c)
        for (int b = 8 * h; b < 8 * h + 8; ++b) rowsel.push_back(16 * c + b);
    }
    char name[32];
    std::snprintf(name, sizeof name, "gm_s2_%d", w);
    std::string s;
    total += xorgen::emit_program(s, name, rows2, F, rowsel, 2, im);
    std::fputs(s.c_str(), stdout);
  }
  // S3: the XOR sums (0/1 map from the K R-coefficient slots), then the twists
  std::vector<uint32_t> M3((size_t)K * K, 0);  // row (H par + i), column slot
  for (int par = 0; par < 2; ++par)
    for (int i = 0; i < H; ++i)
      for (int c = 0; c < F; ++c) {
        if (binom_odd(c, i - c)) M3[(size_t)(H * par + i) * K + 4 * c + par] ^= 1u;
        if (binom_odd(c, i - 1 - c)) M3[(size_t)(H * par + i) * K + 4 * c + par + 2] ^= 1u;
      }
  const auto rows3 = all_bitrows(M3, K, K);
  const int wpq = waves / 2;  // waves per Q
  for (int w = 0; w < waves; ++w) {
    const int par = w / wpq, i0 = 4 * (w % wpq);
    std::vector<int> rowsel;
    for (int i = i0; i < i0 + 4; ++i)
      for (int b = 0; b < 16; ++b) rowsel.push_back(16 * (H * par + i) + b);
    char name[32];
    std::snprintf(name, sizeof name, "gm_s3sum_%d", w);
    std::string s;
    xorgen::InputMap im;
    total += xorgen::emit_program(s, name, rows3, K, rowsel, 4, im);
    std::fputs(s.c_str(), stdout);
  }
  for (int i = 1; i < H; ++i) {
    char name[32];
    std::snprintf(name, sizeof name, "gm_tw%d", i);
    total += (size_t)2 * emit_twist(name, gf16_pow(dinv, (uint32_t)i));  // (applied to both Q)
  }
  // dispatch
  for (const char *st : {"gm_s1_", "gm_s2_", "gm_s3sum_"}) {
    std::printf("  template <typename In>\n  __device__ __forceinline__ static void %s(int w, const In &IN4, uint32_t (&acc)[64]) {\n", st);
    std::printf("    switch (w) {\n");
    for (int w = 0; w < waves; ++w) std::printf("      case %d: %s%d(IN4, acc); break;\n", w, st, w);
    std::printf("      default: break;\n    }\n  }\n");
  }
  std::printf("  // acc (Q coefficients i0..i0+3) *= delta^-i\n");
  std::printf("  __device__ __forceinline__ static void gm_twist(int i, uint32_t (&acc)[16]) {\n    switch (i) {\n");
  for (int i = 1; i < H; ++i) std::printf("      case %d: gm_tw%d(acc); break;\n", i, i);
  std::printf("      default: break;\n    }\n  }\n");
  return total;
}

// Fill programs for one erased set: wave w computes the value at erased point
// E[w] as the fixed combination of the K survivors (Lagrange over S), reading
// survivor j from its own LDS slot S[j].
//   gen_restore fill K N pb e0 e1 ..
static int main_fill(int argc, char **argv) {
  const int K = std::atoi(argv[2]), N = std::atoi(argv[3]), pb = std::atoi(argv[4]);
  std::vector<int> E, S;
  for (int i = 5; i < argc; ++i) E.push_back(std::atoi(argv[i]));
  for (int a = 0; a < N && (int)S.size() < K; ++a)
    if (std::find(E.begin(), E.end(), a) == E.end()) S.push_back(a);
  std::printf("// GENERATED by tools/xorgen/gen_restore fill %d %d %d", K, N, pb);
  for (int e : E) std::printf(" %d", e);
  std::printf(" -- do not edit.\n");
  std::string s;
  const size_t total = xorgen::emit_fill_programs(s, "FillPrograms", K, S, pb);
  std::fputs(s.c_str(), stdout);
  std::fprintf(stderr, "fill K=%d N=%d: %zu XOR instructions per 32 stripes\n", K, N, total);
  return 0;
}

// Small-M syndromes (k_restore_syn's SMALL batch mode, restore_syn.hpp): the
// MS checks of the code restricted to the FIXED point set A = {0..K+MS-1},
//   S_j = sum_{a in A} v_a a^j y_a,  v_a = 1 / prod_{b in A, b != a} (a + b),
// which vanish on every codeword; with at most MS points of A erased (zeroed)
// they determine the erased values through the MS x MS solve W_E^{-1}
// (host).  The download loop's survivor sets are mostly of this shape: the
// first k replicas found, with none or one or two of 0..k-1 lost.  Wave w
// takes points 4w..4w+3 and, for w < MS, point K + w, and computes its share
// of every S_j (one Paar program per wave); the shares meet in the syndrome
// slots K + MS + j through LDS XOR atomics.
static int main_small(int argc, char **argv) {
  if (argc != 5) return 2;
  const int K = std::atoi(argv[2]), MS = std::atoi(argv[3]), pb = std::atoi(argv[4]);
  const int N = K + MS, WV = K / 4;
  if (K % 4 || MS < 1 || MS > WV || 2 * MS > K / 4 || pb < 1) return 2;
  std::vector<uint32_t> W((size_t)MS * N);
  for (int a = 0; a < N; ++a) {
    uint32_t prod = 1;
    for (int b = 0; b < N; ++b)
      if (b != a) prod = gf16_mul(prod, (uint32_t)(a ^ b));
    const uint32_t v = gf16_inv(prod);
    for (int j = 0; j < MS; ++j) W[(size_t)j * N + a] = gf16_mul(v, gf16_vandermonde(a, j));
  }
  std::printf("// GENERATED by tools/xorgen/gen_restore small %d %d %d -- do not edit.\n", K, MS, pb);
  std::printf("// Small-M syndromes over the points 0..%d for k_restore_syn's SMALL batch mode (%d waves).\n", N - 1, WV);
  std::printf("template <> struct SmallSyn<%d, %d> {\n", K, MS);
  std::printf("  static constexpr bool kSmall = true, kPerm = false, kMulti = false;\n  static constexpr int kFill = -1;\n");
  std::printf("  static constexpr bool kScatter = false;\n");
  std::printf("  static constexpr int kM = %d, kN = %d, kSynSlot = %d;  // syndrome j in LDS slot kSynSlot + j\n", MS, N, N);
  std::printf("  static constexpr uint16_t kW[%d][%d] = {\n", MS, N);
  for (int j = 0; j < MS; ++j) {
    std::printf("    {");
    for (int a = 0; a < N; ++a) std::printf("0x%04x%s", W[(size_t)j * N + a], a + 1 < N ? ", " : "");
    std::printf("},\n");
  }
  std::printf("  };\n");
  size_t total = 0;
  for (int w = 0; w < WV; ++w) {
    std::vector<int> pts = {4 * w, 4 * w + 1, 4 * w + 2, 4 * w + 3};
    if (w < MS) pts.push_back(K + w);
    std::vector<uint32_t> Ww((size_t)MS * pts.size());
    for (int j = 0; j < MS; ++j)
      for (size_t i = 0; i < pts.size(); ++i) Ww[(size_t)j * pts.size() + i] = W[(size_t)j * N + pts[i]];
    const auto rows = all_bitrows(Ww, MS, (int)pts.size());
    xorgen::InputMap im;
    im.map = pts;
    char name[32];
    std::snprintf(name, sizeof name, "part%d", w);
    std::string s;
    const size_t ops = xorgen::emit_program(s, name, rows, (int)pts.size(), row_range(0, 16 * MS), pb, im);
    std::fputs(s.c_str(), stdout);
    std::fprintf(stderr, "  %s: %zu ops\n", name, ops);
    total += ops;
  }
  std::printf("  template <typename In>\n  __device__ __forceinline__ static void part(int w, const In &IN4, uint32_t (&acc)[%d]) {\n",
              16 * MS);
  std::printf("    switch (w) {\n");
  for (int w = 0; w < WV; ++w) std::printf("      case %d: part%d(IN4, acc); break;\n", w, w);
  std::printf("      default: break;\n    }\n  }\n");
  std::printf("  static constexpr int kXorOps = %zu;\n};\n", total);
  std::fprintf(stderr, "small K=%d MS=%d: %zu XOR instructions per 32 stripes\n", K, MS, total);
  return 0;
}

// PERM (k_restore_syn's PERM batch regenerate, restore_syn.hpp): survivors
// exactly U = {0..K-1} (K = 2^m: U is the GF(2)-span of 1, x, .., x^(m-1)),
// one target t = K + t' with t' in U.  Q(X) = P(X + t') has the same degree
// and Q(c) = P(c + t') for c in U, so
//   P(t) = Q(K) = sum_{c in U} l_c(K) y_{c + t'},  l_c(K) = prod_{b != c} (K + b) / (c + b):
// ONE fixed program for every target of K..2K-1, its inputs read through the
// runtime address permutation c -> c XOR t'.  Wave w takes points 4w..4w+3.
static int main_perm(int argc, char **argv) {
  if (argc != 4) return 2;
  const int K = std::atoi(argv[2]), pb = std::atoi(argv[3]), WV = K / 4;
  if (K < 4 || (K & (K - 1)) || pb < 1) return 2;
  std::vector<uint32_t> l(K);
  for (int c = 0; c < K; ++c) {
    uint32_t num = 1, den = 1;
    for (int b = 0; b < K; ++b)
      if (b != c) {
        num = gf16_mul(num, (uint32_t)(K ^ b));
        den = gf16_mul(den, (uint32_t)(c ^ b));
      }
    l[c] = gf16_mul(num, gf16_inv(den));
  }
  std::printf("// GENERATED by tools/xorgen/gen_restore perm %d %d -- do not edit.\n", K, pb);
  std::printf("// P(K + t') = sum_c l_c(K) y_(c ^ t') for k_restore_syn's PERM batch regenerate (%d waves).\n", WV);
  std::printf("template <> struct PermSyn<%d> {\n", K);
  std::printf("  static constexpr bool kSmall = false, kPerm = true, kScatter = false, kMulti = false;\n");
  std::printf("  static constexpr int kFill = -1;\n");
  std::printf("  static constexpr uint16_t kL[%d] = {", K);
  for (int c = 0; c < K; ++c) std::printf("0x%04x%s", l[c], c + 1 < K ? ", " : "");
  std::printf("};\n");
  size_t total = 0;
  for (int w = 0; w < WV; ++w) {
    std::vector<uint32_t> Ww(4);
    for (int i = 0; i < 4; ++i) Ww[i] = l[4 * w + i];
    const auto rows = all_bitrows(Ww, 1, 4);
    xorgen::InputMap im;
    im.map = {4 * w, 4 * w + 1, 4 * w + 2, 4 * w + 3};
    char name[32];
    std::snprintf(name, sizeof name, "part%d", w);
    std::string s;
    const size_t ops = xorgen::emit_program(s, name, rows, 4, row_range(0, 16), pb, im);
    std::fputs(s.c_str(), stdout);
    std::fprintf(stderr, "  %s: %zu ops\n", name, ops);
    total += ops;
  }
  std::printf("  template <typename In>\n  __device__ __forceinline__ static void part(int w, const In &IN4, uint32_t (&acc)[16]) {\n");
  std::printf("    switch (w) {\n");
  for (int w = 0; w < WV; ++w) std::printf("      case %d: part%d(IN4, acc); break;\n", w, w);
  std::printf("      default: break;\n    }\n  }\n");
  std::printf("  static constexpr int kXorOps = %zu;\n};\n", total);
  std::fprintf(stderr, "perm K=%d: %zu XOR instructions per 32 stripes\n", K, total);
  return 0;
}

int main(int argc, char **argv) {
  if (argc > 1 && std::string(argv[1]) == "perm") return main_perm(argc, argv);
  if (argc > 1 && std::string(argv[1]) == "fill") return main_fill(argc, argv);
  if (argc > 1 && std::string(argv[1]) == "small") return main_small(argc, argv);
  if (argc < 6 || argc > 8) {
    std::fprintf(stderr, "usage: %s K N WAVES syndrome_block interp_block [half_interp_block [half_split]]\n", argv[0]);
    return 2;
  }
  const int K = std::atoi(argv[1]), N = std::atoi(argv[2]), M = N - K, waves = std::atoi(argv[3]);
  const int syn_pb = std::atoi(argv[4]), int_pb = std::atoi(argv[5]);
  const int hb_pb = argc > 6 ? std::atoi(argv[6]) : 2;
  size_t total_b = 0;
  if ((16 * M) % waves || (16 * K) % waves) {
    std::fprintf(stderr, "16 (N - K) and 16 K must split evenly over the waves\\n");
    return 2;
  }
  // syndrome matrix W (M x N)
  std::vector<uint32_t> W((size_t)M * N);
  for (int a = 0; a < N; ++a) {
    uint32_t prod = 1;
    for (int b = 0; b < N; ++b)
      if (b != a) prod = gf16_mul(prod, (uint32_t)(a ^ b));
    const uint32_t v = gf16_inv(prod);
    for (int j = 0; j < M; ++j) W[(size_t)j * N + a] = gf16_mul(v, gf16_vandermonde(a, j));
  }
  // V_F^{-1} for F = {0..K-1}
  std::vector<uint16_t> nodes(K), inv((size_t)K * K);
  for (int i = 0; i < K; ++i) nodes[i] = (uint16_t)i;
  if (vds_ec_inverse16(K, nodes.data(), inv.data()) != VDS_EC_OK) return 1;
  std::vector<uint32_t> Vi(inv.begin(), inv.end());
  const int syn_rows = 16 * M / waves, int_rows = 16 * K / waves;

  std::printf("// GENERATED by tools/xorgen/gen_restore %d %d %d %d %d %d -- do not edit.\n", K, N, waves, syn_pb, int_pb, hb_pb);
  std::printf("// Syndrome and fixed-interpolation XOR programs for k_restore_syn<%d,%d> with %d waves\n", K, N, waves);
  std::printf("// (points blocked by %d / %d; IN4(g) = planes 4g..4g+3, plane = 16 point + bit).\n", syn_pb, int_pb);
  std::printf("template <> struct RestorePrograms<%d, %d, %d> {\n", K, N, waves);
  std::printf("  static constexpr int kSynRows = %d;  // syndrome bit-rows per wave (wave w: rows %d w ..)\n", syn_rows, syn_rows);
  std::printf("  static constexpr int kIntRows = %d;  // object bit-rows per wave (cells %d w ..)\n", int_rows, int_rows / 16);
  // the syndrome weights v_a a^j, for the host-side solve (row j, column a)
  std::printf("  static constexpr uint16_t kSyndromeW[%d][%d] = {\n", M, N);
  for (int j = 0; j < M; ++j) {
    std::printf("    {");
    for (int a = 0; a < N; ++a) std::printf("0x%04x%s", W[(size_t)j * N + a], a + 1 < N ? ", " : "");
    std::printf("},\n");
  }
  std::printf("  };\n");
  const auto wrows = all_bitrows(W, M, N), vrows = all_bitrows(Vi, K, K);
  size_t total = 0;
  for (int w = 0; w < waves; ++w) {
    char name[64];
    std::snprintf(name, sizeof name, "syndrome%d", w);
    total += emit_program(name, wrows, N, row_range(syn_rows * w, syn_rows), syn_pb);
  }
  // interp_block 0: no direct K-point programs (the kernel uses the
  // additive-FFT stage B only; the direct ones are large for K = 32)
  for (int w = 0; w < waves && int_pb > 0; ++w) {
    char name[64];
    std::snprintf(name, sizeof name, "interp%d", w);
    total += emit_program(name, vrows, K, row_range(int_rows * w, int_rows), int_pb);
  }
  // Half-size interpolation for the one-level additive-FFT interpolation
  // (k_restore_syn stage B): with G = {0, 2, .., K-2} and s(g) = g^2 + g,
  // P(X) = P0(X^2+X) + X P1(X^2+X) where P0 / P1 (degree < K/2) take the
  // values Q0 / Q1 at the K/2 points D = s(G), parked in LDS slots 2i / 2i+1.
  // Wave w computes rows [hb_rows (w % (waves/2)), +hb_rows) of P0 (w < waves/2) or P1.
  const int H = K / 2, hb_parts = waves / 2, hb_rows = 16 * H / hb_parts;
  std::vector<uint16_t> dpts(H), dinv((size_t)H * H);
  for (int i = 0; i < H; ++i) dpts[i] = (uint16_t)(gf16_mul(2 * i, 2 * i) ^ (2 * i));
  if (vds_ec_inverse16(H, dpts.data(), dinv.data()) != VDS_EC_OK) return 1;
  std::vector<uint32_t> Di(dinv.begin(), dinv.end());
  const auto drows = all_bitrows(Di, H, H);
  // Cells (coefficients) of P0 / P1 per part: argv[7] gives the part of each
  // of the H cells (default: contiguous), chosen to balance the programs.
  std::vector<std::vector<int>> part_cells(hb_parts);
  for (int c = 0; c < H; ++c) {
    const int part = argc > 7 ? argv[7][c] - '0' : c / (H / hb_parts);
    if (part < 0 || part >= hb_parts) return 1;
    part_cells[part].push_back(c);
  }
  for (const auto &pc : part_cells)
    if ((int)pc.size() != H / hb_parts) return 1;
  std::printf("  static constexpr int kHalfRows = %d;  // stage-B bit-rows per wave\n", hb_rows);
  std::printf("  // stage-B cell c of part p (wave w: part w %% %d of P0 (w < %d) or P1)\n", hb_parts, hb_parts);
  std::printf("  static constexpr uint8_t kHalfCell[%d][%d] = {", hb_parts, H / hb_parts);
  for (int q = 0; q < hb_parts; ++q) {
    std::printf("{");
    for (int c : part_cells[q]) std::printf("%d, ", c);
    std::printf("}, ");
  }
  std::printf("};\n");
  for (int w = 0; w < waves; ++w) {
    char name[64];
    std::snprintf(name, sizeof name, "interpB%d", w);
    g_im.par = w / hb_parts;
    std::vector<int> rowsel;
    for (int c : part_cells[w % hb_parts])
      for (int b = 0; b < 16; ++b) rowsel.push_back(16 * c + b);
    total_b += emit_program(name, drows, H, rowsel, hb_pb);
  }
  g_im.par = -1;
  std::printf("  template <typename In>\n  __device__ __forceinline__ static void interpB(int w, const In &IN4, uint32_t (&acc)[%d]) {\n", hb_rows);
  std::printf("    switch (w) {\n");
  for (int w = 0; w < waves; ++w) std::printf("      case %d: interpB%d(IN4, acc); break;\n", w, w);
  std::printf("      default: break;\n    }\n  }\n");
  for (const char *kind : {"syndrome", "interp"}) {
    if (kind[0] == 'i' && int_pb == 0) continue;
    std::printf("  template <typename In>\n  __device__ __forceinline__ static void %s(int w, const In &IN4, uint32_t (&acc)[%d]) {\n",
                kind, kind[0] == 's' ? syn_rows : int_rows);
    std::printf("    switch (w) {\n");
    for (int w = 0; w < waves; ++w) std::printf("      case %d: %s%d(IN4, acc); break;\n", w, kind, w);
    std::printf("      default: break;\n    }\n  }\n");
  }
  std::printf("  static constexpr int kXorOps = %zu;\n", total);
  std::printf("  static constexpr int kXorOpsHalf = %zu;  // stage B (all four waves)\n", total_b);
  const size_t total_gm2 = emit_gm2(K, waves);
  std::printf("};\n");
  std::fprintf(stderr, "two-level interpolation: %zu XOR instructions per 32 stripes\n", total_gm2);
  std::fprintf(stderr, "K=%d N=%d waves=%d: %zu XOR instructions per 32 stripes (stage B: %zu)\n", K, N, waves, total,
               total_b);
  return 0;
}
