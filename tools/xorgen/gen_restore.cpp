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
//   gen_restore K N [syndrome_block interp_block] > restore_K_N.inc
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "../../include/vds_ec.h"
#include "../../vds_amd/csrc/gf_common.hpp"
#include "paar.hpp"

using namespace vds_ec;

// Bit-matrix rows of y = M x (M: R x C field constants): output plane 16m+i is
// the XOR of input planes 16j+b with bit i of M[m][j] * x^b set.
static std::vector<std::vector<int>> bitrows(const std::vector<uint32_t> &M, int R, int C, int row0, int rows) {
  std::vector<std::vector<int>> out(16 * rows);
  for (int m = row0; m < row0 + rows; ++m)
    for (int j = 0; j < C; ++j)
      for (int b = 0; b < 16; ++b) {
        const uint32_t v = gf16_mul(M[(size_t)m * C + j], 1u << b);
        for (int i = 0; i < 16; ++i)
          if ((v >> i) & 1) out[16 * (m - row0) + i].push_back(16 * j + b);
      }
  return out;
}

// Emit one block of a program: the block reads the input planes of points
// [p0, p0 + np) (IN4(g) = the 4 planes of group g, a b128 LDS read) and
// accumulates its share into acc[]; `first` assigns instead.  Temps are emitted
// in creation order and each output row is folded in as soon as everything it
// needs exists, so temps die early and register pressure stays bounded.
static size_t emit_block(const xorgen::XorProgram &p, int p0, bool first) {
  const int n = p.ninputs, T = (int)p.temps.size();
  std::vector<bool> used(n, false);
  for (auto &t : p.temps) {
    if (t.first < n) used[t.first] = true;
    if (t.second < n) used[t.second] = true;
  }
  for (auto &r : p.rows)
    for (int x : r)
      if (x < n) used[x] = true;
  std::printf("    {\n");
  for (int g = 0; g < n / 4; ++g)
    if (used[4 * g] || used[4 * g + 1] || used[4 * g + 2] || used[4 * g + 3])
      std::printf("      const auto g%d = IN4(%d);\n", g, 4 * p0 + g);
  auto nm = [&](int id) {
    return id < n ? "g" + std::to_string(id / 4) + "[" + std::to_string(id % 4) + "]" : "t" + std::to_string(id);
  };
  // row o is ready once its largest temp id exists
  std::vector<std::vector<int>> ready_at(T + 1);
  for (size_t o = 0; o < p.rows.size(); ++o) {
    int mx = -1;
    for (int x : p.rows[o])
      if (x >= n) mx = std::max(mx, x - n);
    ready_at[mx + 1].push_back((int)o);
  }
  size_t ops = T;
  auto fold = [&](int o) {
    const auto &r = p.rows[o];
    if (r.empty()) {
      if (first) std::printf("      acc[%d] = 0u;\n", o);
      return;
    }
    std::string acc;
    size_t i = 0;
    if (first) {
      acc = nm(r[0]);
      i = 1;
    } else {
      acc = "acc[" + std::to_string(o) + "]";
    }
    // v_bitop3_b32 (0x96) is a 3-input XOR on gfx950
    while (i < r.size()) {
      if (i + 1 < r.size()) {
        acc = "xor3(" + acc + ", " + nm(r[i]) + ", " + nm(r[i + 1]) + ")";
        i += 2;
      } else {
        acc = "(" + acc + " ^ " + nm(r[i]) + ")";
        i += 1;
      }
      ++ops;
    }
    std::printf("      acc[%d] = %s;\n", o, acc.c_str());
  };
  for (int o : ready_at[0]) fold(o);
  for (int t = 0; t < T; ++t) {
    std::printf("      const uint32_t t%d = %s ^ %s;\n", n + t, nm(p.temps[t].first).c_str(),
                nm(p.temps[t].second).c_str());
    for (int o : ready_at[t + 1]) fold(o);
  }
  std::printf("    }\n");
  return ops;
}

// One wave's program: rows [r0, r0 + nr) of M (R x C), points blocked by `pb`.
static size_t emit_program(const char *name, const std::vector<uint32_t> &M, int C, int r0, int nr, int pb) {
  std::printf("  template <typename In>\n  __device__ __forceinline__ static void %s(const In &IN4, uint32_t (&acc)[%d]) {\n",
              name, 16 * nr);
  size_t ops = 0;
  for (int c0 = 0; c0 < C; c0 += pb) {
    const int cb = std::min(pb, C - c0);
    std::vector<uint32_t> sub((size_t)nr * cb);
    for (int m = 0; m < nr; ++m)
      for (int j = 0; j < cb; ++j) sub[(size_t)m * cb + j] = M[(size_t)(r0 + m) * C + c0 + j];
    ops += emit_block(xorgen::paar(16 * cb, bitrows(sub, nr, cb, 0, nr)), c0, c0 == 0);
  }
  std::printf("  }\n");
  return ops;
}

int main(int argc, char **argv) {
  if (argc != 3 && argc != 5) {
    std::fprintf(stderr, "usage: %s K N [syndrome_block interp_block]\n", argv[0]);
    return 2;
  }
  const int K = std::atoi(argv[1]), N = std::atoi(argv[2]), M = N - K;
  const int syn_pb = argc == 5 ? std::atoi(argv[3]) : 4;
  const int int_pb = argc == 5 ? std::atoi(argv[4]) : 1;
  const int waves = K / 4;
  if (K % 4 || M != waves) {
    std::fprintf(stderr, "layout needs K %% 4 == 0 and N - K == K / 4\n");
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

  std::printf("// GENERATED by tools/xorgen/gen_restore %d %d -- do not edit.\n", K, N);
  std::printf("// Syndrome and fixed-interpolation XOR programs for k_restore_syn<%d,%d>\n", K, N);
  std::printf("// (points blocked by %d / %d; IN4(g) = planes 4g..4g+3, plane = 16 point + bit).\n", syn_pb, int_pb);
  std::printf("template <> struct RestorePrograms<%d, %d> {\n", K, N);
  std::printf("  static constexpr int kWaves = %d;\n", waves);
  // the syndrome weights v_a a^j, for the host-side solve (row j, column a)
  std::printf("  static constexpr uint16_t kSyndromeW[%d][%d] = {\n", M, N);
  for (int j = 0; j < M; ++j) {
    std::printf("    {");
    for (int a = 0; a < N; ++a) std::printf("0x%04x%s", W[(size_t)j * N + a], a + 1 < N ? ", " : "");
    std::printf("},\n");
  }
  std::printf("  };\n");
  size_t total = 0;
  for (int w = 0; w < waves; ++w) {  // wave w: syndrome S_w (16 planes, N points)
    char name[64];
    std::snprintf(name, sizeof name, "syndrome%d", w);
    total += emit_program(name, W, N, w, 1, syn_pb);
  }
  for (int w = 0; w < waves; ++w) {  // wave w: cells 4w..4w+3 (64 planes, points 0..K-1)
    char name[64];
    std::snprintf(name, sizeof name, "interp%d", w);
    total += emit_program(name, Vi, K, 4 * w, 4, int_pb);
  }
  std::printf("  static constexpr int kXorOps = %zu;\n", total);
  std::printf("};\n");
  std::fprintf(stderr, "K=%d N=%d: %zu XOR ops per 32 stripes\n", K, N, total);
  return 0;
}
