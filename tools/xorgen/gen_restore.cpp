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

// One block of a program: a Paar program over the input planes of points
// [p0, p0 + np), turned into emit-ready nodes.  Single-use two-input temps are
// fused into their consumer, so most nodes become one v_bitop3_b32 (a 3-input
// XOR at the issue cost of a 2-input one on gfx950).
struct Block {
  int p0 = 0, n = 0;
  std::vector<std::vector<int>> node;  // operands per temp id (n + t); empty = fused away
  std::vector<std::vector<int>> rows;  // operands per output row (expanded)
  std::vector<bool> group_used;
};

static Block make_block(const xorgen::XorProgram &p, int p0) {
  Block B;
  B.p0 = p0;
  B.n = p.ninputs;
  const int n = p.ninputs, T = (int)p.temps.size();
  std::vector<int> uses(n + T, 0);
  for (auto &t : p.temps) ++uses[t.first], ++uses[t.second];
  for (auto &r : p.rows)
    for (int x : r) ++uses[x];
  B.node.assign(n + T, {});
  std::vector<bool> fused(n + T, false);
  for (int t = 0; t < T; ++t) B.node[n + t] = {p.temps[t].first, p.temps[t].second};
  auto fusable = [&](int c) { return c >= n && uses[c] == 1 && !fused[c] && B.node[c].size() == 2; };
  for (int t = 0; t < T; ++t) {
    auto &o = B.node[n + t];
    for (size_t i = 0; i < o.size() && o.size() < 3; ++i)
      if (fusable(o[i])) {
        const int c = o[i];
        fused[c] = true;
        o.erase(o.begin() + i);
        o.insert(o.end(), B.node[c].begin(), B.node[c].end());
        B.node[c].clear();
        break;
      }
  }
  for (auto &r : p.rows) {
    std::vector<int> e;
    for (int x : r)
      if (fusable(x)) {
        fused[x] = true;
        e.insert(e.end(), B.node[x].begin(), B.node[x].end());
        B.node[x].clear();
      } else {
        e.push_back(x);
      }
    B.rows.push_back(e);
  }
  B.group_used.assign(n / 4, false);
  auto mark = [&](int x) {
    if (x < n) B.group_used[x / 4] = true;
  };
  for (int t = 0; t < T; ++t)
    for (int x : B.node[n + t]) mark(x);
  for (auto &r : B.rows)
    for (int x : r) mark(x);
  return B;
}

// Input point i of a program lives at LDS point i (par < 0) or 2 i + par
// (the half-size interpolations read every other slot).
static int g_par = -1;

static void emit_loads(const Block &B, int bi) {
  for (int g = 0; g < B.n / 4; ++g)
    if (B.group_used[g]) {
      const int pt = B.p0 + g / 4;
      const int lds_pt = g_par < 0 ? pt : 2 * pt + g_par;
      std::printf("    const auto g%d_%d = IN4(%d);\n", bi, g, 4 * lds_pt + g % 4);
    }
}

// Emit a block's XORs; acc[] accumulates (first block: assigns).  Nodes are
// emitted in creation order and every output row is folded in as soon as its
// operands exist, so temps die early and register pressure stays bounded.
static size_t emit_compute(const Block &B, int bi, bool first) {
  const int n = B.n, T = (int)B.node.size() - n;
  auto nm = [&](int id) {
    return id < n ? "g" + std::to_string(bi) + "_" + std::to_string(id / 4) + "[" + std::to_string(id % 4) + "]"
                  : "t" + std::to_string(bi) + "_" + std::to_string(id);
  };
  std::vector<std::vector<int>> ready_at(T + 1);
  for (size_t o = 0; o < B.rows.size(); ++o) {
    int mx = -1;
    for (int x : B.rows[o])
      if (x >= n) mx = std::max(mx, x - n);
    ready_at[mx + 1].push_back((int)o);
  }
  size_t ops = 0;
  auto fold = [&](int o) {
    const auto &r = B.rows[o];
    if (r.empty()) {
      if (first) std::printf("    acc[%d] = 0u;\n", o);
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
    std::printf("    acc[%d] = %s;\n", o, acc.c_str());
  };
  for (int o : ready_at[0]) fold(o);
  for (int t = 0; t < T; ++t) {
    const auto &o = B.node[n + t];
    if (o.size() == 2) {
      std::printf("    const uint32_t %s = %s ^ %s;\n", nm(n + t).c_str(), nm(o[0]).c_str(), nm(o[1]).c_str());
      ++ops;
    } else if (o.size() == 3) {
      std::printf("    const uint32_t %s = xor3(%s, %s, %s);\n", nm(n + t).c_str(), nm(o[0]).c_str(),
                  nm(o[1]).c_str(), nm(o[2]).c_str());
      ++ops;
    }
    for (int r : ready_at[t + 1]) fold(r);
  }
  return ops;
}

// All bit-rows of y = M x for M (R x C field constants): row 16 m + i is the
// set of input planes 16 j + b with bit i of M[m][j] * x^b set.
static std::vector<std::vector<int>> all_bitrows(const std::vector<uint32_t> &M, int R, int C) {
  return bitrows(M, R, C, 0, R);
}

// One wave's program: bit-rows [row0, row0 + nrows) of the map, points
// blocked by `pb`.  The LDS reads of block b + 1 are issued before the XORs of
// block b so their latency hides under them.
static size_t emit_program(const char *name, const std::vector<std::vector<int>> &rows, int C,
                           const std::vector<int> &rowsel, int pb) {
  const int nrows = (int)rowsel.size();
  std::printf("  template <typename In>\n  __device__ __forceinline__ static void %s(const In &IN4, uint32_t (&acc)[%d]) {\n",
              name, nrows);
  std::vector<Block> blocks;
  for (int c0 = 0; c0 < C; c0 += pb) {
    const int cb = std::min(pb, C - c0);
    std::vector<std::vector<int>> sub(nrows);
    for (int r = 0; r < nrows; ++r)
      for (int x : rows[rowsel[r]])
        if (x >= 16 * c0 && x < 16 * (c0 + cb)) sub[r].push_back(x - 16 * c0);
    blocks.push_back(make_block(xorgen::paar(16 * cb, sub), c0));
  }
  size_t ops = 0;
  emit_loads(blocks[0], 0);
  for (size_t b = 0; b < blocks.size(); ++b) {
    if (b + 1 < blocks.size()) emit_loads(blocks[b + 1], (int)b + 1);
    ops += emit_compute(blocks[b], (int)b, b == 0);
    // keep the scheduler from hoisting later blocks' LDS reads (and their
    // registers) above this block
    std::printf("    VDS_SCHED_FENCE();\n");
  }
  std::printf("  }\n");
  std::fprintf(stderr, "  %s: %zu ops\n", name, ops);
  return ops;
}

static std::vector<int> row_range(int row0, int n) {
  std::vector<int> v(n);
  for (int i = 0; i < n; ++i) v[i] = row0 + i;
  return v;
}

int main(int argc, char **argv) {
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
    g_par = w / hb_parts;
    std::vector<int> rowsel;
    for (int c : part_cells[w % hb_parts])
      for (int b = 0; b < 16; ++b) rowsel.push_back(16 * c + b);
    total_b += emit_program(name, drows, H, rowsel, hb_pb);
  }
  g_par = -1;
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
  std::printf("};\n");
  std::fprintf(stderr, "K=%d N=%d waves=%d: %zu XOR instructions per 32 stripes (stage B: %zu)\n", K, N, waves, total,
               total_b);
  return 0;
}
