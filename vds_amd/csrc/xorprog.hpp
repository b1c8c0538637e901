// xorprog.hpp -- straight-line XOR programs for fixed GF(2^16)-linear maps on
// bit-sliced planes (host code).
//
// A linear map y = M x over GF(2^16) (M: R x C field constants) is, on
// bit-sliced planes, a GF(2) bit matrix: output plane 16 m + i is the XOR of
// the input planes 16 j + b with bit i of M[m][j] * x^b set.  Paar's greedy
// common-subexpression elimination turns each wave's rows into a short XOR
// program; single-use two-input temps are fused into their consumer, so most
// nodes become one v_bitop3_b32 (a 3-input XOR at the issue cost of a 2-input
// one on gfx950).  The program is printed as C++ for the restore kernels.
//
// Used offline by tools/xorgen/gen_restore.cpp (the committed
// generated/restore_K_N_wW.inc) and at run time by vds_ec_jit.cpp (the
// pattern-specific fill programs).
#pragma once

#include <algorithm>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "gf_common.hpp"

namespace xorgen {

struct XorProgram {
  int ninputs = 0;
  std::vector<std::pair<int, int>> temps;  // temp id = ninputs + index
  std::vector<std::vector<int>> rows;      // per output: ids to XOR
  size_t xor_count() const {
    size_t n = temps.size();
    for (auto &r : rows) n += r.empty() ? 0 : r.size() - 1;
    return n;
  }
};

// Paar's heuristic: repeatedly factor out the pair of ids that occurs in the
// most rows.  Input: rows[r] = input columns whose XOR is output r.
inline XorProgram paar(int ncols, std::vector<std::vector<int>> rows) {
  XorProgram prog;
  prog.ninputs = ncols;
  const int R = (int)rows.size();
  for (auto &r : rows) std::sort(r.begin(), r.end());
  auto key = [](int a, int b) -> uint64_t {
    if (a > b) std::swap(a, b);
    return (uint64_t(uint32_t(a)) << 32) | uint32_t(b);
  };
  std::unordered_map<uint64_t, int> cnt;
  cnt.reserve(1 << 16);
  std::vector<std::unordered_set<uint64_t>> bucket(R + 2);
  auto add = [&](int a, int b, int d) {
    const uint64_t k = key(a, b);
    int &c = cnt[k];
    if (c > 0) bucket[c].erase(k);
    c += d;
    if (c > 0)
      bucket[c].insert(k);
    else
      cnt.erase(k);
  };
  for (auto &r : rows)
    for (size_t i = 0; i < r.size(); ++i)
      for (size_t j = i + 1; j < r.size(); ++j) add(r[i], r[j], 1);
  // column -> rows containing it
  std::vector<std::vector<int>> col_rows(ncols);
  for (int ri = 0; ri < R; ++ri)
    for (int c : rows[ri]) col_rows[c].push_back(ri);
  int top = R + 1;
  while (true) {
    while (top >= 2 && bucket[top].empty()) --top;
    if (top < 2) break;
    const uint64_t k = *bucket[top].begin();
    const int a = int(k >> 32), b = int(k & 0xFFFFFFFFu);
    const int t = ncols + (int)prog.temps.size();
    prog.temps.push_back({a, b});
    col_rows.emplace_back();
    // rows containing both a and b
    std::vector<int> both;
    {
      auto &ra = col_rows[a], &rb = col_rows[b];
      std::set_intersection(ra.begin(), ra.end(), rb.begin(), rb.end(), std::back_inserter(both));
    }
    for (int ri : both) {
      auto &r = rows[ri];
      for (int x : r) {
        if (x == a || x == b) continue;
        add(a, x, -1);
        add(b, x, -1);
        add(t, x, +1);
      }
      add(a, b, -1);
      r.erase(std::find(r.begin(), r.end(), a));
      r.erase(std::find(r.begin(), r.end(), b));
      r.push_back(t);  // t is the largest id so far: stays sorted
    }
    auto rm = [&](std::vector<int> &v) {
      std::vector<int> out;
      std::set_difference(v.begin(), v.end(), both.begin(), both.end(), std::back_inserter(out));
      v.swap(out);
    };
    rm(col_rows[a]);
    rm(col_rows[b]);
    col_rows[t] = both;
  }
  prog.rows = rows;
  return prog;
}

// Bit-matrix rows of y = M x (M: R x C field constants, row-major), rows
// [row0, row0 + rows): output plane 16 m + i is the XOR of input planes
// 16 j + b with bit i of M[m][j] * x^b set.
inline std::vector<std::vector<int>> bitrows(const std::vector<uint32_t> &M, int R, int C, int row0, int rows) {
  (void)R;
  std::vector<std::vector<int>> out(16 * rows);
  for (int m = row0; m < row0 + rows; ++m)
    for (int j = 0; j < C; ++j)
      for (int b = 0; b < 16; ++b) {
        const uint32_t v = vds_ec::gf16_mul(M[(size_t)m * C + j], 1u << b);
        for (int i = 0; i < 16; ++i)
          if ((v >> i) & 1) out[16 * (m - row0) + i].push_back(16 * j + b);
      }
  return out;
}
inline std::vector<std::vector<int>> all_bitrows(const std::vector<uint32_t> &M, int R, int C) {
  return bitrows(M, R, C, 0, R);
}

// printf into a string
inline void appendf(std::string &s, const char *fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  const int n = std::vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  if (n < (int)sizeof buf) {
    s.append(buf, n > 0 ? (size_t)n : 0);
    return;
  }
  std::string big((size_t)n + 1, '\0');
  va_start(ap, fmt);
  std::vsnprintf(&big[0], big.size(), fmt, ap);
  va_end(ap);
  s.append(big.data(), (size_t)n);
}

// One block of a program: a Paar program over the input planes of points
// [p0, p0 + np), turned into emit-ready nodes (fused xor3s).
struct Block {
  int p0 = 0, n = 0;
  std::vector<std::vector<int>> node;  // operands per temp id (n + t); empty = fused away
  std::vector<std::vector<int>> rows;  // operands per output row (expanded)
  std::vector<bool> group_used;
};

inline Block make_block(const XorProgram &p, int p0) {
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

// Where input point i of a program lives in the LDS: point i (par < 0), 2 i +
// par (the half-size interpolations read every other slot), or map[i] when
// map is set (the fill programs read the survivors' slots).
struct InputMap {
  int par = -1;
  std::vector<int> map;
  int at(int pt) const { return !map.empty() ? map[pt] : par < 0 ? pt : 2 * pt + par; }
};

inline void emit_loads(std::string &s, const Block &B, int bi, const InputMap &im) {
  for (int g = 0; g < B.n / 4; ++g)
    if (B.group_used[g]) {
      const int pt = B.p0 + g / 4;
      appendf(s, "    const auto g%d_%d = IN4(%d);\n", bi, g, 4 * im.at(pt) + g % 4);
    }
}

// Emit a block's XORs; acc[] accumulates (first block: assigns).  Nodes are
// emitted in creation order and every output row is folded in as soon as its
// operands exist, so temps die early and register pressure stays bounded.
inline size_t emit_compute(std::string &s, const Block &B, int bi, bool first) {
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
      if (first) appendf(s, "    acc[%d] = 0u;\n", o);
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
    appendf(s, "    acc[%d] = %s;\n", o, acc.c_str());
  };
  for (int o : ready_at[0]) fold(o);
  for (int t = 0; t < T; ++t) {
    const auto &o = B.node[n + t];
    if (o.size() == 2) {
      appendf(s, "    const uint32_t %s = %s ^ %s;\n", nm(n + t).c_str(), nm(o[0]).c_str(), nm(o[1]).c_str());
      ++ops;
    } else if (o.size() == 3) {
      appendf(s, "    const uint32_t %s = xor3(%s, %s, %s);\n", nm(n + t).c_str(), nm(o[0]).c_str(), nm(o[1]).c_str(),
              nm(o[2]).c_str());
      ++ops;
    }
    for (int r : ready_at[t + 1]) fold(r);
  }
  return ops;
}

// One wave's program: bit-rows rowsel of the map (C input points), points
// blocked by `pb`.  The LDS reads of block b + 1 are issued before the XORs of
// block b so their latency hides under them.  Returns the instruction count.
inline size_t emit_program(std::string &s, const char *name, const std::vector<std::vector<int>> &rows, int C,
                           const std::vector<int> &rowsel, int pb, const InputMap &im, bool prefetch = true) {
  const int nrows = (int)rowsel.size();
  appendf(s, "  template <typename In>\n  __device__ __forceinline__ static void %s(const In &IN4, uint32_t (&acc)[%d]) {\n",
          name, nrows);
  std::vector<Block> blocks;
  for (int c0 = 0; c0 < C; c0 += pb) {
    const int cb = std::min(pb, C - c0);
    std::vector<std::vector<int>> sub(nrows);
    for (int r = 0; r < nrows; ++r)
      for (int x : rows[rowsel[r]])
        if (x >= 16 * c0 && x < 16 * (c0 + cb)) sub[r].push_back(x - 16 * c0);
    blocks.push_back(make_block(paar(16 * cb, sub), c0));
  }
  size_t ops = 0;
  emit_loads(s, blocks[0], 0, im);
  for (size_t b = 0; b < blocks.size(); ++b) {
    if (b > 0 && !prefetch) emit_loads(s, blocks[b], (int)b, im);
    if (b + 1 < blocks.size() && prefetch) emit_loads(s, blocks[b + 1], (int)b + 1, im);
    ops += emit_compute(s, blocks[b], (int)b, b == 0);
    // keep the scheduler from hoisting later blocks' LDS reads (and their
    // registers) above this block
    appendf(s, "    VDS_SCHED_FENCE();\n");
  }
  appendf(s, "  }\n");
  return ops;
}

inline std::vector<int> row_range(int row0, int n) {
  std::vector<int> v(n);
  for (int i = 0; i < n; ++i) v[i] = row0 + i;
  return v;
}

// The fill programs of one survivor set (K survivors among points 0..N-1,
// ascending in `spoints`): program m computes the value at the m-th erased
// point below K -- the points the fixed interpolation from 0..K-1 needs -- as
// the Lagrange combination of the survivors, l_j(e) = prod_{t != j} (e + s_t)
// / (s_j + s_t): the unique polynomial through them, so the bytes equal the
// reference's V_S^{-1} route (chunk.h:290-444) for every input.  Survivor j is
// read from its own LDS slot spoints[j].  Emits `struct NAME { kFill, kPoint,
// fill0.., fill(w, IN4, acc) }`; returns the instruction count.
inline size_t emit_fill_programs(std::string &s, const char *name, int K, const std::vector<int> &spoints, int pb,
                                 bool prefetch = true) {
  std::vector<int> EU;
  for (int a = 0; a < K; ++a)
    if (std::find(spoints.begin(), spoints.end(), a) == spoints.end()) EU.push_back(a);
  std::vector<uint32_t> A(EU.size() * K);
  for (size_t m = 0; m < EU.size(); ++m)
    for (int j = 0; j < K; ++j) {
      uint32_t num = 1, den = 1;
      for (int t = 0; t < K; ++t)
        if (t != j) {
          num = vds_ec::gf16_mul(num, (uint32_t)(EU[m] ^ spoints[t]));
          den = vds_ec::gf16_mul(den, (uint32_t)(spoints[j] ^ spoints[t]));
        }
      A[m * K + j] = vds_ec::gf16_mul(num, vds_ec::gf16_inv(den));
    }
  InputMap im;
  im.map = spoints;
  appendf(s, "struct %s {\n  static constexpr int kFill = %zu;\n  static constexpr bool kScatter = false;\n", name,
          EU.size());
  appendf(s, "  static constexpr bool kSmall = false, kPerm = false, kMulti = false;\n");
  appendf(s, "  static constexpr uint8_t kPoint[%zu] = {", EU.empty() ? (size_t)1 : EU.size());
  for (int e : EU) appendf(s, "%d, ", e);
  appendf(s, "};\n");
  const auto rows = all_bitrows(A, (int)EU.size(), K);
  size_t total = 0;
  for (size_t m = 0; m < EU.size(); ++m) {
    char nm[32];
    std::snprintf(nm, sizeof nm, "fill%zu", m);
    total += emit_program(s, nm, rows, K, row_range(16 * (int)m, 16), pb, im, prefetch);
  }
  appendf(s, "  template <typename In>\n  __device__ __forceinline__ static void fill(int w, const In &IN4, uint32_t (&acc)[16]) {\n");
  appendf(s, "    switch (w) {\n");
  for (size_t m = 0; m < EU.size(); ++m) appendf(s, "      case %zu: fill%zu(IN4, acc); break;\n", m, m);
  appendf(s, "      default: break;\n    }\n  }\n};\n");
  return total;
}

// Column-partitioned fill ("scatter") programs of one survivor set: wave w
// takes the survivors of rank 4w..4w+3 (spoints ascending; the host sorts
// the launch's survivors by point, so these are the ones wave w itself
// stored in stage 1) and computes their share of every erased point below K
// -- the same Lagrange map as emit_fill_programs, partitioned by columns
// instead of rows.  The shares meet in LDS through XOR atomics.  Fewer XORs
// than the row form (k = 16: ~2.1K vs ~2.6K per tile with one Paar block of
// all four survivors; k = 32: ~6.9K vs ~9.8K, balanced over all waves) and
// a quarter of its LDS reads.  Programs cover at most kScatterPart erased
// points each (register pressure).
constexpr int kScatterPart = 4;
// survivors per Paar block of a scatter program (-DVDS_JIT_SPB=n overrides).
// 2 spills 5-7 VGPRs and is still the fastest: same box, three rounds, k=16
// repair 14.13-14.24 ms (2) vs 14.29-14.63 (1) vs 14.43-14.50 (row form);
// 3 or 4 spill 66-174 (profiles/round3/ab/scatter_ab.log).
#ifndef VDS_JIT_SPB
#define VDS_JIT_SPB 2
#endif
#ifndef VDS_JIT_SPREFETCH
#define VDS_JIT_SPREFETCH 1  // (a block's LDS reads issued before the previous block's XORs)
#endif
static_assert(VDS_JIT_SPB >= 1 && VDS_JIT_SPB <= 4, "scatter block size");
constexpr int scatter_block() { return VDS_JIT_SPB; }
// `targets` (optional): the points to compute instead of the erased points
// below K -- the regenerate kernel's targets, every erased point of 0..N-1.
inline size_t emit_fill_scatter(std::string &s, const char *name, int K, const std::vector<int> &spoints,
                                const std::vector<int> *targets = nullptr) {
  std::vector<int> EU;
  if (targets) {
    EU = *targets;
  } else {
    for (int a = 0; a < K; ++a)
      if (std::find(spoints.begin(), spoints.end(), a) == spoints.end()) EU.push_back(a);
  }
  const int F = (int)EU.size(), WV = K / 4, parts = (F + kScatterPart - 1) / kScatterPart;
  std::vector<uint32_t> A((size_t)F * K);
  for (int m = 0; m < F; ++m)
    for (int j = 0; j < K; ++j) {
      uint32_t num = 1, den = 1;
      for (int t = 0; t < K; ++t)
        if (t != j) {
          num = vds_ec::gf16_mul(num, (uint32_t)(EU[m] ^ spoints[t]));
          den = vds_ec::gf16_mul(den, (uint32_t)(spoints[j] ^ spoints[t]));
        }
      A[(size_t)m * K + j] = vds_ec::gf16_mul(num, vds_ec::gf16_inv(den));
    }
  const auto rows = all_bitrows(A, F, K);
  appendf(s, "struct %s {\n  static constexpr int kFill = %d;\n  static constexpr bool kScatter = true;\n", name, F);
  appendf(s, "  static constexpr bool kSmall = false, kPerm = false, kMulti = false;\n");
  appendf(s, "  static constexpr int kParts = %d, kPart = %d;\n", parts, kScatterPart);
  appendf(s, "  static constexpr uint8_t kPoint[%d] = {", F ? F : 1);
  for (int e : EU) appendf(s, "%d, ", e);
  appendf(s, "};\n");
  // the survivors by rank (wave w loaded ranks 4w..4w+3 in stage 1: the
  // kernel serves IN4 from those registers, restore_syn.hpp FillRegIn)
  appendf(s, "  static constexpr uint8_t kSurv[%d] = {", K);
  for (int j = 0; j < K; ++j) appendf(s, "%d, ", spoints[j]);
  appendf(s, "};\n");
  size_t total = 0;
  for (int w = 0; w < WV; ++w)
    for (int q = 0; q < parts; ++q) {
      const int m0 = q * kScatterPart, m1 = std::min(F, m0 + kScatterPart);
      std::vector<std::vector<int>> sub;
      for (int r = 16 * m0; r < 16 * m1; ++r) {
        std::vector<int> row;
        for (int x : rows[r])
          if (x >= 64 * w && x < 64 * w + 64) row.push_back(x - 64 * w);
        sub.push_back(row);
      }
      char nm[48];
      std::snprintf(nm, sizeof nm, "fill%d_%d", w, q);
      InputMap im;  // (this wave's survivors, in their own LDS slots)
      for (int i = 0; i < 4; ++i) im.map.push_back(spoints[4 * w + i]);
      total += emit_program(s, nm, sub, 4, row_range(0, (int)sub.size()), scatter_block(), im,
                            VDS_JIT_SPREFETCH != 0);
    }
  for (int q = 0; q < parts; ++q) {
    appendf(s, "  template <typename In>\n  __device__ __forceinline__ static void fill_part%d(int w, const In &IN4, uint32_t (&acc)[%d]) {\n",
            q, 16 * kScatterPart);
    appendf(s, "    switch (w) {\n");
    for (int w = 0; w < WV; ++w)
      appendf(s, "      case %d: fill%d_%d(IN4, reinterpret_cast<uint32_t(&)[%d]>(acc)); break;\n", w, w, q,
              16 * (std::min(F, q * kScatterPart + kScatterPart) - q * kScatterPart));
    appendf(s, "      default: break;\n    }\n  }\n");
  }
  appendf(s, "  template <typename In>\n  __device__ __forceinline__ static void fill_part(int q, int w, const In &IN4, uint32_t (&acc)[%d]) {\n",
          16 * kScatterPart);
  appendf(s, "    switch (q) {\n");
  for (int q = 0; q < parts; ++q) appendf(s, "      case %d: fill_part%d(w, IN4, acc); break;\n", q, q);
  appendf(s, "      default: break;\n    }\n  }\n};\n");
  return total;
}

// "Own-group" fill of one survivor set (k = 16, four waves; restore only):
// when each wave's interpolation group {4w..4w+3} holds exactly one erased
// point, wave w computes that point from all K survivors -- its own four
// (ranks 4w..4w+3) from its stage-1 registers, the rest from LDS -- and
// hands it to its S1 in registers (restore_syn.hpp OwnIn / kOwn): no LDS
// atomics, no zeroed slots, and no barrier between the fill and S1.  The
// row programs of emit_fill_programs, one per wave.  Returns 0 (nothing
// emitted) when the set does not have one erased point per group.
inline bool fill_own_eligible(int K, const std::vector<int> &spoints) {
  if (K != 16) return false;
  for (int w = 0; w < K / 4; ++w) {
    int e = 0;
    for (int a = 4 * w; a < 4 * w + 4; ++a) e += std::find(spoints.begin(), spoints.end(), a) == spoints.end();
    if (e != 1) return false;
  }
  return true;
}
inline size_t emit_fill_own(std::string &s, const char *name, int K, const std::vector<int> &spoints, int pb,
                            bool prefetch = true) {
  if (!fill_own_eligible(K, spoints)) return 0;
  std::vector<int> EU;  // ascending: EU[w] is the erased point of group w
  for (int a = 0; a < K; ++a)
    if (std::find(spoints.begin(), spoints.end(), a) == spoints.end()) EU.push_back(a);
  const int F = (int)EU.size();
  std::vector<uint32_t> A((size_t)F * K);
  for (int m = 0; m < F; ++m)
    for (int j = 0; j < K; ++j) {
      uint32_t num = 1, den = 1;
      for (int t = 0; t < K; ++t)
        if (t != j) {
          num = vds_ec::gf16_mul(num, (uint32_t)(EU[m] ^ spoints[t]));
          den = vds_ec::gf16_mul(den, (uint32_t)(spoints[j] ^ spoints[t]));
        }
      A[(size_t)m * K + j] = vds_ec::gf16_mul(num, vds_ec::gf16_inv(den));
    }
  InputMap im;
  im.map = spoints;
  appendf(s, "struct %s {\n  static constexpr int kFill = %d;\n  static constexpr bool kScatter = false, kOwn = true;\n",
          name, F);
  appendf(s, "  static constexpr bool kSmall = false, kPerm = false, kMulti = false;\n");
  appendf(s, "  static constexpr uint8_t kPoint[%d] = {", F);
  for (int e : EU) appendf(s, "%d, ", e);
  appendf(s, "};\n  static constexpr uint8_t kSurv[%d] = {", K);
  for (int j = 0; j < K; ++j) appendf(s, "%d, ", spoints[j]);
  appendf(s, "};\n");
  const auto rows = all_bitrows(A, F, K);
  size_t total = 0;
  for (int m = 0; m < F; ++m) {
    char nm[32];
    std::snprintf(nm, sizeof nm, "own%d", m);
    total += emit_program(s, nm, rows, K, row_range(16 * m, 16), pb, im, prefetch);
  }
  appendf(s, "  template <int W, typename In>\n  __device__ __forceinline__ static void own(const In &IN4, uint32_t (&acc)[16]) {\n");
  for (int m = 0; m < F; ++m) appendf(s, "    %sif constexpr (W == %d) own%d(IN4, acc);\n", m ? "else " : "", m, m);
  appendf(s, "  }\n};\n");
  return total;
}

}  // namespace xorgen
