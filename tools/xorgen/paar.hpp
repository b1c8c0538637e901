// paar.hpp -- greedy XOR common-subexpression elimination (Paar's heuristic)
// for a fixed GF(2) matrix.  Used offline to turn the bit-matrix of a
// compile-time GF(2^16) linear map into a short straight-line XOR program.
//
// Input : rows[r] = set of input columns whose XOR is output r.
// Output: temps (t = a ^ b, in creation order, ids >= ncols) and the final
//         rows (each a list of column / temp ids to XOR together).
#pragma once

#include <algorithm>
#include <cstdint>
#include <unordered_map>
#include <unordered_set>
#include <vector>

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
  cnt.reserve(1 << 22);
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

}  // namespace xorgen
