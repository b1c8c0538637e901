// Size XOR programs for candidate decode formulations (offline study tool).
#include <chrono>
#include <cstdio>
#include <vector>

#include "../../include/vds_ec.h"
#include "../../vds_amd/csrc/gf_common.hpp"
#include "../../vds_amd/csrc/xorprog.hpp"

using namespace vds_ec;

// rows for y = M x over GF(2^16), M: R x C constants; planes (m,i) <- (j,b)
static std::vector<std::vector<int>> bitrows(const std::vector<uint16_t> &M, int R, int C) {
  std::vector<std::vector<int>> rows(16 * R);
  for (int m = 0; m < R; ++m)
    for (int j = 0; j < C; ++j)
      for (int b = 0; b < 16; ++b) {
        const uint32_t v = gf16_mul(M[m * C + j], 1u << b);
        for (int i = 0; i < 16; ++i)
          if ((v >> i) & 1) rows[16 * m + i].push_back(16 * j + b);
      }
  return rows;
}

static void report(const char *name, const std::vector<uint16_t> &M, int R, int C, int split) {
  auto t0 = std::chrono::steady_clock::now();
  size_t ones = 0, total = 0;
  auto all = bitrows(M, R, C);
  for (auto &r : all) ones += r.size();
  // split outputs into `split` independent programs (one per wave)
  for (int w = 0; w < split; ++w) {
    std::vector<std::vector<int>> part(all.begin() + w * all.size() / split, all.begin() + (w + 1) * all.size() / split);
    total += xorgen::paar(16 * C, part).xor_count();
  }
  double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  std::printf("%-34s ones=%6zu naive=%6zu paar(split %d)=%6zu  (%.1fs)\n", name, ones, ones - 16 * R, split, total, s);
}

int main() {
  for (int k : {16, 32}) {
    std::vector<uint16_t> nodes(k), M(k * k);
    for (int i = 0; i < k; ++i) nodes[i] = i;
    vds_ec_inverse16(k, nodes.data(), M.data());
    char nm[64];
    std::snprintf(nm, sizeof nm, "V_F^-1 F={0..%d}", k - 1);
    report(nm, M, k, k, 1);
    report(nm, M, k, k, k / 4);
  }
  {  // direct decode matrix for erasures {0,5,10,15} of 20
    std::vector<uint16_t> nodes, M(256);
    for (int r = 0; r < 20; ++r)
      if (r % 5) nodes.push_back(r);
    vds_ec_inverse16(16, nodes.data(), M.data());
    report("V_S^-1 S=20\\{0,5,10,15}", M, 16, 16, 1);
    report("V_S^-1 S=20\\{0,5,10,15}", M, 16, 16, 4);
  }
  {  // syndrome rows: S_j = sum_a v_a a^j c_a, a in 0..19, j < 4
    const int n = 20, m = 4;
    std::vector<uint16_t> W(m * n);
    for (int a = 0; a < n; ++a) {
      uint32_t prod = 1;
      for (int b = 0; b < n; ++b)
        if (b != a) prod = gf16_mul(prod, a ^ b);
      const uint32_t v = gf16_inv(prod);
      for (int j = 0; j < m; ++j) W[j * n + a] = gf16_mul(v, gf16_pow(a, j) * (j || a ? 1 : 1));
    }
    report("syndromes 4 x 20", W, m, n, 1);
    report("syndromes 4 x 20", W, m, n, 4);
  }
  // encode matrix (for reference against Horner)
  {
    std::vector<uint16_t> E(20 * 16);
    for (int r = 0; r < 20; ++r)
      for (int j = 0; j < 16; ++j) E[r * 16 + j] = gf16_vandermonde(r, j);
    report("encode V 20 x 16", E, 20, 16, 4);
  }
}
