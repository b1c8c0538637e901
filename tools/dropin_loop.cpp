// dropin_loop.cpp -- per-call latency of the live upload and download paths
// at the production shape (k = 32, n = 64, 64 KiB objects), one caller thread
// (the reference runs the codec on the single DB thread_apartment,
// database_p.h:302-303).  Prints one JSON line with p50 / p99 / mean per call:
//
//  - save_temp through the UNCHANGED drop-in chunk.h: 64 generators built
//    once (_client ctor, dht_network_client.cpp:57-59), then
//    generators_[r]->write(s, data, size) for r = 0..63 per upload
//    (dht_network_client.cpp:74-79): per write call and per object;
//  - vds_ec_save_temp16_host: the same upload as one call (all 64 replicas,
//    their SHA-256 names and the body hash on the device: upload_data +
//    save_temp, server_api.cpp:12-30, dht_network_client.cpp:62-107);
//  - vds_ec_encode16_host: all 64 replicas, no hashes;
//  - vds_ec_restore16_host: one download (restore_async's chunk_restore from
//    the first 32 replicas found, dht_network_client.cpp:851-901), here 0..31
//    minus one lost replica plus replica 32.
//
//   g++ -O2 -std=c++20 -fcoroutines -I include -I vds_amd/include/vds_data
//       -I vds_amd/include/vds_core_compat tools/dropin_loop.cpp
//       -L vds_amd -lvds_ec -Wl,-rpath,$PWD/vds_amd -o tools/dropin_loop
//   tools/dropin_loop [objects]
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <random>
#include <vector>

#include "chunk.h"
#include "vds_ec.h"

using clk = std::chrono::steady_clock;

namespace {

struct Stats {
  double p50, p99, mean;
};

Stats stats(std::vector<double> us) {
  std::sort(us.begin(), us.end());
  double sum = 0;
  for (double v : us) sum += v;
  auto at = [&](double q) { return us[std::min(us.size() - 1, (size_t)(q * (double)(us.size() - 1) + 0.5))]; };
  return {at(0.50), at(0.99), sum / (double)us.size()};
}

double us_since(clk::time_point t) { return std::chrono::duration<double, std::micro>(clk::now() - t).count(); }

void print(const char *name, const Stats &s, bool comma = true) {
  std::printf("\"%s\": {\"p50_us\": %.2f, \"p99_us\": %.2f, \"mean_us\": %.2f}%s", name, s.p50, s.p99, s.mean,
              comma ? ", " : "");
}

}  // namespace

int main(int argc, char **argv) {
  const int objects = argc > 1 ? std::atoi(argv[1]) : 200;
  constexpr uint16_t k = 32, n = 64;  // MIN_HORCRUX, GENERATE_HORCRUX (dht_network.h:22-25)
  constexpr size_t size = 65536;      // the web client's block (web/src/store/vds_api.jsx:76)
  std::mt19937_64 rng(7);
  std::vector<std::vector<uint8_t>> objs(objects, std::vector<uint8_t>(size));
  for (auto &o : objs)
    for (auto &b : o) b = (uint8_t)rng();
  std::vector<std::unique_ptr<vds::chunk_generator<uint16_t>>> gens;
  for (uint16_t r = 0; r < n; ++r) gens.emplace_back(new vds::chunk_generator<uint16_t>(k, r));
  const uint64_t L = vds_ec_replica_size(2, k, size, 0);
  std::vector<uint8_t> sink(L);
  std::vector<double> call_us, loop_us;
  call_us.reserve((size_t)objects * n);
  auto loop = [&](const std::vector<uint8_t> &data, bool timed) {
    const auto t0 = clk::now();
    for (uint16_t r = 0; r < n; ++r) {
      const auto t1 = clk::now();
      vds::binary_serializer s;
      auto res = gens[r]->write(s, data.data(), data.size());
      if (res.has_error()) {
        std::fprintf(stderr, "write failed: %s\n", res.error()->what());
        std::exit(1);
      }
      sink[r % L] ^= s.get_buffer()[0];
      if (timed) call_us.push_back(us_since(t1));
    }
    if (timed) loop_us.push_back(us_since(t0));
  };
  loop(objs[0], false);  // warm-up: host context, device buffers
  for (int o = 0; o < objects; ++o) loop(objs[o], true);

  std::vector<uint16_t> ids(n);
  for (uint16_t r = 0; r < n; ++r) ids[r] = r;
  std::vector<std::vector<uint8_t>> outs(n, std::vector<uint8_t>(L));
  std::vector<uint8_t *> op(n);
  for (uint16_t r = 0; r < n; ++r) op[r] = outs[r].data();
  std::vector<double> enc_us, st_us, rs_us;
  if (vds_ec_encode16_host(k, ids.data(), n, objs[0].data(), size, op.data(), 0)) return 1;
  for (int o = 0; o < objects; ++o) {
    const auto t = clk::now();
    if (vds_ec_encode16_host(k, ids.data(), n, objs[o].data(), size, op.data(), 0)) return 1;
    enc_us.push_back(us_since(t));
  }
  // the loop's replicas equal the batched call's
  for (uint16_t r = 0; r < n; ++r) {
    vds::binary_serializer s;
    (void)gens[r]->write(s, objs[objects - 1].data(), size);
    for (uint64_t i = 0; i < L; ++i)
      if (s.get_buffer()[i] != outs[r][i]) {
        std::fprintf(stderr, "replica %u differs at %llu\n", r, (unsigned long long)i);
        return 1;
      }
  }
  std::vector<uint8_t> digests((size_t)n * 32), body(32);
  uint32_t rsize = 0;
  if (vds_ec_save_temp16_host(k, n, objs[0].data(), size, op.data(), digests.data(), body.data(), &rsize)) return 1;
  for (int o = 0; o < objects; ++o) {
    const auto t = clk::now();
    if (vds_ec_save_temp16_host(k, n, objs[o].data(), size, op.data(), digests.data(), body.data(), &rsize)) return 1;
    st_us.push_back(us_since(t));
  }
  // one download: survivors 0..32 minus replica 5 (the first 32 found)
  std::vector<uint16_t> nodes;
  std::vector<const uint8_t *> chunks;
  for (uint16_t r = 0; r <= 32; ++r)
    if (r != 5) {
      nodes.push_back(r);
      chunks.push_back(outs[r].data());
    }
  std::vector<uint8_t> back(size + 2 * k);
  uint64_t got = 0;
  if (vds_ec_restore16_host(k, nodes.data(), chunks.data(), L, back.data(), &got, 0)) return 1;
  for (int o = 0; o < objects; ++o) {
    const auto t = clk::now();
    if (vds_ec_restore16_host(k, nodes.data(), chunks.data(), L, back.data(), &got, 0)) return 1;
    rs_us.push_back(us_since(t));
  }
  if (got != size || !std::equal(back.begin(), back.begin() + size, objs[objects - 1].begin())) {
    std::fprintf(stderr, "restore differs\n");
    return 1;
  }
  const Stats sl = stats(loop_us);
  std::printf("{\"shape\": \"k=32, n=64, 64 KiB object, one caller thread\", \"objects\": %d, ", objects);
  print("dropin_write_call", stats(call_us));
  print("dropin_write_loop_per_object", sl);
  std::printf("\"dropin_loop_MiBps\": %.1f, ", size / sl.mean / 1.048576);
  print("save_temp16_host_per_object", stats(st_us));
  print("encode16_host_per_object", stats(enc_us));
  print("restore16_host_per_object", stats(rs_us));
  std::printf("\"reference_cpu_us_per_object\": 11000}\n");
  return 0;
}
