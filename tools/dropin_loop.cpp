// dropin_loop.cpp -- the unchanged caller loop through the drop-in chunk.h
// (VERDICT r2 #6): save_temp builds 64 generators once (_client ctor,
// dht_network_client.cpp:57-59) and calls generators_[r]->write(s, data,
// size) for r = 0..63 on every 64 KiB upload (dht_network_client.cpp:74-79).
// Each call is one synchronous vds_ec_encode16_host of one replica.  Times
// that loop per object, and beside it the batched call a caller could adopt
// (vds_ec_encode16_host, all 64 replicas at once).  Prints one JSON line.
//
//   g++ -O2 -std=c++20 -fcoroutines -I include -I vds_amd/include/vds_data
//       -I vds_amd/include/vds_core_compat tools/dropin_loop.cpp
//       -L vds_amd -lvds_ec -Wl,-rpath,$PWD/vds_amd -o tools/dropin_loop
//   tools/dropin_loop [objects]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <random>
#include <vector>

#include "chunk.h"
#include "vds_ec.h"

using clk = std::chrono::steady_clock;

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
  auto loop = [&](const std::vector<uint8_t> &data) {
    for (uint16_t r = 0; r < n; ++r) {
      vds::binary_serializer s;
      auto res = gens[r]->write(s, data.data(), data.size());
      if (res.has_error()) {
        std::fprintf(stderr, "write failed: %s\n", res.error()->what());
        std::exit(1);
      }
      sink[r % L] ^= s.get_buffer()[0];
    }
  };
  loop(objs[0]);  // warm-up: host context, device buffers
  const auto t0 = clk::now();
  for (int o = 0; o < objects; ++o) loop(objs[o]);
  const double per_obj = std::chrono::duration<double>(clk::now() - t0).count() / objects;

  std::vector<uint16_t> ids(n);
  for (uint16_t r = 0; r < n; ++r) ids[r] = r;
  std::vector<std::vector<uint8_t>> outs(n, std::vector<uint8_t>(L));
  std::vector<uint8_t *> op(n);
  for (uint16_t r = 0; r < n; ++r) op[r] = outs[r].data();
  vds_ec_encode16_host(k, ids.data(), n, objs[0].data(), size, op.data(), 0);
  const auto t1 = clk::now();
  for (int o = 0; o < objects; ++o)
    if (vds_ec_encode16_host(k, ids.data(), n, objs[o].data(), size, op.data(), 0)) return 1;
  const double per_obj_batch = std::chrono::duration<double>(clk::now() - t1).count() / objects;
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
  std::printf("{\"shape\": \"k=32, n=64, 64 KiB object\", \"objects\": %d, "
              "\"per_replica_loop_us_per_object\": %.1f, \"per_replica_call_us\": %.2f, "
              "\"per_replica_loop_MiBps\": %.1f, \"batched_call_us_per_object\": %.1f, \"batched_MiBps\": %.1f, "
              "\"reference_cpu_us_per_object\": 11000}\n",
              objects, per_obj * 1e6, per_obj * 1e6 / n, size / per_obj / (1 << 20), per_obj_batch * 1e6,
              size / per_obj_batch / (1 << 20));
  return 0;
}
