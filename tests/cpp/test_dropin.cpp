// Re-hosts lboss75/vds tests/test_vds_data (gf_tests.cpp, chunk_tests.cpp) on
// the drop-in headers vds_amd/include/vds_data/, unchanged in substance but
// seeded (the reference seeds std::srand(time(0)), test_vds_data.cpp:8-13)
// and without gtest (not installed in this image).
//
//   test_dropin gf      -- gf_tests.test_mul / test_math          (no GPU)
//   test_dropin chunk   -- chunk_tests.test_chunks{,16,_storage}  (GPU)
//                          + chunk_output_async == one-shot write
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#include "chunk.h"
#include "chunk_storage.h"
#include "gf.h"

static int g_fail = 0;
#define ASSERT_EQ(a, b)                                                                      \
  do {                                                                                       \
    if (!((a) == (b))) {                                                                     \
      std::printf("FAIL %s:%d %s == %s\n", __FILE__, __LINE__, #a, #b);                      \
      ++g_fail;                                                                              \
      return;                                                                                \
    }                                                                                        \
  } while (0)
#define GET_EXPECTED_TEST(var, v)                                                            \
  auto __r##var = (v);                                                                       \
  if (__r##var.has_error()) {                                                                \
    std::printf("FAIL %s:%d %s\n", __FILE__, __LINE__, __r##var.error()->what());             \
    ++g_fail;                                                                                \
    return;                                                                                  \
  }                                                                                          \
  auto var = std::move(__r##var.value());

// gf_tests.cpp:9-38
static void gf_test_mul() {
  static uint8_t original[8][8] = {{0, 0, 0, 0, 0, 0, 0, 0}, {0, 1, 2, 3, 4, 5, 6, 7}, {0, 2, 4, 6, 3, 1, 7, 5},
                                   {0, 3, 6, 5, 7, 4, 1, 2}, {0, 4, 3, 7, 6, 2, 5, 1}, {0, 5, 1, 4, 2, 7, 3, 6},
                                   {0, 6, 7, 1, 5, 3, 2, 4}, {0, 7, 5, 2, 1, 6, 4, 3}};
  for (uint8_t i = 1; i < 8; ++i)
    for (uint8_t j = 1; j < 8; ++j) {
      uint8_t l[1] = {i}, r[1] = {j}, res[1] = {original[i][j]};
      ASSERT_EQ(vds::gf<3>(res), vds::gf<3>(l) * vds::gf<3>(r));
    }
}

// gf_tests.cpp:41-64
static void gf_test_math() {
  vds::gf_math<uint8_t> math;
  for (int i = 0; i < 1000; ++i) {
    uint8_t x = std::rand() & 0xFF, y = std::rand() & 0xFF;
    uint8_t gx[] = {x}, gy[] = {y};
    uint8_t z = (vds::gf<8>(gx) * vds::gf<8>(gy)).data()[0];
    uint8_t p = (vds::gf<8>(gx) + vds::gf<8>(gy)).data()[0];
    ASSERT_EQ(math.mul(x, y), z);
    ASSERT_EQ(math.mul(y, x), z);
    if (z != 0) {
      ASSERT_EQ(math.div(z, x), y);
      ASSERT_EQ(math.div(z, y), x);
    }
    ASSERT_EQ(math.add(x, y), p);
    ASSERT_EQ(math.sub(p, x), y);
  }
  // the production field against gf<16>
  static vds::gf_math<uint16_t> m16;
  for (int i = 0; i < 100000; ++i) {
    uint16_t x = std::rand() & 0xFFFF, y = std::rand() & 0xFFFF;
    uint8_t gx[] = {uint8_t(x), uint8_t(x >> 8)}, gy[] = {uint8_t(y), uint8_t(y >> 8)};
    auto z = vds::gf<16>(gx) * vds::gf<16>(gy);
    ASSERT_EQ(m16.mul(x, y), uint16_t(z.data()[0] | (z.data()[1] << 8)));
    if (x && y) ASSERT_EQ(m16.div(m16.mul(x, y), y), x);
  }
}

template <typename cell>
static void chunk_roundtrip(int limit) {
  int size = 1 + std::rand() % 1000;
  size -= size % 3;
  std::vector<cell> data(size);
  for (auto &d : data) d = cell(std::rand() & limit);
  int r1 = std::rand() % 256, r2, r3;
  do r2 = std::rand() % 256; while (r2 == r1);
  do r3 = std::rand() % 256; while (r3 == r1 || r3 == r2);
  vds::chunk_generator<cell> g1(3, cell(r1)), g2(3, cell(r2)), g3(3, cell(r3));
  vds::chunk<cell> c1(g1, data.data(), size), c2(g2, data.data(), size), c3(g3, data.data(), size);
  std::vector<cell> result;
  cell ns[] = {cell(r1), cell(r2), cell(r3)};
  const vds::chunk<cell> *chunks[] = {&c1, &c2, &c3};
  vds::chunk_restore<cell>(3, ns).restore(result, chunks);
  ASSERT_EQ(size_t(size), result.size());
  for (int i = 0; i < size; ++i) ASSERT_EQ(data[i], result[i]);
}

// chunk_tests.cpp:112-162
static void chunk_test_storage() {
  const uint16_t horcrux_count = 1000, min_horcrux = 800;
  int size = 2000 + std::rand() % 4001;
  std::vector<uint8_t> data(size);
  for (auto &d : data) d = uint8_t(std::rand());
  vds::chunk_storage storage(min_horcrux);
  std::unordered_map<uint16_t, vds::const_data_buffer> horcruxes;
  while (horcruxes.size() < min_horcrux) {
    uint16_t replica;
    do replica = uint16_t(std::rand() % horcrux_count); while (horcruxes.count(replica));
    GET_EXPECTED_TEST(hr, storage.generate_replica(replica, data.data(), size));
    horcruxes[replica] = hr;
  }
  GET_EXPECTED_TEST(result, storage.restore_data(horcruxes));
  ASSERT_EQ(size_t(size), result.size());
  ASSERT_EQ(0, std::memcmp(data.data(), result.data(), size));
}

// The repair route of sync_process.cpp:313-335 (restore_data, then
// generate_replica of the missing replicas) against the fused
// regenerate_replicas, and the batched replica names against the replicas.
static void chunk_test_regenerate() {
  const uint16_t k = 16, n = 20;
  const int size = 3 * 65536 + std::rand() % 5000;
  std::vector<uint8_t> data(size);
  for (auto &d : data) d = uint8_t(std::rand());
  vds::chunk_storage storage(k);
  std::vector<uint16_t> ids(n);
  for (uint16_t i = 0; i < n; ++i) ids[i] = i;
  std::vector<vds::const_data_buffer> names;
  GET_EXPECTED_TEST(reps, storage.generate_replicas(ids, data.data(), size, names));
  ASSERT_EQ(size_t(n), reps.size());
  ASSERT_EQ(size_t(n), names.size());
  std::unordered_map<uint16_t, vds::const_data_buffer> survivors;
  for (uint16_t r = 0; r < n; ++r)
    if (r % 5) survivors[r] = reps[r];
  GET_EXPECTED_TEST(object, storage.restore_data(survivors));
  const std::vector<uint16_t> lost = {0, 5, 10, 15};
  GET_EXPECTED_TEST(fused, storage.regenerate_replicas(survivors, lost));
  for (size_t i = 0; i < lost.size(); ++i) {
    GET_EXPECTED_TEST(again, storage.generate_replica(lost[i], object.data(), object.size()));
    ASSERT_EQ(again.size(), fused[i].size());
    ASSERT_EQ(0, std::memcmp(again.data(), fused[i].data(), again.size()));
    ASSERT_EQ(0, std::memcmp(reps[lost[i]].data(), fused[i].data(), again.size()));
  }
  // batched restore_data: the same objects as one call per object
  std::vector<std::unordered_map<uint16_t, vds::const_data_buffer>> batch = {survivors, survivors};
  batch[1].erase(1);
  batch[1][0] = reps[0];
  GET_EXPECTED_TEST(objects, storage.restore_datas(batch));
  ASSERT_EQ(size_t(2), objects.size());
  for (auto &o : objects) {
    ASSERT_EQ(object.size(), o.size());
    ASSERT_EQ(0, std::memcmp(object.data(), o.data(), o.size()));
  }
  batch[0].erase(2);  // k - 1 horcruxes: restore_data's error
  ASSERT_EQ(false, storage.restore_datas(batch).has_value());
  // names: the replica hash is a function of the bytes only
  for (uint16_t r = 0; r < n; ++r) {
    ASSERT_EQ(size_t(32), names[r].size());
    for (uint16_t q = 0; q < r; ++q) ASSERT_EQ(false, std::memcmp(names[r].data(), names[q].data(), 32) == 0);
  }
}

// chunk_output_async (chunk.h:116-176) is byte-identical to one-shot write.
struct collect : vds::stream_output_async<uint8_t> {
  std::vector<uint8_t> bytes;
  bool closed = false;
  vds::async_task<vds::expected<void>> write_async(const uint8_t *d, size_t len) override {
    if (len == 0) closed = true;
    else bytes.insert(bytes.end(), d, d + len);
    co_return vds::expected<void>();
  }
};

static void chunk_test_output_async() {
  for (size_t size : {size_t(0), size_t(5), size_t(32 * 1024), size_t(32 * 1024 * 3 + 17), size_t(100000)}) {
    std::vector<uint8_t> data(size);
    for (auto &d : data) d = uint8_t(std::rand());
    vds::chunk_generator<uint16_t> g(16, 7);
    auto sink = std::make_shared<collect>();
    vds::chunk_output_async<uint16_t> out(g, sink);
    size_t pos = 0;
    while (pos < size) {  // ragged pieces
      size_t l = std::min(size - pos, size_t(1 + std::rand() % 9000));
      auto r = out.write_async(data.data() + pos, l).get();
      ASSERT_EQ(false, r.has_error());
      pos += l;
    }
    auto r = out.write_async(nullptr, 0).get();
    ASSERT_EQ(false, r.has_error());
    ASSERT_EQ(true, sink->closed);
    vds::binary_serializer s;
    auto w = g.write(s, data.data(), size);
    ASSERT_EQ(false, w.has_error());
    ASSERT_EQ(s.size(), sink->bytes.size());
    ASSERT_EQ(0, std::memcmp(s.get_buffer(), sink->bytes.data(), s.size()));
  }
}

int main(int argc, char **argv) {
  const std::string mode = argc > 1 ? argv[1] : "gf";
  std::srand(argc > 2 ? std::atoi(argv[2]) : 12345);
  if (mode == "gf") {
    gf_test_mul();
    gf_test_math();
  } else {
    for (int i = 0; i < 20; ++i) chunk_roundtrip<uint8_t>(0xFF);
    for (int i = 0; i < 20; ++i) chunk_roundtrip<uint16_t>(0xFFFF);
    chunk_test_storage();
    chunk_test_regenerate();
    chunk_test_output_async();
  }
  std::printf("%s %s (%d failures)\n", mode.c_str(), g_fail ? "FAILED" : "OK", g_fail);
  return g_fail ? 1 : 0;
}
