// chunk_storage.cpp -- drop-in for lboss75/vds kernel/vds_data/chunk_storage.cpp
// (chunk_storage.cpp:10-86) on the MI355X codec.
#include "chunk_storage.h"

#include <map>
#include <memory>

#include "chunk.h"

namespace vds {

class _chunk_storage {
 public:
  explicit _chunk_storage(uint16_t min_horcrux) : min_horcrux_(min_horcrux) {}

  // chunk_storage.cpp:41-60: lazily cached generator per replica, then write.
  expected<const_data_buffer> generate_replica(uint16_t replica, const void *data, size_t size) {
    auto p = generators_.find(replica);
    if (p == generators_.end())
      p = generators_.emplace(replica, std::make_unique<chunk_generator<uint16_t>>(min_horcrux_, replica)).first;
    binary_serializer s;
    CHECK_EXPECTED(p->second->write(s, data, size));
    return s.move_data();
  }

  expected<std::vector<const_data_buffer>> generate_replicas(const std::vector<uint16_t> &replicas, const void *data,
                                                             size_t size) {
    const uint64_t len = vds_ec_replica_size(2, min_horcrux_, size, 0);
    std::vector<std::vector<uint8_t>> bufs(replicas.size(), std::vector<uint8_t>(len ? len : 1));
    std::vector<uint8_t *> outs(replicas.size());
    for (size_t i = 0; i < replicas.size(); ++i) outs[i] = bufs[i].data();
    const int rc = vds_ec_encode16_host(min_horcrux_, replicas.data(), uint32_t(replicas.size()),
                                        static_cast<const uint8_t *>(data), size, outs.data(), 0);
    if (rc != VDS_EC_OK) return make_unexpected<std::runtime_error>(vds_ec_strerror(rc));
    std::vector<const_data_buffer> result;
    result.reserve(replicas.size());
    for (auto &b : bufs) result.emplace_back(b.data(), len);
    return result;
  }

  expected<std::vector<const_data_buffer>> generate_replicas(const std::vector<uint16_t> &replicas, const void *data,
                                                             size_t size, std::vector<const_data_buffer> &hashes) {
    const uint64_t len = vds_ec_replica_size(2, min_horcrux_, size, 0);
    std::vector<std::vector<uint8_t>> bufs(replicas.size(), std::vector<uint8_t>(len ? len : 1));
    std::vector<uint8_t *> outs(replicas.size());
    for (size_t i = 0; i < replicas.size(); ++i) outs[i] = bufs[i].data();
    std::vector<uint8_t> names(32 * (replicas.size() ? replicas.size() : 1));
    const int rc = vds_ec_encode16_hash_host(min_horcrux_, replicas.data(), uint32_t(replicas.size()),
                                             static_cast<const uint8_t *>(data), size, outs.data(), names.data(), 0);
    if (rc != VDS_EC_OK) return make_unexpected<std::runtime_error>(vds_ec_strerror(rc));
    std::vector<const_data_buffer> result;
    hashes.clear();
    for (size_t i = 0; i < bufs.size(); ++i) {
      result.emplace_back(bufs[i].data(), len);
      hashes.emplace_back(names.data() + 32 * i, 32);
    }
    return result;
  }

  expected<std::vector<const_data_buffer>> regenerate_replicas(
      const std::unordered_map<uint16_t, const_data_buffer> &horcruxes, const std::vector<uint16_t> &targets) {
    if (min_horcrux_ != horcruxes.size()) return make_unexpected<std::runtime_error>("Error at restoring data");
    const size_t size = horcruxes.begin()->second.size();
    std::vector<uint16_t> nodes;
    std::vector<const uint8_t *> chunks;
    for (auto &p : horcruxes) {
      if (size != p.second.size()) return make_unexpected<std::runtime_error>("Error at restoring data");
      nodes.push_back(p.first);
      chunks.push_back(p.second.data());
    }
    std::vector<std::vector<uint8_t>> bufs(targets.size(), std::vector<uint8_t>(size ? size : 1));
    std::vector<uint8_t *> outs(targets.size());
    for (size_t i = 0; i < targets.size(); ++i) outs[i] = bufs[i].data();
    const int rc = vds_ec_regenerate16_host(min_horcrux_, nodes.data(), chunks.data(), size, targets.data(),
                                            uint32_t(targets.size()), outs.data());
    if (rc != VDS_EC_OK) return make_unexpected<std::runtime_error>(vds_ec_strerror(rc));
    std::vector<const_data_buffer> result;
    for (auto &b : bufs) result.emplace_back(b.data(), size);
    return result;
  }

  expected<std::vector<const_data_buffer>> restore_datas(
      const std::vector<std::unordered_map<uint16_t, const_data_buffer>> &objects) {
    const size_t count = objects.size();
    std::vector<uint16_t> nodes;
    std::vector<const uint8_t *> chunks;
    std::vector<uint64_t> sizes(count), out_sizes(count);
    for (size_t o = 0; o < count; ++o) {  // the checks of restore_data (chunk_storage.cpp:65-77)
      const auto &h = objects[o];
      if (min_horcrux_ != h.size()) return make_unexpected<std::runtime_error>("Error at restoring data");
      sizes[o] = h.begin()->second.size();
      for (auto &p : h) {
        if (sizes[o] != p.second.size()) return make_unexpected<std::runtime_error>("Error at restoring data");
        nodes.push_back(p.first);
        chunks.push_back(p.second.data());
      }
    }
    std::vector<std::vector<uint8_t>> bufs(count);
    std::vector<uint8_t *> outs(count);
    for (size_t o = 0; o < count; ++o) {
      bufs[o].resize(sizes[o] * min_horcrux_ ? sizes[o] * min_horcrux_ : 1);  // >= any restored length
      outs[o] = bufs[o].data();
      out_sizes[o] = bufs[o].size();
    }
    const int rc = vds_ec_restore16_host_batch(min_horcrux_, nodes.data(), chunks.data(), sizes.data(),
                                               uint32_t(count), outs.data(), out_sizes.data(), 0, 0);
    if (rc == VDS_EC_ERESTORE) return make_unexpected<std::runtime_error>("Fatal error at chunk_restore::restore");
    if (rc != VDS_EC_OK) return make_unexpected<std::runtime_error>(vds_ec_strerror(rc));
    std::vector<const_data_buffer> result;
    result.reserve(count);
    for (size_t o = 0; o < count; ++o) result.emplace_back(bufs[o].data(), out_sizes[o]);
    return result;
  }

  // chunk_storage.cpp:62-86: exactly k equal-size horcruxes.
  expected<const_data_buffer> restore_data(const std::unordered_map<uint16_t, const_data_buffer> &horcruxes) {
    if (min_horcrux_ != horcruxes.size()) return make_unexpected<std::runtime_error>("Error at restoring data");
    const size_t size = horcruxes.begin()->second.size();
    std::vector<uint16_t> replicas;
    std::vector<const_data_buffer> datas;
    for (auto &p : horcruxes) {
      if (size != p.second.size()) return make_unexpected<std::runtime_error>("Error at restoring data");
      replicas.push_back(p.first);
      datas.push_back(p.second);
    }
    chunk_restore<uint16_t> restore(min_horcrux_, replicas.data());
    return restore.restore(datas);
  }

 private:
  uint16_t min_horcrux_;
  std::map<uint16_t, std::unique_ptr<chunk_generator<uint16_t>>> generators_;
};

chunk_storage::chunk_storage(uint16_t min_horcrux) : impl_(new _chunk_storage(min_horcrux)) {}

expected<std::vector<const_data_buffer>> chunk_storage::restore_datas(
    const std::vector<std::unordered_map<uint16_t, const_data_buffer>> &objects) {
  return impl_->restore_datas(objects);
}
chunk_storage::~chunk_storage() { delete impl_; }

expected<const_data_buffer> chunk_storage::generate_replica(uint16_t replica, const void *data, size_t size) {
  return impl_->generate_replica(replica, data, size);
}

expected<std::vector<const_data_buffer>> chunk_storage::generate_replicas(const std::vector<uint16_t> &replicas,
                                                                          const void *data, size_t size) {
  return impl_->generate_replicas(replicas, data, size);
}

expected<std::vector<const_data_buffer>> chunk_storage::generate_replicas(const std::vector<uint16_t> &replicas,
                                                                          const void *data, size_t size,
                                                                          std::vector<const_data_buffer> &hashes) {
  return impl_->generate_replicas(replicas, data, size, hashes);
}

expected<std::vector<const_data_buffer>> chunk_storage::regenerate_replicas(
    const std::unordered_map<uint16_t, const_data_buffer> &horcruxes, const std::vector<uint16_t> &targets) {
  return impl_->regenerate_replicas(horcruxes, targets);
}

expected<const_data_buffer> chunk_storage::restore_data(
    const std::unordered_map<uint16_t, const_data_buffer> &horcruxes) {
  return impl_->restore_data(horcruxes);
}

}  // namespace vds
