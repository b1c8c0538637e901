// chunk_storage.h -- drop-in for lboss75/vds kernel/vds_data/chunk_storage.h
// (chunk_storage.h:13-34): same class, same signatures.
#ifndef __VDS_DATA_CHUNK_STORAGE_H_
#define __VDS_DATA_CHUNK_STORAGE_H_

#include <unordered_map>
#include <vector>

#include "binary_serialize.h"

namespace vds {
class _chunk_storage;

class chunk_storage {
 public:
  chunk_storage(uint16_t min_horcrux);
  ~chunk_storage();

  expected<const_data_buffer> generate_replica(uint16_t replica, const void *data, size_t size);

  expected<const_data_buffer> restore_data(const std::unordered_map<uint16_t, const_data_buffer> &horcruxes);

  // Batched form for the save_temp / save_data loops (dht_network_client.cpp:
  // 74-104, 588-655): every requested replica from one device pass.
  expected<std::vector<const_data_buffer>> generate_replicas(const std::vector<uint16_t> &replicas,
                                                             const void *data, size_t size);

  // generate_replicas plus each replica's SHA-256 name (the replica_hash of
  // dht_network_client.cpp:79 / :593), computed on the device.
  expected<std::vector<const_data_buffer>> generate_replicas(const std::vector<uint16_t> &replicas,
                                                             const void *data, size_t size,
                                                             std::vector<const_data_buffer> &hashes);

  // Batched restore_data: object o from the k equal-size horcruxes of
  // objects[o] (one device pass per object over every GPU, pinned staging);
  // the same results and errors as restore_data per object.
  expected<std::vector<const_data_buffer>> restore_datas(
      const std::vector<std::unordered_map<uint16_t, const_data_buffer>> &objects);

  // Repair without materialising the object (sync_process.cpp:313-335 does
  // restore_data + generate_replica): replicas `targets` from exactly
  // min_horcrux equal-size horcruxes, byte-identical to that route.
  expected<std::vector<const_data_buffer>> regenerate_replicas(
      const std::unordered_map<uint16_t, const_data_buffer> &horcruxes, const std::vector<uint16_t> &targets);

 private:
  friend class ichunk_storage;
  _chunk_storage *const impl_;
};
}  // namespace vds

#endif  // __VDS_DATA_CHUNK_STORAGE_H_
