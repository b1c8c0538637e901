// binary_serialize.h (compat) -- the byte sink chunk_generator::write appends
// to; big-endian integers as kernel/vds_core/binary_serialize.cpp:18-22.
#pragma once

#include <cstdint>
#include <vector>

#include "const_data_buffer.h"
#include "expected.h"

namespace vds {

class binary_serializer {
 public:
  expected<void> put(uint8_t v) {
    buf_.push_back(v);
    return expected<void>();
  }
  expected<void> put(uint16_t v) {
    buf_.push_back(uint8_t(v >> 8));
    buf_.push_back(uint8_t(v));
    return expected<void>();
  }
  expected<void> push_data(const void *data, size_t size, bool serialize_size = true) {
    if (serialize_size) return make_unexpected<std::runtime_error>("compat serializer: sized push unsupported");
    const uint8_t *p = static_cast<const uint8_t *>(data);
    buf_.insert(buf_.end(), p, p + size);
    return expected<void>();
  }
  // Reserve `size` bytes at the end and return where they start (drop-in fast
  // path: the device writes straight into the serializer's storage).
  uint8_t *append_uninitialized(size_t size) {
    const size_t at = buf_.size();
    buf_.resize(at + size);
    return buf_.data() + at;
  }
  const uint8_t *get_buffer() const { return buf_.data(); }
  size_t size() const { return buf_.size(); }
  const_data_buffer move_data() { return const_data_buffer(std::move(buf_)); }

 private:
  std::vector<uint8_t> buf_;
};

inline expected<void> operator<<(binary_serializer &s, uint8_t v) { return s.put(v); }
inline expected<void> operator<<(binary_serializer &s, uint16_t v) { return s.put(v); }

}  // namespace vds
