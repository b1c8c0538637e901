// const_data_buffer.h (compat) -- owned byte buffer with the accessors the
// codec uses (kernel/vds_core/const_data_buffer.h:19-150).
#pragma once

#include <cstdint>
#include <cstring>
#include <vector>

namespace vds {

class const_data_buffer {
 public:
  const_data_buffer() = default;
  const_data_buffer(const void *data, size_t len)
      : bytes_(static_cast<const uint8_t *>(data), static_cast<const uint8_t *>(data) + len) {}
  explicit const_data_buffer(std::vector<uint8_t> &&v) : bytes_(std::move(v)) {}
  const uint8_t *data() const { return bytes_.data(); }
  uint8_t *data() { return bytes_.data(); }
  size_t size() const { return bytes_.size(); }
  void resize(size_t len) { bytes_.resize(len); }
  uint8_t operator[](size_t i) const { return bytes_[i]; }
  bool operator==(const const_data_buffer &o) const { return bytes_ == o.bytes_; }

 private:
  std::vector<uint8_t> bytes_;
};

}  // namespace vds
