// chunk.h -- drop-in for lboss75/vds kernel/vds_data/chunk.h (chunk.h:17-446).
//
// Keeps the template API the callers compile against (chunk, chunk_generator,
// chunk_restore, chunk_output_async) and forwards the
// uint8_t / uint16_t instantiations to the MI355X codec through the C ABI
// (include/vds_ec.h).  Every data-path call runs the HIP kernels; when no GPU
// is usable the calls return make_unexpected<std::runtime_error> (or, from a
// constructor that cannot report, abort) -- there is no CPU fallback.
//
// Differences from the reference, on invalid input only:
//  * chunk_restore with repeated replica ids: the reference computes garbage
//    (its validation is vds_assert, compiled out); here restore() returns an
//    error and multipliers() is all-zero.
//  * chunk_generator and chunk_restore are neither copyable nor movable (the
//    copy operations are deleted; the reference's implicit copy would
//    double-free multipliers_).  Every caller holds them by unique_ptr or as
//    a local, which compiles unchanged.
#ifndef __VDS_DATA_CHUNK_H_
#define __VDS_DATA_CHUNK_H_

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <memory>
#include <stdexcept>
#include <vector>

#include "binary_serialize.h"
#include "gf.h"
#include "stream.h"
#include "vds_debug.h"
#include "vds_ec.h"

namespace vds {

namespace chunk_detail {

template <typename cell_type> struct codec;

template <> struct codec<uint16_t> {
  static int multipliers(uint16_t k, uint16_t n, uint16_t *out) { return vds_ec_multipliers16(k, n, out); }
  static int inverse(uint16_t k, const uint16_t *n, uint16_t *out) { return vds_ec_inverse16(k, n, out); }
  static int encode(uint16_t k, uint16_t n, const uint8_t *d, uint64_t size, uint8_t *out, unsigned flags) {
    uint8_t *outs[1] = {out};
    return vds_ec_encode16_host(k, &n, 1, d, size, outs, flags);
  }
  static int restore(uint16_t k, const uint16_t *n, const uint8_t *const *c, uint64_t size, uint8_t *out,
                     uint64_t *out_size, unsigned flags) {
    return vds_ec_restore16_host(k, n, c, size, out, out_size, flags);
  }
};

template <> struct codec<uint8_t> {
  static int multipliers(uint8_t k, uint8_t n, uint8_t *out) { return vds_ec_multipliers8(k, n, out); }
  static int inverse(uint8_t k, const uint8_t *n, uint8_t *out) { return vds_ec_inverse8(k, n, out); }
  static int encode(uint8_t k, uint8_t n, const uint8_t *d, uint64_t size, uint8_t *out, unsigned flags) {
    uint8_t *outs[1] = {out};
    return vds_ec_encode8_host(k, &n, 1, d, size, outs, flags);
  }
  static int restore(uint8_t k, const uint8_t *n, const uint8_t *const *c, uint64_t size, uint8_t *out,
                     uint64_t *out_size, unsigned flags) {
    return vds_ec_restore8_host(k, n, c, size, out, out_size, flags);
  }
};

[[noreturn]] inline void fail(const char *where, int status) {
#if __cpp_exceptions
  throw std::runtime_error(std::string(where) + ": " + vds_ec_strerror(status));
#else
  std::fprintf(stderr, "%s: %s\n", where, vds_ec_strerror(status));
  std::abort();
#endif
}

}  // namespace chunk_detail

template <typename cell_type>
class chunk_generator;

template <typename cell_type>
class chunk_restore;

template <typename cell_type>
class chunk {
 public:
  chunk(cell_type k, cell_type n, const std::vector<cell_type> &data) : k_(k), n_(n), data_(data) {}
  // Cell-array encode (chunk.h:206-224): ceil(len/k) cells, short stripe zero-padded.
  chunk(const chunk_generator<cell_type> &generator, const cell_type *data, size_t len)
      : k_(generator.k()), n_(generator.n()) {
    data_.resize(k_ ? (len + k_ - 1) / k_ : 0);
    if (data_.empty()) return;
    const int rc = chunk_detail::codec<cell_type>::encode(k_, n_, reinterpret_cast<const uint8_t *>(data),
                                                          len * sizeof(cell_type),
                                                          reinterpret_cast<uint8_t *>(data_.data()), VDS_EC_F_CELLS);
    if (rc != VDS_EC_OK) chunk_detail::fail("chunk::chunk", rc);
  }
  ~chunk() {}

  const std::vector<cell_type> &data() const { return data_; }
  static gf_math<cell_type> &math() { return math_; }

 private:
  cell_type k_;
  cell_type n_;
  std::vector<cell_type> data_;
  static gf_math<cell_type> math_;

  friend class chunk_generator<cell_type>;
  friend class chunk_restore<cell_type>;
};

template <typename cell_type>
gf_math<cell_type> chunk<cell_type>::math_;

template <typename cell_type>
class chunk_generator {
 public:
  chunk_generator(cell_type k, cell_type n) : k_(k), n_(n), multipliers_(new cell_type[k ? k : 1]) {
    chunk_detail::codec<cell_type>::multipliers(k, n, multipliers_);
  }
  ~chunk_generator() { delete[] multipliers_; }
  chunk_generator(const chunk_generator &) = delete;
  chunk_generator &operator=(const chunk_generator &) = delete;

  cell_type k() const { return k_; }
  cell_type n() const { return n_; }
  const cell_type *multipliers() const { return multipliers_; }

  // chunk.h:245-281: append replica n_ of data[0..size) (+ BE16 trailer).
  expected<void> write(binary_serializer &s, const void *data, size_t size, bool write_padding = true) {
    const unsigned flags = write_padding ? 0u : VDS_EC_F_NO_TRAILER;
    const uint64_t len = vds_ec_replica_size(sizeof(cell_type), k_, size, flags);
    std::vector<uint8_t> tmp(len ? len : 1);
    const int rc = chunk_detail::codec<cell_type>::encode(k_, n_, static_cast<const uint8_t *>(data), size,
                                                          tmp.data(), flags);
    if (rc != VDS_EC_OK) return make_unexpected<std::runtime_error>(vds_ec_strerror(rc));
    return s.push_data(tmp.data(), len, false);
  }

  // chunk.h:283-287
  expected<void> write_padding(binary_serializer &s, uint64_t size) {
    return (s << uint16_t(size % (sizeof(cell_type) * k_)));
  }

 private:
  cell_type k_;
  cell_type n_;
  cell_type *multipliers_;

  friend class chunk<cell_type>;
};

template <typename cell_type>
class chunk_restore {
 public:
  // chunk.h:290-375: multipliers_ = V^{-1}, V[i][c] = n[i]^c.
  chunk_restore(cell_type k, const cell_type *n)
      : k_(k), nodes_(n, n + k), multipliers_(new cell_type[size_t(k) * k ? size_t(k) * k : 1]()) {
    status_ = chunk_detail::codec<cell_type>::inverse(k, n, multipliers_);
  }
  ~chunk_restore() { delete[] multipliers_; }
  chunk_restore(const chunk_restore &) = delete;
  chunk_restore &operator=(const chunk_restore &) = delete;

  // chunk.h:383-400: cell arrays, appended to result, not trimmed.
  void restore(std::vector<cell_type> &result, const chunk<cell_type> **chunks) {
    if (status_ != VDS_EC_OK) chunk_detail::fail("chunk_restore::restore", status_);
    const size_t cells = chunks[0]->data_.size();
    std::vector<const uint8_t *> ptrs(k_);
    for (size_t j = 0; j < k_; ++j) ptrs[j] = reinterpret_cast<const uint8_t *>(chunks[j]->data_.data());
    const size_t at = result.size();
    result.resize(at + cells * k_);
    uint64_t out_size = 0;
    const int rc = chunk_detail::codec<cell_type>::restore(k_, nodes_.data(), ptrs.data(), cells * sizeof(cell_type),
                                                           reinterpret_cast<uint8_t *>(result.data() + at),
                                                           &out_size, VDS_EC_F_CELLS);
    if (rc != VDS_EC_OK) chunk_detail::fail("chunk_restore::restore", rc);
  }

  // chunk.h:402-444: decode the byte object from k replicas (trailer-trimmed).
  expected<const_data_buffer> restore(const std::vector<const_data_buffer> &chunks) {
    if (status_ != VDS_EC_OK) return make_unexpected<std::runtime_error>(vds_ec_strerror(status_));
    if (chunks.size() < k_) return make_unexpected<std::runtime_error>("Fatal error at chunk_restore::restore");
    const size_t size = chunks[0].size();
    std::vector<const uint8_t *> ptrs(k_);
    for (size_t j = 0; j < k_; ++j) {
      if (chunks[j].size() != size) return make_unexpected<std::runtime_error>("Fatal error at chunk_restore::restore");
      ptrs[j] = chunks[j].data();
    }
    std::vector<uint8_t> out(size * k_ ? size * k_ : 1);
    uint64_t out_size = 0;
    const int rc =
        chunk_detail::codec<cell_type>::restore(k_, nodes_.data(), ptrs.data(), size, out.data(), &out_size, 0);
    if (rc == VDS_EC_ERESTORE) return make_unexpected<std::runtime_error>("Fatal error at chunk_restore::restore");
    if (rc != VDS_EC_OK) return make_unexpected<std::runtime_error>(vds_ec_strerror(rc));
    // (const void*, size_t) is the constructor both the real vds_core and the compat type have
    return const_data_buffer(out.data(), out_size);
  }

  const cell_type *multipliers() const { return multipliers_; }

 private:
  cell_type k_;
  std::vector<cell_type> nodes_;
  cell_type *multipliers_;
  int status_ = VDS_EC_OK;
};

// chunk.h:116-176: streaming encoder.  Full buffers of 1024*k cells are
// encoded without trailer; the final call writes the tail with its trailer
// (or just the trailer), then forwards end-of-stream.  Byte-identical to a
// one-shot write of the whole input.
template <typename cell_type>
class chunk_output_async : public stream_output_async<uint8_t> {
 public:
  chunk_output_async(chunk_generator<cell_type> &generator, const std::shared_ptr<stream_output_async<uint8_t>> &target)
      : generator_(generator), target_(target), size_(0),
        buffer_(size_t(1024) * generator.k() * sizeof(cell_type)), buffer_position_(0) {
    vds_assert(!!target_);
  }

  async_task<expected<void>> write_async(const uint8_t *data, size_t len) override {
    const size_t block = buffer_.size();
    if (0 != len) {
      size_ += len;
      while (len > 0) {
        const size_t l = std::min(len, block - buffer_position_);
        std::memcpy(buffer_.data() + buffer_position_, data, l);
        data += l;
        len -= l;
        buffer_position_ += l;
        if (buffer_position_ == block) {
          binary_serializer s;
          CHECK_EXPECTED_ASYNC(generator_.write(s, buffer_.data(), buffer_position_, false));
          CHECK_EXPECTED_ASYNC(co_await target_->write_async(s.get_buffer(), s.size()));
          buffer_position_ = 0;
        }
      }
    } else {
      binary_serializer s;
      if (0 != buffer_position_) {
        CHECK_EXPECTED_ASYNC(generator_.write(s, buffer_.data(), buffer_position_));
      } else {
        CHECK_EXPECTED_ASYNC(generator_.write_padding(s, size_));
      }
      CHECK_EXPECTED_ASYNC(co_await target_->write_async(s.get_buffer(), s.size()));
      CHECK_EXPECTED_ASYNC(co_await target_->write_async(nullptr, 0));
    }
    co_return expected<void>();
  }

 private:
  chunk_generator<cell_type> &generator_;
  std::shared_ptr<stream_output_async<uint8_t>> target_;
  uint64_t size_;
  std::vector<uint8_t> buffer_;
  size_t buffer_position_;
};

}  // namespace vds

#endif  // __VDS_DATA_CHUNK_H_
