// expected.h (compat) -- the subset of lboss75/vds kernel/vds_core/expected.h
// (expected.h:27-167) that the codec API is written in.  Used only for the
// standalone build of the drop-in; inside the vds tree the real vds_core
// header is found first on the include path.
#pragma once

#include <exception>
#include <memory>
#include <stdexcept>
#include <type_traits>
#include <utility>

namespace vds {

class unexpected {
 public:
  explicit unexpected(std::unique_ptr<std::exception> &&e) : error_(std::move(e)) {}
  std::unique_ptr<std::exception> &error() { return error_; }
  const std::unique_ptr<std::exception> &error() const { return error_; }

 private:
  std::unique_ptr<std::exception> error_;
};

template <typename E, typename... Args>
inline unexpected make_unexpected(Args &&...args) {
  return unexpected(std::make_unique<E>(std::forward<Args>(args)...));
}

template <typename T>
class [[nodiscard]] expected {
 public:
  template <typename... A>
  expected(A &&...v) : has_value_(true), value_(std::forward<A>(v)...) {}
  expected(expected &&o) noexcept : has_value_(o.has_value_), value_(std::move(o.value_)), error_(std::move(o.error_)) {}
  expected(unexpected &&u) : has_value_(false), value_(), error_(std::move(u.error())) {}
  expected &operator=(expected &&o) noexcept {
    has_value_ = o.has_value_;
    value_ = std::move(o.value_);
    error_ = std::move(o.error_);
    return *this;
  }
  bool has_value() const { return has_value_; }
  bool has_error() const { return !!error_; }
  T &value() { return value_; }
  const T &value() const { return value_; }
  std::unique_ptr<std::exception> &error() { return error_; }
  const std::unique_ptr<std::exception> &error() const { return error_; }

 private:
  bool has_value_;
  T value_;
  std::unique_ptr<std::exception> error_;
};

template <>
class [[nodiscard]] expected<void> {
 public:
  expected() = default;
  expected(expected &&) noexcept = default;
  expected(unexpected &&u) : error_(std::move(u.error())) {}
  expected &operator=(expected &&) noexcept = default;
  bool has_value() const { return !error_; }
  bool has_error() const { return !!error_; }
  void value() const {}
  std::unique_ptr<std::exception> &error() { return error_; }
  const std::unique_ptr<std::exception> &error() const { return error_; }

 private:
  std::unique_ptr<std::exception> error_;
};

}  // namespace vds

#define CHECK_EXPECTED(v)                                                      \
  {                                                                            \
    auto __vds_r = (v);                                                        \
    if (__vds_r.has_error()) return vds::unexpected(std::move(__vds_r.error())); \
  }
#define GET_EXPECTED(var, v)                                                          \
  auto __vds_r##var = (v);                                                            \
  if (__vds_r##var.has_error()) return vds::unexpected(std::move(__vds_r##var.error())); \
  auto var = std::move(__vds_r##var.value());
#define CHECK_EXPECTED_ASYNC(v)                                                    \
  {                                                                                \
    auto __vds_r = (v);                                                            \
    if (__vds_r.has_error()) co_return vds::unexpected(std::move(__vds_r.error())); \
  }
