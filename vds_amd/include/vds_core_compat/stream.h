// stream.h (compat) -- async_task / stream_output_async as used by
// chunk_output_async (kernel/vds_core/stream.h:15-23).  The reference builds
// on the coroutines TS with libc++; this standalone stand-in is a minimal,
// eagerly-run C++20 coroutine task so the drop-in's chunk_output_async can be
// compiled and tested outside the vds tree.
#pragma once

#include <coroutine>
#include <exception>
#include <memory>
#include <optional>
#include <utility>

#include "expected.h"

namespace vds {

template <typename T>
class async_task {
 public:
  struct promise_type {
    std::optional<T> value;
    async_task get_return_object() { return async_task(std::coroutine_handle<promise_type>::from_promise(*this)); }
    std::suspend_never initial_suspend() noexcept { return {}; }
    std::suspend_always final_suspend() noexcept { return {}; }
    template <typename U>
    void return_value(U &&v) { value.emplace(std::forward<U>(v)); }
    void unhandled_exception() { std::terminate(); }
  };
  explicit async_task(std::coroutine_handle<promise_type> h) : h_(h) {}
  async_task(async_task &&o) noexcept : h_(std::exchange(o.h_, {})) {}
  ~async_task() {
    if (h_) h_.destroy();
  }
  // Everything here completes synchronously, so awaiting just yields the value.
  bool await_ready() const noexcept { return true; }
  void await_suspend(std::coroutine_handle<>) const noexcept {}
  T await_resume() { return std::move(*h_.promise().value); }
  T get() { return std::move(*h_.promise().value); }

 private:
  std::coroutine_handle<promise_type> h_;
};

template <typename item_type>
class stream_output_async : public std::enable_shared_from_this<stream_output_async<item_type>> {
 public:
  virtual ~stream_output_async() {}
  virtual async_task<expected<void>> write_async(const item_type *data, size_t len) = 0;
};

}  // namespace vds
