// types.h (compat) -- safe_cast (kernel/vds_core/types.h:42-65).
#pragma once
#include "vds_debug.h"
namespace vds {
template <typename T>
class safe_cast {
 public:
  template <typename S>
  safe_cast(S v) : value_((T)v) {
    vds_assert(v == (S)value_);
  }
  operator T() const { return value_; }

 private:
  T value_;
};
}  // namespace vds
