// vds_debug.h (compat) -- vds_assert as in kernel/vds_core/vds_debug.h:11-15.
#pragma once
#include <stdexcept>
#if __cpp_exceptions
#define vds_assert(exp) \
  if (!(exp)) { throw std::runtime_error("Accert " #exp); }
#else
#define vds_assert(exp)
#endif
