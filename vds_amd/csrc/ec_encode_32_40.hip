// ec_encode_32_40.hip -- k_encode_bs<32,40>, C4 (BASELINE configs[3]): one
// translation unit per shape so the builds compile them in parallel.
#include "ec_encode.hpp"

namespace vds_ec {

hipError_t launch_encode_fast_32_40(const FastEncodeArgs &a, hipStream_t s) {
  return launch_encode_bs<32, 40, 5, 8>(a, s);
}

}  // namespace vds_ec
