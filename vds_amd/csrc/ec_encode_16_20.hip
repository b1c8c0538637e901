// ec_encode_16_20.hip -- k_encode_bs<16,20>, the headline shape (BASELINE configs[1]): one
// translation unit per shape so the builds compile them in parallel.
#include "ec_encode.hpp"

namespace vds_ec {

hipError_t launch_encode_fast_16_20(const FastEncodeArgs &a, hipStream_t s) {
  return launch_encode_bs<16, 20, 5, 4>(a, s);
}

}  // namespace vds_ec
