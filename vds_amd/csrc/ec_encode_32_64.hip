// ec_encode_32_64.hip -- k_encode_bs<32,64>, the live production shape (dht_network.h:22-25): one
// translation unit per shape so the builds compile them in parallel.
#include "ec_encode.hpp"

namespace vds_ec {

hipError_t launch_encode_fast_32_64(const FastEncodeArgs &a, hipStream_t s) {
  return launch_encode_bs<32, 64, 8, 8>(a, s);
}

}  // namespace vds_ec
