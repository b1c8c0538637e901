// ec_encode.hip -- dispatch of the bit-sliced encode k_encode_bs<K,N>
// (ec_encode.hpp) to its per-shape translation units, and the k = 4
// instantiation (chunk_generator<uint16_t>::write, chunk.h:245-281).
#include "ec_encode.hpp"

namespace vds_ec {

hipError_t launch_encode_fast_16_20(const FastEncodeArgs &a, hipStream_t s);
hipError_t launch_encode_fast_32_40(const FastEncodeArgs &a, hipStream_t s);
hipError_t launch_encode_fast_32_64(const FastEncodeArgs &a, hipStream_t s);

bool has_encode_fast(uint32_t k, uint32_t n) {
  return (k == 16 && n == 20) || (k == 32 && n == 40) || (k == 32 && n == 64) || (k == 4 && n == 6);
}

hipError_t launch_encode_fast(uint32_t k, uint32_t n, const FastEncodeArgs &a, hipStream_t s) {
  if (k == 16 && n == 20) return launch_encode_fast_16_20(a, s);
  if (k == 32 && n == 40) return launch_encode_fast_32_40(a, s);
  if (k == 32 && n == 64) return launch_encode_fast_32_64(a, s);  // the live shape (dht_network.h:22-25)
  if (k == 4 && n == 6) return launch_encode_bs<4, 6, 6, 1>(a, s);
  return hipErrorNotSupported;
}

}  // namespace vds_ec
