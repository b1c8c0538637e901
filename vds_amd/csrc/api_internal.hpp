// api_internal.hpp -- host runtime internals shared by the C ABI's
// translation units (internal to libvds_ec.so):
//   vds_ec_api.cpp      argument validation, host field arithmetic and the
//                       inverse, encode / restore / regenerate dispatch, host
//                       staging contexts, the C ABI itself;
//   api_param_ring.cpp  the stream-ordered parameter ring;
//   api_batch.cpp       batched per-object-survivor restore / regenerate
//                       planning (routes, erased-set plans, tiles);
//   api_host_batch.cpp  caller-pinned slabs, the multi-GPU host batches and
//                       the stripe-range split.
#pragma once

#include "../../include/vds_ec.h"

#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <array>
#include <climits>
#include <condition_variable>
#include <cstdint>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <sched.h>
#include <shared_mutex>
#include <thread>
#include <unordered_map>
#include <vector>

#include "ec_internal.hpp"
#include "gf_common.hpp"

namespace vds_ec {
namespace api {

struct HostCtx;
struct RestorePlan;

inline hipStream_t as_stream(void *s) { return reinterpret_cast<hipStream_t>(s); }

// ------------------------------------------------- host field arithmetic
// log / antilog tables for the host's k x k and M x M work (gf.h:193-253's
// tables; the kernels never use them).  Built once, 384 KiB.
struct Gf16Tables {
  uint16_t log[65536];
  uint16_t exp[2 * 65535];
  Gf16Tables() {
    uint32_t v = 1;
    for (uint32_t l = 0; l < 65535; ++l) {
      exp[l] = exp[l + 65535] = (uint16_t)v;
      log[v] = (uint16_t)l;
      v = gf16_mul(v, 2);
    }
    log[0] = 0;
  }
};

// ------------------------------------------------ stream-ordered parameters
// Kernel parameters too large for the kernel arguments (k > 32 inverses, k >
// 64 chunk tables, regenerate coefficients beyond kInlineCoef) ride a
// per-device ring of pinned host + device slots, so the *_device entry points
// enqueue without synchronising.  A slot's bytes are written on the host,
// copied with hipMemcpyAsync on the caller's stream, and an event recorded
// after the kernels that read them; a slot is reused only once its event has
// completed, and hipEventSynchronize blocks only when the ring has wrapped
// round inside the GPU's queue.  (The round-1 version copied a std::vector
// on the caller's stack with hipMemcpyAsync and freed a hipMallocAsync
// buffer in a destructor: the copy could read the vector after it was gone
// -- the likely cause of that round's fault)  Growing a slot
// allocates, which synchronises; slots only grow.
struct ParamSlot {
  uint8_t *h = nullptr, *d = nullptr;
  size_t cap = 0;
  hipEvent_t ev = nullptr;
  hipEvent_t copied = nullptr;  // the host -> device copy on the ring's copy stream
  bool pending = false;  // its event guards the device copy's readers
  bool busy = false;     // acquired, not yet released
  uint64_t stamp = 0;    // when last acquired (ParamRing::clock)
};

// --------------------------------------------------------- restore core
// Optional layout facts the host path knows: chunks contiguous at a pitch,
// and a device copy of a large inverse already staged.
struct ChunkLayout {
  const uint8_t *base = nullptr;
  uint64_t pitch = 0;
  const uint16_t *matrix_dev = nullptr;
};

struct Copy {
  uint8_t *dst;
  const uint8_t *src;
  size_t len;
};

// ---------------------------------------------- caller-pinned host memory
// Buffers the caller allocated with vds_ec_host_alloc or registered with
// vds_ec_host_register (page-locked, mapped, portable across devices).  A
// host batch whose group of objects (or replicas) lies in one such range as
// one contiguous slab skips the staging copies: the H2D DMA reads the
// caller's bytes, and the push kernel writes the results straight into the
// caller's pages.  Lookups are per group, not per object.
constexpr int kPinnedMaxDev = 64;
struct PinnedRange {
  uint64_t bytes;
  bool owned;  // vds_ec_host_alloc (freed by vds_ec_host_free) vs registered
  // the device address of the range's first byte, per device: resolved on
  // each device the first time a host batch there uses the range (a mapped
  // host range need not have the same address on every device)
  uint8_t *dev[kPinnedMaxDev] = {};
};
struct PinnedRegistry {
  std::mutex mu;
  std::map<uintptr_t, PinnedRange> ranges;  // by start address
};

int hip_status(hipError_t e);
int device_ready();
int inverse16(uint32_t k, const uint16_t *nodes, uint16_t *out);
bool restore_path_override_bs();
bool syn_solve(uint32_t k, uint32_t n, SynRestoreArgs &sa);
int encode_device(unsigned cb, uint32_t k, const uint16_t *replicas, uint32_t n, const uint8_t *in,
                  uint64_t size, uint64_t in_stride, uint32_t count, uint8_t *const *outs,
                  uint64_t out_stride, unsigned flags, hipStream_t s);
hipError_t param_acquire_n(int cnt, const size_t *bytes, ParamSlot **out);
hipError_t param_commit(ParamSlot *sl, size_t bytes, hipStream_t s);
hipError_t param_release(ParamSlot *sl, hipStream_t s);
hipError_t param_stage(const std::vector<uint8_t> &blob, hipStream_t s, const uint8_t **dev, ParamSlot **out);
int restore_device(unsigned cb, uint32_t k, const uint16_t *nodes, const uint16_t *matrix, const uint8_t *const *chunks,
                   uint64_t chunk_size, uint64_t chunk_stride, uint64_t out_len, uint32_t count,
                   uint8_t *out, uint64_t out_stride, unsigned flags, hipStream_t s,
                   const ChunkLayout &layout = ChunkLayout());
uint64_t restored_len(unsigned cb, uint32_t k, uint64_t chunk_size, uint16_t padding, unsigned flags,
                      bool *ok);
void parallel_copy(const std::vector<Copy> &parts_in);
extern std::atomic<uint64_t> g_host_ctx_created;
int regenerate_device(unsigned cb, uint32_t k, const uint16_t *nodes, const uint8_t *const *chunks,
                      uint64_t chunk_size, uint64_t chunk_stride, uint32_t count, const uint16_t *targets,
                      uint32_t nt, uint8_t *const *outs, uint64_t out_stride, hipStream_t s);
bool ids_distinct(uint32_t k, const uint16_t *nd);
int restore_batch_device(uint32_t k, uint32_t count, const uint16_t *nodes, const uint8_t *const *chunks,
                         const uint64_t *chunk_sizes, const uint16_t *paddings, uint8_t *const *outs, unsigned flags,
                         hipStream_t s);
int regenerate_batch_device(uint32_t k, uint32_t count, const uint16_t *nodes, const uint8_t *const *chunks,
                            const uint64_t *chunk_sizes, uint32_t nt, const uint16_t *targets, uint8_t *const *outs,
                            hipStream_t s);
PinnedRegistry &pinned_registry();
int encode_host_batch(uint32_t k, const uint16_t *replicas, uint32_t n, const uint8_t *const *objs,
                      const uint64_t *sizes, uint32_t count, uint8_t *const *outs, unsigned flags, int max_devices);
int restore_host_batch(uint32_t k, const uint16_t *nodes, const uint8_t *const *chunks, const uint64_t *chunk_sizes,
                       uint32_t count, uint8_t *const *outs, uint64_t *out_sizes, unsigned flags, int max_devices);
int encode_range(uint32_t k, const uint16_t *replicas, uint32_t n, const uint8_t *in, uint64_t size, uint64_t t0,
                 uint64_t t1, uint8_t *const *outs, unsigned flags, hipStream_t s);
int range_restore_len(uint32_t k, uint64_t chunk_size, uint16_t padding, unsigned flags, uint64_t *E, uint64_t *nst);
int restore_range(uint32_t k, const uint16_t *nodes, const uint16_t *matrix, const uint8_t *const *chunks,
                  uint64_t t0, uint64_t t1, uint64_t E, uint8_t *out, unsigned flags, hipStream_t s);
int encode_host_split(uint32_t k, const uint16_t *replicas, uint32_t n, const uint8_t *data, uint64_t size,
                      uint8_t *const *outs, unsigned flags, int max_devices, uint32_t parts);
int restore_host_split(uint32_t k, const uint16_t *nodes, const uint8_t *const *chunks, uint64_t chunk_size,
                       uint8_t *out, uint64_t *out_size, unsigned flags, int max_devices, uint32_t parts);const Gf16Tables &gf16_tables();

inline uint32_t gf16_mul_fast(uint32_t a, uint32_t b) {
  if (!a || !b) return 0;
  const Gf16Tables &t = gf16_tables();
  return t.exp[t.log[a] + t.log[b]];
}

inline uint32_t gf16_inv_fast(uint32_t a) {
  if (!a) return 0;
  const Gf16Tables &t = gf16_tables();
  return t.exp[65535 - t.log[a]];
}

template <typename T>
size_t blob_append(std::vector<uint8_t> &blob, const T *p, size_t n) {
  const size_t off = (blob.size() + 15) & ~size_t(15);
  blob.resize(off + sizeof(T) * n);
  std::memcpy(blob.data() + off, p, sizeof(T) * n);
  return off;
}

template <typename Id>
int check_restore_args(uint32_t k, const Id *nodes, const uint8_t *const *chunks, uint64_t chunk_size) {
  if (k == 0 || !nodes || !chunks) return VDS_EC_EINVAL;
  for (uint32_t j = 0; j < k; ++j)
    if (!chunks[j] && chunk_size) return VDS_EC_EINVAL;
  return VDS_EC_OK;
}

}  // namespace api
}  // namespace vds_ec
