// ec_device.hpp -- device-side helpers shared by the kernel translation units
// (ec_generic.hip, ec_encode.hip, ec_restore_bs.hip, ec_restore_syn.hip).
// Internal to libvds_ec.so.
#pragma once

#ifndef __HIPCC_RTC__  // (hiprtc: device code only, vds_ec_jit.cpp)
#include <hip/hip_runtime.h>

#include <atomic>
#endif
#include <cstdint>

#include "bitslice.hpp"
#include "ec_internal.hpp"

namespace vds_ec {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) const volatile u32x4 lds_u32x4;
typedef __attribute__((address_space(3))) volatile u32x4 lds_v4;
typedef __attribute__((address_space(3))) volatile u32x2 lds_v2;
typedef __attribute__((address_space(3))) char lds_char;

// Streaming (non-temporal) global accesses of the data path, by bit:
// 1 = encode replica stores, 2 = encode object loads, 4 = restore survivor
// loads, 8 = restore / regenerate stores.  Every byte is read or written
// exactly once, so nothing is lost by not keeping it in L2.  Only whole-line
// wave accesses use them: k_restore_bs's 4-byte strided stores and loads ran
// 3.4x slower non-temporal (live shape repair 212 -> 79 GiB/s).  Same-box A/B
// (512 x 64 MiB, 3 rounds): none 840, {1,4,8} 859, all four 856 GiB/s.
constexpr int kNonTemporal = 1 | 4 | 8;

// The pointers are global memory: the explicit address space keeps pointers
// the kernel read from memory (batch descriptors) from becoming flat_
// accesses, which also count against lgkmcnt and retire out of order.
template <class T>
using gmem = __attribute__((address_space(1))) T;
template <int BIT, class T>
__device__ __forceinline__ T g_ld(const void *p) {
  const gmem<T> *q = (const gmem<T> *)p;
  if constexpr ((kNonTemporal & BIT) != 0) return __builtin_nontemporal_load(q);
  else return *q;
}
template <int BIT, class T>
__device__ __forceinline__ void g_st(void *p, T v) {
  gmem<T> *q = (gmem<T> *)p;
  if constexpr ((kNonTemporal & BIT) != 0) __builtin_nontemporal_store(v, q);
  else *q = v;
}
// A wave-uniform read of a launch table the kernel never writes (batch
// descriptors): the constant address space lets a uniform address become an
// s_load into SGPRs instead of a per-lane vector load.
template <class T>
__device__ __forceinline__ T s_ld(const T *p) {
  return *(const __attribute__((address_space(4))) T *)p;
}
// Byte i of a wave-uniform launch table (e.g. a kernel argument's uint8_t
// array at a runtime index; `arr` 4-byte aligned).  gfx950 has no sub-dword
// scalar load: a plain arr[i] becomes a *vector* global_load_ubyte, whose
// s_waitcnt vmcnt(0) then waits for every load and store the wave has in
// flight -- at the top of a tile loop, the previous tile's stores and the
// prefetched next tile.  Load the aligned dword with s_load and extract the
// byte instead.  (No pointer-to-integer casts: on a kernel argument they
// force a private copy of the whole argument struct.)
__device__ __forceinline__ uint32_t s_ld_u8(const uint8_t *arr, int i) {
  const uint32_t w = s_ld(reinterpret_cast<const uint32_t *>(arr) + (i >> 2));
  return (w >> (8 * (i & 3))) & 0xFFu;
}

// The 16 planes of one cell from LDS as four ds_read_b128.  A volatile
// 128-bit load through an LDS (address_space(3)) pointer keeps the compiler
// from splitting the reads into ds_read2_b32 / ds_read_b64, which
// bank-conflict at the encode's padding.
__device__ __forceinline__ Plane16 lds_planes(const uint32_t *p) {
  Plane16 x;
  lds_u32x4 *q = (lds_u32x4 *)(p);
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const u32x4 v = q[m];
    x.p[4 * m + 0] = v.x;
    x.p[4 * m + 1] = v.y;
    x.p[4 * m + 2] = v.z;
    x.p[4 * m + 3] = v.w;
  }
  return x;
}

// Tile order of the persistent tile loops.  Workgroups are dealt round-robin
// over the 8 XCDs (workgroup b on XCD b mod 8), so a grid stride of single
// tiles puts adjacent tiles -- adjacent 4 KiB pieces of every replica stream
// -- on different XCDs.  With VDS_XCD_TILES each XCD instead walks its own
// contiguous eighth of the tiles, its workgroups side by side
// (tools/ubench/hbm_write.hip, the encode's 20-stream store shape: 5.24 ->
// 5.47-5.61 TB/s).  Any order is correct; this one is for speed only.
#ifndef VDS_XCD_TILES
#define VDS_XCD_TILES 1
#endif
struct TileRange {
  uint32_t first, end, step;
};
__device__ __forceinline__ TileRange tile_range(uint32_t total) {
#if VDS_XCD_TILES
  const uint32_t g = gridDim.x;
  if ((g & 7u) == 0 && total >= g) {  // (every XCD range then has >= g/8 tiles)
    const uint32_t x = blockIdx.x & 7u;
    const uint32_t lo = (uint32_t)((uint64_t)total * x / 8), hi = (uint32_t)((uint64_t)total * (x + 1) / 8);
    return {lo + (blockIdx.x >> 3), hi, g >> 3};
  }
#endif
  return {blockIdx.x, total, gridDim.x};
}

// ------------------------------------------------------------ host helpers
#ifndef __HIPCC_RTC__

// Study overrides of the fast kernels' grids (workgroups), compile-time:
// -DVDS_ENC_GRID=n / -DVDS_SYN_GRID=n (0 = the default sizing), and
// -DVDS_ENC_LDS_EXTRA=bytes of unused LDS per encode workgroup (runs the
// encode at fewer workgroups per CU; diagnostic).
#ifndef VDS_ENC_GRID
#define VDS_ENC_GRID 0
#endif
#ifndef VDS_SYN_GRID
#define VDS_SYN_GRID 0
#endif
#ifndef VDS_ENC_LDS_EXTRA
#define VDS_ENC_LDS_EXTRA 0
#endif

// hipFuncSetAttribute(MaxDynamicSharedMemorySize) once per (kernel, device):
// the attribute is per device, and the multi-GPU host batches launch from one
// thread per device concurrently.
template <class Kernel>
hipError_t ensure_lds_attr(Kernel *k, int bytes) {
  constexpr int kMaxDev = 64;
  static std::atomic<int> done[kMaxDev];  // 0 = not yet, 1 = set
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  if (dev >= 0 && dev < kMaxDev && done[dev].load(std::memory_order_acquire)) return hipSuccess;
  e = hipFuncSetAttribute(reinterpret_cast<const void *>(k), hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  if (e == hipSuccess && dev >= 0 && dev < kMaxDev) done[dev].store(1, std::memory_order_release);
  return e;
}

#endif  // __HIPCC_RTC__

}  // namespace vds_ec
