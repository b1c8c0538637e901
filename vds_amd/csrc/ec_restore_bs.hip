// ec_restore_bs.hip -- k_restore_bs<K>: bit-sliced restore with the k x k
// inverse as wave-uniform runtime constants (chunk_restore<uint16_t>::restore,
// chunk.h:402-444), K in {16, 32}, any k survivors.  Also the regenerate mode
// (rows V_targets V_S^{-1}: replicas straight from the survivors) for
// survivor sets outside the syndrome kernel's points, e.g. the live n = 64
// shape.
#include "ec_device.hpp"

namespace vds_ec {

template <int K>
struct RestoreShape {
  static constexpr int kPerWave = 4;           // survivors loaded / outputs computed per wave
  static constexpr int kWaves = K / kPerWave;
  static constexpr int kThreads = 64 * kWaves;
  static constexpr int kSetWords = K * 16 + 4;
  static constexpr int kLdsBytes = 64 * kSetWords * 4;
  static_assert(K % 8 == 0, "restore fast path needs k % 8 == 0");
};

// slot i (0..31) of lane l <-> stripe stripe0 + 8 l + 512 (i / 8) + (i % 8);
// bit position pi of a plane <-> slot (pi < 16 ? 2 pi : 2 (pi - 16) + 1).
__device__ __forceinline__ uint64_t restore_slot_stripe(int lane, int slot) {
  return 8u * lane + 512u * (slot >> 3) + (slot & 7);
}

// Tiles in 512-stripe groups (1 KiB of every survivor): group q of tile t is
// global group 4 t + q = group r of object o (groups_per_obj per object).
// STREAM: tiles may straddle objects (small objects, groups_per_obj % 4 != 0).
__device__ __forceinline__ void restore_group(const FastRestoreArgs &a, uint32_t tile, uint32_t q, uint32_t &o,
                                              uint32_t &r) {
  const uint32_t g = 4u * tile + q;
  o = g / a.groups_per_obj;
  r = g - o * a.groups_per_obj;
}

template <int K, bool STREAM>
__device__ __forceinline__ void restore_load(u32x4 (&Q)[RestoreShape<K>::kPerWave][4], const FastRestoreArgs &a,
                                             uint32_t tile, int lane, int wave) {
  using S = RestoreShape<K>;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    uint32_t o, r;
    restore_group(a, tile, STREAM ? q : 0, o, r);
    const uint64_t off = (uint64_t)o * a.chunk_stride + 1024ull * (STREAM ? r : r + q) + 16 * lane;
#pragma unroll
    for (int s = 0; s < S::kPerWave; ++s) Q[s][q] = *reinterpret_cast<const u32x4 *>(a.chunks[wave * S::kPerWave + s] + off);
  }
}

template <int K, bool STREAM, bool REGEN>
__global__ __launch_bounds__((RestoreShape<K>::kThreads), 2) void k_restore_bs(FastRestoreArgs a) {
  using S = RestoreShape<K>;
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint32_t *my_set = lds + lane * S::kSetWords;

  u32x4 Q[S::kPerWave][4];
  uint32_t tile = blockIdx.x;
  if (tile < a.total_tiles) restore_load<K, STREAM>(Q, a, tile, lane, wave);
  for (; tile < a.total_tiles; tile += gridDim.x) {
    uint32_t W[S::kPerWave][16];
#pragma unroll
    for (int s = 0; s < S::kPerWave; ++s)
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int d = 0; d < 4; ++d) W[s][4 * q + d] = Q[s][q][d];
    // ---- transpose this wave's survivors to planes: W[x] = plane of cell bit x^8
#pragma unroll
    for (int s = 0; s < S::kPerWave; ++s) {
      const int j = wave * S::kPerWave + s;
      transpose16x2(W[s]);
#pragma unroll
      for (int m = 0; m < 4; ++m)
        *reinterpret_cast<uint4 *>(my_set + j * 16 + 4 * m) =
            make_uint4(W[s][4 * (m ^ 2)], W[s][4 * (m ^ 2) + 1], W[s][4 * (m ^ 2) + 2], W[s][4 * (m ^ 2) + 3]);
    }
    __syncthreads();
    const uint32_t next = tile + gridDim.x;
    if (next < a.total_tiles) restore_load<K, STREAM>(Q, a, next, lane, wave);
    // ---- outputs m = wave*kPerWave + s : sum_j M[m][j] * Y_j
    Plane16 acc[S::kPerWave];
#pragma unroll
    for (int s = 0; s < S::kPerWave; ++s) acc[s] = plane_zero();
    Plane16 yn = lds_planes(my_set);  // one survivor ahead
#pragma clang loop unroll(disable)
    for (int j = 0; j < K; ++j) {
      const Plane16 y = yn;
      if (j + 1 < K) yn = lds_planes(my_set + (j + 1) * 16);
      uint32_t c[S::kPerWave];
#pragma unroll
      for (int s = 0; s < S::kPerWave; ++s) {
        const uint32_t idx = (wave * S::kPerWave + s) * K + j;
        c[s] = (a.matrix2[idx >> 1] >> (16 * (idx & 1))) & 0xFFFFu;
      }
      plane_mac_rt<S::kPerWave>(acc, y, c);
    }
    if constexpr (REGEN) {
      // ---- regenerate: output m is replica regen[m]'s cells for the same
      // stripes the survivors were loaded from; undo the load transpose and
      // store with the load's addressing (1 KiB per wave-instruction)
#pragma unroll
      for (int s = 0; s < S::kPerWave; ++s) {
        const uint32_t m = wave * S::kPerWave + s;
        if (m >= a.nt) continue;
        uint32_t W[16];
#pragma unroll
        for (int b = 0; b < 16; ++b) W[b ^ 8] = acc[s].p[b];
        transpose16x2(W);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          uint32_t o, r;
          restore_group(a, tile, STREAM ? q : 0, o, r);
          uint8_t *dst = a.regen[m] + (uint64_t)o * a.out_stride + 1024ull * (STREAM ? r : r + q) + 16 * lane;
          *reinterpret_cast<u32x4 *>(dst) = u32x4{W[4 * q], W[4 * q + 1], W[4 * q + 2], W[4 * q + 3]};
        }
      }
      __syncthreads();
      continue;
    }
    // ---- back to big-endian cells: word group w' = cells (2w', 2w'+1)
#pragma unroll
    for (int g = 0; g < S::kPerWave / 2; ++g) {
      uint32_t rows[32];
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int jb = 0; jb < 16; ++jb) rows[16 * h + jb] = acc[2 * g + h].p[jb ^ 8];
      transpose32(rows);
      const int wg = (wave * S::kPerWave) / 2 + g;
      // slot 8q+e <-> stripe 8 lane + 512 q + e of the tile (group q); plane bit
      // pi <-> slot (pi < 16 ? 2 pi : 2 (pi-16) + 1)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        uint32_t o, r;
        restore_group(a, tile, STREAM ? q : 0, o, r);
        uint8_t *base = a.out + (uint64_t)o * a.out_stride + ((uint64_t)512 * (STREAM ? r : r + q) + 8u * lane) * (2 * K) +
                        4 * wg;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int slot = 8 * q + e;
          const int pi = (slot & 1) ? 16 + (slot >> 1) : (slot >> 1);
          *reinterpret_cast<uint32_t *>(base + e * (2 * K)) = rows[pi];
        }
      }
    }
    __syncthreads();
  }
}

template <int K, bool STREAM, bool REGEN>
static hipError_t launch_restore_bs_k(const FastRestoreArgs &a, hipStream_t s) {
  using S = RestoreShape<K>;
  hipError_t e = ensure_lds_attr(&k_restore_bs<K, STREAM, REGEN>, S::kLdsBytes);
  if (e != hipSuccess) return e;
  const int blocks_per_cu = (160 * 1024) / S::kLdsBytes;
  int grid = 256 * (blocks_per_cu > 0 ? blocks_per_cu : 1);
  if ((uint32_t)grid > a.total_tiles) grid = (int)a.total_tiles;
  if (grid == 0) return hipSuccess;
  hipLaunchKernelGGL((k_restore_bs<K, STREAM, REGEN>), dim3(grid), dim3(S::kThreads), S::kLdsBytes, s, a);
  return hipGetLastError();
}

bool has_restore_fast(uint32_t k) { return k == 16 || k == 32; }

template <int K>
static hipError_t launch_restore_bs_kk(const FastRestoreArgs &a, hipStream_t s, bool regen) {
  const bool stream = a.groups_per_obj % 4 != 0;
  if (regen) return stream ? launch_restore_bs_k<K, true, true>(a, s) : launch_restore_bs_k<K, false, true>(a, s);
  return stream ? launch_restore_bs_k<K, true, false>(a, s) : launch_restore_bs_k<K, false, false>(a, s);
}

hipError_t launch_restore_fast(uint32_t k, const FastRestoreArgs &a, hipStream_t s, bool regen) {
  if (k == 16) return launch_restore_bs_kk<16>(a, s, regen);
  if (k == 32) return launch_restore_bs_kk<32>(a, s, regen);
  return hipErrorNotSupported;
}

}  // namespace vds_ec
