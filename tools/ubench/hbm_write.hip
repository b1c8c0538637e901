// hbm_write.hip -- write-side HBM ceiling sweep (offline study tool, not
// product code): is ~5.4 TB/s the most a write-only stream reaches on this
// part, or only what tools/ubench/hbm_shape.hip's launch shapes reach?
// Sweeps block size, grid, stores per lane per iteration (ILP) and cache
// policy (plain / non-temporal) for a grid-strided 16-byte store stream into
// a buffer far larger than the 256 MiB Infinity Cache, plus the same shapes
// for a read stream and a copy.
//
//   hipcc --offload-arch=gfx950 -O3 -o hbm_write hbm_write.hip && ./hbm_write [GiB]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                      \
  do {                                                             \
    hipError_t e_ = (x);                                           \
    if (e_ != hipSuccess) {                                        \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); \
      std::exit(1);                                                \
    }                                                              \
  } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ void st(u32x4 *p, u32x4 v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}
template <bool NT>
__device__ __forceinline__ u32x4 ld(const u32x4 *p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}

// U stores per lane per iteration, each a whole block-wide 16-B store stream
template <int B, int U, bool NT>
__global__ __launch_bounds__(B) void k_write(u32x4 *out, uint64_t n) {
  const uint64_t step = (uint64_t)gridDim.x * B;
  for (uint64_t i = blockIdx.x * (uint64_t)B * U + threadIdx.x; i < n; i += step * U) {
#pragma unroll
    for (int u = 0; u < U; ++u) st<NT>(out + i + (uint64_t)u * B, u32x4{(uint32_t)i, (uint32_t)u, 2u, 3u});
  }
}

template <int B, int U, bool NT>
__global__ __launch_bounds__(B) void k_read(const u32x4 *in, u32x4 *sink, uint64_t n) {
  const uint64_t step = (uint64_t)gridDim.x * B;
  u32x4 acc = {0, 0, 0, 0};
  for (uint64_t i = blockIdx.x * (uint64_t)B * U + threadIdx.x; i < n; i += step * U) {
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= ld<NT>(in + i + (uint64_t)u * B);
  }
  if (acc.x == 0x12345678u) sink[0] = acc;
}

template <int B, int U, bool NT>
__global__ __launch_bounds__(B) void k_copy(const u32x4 *in, u32x4 *out, uint64_t n) {
  const uint64_t step = (uint64_t)gridDim.x * B;
  for (uint64_t i = blockIdx.x * (uint64_t)B * U + threadIdx.x; i < n; i += step * U) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ld<NT>(in + i + (uint64_t)u * B);
#pragma unroll
    for (int u = 0; u < U; ++u) st<NT>(out + i + (uint64_t)u * B, v[u]);
  }
}

// The encode's store shape: NR replica streams (rep_stride apart), each tile
// writes CH bytes per replica as dword stores (256 B per wave-instruction),
// 4 waves per workgroup, NR/4 replicas each.  MAP 0: tile t on workgroup
// t mod grid (the encode's order; workgroup b runs on XCD b mod 8, so
// adjacent tiles are on different XCDs); MAP 1: each XCD walks its own
// contiguous eighth of the tiles (adjacent tiles on one XCD).
template <int NR, int CH, int MAP, bool WIDE = false>
__global__ __launch_bounds__(256) void k_encw(uint8_t *reps, uint64_t tiles, uint64_t rep_stride) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint64_t G = gridDim.x, x = blockIdx.x % 8, j = blockIdx.x / 8, per_x = tiles / 8;
  for (uint64_t k = 0;; ++k) {
    uint64_t t;
    if constexpr (MAP == 0) {
      t = k * G + blockIdx.x;
      if (t >= tiles) break;
    } else {
      const uint64_t i = k * (G / 8) + j;
      if (i >= per_x) break;
      t = x * per_x + i;
    }
#pragma unroll
    for (int s = 0; s < NR / 4; ++s) {
      const int r = (NR / 4) * wave + s;
      if constexpr (WIDE) {
        u32x4 *d = (u32x4 *)(reps + (uint64_t)r * rep_stride + t * CH) + lane;
#pragma unroll
        for (int q = 0; q < CH / 1024; ++q) __builtin_nontemporal_store(u32x4{(uint32_t)t, (uint32_t)r, (uint32_t)q, 0u}, d + 64 * q);
      } else {
        uint32_t *d = (uint32_t *)(reps + (uint64_t)r * rep_stride + t * CH) + lane;
#pragma unroll
        for (int q = 0; q < CH / 256; ++q) __builtin_nontemporal_store((uint32_t)(t ^ r ^ q), d + 64 * q);
      }
    }
  }
}

int main(int argc, char **argv) {
  const uint64_t gib = argc > 1 ? atoi(argv[1]) : 4;
  const uint64_t bytes = gib << 30, n = bytes / 16;
  u32x4 *a, *b;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&b, bytes));
  CK(hipMemset(a, 1, bytes));
  CK(hipMemset(b, 2, bytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto time = [&](auto launch, double moved, const char *name) {
    launch();
    CK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int it = 0; it < 5; ++it) {
      CK(hipEventRecord(e0));
      launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (ms < best) best = ms;
    }
    std::printf("%-40s best %8.3f ms %7.1f GB/s\n", name, best, moved / (best * 1e-3) / 1e9);
    std::fflush(stdout);
  };
#define SWEEP(B, U, NT)                                                                                          \
  for (int grid : {256, 512, 1024, 2048, 4096}) {                                                              \
    char nm[96];                                                                                               \
    std::snprintf(nm, sizeof nm, "write B%d U%d nt%d grid %d", B, U, (int)NT, grid);                           \
    time([&] { hipLaunchKernelGGL((k_write<B, U, NT>), dim3(grid), dim3(B), 0, 0, b, n); }, 1.0 * bytes, nm); \
    std::snprintf(nm, sizeof nm, "read  B%d U%d nt%d grid %d", B, U, (int)NT, grid);                           \
    time([&] { hipLaunchKernelGGL((k_read<B, U, NT>), dim3(grid), dim3(B), 0, 0, a, b, n); }, 1.0 * bytes, nm); \
    std::snprintf(nm, sizeof nm, "copy  B%d U%d nt%d grid %d", B, U, (int)NT, grid);                           \
    time([&] { hipLaunchKernelGGL((k_copy<B, U, NT>), dim3(grid), dim3(B), 0, 0, a, b, n); }, 2.0 * bytes, nm); \
  }
  {
#define ENCW(NR, CH, MAP, W)                                                                                \
  for (int grid : {256, 512, 1024}) {                                                                      \
    const uint64_t rs = (bytes / (NR)) & ~(uint64_t)((CH) - 1), tiles = (rs / (CH)) & ~7ull;               \
    char nm[96];                                                                                           \
    std::snprintf(nm, sizeof nm, "encw streams %d chunk %dK map %d wide %d grid %d", NR, (CH) / 1024, MAP, W, grid);  \
    time([&] { hipLaunchKernelGGL((k_encw<NR, CH, MAP, W>), dim3(grid), dim3(256), 0, 0, (uint8_t *)b, tiles, rs); }, \
         (double)(NR) * tiles * (CH), nm);                                                                 \
  }
    ENCW(4, 4096, 0, false) ENCW(4, 4096, 0, true) ENCW(4, 4096, 1, false) ENCW(4, 4096, 1, true)
    ENCW(20, 4096, 0, false) ENCW(20, 4096, 0, true) ENCW(20, 4096, 1, false) ENCW(20, 4096, 1, true)
  }
  if (argc > 2) return 0;
  SWEEP(256, 1, false)
  SWEEP(256, 4, false)
  SWEEP(256, 4, true)
  SWEEP(1024, 1, false)
  SWEEP(1024, 4, false)
  SWEEP(1024, 4, true)
  SWEEP(512, 8, true)
  SWEEP(512, 8, false)
  return 0;
}
