// hbm_pipe.hip -- achievable HBM rate of the codec's two traffic shapes with
// the loads software-pipelined one tile ahead (offline study tool, not
// product code; tools/ubench/hbm_mix.hip had no prefetch, so its stores and
// the next tile's loads never overlapped).
//
// Encode shape (k=16, n=20): per 64 KiB tile, 256 threads read 16 x 1 KiB
// per wave, then each of the 4 waves writes 5 replicas x 4 KiB at
// replica r of object o = out + r * objects * L + o * L (bench.py's layout):
//   W=4  -> 16 dword stores per replica (256 B per wave-instruction, the
//           layout k_encode_bs writes)
//   W=16 -> 4 dwordx4 stores per replica (1 KiB per wave-instruction)
// Restore shape (k=16): per tile, wave w reads 4 survivors x 4 KiB (from 16
// different replica arrays), then writes 16 KiB of the 64 KiB output tile.
// NT = non-temporal stores (and loads for the restore shape), PF = tiles of
// loads in flight ahead of the one being stored (1 or 2).
//
//   hipcc --offload-arch=gfx950 -O3 -o hbm_pipe hbm_pipe.hip && ./hbm_pipe [objects]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                          \
  do {                                                                 \
    hipError_t e_ = (x);                                               \
    if (e_ != hipSuccess) {                                            \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));     \
      std::exit(1);                                                    \
    }                                                                  \
  } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kTile = 65536;

template <bool NT, class T>
__device__ __forceinline__ void st(T *p, T v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}
template <bool NT, class T>
__device__ __forceinline__ T ld(const T *p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}

template <int W, bool NT, int PF>
__global__ __launch_bounds__(256, 2) void k_enc(const uint8_t *in, uint8_t *out, uint64_t tiles, uint32_t tpo,
                                                 uint32_t objects) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint64_t L = (uint64_t)(kTile / 16) * tpo;  // replica bytes per object
  // 64 KiB per tile = 4 waves x 16 KiB: each wave reads 16 x 1 KiB below
  uint64_t t = blockIdx.x;
  u32x4 A[PF][16];
  auto load16 = [&](u32x4(&D)[16], uint64_t tt) {
    const u32x4 *src = (const u32x4 *)(in + tt * kTile) + wave * 1024 + lane;
#pragma unroll
    for (int i = 0; i < 16; ++i) D[i] = src[i * 64];
  };
#pragma unroll
  for (int p = 0; p < PF; ++p)
    if (t + p * gridDim.x < tiles) load16(A[p], t + p * gridDim.x);
  for (; t < tiles; t += gridDim.x) {
    u32x4 acc = A[0][0];
#pragma unroll
    for (int i = 1; i < 16; ++i) acc ^= A[0][i];
#pragma unroll
    for (int p = 0; p + 1 < PF; ++p)
#pragma unroll
      for (int i = 0; i < 16; ++i) A[p][i] = A[p + 1][i];
    const uint64_t nx = t + PF * gridDim.x;
    if (nx < tiles) load16(A[PF - 1], nx);
    // a few real cycles of dependency so the stores are data-dependent
    const uint32_t o = t / tpo, ti = t % tpo;
#pragma unroll
    for (int s = 0; s < 5; ++s) {
      const int r = wave * 5 + s;
      uint8_t *dst = out + (uint64_t)r * objects * L + o * L + (uint64_t)ti * (kTile / 16);
      if constexpr (W == 4) {
        uint32_t *d = (uint32_t *)dst + lane;
#pragma unroll
        for (int j = 0; j < 16; ++j) st<NT>(d + 64 * j, acc[j & 3] ^ (uint32_t)(r + j));
      } else {
        u32x4 *d = (u32x4 *)dst + lane;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          u32x4 v = acc;
          v.x ^= (uint32_t)(r + j);
          st<NT>(d + 64 * j, v);
        }
      }
    }
  }
}

// restore shape: survivors are replicas 4..19 of the encode layout (4 KiB per
// tile each), output tile 64 KiB contiguous
template <bool NT, int PF>
__global__ __launch_bounds__(256, 2) void k_res(const uint8_t *reps, uint8_t *out, uint64_t tiles, uint32_t tpo,
                                                 uint32_t objects) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint64_t L = (uint64_t)(kTile / 16) * tpo;
  u32x4 A[PF][16];
  auto load16 = [&](u32x4(&D)[16], uint64_t tt) {
    const uint32_t o = tt / tpo, ti = tt % tpo;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const u32x4 *src = (const u32x4 *)(reps + (uint64_t)(4 + wave * 4 + s) * objects * L + o * L +
                                         (uint64_t)ti * (kTile / 16)) + lane;
#pragma unroll
      for (int q = 0; q < 4; ++q) D[4 * s + q] = ld<NT>(src + 64 * q);
    }
  };
  uint64_t t = blockIdx.x;
#pragma unroll
  for (int p = 0; p < PF; ++p)
    if (t + p * gridDim.x < tiles) load16(A[p], t + p * gridDim.x);
  for (; t < tiles; t += gridDim.x) {
    u32x4 acc = A[0][0];
#pragma unroll
    for (int i = 1; i < 16; ++i) acc ^= A[0][i];
#pragma unroll
    for (int p = 0; p + 1 < PF; ++p)
#pragma unroll
      for (int i = 0; i < 16; ++i) A[p][i] = A[p + 1][i];
    const uint64_t nx = t + PF * gridDim.x;
    if (nx < tiles) load16(A[PF - 1], nx);
    u32x4 *d = (u32x4 *)(out + t * kTile + wave * 16384) + lane;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      u32x4 v = acc;
      v.y ^= (uint32_t)j;
      st<NT>(d + 64 * j, v);
    }
  }
}

__global__ __launch_bounds__(256) void k_copy(const u32x4 *in, u32x4 *out, uint64_t n) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) out[i] = in[i];
}

int main(int argc, char **argv) {
  const uint32_t objects = argc > 1 ? atoi(argv[1]) : 128;
  const uint64_t obj = 64ull << 20;
  const uint32_t tpo = obj / kTile;
  const uint64_t tiles = (uint64_t)objects * tpo;
  uint8_t *in, *reps, *out;
  CK(hipMalloc(&in, objects * obj));
  CK(hipMalloc(&reps, objects * obj * 20 / 16));
  CK(hipMalloc(&out, objects * obj));
  CK(hipMemset(in, 1, objects * obj));
  CK(hipMemset(reps, 2, objects * obj * 20 / 16));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto time = [&](auto launch, double bytes, const char *name) {
    launch();
    CK(hipDeviceSynchronize());
    float best = 1e30f, sum = 0;
    for (int it = 0; it < 5; ++it) {
      CK(hipEventRecord(e0));
      launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (ms < best) best = ms;
      sum += ms;
    }
    std::printf("%-40s best %8.3f ms %7.1f GB/s  mean %7.1f GB/s\n", name, best, bytes / (best * 1e-3) / 1e9,
                bytes / (sum / 5 * 1e-3) / 1e9);
    std::fflush(stdout);
  };
  const double enc_bytes = (double)objects * obj * (1.0 + 20.0 / 16);
  const double res_bytes = (double)objects * obj * 2.0;
  const uint64_t n16 = objects * obj / 16;
  for (int grid : {1024, 4096}) {
    char nm[96];
    std::snprintf(nm, sizeof nm, "copy float4 grid %d", grid);
    time([&] { hipLaunchKernelGGL(k_copy, dim3(grid), dim3(256), 0, 0, (const u32x4 *)in, (u32x4 *)out, n16); },
         2.0 * objects * obj, nm);
  }
#define ENC(W, NT, PF)                                                                                       \
  for (int grid : {512, 1024}) {                                                                             \
    char nm[96];                                                                                             \
    std::snprintf(nm, sizeof nm, "enc W%d nt%d pf%d grid %d", W, NT, PF, grid);                              \
    time([&] { hipLaunchKernelGGL((k_enc<W, NT, PF>), dim3(grid), dim3(256), 0, 0, in, reps, tiles, tpo, objects); }, \
         enc_bytes, nm);                                                                                     \
  }
  ENC(4, false, 1) ENC(4, true, 1) ENC(16, false, 1) ENC(16, true, 1) ENC(4, true, 2) ENC(16, true, 2)
#define RES(NT, PF)                                                                                          \
  for (int grid : {512, 1024}) {                                                                             \
    char nm[96];                                                                                             \
    std::snprintf(nm, sizeof nm, "res nt%d pf%d grid %d", NT, PF, grid);                                     \
    time([&] { hipLaunchKernelGGL((k_res<NT, PF>), dim3(grid), dim3(256), 0, 0, reps, out, tiles, tpo, objects); }, \
         res_bytes, nm);                                                                                     \
  }
  RES(false, 1) RES(true, 1) RES(false, 2) RES(true, 2)
  return 0;
}
