// hbm_shape.hip -- what the restore's traffic shape can reach on HBM (offline
// study tool, not product code).  tools/ubench/hbm_pipe.hip measured the
// k=16 restore shape (16 survivors x 4 KiB read from 16 replica arrays, 64
// KiB written contiguous per tile) at 4.2-4.6 TB/s against 5.7 TB/s for a
// float4 copy and 5.4 TB/s for the encode shape.  This sweeps what might
// explain the gap:
//   CH   = bytes of each survivor per tile (4, 8 or 16 KiB; the output tile is
//          16 CH), so each read stream is CH contiguous per workgroup visit
//   WV   = waves per workgroup (4 or 8; 8 waves read 2 survivors each)
// plus read-only / write-only streams and copies at several occupancies as
// references.  Prints GB/s of (bytes read + written) / kernel time.
//
// The encode shape (one 16 CH object read, 20 replica chunks of CH written
// per tile) is swept the same way.
//
//   hipcc --offload-arch=gfx950 -O3 -o hbm_shape hbm_shape.hip && ./hbm_shape [objects] [mode: 1 res, 2 enc, 3 both]
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

template <class T>
__device__ __forceinline__ void stn(T *p, T v) { __builtin_nontemporal_store(v, p); }
template <class T>
__device__ __forceinline__ T ldn(const T *p) { return __builtin_nontemporal_load(p); }

// survivors: replicas 4..19 of a [20][objects][L] array, L = objects' replica bytes
template <int CH, int WV>
__global__ __launch_bounds__(64 * WV, 1) void k_res(const uint8_t *reps, uint8_t *out, uint64_t tiles, uint32_t tpo,
                                                     uint64_t L, uint32_t objects) {
  constexpr int SPW = 16 / WV;            // survivors per wave
  constexpr int LPS = CH / 1024;          // 1 KiB loads per survivor
  constexpr int NL = SPW * LPS;           // loads per lane per tile
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  u32x4 A[NL];
  auto load = [&](uint64_t tt) {
    const uint64_t o = tt / tpo, ti = tt % tpo;
#pragma unroll
    for (int s = 0; s < SPW; ++s) {
      const u32x4 *src = (const u32x4 *)(reps + (uint64_t)(4 + wave * SPW + s) * objects * L + o * L + ti * CH) + lane;
#pragma unroll
      for (int q = 0; q < LPS; ++q) A[s * LPS + q] = ldn(src + 64 * q);
    }
  };
  uint64_t t = blockIdx.x;
  if (t < tiles) load(t);
  for (; t < tiles; t += gridDim.x) {
    u32x4 acc = A[0];
#pragma unroll
    for (int i = 1; i < NL; ++i) acc ^= A[i];
    if (t + gridDim.x < tiles) load(t + gridDim.x);
    u32x4 *d = (u32x4 *)(out + t * (16ull * CH) + (uint64_t)wave * (16 * CH / WV)) + lane;
#pragma unroll
    for (int j = 0; j < 16 * CH / WV / 1024; ++j) {
      u32x4 v = acc;
      v.y ^= (uint32_t)j;
      stn(d + 64 * j, v);
    }
  }
}

// encode shape: per tile read 16 CH contiguous (the object), write 20
// replicas x CH (replica r of object o at r * objects * L + o * L); 4 waves,
// wave w writes replicas 5w..5w+4 with dword (W = 4: 256 B per
// wave-instruction, k_encode_bs's store shape) or dwordx4 stores
template <int CH, int W>
__global__ __launch_bounds__(256, 1) void k_enc(const uint8_t *in, uint8_t *reps, uint64_t tiles, uint32_t tpo,
                                                 uint64_t L, uint32_t objects) {
  constexpr int NL = 16 * CH / 4 / 1024;  // 1 KiB loads per wave
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  u32x4 A[NL];
  auto load = [&](uint64_t tt) {
    const u32x4 *src = (const u32x4 *)(in + tt * (16ull * CH) + (uint64_t)wave * (4 * CH)) + lane;
#pragma unroll
    for (int q = 0; q < NL; ++q) A[q] = ldn(src + 64 * q);
  };
  uint64_t t = blockIdx.x;
  if (t < tiles) load(t);
  for (; t < tiles; t += gridDim.x) {
    u32x4 acc = A[0];
#pragma unroll
    for (int i = 1; i < NL; ++i) acc ^= A[i];
    if (t + gridDim.x < tiles) load(t + gridDim.x);
    const uint64_t o = t / tpo, ti = t % tpo;
#pragma unroll
    for (int s = 0; s < 5; ++s) {
      const int r = 5 * wave + s;
      uint8_t *dst = reps + (uint64_t)r * objects * L + o * L + ti * CH;
      if constexpr (W == 4) {
        uint32_t *d = (uint32_t *)dst + lane;
#pragma unroll
        for (int j = 0; j < CH / 256; ++j) stn(d + 64 * j, acc[j & 3] ^ (uint32_t)(r + j));
      } else {
        u32x4 *d = (u32x4 *)dst + lane;
#pragma unroll
        for (int j = 0; j < CH / 1024; ++j) {
          u32x4 v = acc;
          v.x ^= (uint32_t)(r + j);
          stn(d + 64 * j, v);
        }
      }
    }
  }
}

__global__ __launch_bounds__(256) void k_copy(const u32x4 *in, u32x4 *out, uint64_t n) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) out[i] = in[i];
}

// copy with 4 independent 16-B loads per lane in flight
__global__ __launch_bounds__(256) void k_copy4(const u32x4 *in, u32x4 *out, uint64_t n) {
  const uint64_t step = (uint64_t)gridDim.x * 256;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i + 3 * step < n; i += 4 * step) {
    u32x4 a = ldn(in + i), b = ldn(in + i + step), c = ldn(in + i + 2 * step), d = ldn(in + i + 3 * step);
    stn(out + i, a);
    stn(out + i + step, b);
    stn(out + i + 2 * step, c);
    stn(out + i + 3 * step, d);
  }
}

__global__ __launch_bounds__(256) void k_read(const u32x4 *in, u32x4 *sink, uint64_t n) {
  const uint64_t step = (uint64_t)gridDim.x * 256;
  u32x4 acc = {0, 0, 0, 0};
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i + 3 * step < n; i += 4 * step)
    acc ^= ldn(in + i) ^ ldn(in + i + step) ^ ldn(in + i + 2 * step) ^ ldn(in + i + 3 * step);
  if (acc.x == 0x12345678u) sink[0] = acc;
}

__global__ __launch_bounds__(256) void k_write(u32x4 *out, uint64_t n) {
  const uint64_t step = (uint64_t)gridDim.x * 256;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += step) stn(out + i, u32x4{(uint32_t)i, 1u, 2u, 3u});
}

int main(int argc, char **argv) {
  const uint32_t objects = argc > 1 ? atoi(argv[1]) : 128;
  const uint64_t obj = 64ull << 20;
  const uint64_t L = obj / 16;
  uint8_t *reps, *out;
  CK(hipMalloc(&reps, objects * L * 20));
  CK(hipMalloc(&out, objects * obj));
  CK(hipMemset(reps, 2, objects * L * 20));
  CK(hipMemset(out, 3, objects * obj));
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
    std::printf("%-36s best %8.3f ms %7.1f GB/s  mean %7.1f GB/s\n", name, best, bytes / (best * 1e-3) / 1e9,
                bytes / (sum / 5 * 1e-3) / 1e9);
    std::fflush(stdout);
  };
  const uint64_t n16 = objects * obj / 16;
  const u32x4 *src = (const u32x4 *)reps;
  for (int grid : {512, 1024, 2048}) {
    char nm[96];
    std::snprintf(nm, sizeof nm, "copy grid %d", grid);
    time([&] { hipLaunchKernelGGL(k_copy, dim3(grid), dim3(256), 0, 0, src, (u32x4 *)out, n16); }, 2.0 * n16 * 16, nm);
    std::snprintf(nm, sizeof nm, "copy4 nt grid %d", grid);
    time([&] { hipLaunchKernelGGL(k_copy4, dim3(grid), dim3(256), 0, 0, src, (u32x4 *)out, n16); }, 2.0 * n16 * 16, nm);
    std::snprintf(nm, sizeof nm, "read4 nt grid %d", grid);
    time([&] { hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, 0, src, (u32x4 *)out, n16); }, 1.0 * n16 * 16, nm);
    std::snprintf(nm, sizeof nm, "write nt grid %d", grid);
    time([&] { hipLaunchKernelGGL(k_write, dim3(grid), dim3(256), 0, 0, (u32x4 *)out, n16); }, 1.0 * n16 * 16, nm);
  }
#define RES(CH, WV)                                                                                                  \
  for (int grid : {256, 512, 1024}) {                                                                               \
    const uint32_t tpo = (uint32_t)(L / (CH));                                                                       \
    const uint64_t tiles = (uint64_t)objects * tpo;                                                                  \
    char nm[96];                                                                                                     \
    std::snprintf(nm, sizeof nm, "res ch%dK wv%d grid %d", (CH) / 1024, WV, grid);                                   \
    time([&] { hipLaunchKernelGGL((k_res<CH, WV>), dim3(grid), dim3(64 * (WV)), 0, 0, reps, out, tiles, tpo, L, objects); }, \
         2.0 * objects * obj, nm);                                                                                   \
  }
  const int mode = argc > 2 ? atoi(argv[2]) : 3;
  if (mode & 1) { RES(4096, 4) RES(4096, 8) RES(8192, 4) RES(8192, 8) RES(16384, 8) }
#define ENC(CH, W)                                                                                                   \
  for (int grid : {256, 384, 512, 1024}) {                                                                          \
    const uint32_t tpo = (uint32_t)(L / (CH));                                                                       \
    const uint64_t tiles = (uint64_t)objects * tpo;                                                                  \
    char nm[96];                                                                                                     \
    std::snprintf(nm, sizeof nm, "enc ch%dK W%d grid %d", (CH) / 1024, W, grid);                                     \
    time([&] { hipLaunchKernelGGL((k_enc<CH, W>), dim3(grid), dim3(256), 0, 0, out, reps, tiles, tpo, L, objects); }, \
         (double)objects * obj * (1.0 + 20.0 / 16), nm);                                                             \
  }
  if (mode & 2) { ENC(4096, 4) ENC(4096, 16) ENC(8192, 4) ENC(8192, 16) ENC(16384, 16) }
  return 0;
}
