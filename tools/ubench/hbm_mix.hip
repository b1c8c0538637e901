// hbm_mix.hip -- achievable HBM rate for the encode's traffic mix (offline
// study tool, not product code).
//
// Every kernel reads a 64 KiB tile per workgroup iteration and writes
// `reps` x (tile / ratio) bytes with ideal 16-byte-per-lane instructions:
//   layout 0: replica r of object o at r * (objects * L) + o * L  (bench.py's layout)
//   layout 1: the tile's whole output contiguous (one write stream)
// and a plain copy (read N, write N) for reference.  Prints GB/s of
// (bytes read + bytes written) / kernel time.
//
//   hipcc --offload-arch=gfx950 -O3 -o hbm_mix hbm_mix.hip && ./hbm_mix
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));             \
      std::exit(1);                                                            \
    }                                                                          \
  } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kTile = 65536;

// One workgroup of 256 threads per tile: 64 KiB in = 16 dwordx4 per lane
// (4 KiB per wave-instruction across the workgroup), output `reps` chunks
// of kTile / ratio bytes.
__global__ __launch_bounds__(256) void k_mix(const uint8_t *in, uint8_t *out, uint64_t tiles, uint32_t tiles_per_obj,
                                             uint32_t objects, int reps, int ratio, int layout) {
  const uint32_t chunk = kTile / ratio;  // bytes per replica per tile
  const uint64_t L = (uint64_t)chunk * tiles_per_obj;
  for (uint64_t t = blockIdx.x; t < tiles; t += gridDim.x) {
    const u32x4 *src = (const u32x4 *)(in + t * kTile);
    u32x4 acc = {0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < kTile / 16 / 256; ++i) {
      const u32x4 v = src[i * 256 + threadIdx.x];
      acc ^= v;
    }
    const uint32_t o = t / tiles_per_obj, ti = t % tiles_per_obj;
    for (int r = 0; r < reps; ++r) {
      uint8_t *dst = layout == 0 ? out + (uint64_t)r * objects * L + o * L + (uint64_t)ti * chunk
                                 : out + t * (uint64_t)chunk * reps + (uint64_t)r * chunk;
      for (uint32_t b = threadIdx.x * 16; b < chunk; b += 256 * 16) {
        u32x4 v = acc;
        v.x ^= r;
        *(u32x4 *)(dst + b) = v;
      }
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
  uint8_t *in, *out;
  CK(hipMalloc(&in, objects * obj));
  CK(hipMalloc(&out, objects * obj * 3 / 2));
  CK(hipMemset(in, 1, objects * obj));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto time = [&](auto launch, double bytes, const char *name) {
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
    std::printf("%-44s %8.3f ms  %7.1f GB/s\n", name, best, bytes / (best * 1e-3) / 1e9);
  };
  const uint64_t n16 = objects * obj / 16;
  for (int grid : {1024, 4096}) {
    char nm[96];
    std::snprintf(nm, sizeof nm, "copy (read N, write N) grid %d", grid);
    time([&] { hipLaunchKernelGGL(k_copy, dim3(grid), dim3(256), 0, 0, (const u32x4 *)in, (u32x4 *)out, n16); },
         2.0 * objects * obj, nm);
  }
  struct Cfg { int reps, ratio; const char *what; } cfgs[] = {{20, 16, "k16 n20"}, {40, 32, "k32 n40"}, {1, 1, "1 rep"}};
  for (auto c : cfgs)
    for (int layout : {0, 1})
      for (int grid : {512, 1024, 2048}) {
        char nm[96];
        std::snprintf(nm, sizeof nm, "mix %s layout %d grid %d", c.what, layout, grid);
        const double bytes = (double)objects * obj * (1.0 + (double)c.reps / c.ratio);
        time([&] { hipLaunchKernelGGL(k_mix, dim3(grid), dim3(256), 0, 0, in, out, tiles, tpo, objects, c.reps, c.ratio, layout); },
             bytes, nm);
      }
  return 0;
}
