// pcie_duplex.hip -- why do H2D + D2H together move only one direction's
// bytes?  Host <-> device transfer ceilings by mechanism:
//   sdma_h2d / sdma_d2h      hipMemcpyAsync from / to pinned host memory
//   sdma_both                both at once on two streams
//   pull_h2d                 a kernel reads pinned host memory (mapped) and
//                            writes device memory (zero-copy read over PCIe)
//   push_d2h                 a kernel reads device memory and writes mapped
//                            pinned host memory
//   pull + sdma_d2h, push + sdma_h2d, pull + push   concurrently
// Prints one JSON line of GB/s (each direction's bytes / the time of the
// whole concurrent step).
//   hipcc --offload-arch=gfx950 -O3 tools/ubench/pcie_duplex.hip -o tools/ubench/pcie_duplex
//   tools/ubench/pcie_duplex [MiB]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <functional>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                             \
    }                                                                           \
  } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ void k_copy(const u32x4 *__restrict__ src, u32x4 *__restrict__ dst, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    dst[i] = __builtin_nontemporal_load(src + i);
}

static double best_of(int reps, const std::function<void()> &step) {
  step();
  CK(hipDeviceSynchronize());
  double best = 1e30;
  for (int r = 0; r < reps; ++r) {
    auto t0 = std::chrono::steady_clock::now();
    step();
    CK(hipDeviceSynchronize());
    double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (dt < best) best = dt;
  }
  return best;
}

int main(int argc, char **argv) {
  const size_t mib = argc > 1 ? std::strtoul(argv[1], nullptr, 10) : 256;
  const size_t N = mib << 20, n4 = N / 16;
  uint8_t *hA, *hB, *dA, *dB, *dC, *dD;
  CK(hipHostMalloc(&hA, N, hipHostMallocMapped));
  CK(hipHostMalloc(&hB, N, hipHostMallocMapped));
  for (size_t i = 0; i < N; i += 4096) hA[i] = hB[i] = (uint8_t)i;
  CK(hipMalloc(&dA, N));
  CK(hipMalloc(&dB, N));
  CK(hipMalloc(&dC, N));
  CK(hipMalloc(&dD, N));
  CK(hipMemset(dA, 1, N));
  CK(hipMemset(dB, 2, N));
  uint8_t *hAd, *hBd;  // device views of the mapped host buffers
  CK(hipHostGetDevicePointer((void **)&hAd, hA, 0));
  CK(hipHostGetDevicePointer((void **)&hBd, hB, 0));
  hipStream_t s1, s2;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  const int grid = 1024, block = 256;
  auto pull = [&](hipStream_t s) {  // host -> device by a kernel
    hipLaunchKernelGGL(k_copy, dim3(grid), dim3(block), 0, s, (const u32x4 *)hAd, (u32x4 *)dC, n4);
  };
  auto push = [&](hipStream_t s) {  // device -> host by a kernel
    hipLaunchKernelGGL(k_copy, dim3(grid), dim3(block), 0, s, (const u32x4 *)dD, (u32x4 *)hBd, n4);
  };
  auto gb = [&](double t) { return N / t / 1e9; };
  const int R = 5;
  double t;
  std::printf("{\"bytes\": %zu", N);
  t = best_of(R, [&] { CK(hipMemcpyAsync(dA, hA, N, hipMemcpyHostToDevice, s1)); });
  std::printf(", \"sdma_h2d\": %.2f", gb(t));
  t = best_of(R, [&] { CK(hipMemcpyAsync(hB, dB, N, hipMemcpyDeviceToHost, s1)); });
  std::printf(", \"sdma_d2h\": %.2f", gb(t));
  t = best_of(R, [&] {
    CK(hipMemcpyAsync(dA, hA, N, hipMemcpyHostToDevice, s1));
    CK(hipMemcpyAsync(hB, dB, N, hipMemcpyDeviceToHost, s2));
  });
  std::printf(", \"sdma_both_each\": %.2f", gb(t));
  t = best_of(R, [&] { pull(s1); });
  std::printf(", \"pull_h2d\": %.2f", gb(t));
  t = best_of(R, [&] { push(s1); });
  std::printf(", \"push_d2h\": %.2f", gb(t));
  t = best_of(R, [&] {
    pull(s1);
    CK(hipMemcpyAsync(hB, dB, N, hipMemcpyDeviceToHost, s2));
  });
  std::printf(", \"pull_plus_sdma_d2h_each\": %.2f", gb(t));
  t = best_of(R, [&] {
    push(s1);
    CK(hipMemcpyAsync(dA, hA, N, hipMemcpyHostToDevice, s2));
  });
  std::printf(", \"push_plus_sdma_h2d_each\": %.2f", gb(t));
  t = best_of(R, [&] {
    pull(s1);
    push(s2);
  });
  std::printf(", \"pull_plus_push_each\": %.2f", gb(t));
  std::printf("}\n");
  return 0;
}
