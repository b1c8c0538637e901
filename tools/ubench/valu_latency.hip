// Microbenchmark: chip-wide issue rate of the XOR-family VALU instructions the
// bit-sliced kernels are made of (v_xor_b32, v_bitop3_b32 with VGPR / SGPR
// operands, v_bfi_b32, v_perm_b32), 8 independent chains, 1..4 waves per
// SIMD.  Sizes the instruction budget of the XOR-program generator.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

enum Op { XOR2, BITOP3_V, BITOP3_S, BFI, PERM, PERM_V, LSHL, BITOP3_LIT, ALIGNBIT, DPP, AND_LIT, LSHL_OR };

template <int OP>
__global__ __launch_bounds__(1024) void k_rate(uint32_t *out, uint32_t seed, int iters) {
  constexpr int C = 8;
  uint32_t v[C], w[C];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    v[c] = seed * (threadIdx.x + 1) + c;
    w[c] = (seed ^ threadIdx.x) * 2654435761u + 7 * c;
  }
  const uint32_t k = seed + 99u;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
      for (int c = 0; c < C; ++c) {
        if constexpr (OP == XOR2) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(v[c]) : "v"(w[c]));
        if constexpr (OP == BITOP3_V)
          asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(v[c]) : "v"(w[c]), "v"(w[(c + 1) % C]));
        if constexpr (OP == BITOP3_S)
          asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(v[c]) : "v"(w[c]), "s"(k));
        if constexpr (OP == BFI) asm volatile("v_bfi_b32 %0, %1, %0, %2" : "+v"(v[c]) : "v"(w[c]), "v"(w[(c + 1) % C]));
        if constexpr (OP == PERM) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(v[c]) : "v"(w[c]), "s"(k));
        if constexpr (OP == PERM_V) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(v[c]) : "v"(w[c]), "v"(w[(c + 1) % C]));
        if constexpr (OP == LSHL) asm volatile("v_lshlrev_b32 %0, 4, %0" : "+v"(v[c]));
        if constexpr (OP == BITOP3_LIT)
          asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0xca" : "+v"(v[c]) : "v"(w[c]), "v"(k));
        if constexpr (OP == ALIGNBIT) asm volatile("v_alignbit_b32 %0, %0, %1, 4" : "+v"(v[c]) : "v"(w[c]));
        if constexpr (OP == DPP) asm volatile("v_mov_b32_dpp %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(v[c]) : "v"(w[c]));
        if constexpr (OP == AND_LIT) asm volatile("v_and_b32 %0, 0x0f0f0f0f, %0" : "+v"(v[c]));
        if constexpr (OP == LSHL_OR) asm volatile("v_lshl_or_b32 %0, %0, 4, %1" : "+v"(v[c]) : "v"(w[c]));
      }
    // keep w live and changing so nothing is hoisted
#pragma unroll
    for (int c = 0; c < C; ++c) w[c] += 1;
  }
  uint32_t acc = 0;
#pragma unroll
  for (int c = 0; c < C; ++c) acc ^= v[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int OP>
static void run(const char *name, int waves_per_cu) {
  uint32_t *out;
  const int threads = 64 * waves_per_cu;
  (void)hipMalloc(&out, sizeof(uint32_t) * threads * 256);
  const int iters = 4000;
  hipLaunchKernelGGL(k_rate<OP>, dim3(256), dim3(threads), 0, 0, out, 7u, iters);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  (void)hipEventRecord(a);
  hipLaunchKernelGGL(k_rate<OP>, dim3(256), dim3(threads), 0, 0, out, 7u, iters);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  const double instr = (double)iters * 64;  // measured op instructions per wave (+8 adds per iter ignored)
  std::printf("%-9s waves/SIMD=%d  chip wave-instr/ns=%.1f  ns/instr/wave=%.3f\n", name, waves_per_cu / 4,
              256.0 * waves_per_cu * instr / (ms * 1e6), ms * 1e6 / instr);
  (void)hipFree(out);
}

int main(int argc, char **argv) {
  // waves per CU to sweep (default 8 and 16 = 2 and 4 waves per SIMD)
  int ws[8] = {8, 16}, nw = 2;
  if (argc > 1) {
    nw = 0;
    for (int i = 1; i < argc && nw < 8; ++i) ws[nw++] = atoi(argv[i]);
  }
  for (int wi = 0; wi < nw; ++wi) {
    const int w = ws[wi];
    run<XOR2>("xor2", w);
    run<BITOP3_V>("bitop3_v", w);
    run<BITOP3_S>("bitop3_s", w);
    run<BITOP3_LIT>("bfi_as_bitop3_vmask", w);
    run<BFI>("bfi", w);
    run<PERM>("perm_s", w);
    run<PERM_V>("perm_v", w);
    run<LSHL>("lshl", w);
    run<ALIGNBIT>("alignbit", w);
    run<DPP>("mov_dpp", w);
    run<AND_LIT>("and_lit", w);
    run<LSHL_OR>("lshl_or", w);
  }
  return 0;
}
