// ec_generic.hip -- the any-shape kernels of the object-chunk erasure codec.
//
// One lane per output cell with the carry-less field multiply: any k, any
// replica ids, 8- or 16-bit cells.  They handle the tails of the bit-sliced
// kernels (partial tiles, the last partial stripe, trailers) and every shape
// those are not instantiated for (e.g. chunk_storage's 800-of-1000 ids, the
// uint8_t template, the cell-array test paths).  Plus the synthetic-object
// generator used by bench.py and the tests.
#include <mutex>

#include "ec_device.hpp"

namespace vds_ec {

template <int CB>
__device__ __forceinline__ uint32_t gf_mul_cell(uint32_t a, uint32_t b) {
  if constexpr (CB == 2)
    return gf16_mul(a, b);
  else
    return gf8_mul(a, b);
}

// Cell j of stripe t of an object, zero beyond `size` (chunk.h:254-260).
template <int CB>
__device__ __forceinline__ uint32_t read_cell(const uint8_t *obj, uint64_t size, uint64_t t, uint32_t j,
                                              uint32_t k, bool native) {
  const uint64_t pos = (t * k + j) * CB;
  if constexpr (CB == 1) {
    return pos < size ? obj[pos] : 0u;
  } else {
    if (native) {  // cell arrays: whole native uint16 cells (chunk.h:213-221)
      return pos + 1 < size ? (uint32_t)(obj[pos] | (obj[pos + 1] << 8)) : 0u;
    }
    uint32_t hi = pos < size ? obj[pos] : 0u;
    uint32_t lo = pos + 1 < size ? obj[pos + 1] : 0u;
    return (hi << 8) | lo;
  }
}

template <int CB>
__global__ void k_encode_generic(GenericEncodeArgs a) {
  const uint64_t per_rep = a.t_count + (a.write_trailer ? 1 : 0);
  const uint64_t total = per_rep * a.nrep * (uint64_t)a.count;
  const bool native = (a.flags & 0x2u) != 0;
  for (uint64_t idx = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; idx < total;
       idx += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t ti = idx % per_rep;
    const uint64_t rest = idx / per_rep;
    const uint32_t i = (uint32_t)(rest % a.nrep);
    const uint32_t o = (uint32_t)(rest / a.nrep);
    uint8_t *out = a.outs[i] + (uint64_t)o * a.out_stride;
    if (ti == a.t_count) {
      // trailer BE16(size % (k*cell)) after the T cells (chunk.h:273-275)
      const uint64_t pad = a.size % ((uint64_t)a.k * CB);
      out[a.stripes * CB] = (uint8_t)(pad >> 8);
      out[a.stripes * CB + 1] = (uint8_t)(pad & 0xFF);
      continue;
    }
    const uint64_t t = a.t_begin + ti;
    const uint8_t *obj = a.in + (uint64_t)o * a.in_stride;
    const uint32_t node = a.nodes[i];
    uint32_t acc = 0;
    for (int32_t j = (int32_t)a.k - 1; j >= 0; --j)  // Horner: sum_j node^j x_j
      acc = gf_mul_cell<CB>(acc, node) ^ read_cell<CB>(obj, a.size, t, (uint32_t)j, a.k, native);
    if constexpr (CB == 2) {
      if (native) {
        out[2 * t] = (uint8_t)(acc & 0xFF);
        out[2 * t + 1] = (uint8_t)(acc >> 8);
      } else {
        out[2 * t] = (uint8_t)(acc >> 8);  // binary_serialize.cpp:18-22
        out[2 * t + 1] = (uint8_t)(acc & 0xFF);
      }
    } else {
      out[t] = (uint8_t)acc;
    }
  }
}

template <int CB>
__global__ void k_restore_generic(GenericRestoreArgs a) {
  const uint64_t per_obj = a.t_count * a.k;
  const uint64_t total = per_obj * a.count;
  const bool native = (a.flags & 0x2u) != 0;
  for (uint64_t idx = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; idx < total;
       idx += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t o = (uint32_t)(idx / per_obj);
    const uint64_t r = idx % per_obj;
    const uint64_t t = a.t_begin + r / a.k;
    const uint32_t m = (uint32_t)(r % a.k);
    const uint64_t pos = (t * a.k + m) * CB;
    if (pos >= a.out_len) continue;
    uint32_t acc = 0;
    const uint64_t row = (uint64_t)m * a.k;
    for (uint32_t j = 0; j < a.k; ++j) {
      const uint8_t *base = a.chunk_pitch ? a.chunk_base + (uint64_t)j * a.chunk_pitch
                                          : (a.chunk_table ? a.chunk_table[j] : a.chunk_ptr[j]);
      const uint8_t *c = base + (uint64_t)o * a.chunk_stride + t * CB;
      const uint64_t e = row + j;
      const uint32_t coef = a.matrix_dev ? a.matrix_dev[e] : (a.matrix_inline[e >> 1] >> (16 * (e & 1))) & 0xFFFFu;
      uint32_t cell;
      if constexpr (CB == 2)
        cell = native ? (uint32_t)(c[0] | (c[1] << 8)) : (uint32_t)((c[0] << 8) | c[1]);
      else
        cell = c[0];
      acc ^= gf_mul_cell<CB>(coef, cell);
    }
    uint8_t *out = a.out + (uint64_t)o * a.out_stride;
    if constexpr (CB == 2) {
      const uint8_t b0 = native ? (uint8_t)(acc & 0xFF) : (uint8_t)(acc >> 8);
      const uint8_t b1 = native ? (uint8_t)(acc >> 8) : (uint8_t)(acc & 0xFF);
      out[pos] = b0;
      if (pos + 1 < a.out_len) out[pos + 1] = b1;  // trimmed to E bytes (chunk.h:437-439)
    } else {
      out[pos] = (uint8_t)acc;
    }
  }
}

template <int CB>
__global__ void k_regen_generic(RegenArgs a) {
  const uint64_t per = a.t_count + 1;  // cells + the trailer
  const uint64_t total = per * a.nt * (uint64_t)a.count;
  for (uint64_t idx = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; idx < total;
       idx += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t ti = idx % per;
    const uint64_t rest = idx / per;
    const uint32_t i = (uint32_t)(rest % a.nt);
    const uint32_t o = (uint32_t)(rest / a.nt);
    uint8_t *out = a.outs[i] + (uint64_t)o * a.out_stride;
    auto chunk = [&](uint32_t j) {
      return (a.chunk_table ? a.chunk_table[j] : a.chunk_ptr[j]) + (uint64_t)o * a.chunk_stride;
    };
    if (ti == a.t_count) {  // trailer BE16(size % (k*cell)), identical in every replica (chunk.h:273-275)
      const uint8_t *c0 = chunk(0);
      out[a.T * CB] = c0[a.T * CB];
      out[a.T * CB + 1] = c0[a.T * CB + 1];
      continue;
    }
    const uint64_t t = a.t_begin + ti;
    uint32_t acc = 0;
    for (uint32_t j = 0; j < a.k; ++j) {
      const uint64_t e = (uint64_t)i * a.k + j;
      const uint32_t coef = a.coef_dev ? a.coef_dev[e] : (a.coef_inline[e >> 1] >> (16 * (e & 1))) & 0xFFFFu;
      const uint8_t *c = chunk(j) + t * CB;
      const uint32_t cell = CB == 2 ? (uint32_t)((c[0] << 8) | c[1]) : (uint32_t)c[0];
      acc ^= gf_mul_cell<CB>(coef, cell);
    }
    if constexpr (CB == 2) {
      out[2 * t] = (uint8_t)(acc >> 8);  // binary_serialize.cpp:18-22
      out[2 * t + 1] = (uint8_t)(acc & 0xFF);
    } else {
      out[t] = (uint8_t)acc;
    }
  }
}

// ============================================================ regenerate tail
// (RegenTailArgs, ec_internal.hpp): the last cell and the trailer of every
// target replica as restore (trimmed to E) + re-encode writes them.

__device__ __forceinline__ uint32_t be16_at(const uint8_t *p) { return (uint32_t)((p[0] << 8) | p[1]); }
__device__ __forceinline__ void put_be16(uint8_t *p, uint32_t v) {
  p[0] = (uint8_t)(v >> 8);
  p[1] = (uint8_t)(v & 0xFF);
}
// Decoded cell j of the last stripe as the reference's trimmed object holds
// it: bytes [0, p) of the stripe kept (cell j = bytes 2j, 2j+1).
__device__ __forceinline__ uint32_t trim_cell(uint32_t u, uint32_t j, uint32_t p) {
  return 2 * j + 1 < p ? u : (2 * j + 1 == p ? (u & 0xFF00u) : 0u);
}

// One survivor set, host inverse: workgroup per object.  Threads j < J =
// ceil(p/2) decode cell j of the last stripe (row j of V_S^{-1}), trimmed,
// into LDS; then each target is a Horner over those J cells.
__global__ void k_regen_tail(RegenTailArgs a) {
  extern __shared__ uint16_t tail_cells[];
  const uint64_t L = a.chunk_size, T = (L - 2) / 2;
  for (uint32_t o = blockIdx.x; o < a.count; o += gridDim.x) {
    auto chunk = [&](uint32_t j) {
      return (a.chunk_table ? a.chunk_table[j] : a.chunk_ptr[j]) + (uint64_t)o * a.chunk_stride;
    };
    const uint32_t p = be16_at(chunk(0) + L - 2);
    if (p > 2 * a.k) continue;  // no chunk_size-byte reference answer (ec_internal.hpp)
    const uint32_t trailer = p == 2 * a.k ? 0u : p;
    for (uint32_t i = threadIdx.x; i < a.nt; i += blockDim.x) put_be16(a.outs[i] + (uint64_t)o * a.out_stride + 2 * T, trailer);
    if (p == 0 || p == 2 * a.k || T == 0) continue;  // nothing trimmed
    const uint32_t J = (p + 1) / 2;
    for (uint32_t j = threadIdx.x; j < J; j += blockDim.x) {
      uint32_t u = 0;
      for (uint32_t s = 0; s < a.k; ++s) {
        const uint64_t e = (uint64_t)j * a.k + s;
        const uint32_t coef = a.matrix_dev ? a.matrix_dev[e] : (a.matrix_inline[e >> 1] >> (16 * (e & 1))) & 0xFFFFu;
        u ^= gf16_mul(coef, be16_at(chunk(s) + 2 * (T - 1)));
      }
      tail_cells[j] = (uint16_t)trim_cell(u, j, p);
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < a.nt; i += blockDim.x) {
      uint32_t acc = 0;  // sum_j cell_j t^j (chunk.h:251-265)
      for (uint32_t j = J; j-- > 0;) acc = gf16_mul(acc, a.targets[i]) ^ tail_cells[j];
      put_be16(a.outs[i] + (uint64_t)o * a.out_stride + 2 * (T - 1), acc);
    }
    __syncthreads();
  }
}

__device__ __forceinline__ uint32_t wave_xor(uint32_t v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v ^= __shfl_xor(v, off);
  return v;
}

// Batched syndrome regenerate: one wave per object, its survivor set its own
// (k <= 64), so the last stripe is interpolated here.  Lane s holds survivor
// s (point a_s, cell c_s); with N(z) = prod_s (z + a_s) the decoded stripe is
//   U(z) = sum_s w_s N(z) / (z + a_s),  w_s = c_s / prod_{j != s} (a_s + a_j)
// (Lagrange; the unique polynomial through the survivors, as V_S^{-1} c).
// The quotients q_s(z) = N(z) / (z + a_s) come out top coefficient first
// (q_{s,m-1} = N_m + a_s q_{s,m}), so U_m = sum_s w_s q_{s,m} arrives in the
// order a Horner evaluation of the targets consumes it.
// (rt: an RT object -- survivor points rt.spoint in slot order, targets
// rt.epoint[0..ne); otherwise the plan's points and erased points)
__global__ void k_regen_tail_batch(uint32_t k, uint32_t m, const SynBatchObj *objs, const SynBatchPlan *plans,
                                   uint32_t count, bool rt) {
  const int lane = threadIdx.x & 63;
  const uint32_t waves = blockDim.x / 64;
  for (uint32_t o = blockIdx.x * waves + (threadIdx.x >> 6); o < count; o += gridDim.x * waves) {
    const SynBatchObj &d = objs[o];
    const uint8_t *const points = rt ? d.rt.spoint : plans[d.plan].point;
    const uint8_t *const tpoints = rt ? d.rt.epoint : plans[d.plan].erased;
    const uint32_t nt = rt ? d.rt.ne : m;
    const uint64_t L = d.chunk_len, T = (L - 2) / 2;
    const uint32_t p = be16_at(d.chunks[d.first] + L - 2);
    if (p > 2 * k) continue;
    const uint32_t trailer = p == 2 * k ? 0u : p;
    uint8_t *const rg = lane < (int)nt ? d.regen[lane] : nullptr;
    const uint32_t t = lane < (int)nt ? tpoints[lane] : 0u;
    if (rg) put_be16(rg + 2 * T, trailer);
    if (p == 0 || p == 2 * k || T == 0) continue;
    const bool live = lane < (int)k;
    const uint32_t as = live ? points[lane] : 0u;
    const uint32_t cs = live ? be16_at(d.chunks[lane] + 2 * (T - 1)) : 0u;
    uint32_t Nm = lane == 0 ? 1u : 0u;  // lane m: coefficient m of N (N_k = 1 implicit)
    uint32_t D = 1;
    for (uint32_t j = 0; j < k; ++j) {
      const uint32_t aj = __shfl(as, (int)j);
      const uint32_t up = __shfl_up(Nm, 1);
      Nm = (lane == 0 ? 0u : up) ^ gf16_mul(aj, Nm);
      D = gf16_mul(D, j == (uint32_t)lane ? 1u : (as ^ aj));
    }
    const uint32_t w = live ? gf16_mul(cs, gf16_inv(D)) : 0u;
    const uint32_t J = (p + 1) / 2;
    uint32_t q = 1, acc = 0;
    for (uint32_t mm = k; mm-- > 0;) {
      if (mm < J) {  // (cells mm >= J are trimmed to zero: acc stays 0 above them)
        const uint32_t u = trim_cell(wave_xor(gf16_mul(w, q)), mm, p);
        acc = gf16_mul(acc, t) ^ u;
      }
      if (mm > 0) q = __shfl(Nm, (int)mm) ^ gf16_mul(as, q);
    }
    if (rg) put_be16(rg + 2 * (T - 1), acc);
  }
}

// GF(2^16) log / exp tables (generator x = 2 of kPoly16, as the reference's
// gf_math<uint16_t>, gf.h:193-253): the RT coefficient kernel's products
// become sums of logs.  g_exp16 is 3 x 65535 long so a sum of three reduced
// logs needs no reduction.  Built once per device by k_gf16_tables.
__device__ uint16_t g_log16[65536];
__device__ uint16_t g_exp16[3 * 65535];

__global__ void k_gf16_tables() {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 65535) return;
  uint32_t r = 1, b = 2, e = i;  // 2^i
  while (e) {
    if (e & 1u) r = gf16_mul(r, b);
    b = gf16_mul(b, b);
    e >>= 1;
  }
  g_exp16[i] = g_exp16[i + 65535] = g_exp16[i + 2 * 65535] = (uint16_t)r;
  g_log16[r] = (uint16_t)i;
  if (i == 0) g_log16[0] = 0;  // (never read: zero factors are handled apart)
}

__device__ __forceinline__ uint32_t glog(uint32_t x) { return g_log16[x]; }
__device__ __forceinline__ uint32_t mod65535(uint32_t x) {
  x = (x & 0xFFFFu) + (x >> 16);
  x = (x & 0xFFFFu) + (x >> 16);
  return x >= 65535u ? x - 65535u : x;
}
__device__ __forceinline__ uint32_t spread16(uint32_t c) { return (c & 0xFFu) | ((c & 0xFF00u) << 8); }

// RT coefficient rows (SynBatchRt): one wave per object, lane j = slot j
// holding point a_j.  Row m, column j is the Lagrange basis polynomial of
// slot j evaluated at t = epoint[m]:
//   l_j(t) = prod_i (t + a_i) / ((t + a_j) D_j),  D_j = prod_{i != j} (a_j + a_i),
// in logs: the row's sum over the lanes (butterfly), minus the lane's two
// logs, one exp lookup.  t equal to a slot's point gives the unit row.  k <=
// 32: the wave's two halves take two rows at a time (32-lane segments).
// (Round 3 multiplied with the carry-less gf16_mul -- ~70 VALU each, prefix
// and suffix scans per row: 190-200 us per live p = 0.25 call.)
// RT2 objects (SynBatchRt::mode 1, ec_internal.hpp): c[m][jj] = F_m G_jj /
// (e_m + b_jj), F_m = Z(e_m) prod_i (e_m + b_i), G_jj = 1 / (Z(b_jj)
// prod_{i != jj} (b_jj + b_i)), Z(x) = prod over the survivors below k.
// Stored spread (SynBatchRt::coef).
__global__ void k_rt_coefs(uint32_t k, const SynBatchObj *objs, uint32_t count) {
  const int lane = threadIdx.x & 63;
  const int seg = k <= 32 ? 32 : 64;  // lanes per row
  const int j = lane & (seg - 1);     // slot of this lane
  const int half = lane / seg;        // row of this lane within a pass
  const uint32_t per_pass = 64 / seg;
  const uint32_t waves = blockDim.x / 64;
  for (uint32_t o = blockIdx.x * waves + (threadIdx.x >> 6); o < count; o += gridDim.x * waves) {
    const SynBatchRt &r = objs[o].rt;
    const uint32_t ne = r.ne;
    if (ne == 0) continue;
    uint32_t *const out = const_cast<uint32_t *>(r.coef);
    if (r.mode == 1) {
      const uint64_t erased = r.borrowed;  // (the erased points below k: the borrowed slots)
      // lanes 0..ne-1: x = e_m; lanes 16..16+ne-1: x = b_jj; log Z(x) over the survivors below k
      const int q = lane & 15;
      const bool isb = lane >= 16 && lane < 32;
      const uint32_t em = q < (int)ne ? r.epoint[q] : 0u;
      const uint32_t x = q < (int)ne ? (isb ? r.spoint[em] : em) : 0u;
      uint32_t lz = 0;
      for (uint32_t a = 0; a < k; ++a)
        if (!((erased >> a) & 1u)) lz += glog(x ^ a);
      // log F_m (lanes 0..15), log of 1 / G_jj (lanes 16..31)
      for (uint32_t i = 0; i < ne; ++i) {
        const uint32_t bi = __shfl(x, 16 + (int)i);
        if (!(isb && (uint32_t)q == i)) lz += glog(x ^ bi);
      }
      const uint32_t lfg = mod65535(lz);
      for (uint32_t pr = (uint32_t)lane; pr < 64u * ((ne * ne + 63) / 64); pr += 64) {
        const uint32_t m = pr / ne, jj = pr % ne;
        const bool ok = pr < ne * ne;
        const uint32_t lF = __shfl(lfg, ok ? (int)m : 0), lG = __shfl(lfg, ok ? 16 + (int)jj : 16);
        const uint32_t e = __shfl(x, ok ? (int)m : 0), b = __shfl(x, ok ? 16 + (int)jj : 16);
        if (ok) {  // F G / (e + b): lF - lG - log(e + b), shifted positive
          const uint32_t c = g_exp16[lF + (65535u - lG) + (65535u - glog(e ^ b))];
          out[(uint64_t)m * k + jj] = spread16(c);
        }
      }
      continue;
    }
    const bool live = j < (int)k;
    const uint32_t a = live ? r.spoint[j] : 0u;
    // log D_j
    uint32_t ld = 0;
    for (uint32_t i = 0; i < k; ++i) {
      const uint32_t ai = __shfl(a, (int)i);
      if (i != (uint32_t)j) ld += glog(a ^ ai);
    }
    const uint32_t nld = 65535u - mod65535(ld);  // log of 1 / D_j
    for (uint32_t m0 = 0; m0 < ne; m0 += per_pass) {
      const uint32_t m = m0 + (uint32_t)half;
      const uint32_t f = live && m < ne ? (r.epoint[m] ^ a) : 1u;  // (dead lanes: log 1 = 0)
      const bool zero = f == 0u;                                   // t is this slot's point
      const uint64_t zb = __ballot(zero);
      const bool row_zero = ((zb >> (half * seg)) & (seg == 64 ? ~0ull : 0xFFFFFFFFull)) != 0;
      uint32_t lf = zero ? 0u : glog(f);
      uint32_t sum = lf;
      for (int off = 1; off < seg; off <<= 1) sum += __shfl_xor(sum, off);
      if (live && m < ne) {
        uint32_t c;
        if (row_zero)
          c = zero ? 1u : 0u;
        else  // prod_i f_i / f_j / D_j
          c = g_exp16[mod65535(sum) + (65535u - lf) + nld];
        out[(uint64_t)m * k + j] = spread16(c);
      }
    }
  }
}

static std::mutex g_tables_mu;
static uint64_t g_tables_ready = 0;  // bit d: device d has the log / exp tables (g_tables_mu)

// Built once per device on a private stream, which this thread then waits
// for: the caller's stream is neither synchronised nor used, so a
// stream-ordered *_device call that gets here first still only enqueues on
// it; every later launch on any stream sees the finished tables.
// While a stream of the process is being captured in global mode, creating
// and synchronising a stream are prohibited calls that would invalidate that
// capture; this thread switches to relaxed capture mode for the build and
// back, so the build cannot.  (Capturing the batch entry points
// themselves in a graph is not supported: their descriptors live in pinned
// parameter slots that later calls reuse, api_param_ring.cpp.)
static hipError_t ensure_gf16_tables() {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  std::lock_guard<std::mutex> g(g_tables_mu);
  if (dev < 64 && ((g_tables_ready >> dev) & 1u)) return hipSuccess;
  hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;
  if ((e = hipThreadExchangeStreamCaptureMode(&mode)) != hipSuccess) return e;
  hipStream_t own = nullptr;
  e = hipStreamCreateWithFlags(&own, hipStreamNonBlocking);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(k_gf16_tables, dim3((65535 + 255) / 256), dim3(256), 0, own);
    e = hipGetLastError();
    if (e == hipSuccess) e = hipStreamSynchronize(own);
    (void)hipStreamDestroy(own);
  }
  (void)hipThreadExchangeStreamCaptureMode(&mode);  // (the caller's mode again)
  if (e != hipSuccess) return e;
  if (dev < 64) g_tables_ready |= 1ull << dev;
  return hipSuccess;
}

// ============================================================ host push copy
// Device -> host copy by a kernel storing into mapped pinned host memory.
// On the MI355X box the two SDMA directions together move only one
// direction's bytes (57 GB/s total: H2D + D2H on two streams at 28.5 each),
// but a kernel's stores over PCIe run beside an SDMA H2D: 42.7 + 42.7 GB/s
// (tools/ubench/pcie_duplex.hip).  The host batches therefore take their
// results out this way while the next group's input comes in by SDMA.
typedef uint32_t copy_u32x4 __attribute__((ext_vector_type(4)));
__global__ void k_push(uint8_t *dst, const uint8_t *src, uint64_t bytes) {
  const uint64_t n16 = bytes / 16;
  const uint64_t step = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t i0 = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  for (uint64_t i = i0; i < n16; i += step)
    __builtin_nontemporal_store(__builtin_nontemporal_load(reinterpret_cast<const copy_u32x4 *>(src) + i),
                                reinterpret_cast<copy_u32x4 *>(dst) + i);
  for (uint64_t b = 16 * n16 + i0; b < bytes; b += step) dst[b] = src[b];
}

// ============================================================== synthetic data

__global__ void k_fill_splitmix(uint8_t *dst, uint64_t size, uint64_t seed) {
  const uint64_t words = (size + 7) / 8;
  for (uint64_t w = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; w < words;
       w += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t z = seed + (w + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    if (8 * w + 8 <= size) {
      *reinterpret_cast<uint64_t *>(dst + 8 * w) = z;
    } else {
      for (uint64_t b = 0; 8 * w + b < size; ++b) dst[8 * w + b] = (uint8_t)(z >> (8 * b));
    }
  }
}

static int grid_for(uint64_t work, int block) {
  uint64_t g = (work + block - 1) / block;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  return (int)g;
}

hipError_t launch_encode_generic(const GenericEncodeArgs &a, hipStream_t s) {
  const uint64_t work = (a.t_count + (a.write_trailer ? 1 : 0)) * a.nrep * (uint64_t)a.count;
  if (work == 0) return hipSuccess;
  const int grid = grid_for(work, 256);
  if (a.cell_bytes == 2)
    hipLaunchKernelGGL(k_encode_generic<2>, dim3(grid), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL(k_encode_generic<1>, dim3(grid), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_restore_generic(const GenericRestoreArgs &a, hipStream_t s) {
  const uint64_t work = a.t_count * a.k * (uint64_t)a.count;
  if (work == 0) return hipSuccess;
  const int grid = grid_for(work, 256);
  if (a.cell_bytes == 2)
    hipLaunchKernelGGL(k_restore_generic<2>, dim3(grid), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL(k_restore_generic<1>, dim3(grid), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_regen_generic(const RegenArgs &a, hipStream_t s) {
  const uint64_t work = (a.t_count + 1) * a.nt * (uint64_t)a.count;
  if (work == 0) return hipSuccess;
  const int grid = grid_for(work, 256);
  if (a.cell_bytes == 2)
    hipLaunchKernelGGL(k_regen_generic<2>, dim3(grid), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL(k_regen_generic<1>, dim3(grid), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_regen_tail(const RegenTailArgs &a, hipStream_t s) {
  if (a.count == 0 || a.nt == 0 || a.chunk_size < 2) return hipSuccess;
  // J = ceil(p / 2) <= 32768 cells (p is 16 bits)
  const int lds = 2 * (int)(a.k < 32768u ? a.k : 32768u);
  hipError_t e = ensure_lds_attr(&k_regen_tail, lds);
  if (e != hipSuccess) return e;
  const uint32_t grid = a.count < 4096u ? a.count : 4096u;
  hipLaunchKernelGGL(k_regen_tail, dim3(grid), dim3(256), lds, s, a);
  return hipGetLastError();
}

hipError_t launch_regen_tail_batch(uint32_t k, uint32_t m, const SynBatchObj *objs, const SynBatchPlan *plans,
                                   uint32_t count, hipStream_t s) {
  if (count == 0) return hipSuccess;
  if (k > 64 || m > (uint32_t)kMaxFastK / 4) return hipErrorInvalidValue;
  const uint32_t waves = 4, grid = (count + waves - 1) / waves < 8192u ? (count + waves - 1) / waves : 8192u;
  hipLaunchKernelGGL(k_regen_tail_batch, dim3(grid), dim3(64 * waves), 0, s, k, m, objs, plans, count, false);
  return hipGetLastError();
}

hipError_t launch_regen_tail_rt(uint32_t k, const SynBatchObj *objs, uint32_t count, hipStream_t s) {
  if (count == 0) return hipSuccess;
  if (k > 64) return hipErrorInvalidValue;
  const uint32_t waves = 4, grid = (count + waves - 1) / waves < 8192u ? (count + waves - 1) / waves : 8192u;
  hipLaunchKernelGGL(k_regen_tail_batch, dim3(grid), dim3(64 * waves), 0, s, k, 0u, objs, nullptr, count, true);
  return hipGetLastError();
}

hipError_t launch_rt_coefs(uint32_t k, const SynBatchObj *objs, uint32_t count, hipStream_t s) {
  if (count == 0) return hipSuccess;
  if (k > 64) return hipErrorInvalidValue;
  const hipError_t te = ensure_gf16_tables();
  if (te != hipSuccess) return te;
  const uint32_t waves = 4, grid = (count + waves - 1) / waves < 8192u ? (count + waves - 1) / waves : 8192u;
  hipLaunchKernelGGL(k_rt_coefs, dim3(grid), dim3(64 * waves), 0, s, k, objs, count);
  return hipGetLastError();
}

hipError_t launch_push(uint8_t *dst_host_dev, const uint8_t *src, uint64_t bytes, hipStream_t s) {
  if (bytes == 0) return hipSuccess;
  if (((uintptr_t)dst_host_dev | (uintptr_t)src) & 15u) return hipErrorInvalidValue;
  uint64_t g = (bytes / 16 + 255) / 256;
  const uint32_t grid = (uint32_t)(g < 1 ? 1 : (g > 512 ? 512 : g));
  hipLaunchKernelGGL(k_push, dim3(grid), dim3(256), 0, s, dst_host_dev, src, bytes);
  return hipGetLastError();
}

hipError_t launch_fill_splitmix(uint8_t *dst, uint64_t size, uint64_t seed, hipStream_t s) {
  if (size == 0) return hipSuccess;
  const int grid = grid_for((size + 7) / 8, 256);
  hipLaunchKernelGGL(k_fill_splitmix, dim3(grid), dim3(256), 0, s, dst, size, seed);
  return hipGetLastError();
}

}  // namespace vds_ec
