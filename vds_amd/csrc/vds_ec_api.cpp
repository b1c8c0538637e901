// vds_ec_api.cpp -- the C ABI declared in include/vds_ec.h.
// (api_internal.hpp lists the host runtime's other translation units.)
//
// Host-side runtime of the codec: argument validation mirroring the
// reference's contracts (chunk.h, chunk_storage.cpp), the Vandermonde
// inverse (the chunk_restore constructor), dispatch between the bit-sliced
// and generic kernels, host-memory staging and the multi-GPU batch driver.
// All data-path arithmetic runs in the HIP kernels (ec_*.hip); the
// only host arithmetic is on k x k matrices and tables.
#include "api_internal.hpp"

using namespace vds_ec;
using namespace vds_ec::api;

namespace vds_ec {
namespace api {

constexpr int kVersion = 100;  // 0.1.0


int hip_status(hipError_t e) {
  if (e == hipSuccess) return VDS_EC_OK;
  static const bool debug = std::getenv("VDS_EC_DEBUG") != nullptr;
  if (debug) std::fprintf(stderr, "vds_ec: HIP error %d (%s)\n", (int)e, hipGetErrorString(e));
  if (e == hipErrorOutOfMemory) return VDS_EC_ENOMEM;
  if (e == hipErrorNoDevice || e == hipErrorInvalidDevice || e == hipErrorInsufficientDriver)
    return VDS_EC_ENODEV;
  return VDS_EC_EHIP;
}

int device_ready() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return VDS_EC_ENODEV;
  return VDS_EC_OK;
}

const Gf16Tables &gf16_tables() {
  static const Gf16Tables *t = new Gf16Tables();  // never freed
  return *t;
}

// ---------------------------------------------------------------- inverse
// M = V^{-1} for V[i][c] = a_i^c, by Lagrange: column i of M holds the
// coefficients of prod_{j!=i} (z - a_j) / (a_i - a_j).  V^{-1} is unique, so
// this equals the reference's cross-multiplied Gauss-Jordan
// (chunk.h:290-375) bit for bit whenever the nodes are distinct.
template <typename Mul, typename Inv>
int lagrange_inverse(uint32_t k, const uint32_t *a, uint16_t *out, Mul mul, Inv inv) {
  std::vector<uint32_t> N(k + 1, 0), q(k);
  N[0] = 1;
  for (uint32_t j = 0; j < k; ++j) {  // N(z) = prod (z + a_j)
    for (uint32_t d = j + 1; d > 0; --d) N[d] = N[d - 1] ^ mul(a[j], N[d]);
    N[0] = mul(a[j], N[0]);
  }
  for (uint32_t i = 0; i < k; ++i) {
    q[k - 1] = N[k];  // synthetic division by (z + a_i)
    for (uint32_t m = k - 1; m > 0; --m) q[m - 1] = N[m] ^ mul(a[i], q[m]);
    uint32_t d = 0;  // Q_i(a_i) = prod_{j != i} (a_i + a_j)
    for (uint32_t m = k; m > 0; --m) d = mul(d, a[i]) ^ q[m - 1];
    if (d == 0) return VDS_EC_ESINGULAR;
    const uint32_t di = inv(d);
    for (uint32_t m = 0; m < k; ++m) out[(size_t)m * k + i] = (uint16_t)mul(q[m], di);
  }
  return VDS_EC_OK;
}

int inverse16(uint32_t k, const uint16_t *nodes, uint16_t *out) {
  std::vector<uint32_t> a(nodes, nodes + k);
  return lagrange_inverse(
      k, a.data(), out, [](uint32_t x, uint32_t y) { return gf16_mul_fast(x, y); },
      [](uint32_t x) { return gf16_inv_fast(x); });
}

int inverse8(uint32_t k, const uint8_t *nodes, uint16_t *out) {
  std::vector<uint32_t> a(nodes, nodes + k);
  return lagrange_inverse(
      k, a.data(), out, [](uint32_t x, uint32_t y) { return (uint32_t)gf8_mul(x, y); },
      [](uint32_t x) { return (uint32_t)gf8_inv(x); });
}

// ------------------------------------------------- syndrome restore plan
// The erasure-pattern-independent kernel k_restore_syn<K,N> applies when the
// survivors are K distinct points of 0..N-1 for a compiled (K, N).  The host
// part is the M x M solve matrix R = W_E^{-1}, W_E[j][i] = v_{e_i} e_i^j
// (M = N - K, E = the erased points): with S_j = sum_{a survives} W[j][a] c_a,
// every codeword has sum_a W[j][a] c_a = 0, so W_E c_E = S.  Any K survivor
// values lie on exactly one polynomial of degree < K, so the recovered
// replicas and the interpolated object equal V_S^{-1} applied to the
// survivors (the reference's chunk.h:290-375 route) for every input.
// (a -DVDS_RESTORE_PATH_BS=1 build sends every restore to k_restore_bs: A/B)
#ifndef VDS_RESTORE_PATH_BS
#define VDS_RESTORE_PATH_BS 0
#endif
bool restore_path_override_bs() { return VDS_RESTORE_PATH_BS != 0; }

// The syndrome kernel's point assignment for a survivor list: eligible when
// the k ids are distinct points of 0..k+k/4-1 for a compiled (k, n); fills
// sa.point / sa.erased and the erased set as a bitmask (the plan's key).
bool syn_points(uint32_t k, const uint16_t *nodes, SynRestoreArgs &sa, uint32_t *n_out, uint64_t *key) {
  if (!nodes || restore_path_override_bs()) return false;
  const uint32_t n = k + k / 4;
  if (k % 4 || !has_restore_syn(k, n)) return false;
  uint64_t seen = 0;
  for (uint32_t j = 0; j < k; ++j) {
    if (nodes[j] >= n || ((seen >> nodes[j]) & 1u)) return false;
    seen |= 1ull << nodes[j];
    sa.point[j] = (uint8_t)nodes[j];
  }
  uint32_t e = 0;
  for (uint32_t a = 0; a < n; ++a)
    if (!((seen >> a) & 1u)) sa.erased[e++] = (uint8_t)a;
  *n_out = n;
  *key = ~seen & ((1ull << n) - 1);
  return true;
}

// R = W_E^{-1} as the kernel's bit selections (sa.erased set by syn_points).
bool syn_solve(uint32_t k, uint32_t n, SynRestoreArgs &sa) {
  const uint16_t *W = restore_syn_weights(k, n);
  const uint32_t m = n - k;
  // Gauss-Jordan on [W_E | I] (m <= 8)
  uint32_t A[8 * 16] = {};
  for (uint32_t j = 0; j < m; ++j) {
    for (uint32_t i = 0; i < m; ++i) A[j * 2 * m + i] = W[j * n + sa.erased[i]];
    A[j * 2 * m + m + j] = 1;
  }
  for (uint32_t c = 0; c < m; ++c) {
    uint32_t piv = c;
    while (piv < m && A[piv * 2 * m + c] == 0) ++piv;
    if (piv == m) return false;  // cannot happen for distinct points
    if (piv != c)
      for (uint32_t x = 0; x < 2 * m; ++x) std::swap(A[c * 2 * m + x], A[piv * 2 * m + x]);
    const uint32_t iv = gf16_inv_fast(A[c * 2 * m + c]);
    for (uint32_t x = 0; x < 2 * m; ++x) A[c * 2 * m + x] = gf16_mul_fast(A[c * 2 * m + x], iv);
    for (uint32_t r = 0; r < m; ++r) {
      const uint32_t f = A[r * 2 * m + c];
      if (r == c || f == 0) continue;
      for (uint32_t x = 0; x < 2 * m; ++x) A[r * 2 * m + x] ^= gf16_mul_fast(f, A[c * 2 * m + x]);
    }
  }
  // R[i][j]: row i = the erased point the kernel's wave i recovers
  std::memset(sa.solve_sel, 0, sizeof sa.solve_sel);
  for (uint32_t i = 0; i < m; ++i)
    for (uint32_t j = 0; j < m; ++j) {
      const uint32_t r = A[i * 2 * m + m + j];
      for (uint32_t b = 0; b < 16; ++b)
        if ((r >> b) & 1u) sa.solve_sel[i][b >> 2] |= 1u << (8 * (b & 3) + j);
    }
  return true;
}

bool plan_restore_syn(uint32_t k, const uint16_t *nodes, SynRestoreArgs &sa, uint32_t *n_out) {
  uint64_t key = 0;
  return syn_points(k, nodes, sa, n_out, &key) && syn_solve(k, *n_out, sa);
}

// ---------------------------------------------------------- encode core
// The zero trailers of a launch that covers every stripe are written by the
// bit-sliced kernel's stores (fa.trailer0); other launches get a generic one.

int encode_device(unsigned cb, uint32_t k, const uint16_t *replicas, uint32_t n, const uint8_t *in,
                  uint64_t size, uint64_t in_stride, uint32_t count, uint8_t *const *outs,
                  uint64_t out_stride, unsigned flags, hipStream_t s) {
  if (k == 0 || (n > 0 && (!replicas || !outs)) || (count > 0 && size > 0 && !in)) return VDS_EC_EINVAL;
  if (n == 0 || count == 0) return VDS_EC_OK;
  for (uint32_t i = 0; i < n; ++i)
    if (!outs[i]) return VDS_EC_EINVAL;
  int rc = device_ready();
  if (rc) return rc;
  const bool cells = (flags & VDS_EC_F_CELLS) != 0;
  const bool trailer = !(flags & (VDS_EC_F_NO_TRAILER | VDS_EC_F_CELLS));
  const uint64_t stripe_bytes = (uint64_t)k * cb;
  const uint64_t T = (size + stripe_bytes - 1) / stripe_bytes;

  // Bit-sliced path: 16-bit byte-API cells, replicas exactly 0..n-1.  It
  // covers the first gpo 128-stripe groups of every object, taken as one
  // stream of 2048-stripe tiles: with F = full stripes per object, gpo = F/128
  // when 128 | F (tiles may straddle objects, k >= 8), else gpo = 16 floor(F/2048)
  // (whole tiles per object).  The rest is generic.
  const uint64_t F = size / stripe_bytes;  // stripes with no zero padding
  uint64_t gpo = 0, fast_groups = 0;
  bool contiguous = true;
  for (uint32_t i = 0; i < n; ++i) contiguous &= (replicas[i] == i);
  if (cb == 2 && !cells && contiguous && has_encode_fast(k, n) && ((uintptr_t)in | in_stride) % 4 == 0) {
    if (F % 128 == 0 && (k >= 8 || F % kTileStripes == 0))
      gpo = F / 128;
    else
      gpo = 16 * (F / kTileStripes);
    const uint64_t total = gpo * count / 16;
    if (gpo > 0 && gpo <= 0xFFFFFFFFull && total > 0 && total <= 0xFFFFFFFFull) {
      FastEncodeArgs fa{};
      fa.in = in;
      fa.in_stride = in_stride;
      fa.out_stride = out_stride;
      fa.groups_per_obj = (uint32_t)gpo;
      fa.total_tiles = (uint32_t)total;
      // every stripe of every object in the launch, size a multiple of 2k:
      // the zero trailers ride the bit-sliced stores (k >= 8, map 3)
      fa.trailer0 = (trailer && k >= 8 && 128 * gpo == T && size % stripe_bytes == 0 &&
                     total * 16 == gpo * count)
                        ? 1u
                        : 0u;
      for (uint32_t i = 0; i < n; ++i) fa.outs[i] = outs[i];
      hipError_t e = launch_encode_fast(k, n, fa, s);
      if (e != hipSuccess) return hip_status(e);
      fast_groups = total * 16;
    }
  }
  // Generic path for the rest (+ trailers), in launches of <= 64 replicas:
  // objects [0, o_full) need only their partial stripe and trailer, object
  // o_full its uncovered tail, objects after it everything.
  const uint64_t o_full = fast_groups ? fast_groups / gpo : 0;
  struct Part {
    uint64_t o0, cnt, t_begin;
  };
  const bool trailers_done = fast_groups && trailer && k >= 8 && 128 * gpo == T &&
                             size % stripe_bytes == 0 && fast_groups == gpo * count;  // (fa.trailer0 above)
  Part parts[3] = {{0, trailers_done ? 0 : o_full, 128 * gpo},
                   {o_full, o_full < count ? 1u : 0u, fast_groups ? 128 * (fast_groups - o_full * gpo) : 0},
                   {o_full + 1, o_full + 1 < count ? count - o_full - 1 : 0, 0}};
  if (!fast_groups) {
    parts[0] = {0, count, 0};
    parts[1].cnt = parts[2].cnt = 0;
  }
  for (const Part &pt : parts) {
    if (pt.cnt == 0) continue;
    for (uint32_t base = 0; base < n; base += kMaxLaunchReplicas) {
      GenericEncodeArgs ga{};
      ga.in = in + pt.o0 * in_stride;
      ga.size = size;
      ga.in_stride = in_stride;
      ga.count = (uint32_t)pt.cnt;
      ga.k = k;
      ga.cell_bytes = cb;
      ga.flags = flags;
      ga.nrep = (n - base) < (uint32_t)kMaxLaunchReplicas ? (n - base) : (uint32_t)kMaxLaunchReplicas;
      ga.t_begin = pt.t_begin;
      ga.t_count = T - pt.t_begin;
      ga.stripes = T;
      ga.write_trailer = trailer ? 1 : 0;
      ga.out_stride = out_stride;
      for (uint32_t i = 0; i < ga.nrep; ++i) {
        ga.nodes[i] = replicas[base + i];
        ga.outs[i] = outs[base + i] + pt.o0 * out_stride;
      }
      hipError_t e = launch_encode_generic(ga, s);
      if (e != hipSuccess) return hip_status(e);
    }
  }
  return VDS_EC_OK;
}

// ------------------------------------------------------- restore planning
// Which kernels restore_device runs for these parameters (shared with the
// vds_ec_restore16_path query, so the two cannot disagree):
//   3 = k_restore_syn over the whole 2048-stripe tiles of every object,
//   2 = k_restore_bs over 512-stripe groups (whole tiles per object, or a
//       stream of tiles across objects when the groups of an object are not
//       a multiple of 4),
//   1 = the generic kernel only.
// F counts the stripes whose k cells all land in the output (out_len / 2k:
// one fewer than the replica's cells when the trailer's padding is non-zero).
struct RestorePlan {
  int path = 1;
  uint64_t tiles = 0;  // path 3: tiles per object
  uint64_t gpo = 0;    // path 2: 512-stripe groups per object
  SynRestoreArgs sa{};
  uint32_t syn_n = 0;
};

RestorePlan plan_restore(unsigned cb, uint32_t k, const uint16_t *nodes, uint64_t out_len, uint32_t count,
                         unsigned flags) {
  RestorePlan p;
  const bool cells = (flags & VDS_EC_F_CELLS) != 0;
  if (cb != 2 || cells || k == 0 || count == 0) return p;
  const uint64_t F = out_len / (2ull * k);
  // (objects under one tile go to the bit-sliced kernel's stream mode,
  // whatever the survivor set)
  if (F >= kTileStripes && plan_restore_syn(k, nodes, p.sa, &p.syn_n)) {
    const uint64_t tiles = F / kTileStripes;
    if (tiles * count <= 0xFFFFFFFFull) {
      p.path = 3;
      p.tiles = tiles;
      return p;
    }
  }
  if (has_restore_fast(k)) {
    // 512-stripe groups; tiles of 4 groups may straddle objects when 512 | F
    const uint64_t gpo = F % 512 == 0 ? F / 512 : 4 * (F / kTileStripes);
    const uint64_t total = gpo * count / 4;
    if (gpo > 0 && gpo <= 0xFFFFFFFFull && total > 0 && total <= 0xFFFFFFFFull) {
      p.path = 2;
      p.gpo = gpo;
    }
  }
  return p;
}

int restore_device(unsigned cb, uint32_t k, const uint16_t *nodes, const uint16_t *matrix, const uint8_t *const *chunks,
                   uint64_t chunk_size, uint64_t chunk_stride, uint64_t out_len, uint32_t count,
                   uint8_t *out, uint64_t out_stride, unsigned flags, hipStream_t s,
                   const ChunkLayout &layout) {
  if (count == 0 || out_len == 0) return VDS_EC_OK;
  int rc = device_ready();
  if (rc) return rc;
  // Every cell of a chunk, the trailer cell included: with a corrupt trailer
  // the reference decodes that row too (chunk.h:421-441).
  const uint64_t cells_per_chunk = chunk_size / cb;
  const uint64_t stripe_bytes = (uint64_t)k * cb;
  uint64_t need = (out_len + stripe_bytes - 1) / stripe_bytes;  // stripes that produce output
  if (need > cells_per_chunk) need = cells_per_chunk;

  // The fast kernels cover the first `per_obj` stripes of every object (or,
  // in stream mode, the first `fast_total` stripes of the batch taken as one
  // stream of objects of F full output stripes each); the generic kernel the rest.
  const uint64_t F = out_len / stripe_bytes;  // stripes whose k cells all land in the output
  uint64_t per_obj = 0, fast_total = 0;       // fast stripes: per object (whole tiles) / stream
  RestorePlan plan = plan_restore(cb, k, nodes, out_len, count, flags);
  if (plan.path == 3) {
    SynRestoreArgs &sa = plan.sa;
    for (uint32_t j = 0; j < k; ++j) sa.chunks[j] = chunks[j];
    sa.chunk_stride = chunk_stride;
    sa.out = out;
    sa.out_stride = out_stride;
    sa.tiles_per_obj = (uint32_t)plan.tiles;
    sa.total_tiles = (uint32_t)(plan.tiles * count);
    // the survivor set's own kernel once it is compiled (vds_ec_jit.cpp)
    const hipFunction_t jf = jit_restore_function(k, plan.syn_n, sa);
    hipError_t e = jf ? launch_restore_syn_jit(jf, k, plan.syn_n, sa, s) : launch_restore_syn(k, plan.syn_n, sa, s);
    if (e != hipSuccess) return hip_status(e);
    per_obj = plan.tiles * kTileStripes;
  } else if (plan.path == 2) {
    const uint64_t gpo = plan.gpo, total = gpo * count / 4;
    FastRestoreArgs fa{};
    for (uint32_t j = 0; j < k; ++j) fa.chunks[j] = chunks[j];
    fa.chunk_stride = chunk_stride;
    fa.out = out;
    fa.out_stride = out_stride;
    fa.groups_per_obj = (uint32_t)gpo;
    fa.total_tiles = (uint32_t)total;
    for (uint32_t i = 0; i < k * k; ++i) fa.matrix2[i >> 1] |= uint32_t(matrix[i]) << (16 * (i & 1));
    hipError_t e = launch_restore_fast(k, fa, s);
    if (e != hipSuccess) return hip_status(e);
    if (gpo % 4 == 0)
      per_obj = 512 * gpo;
    else
      fast_total = 512 * 4 * total;
  }
  // generic remainder: [0, o_full) from per_obj (or F), object o_full from its
  // covered prefix, objects after it from 0
  struct Part {
    uint64_t o0, cnt, t_begin;
  };
  Part parts[3] = {{0, count, per_obj}, {0, 0, 0}, {0, 0, 0}};
  if (fast_total) {
    const uint64_t o_full = fast_total / F;
    parts[0] = {0, o_full, F};
    parts[1] = {o_full, o_full < count ? 1u : 0u, fast_total - o_full * F};
    parts[2] = {o_full + 1, o_full + 1 < count ? count - o_full - 1 : 0, 0};
  }
  bool any = false;
  for (const Part &pt : parts) any |= pt.cnt > 0 && need > pt.t_begin;
  if (any) {
    GenericRestoreArgs ga{};
    // Parameters that do not fit in the kernel arguments (k > 32 inverse,
    // k > 64 chunk table) ride the stream-ordered parameter ring.
    std::vector<uint8_t> blob;
    size_t off_table = SIZE_MAX, off_matrix = SIZE_MAX;
    const bool use_table = !layout.pitch && k > (uint32_t)kInlineChunks;
    if (use_table) off_table = blob_append(blob, chunks, k);
    if (k <= (uint32_t)kInlineMatrixK) {
      for (uint32_t i = 0; i < k * k; ++i) ga.matrix_inline[i >> 1] |= uint32_t(matrix[i]) << (16 * (i & 1));
    } else if (layout.matrix_dev) {
      ga.matrix_dev = layout.matrix_dev;
    } else {
      off_matrix = blob_append(blob, matrix, (size_t)k * k);
    }
    hipError_t e = hipSuccess;
    ParamSlot *slot = nullptr;
    if (!blob.empty()) {
      const uint8_t *d = nullptr;
      e = param_stage(blob, s, &d, &slot);
      if (e == hipSuccess && off_table != SIZE_MAX) ga.chunk_table = reinterpret_cast<const uint8_t *const *>(d + off_table);
      if (e == hipSuccess && off_matrix != SIZE_MAX) ga.matrix_dev = reinterpret_cast<const uint16_t *>(d + off_matrix);
    }
    const bool tmp_table = use_table;
    for (const Part &pt : parts) {
      if (e != hipSuccess || pt.cnt == 0 || need <= pt.t_begin) continue;
      if (tmp_table && pt.o0) {  // (k > 64: only reached without the fast path, i.e. o0 == 0)
        e = hipErrorInvalidValue;
        break;
      }
      if (layout.pitch) {
        ga.chunk_base = layout.base + pt.o0 * chunk_stride;
        ga.chunk_pitch = layout.pitch;
      } else if (!tmp_table) {
        for (uint32_t j = 0; j < k; ++j) ga.chunk_ptr[j] = chunks[j] + pt.o0 * chunk_stride;
      }
      ga.chunk_stride = chunk_stride;
      ga.count = (uint32_t)pt.cnt;
      ga.k = k;
      ga.cell_bytes = cb;
      ga.flags = flags;
      ga.t_begin = pt.t_begin;
      ga.t_count = need - pt.t_begin;
      ga.out = out + pt.o0 * out_stride;
      ga.out_stride = out_stride;
      ga.out_len = out_len;
      e = launch_restore_generic(ga, s);
    }
    if (slot) {
      const hipError_t re = param_release(slot, s);
      if (e == hipSuccess) e = re;
    }
    if (e != hipSuccess) return hip_status(e);
  }
  return VDS_EC_OK;
}

uint64_t restored_len(unsigned cb, uint32_t k, uint64_t chunk_size, uint16_t padding, unsigned flags,
                      bool *ok) {
  *ok = true;
  if (flags & VDS_EC_F_CELLS) return (chunk_size / cb) * k * cb;  // chunk.h:388-399, untrimmed
  if (chunk_size < 2) {
    *ok = false;
    return 0;
  }
  // chunk.h:415-419 (size_t arithmetic; wraps exactly like the reference)
  uint64_t e = (chunk_size - 2) * k;
  if (padding != 0) {
    e -= (uint64_t)k * cb;
    e += padding;
  }
  // The reference's loop produces at most (chunk_size/cb)*k*cb bytes before
  // reporting "Fatal error at chunk_restore::restore" (chunk.h:421-443).
  const uint64_t produced = (chunk_size / cb) * k * cb;
  if (e > produced) *ok = false;
  return e;
}

// The copies, split over up to 8 threads by bytes: one thread's memcpy into
// pinned memory runs far below host memory bandwidth (28 vs 113 GB/s with 8).
// Copies that continue each other on both sides (a caller's objects or
// replicas in one slab) are merged first: the live shape's 2 KiB replicas
// would otherwise cost a memcpy call each.
void parallel_copy(const std::vector<Copy> &parts_in) {
  std::vector<Copy> parts;
  parts.reserve(parts_in.size());
  for (const Copy &c : parts_in) {
    if (c.len == 0) continue;
    if (!parts.empty() && parts.back().dst + parts.back().len == c.dst && parts.back().src + parts.back().len == c.src)
      parts.back().len += c.len;
    else
      parts.push_back(c);
  }
  size_t total = 0;
  for (const Copy &c : parts) total += c.len;
  const size_t kMinPerThread = 8u << 20;
  size_t nt = std::min<size_t>(total / kMinPerThread, 8);
  if (nt <= 1) {
    for (const Copy &c : parts) std::memcpy(c.dst, c.src, c.len);
    return;
  }
  // thread t copies bytes [total t / nt, total (t+1) / nt) of the concatenation
  auto run = [&](size_t t) {
    const size_t lo = total * t / nt, hi = total * (t + 1) / nt;
    size_t at = 0;
    for (const Copy &c : parts) {
      const size_t b = std::max(lo, at), e = std::min(hi, at + c.len);
      if (b < e) std::memcpy(c.dst + (b - at), c.src + (b - at), e - b);
      at += c.len;
      if (at >= hi) break;
    }
  };
  std::vector<std::thread> th;
  for (size_t t = 1; t < nt; ++t) th.emplace_back(run, t);
  run(0);
  for (auto &t : th) t.join();
}

// --------------------------------------------------------- host staging
// Per (thread, device) staging context.  When a thread exits, its contexts go
// back to a process-wide pool, from which the next thread that needs one on
// that device takes it: short-lived caller threads reuse the pinned and
// device buffers instead of leaking a set each.  (Nothing is freed in the
// thread-exit hook: at process exit it would race the HIP runtime's own
// teardown.  Every host entry point waits for its stream before returning, so
// a pooled context has no work in flight.)
struct HostCtx {
  hipStream_t stream = nullptr;
  uint8_t *d_in = nullptr;
  size_t d_in_cap = 0;
  uint8_t *d_out = nullptr;
  size_t d_out_cap = 0;
  uint8_t *d_param = nullptr;  // large k x k inverses (k > kInlineMatrixK)
  size_t d_param_cap = 0;
  // Pinned staging: the caller's (pageable) input is gathered into h_in and
  // crosses PCIe as one DMA; results are pushed by a kernel into the mapped
  // h_out (device view h_out_dev) and scattered from there.  One transfer
  // each way instead of one per chunk / replica: the per-transfer cost of
  // pageable copies (tens of us) dominated the drop-in calls' small objects.
  uint8_t *h_in = nullptr;
  size_t h_in_cap = 0;
  uint8_t *h_out = nullptr, *h_out_dev = nullptr;
  size_t h_out_cap = 0;
  // Replica window of the last encode (see encode_host): h_out holds
  // replicas win_first .. win_first + win_n - 1 of the object whose bytes are
  // still in h_in[0, win_size).
  bool win_valid = false;
  unsigned win_cb = 0, win_flags = 0;
  uint32_t win_k = 0, win_n = 0;
  uint32_t win_first = 0, win_last_single = 0;
  uint64_t win_size = 0;
  int grow(uint8_t **p, size_t *cap, size_t want) {
    if (want <= *cap) return VDS_EC_OK;
    if (*p) {
      (void)hipStreamSynchronize(stream);
      (void)hipFree(*p);
    }
    *p = nullptr;
    *cap = 0;
    if (hipMalloc(p, want) != hipSuccess) return VDS_EC_ENOMEM;
    *cap = want;
    return VDS_EC_OK;
  }
  int grow_pinned(size_t in_b, size_t out_b) {
    in_b = std::max<size_t>(in_b, 64);
    out_b = std::max<size_t>(out_b, 64);
    if (in_b > h_in_cap || out_b > h_out_cap) (void)hipStreamSynchronize(stream);
    if (in_b > h_in_cap) {
      win_valid = false;
      if (h_in) (void)hipHostFree(h_in);
      h_in = nullptr;
      h_in_cap = 0;
      if (hipHostMalloc(&h_in, in_b, 0) != hipSuccess) return VDS_EC_ENOMEM;
      h_in_cap = in_b;
    }
    if (out_b > h_out_cap) {
      win_valid = false;
      if (h_out) (void)hipHostFree(h_out);
      h_out = h_out_dev = nullptr;
      h_out_cap = 0;
      if (hipHostMalloc(&h_out, out_b, hipHostMallocMapped) != hipSuccess ||
          hipHostGetDevicePointer(reinterpret_cast<void **>(&h_out_dev), h_out, 0) != hipSuccess)
        return VDS_EC_ENOMEM;
      h_out_cap = out_b;
    }
    return VDS_EC_OK;
  }
  int ensure(size_t in_bytes, size_t out_bytes) {
    if (!stream && hipStreamCreateWithFlags(&stream, hipStreamNonBlocking) != hipSuccess) return VDS_EC_ENODEV;
    int rc = grow(&d_in, &d_in_cap, in_bytes);
    if (!rc) rc = grow(&d_out, &d_out_cap, out_bytes);
    return rc ? rc : grow_pinned(in_bytes, out_bytes);
  }
  // d_in[0, size) <- data through h_in (invalidates the replica window)
  int stage_in(const uint8_t *data, uint64_t size) {
    win_valid = false;
    if (size == 0) return VDS_EC_OK;
    parallel_copy({{h_in, data, size}});
    return hip_status(hipMemcpyAsync(d_in, h_in, size, hipMemcpyHostToDevice, stream));
  }
  // h_out[0, bytes) <- d_out[0, bytes), then wait for the stream
  int push_out_and_wait(uint64_t bytes) {
    hipError_t e = launch_push(h_out_dev, d_out, bytes, stream);
    if (e != hipSuccess) return hip_status(e);
    return hip_status(hipStreamSynchronize(stream));
  }
};

std::atomic<uint64_t> g_host_ctx_created{0};
struct HostCtxPool {
  std::mutex mu;
  std::vector<std::vector<HostCtx *>> idle;  // per device
};
HostCtxPool &host_ctx_pool() {
  static HostCtxPool *p = new HostCtxPool();  // never freed: outlives every thread
  return *p;
}
struct HostCtxOwner {  // a thread's contexts; back to the pool at thread exit
  std::vector<HostCtx *> per_device;
  ~HostCtxOwner() {
    HostCtxPool &p = host_ctx_pool();
    std::lock_guard<std::mutex> g(p.mu);
    for (size_t d = 0; d < per_device.size(); ++d) {
      if (!per_device[d]) continue;
      per_device[d]->win_valid = false;  // (the replica window belongs to this thread's calls)
      if (p.idle.size() <= d) p.idle.resize(d + 1);
      p.idle[d].push_back(per_device[d]);
    }
  }
};

HostCtx *host_ctx() {
  thread_local HostCtxOwner own;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0) return nullptr;
  if ((size_t)dev >= own.per_device.size()) own.per_device.resize(dev + 1, nullptr);
  if (!own.per_device[dev]) {
    HostCtxPool &p = host_ctx_pool();
    std::lock_guard<std::mutex> g(p.mu);
    if ((size_t)dev < p.idle.size() && !p.idle[dev].empty()) {
      own.per_device[dev] = p.idle[dev].back();
      p.idle[dev].pop_back();
    } else {
      own.per_device[dev] = new HostCtx();
      g_host_ctx_created.fetch_add(1, std::memory_order_relaxed);
    }
  }
  return own.per_device[dev];
}

// Contexts created and pooled so far (vds_ec_host_ctx_stats).
size_t host_ctx_pooled() {
  HostCtxPool &p = host_ctx_pool();
  std::lock_guard<std::mutex> g(p.mu);
  size_t n = 0;
  for (const auto &v : p.idle) n += v.size();
  return n;
}

// Host-buffer encode.  The drop-in chunk_generator<T>::write encodes one
// replica per call, and the caller that matters (_client::save_temp,
// dht_network_client.cpp:74-79) calls it for replicas 0..n-1 of the same
// bytes in turn.  So a single-replica call whose input equals the previous
// call's (compared byte for byte with the copy kept in h_in) and whose id
// follows that call's id encodes a window of the next replicas at once
// (kWindowBytes of output at most, up to kWindowReplicas); later calls in
// the window are served from h_out without touching the device.  The bytes
// are the encode of the current input in every case -- the window is only
// used when the input is identical -- so callers see no difference but the
// time.
constexpr uint32_t kWindowReplicas = 64;
constexpr uint64_t kWindowBytes = 8ull << 20;

int encode_host(unsigned cb, uint32_t k, const uint16_t *replicas, uint32_t n, const uint8_t *data,
                uint64_t size, uint8_t *const *outs, unsigned flags) {
  if (k == 0 || (n > 0 && (!replicas || !outs)) || (size > 0 && !data)) return VDS_EC_EINVAL;
  int rc = device_ready();
  if (rc) return rc;
  if (n == 0) return VDS_EC_OK;
  for (uint32_t i = 0; i < n; ++i)
    if (!outs[i]) return VDS_EC_EINVAL;
  const uint64_t L = vds_ec_replica_size(cb, k, size, flags);
  HostCtx *cp = host_ctx();
  if (!cp) return VDS_EC_ENODEV;
  HostCtx &c = *cp;
  const uint32_t max_id = cb == 1 ? 255u : 65535u;
  std::vector<uint16_t> ids(replicas, replicas + n);
  bool same_input = false;
  if (n == 1 && c.win_valid && c.win_cb == cb && c.win_k == k && c.win_flags == flags && c.win_size == size &&
      (size == 0 || std::memcmp(c.h_in, data, size) == 0)) {
    same_input = true;
    const uint32_t r = replicas[0];
    if (r >= c.win_first && r < c.win_first + c.win_n) {
      if (L) std::memcpy(outs[0], c.h_out + (uint64_t)(r - c.win_first) * L, L);
      c.win_last_single = r;
      return VDS_EC_OK;
    }
    if (r == c.win_last_single + 1 && r <= max_id) {
      // the per-replica loop: take the next replicas too
      const uint64_t by_bytes = L ? std::max<uint64_t>(1, kWindowBytes / L) : kWindowReplicas;
      const uint32_t w = (uint32_t)std::min<uint64_t>({kWindowReplicas, by_bytes, (uint64_t)max_id - r + 1});
      ids.resize(w);
      for (uint32_t i = 0; i < w; ++i) ids[i] = (uint16_t)(r + i);
    }
  }
  const uint32_t nw = (uint32_t)ids.size();
  c.win_valid = false;
  rc = c.ensure(size ? size : 1, L * nw ? L * nw : 1);
  if (rc) return rc;
  hipError_t e = hipSuccess;
  if (size) {
    if (!same_input) parallel_copy({{c.h_in, data, size}});
    e = hipMemcpyAsync(c.d_in, c.h_in, size, hipMemcpyHostToDevice, c.stream);
  }
  if (e != hipSuccess) return hip_status(e);
  std::vector<uint8_t *> douts(nw);
  for (uint32_t i = 0; i < nw; ++i) douts[i] = c.d_out + (uint64_t)i * L;
  rc = encode_device(cb, k, ids.data(), nw, c.d_in, size, size, 1, douts.data(), 0, flags, c.stream);
  if (rc) return rc;
  if ((rc = c.push_out_and_wait(L * nw))) return rc;
  std::vector<Copy> parts(n);
  for (uint32_t i = 0; i < n; ++i) parts[i] = {outs[i], c.h_out + (uint64_t)i * L, L};
  parallel_copy(parts);
  if (n == 1) {
    c.win_valid = true;
    c.win_cb = cb;
    c.win_k = k;
    c.win_flags = flags;
    c.win_size = size;
    c.win_first = ids[0];
    c.win_n = nw;
    c.win_last_single = ids[0];
  }
  return VDS_EC_OK;
}

int restore_host(unsigned cb, uint32_t k, const uint16_t *nodes, const uint16_t *matrix, const uint8_t *const *chunks,
                 uint64_t chunk_size, uint64_t out_len, uint8_t *out, unsigned flags) {
  HostCtx *cp = host_ctx();
  if (!cp) return VDS_EC_ENODEV;
  HostCtx &c = *cp;
  const uint64_t in_bytes = chunk_size * k;
  int rc = c.ensure(in_bytes ? in_bytes : 1, out_len ? out_len : 1);
  if (rc) return rc;
  c.win_valid = false;  // h_in is overwritten
  // chunks staged contiguously (chunk j at + j*chunk_size), one DMA
  std::vector<Copy> in(k);
  for (uint32_t j = 0; j < k; ++j) in[j] = {c.h_in + (uint64_t)j * chunk_size, chunks[j], chunk_size};
  parallel_copy(in);
  if (in_bytes) {
    hipError_t e = hipMemcpyAsync(c.d_in, c.h_in, in_bytes, hipMemcpyHostToDevice, c.stream);
    if (e != hipSuccess) return hip_status(e);
  }
  ChunkLayout layout;
  layout.base = c.d_in;
  layout.pitch = chunk_size ? chunk_size : 1;
  if (k > (uint32_t)kInlineMatrixK) {
    rc = c.grow(&c.d_param, &c.d_param_cap, sizeof(uint16_t) * (size_t)k * k);
    if (rc) return rc;
    hipError_t e = hipMemcpyAsync(c.d_param, matrix, sizeof(uint16_t) * (size_t)k * k, hipMemcpyHostToDevice,
                                  c.stream);
    if (e != hipSuccess) return hip_status(e);
    layout.matrix_dev = reinterpret_cast<const uint16_t *>(c.d_param);
  }
  std::vector<const uint8_t *> dchunks(k);
  for (uint32_t j = 0; j < k; ++j) dchunks[j] = c.d_in + (uint64_t)j * chunk_size;
  rc = restore_device(cb, k, nodes, matrix, dchunks.data(), chunk_size, 0, out_len, 1, c.d_out, 0, flags, c.stream,
                      layout);
  if (rc) return rc;
  if ((rc = c.push_out_and_wait(out_len))) return rc;
  if (out_len) parallel_copy({{out, c.h_out, out_len}});
  return VDS_EC_OK;
}

// ------------------------------------------------------ regenerate core
// Replicas `targets` of objects restored from k survivors, without
// materialising the object: replica t = P(t) stripe by stripe, with P the
// polynomial through the survivors.  This is what sync_process's repair does
// with restore_async + save_data (sync_process.cpp:313-335,
// dht_network_client.cpp:582-658) -- decode, then re-encode -- fused.  The
// main kernels write P(t) of the untrimmed decode; the tail kernel then
// rewrites the last cell and the trailer as the route does (the decoded
// object trimmed to E bytes, the last stripe zero-padded on re-encode), so
// the bytes equal the reference's for any survivors, codeword or not
// (RegenTailArgs, ec_internal.hpp).
int regenerate_device(unsigned cb, uint32_t k, const uint16_t *nodes, const uint8_t *const *chunks,
                      uint64_t chunk_size, uint64_t chunk_stride, uint32_t count, const uint16_t *targets,
                      uint32_t nt, uint8_t *const *outs, uint64_t out_stride, hipStream_t s) {
  if (k == 0 || !nodes || !chunks || (nt > 0 && (!targets || !outs))) return VDS_EC_EINVAL;
  if (chunk_size < 2 || (chunk_size - 2) % cb) return VDS_EC_EINVAL;  // cells + BE16 trailer
  for (uint32_t j = 0; j < k; ++j)
    if (!chunks[j]) return VDS_EC_EINVAL;
  for (uint32_t i = 0; i < nt; ++i)
    if (!outs[i]) return VDS_EC_EINVAL;
  if (nt == 0 || count == 0) return VDS_EC_OK;
  int rc = device_ready();
  if (rc) return rc;
  std::vector<uint16_t> inv((size_t)k * k);
  if (cb == 2) {
    rc = inverse16(k, nodes, inv.data());
  } else {
    std::vector<uint8_t> n8(nodes, nodes + k);
    rc = inverse8(k, n8.data(), inv.data());
  }
  if (rc) return rc;
  const uint64_t T = (chunk_size - 2) / cb;
  uint64_t fast_stripes = 0;
  // coef[i][j] = sum_m t_i^m inv[m][j]  (P_m = sum_j inv[m][j] c_j): replica
  // t_i as a combination of the survivors
  auto coefs = [&](uint32_t base, uint32_t cnt) {
    std::vector<uint16_t> coef((size_t)cnt * k, 0);
    for (uint32_t i = 0; i < cnt; ++i) {
      const uint32_t t = targets[base + i];
      for (uint32_t m = 0; m < k; ++m) {
        const uint32_t tm = cb == 2 ? gf16_vandermonde(t, m) : (m == 0 ? 1u : gf8_pow(t, m));
        if (!tm) continue;
        for (uint32_t j = 0; j < k; ++j) {
          const uint32_t v = inv[(size_t)m * k + j];
          coef[(size_t)i * k + j] ^= (uint16_t)(cb == 2 ? gf16_mul(tm, v) : gf8_mul(tm, v));
        }
      }
    }
    return coef;
  };
  // objects [o0, o0 + cnt) still need cells [t_begin, T) and the trailer
  struct Part {
    uint64_t o0, cnt, t_begin;
  };
  Part parts[3] = {{0, count, 0}, {0, 0, 0}, {0, 0, 0}};
  SynRestoreArgs sa{};
  uint32_t syn_n = 0;
  if (cb == 2 && plan_restore_syn(k, nodes, sa, &syn_n)) {
    // the fast kernel regenerates erased points only: every target must be one
    bool all = true;
    for (uint32_t i = 0; i < nt && all; ++i) {
      bool hit = false;
      for (uint32_t w = 0; w < syn_n - k; ++w)
        if (sa.erased[w] == targets[i] && !sa.regen[w]) {  // (a repeated target: generic path)
          sa.regen[w] = outs[i];
          hit = true;
        }
      all = hit;
    }
    const uint64_t tiles = T / kTileStripes;
    const uint64_t total = tiles * count;
    if (all && tiles > 0 && total <= 0xFFFFFFFFull) {
      for (uint32_t j = 0; j < k; ++j) sa.chunks[j] = chunks[j];
      sa.chunk_stride = chunk_stride;
      sa.regen_stride = out_stride;
      sa.tiles_per_obj = (uint32_t)tiles;
      sa.total_tiles = (uint32_t)total;
      const hipFunction_t jf = jit_restore_function(k, syn_n, sa, true);  // (the set's own kernel, vds_ec_jit.cpp)
      hipError_t e = jf ? launch_restore_syn_jit(jf, k, syn_n, sa, s) : launch_restore_syn(k, syn_n, sa, s, true);
      if (e != hipSuccess) return hip_status(e);
      fast_stripes = tiles * kTileStripes;
      parts[0].t_begin = fast_stripes;
    }
  }
  if (!fast_stripes && cb == 2 && has_restore_fast(k) && nt <= k) {
    // any survivors, any targets (e.g. the live n = 64 shape): the
    // runtime-coefficient bit-sliced kernel with the nt x k combination rows,
    // over 512-stripe groups (tiles of four may straddle objects when 512 | T)
    const uint64_t gpo = T % 512 == 0 ? T / 512 : 4 * (T / kTileStripes);
    const uint64_t total = gpo * count / 4;
    if (gpo > 0 && gpo <= 0xFFFFFFFFull && total > 0 && total <= 0xFFFFFFFFull) {
      FastRestoreArgs fa{};
      for (uint32_t j = 0; j < k; ++j) fa.chunks[j] = chunks[j];
      fa.chunk_stride = chunk_stride;
      fa.out_stride = out_stride;
      fa.groups_per_obj = (uint32_t)gpo;
      fa.total_tiles = (uint32_t)total;
      fa.nt = nt;
      for (uint32_t i = 0; i < nt; ++i) fa.regen[i] = outs[i];
      const std::vector<uint16_t> coef = coefs(0, nt);
      for (size_t x = 0; x < coef.size(); ++x) fa.matrix2[x >> 1] |= uint32_t(coef[x]) << (16 * (x & 1));
      hipError_t e = launch_restore_fast(k, fa, s, true);
      if (e != hipSuccess) return hip_status(e);
      if (gpo % 4 == 0) {
        fast_stripes = 512 * gpo;
        parts[0].t_begin = fast_stripes;
      } else {  // stream: the first 2048 * total stripes of the objects taken as one stream
        const uint64_t fast_total = (uint64_t)kTileStripes * total, o_full = fast_total / T;
        fast_stripes = fast_total;
        parts[0] = {0, o_full, T};
        parts[1] = {o_full, o_full < count ? 1u : 0u, fast_total - o_full * T};
        parts[2] = {o_full + 1, o_full + 1 < count ? count - o_full - 1 : 0, 0};
      }
    }
  }
  // generic path: the remaining cells and the trailers, <= 64 targets per
  // launch; a k > 64 chunk table and coefficient blocks beyond kInlineCoef
  // ride the stream-ordered parameter ring (one staged blob for the call)
  std::vector<uint8_t> blob;
  const bool tmp_table = k > (uint32_t)kInlineChunks;
  const size_t off_table = tmp_table ? blob_append(blob, chunks, k) : SIZE_MAX;
  // the tail's V_S^{-1} (regen_tail below)
  const size_t off_inv = cb == 2 && k > (uint32_t)kInlineMatrixK ? blob_append(blob, inv.data(), inv.size()) : SIZE_MAX;
  std::vector<std::vector<uint16_t>> coef_blocks;
  std::vector<size_t> coef_off;
  for (uint32_t base = 0; base < nt; base += kMaxLaunchReplicas) {
    coef_blocks.push_back(coefs(base, std::min<uint32_t>(nt - base, kMaxLaunchReplicas)));
    const auto &c = coef_blocks.back();
    coef_off.push_back(c.size() > (size_t)kInlineCoef ? blob_append(blob, c.data(), c.size()) : SIZE_MAX);
  }
  hipError_t e = hipSuccess;
  ParamSlot *slot = nullptr;
  const uint8_t *dparam = nullptr;
  if (!blob.empty()) e = param_stage(blob, s, &dparam, &slot);
  for (uint32_t base = 0, bi = 0; base < nt && e == hipSuccess; base += kMaxLaunchReplicas, ++bi) {
    RegenArgs ga{};
    ga.nt = std::min<uint32_t>(nt - base, kMaxLaunchReplicas);
    if (tmp_table) ga.chunk_table = reinterpret_cast<const uint8_t *const *>(dparam + off_table);
    const std::vector<uint16_t> &coef = coef_blocks[bi];
    if (coef_off[bi] == SIZE_MAX) {
      for (size_t x = 0; x < coef.size(); ++x) ga.coef_inline[x >> 1] |= uint32_t(coef[x]) << (16 * (x & 1));
    } else {
      ga.coef_dev = reinterpret_cast<const uint16_t *>(dparam + coef_off[bi]);
    }
    ga.chunk_stride = chunk_stride;
    ga.k = k;
    ga.cell_bytes = cb;
    ga.T = T;
    ga.out_stride = out_stride;
    for (const Part &pt : parts) {
      if (e != hipSuccess || pt.cnt == 0) continue;
      if (tmp_table && pt.o0) {  // (k > 64: never with a fast path, so o0 == 0)
        e = hipErrorInvalidValue;
        break;
      }
      if (!tmp_table)
        for (uint32_t j = 0; j < k; ++j) ga.chunk_ptr[j] = chunks[j] + pt.o0 * chunk_stride;
      for (uint32_t i = 0; i < ga.nt; ++i) ga.outs[i] = outs[base + i] + pt.o0 * out_stride;
      ga.count = (uint32_t)pt.cnt;
      ga.t_begin = pt.t_begin;
      ga.t_count = T - pt.t_begin;
      e = launch_regen_generic(ga, s);
    }
  }
  // the reference route's last cell and trailer (trim to E, then re-encode),
  // over what the kernels above wrote (same stream)
  for (uint32_t base = 0; cb == 2 && base < nt && e == hipSuccess; base += kMaxLaunchReplicas) {
    RegenTailArgs ta{};
    if (tmp_table)
      ta.chunk_table = reinterpret_cast<const uint8_t *const *>(dparam + off_table);
    else
      for (uint32_t j = 0; j < k; ++j) ta.chunk_ptr[j] = chunks[j];
    ta.chunk_stride = chunk_stride;
    if (off_inv != SIZE_MAX)
      ta.matrix_dev = reinterpret_cast<const uint16_t *>(dparam + off_inv);
    else
      for (uint32_t i = 0; i < k * k; ++i) ta.matrix_inline[i >> 1] |= uint32_t(inv[i]) << (16 * (i & 1));
    ta.chunk_size = chunk_size;
    ta.k = k;
    ta.count = count;
    ta.nt = std::min<uint32_t>(nt - base, kMaxLaunchReplicas);
    for (uint32_t i = 0; i < ta.nt; ++i) {
      ta.targets[i] = targets[base + i];
      ta.outs[i] = outs[base + i];
    }
    ta.out_stride = out_stride;
    e = launch_regen_tail(ta, s);
  }
  if (slot) {
    const hipError_t re = param_release(slot, s);
    if (e == hipSuccess) e = re;
  }
  return hip_status(e);
}

int regenerate_host(unsigned cb, uint32_t k, const uint16_t *nodes, const uint8_t *const *chunks, uint64_t chunk_size,
                    const uint16_t *targets, uint32_t nt, uint8_t *const *outs) {
  if (k == 0 || !nodes || !chunks || (nt > 0 && (!targets || !outs))) return VDS_EC_EINVAL;
  if (chunk_size < 2 || (chunk_size - 2) % cb) return VDS_EC_EINVAL;
  for (uint32_t j = 0; j < k; ++j)
    if (!chunks[j]) return VDS_EC_EINVAL;
  for (uint32_t i = 0; i < nt; ++i)
    if (!outs[i]) return VDS_EC_EINVAL;
  // The reference route restores first (chunk.h:402-444, with chunks[0]'s
  // trailer p): a trailer it cannot restore with fails there ("Fatal
  // error"), and p > 2k would re-encode to a replica longer than chunk_size.
  if (cb == 2) {
    const uint16_t p = (uint16_t)((chunks[0][chunk_size - 2] << 8) | chunks[0][chunk_size - 1]);
    bool ok = true;
    (void)restored_len(2, k, chunk_size, p, 0, &ok);
    if (!ok || p > 2 * k) return VDS_EC_ERESTORE;
  }
  int rc = device_ready();
  if (rc) return rc;
  if (nt == 0) return VDS_EC_OK;
  HostCtx *cp = host_ctx();
  if (!cp) return VDS_EC_ENODEV;
  HostCtx &c = *cp;
  rc = c.ensure(chunk_size * k, chunk_size * nt);
  if (rc) return rc;
  c.win_valid = false;
  std::vector<const uint8_t *> dchunks(k);
  std::vector<Copy> in(k);
  for (uint32_t j = 0; j < k; ++j) {
    dchunks[j] = c.d_in + (uint64_t)j * chunk_size;
    in[j] = {c.h_in + (uint64_t)j * chunk_size, chunks[j], chunk_size};
  }
  parallel_copy(in);
  hipError_t e = hipMemcpyAsync(c.d_in, c.h_in, chunk_size * k, hipMemcpyHostToDevice, c.stream);
  if (e != hipSuccess) return hip_status(e);
  std::vector<uint8_t *> douts(nt);
  for (uint32_t i = 0; i < nt; ++i) douts[i] = c.d_out + (uint64_t)i * chunk_size;
  rc = regenerate_device(cb, k, nodes, dchunks.data(), chunk_size, 0, 1, targets, nt, douts.data(), 0, c.stream);
  if (rc) return rc;
  if ((rc = c.push_out_and_wait(chunk_size * nt))) return rc;
  std::vector<Copy> parts(nt);
  for (uint32_t i = 0; i < nt; ++i) parts[i] = {outs[i], c.h_out + (uint64_t)i * chunk_size, chunk_size};
  parallel_copy(parts);
  return VDS_EC_OK;
}

// The k replica ids of one object pairwise distinct (else V_S is singular).
// The batch entry points check every object with this before anything is
// enqueued, so a bad object fails the call without partial output.
bool ids_distinct(uint32_t k, const uint16_t *nd) {
  uint64_t seen = 0;
  bool wide = false;
  for (uint32_t j = 0; j < k; ++j) {
    if (nd[j] >= 64) {
      wide = true;
      continue;
    }
    if ((seen >> nd[j]) & 1u) return false;
    seen |= 1ull << nd[j];
  }
  if (!wide) return true;
  std::vector<uint16_t> v(nd, nd + k);
  std::sort(v.begin(), v.end());
  return std::adjacent_find(v.begin(), v.end()) == v.end();
}

}  // namespace api
}  // namespace vds_ec

// ====================================================================== C ABI

extern "C" {

const char *vds_ec_strerror(int status) {
  switch (status) {
    case VDS_EC_OK: return "ok";
    case VDS_EC_EINVAL: return "invalid argument";
    case VDS_EC_ENODEV: return "no usable GPU (vds_ec has no CPU fallback)";
    case VDS_EC_ENOMEM: return "device or pinned allocation failed";
    case VDS_EC_ESINGULAR: return "replica ids are not distinct (singular Vandermonde matrix)";
    case VDS_EC_ERESTORE: return "Fatal error at chunk_restore::restore";
    case VDS_EC_EHIP: return "HIP runtime error";
    case VDS_EC_EB64_LENGTH: return "Non-Valid base64!";
    case VDS_EC_EB64_PADDING: return "Invalid Padding in Base 64!";
    case VDS_EC_EB64_CHAR: return "Non-Valid Character in Base 64!";
    default: return "unknown vds_ec status";
  }
}

int vds_ec_version(void) { return kVersion; }

int vds_ec_host_ctx_stats(uint64_t *created, uint64_t *pooled) {
  if (created) *created = g_host_ctx_created.load(std::memory_order_relaxed);
  if (pooled) *pooled = host_ctx_pooled();
  return VDS_EC_OK;
}

int vds_ec_device_count(int *count) {
  if (!count) return VDS_EC_EINVAL;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
  *count = n;
  return VDS_EC_OK;
}

uint64_t vds_ec_replica_size(unsigned cell_bytes, unsigned k, uint64_t size, unsigned flags) {
  if (k == 0 || (cell_bytes != 1 && cell_bytes != 2)) return 0;
  const uint64_t stripe = (uint64_t)cell_bytes * k;
  const uint64_t cells = (size + stripe - 1) / stripe;
  const bool trailer = !(flags & (VDS_EC_F_NO_TRAILER | VDS_EC_F_CELLS));
  return cells * cell_bytes + (trailer ? 2 : 0);
}

uint64_t vds_ec_restored_size(unsigned cell_bytes, unsigned k, uint64_t replica_size, uint16_t padding) {
  bool ok = true;
  uint64_t e = restored_len(cell_bytes, k, replica_size, padding, 0, &ok);
  return ok ? e : 0;
}

int vds_ec_gf16_tables(uint16_t *value2log, uint16_t *log2value) {
  if (!value2log || !log2value) return VDS_EC_EINVAL;
  // gf.h:197-216: log2value[l] = x^l for l < 65535, value2log inverse,
  // value2log[0] = 0 and log2value[65535] = 0 (never read).
  std::memset(value2log, 0, 65536 * sizeof(uint16_t));
  std::memset(log2value, 0, 65536 * sizeof(uint16_t));
  uint32_t v = 1;
  for (uint32_t l = 0; l < 65535; ++l) {
    log2value[l] = (uint16_t)v;
    value2log[v] = (uint16_t)l;
    v = gf16_mul(v, 2);
  }
  return VDS_EC_OK;
}

int vds_ec_gf8_tables(uint8_t *value2log, uint8_t *log2value) {
  if (!value2log || !log2value) return VDS_EC_EINVAL;
  std::memset(value2log, 0, 256);
  std::memset(log2value, 0, 256);
  uint32_t v = 1;
  for (uint32_t l = 0; l < 255; ++l) {
    log2value[l] = (uint8_t)v;
    value2log[v] = (uint8_t)l;
    v = gf8_mul(v, 2);
  }
  return VDS_EC_OK;
}

int vds_ec_multipliers16(uint16_t k, uint16_t node, uint16_t *out) {
  if (!out && k) return VDS_EC_EINVAL;
  for (uint32_t j = 0; j < k; ++j) out[j] = gf16_vandermonde(node, j);
  return VDS_EC_OK;
}

int vds_ec_multipliers8(uint8_t k, uint8_t node, uint8_t *out) {
  if (!out && k) return VDS_EC_EINVAL;
  for (uint32_t j = 0; j < k; ++j) out[j] = j == 0 ? 1 : gf8_pow(node, j);
  return VDS_EC_OK;
}

int vds_ec_inverse16(uint16_t k, const uint16_t *nodes, uint16_t *out) {
  if (k == 0 || !nodes || !out) return VDS_EC_EINVAL;
  return inverse16(k, nodes, out);
}

int vds_ec_inverse8(uint8_t k, const uint8_t *nodes, uint8_t *out) {
  if (k == 0 || !nodes || !out) return VDS_EC_EINVAL;
  std::vector<uint16_t> m((size_t)k * k);
  int rc = inverse8(k, nodes, m.data());
  if (rc) return rc;
  for (size_t i = 0; i < m.size(); ++i) out[i] = (uint8_t)m[i];
  return VDS_EC_OK;
}

int vds_ec_encode16_device(uint16_t k, const uint16_t *replicas, uint32_t n, const uint8_t *in,
                           uint64_t size, uint64_t in_stride, uint32_t count, uint8_t *const *outs,
                           uint64_t out_stride, unsigned flags, void *stream) {
  return encode_device(2, k, replicas, n, in, size, in_stride, count, outs, out_stride, flags, as_stream(stream));
}

int vds_ec_encode8_device(uint8_t k, const uint8_t *replicas, uint32_t n, const uint8_t *in,
                          uint64_t size, uint64_t in_stride, uint32_t count, uint8_t *const *outs,
                          uint64_t out_stride, unsigned flags, void *stream) {
  if (n > 0 && !replicas) return VDS_EC_EINVAL;
  std::vector<uint16_t> ids(replicas, replicas + n);
  return encode_device(1, k, ids.data(), n, in, size, in_stride, count, outs, out_stride, flags, as_stream(stream));
}

int vds_ec_restore16_device(uint16_t k, const uint16_t *nodes, const uint8_t *const *chunks,
                            uint64_t chunk_size, uint64_t chunk_stride, uint16_t padding,
                            uint32_t count, uint8_t *out, uint64_t out_stride, unsigned flags,
                            void *stream) {
  int rc = check_restore_args(k, nodes, chunks, chunk_size);
  if (rc) return rc;
  bool ok = true;
  const uint64_t len = restored_len(2, k, chunk_size, padding, flags, &ok);
  if (!ok) return VDS_EC_ERESTORE;
  if (len && count && !out) return VDS_EC_EINVAL;
  std::vector<uint16_t> m((size_t)k * k);
  rc = inverse16(k, nodes, m.data());
  if (rc) return rc;
  return restore_device(2, k, nodes, m.data(), chunks, chunk_size, chunk_stride, len, count, out, out_stride, flags,
                        as_stream(stream));
}

int vds_ec_restore8_device(uint8_t k, const uint8_t *nodes, const uint8_t *const *chunks,
                           uint64_t chunk_size, uint64_t chunk_stride, uint16_t padding,
                           uint32_t count, uint8_t *out, uint64_t out_stride, unsigned flags,
                           void *stream) {
  int rc = check_restore_args(k, nodes, chunks, chunk_size);
  if (rc) return rc;
  bool ok = true;
  const uint64_t len = restored_len(1, k, chunk_size, padding, flags, &ok);
  if (!ok) return VDS_EC_ERESTORE;
  if (len && count && !out) return VDS_EC_EINVAL;
  std::vector<uint16_t> m((size_t)k * k);
  rc = inverse8(k, nodes, m.data());
  if (rc) return rc;
  return restore_device(1, k, nullptr, m.data(), chunks, chunk_size, chunk_stride, len, count, out, out_stride, flags,
                        as_stream(stream));
}

int vds_ec_encode16_host(uint16_t k, const uint16_t *replicas, uint32_t n, const uint8_t *data,
                         uint64_t size, uint8_t *const *outs, unsigned flags) {
  return encode_host(2, k, replicas, n, data, size, outs, flags);
}

int vds_ec_encode8_host(uint8_t k, const uint8_t *replicas, uint32_t n, const uint8_t *data,
                        uint64_t size, uint8_t *const *outs, unsigned flags) {
  if (n > 0 && !replicas) return VDS_EC_EINVAL;
  std::vector<uint16_t> ids(replicas, replicas + n);
  return encode_host(1, k, ids.data(), n, data, size, outs, flags);
}

int vds_ec_restore16_host(uint16_t k, const uint16_t *nodes, const uint8_t *const *chunks,
                          uint64_t chunk_size, uint8_t *out, uint64_t *out_size, unsigned flags) {
  int rc = check_restore_args(k, nodes, chunks, chunk_size);
  if (rc) return rc;
  rc = device_ready();
  if (rc) return rc;
  const bool cells = (flags & VDS_EC_F_CELLS) != 0;
  const uint16_t padding =
      (cells || chunk_size < 2) ? 0 : (uint16_t)((chunks[0][chunk_size - 2] << 8) | chunks[0][chunk_size - 1]);
  bool ok = true;
  const uint64_t len = restored_len(2, k, chunk_size, padding, flags, &ok);
  if (!ok) return VDS_EC_ERESTORE;
  if (len && !out) return VDS_EC_EINVAL;
  std::vector<uint16_t> m((size_t)k * k);
  rc = inverse16(k, nodes, m.data());
  if (rc) return rc;
  rc = restore_host(2, k, nodes, m.data(), chunks, chunk_size, len, out, flags);
  if (rc == VDS_EC_OK && out_size) *out_size = len;
  return rc;
}

int vds_ec_restore8_host(uint8_t k, const uint8_t *nodes, const uint8_t *const *chunks,
                         uint64_t chunk_size, uint8_t *out, uint64_t *out_size, unsigned flags) {
  int rc = check_restore_args(k, nodes, chunks, chunk_size);
  if (rc) return rc;
  rc = device_ready();
  if (rc) return rc;
  const bool cells = (flags & VDS_EC_F_CELLS) != 0;
  const uint16_t padding =
      (cells || chunk_size < 2) ? 0 : (uint16_t)((chunks[0][chunk_size - 2] << 8) | chunks[0][chunk_size - 1]);
  bool ok = true;
  const uint64_t len = restored_len(1, k, chunk_size, padding, flags, &ok);
  if (!ok) return VDS_EC_ERESTORE;
  if (len && !out) return VDS_EC_EINVAL;
  std::vector<uint16_t> m((size_t)k * k);
  rc = inverse8(k, nodes, m.data());
  if (rc) return rc;
  rc = restore_host(1, k, nullptr, m.data(), chunks, chunk_size, len, out, flags);
  if (rc == VDS_EC_OK && out_size) *out_size = len;
  return rc;
}

int vds_ec_host_alloc(uint64_t bytes, void **ptr) {
  if (!ptr || bytes == 0) return VDS_EC_EINVAL;
  *ptr = nullptr;
  int rc = device_ready();
  if (rc) return rc;
  void *p = nullptr;
  if (hipHostMalloc(&p, bytes, hipHostMallocMapped | hipHostMallocPortable) != hipSuccess) return VDS_EC_ENOMEM;
  void *d = nullptr;
  if (hipHostGetDevicePointer(&d, p, 0) != hipSuccess) {
    (void)hipHostFree(p);
    return VDS_EC_EHIP;
  }
  PinnedRange pr{bytes, true};
  int dev = 0;
  if (hipGetDevice(&dev) == hipSuccess && dev >= 0 && dev < kPinnedMaxDev) pr.dev[dev] = static_cast<uint8_t *>(d);
  PinnedRegistry &r = pinned_registry();
  std::lock_guard<std::mutex> g(r.mu);
  r.ranges[reinterpret_cast<uintptr_t>(p)] = pr;
  *ptr = p;
  return VDS_EC_OK;
}

int vds_ec_host_free(void *ptr) {
  if (!ptr) return VDS_EC_OK;
  PinnedRegistry &r = pinned_registry();
  {
    std::lock_guard<std::mutex> g(r.mu);
    auto it = r.ranges.find(reinterpret_cast<uintptr_t>(ptr));
    if (it == r.ranges.end() || !it->second.owned) return VDS_EC_EINVAL;
    r.ranges.erase(it);
  }
  return hip_status(hipHostFree(ptr));
}

int vds_ec_host_register(void *ptr, uint64_t bytes) {
  if (!ptr || bytes == 0) return VDS_EC_EINVAL;
  int rc = device_ready();
  if (rc) return rc;
  if (hipHostRegister(ptr, bytes, hipHostRegisterMapped | hipHostRegisterPortable) != hipSuccess) return VDS_EC_EHIP;
  void *d = nullptr;
  if (hipHostGetDevicePointer(&d, ptr, 0) != hipSuccess) {
    (void)hipHostUnregister(ptr);
    return VDS_EC_EHIP;
  }
  PinnedRange pr{bytes, false};
  int dev = 0;
  if (hipGetDevice(&dev) == hipSuccess && dev >= 0 && dev < kPinnedMaxDev) pr.dev[dev] = static_cast<uint8_t *>(d);
  PinnedRegistry &r = pinned_registry();
  std::lock_guard<std::mutex> g(r.mu);
  r.ranges[reinterpret_cast<uintptr_t>(ptr)] = pr;
  return VDS_EC_OK;
}

int vds_ec_host_unregister(void *ptr) {
  PinnedRegistry &r = pinned_registry();
  {
    std::lock_guard<std::mutex> g(r.mu);
    auto it = r.ranges.find(reinterpret_cast<uintptr_t>(ptr));
    if (it == r.ranges.end() || it->second.owned) return VDS_EC_EINVAL;
    r.ranges.erase(it);
  }
  return hip_status(hipHostUnregister(ptr));
}

int vds_ec_encode16_host_batch(uint16_t k, const uint16_t *replicas, uint32_t n,
                               const uint8_t *const *objs, const uint64_t *sizes, uint32_t count,
                               uint8_t *const *outs, unsigned flags, int max_devices) {
  return encode_host_batch(k, replicas, n, objs, sizes, count, outs, flags, max_devices);
}

int vds_ec_restore16_host_batch(uint16_t k, const uint16_t *nodes, const uint8_t *const *chunks,
                                const uint64_t *chunk_sizes, uint32_t count, uint8_t *const *outs, uint64_t *out_sizes,
                                unsigned flags, int max_devices) {
  return restore_host_batch(k, nodes, chunks, chunk_sizes, count, outs, out_sizes, flags, max_devices);
}

int vds_ec_encode16_range_device(uint16_t k, const uint16_t *replicas, uint32_t n, const uint8_t *in, uint64_t size,
                                 uint64_t t0, uint64_t t1, uint8_t *const *outs, unsigned flags, void *stream) {
  return encode_range(k, replicas, n, in, size, t0, t1, outs, flags, as_stream(stream));
}

int vds_ec_restore16_range_device(uint16_t k, const uint16_t *nodes, const uint8_t *const *chunks, uint64_t chunk_size,
                                  uint16_t padding, uint64_t t0, uint64_t t1, uint8_t *out, unsigned flags,
                                  void *stream) {
  int rc = check_restore_args(k, nodes, chunks, chunk_size);
  if (rc) return rc;
  uint64_t E = 0, nst = 0;
  if ((rc = range_restore_len(k, chunk_size, padding, flags, &E, &nst))) return rc;
  if (t0 > t1 || t1 > nst || (E && !out)) return VDS_EC_EINVAL;
  if (t0 == t1) return VDS_EC_OK;
  std::vector<uint16_t> m((size_t)k * k);
  if ((rc = inverse16(k, nodes, m.data()))) return rc;
  return restore_range(k, nodes, m.data(), chunks, t0, t1, E, out, flags, as_stream(stream));
}

int vds_ec_encode16_host_split(uint16_t k, const uint16_t *replicas, uint32_t n, const uint8_t *data, uint64_t size,
                               uint8_t *const *outs, unsigned flags, int max_devices, uint32_t parts) {
  return encode_host_split(k, replicas, n, data, size, outs, flags, max_devices, parts);
}

int vds_ec_restore16_host_split(uint16_t k, const uint16_t *nodes, const uint8_t *const *chunks, uint64_t chunk_size,
                                uint8_t *out, uint64_t *out_size, unsigned flags, int max_devices, uint32_t parts) {
  return restore_host_split(k, nodes, chunks, chunk_size, out, out_size, flags, max_devices, parts);
}

int vds_ec_sha256_device(const uint8_t *base, uint64_t len, uint64_t stride, uint32_t count, uint8_t *digests,
                         void *stream) {
  if (count && (!digests || (len && !base))) return VDS_EC_EINVAL;
  if (count == 0) return VDS_EC_OK;
  int rc = device_ready();
  if (rc) return rc;
  return hip_status(launch_sha256(base, len, stride, count, digests, as_stream(stream)));
}

int vds_ec_encode16_hash_host(uint16_t k, const uint16_t *replicas, uint32_t n, const uint8_t *data, uint64_t size,
                              uint8_t *const *outs, uint8_t *digests, unsigned flags) {
  if (k == 0 || (n > 0 && (!replicas || !outs || !digests)) || (size > 0 && !data)) return VDS_EC_EINVAL;
  int rc = device_ready();
  if (rc) return rc;
  if (n == 0) return VDS_EC_OK;
  const uint64_t L = vds_ec_replica_size(2, k, size, flags);
  HostCtx *cp = host_ctx();
  if (!cp) return VDS_EC_ENODEV;
  HostCtx &c = *cp;
  // replicas, then the digests at a 16-byte aligned offset: one push out
  const uint64_t dig = (L * n + 15) & ~15ull;
  rc = c.ensure(size ? size : 1, dig + 32ull * n);
  if (!rc) rc = c.stage_in(data, size);
  if (rc) return rc;
  std::vector<uint8_t *> douts(n);
  for (uint32_t i = 0; i < n; ++i) douts[i] = c.d_out + (uint64_t)i * L;
  // (an error after the first enqueue drains the stream before returning:
  // the next call on this thread reuses c's buffers)
  auto drained = [&](int r) {
    (void)hipStreamSynchronize(c.stream);
    return r;
  };
  rc = encode_device(2, k, replicas, n, c.d_in, size, size, 1, douts.data(), 0, flags, c.stream);
  if (rc) return drained(rc);
  // the replica hashes of save_temp / save_data (dht_network_client.cpp:79, :593), on the device
  hipError_t e = launch_sha256(c.d_out, L, L, n, c.d_out + dig, c.stream);
  if (e != hipSuccess) return drained(hip_status(e));
  if ((rc = c.push_out_and_wait(dig + 32ull * n))) return rc;
  std::vector<Copy> parts(n);
  for (uint32_t i = 0; i < n; ++i) parts[i] = {outs[i], c.h_out + (uint64_t)i * L, L};
  parts.push_back({digests, c.h_out + dig, 32ull * n});
  parallel_copy(parts);
  return VDS_EC_OK;
}

int vds_ec_save_temp16_host(uint16_t k, uint32_t n, const uint8_t *data, uint64_t size, uint8_t *const *outs,
                            uint8_t *replica_digests, uint8_t *data_digest, uint32_t *replica_size) {
  if (k == 0 || (n > 0 && (!outs || !replica_digests)) || !data_digest || (size > 0 && !data)) return VDS_EC_EINVAL;
  int rc = device_ready();
  if (rc) return rc;
  const uint64_t L = vds_ec_replica_size(2, k, size, 0);
  if (replica_size) *replica_size = (uint32_t)L;  // save_temp: replica 0's size (dht_network_client.cpp:81-83)
  if (n == 0) {  // only the body hash: nothing to stage or encode
    sha256_host(data, size, data_digest);
    return VDS_EC_OK;
  }
  HostCtx *cp = host_ctx();
  if (!cp) return VDS_EC_ENODEV;
  HostCtx &c = *cp;
  // replicas, then n digests at a 16-byte aligned offset: one push out
  const uint64_t dig = (L * n + 15) & ~15ull;
  rc = c.ensure(size ? size : 1, dig + 32ull * n);
  if (!rc) rc = c.stage_in(data, size);
  if (rc) return rc;
  // (an error after the first enqueue drains the stream before returning:
  // the next call on this thread reuses c's buffers)
  auto drained = [&](int r) {
    (void)hipStreamSynchronize(c.stream);
    return r;
  };
  std::vector<Copy> parts;
  std::vector<uint16_t> ids(n);
  std::vector<uint8_t *> douts(n);
  for (uint32_t i = 0; i < n; ++i) {
    ids[i] = (uint16_t)i;
    douts[i] = c.d_out + (uint64_t)i * L;
    parts.push_back({outs[i], c.h_out + (uint64_t)i * L, L});
  }
  rc = encode_device(2, k, ids.data(), n, c.d_in, size, size, 1, douts.data(), 0, 0, c.stream);
  if (rc) return drained(rc);
  hipError_t e = launch_sha256(c.d_out, L, L, n, c.d_out + dig, c.stream);  // save_temp's replica names (:79)
  if (e != hipSuccess) return drained(hip_status(e));
  e = launch_push(c.h_out_dev, c.d_out, dig + 32ull * n, c.stream);
  if (e != hipSuccess) return drained(hip_status(e));
  parts.push_back({replica_digests, c.h_out + dig, 32ull * n});
  // upload_data's hash of the body (server_api.cpp:16) on this thread while
  // the device works: one sequential chain, ~3 us a block in a GPU lane
  // (sha256_host.cpp)
  sha256_host(data, size, data_digest);
  if ((rc = hip_status(hipStreamSynchronize(c.stream)))) return rc;
  parallel_copy(parts);
  return VDS_EC_OK;
}

int vds_ec_replica_paths(const uint8_t *digests, uint32_t count, char *out) {
  if (count && (!digests || !out)) return VDS_EC_EINVAL;
  static const char kB64[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789#_";  // '+' '/' replaced
  for (uint32_t i = 0; i < count; ++i) {
    const uint8_t *d = digests + 32ull * i;
    char b64[45];
    int n = 0;
    for (int p = 0; p + 2 < 32; p += 3) {  // 10 full groups
      const uint32_t t = (uint32_t(d[p]) << 16) | (uint32_t(d[p + 1]) << 8) | d[p + 2];
      for (int s = 18; s >= 0; s -= 6) b64[n++] = kB64[(t >> s) & 63];
    }
    const uint32_t t = (uint32_t(d[30]) << 16) | (uint32_t(d[31]) << 8);  // 2 bytes left: 3 chars + '='
    b64[n++] = kB64[(t >> 18) & 63];
    b64[n++] = kB64[(t >> 12) & 63];
    b64[n++] = kB64[(t >> 6) & 63];
    b64[n++] = '=';
    char *o = out + (size_t)VDS_EC_PATH_BYTES * i;
    std::memcpy(o, b64, 10);
    o[10] = '/';
    std::memcpy(o + 11, b64 + 10, 10);
    o[21] = '/';
    std::memcpy(o + 22, b64 + 20, 24);
    o[46] = 0;
    o[47] = 0;
  }
  return VDS_EC_OK;
}

int vds_ec_regenerate16_device(uint16_t k, const uint16_t *nodes, const uint8_t *const *chunks, uint64_t chunk_size,
                               uint64_t chunk_stride, uint32_t count, const uint16_t *targets, uint32_t ntargets,
                               uint8_t *const *outs, uint64_t out_stride, void *stream) {
  return regenerate_device(2, k, nodes, chunks, chunk_size, chunk_stride, count, targets, ntargets, outs, out_stride,
                           as_stream(stream));
}

int vds_ec_regenerate16_host(uint16_t k, const uint16_t *nodes, const uint8_t *const *chunks, uint64_t chunk_size,
                             const uint16_t *targets, uint32_t ntargets, uint8_t *const *outs) {
  return regenerate_host(2, k, nodes, chunks, chunk_size, targets, ntargets, outs);
}

int vds_ec_restore16_batch_device(uint16_t k, uint32_t count, const uint16_t *nodes, const uint8_t *const *chunks,
                                  const uint64_t *chunk_sizes, const uint16_t *paddings, uint8_t *const *outs,
                                  unsigned flags, void *stream) {
  return restore_batch_device(k, count, nodes, chunks, chunk_sizes, paddings, outs, flags, as_stream(stream));
}

int vds_ec_regenerate16_batch_device(uint16_t k, uint32_t count, const uint16_t *nodes, const uint8_t *const *chunks,
                                     const uint64_t *chunk_sizes, uint32_t ntargets, const uint16_t *targets,
                                     uint8_t *const *outs, void *stream) {
  return regenerate_batch_device(k, count, nodes, chunks, chunk_sizes, ntargets, targets, outs, as_stream(stream));
}

int vds_ec_regenerate16_path(uint16_t k, const uint16_t *nodes, const uint16_t *targets, uint32_t ntargets,
                             uint64_t chunk_size) {
  if (k == 0 || !nodes || (ntargets && !targets) || chunk_size < 2) return 0;
  SynRestoreArgs sa{};
  uint32_t n = 0;
  const uint64_t T = (chunk_size - 2) / 2;
  bool syn = T >= kTileStripes && plan_restore_syn(k, nodes, sa, &n);
  for (uint32_t i = 0; syn && i < ntargets; ++i) {  // (mirrors regenerate_device's choice)
    bool hit = false;
    for (uint32_t w = 0; w < n - k; ++w)
      if (sa.erased[w] == targets[i] && !sa.regen[w]) {
        sa.regen[w] = reinterpret_cast<uint8_t *>(1);
        hit = true;
      }
    syn = hit;
  }
  if (syn) return jit_ready(k, n, sa, true) ? 4 : 3;
  const uint64_t gpo = T % 512 == 0 ? T / 512 : 4 * (T / kTileStripes);
  return (has_restore_fast(k) && ntargets <= k && gpo > 0) ? 2 : 1;
}

int vds_ec_fill_splitmix_device(uint8_t *dst, uint64_t size, uint64_t seed, void *stream) {
  if (size && !dst) return VDS_EC_EINVAL;
  int rc = device_ready();
  if (rc) return rc;
  return hip_status(launch_fill_splitmix(dst, size, seed, as_stream(stream)));
}

int vds_ec_encode16_path(uint16_t k, const uint16_t *replicas, uint32_t n, uint64_t size) {
  bool contiguous = replicas != nullptr;
  for (uint32_t i = 0; contiguous && i < n; ++i) contiguous &= (replicas[i] == i);
  // (for a batch of at least one 2048-stripe tile of full stripes)
  const uint64_t F = k ? size / (2ull * k) : 0;
  const bool fast = F >= kTileStripes || (F > 0 && F % 128 == 0 && k >= 8);
  return (contiguous && has_encode_fast(k, n) && fast) ? 2 : 1;
}

int vds_ec_restore16_path(uint16_t k, const uint16_t *nodes, uint64_t chunk_size, uint16_t padding, uint32_t count) {
  bool ok = true;
  const uint64_t len = restored_len(2, k, chunk_size, padding, 0, &ok);
  if (!ok || k == 0) return 1;
  const int path = plan_restore(2, k, nodes, len, count, 0).path;
  return path == 3 && jit_enabled() && vds_ec_jit_ready16(k, nodes) ? 4 : path;
}

}  // extern "C"
