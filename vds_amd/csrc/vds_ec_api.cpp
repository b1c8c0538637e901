// vds_ec_api.cpp -- the C ABI declared in include/vds_ec.h.
//
// Host-side runtime of the codec: argument validation mirroring the
// reference's contracts (chunk.h, chunk_storage.cpp), the Vandermonde
// inverse (the chunk_restore constructor), dispatch between the bit-sliced
// and generic kernels, host-memory staging and the multi-GPU batch driver.
// All data-path arithmetic runs in the HIP kernels (ec_*.hip); the
// only host arithmetic is on k x k matrices and tables.
#include "../../include/vds_ec.h"

#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <array>
#include <climits>
#include <condition_variable>
#include <cstdint>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <vector>

#include "ec_internal.hpp"
#include "gf_common.hpp"

using namespace vds_ec;

namespace {

constexpr int kVersion = 100;  // 0.1.0

inline hipStream_t as_stream(void *s) { return reinterpret_cast<hipStream_t>(s); }

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

// ------------------------------------------------- host field arithmetic
// log / antilog tables for the host's k x k and M x M work (gf.h:193-253's
// tables; the kernels never use them).  Built once, 384 KiB.
struct Gf16Tables {
  uint16_t log[65536];
  uint16_t exp[2 * 65535];
  Gf16Tables() {
    uint32_t v = 1;
    for (uint32_t l = 0; l < 65535; ++l) {
      exp[l] = exp[l + 65535] = (uint16_t)v;
      log[v] = (uint16_t)l;
      v = gf16_mul(v, 2);
    }
    log[0] = 0;
  }
};

const Gf16Tables &gf16_tables() {
  static const Gf16Tables *t = new Gf16Tables();  // never freed
  return *t;
}

inline uint32_t gf16_mul_fast(uint32_t a, uint32_t b) {
  if (!a || !b) return 0;
  const Gf16Tables &t = gf16_tables();
  return t.exp[t.log[a] + t.log[b]];
}

inline uint32_t gf16_inv_fast(uint32_t a) {
  if (!a) return 0;
  const Gf16Tables &t = gf16_tables();
  return t.exp[65535 - t.log[a]];
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
bool restore_path_override_bs() {
  static const bool bs = [] {
    const char *v = std::getenv("VDS_EC_RESTORE_PATH");
    return v && std::strcmp(v, "bs") == 0;
  }();
  return bs;
}

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
// bit-sliced kernel's stores (VDS_EC_ENC_TRAILER=0: by a generic launch, A/B).
bool fold_trailers() {
  static const bool on = [] {
    const char *v = std::getenv("VDS_EC_ENC_TRAILER");
    return !(v && v[0] == '0');
  }();
  return on;
}

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
      fa.trailer0 = (fold_trailers() && trailer && k >= 8 && 128 * gpo == T && size % stripe_bytes == 0 &&
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
  const bool trailers_done = fold_trailers() && fast_groups && trailer && k >= 8 && 128 * gpo == T &&
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

// ------------------------------------------------ stream-ordered parameters
// Kernel parameters too large for the kernel arguments (k > 32 inverses, k >
// 64 chunk tables, regenerate coefficients beyond kInlineCoef) ride a
// per-device ring of pinned host + device slots, so the *_device entry points
// enqueue without synchronising.  A slot's bytes are written on the host,
// copied with hipMemcpyAsync on the caller's stream, and an event recorded
// after the kernels that read them; a slot is reused only once its event has
// completed, and hipEventSynchronize blocks only when the ring has wrapped
// round inside the GPU's queue.  (The round-1 version copied a std::vector
// on the caller's stack with hipMemcpyAsync and freed a hipMallocAsync
// buffer in a destructor: the copy could read the vector after it was gone
// -- the likely cause of that round's fault)  Growing a slot
// allocates, which synchronises; slots only grow.
struct ParamSlot {
  uint8_t *h = nullptr, *d = nullptr;
  size_t cap = 0;
  hipEvent_t ev = nullptr;
  hipEvent_t copied = nullptr;  // the host -> device copy on the ring's copy stream
  bool pending = false;  // its event guards the device copy's readers
  bool busy = false;     // acquired, not yet released
  uint64_t stamp = 0;    // when last acquired (ParamRing::clock)
};

struct ParamRing {
  static constexpr int kSlots = 16;
  std::mutex mu;
  std::condition_variable freed;  // a slot was released
  ParamSlot slot[kSlots];
  unsigned next = 0;
  uint64_t clock = 0;
  hipStream_t copy = nullptr;  // the copies run here, beside the caller's kernels
};

ParamRing *param_ring() {
  static std::mutex m;
  static std::vector<ParamRing *> rings;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0) return nullptr;
  std::lock_guard<std::mutex> g(m);
  if ((size_t)dev >= rings.size()) rings.resize(dev + 1, nullptr);
  if (!rings[dev]) rings[dev] = new ParamRing();  // never freed: outlives every caller
  return rings[dev];
}

// `cnt` slots of at least bytes[i] each, whose host sides the caller may
// write (out[i]->h); then param_commit copies one to the device on the
// caller's stream, and param_release after the launches reading it.  A slot
// stays reserved (busy) from acquire to release, so threads sharing the ring
// never write one another's.  The cnt slots are reserved together, under one
// hold of the ring's lock: a caller never holds a slot while it waits for
// another (two batch builders each holding one of the last slots and waiting
// for a second would deadlock), so with cnt <= 2 < kSlots every waiter is
// eventually served.
hipError_t param_acquire_n(int cnt, const size_t *bytes, ParamSlot **out) {
  for (int i = 0; i < cnt; ++i) out[i] = nullptr;
  if (cnt <= 0) return hipSuccess;
  ParamRing *r = param_ring();
  if (!r) return hipErrorNoDevice;
  if (cnt > ParamRing::kSlots / 2) return hipErrorInvalidValue;
  std::unique_lock<std::mutex> g(r->mu);
  hipError_t e = hipSuccess;
  if (!r->copy && (e = hipStreamCreateWithFlags(&r->copy, hipStreamNonBlocking)) != hipSuccess) return e;
  // per slot, first choice: an idle slot already big enough whose readers are
  // done (no allocation, no wait); second, once kAhead slots are big enough
  // but all still being read: the least recently used of them (its event
  // wait below keeps the caller at most kAhead calls ahead of the GPU); else
  // the next idle slot in rotation, grown; with fewer than cnt idle slots,
  // take none and wait for a release.  (Always growing let a caller that
  // plans faster than the GPU runs grow a new slot on nearly every call of a
  // loop -- pinned and device allocations, milliseconds each; always waiting
  // on the one big slot made every call wait for the previous one's kernels,
  // live repair 1020 -> 788 GiB/s.)
  constexpr int kAhead = 3;
  ParamSlot *sp[ParamRing::kSlots / 2] = {};
  bool pending[ParamRing::kSlots / 2] = {};
  for (;;) {
    int got = 0;
    for (; got < cnt; ++got) {
      ParamSlot *p = nullptr;
      for (int i = 0; i < ParamRing::kSlots && !p; ++i) {
        ParamSlot &c = r->slot[(r->next + i) % ParamRing::kSlots];
        if (!c.busy && c.cap >= bytes[got] && (!c.pending || hipEventQuery(c.ev) == hipSuccess)) p = &c;
      }
      if (!p) {
        int big = 0;
        ParamSlot *lru = nullptr;
        for (int i = 0; i < ParamRing::kSlots; ++i) {
          ParamSlot &c = r->slot[i];
          if (c.busy || c.cap < bytes[got]) continue;
          ++big;
          if (!lru || c.stamp < lru->stamp) lru = &c;
        }
        if (big >= kAhead) p = lru;
      }
      for (int i = 0; i < ParamRing::kSlots && !p; ++i) {
        ParamSlot &c = r->slot[r->next++ % ParamRing::kSlots];
        if (!c.busy) p = &c;
      }
      if (!p) break;
      p->busy = true;
      p->stamp = ++r->clock;
      sp[got] = p;
    }
    if (got == cnt) break;
    for (int i = 0; i < got; ++i) sp[i]->busy = false;  // (none held while waiting)
    r->freed.wait(g);
  }
  for (int i = 0; i < cnt; ++i) {  // reserved: from here on only this thread touches them
    pending[i] = sp[i]->pending;
    sp[i]->pending = false;
  }
  g.unlock();  // (the event waits and any allocation run outside the ring's lock)
  for (int i = 0; i < cnt && e == hipSuccess; ++i) {
    ParamSlot &sl = *sp[i];
    if (pending[i]) e = hipEventSynchronize(sl.ev);
    if (e == hipSuccess && !sl.ev) e = hipEventCreateWithFlags(&sl.ev, hipEventDisableTiming);
    if (e == hipSuccess && !sl.copied) e = hipEventCreateWithFlags(&sl.copied, hipEventDisableTiming);
    if (e == hipSuccess && bytes[i] > sl.cap) {
      // grown to a power of two (at least 64 KiB): the batch calls' tables
      // vary a little from call to call, and each growth frees device memory
      // (hipFree waits for the device) -- a few ms inside a repair loop
      size_t cap = 64u << 10;
      while (cap < bytes[i]) cap *= 2;
      if (sl.h) (void)hipHostFree(sl.h);
      if (sl.d) (void)hipFree(sl.d);
      sl.h = sl.d = nullptr;
      sl.cap = 0;
      e = hipHostMalloc(&sl.h, cap, 0);
      if (e == hipSuccess) e = hipMalloc(&sl.d, cap);
      if (e == hipSuccess) sl.cap = cap;
    }
  }
  if (e != hipSuccess) {  // all of them back, unused (nothing was enqueued on them)
    std::lock_guard<std::mutex> g2(r->mu);
    for (int i = 0; i < cnt; ++i) sp[i]->busy = false;
    r->freed.notify_all();
    return e;
  }
  for (int i = 0; i < cnt; ++i) out[i] = sp[i];
  return hipSuccess;
}

hipError_t param_acquire(size_t bytes, ParamSlot **out) { return param_acquire_n(1, &bytes, out); }

// The copy runs on the ring's copy stream and s waits for it, so the copy
// for one call overlaps the kernels of the call before it on s.  (The slot's
// previous readers are done: acquire waited for its event.)
hipError_t param_commit(ParamSlot *sl, size_t bytes, hipStream_t s) {
  if (!bytes) return hipSuccess;
  ParamRing *r = param_ring();
  if (!r || !r->copy) return hipErrorNoDevice;
  hipError_t e = hipMemcpyAsync(sl->d, sl->h, bytes, hipMemcpyHostToDevice, r->copy);
  if (e == hipSuccess) e = hipEventRecord(sl->copied, r->copy);
  if (e == hipSuccess) e = hipStreamWaitEvent(s, sl->copied, 0);
  return e;
}

hipError_t param_release(ParamSlot *sl, hipStream_t s) {
  ParamRing *r = param_ring();
  if (!r || !sl) return hipSuccess;
  std::lock_guard<std::mutex> g(r->mu);
  const hipError_t e = hipEventRecord(sl->ev, s);
  sl->pending = e == hipSuccess;
  sl->busy = false;
  r->freed.notify_all();  // (waiters need one or two slots: each re-checks)
  return e;
}

// Stage blob into a device slot on stream s; *dev receives the device
// address.  Call param_release(slot, s) after the launches reading it.
hipError_t param_stage(const std::vector<uint8_t> &blob, hipStream_t s, const uint8_t **dev, ParamSlot **out) {
  hipError_t e = param_acquire(blob.size(), out);
  if (e != hipSuccess) return e;
  std::memcpy((*out)->h, blob.data(), blob.size());
  *dev = (*out)->d;
  e = param_commit(*out, blob.size(), s);
  if (e != hipSuccess) {
    (void)param_release(*out, s);
    *out = nullptr;
  }
  return e;
}

template <typename T>
size_t blob_append(std::vector<uint8_t> &blob, const T *p, size_t n) {
  const size_t off = (blob.size() + 15) & ~size_t(15);
  blob.resize(off + sizeof(T) * n);
  std::memcpy(blob.data() + off, p, sizeof(T) * n);
  return off;
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

// --------------------------------------------------------- restore core
// Optional layout facts the host path knows: chunks contiguous at a pitch,
// and a device copy of a large inverse already staged.
struct ChunkLayout {
  const uint8_t *base = nullptr;
  uint64_t pitch = 0;
  const uint16_t *matrix_dev = nullptr;
};

int restore_device(unsigned cb, uint32_t k, const uint16_t *nodes, const uint16_t *matrix, const uint8_t *const *chunks,
                   uint64_t chunk_size, uint64_t chunk_stride, uint64_t out_len, uint32_t count,
                   uint8_t *out, uint64_t out_stride, unsigned flags, hipStream_t s,
                   const ChunkLayout &layout = ChunkLayout()) {
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

struct Copy {
  uint8_t *dst;
  const uint8_t *src;
  size_t len;
};

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

template <typename Id>
int check_restore_args(uint32_t k, const Id *nodes, const uint8_t *const *chunks, uint64_t chunk_size) {
  if (k == 0 || !nodes || !chunks) return VDS_EC_EINVAL;
  for (uint32_t j = 0; j < k; ++j)
    if (!chunks[j] && chunk_size) return VDS_EC_EINVAL;
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

// ------------------------------------------------ batched device restore
// Many objects, each with its own survivor set, size and output, as the
// download and repair loops meet them (restore_async gathers the first k
// replicas found PER OBJECT, dht_network_client.cpp:851-901; sync_process
// repairs object by object, sync_process.cpp:313-335).  Objects whose
// survivors lie within the syndrome kernel's points go to ONE launch of
// k_restore_syn in batch mode over every half-tile (kHalfStripes stripes) of
// every such object, the halves of one erased set paired into tiles; objects
// of a compiled k whose survivors lie elsewhere go to ONE launch of its
// runtime-coefficient (RT) mode; the rest fall back to one restore_device /
// regenerate_device call each, on the same stream.  Nothing synchronises.
//
// An erased set's plan (the M x M solve) never changes, so solved plans are
// kept process-wide: a repair loop meets the same few loss patterns again and
// again.  (Bounded: past kMax entries the store is cleared.)
struct SynPlanStore {
  static constexpr size_t kMax = 1u << 16;
  std::mutex mu;
  std::unordered_map<uint64_t, SynBatchPlan> map;
};

SynPlanStore &syn_plan_store() {
  static SynPlanStore *st = new SynPlanStore();  // never freed: outlives every caller
  return *st;
}

// The SMALL plan of survivor set `seen` within A = {0..k+ms-1}: A's ms erased
// points ascending (then the syndrome slots, which stage 1 zeroes too), the
// survivors ascending, R = W_E^{-1} of the ms checks over A as bit masks, and
// nrec = the erased points below k (the rows a restore needs).
bool small_plan_solve(uint32_t k, uint32_t ms, uint64_t seen, SynBatchPlan &p) {
  const uint16_t *W = restore_small_weights(k, ms);
  const uint32_t na = k + ms;
  if (!W || ms > (uint32_t)kSmallMaxM) return false;
  uint32_t e = 0, j = 0, nrec = 0;
  for (uint32_t a = 0; a < na; ++a) {
    if ((seen >> a) & 1u) {
      p.point[j++] = (uint8_t)a;
    } else {
      p.erased[e++] = (uint8_t)a;
      nrec += a < k;
    }
  }
  if (j != k || e != ms) return false;
  for (uint32_t i = ms; i < kMaxFastK / 4; ++i) p.erased[i] = (uint8_t)(na + std::min(i - ms, ms - 1));
  // [W_E | I] -> [I | R] (ms <= 2; W_E[j][i] = v_e e^j at erased point i)
  uint32_t A[kSmallMaxM][2 * kSmallMaxM] = {};
  for (uint32_t r = 0; r < ms; ++r) {
    for (uint32_t i = 0; i < ms; ++i) A[r][i] = W[r * na + p.erased[i]];
    A[r][ms + r] = 1;
  }
  for (uint32_t c = 0; c < ms; ++c) {
    uint32_t piv = c;
    while (piv < ms && A[piv][c] == 0) ++piv;
    if (piv == ms) return false;
    if (piv != c)
      for (uint32_t x = 0; x < 2 * ms; ++x) std::swap(A[c][x], A[piv][x]);
    const uint32_t iv = gf16_inv_fast(A[c][c]);
    for (uint32_t x = 0; x < 2 * ms; ++x) A[c][x] = gf16_mul_fast(A[c][x], iv);
    for (uint32_t r = 0; r < ms; ++r) {
      const uint32_t f = A[r][c];
      if (r == c || f == 0) continue;
      for (uint32_t x = 0; x < 2 * ms; ++x) A[r][x] ^= gf16_mul_fast(f, A[c][x]);
    }
  }
  std::memset(p.small_mask, 0, sizeof p.small_mask);
  for (uint32_t m = 0; m < ms; ++m)
    for (uint32_t jj = 0; jj < ms; ++jj) {
      const uint32_t r = A[m][ms + jj];
      for (uint32_t b = 0; b < 16; ++b) {
        const uint32_t v = gf16_mul_fast(r, 1u << b);
        for (uint32_t i = 0; i < 16; ++i)
          if ((v >> i) & 1u) p.small_mask[m][jj][i] |= (uint16_t)(1u << b);
      }
    }
  p.nrec = nrec;
  return true;
}

// The plan of the erased set ~seen (k, n = k + k/4 compiled; or, ms > 0, the
// SMALL plan over 0..k+ms-1): points and erased points ascending, the solve
// from the store or computed.
bool syn_plan(uint32_t k, uint32_t n, uint64_t seen, SynBatchPlan *out, uint32_t ms = 0) {
  if (ms) n = k + ms;
  const uint64_t key = (~seen & ((1ull << n) - 1)) | ((uint64_t)k << 56) | ((uint64_t)ms << 48);
  SynPlanStore &st = syn_plan_store();
  {
    std::lock_guard<std::mutex> g(st.mu);
    auto it = st.map.find(key);
    if (it != st.map.end()) {
      *out = it->second;
      return true;
    }
  }
  SynBatchPlan p{};
  if (ms) {
    if (!small_plan_solve(k, ms, seen, p)) return false;
  } else {
    SynRestoreArgs sa{};
    uint32_t e = 0, j = 0;
    for (uint32_t a = 0; a < n; ++a) {
      if ((seen >> a) & 1u)
        sa.point[j++] = (uint8_t)a;
      else
        sa.erased[e++] = (uint8_t)a;
    }
    if (j != k || !syn_solve(k, n, sa)) return false;
    std::memcpy(p.erased, sa.erased, sizeof p.erased);
    std::memcpy(p.point, sa.point, sizeof p.point);
    std::memcpy(p.solve_sel, sa.solve_sel, sizeof p.solve_sel);
  }
  std::lock_guard<std::mutex> g(st.mu);
  if (st.map.size() >= SynPlanStore::kMax) st.map.clear();
  st.map.emplace(key, p);
  *out = p;
  return true;
}

// ------------------------------------------------------ host thread pool
// The batch planners' per-object passes run over a few worker threads: the
// live repair loop plans 16,384 objects per call, and one thread took longer
// (3.3 ms) than the kernels it feeds.  Workers start once and wait for a job;
// a caller that finds the pool busy (another thread's batch) runs its parts
// inline.
class HostPool {
 public:
  static HostPool &get() {
    static HostPool *p = new HostPool();  // never freed: detached workers outlive every caller
    return *p;
  }
  // fn(part) for every part in [0, parts), over the workers and the caller.
  template <class F>
  void run(unsigned parts, F &&fn) {
    std::unique_lock<std::mutex> busy(run_mu_, std::try_to_lock);
    if (parts <= 1 || !busy.owns_lock() || nworkers_ == 0) {
      for (unsigned p = 0; p < parts; ++p) fn(p);
      return;
    }
    auto job = std::make_shared<Job>();
    job->fn = [&fn](unsigned p) { fn(p); };
    job->parts = parts;
    {
      std::lock_guard<std::mutex> g(mu_);
      cur_ = job;
      ++gen_;
    }
    cv_.notify_all();
    work(*job);
    std::unique_lock<std::mutex> g(job->m);
    job->cv.wait(g, [&] { return job->done.load() == job->parts; });
  }

 private:
  struct Job {
    std::function<void(unsigned)> fn;
    unsigned parts = 0;
    std::atomic<unsigned> next{0}, done{0};
    std::mutex m;
    std::condition_variable cv;
  };
  HostPool() {
    const unsigned hw = std::thread::hardware_concurrency();
    nworkers_ = hw > 1 ? std::min(hw - 1, 7u) : 0u;
    for (unsigned i = 0; i < nworkers_; ++i) std::thread([this] { loop(); }).detach();
  }
  static void work(Job &j) {
    for (;;) {
      const unsigned p = j.next.fetch_add(1);
      if (p >= j.parts) return;
      j.fn(p);
      if (j.done.fetch_add(1) + 1 == j.parts) {
        std::lock_guard<std::mutex> g(j.m);
        j.cv.notify_all();
      }
    }
  }
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      std::shared_ptr<Job> j;
      {
        std::unique_lock<std::mutex> g(mu_);
        cv_.wait(g, [&] { return gen_ != seen; });
        seen = gen_;
        j = cur_;
      }
      if (j) work(*j);
    }
  }
  std::mutex run_mu_, mu_;
  std::condition_variable cv_;
  std::shared_ptr<Job> cur_;
  uint64_t gen_ = 0;
  unsigned nworkers_ = 0;
};

// fn(o0, o1) over [0, count) in ranges of at least kMinPer objects.
template <class F>
void parallel_objects(uint32_t count, F &&fn) {
  constexpr uint32_t kMinPer = 1024;
  const unsigned parts = std::min<uint32_t>(8, std::max<uint32_t>(1, count / kMinPer));
  HostPool::get().run(parts, [&](unsigned p) {
    fn((uint32_t)((uint64_t)count * p / parts), (uint32_t)((uint64_t)count * (p + 1) / parts));
  });
}

// The first failure of a parallel validation pass: the lowest object's.
struct FirstError {
  std::mutex mu;
  uint32_t obj = UINT32_MAX;
  int rc = VDS_EC_OK;
  void note(uint32_t o, int r) {
    std::lock_guard<std::mutex> g(mu);
    if (o < obj) {
      obj = o;
      rc = r;
    }
  }
};

// Per-object facts of a batch call, from one parallel pass.  Routes:
// kRouteSyn = survivors within the syndrome kernel's points (k_restore_syn
// batch, by erased-set plan); kRouteRt = any other survivors of a compiled k
// with ids < 256 (the RT batch: per-object coefficient rows); kRouteOne =
// the rest (other k, cell arrays), one restore_device / regenerate_device
// per object; kRouteSkip = nothing to write.
enum : uint8_t { kRouteSkip, kRouteSyn, kRouteRt, kRouteOne };
struct BatchObjInfo {
  uint64_t seen;    // survivor ids below 64 as bits
  uint32_t halves;  // half tiles (kHalfStripes stripes) of its output
  uint16_t rows;    // RT rows: restore, its erased points below k; regenerate, its targets
  uint8_t route;
  uint8_t parts;    // RT descriptors (regenerate: rows in groups of at most n - k)
  uint8_t ms;       // kRouteSyn: SMALL ms (1, 2) over 0..k+ms-1, kMsPerm, or 0 = the N = k + k/4 kernel
  uint16_t target;  // kMsPerm: the one target
};

// (BatchObjInfo::ms of the PERM regenerate: survivors exactly 0..k-1, one
// target in k..2k-1)
constexpr uint8_t kMsPerm = 3;

// The SMALL batch kernels (VDS_EC_SMALL=0 routes their objects to the
// N = k + k/4 syndrome kernel instead: A/B).
bool small_enabled() {
  static const bool on = [] {
    const char *v = std::getenv("VDS_EC_SMALL");
    return !(v && v[0] == '0');
  }();
  return on;
}
// The smallest SMALL ms whose points 0..k+ms-1 hold every survivor (maxid), or 0.
uint8_t small_ms_for(uint32_t k, uint32_t maxid) {
  if (!small_enabled()) return 0;
  for (uint32_t ms = 1; ms <= (uint32_t)kSmallMaxM; ++ms)
    if (maxid < k + ms && has_restore_small(k, ms)) return (uint8_t)ms;
  return 0;
}

// The survivor ids of one object: those below 64 as bits, the largest; false
// when two coincide (V_S singular).
inline bool id_set(uint32_t k, const uint16_t *nd, uint64_t *seen, uint32_t *maxid) {
  uint64_t m = 0;
  uint32_t mx = 0;
  bool wide = false;
  for (uint32_t j = 0; j < k; ++j) {
    const uint32_t a = nd[j];
    mx = a > mx ? a : mx;
    if (a >= 64) {
      wide = true;
    } else {
      if ((m >> a) & 1u) return false;
      m |= 1ull << a;
    }
  }
  *seen = m;
  *maxid = mx;
  return !wide || ids_distinct(k, nd);
}

// Host-side builder of one k_restore_syn batch launch, written straight into
// a pinned parameter slot: objs (and the empty object), then tiles, then
// plans.  plan_of() (serial) resolves survivor sets to plans; fill() writes
// descriptor i and may run on several threads for distinct i.
struct SynBatchBuild {
  uint32_t k, n;
  bool regen = false;
  // plans [0, cls_end[0]) are SMALL ms = 1, [cls_end[0], cls_end[1]) ms = 2,
  // [cls_end[1], cls_end[2]) PERM, the rest the N = k + k/4 syndrome
  // kernel's (batch_begin resolves them in that order); each class is one
  // launch over its plans' tiles
  uint32_t cls_end[3] = {0, 0, 0};
  uint32_t perm_idx[64];  // PERM plan of target t (k <= t < 2k), or UINT32_MAX
  ParamSlot *slot = nullptr;
  size_t cap_objs = 0, cap_tiles = 0, cap_plans = 0, o_tiles = 0, o_plans = 0;
  SynBatchObj *objs = nullptr;
  uint32_t nobj = 0;
  std::vector<uint32_t> obj_plan, obj_halves;
  std::vector<SynBatchPlan> plans;
  // survivor set -> plans[]: open addressing, linear probing (a set is a
  // nonzero bitmask; 0 marks a free entry)
  std::vector<uint64_t> hkey;
  std::vector<uint32_t> hval;
  std::vector<uint32_t> hused;  // entries of hkey in use (cleared one by one when the table is reused)
  std::vector<uint64_t> first_, used_;
  std::vector<SynBatchPlan> sorted_;  // (batch_begin's class order; swapped with plans)
  unsigned hshift = 64;

  static size_t up16(size_t x) { return (x + 15) & ~size_t(15); }

  // A builder is per thread and reused (batch_scratch): the vectors keep
  // their capacity, so a steady stream of calls allocates nothing.
  void reset(uint32_t k_, uint32_t n_) {
    k = k_;
    n = n_;
    regen = false;
    cls_end[0] = cls_end[1] = cls_end[2] = 0;
    slot = nullptr;
    cap_objs = cap_tiles = cap_plans = o_tiles = o_plans = 0;
    objs = nullptr;
    nobj = 0;
    plans.clear();
  }

  // The slot bytes for `count` objects of `halves` half tiles; then attach().
  size_t layout(uint32_t count, uint64_t halves) {
    nobj = count;
    cap_objs = (size_t)count + 1;
    cap_tiles = (size_t)((halves + count + 1) / 2 + 1);  // pairs within each plan: <= (halves + plans) / 2
    cap_plans = count;
    o_tiles = up16(cap_objs * sizeof(SynBatchObj));
    o_plans = up16(o_tiles + cap_tiles * sizeof(SynBatchTile));
    return o_plans + cap_plans * sizeof(SynBatchPlan);
  }
  void attach(ParamSlot *sl) {
    slot = sl;
    objs = reinterpret_cast<SynBatchObj *>(slot->h);
    const uint32_t count = nobj;
    obj_plan.assign(count, 0);
    obj_halves.assign(count, 0);
    unsigned bits = 4;
    while ((1ull << bits) < 2ull * count) ++bits;
    if (hkey.size() != (1ull << bits)) {
      hkey.assign(1ull << bits, 0);
      hval.assign(1ull << bits, 0);
    } else {
      for (const uint32_t x : hused) hkey[x] = 0;
    }
    hused.clear();
    hshift = 64 - bits;
    for (uint32_t &x : perm_idx) x = UINT32_MAX;
  }
  // The plan of survivor set `seen` (UINT32_MAX: no solve; not for distinct
  // points); ms > 0: the SMALL plan over 0..k+ms-1 (a set always resolves to
  // the same ms within a call: the route is a function of the set).
  uint32_t plan_of(uint64_t seen, uint32_t ms = 0, uint32_t target = 0) {
    if (ms == kMsPerm) {  // survivors 0..k-1, one target t in k..2k-1: a plan per t
      if (target < k || target >= 2 * k || target >= 64) return UINT32_MAX;
      if (perm_idx[target] != UINT32_MAX) return perm_idx[target];
      SynBatchPlan pl{};
      for (uint32_t j = 0; j < k; ++j) pl.point[j] = (uint8_t)j;
      for (uint32_t i = 0; i < kMaxFastK / 4; ++i) pl.erased[i] = (uint8_t)target;
      pl.cls = 3;  // (kClsPerm)
      perm_idx[target] = (uint32_t)plans.size();
      plans.push_back(pl);
      return perm_idx[target];
    }
    // (keyed by set AND ms: a regenerate's route also depends on its targets,
    // so one set may meet two SMALL sizes in a call)
    const uint64_t hk = seen | ((uint64_t)ms << 56);
    const size_t mask = hkey.size() - 1;
    size_t i = (size_t)((hk * 0x9E3779B97F4A7C15ull) >> hshift);
    while (hkey[i] != 0 && hkey[i] != hk) i = (i + 1) & mask;
    if (hkey[i] == hk) return hval[i];
    SynBatchPlan pl;
    if (!syn_plan(k, n, seen, &pl, ms)) return UINT32_MAX;
    if (ms && regen) pl.nrec = ms;  // (regenerate: every erased point of A is a target candidate)
    pl.cls = ms;                    // (kClsSyn = 0, kClsSmall1 / 2 = ms)
    const uint32_t p = (uint32_t)plans.size();
    plans.push_back(pl);
    hkey[i] = hk;
    hval[i] = p;
    hused.push_back((uint32_t)i);
    return p;
  }
  // Descriptor i: survivors in the plan's point order (ascending ids).
  SynBatchObj &fill(uint32_t i, uint64_t seen, const uint16_t *nd, const uint8_t *const *chunks, uint32_t plan,
                    uint32_t halves) {
    uint8_t pos[64];
    for (uint32_t j = 0; j < k; ++j) pos[nd[j]] = (uint8_t)j;
    SynBatchObj &d = objs[i];
    uint32_t j = 0;
    for (uint64_t b = seen; b; b &= b - 1, ++j) {
      const uint32_t at = pos[__builtin_ctzll(b)];
      d.chunks[j] = chunks[at];
      if (at == 0) d.first = j;
    }
    d.plan = plan;
    obj_plan[i] = plan;
    obj_halves[i] = halves;
    return d;
  }
  // Pair the halves of each plan into tiles, stage and launch (regenerate:
  // the last half of every object also copies its trailer cell, and the tail
  // kernel then writes the reference route's last cell and trailer).
  int launch(bool regen, hipStream_t s) {
    if (nobj == 0) return hip_status(param_release(slot, s));
    const uint32_t empty = nobj;
    std::memset(&objs[empty], 0, sizeof(SynBatchObj));
    std::vector<uint64_t> &first = first_, &used = used_;
    first.assign(plans.size() + 1, 0);  // tile offset of each plan
    used.assign(plans.size(), 0);
    for (uint32_t o = 0; o < nobj; ++o) first[obj_plan[o] + 1] += obj_halves[o];
    for (size_t p = 0; p < plans.size(); ++p) first[p + 1] = first[p] + (first[p + 1] + 1) / 2;
    const uint64_t ntiles = first[plans.size()];
    if (ntiles > cap_tiles || ntiles > 0xFFFFFFFFull) {
      (void)param_release(slot, s);
      return VDS_EC_EINVAL;
    }
    // classes (plans resolved class by class: contiguous plan and tile ranges)
    const uint32_t bound[4] = {cls_end[0], cls_end[1], cls_end[2], (uint32_t)plans.size()};
    int ncls = 0;
    for (int c = 0, q0 = 0; c < 4; q0 = bound[c], ++c) ncls += first[bound[c]] > first[q0];
    // MULTI (ncls > 1): tile t goes to position pos(t), so that each XCD's
    // contiguous eighth of the launch (tile_range) gets every eighth tile --
    // the same mix of classes, whose tiles cost differently
    const uint64_t R = ntiles;
    auto pos = [&](uint64_t t) -> uint64_t {
      if (ncls <= 1) return t;
      const uint64_t r = t % 8;
      return r * (R / 8) + std::min<uint64_t>(r, R % 8) + t / 8;
    };
    SynBatchTile *tiles = reinterpret_cast<SynBatchTile *>(slot->h + o_tiles);
    for (size_t p = 0; p < plans.size(); ++p)
      for (uint64_t t = first[p]; t < first[p + 1]; ++t)
        tiles[pos(t)] = SynBatchTile{{empty, empty}, {0, 0}, (uint32_t)p, 0, 0, 0};
    for (uint32_t o = 0; o < nobj; ++o) {
      const uint32_t p = obj_plan[o];
      for (uint32_t h = 0; h < obj_halves[o]; ++h) {
        const uint64_t i = used[p]++;
        SynBatchTile &t = tiles[pos(first[p] + i / 2)];
        t.obj[i & 1] = o;
        t.stripe0[i & 1] = h * kHalfStripes;
        if (regen && h + 1 == obj_halves[o]) t.trailer |= 1u << (i & 1);
      }
    }
    std::memcpy(slot->h + o_plans, plans.data(), plans.size() * sizeof(SynBatchPlan));
    hipError_t e = param_commit(slot, o_plans + plans.size() * sizeof(SynBatchPlan), s);
    if (e == hipSuccess) {
      SynRestoreArgs sa{};
      sa.objs = reinterpret_cast<const SynBatchObj *>(slot->d);
      sa.plans = reinterpret_cast<const SynBatchPlan *>(slot->d + o_plans);
      const SynBatchTile *dt = reinterpret_cast<const SynBatchTile *>(slot->d + o_tiles);
      // one launch: the MULTI kernel over every class's tiles when there is
      // more than one class (no class waits for another launch's tail), else
      // the class's own kernel
      if (ncls > 1) {
        sa.tiles = dt;
        sa.total_tiles = (uint32_t)ntiles;
        e = launch_restore_multi_batch(k, sa, s, regen);
      }
      uint32_t p0 = 0;
      for (int c = 0; c < 4 && e == hipSuccess && ncls == 1; ++c) {
        const uint64_t t0 = first[p0], t1 = first[bound[c]];
        p0 = bound[c];
        if (t1 == t0) continue;
        sa.tiles = dt + t0;
        sa.total_tiles = (uint32_t)(t1 - t0);
        e = c < 2 ? launch_restore_small_batch(k, (uint32_t)c + 1, sa, s, regen)
            : c == 2 ? (regen ? launch_regen_perm_batch(k, sa, s) : hipErrorInvalidValue)
                     : launch_restore_syn_batch(k, n, sa, s, regen);
      }
      // (reads the same tables, so before the slot is released)
      if (e == hipSuccess && regen) e = launch_regen_tail_batch(k, n - k, sa.objs, sa.plans, nobj, s);
    }
    const hipError_t re = param_release(slot, s);
    if (e == hipSuccess) e = re;
    return hip_status(e);
  }
  void abandon(hipStream_t s) {
    if (slot) (void)param_release(slot, s);  // (nothing was copied from it)
  }
};

// Host-side builder of one RT launch (SynBatchRt, ec_internal.hpp): objects
// whose survivors are outside the syndrome kernel's points, each with its own
// coefficient rows.  Any two objects may share a tile (the kernel reads each
// half's own rows); the tile's row count is the larger of its halves', so
// halves are paired in order of row count.  One pinned slot holds the
// objects, the tiles and -- device side only, written by the coefficient
// kernel -- the rows.  fill() may run on several threads for distinct i.
// RT2 rows for the k = 32 restore's RT objects (VDS_EC_RT2=0: every RT
// object takes the k-slot combination, A/B)
bool rt2_enabled() {
  static const bool on = [] {
    const char *v = std::getenv("VDS_EC_RT2");
    return !(v && v[0] == '0');
  }();
  return on;
}

struct RtBatchBuild {
  uint32_t k, n;
  bool rt2 = false;  // restore: objects that qualify take RT2 rows (SynBatchRt::mode)
  ParamSlot *slot = nullptr;
  size_t cap_tiles = 0, o_tiles = 0, o_coef = 0;
  uint64_t cap_rows = 0;
  SynBatchObj *objs = nullptr;
  uint32_t nobj = 0;
  std::vector<uint32_t> obj_halves, cnt_, order_;

  static size_t up16(size_t x) { return (x + 15) & ~size_t(15); }

  void reset(uint32_t k_, uint32_t n_) {  // (reused per thread, as SynBatchBuild)
    k = k_;
    n = n_;
    rt2 = false;
    slot = nullptr;
    cap_tiles = o_tiles = o_coef = 0;
    cap_rows = 0;
    objs = nullptr;
    nobj = 0;
  }

  // The slot bytes for `count` descriptors of `halves` half tiles and `rows`
  // coefficient rows; then attach().
  size_t layout(uint32_t count, uint64_t halves, uint64_t rows) {
    nobj = count;
    cap_tiles = (size_t)(halves + 1) / 2 + 1;
    cap_rows = rows;
    o_tiles = up16(((size_t)count + 1) * sizeof(SynBatchObj));
    o_coef = up16(o_tiles + cap_tiles * sizeof(SynBatchTile));
    return o_coef + cap_rows * k * sizeof(uint32_t) + 16;
  }
  void attach(ParamSlot *sl) {
    slot = sl;
    objs = reinterpret_cast<SynBatchObj *>(slot->h);
    obj_halves.assign(nobj, 0);
  }
  // Descriptor i of survivors nd (chunks ch; ids < 256), rows at the points
  // rowp[0..ne) stored from row `row0` of the slot's coefficient area: slot a
  // < k holds point a if it survives, else the next survivor beyond k - 1.
  SynBatchObj &fill(uint32_t i, const uint16_t *nd, const uint8_t *const *ch, const uint8_t *rowp, uint32_t ne,
                    uint64_t row0, uint32_t halves) {
    SynBatchObj &d = objs[i];
    int at[kMaxFastK];
    for (uint32_t a = 0; a < k; ++a) at[a] = -1;
    uint32_t extra[kMaxFastK], nx = 0;
    for (uint32_t j = 0; j < k; ++j) {
      if (nd[j] < k)
        at[nd[j]] = (int)j;
      else
        extra[nx++] = j;
    }
    uint64_t borrowed = 0;
    for (uint32_t a = 0, x = 0; a < k; ++a) {
      uint32_t j;
      if (at[a] >= 0) {
        j = (uint32_t)at[a];
      } else {
        j = extra[x++];
        borrowed |= 1ull << a;
      }
      d.chunks[a] = ch[j];
      d.rt.spoint[a] = (uint8_t)nd[j];
      if (j == 0) d.first = a;
    }
    d.rt.borrowed = borrowed;
    d.rt.ne = ne;
    // RT2 (ec_internal.hpp): k = 32, 1..kRt2MaxRows rows, every borrowed
    // survivor in k..2k-1 (the PERM program's coset)
    bool two = rt2 && k == 32 && ne >= 1 && ne <= kRt2MaxRows;
    for (uint32_t a = 0; two && a < k; ++a)
      if (((borrowed >> a) & 1u) && d.rt.spoint[a] >= 2 * k) two = false;
    d.rt.mode = two ? 1u : 0u;
    for (uint32_t m = 0; m < ne; ++m) d.rt.epoint[m] = rowp[m];
    d.rt.coef = reinterpret_cast<const uint32_t *>(slot->d + o_coef + row0 * k * sizeof(uint32_t));
    d.plan = 0;
    obj_halves[i] = halves;
    return d;
  }
  int launch(bool regen, hipStream_t s) {
    if (nobj == 0) return hip_status(param_release(slot, s));
    const uint32_t empty = nobj;
    std::memset(&objs[empty], 0, sizeof(SynBatchObj));
    // objects by (mode, row count) (counting sort: RT2 objects first), halves
    // paired in that order; a tile never pairs the two modes (the kernel's
    // phase 2 is per tile)
    const uint32_t kKeys = kMaxFastK + 1;
    std::vector<uint32_t> &cnt = cnt_, &order = order_;
    cnt.assign(2 * kKeys + 1, 0);
    order.resize(nobj);
    auto key = [&](uint32_t o) { return (objs[o].rt.mode == 1u ? 0u : kKeys) + objs[o].rt.ne; };
    for (uint32_t o = 0; o < nobj; ++o) ++cnt[key(o) + 1];
    for (uint32_t r = 1; r < cnt.size(); ++r) cnt[r] += cnt[r - 1];
    for (uint32_t o = 0; o < nobj; ++o) order[cnt[key(o)]++] = o;
    uint64_t total = 0;
    for (uint32_t o = 0; o < nobj; ++o) total += obj_halves[o];
    if ((total + 2) / 2 > cap_tiles || (total + 2) / 2 > 0xFFFFFFFFull) {  // (+1 half: the mode boundary)
      (void)param_release(slot, s);
      return VDS_EC_EINVAL;
    }
    SynBatchTile *tiles = reinterpret_cast<SynBatchTile *>(slot->h + o_tiles);
    uint64_t i = 0;
    for (const uint32_t o : order) {
      if ((i & 1) && tiles[i / 2].mode != objs[o].rt.mode) ++i;  // (the other mode starts a new tile)
      for (uint32_t h = 0; h < obj_halves[o]; ++h, ++i) {
        SynBatchTile &t = tiles[i / 2];
        if ((i & 1) == 0) t = SynBatchTile{{empty, empty}, {0, 0}, 0, 0, 0, objs[o].rt.mode};
        t.obj[i & 1] = o;
        t.stripe0[i & 1] = h * kHalfStripes;
        t.nm = std::max(t.nm, objs[o].rt.ne);
        if (regen && h + 1 == obj_halves[o]) t.trailer |= 1u << (i & 1);
      }
    }
    const uint64_t ntiles = (i + 1) / 2;
    hipError_t e = param_commit(slot, o_tiles + ntiles * sizeof(SynBatchTile), s);
    const SynBatchObj *dobjs = reinterpret_cast<const SynBatchObj *>(slot->d);
    if (e == hipSuccess) e = launch_rt_coefs(k, dobjs, nobj, s);
    if (e == hipSuccess) {
      SynRestoreArgs sa{};
      sa.objs = dobjs;
      sa.tiles = reinterpret_cast<const SynBatchTile *>(slot->d + o_tiles);
      sa.total_tiles = (uint32_t)ntiles;
      e = launch_restore_rt_batch(k, n, sa, s, regen);
    }
    if (e == hipSuccess && regen) e = launch_regen_tail_rt(k, dobjs, nobj, s);
    const hipError_t re = param_release(slot, s);
    if (e == hipSuccess) e = re;
    return hip_status(e);
  }
  void abandon(hipStream_t s) {
    if (slot) (void)param_release(slot, s);
  }
};

// Prefix indices of the routed objects: syn[o] / rt[o] = descriptor index,
// rtrow[o] = first coefficient row; counts and half / row totals.
struct BatchIndex {
  std::vector<uint32_t> syn, rt;
  std::vector<uint64_t> rtrow;
  uint32_t nsyn = 0, nrt = 0;
  uint64_t syn_halves = 0, rt_halves = 0, rt_rows = 0;
  void build(const std::vector<BatchObjInfo> &info) {
    const uint32_t count = (uint32_t)info.size();
    nsyn = nrt = 0;
    syn_halves = rt_halves = rt_rows = 0;
    syn.assign(count, 0);
    rt.assign(count, 0);
    rtrow.assign(count, 0);
    for (uint32_t o = 0; o < count; ++o) {
      const BatchObjInfo &f = info[o];
      if (f.route == kRouteSyn) {
        syn[o] = nsyn++;
        syn_halves += f.halves;
      } else if (f.route == kRouteRt) {
        rt[o] = nrt;
        rtrow[o] = rt_rows;
        nrt += f.parts;
        rt_halves += (uint64_t)f.parts * f.halves;
        rt_rows += f.rows;
      }
    }
  }
};

// VDS_EC_HOST_TRACE=1: the batched calls print their host phases (us) to
// stderr (planning cost study).
struct HostTrace {
  const char *name;
  bool on;
  std::chrono::steady_clock::time_point t0, last;
  char buf[256];
  int len = 0;
  explicit HostTrace(const char *n) : name(n), on(enabled()) {
    if (on) t0 = last = std::chrono::steady_clock::now();
  }
  static bool enabled() {
    static const bool e = std::getenv("VDS_EC_HOST_TRACE") != nullptr;
    return e;
  }
  void mark(const char *phase) {
    if (!on) return;
    const auto now = std::chrono::steady_clock::now();
    const double us = std::chrono::duration<double, std::micro>(now - last).count();
    last = now;
    if (len < (int)sizeof buf - 40) len += std::snprintf(buf + len, sizeof buf - len, " %s=%.0f", phase, us);
  }
  ~HostTrace() {
    if (!on) return;
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    std::fprintf(stderr, "vds_ec host %s:%s total=%.0f us\n", name, buf, us);
  }
};

// Acquire both builders' slots (together: see param_acquire_n), resolve the
// syndrome objects' plans (serial: the plan store and the per-call hash).
// The batch calls' per-object tables, per thread and reused: at 16K objects
// a call's fresh vectors came from mmap and paid their page faults every
// call (~100 us of the planning at loss 0.25).
struct BatchScratch {
  std::vector<uint64_t> lens;
  std::vector<BatchObjInfo> info;
  std::vector<uint32_t> plan;
  BatchIndex ix;
  SynBatchBuild bb;
  RtBatchBuild rb;
};
BatchScratch &batch_scratch() {
  thread_local BatchScratch sc;
  return sc;
}

int batch_begin(const std::vector<BatchObjInfo> &info, const BatchIndex &ix, SynBatchBuild &bb, RtBatchBuild &rb,
                std::vector<uint32_t> &plan, hipStream_t s, HostTrace *ht) {
  size_t bytes[2];
  ParamSlot *sl[2] = {};
  int nb = 0;
  if (ix.nsyn) bytes[nb++] = bb.layout(ix.nsyn, ix.syn_halves);
  if (ix.nrt) bytes[nb++] = rb.layout(ix.nrt, ix.rt_halves, ix.rt_rows);
  const hipError_t e = param_acquire_n(nb, bytes, sl);
  if (e != hipSuccess) return hip_status(e);
  if (ht) ht->mark("acquire");
  nb = 0;
  if (ix.nsyn) bb.attach(sl[nb++]);
  if (ix.nrt) rb.attach(sl[nb++]);
  if (ht) ht->mark("attach");
  if (ix.nsyn) {
    // One pass resolves every object's plan (first seen, first numbered);
    // then the plans are renumbered class by class -- SMALL ms = 1, ms = 2,
    // PERM, the N = k + k/4 kernel's (SynBatchBuild::cls_end) -- so each
    // class's tiles are contiguous.  (Four passes, one per class, cost ~30 us
    // more at 16K objects; finding the distinct sets in parallel and
    // resolving each once measured slower still: 110 -> 245 us.)
    const uint32_t count = (uint32_t)info.size();
    plan.assign(count, 0);
    for (uint32_t o = 0; o < count; ++o)
      if (info[o].route == kRouteSyn &&
          (plan[o] = bb.plan_of(info[o].seen, info[o].ms, info[o].target)) == UINT32_MAX) {
        bb.abandon(s);
        if (ix.nrt) rb.abandon(s);
        return VDS_EC_ESINGULAR;
      }
    if (ht) ht->mark("plans");
    const size_t np = bb.plans.size();
    auto rank = [](uint32_t cls) { return cls == 1 ? 0 : cls == 2 ? 1 : cls == 3 ? 2 : 3; };
    std::vector<uint32_t> order(np), remap(np);
    uint32_t cnt[5] = {0, 0, 0, 0, 0};
    for (size_t p = 0; p < np; ++p) ++cnt[rank(bb.plans[p].cls) + 1];
    for (int c = 1; c < 5; ++c) cnt[c] += cnt[c - 1];
    for (int c = 0; c < 3; ++c) bb.cls_end[c] = cnt[c + 1];
    for (size_t p = 0; p < np; ++p) {
      const uint32_t q = cnt[rank(bb.plans[p].cls)]++;
      order[q] = (uint32_t)p;
      remap[p] = q;
    }
    std::vector<SynBatchPlan> &sorted = bb.sorted_;
    sorted.resize(np);
    for (size_t q = 0; q < np; ++q) sorted[q] = bb.plans[order[q]];
    bb.plans.swap(sorted);
    for (uint32_t o = 0; o < count; ++o)
      if (info[o].route == kRouteSyn) plan[o] = remap[plan[o]];
  }
  return VDS_EC_OK;
}

int batch_launch(const BatchIndex &ix, SynBatchBuild &bb, RtBatchBuild &rb, bool regen, hipStream_t s) {
  int rc = ix.nsyn ? bb.launch(regen, s) : VDS_EC_OK;
  if (rc) {
    if (ix.nrt) rb.abandon(s);
    return rc;
  }
  return ix.nrt ? rb.launch(regen, s) : VDS_EC_OK;
}

int restore_batch_device(uint32_t k, uint32_t count, const uint16_t *nodes, const uint8_t *const *chunks,
                         const uint64_t *chunk_sizes, const uint16_t *paddings, uint8_t *const *outs, unsigned flags,
                         hipStream_t s) {
  if (k == 0 || (count && (!nodes || !chunks || !chunk_sizes || !paddings || !outs))) return VDS_EC_EINVAL;
  if (count == 0) return VDS_EC_OK;
  const uint32_t n = k + k / 4;
  const bool batch_ok = !(flags & VDS_EC_F_CELLS) && k % 4 == 0 && has_restore_syn(k, n);
  const bool syn = batch_ok && !restore_path_override_bs();
  HostTrace ht("restore_batch");
  // pass 1 (parallel): every object validated before anything is enqueued,
  // its route and sizes
  BatchScratch &sc = batch_scratch();
  std::vector<uint64_t> &lens = sc.lens;
  std::vector<BatchObjInfo> &info = sc.info;
  lens.assign(count, 0);
  info.assign(count, BatchObjInfo{});
  FirstError err;
  parallel_objects(count, [&](uint32_t o0, uint32_t o1) {
    for (uint32_t o = o0; o < o1; ++o) {
      const uint16_t *nd = nodes + (uint64_t)o * k;
      int rc = check_restore_args(k, nd, chunks + (uint64_t)o * k, chunk_sizes[o]);
      bool ok = true;
      if (!rc) lens[o] = restored_len(2, k, chunk_sizes[o], paddings[o], flags, &ok);
      if (!rc && !ok) rc = VDS_EC_ERESTORE;
      if (!rc && lens[o] && !outs[o]) rc = VDS_EC_EINVAL;
      BatchObjInfo f{};
      uint32_t maxid = 0;
      if (!rc && lens[o] && !id_set(k, nd, &f.seen, &maxid)) rc = VDS_EC_ESINGULAR;
      if (rc) {
        err.note(o, rc);
        return;
      }
      const uint64_t need = (lens[o] + 2ull * k - 1) / (2ull * k);  // stripes that produce output
      f.halves = (uint32_t)std::min<uint64_t>((need + kHalfStripes - 1) / kHalfStripes, UINT32_MAX);
      // (SynBatchTile::stripe0 is 32-bit: objects past 2^32 stripes take the per-object path)
      const bool fits = need <= 0xFFFFFFFFull - kHalfStripes;
      if (need == 0) {
        f.route = kRouteSkip;
      } else if (syn && fits && maxid < n) {
        f.route = kRouteSyn;
        f.ms = small_ms_for(k, maxid);
      } else if (batch_ok && fits && maxid < 256) {
        f.route = kRouteRt;
        f.parts = 1;
        f.rows = (uint16_t)(k - __builtin_popcountll(f.seen & ((1ull << k) - 1)));  // erased points below k
      } else {
        f.route = kRouteOne;
      }
      info[o] = f;
    }
  });
  if (err.rc) return err.rc;
  int rc = device_ready();
  if (rc) return rc;
  ht.mark("pass1");
  BatchIndex &ix = sc.ix;
  ix.build(info);
  SynBatchBuild &bb = sc.bb;
  bb.reset(k, n);
  RtBatchBuild &rb = sc.rb;
  rb.reset(k, n);
  rb.rt2 = rt2_enabled();  // (restore only; RtBatchBuild::fill decides per object)
  std::vector<uint32_t> &plan = sc.plan;
  ht.mark("index");
  if ((rc = batch_begin(info, ix, bb, rb, plan, s, &ht))) return rc;
  ht.mark("begin");
  // pass 2 (parallel): the descriptors
  parallel_objects(count, [&](uint32_t o0, uint32_t o1) {
    for (uint32_t o = o0; o < o1; ++o) {
      const BatchObjInfo &f = info[o];
      const uint16_t *nd = nodes + (uint64_t)o * k;
      const uint8_t *const *ch = chunks + (uint64_t)o * k;
      SynBatchObj *d;
      if (f.route == kRouteSyn) {
        d = &bb.fill(ix.syn[o], f.seen, nd, ch, plan[o], f.halves);
      } else if (f.route == kRouteRt) {
        uint8_t rowp[kMaxFastK];
        uint32_t ne = 0;
        for (uint64_t b = ~f.seen & ((1ull << k) - 1); b; b &= b - 1) rowp[ne++] = (uint8_t)__builtin_ctzll(b);
        d = &rb.fill(ix.rt[o], nd, ch, rowp, ne, ix.rtrow[o], f.halves);
      } else {
        continue;
      }
      d->out = outs[o];
      std::memset(d->regen, 0, sizeof d->regen);
      d->out_len = lens[o];
      d->chunk_len = chunk_sizes[o];
    }
  });
  ht.mark("pass2");
  if ((rc = batch_launch(ix, bb, rb, false, s))) return rc;
  ht.mark("launch");
  for (uint32_t o = 0; o < count; ++o) {
    if (info[o].route != kRouteOne) continue;
    std::vector<uint16_t> m((size_t)k * k);
    rc = inverse16(k, nodes + (uint64_t)o * k, m.data());
    if (rc) return rc;
    rc = restore_device(2, k, nodes + (uint64_t)o * k, m.data(), chunks + (uint64_t)o * k, chunk_sizes[o], 0, lens[o], 1,
                        outs[o], 0, flags, s);
    if (rc) return rc;
  }
  return VDS_EC_OK;
}

int regenerate_batch_device(uint32_t k, uint32_t count, const uint16_t *nodes, const uint8_t *const *chunks,
                            const uint64_t *chunk_sizes, uint32_t nt, const uint16_t *targets, uint8_t *const *outs,
                            hipStream_t s) {
  if (k == 0 || (count && (!nodes || !chunks || !chunk_sizes || (nt && (!targets || !outs))))) return VDS_EC_EINVAL;
  if (count == 0 || nt == 0) return VDS_EC_OK;
  // Routes as restore_batch_device's; the syndrome kernel only when every
  // target is one of the object's erased points (each at most once: wave w
  // recovers the w-th erased point, ascending); an RT object carries at most
  // n - k rows, so one with more targets becomes several descriptors, each
  // re-reading its survivors.
  const uint32_t n = k + k / 4, R = n - k;
  const bool batch_ok = k % 4 == 0 && has_restore_syn(k, n);
  const bool syn = batch_ok && !restore_path_override_bs();
  HostTrace ht("regenerate_batch");
  BatchScratch &sc = batch_scratch();
  std::vector<BatchObjInfo> &info = sc.info;
  info.assign(count, BatchObjInfo{});
  FirstError err;
  parallel_objects(count, [&](uint32_t o0, uint32_t o1) {
    for (uint32_t o = o0; o < o1; ++o) {
      const uint16_t *nd = nodes + (uint64_t)o * k;
      const uint16_t *tg = targets + (uint64_t)o * nt;
      int rc = VDS_EC_OK;
      if (chunk_sizes[o] < 2 || (chunk_sizes[o] - 2) % 2) rc = VDS_EC_EINVAL;  // cells + BE16 trailer
      for (uint32_t j = 0; !rc && j < k; ++j)
        if (!chunks[(uint64_t)o * k + j]) rc = VDS_EC_EINVAL;
      for (uint32_t i = 0; !rc && i < nt; ++i)
        if (!outs[(uint64_t)o * nt + i]) rc = VDS_EC_EINVAL;
      BatchObjInfo f{};
      uint32_t maxid = 0;
      if (!rc && !id_set(k, nd, &f.seen, &maxid)) rc = VDS_EC_ESINGULAR;
      if (rc) {
        err.note(o, rc);
        return;
      }
      const uint64_t T = (chunk_sizes[o] - 2) / 2;
      f.halves = (uint32_t)std::min<uint64_t>(T ? (T + kHalfStripes - 1) / kHalfStripes : 1, UINT32_MAX);
      const bool fits = T <= 0xFFFFFFFFull - kHalfStripes;
      bool ok = syn && fits && maxid < n;
      const uint64_t erased = ~f.seen & ((1ull << n) - 1);
      uint64_t hit = 0;
      uint32_t tmax = 0;
      for (uint32_t i = 0; i < nt; ++i) {
        const uint32_t t = tg[i];
        tmax = t > tmax ? t : tmax;
        if (ok) {
          ok = t < n && ((erased >> t) & 1u) && !((hit >> t) & 1u);
          if (ok) hit |= 1ull << t;
        }
      }
      if (small_enabled() && fits && nt == 1 && (k == 16 || k == 32) && maxid < k && tg[0] >= k && tg[0] < 2 * k) {
        f.route = kRouteSyn;  // survivors exactly 0..k-1 (k distinct ids below k), one target in k..2k-1
        f.ms = kMsPerm;
        f.target = tg[0];
      } else if (ok) {
        f.route = kRouteSyn;
        f.ms = small_ms_for(k, std::max(maxid, tmax));  // (every target an erased point of 0..k+ms-1)
      } else if (batch_ok && fits && maxid < 256 && tmax < 256) {
        f.route = kRouteRt;
        f.parts = (uint8_t)((nt + R - 1) / R);
        f.rows = (uint16_t)nt;
      } else {
        f.route = kRouteOne;
      }
      info[o] = f;
    }
  });
  if (err.rc) return err.rc;
  int rc = device_ready();
  if (rc) return rc;
  for (const BatchObjInfo &f : info)  // (RT descriptors per object: nt / (n - k) rounded up, < 256)
    if (f.route == kRouteRt && (uint32_t)f.parts * R < nt) return VDS_EC_EINVAL;
  ht.mark("pass1");
  BatchIndex &ix = sc.ix;
  ix.build(info);
  SynBatchBuild &bb = sc.bb;
  bb.reset(k, n);
  bb.regen = true;
  RtBatchBuild &rb = sc.rb;
  rb.reset(k, n);
  std::vector<uint32_t> &plan = sc.plan;
  ht.mark("index");
  if ((rc = batch_begin(info, ix, bb, rb, plan, s, &ht))) return rc;
  ht.mark("begin");
  parallel_objects(count, [&](uint32_t o0, uint32_t o1) {
    for (uint32_t o = o0; o < o1; ++o) {
      const BatchObjInfo &f = info[o];
      const uint16_t *nd = nodes + (uint64_t)o * k;
      const uint8_t *const *ch = chunks + (uint64_t)o * k;
      const uint16_t *tg = targets + (uint64_t)o * nt;
      uint8_t *const *os = outs + (uint64_t)o * nt;
      if (f.route == kRouteSyn) {
        SynBatchObj &d = bb.fill(ix.syn[o], f.seen, nd, ch, plan[o], f.halves);
        std::memset(d.regen, 0, sizeof d.regen);
        if (f.ms == kMsPerm) {
          d.regen[0] = os[0];  // (the plan's erased[0] is the target)
        } else {
          const uint32_t np = f.ms ? k + f.ms : n;  // the plan's points
          const uint64_t erased = ~f.seen & ((1ull << np) - 1);
          for (uint32_t i = 0; i < nt; ++i)
            d.regen[__builtin_popcountll(erased & ((1ull << tg[i]) - 1))] = os[i];
        }
        d.out = nullptr;
        d.out_len = 0;
        d.chunk_len = chunk_sizes[o];
      } else if (f.route == kRouteRt) {
        for (uint32_t part = 0, i0 = 0; part < f.parts; ++part, i0 += R) {
          const uint32_t cnt = std::min(R, nt - i0);
          uint8_t rowp[kMaxFastK / 4];
          for (uint32_t i = 0; i < cnt; ++i) rowp[i] = (uint8_t)tg[i0 + i];
          SynBatchObj &d = rb.fill(ix.rt[o] + part, nd, ch, rowp, cnt, ix.rtrow[o] + i0, f.halves);
          std::memset(d.regen, 0, sizeof d.regen);
          for (uint32_t i = 0; i < cnt; ++i) d.regen[i] = os[i0 + i];
          d.out = nullptr;
          d.out_len = 0;
          d.chunk_len = chunk_sizes[o];
        }
      }
    }
  });
  ht.mark("pass2");
  if ((rc = batch_launch(ix, bb, rb, true, s))) return rc;
  ht.mark("launch");
  for (uint32_t o = 0; o < count; ++o) {
    if (info[o].route != kRouteOne) continue;
    rc = regenerate_device(2, k, nodes + (uint64_t)o * k, chunks + (uint64_t)o * k, chunk_sizes[o], 0, 1,
                           targets + (uint64_t)o * nt, nt, outs + (uint64_t)o * nt, 0, s);
    if (rc) return rc;
  }
  return VDS_EC_OK;
}

// ---------------------------------------------- caller-pinned host memory
// Buffers the caller allocated with vds_ec_host_alloc or registered with
// vds_ec_host_register (page-locked, mapped, portable across devices).  A
// host batch whose group of objects (or replicas) lies in one such range as
// one contiguous slab skips the staging copies: the H2D DMA reads the
// caller's bytes, and the push kernel writes the results straight into the
// caller's pages.  Lookups are per group, not per object.
constexpr int kPinnedMaxDev = 64;
struct PinnedRange {
  uint64_t bytes;
  bool owned;  // vds_ec_host_alloc (freed by vds_ec_host_free) vs registered
  // the device address of the range's first byte, per device: resolved on
  // each device the first time a host batch there uses the range (a mapped
  // host range need not have the same address on every device)
  uint8_t *dev[kPinnedMaxDev] = {};
};
struct PinnedRegistry {
  std::mutex mu;
  std::map<uintptr_t, PinnedRange> ranges;  // by start address
};
PinnedRegistry &pinned_registry() {
  static PinnedRegistry *r = new PinnedRegistry();  // never freed: outlives every caller
  return *r;
}
// The address, on the calling thread's current device, of host bytes
// [p, p + len) when they lie in one pinned range, else nullptr (then the
// caller stages the bytes as for pageable memory).
uint8_t *pinned_device_ptr(const void *p, uint64_t len) {
  if (!p) return nullptr;
  PinnedRegistry &r = pinned_registry();
  std::lock_guard<std::mutex> g(r.mu);
  if (r.ranges.empty()) return nullptr;
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  auto it = r.ranges.upper_bound(a);
  if (it == r.ranges.begin()) return nullptr;
  --it;
  if (a + len > it->first + it->second.bytes) return nullptr;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kPinnedMaxDev) return nullptr;
  uint8_t *&d = it->second.dev[dev];
  if (!d) {
    void *q = nullptr;
    if (hipHostGetDevicePointer(&q, reinterpret_cast<void *>(it->first), 0) != hipSuccess || !q) return nullptr;
    d = static_cast<uint8_t *>(q);
  }
  return d + (a - it->first);
}

// The D2H of a pinned slab by the push kernel (default) or by the copy
// engine (VDS_EC_PIN_D2H=dma, A/B).
bool pinned_d2h_dma() {
  static const bool dma = [] {
    const char *v = std::getenv("VDS_EC_PIN_D2H");
    return v && std::strcmp(v, "dma") == 0;
  }();
  return dma;
}

// ------------------------------------------------- multi-GPU host batch
// Host-resident objects, many per launch: runs of consecutive objects of one
// size are packed into groups of up to kGroupBytes of input, and the groups
// go round-robin to the devices (one host thread each).  Per device a ring of
// kSlots pinned slots keeps the host copies of one group (gathered into, or
// scattered out of, pinned staging by a few threads), the DMA of another and
// the kernels of a third in flight together.  Staging is kept across calls:
// hipHostMalloc of hundreds of MiB costs more than the encode it feeds.
// The bound is PCIe: input + every replica cross it, and on the MI355X box
// its two directions together carry about one direction's 57 GB/s
// (tools/ubench/pcie.py).
constexpr uint64_t kGroupBytes = 64ull << 20;

struct BatchSlot {
  hipStream_t stream = nullptr;
  uint8_t *h_in = nullptr, *h_out = nullptr, *d_in = nullptr, *d_out = nullptr;
  uint8_t *h_out_dev = nullptr;  // device view of the mapped h_out
  size_t in_cap = 0, out_cap = 0;
  bool busy = false;
  std::vector<Copy> out_parts;  // the scatter of h_out once the stream is done
  size_t d_in_cap = 0, d_out_cap = 0;
  // pinned host staging of at least in_b / out_b bytes (1 when the group's
  // caller slabs are pinned and nothing is staged)
  int reserve(size_t in_b, size_t out_b) {
    if (!stream && hipStreamCreateWithFlags(&stream, hipStreamNonBlocking) != hipSuccess) return VDS_EC_ENODEV;
    in_b = std::max<size_t>(in_b, 1);
    out_b = std::max<size_t>(out_b, 1);
    if (in_b > in_cap) {
      if (h_in) (void)hipHostFree(h_in);
      h_in = nullptr;
      in_cap = 0;
      if (hipHostMalloc(&h_in, in_b, 0) != hipSuccess) return VDS_EC_ENOMEM;
      in_cap = in_b;
    }
    if (out_b > out_cap) {
      if (h_out) (void)hipHostFree(h_out);
      h_out = h_out_dev = nullptr;
      out_cap = 0;
      if (hipHostMalloc(&h_out, out_b, hipHostMallocMapped) != hipSuccess ||
          hipHostGetDevicePointer(reinterpret_cast<void **>(&h_out_dev), h_out, 0) != hipSuccess)
        return VDS_EC_ENOMEM;
      out_cap = out_b;
    }
    return VDS_EC_OK;
  }
  // device buffers of at least in_b / out_b bytes
  int reserve_dev(size_t in_b, size_t out_b) {
    in_b = std::max<size_t>(in_b, 1);
    out_b = std::max<size_t>(out_b, 1);
    if (in_b > d_in_cap) {
      if (d_in) (void)hipFree(d_in);
      d_in = nullptr;
      d_in_cap = 0;
      if (hipMalloc(&d_in, in_b) != hipSuccess) return VDS_EC_ENOMEM;
      d_in_cap = in_b;
    }
    if (out_b > d_out_cap) {
      if (d_out) (void)hipFree(d_out);
      d_out = nullptr;
      d_out_cap = 0;
      if (hipMalloc(&d_out, out_b) != hipSuccess) return VDS_EC_ENOMEM;
      d_out_cap = out_b;
    }
    return VDS_EC_OK;
  }
  // d_out[0, bytes) -> h_out by a kernel on the slot's stream: the copy
  // engines would serialise it with the next group's H2D (see launch_push)
  int push_out(uint64_t bytes) { return hip_status(launch_push(h_out_dev, d_out, bytes, stream)); }
  // wait for the slot's group and copy its results out
  int drain() {
    if (!busy) return VDS_EC_OK;
    busy = false;
    hipError_t e = hipStreamSynchronize(stream);
    if (e != hipSuccess) return hip_status(e);
    parallel_copy(out_parts);
    out_parts.clear();
    return VDS_EC_OK;
  }
};

struct BatchRing {
  static constexpr int kSlots = 3;
  std::mutex mu;  // one batch call per device at a time
  BatchSlot slot[kSlots];
};

BatchRing *batch_ring(int dev) {
  static std::mutex m;
  static std::vector<BatchRing *> rings;
  std::lock_guard<std::mutex> g(m);
  if (dev < 0) return nullptr;
  if ((size_t)dev >= rings.size()) rings.resize(dev + 1, nullptr);
  if (!rings[dev]) rings[dev] = new BatchRing();  // never freed: outlives every caller
  return rings[dev];
}

struct Group {
  uint32_t o0, cnt;
};

// Runs of consecutive objects with equal key(o), at most kGroupBytes of
// bytes(o) each (and at least one object).
template <typename Key, typename Bytes>
std::vector<Group> make_groups(uint32_t count, Key key, Bytes bytes) {
  std::vector<Group> g;
  uint64_t acc = 0;
  for (uint32_t o = 0; o < count; ++o) {
    const uint64_t b = bytes(o);
    if (!g.empty() && key(o) == key(g.back().o0) && acc + b <= kGroupBytes) {
      ++g.back().cnt;
      acc += b;
    } else {
      g.push_back({o, 1});
      acc = b;
    }
  }
  return g;
}

// Run enqueue(slot, group) for the groups of each device on its ring; a slot
// is drained before it is refilled and every slot at the end.
template <typename Enqueue>
int run_host_batch(const std::vector<Group> &groups, int ndev, Enqueue enqueue) {
  std::atomic<int> status{VDS_EC_OK};
  auto worker = [&](int dev) {
    if (hipSetDevice(dev) != hipSuccess) {
      status = VDS_EC_ENODEV;
      return;
    }
    BatchRing *ring = batch_ring(dev);
    if (!ring) {
      status = VDS_EC_ENODEV;
      return;
    }
    std::lock_guard<std::mutex> hold(ring->mu);
    int si = 0;
    for (size_t g = dev; g < groups.size() && status.load() == VDS_EC_OK; g += ndev) {
      BatchSlot &s = ring->slot[si];
      si = (si + 1) % BatchRing::kSlots;
      int rc = s.drain();
      if (rc == VDS_EC_OK) {
        rc = enqueue(s, groups[g]);
        s.busy = true;  // (on failure too: whatever was enqueued is waited for, nothing copied out)
        if (rc) s.out_parts.clear();
      }
      if (rc) {
        status = rc;
        break;
      }
    }
    for (auto &s : ring->slot) {
      const int rc = s.drain();
      if (rc && status.load() == VDS_EC_OK) status = rc;
      s.out_parts.clear();
    }
  };
  std::vector<std::thread> threads;
  for (int d = 0; d < ndev && (size_t)d < groups.size(); ++d) threads.emplace_back(worker, d);
  for (auto &t : threads) t.join();
  return status.load();
}

int batch_devices(int max_devices, int *ndev) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return VDS_EC_ENODEV;
  if (max_devices > 0 && max_devices < n) n = max_devices;
  *ndev = n;
  return VDS_EC_OK;
}

int encode_host_batch(uint32_t k, const uint16_t *replicas, uint32_t n, const uint8_t *const *objs,
                      const uint64_t *sizes, uint32_t count, uint8_t *const *outs, unsigned flags, int max_devices) {
  if (k == 0 || (count && (!objs || !sizes || !outs)) || (n && !replicas)) return VDS_EC_EINVAL;
  int ndev = 0;
  int rc = batch_devices(max_devices, &ndev);
  if (rc) return rc;
  if (count == 0 || n == 0) return VDS_EC_OK;
  for (uint32_t o = 0; o < count; ++o) {
    if (sizes[o] && !objs[o]) return VDS_EC_EINVAL;
    for (uint32_t i = 0; i < n; ++i)
      if (!outs[(uint64_t)o * n + i]) return VDS_EC_EINVAL;
  }
  const std::vector<Group> groups = make_groups(
      count, [&](uint32_t o) { return sizes[o]; },
      [&](uint32_t o) { return sizes[o] + (uint64_t)n * vds_ec_replica_size(2, k, sizes[o], flags); });
  return run_host_batch(groups, ndev, [&](BatchSlot &s, const Group &g) -> int {
    const uint64_t size = sizes[g.o0], L = vds_ec_replica_size(2, k, size, flags), m = g.cnt;
    // caller-pinned slabs (vds_ec_host_alloc / _register): no staging copies
    bool in_slab = size > 0, out_slab = L > 0;
    for (uint64_t o = 1; o < m && in_slab; ++o) in_slab = objs[g.o0 + o] == objs[g.o0] + o * size;
    uint8_t *const out0 = outs[(uint64_t)g.o0 * n];
    for (uint64_t i = 1; i < m * n && out_slab; ++i) out_slab = outs[(uint64_t)g.o0 * n + i] == out0 + i * L;
    const bool in_direct = in_slab && pinned_device_ptr(objs[g.o0], m * size);
    uint8_t *const out_dev = out_slab ? pinned_device_ptr(out0, m * n * L) : nullptr;
    int rc = s.reserve(in_direct ? 1 : m * size, out_dev ? 1 : m * n * L);
    if (rc) return rc;
    if (!in_direct) {
      std::vector<Copy> in(m);
      for (uint64_t o = 0; o < m; ++o) in[o] = {s.h_in + o * size, objs[g.o0 + o], size};
      parallel_copy(in);
    }
    // (the device input buffer, in the staging slot too: sized for the group)
    rc = s.reserve_dev(m * size, m * n * L);
    if (rc) return rc;
    hipError_t e = size ? hipMemcpyAsync(s.d_in, in_direct ? objs[g.o0] : s.h_in, m * size, hipMemcpyHostToDevice,
                                         s.stream)
                        : hipSuccess;
    if (e != hipSuccess) return hip_status(e);
    // replica i of the group's object o at d_out + (o n + i) L: the order of
    // outs[], so a caller's slab of replicas is one copy out
    std::vector<uint8_t *> douts(n);
    for (uint32_t i = 0; i < n; ++i) douts[i] = s.d_out + (uint64_t)i * L;
    rc = encode_device(2, k, replicas, n, s.d_in, size, size, (uint32_t)m, douts.data(), n * L, flags, s.stream);
    if (rc) return rc;
    if (out_dev) {  // straight into the caller's pinned slab
      s.out_parts.clear();
      return hip_status(((reinterpret_cast<uintptr_t>(out_dev) & 15u) == 0 && !pinned_d2h_dma())
                            ? launch_push(out_dev, s.d_out, m * n * L, s.stream)
                            : hipMemcpyAsync(out0, s.d_out, m * n * L, hipMemcpyDeviceToHost, s.stream));
    }
    if ((rc = s.push_out(m * n * L))) return rc;
    s.out_parts.resize(m * n);
    for (uint64_t o = 0; o < m; ++o)
      for (uint32_t i = 0; i < n; ++i)
        s.out_parts[o * n + i] = {outs[(g.o0 + o) * n + i], s.h_out + (o * n + i) * L, L};
    return VDS_EC_OK;
  });
}

int restore_host_batch(uint32_t k, const uint16_t *nodes, const uint8_t *const *chunks, const uint64_t *chunk_sizes,
                       uint32_t count, uint8_t *const *outs, uint64_t *out_sizes, unsigned flags, int max_devices) {
  if (k == 0 || (count && (!nodes || !chunks || !chunk_sizes || !outs || !out_sizes))) return VDS_EC_EINVAL;
  int ndev = 0;
  int rc = batch_devices(max_devices, &ndev);
  if (rc) return rc;
  if (count == 0) return VDS_EC_OK;
  // Validate every object before any transfer, as restore16_host does per
  // object (chunk.h:415-419 lengths; the trailer of the first chunk), so a
  // bad object fails the call without partial output.
  const bool cells = (flags & VDS_EC_F_CELLS) != 0;
  std::vector<uint64_t> lens(count);
  std::vector<uint16_t> pads(count);
  for (uint32_t o = 0; o < count; ++o) {
    const uint64_t cs = chunk_sizes[o];
    rc = check_restore_args(k, nodes + (uint64_t)o * k, chunks + (uint64_t)o * k, cs);
    if (rc) return rc;
    const uint8_t *c0 = chunks[(uint64_t)o * k];
    pads[o] = (cells || cs < 2) ? 0 : (uint16_t)((c0[cs - 2] << 8) | c0[cs - 1]);
    bool ok = true;
    lens[o] = restored_len(2, k, cs, pads[o], flags, &ok);
    if (!ok) return VDS_EC_ERESTORE;
    if (lens[o] > out_sizes[o] || (lens[o] && !outs[o])) return VDS_EC_EINVAL;
    if (lens[o] && !ids_distinct(k, nodes + (uint64_t)o * k)) return VDS_EC_ESINGULAR;
  }
  // the most a group's object can restore to: (chunk_size - 2) k plus a
  // corrupt trailer's excess, bounded by restored_len's own checks
  const std::vector<Group> groups = make_groups(
      count, [&](uint32_t o) { return chunk_sizes[o]; }, [&](uint32_t o) { return chunk_sizes[o] * (k + 1); });
  rc = run_host_batch(groups, ndev, [&](BatchSlot &s, const Group &g) -> int {
    const uint64_t cs = chunk_sizes[g.o0], m = g.cnt;
    uint64_t cap = 1;
    for (uint64_t o = 0; o < m; ++o) cap = std::max(cap, lens[g.o0 + o]);
    // caller-pinned slabs: the survivors as [objects][k][cs], the outputs
    // back to back at one length
    const uint8_t *const c0 = chunks[(uint64_t)g.o0 * k];
    bool in_slab = cs > 0;
    for (uint64_t i = 1; i < m * k && in_slab; ++i) in_slab = chunks[(uint64_t)g.o0 * k + i] == c0 + i * cs;
    const bool in_direct = in_slab && pinned_device_ptr(c0, m * k * cs);
    bool out_slab = cap > 0;
    for (uint64_t o = 0; o < m && out_slab; ++o)
      out_slab = lens[g.o0 + o] == cap && outs[g.o0 + o] == outs[g.o0] + o * cap;
    uint8_t *const out_dev = out_slab ? pinned_device_ptr(outs[g.o0], m * cap) : nullptr;
    int rc = s.reserve(in_direct ? 1 : m * k * cs, out_dev ? 1 : m * cap);
    if (rc) return rc;
    rc = s.reserve_dev(m * k * cs, m * cap);
    if (rc) return rc;
    std::vector<Copy> in(in_direct ? 0 : m * k);
    std::vector<const uint8_t *> dchunks(m * k);
    for (uint64_t o = 0; o < m; ++o)
      for (uint32_t j = 0; j < k; ++j) {
        if (!in_direct) in[o * k + j] = {s.h_in + (o * k + j) * cs, chunks[(g.o0 + o) * k + j], cs};
        dchunks[o * k + j] = s.d_in + (o * k + j) * cs;
      }
    parallel_copy(in);
    hipError_t e = cs ? hipMemcpyAsync(s.d_in, in_direct ? c0 : s.h_in, m * k * cs, hipMemcpyHostToDevice, s.stream)
                      : hipSuccess;
    if (e != hipSuccess) return hip_status(e);
    std::vector<uint64_t> csz(m, cs);
    std::vector<uint8_t *> douts(m);
    for (uint64_t o = 0; o < m; ++o) douts[o] = s.d_out + o * cap;
    rc = restore_batch_device(k, (uint32_t)m, nodes + (uint64_t)g.o0 * k, dchunks.data(), csz.data(),
                              pads.data() + g.o0, douts.data(), flags, s.stream);
    if (rc) return rc;
    s.out_parts.clear();
    if (out_dev)  // straight into the caller's pinned slab
      return hip_status(((reinterpret_cast<uintptr_t>(out_dev) & 15u) == 0 && !pinned_d2h_dma())
                            ? launch_push(out_dev, s.d_out, m * cap, s.stream)
                            : hipMemcpyAsync(outs[g.o0], s.d_out, m * cap, hipMemcpyDeviceToHost, s.stream));
    if ((rc = s.push_out(m * cap))) return rc;
    for (uint64_t o = 0; o < m; ++o)
      if (lens[g.o0 + o]) s.out_parts.push_back({outs[g.o0 + o], s.h_out + o * cap, lens[g.o0 + o]});
    return VDS_EC_OK;
  });
  if (rc == VDS_EC_OK)
    for (uint32_t o = 0; o < count; ++o) out_sizes[o] = lens[o];
  return rc;
}

// ------------------------------------------------ stripe-range split
// One object split by stripe range [t0, t1): cell t of every
// replica depends on stripe t only, so a range is encoded as an object of its
// own -- the slice of input bytes [2k t0, 2k t1) (the object's last range: to
// its end, zero-padded and with the trailer, whose value depends only on
// size mod 2k) -- into replica bytes [2 t0, 2 t1).  Restore likewise writes
// output bytes [2k t0, min(2k t1, E)) from the survivors' cells [t0, t1).
int encode_range(uint32_t k, const uint16_t *replicas, uint32_t n, const uint8_t *in, uint64_t size, uint64_t t0,
                 uint64_t t1, uint8_t *const *outs, unsigned flags, hipStream_t s) {
  if (k == 0 || (flags & VDS_EC_F_CELLS) || (n && (!replicas || !outs))) return VDS_EC_EINVAL;
  const uint64_t sb = 2ull * k, T = (size + sb - 1) / sb;
  if (t0 > t1 || t1 > T || (t0 == t1 && T != 0)) return VDS_EC_EINVAL;
  const bool last = t1 == T;
  const uint64_t slice = last ? size - sb * t0 : sb * (t1 - t0);
  std::vector<uint8_t *> o(n);
  for (uint32_t i = 0; i < n; ++i) {
    if (!outs[i]) return VDS_EC_EINVAL;
    o[i] = outs[i] + 2 * t0;
  }
  return encode_device(2, k, replicas, n, in + sb * t0, slice, slice, 1, o.data(), 0,
                       last ? flags : (flags | VDS_EC_F_NO_TRAILER), s);
}

// restored length and stripes of an object from its trailer padding
int range_restore_len(uint32_t k, uint64_t chunk_size, uint16_t padding, unsigned flags, uint64_t *E, uint64_t *nst) {
  if (flags & VDS_EC_F_CELLS) return VDS_EC_EINVAL;
  bool ok = true;
  *E = restored_len(2, k, chunk_size, padding, flags, &ok);
  if (!ok) return VDS_EC_ERESTORE;
  *nst = (*E + 2ull * k - 1) / (2ull * k);
  return VDS_EC_OK;
}

int restore_range(uint32_t k, const uint16_t *nodes, const uint16_t *matrix, const uint8_t *const *chunks,
                  uint64_t t0, uint64_t t1, uint64_t E, uint8_t *out, unsigned flags, hipStream_t s) {
  const uint64_t sb = 2ull * k;
  std::vector<const uint8_t *> c(k);
  for (uint32_t j = 0; j < k; ++j) c[j] = chunks[j] + 2 * t0;
  const uint64_t len = std::min(sb * t1, E) - sb * t0;
  return restore_device(2, k, nodes, matrix, c.data(), 2 * (t1 - t0), 0, len, 1, out + sb * t0, 0, flags, s);
}

// Split [0, T) into `parts` ranges of whole 2048-stripe tiles (the last
// takes the rest; fewer ranges when there are fewer tiles).
std::vector<std::pair<uint64_t, uint64_t>> stripe_ranges(uint64_t T, uint32_t parts) {
  std::vector<std::pair<uint64_t, uint64_t>> r;
  const uint64_t tiles = (T + kTileStripes - 1) / kTileStripes;
  const uint64_t p = std::max<uint64_t>(1, std::min<uint64_t>(parts, tiles));
  uint64_t at = 0;
  for (uint64_t i = 0; i < p; ++i) {
    const uint64_t end = i + 1 == p ? T : std::min(T, (tiles * (i + 1) / p) * kTileStripes);
    r.push_back({at, end});
    at = end;
  }
  return r;
}

int encode_host_split(uint32_t k, const uint16_t *replicas, uint32_t n, const uint8_t *data, uint64_t size,
                      uint8_t *const *outs, unsigned flags, int max_devices, uint32_t parts) {
  if (k == 0 || (flags & VDS_EC_F_CELLS) || (n && (!replicas || !outs)) || (size && !data)) return VDS_EC_EINVAL;
  int ndev = 0;
  int rc = batch_devices(max_devices, &ndev);
  if (rc) return rc;
  if (n == 0) return VDS_EC_OK;
  for (uint32_t i = 0; i < n; ++i)
    if (!outs[i]) return VDS_EC_EINVAL;
  const uint64_t sb = 2ull * k, T = (size + sb - 1) / sb;
  const auto ranges = stripe_ranges(T, parts ? parts : (uint32_t)ndev);
  std::vector<Group> groups;
  for (uint32_t r = 0; r < ranges.size(); ++r) groups.push_back({r, 1});
  const bool trailer = !(flags & VDS_EC_F_NO_TRAILER);
  return run_host_batch(groups, ndev, [&](BatchSlot &s, const Group &g) -> int {
    const auto [t0, t1] = ranges[g.o0];
    const bool last = t1 == T;
    const uint64_t in_b = last ? size - sb * t0 : sb * (t1 - t0);
    const uint64_t Lr = 2 * (t1 - t0) + (last && trailer ? 2 : 0);  // replica bytes of the range
    int rc = s.reserve(in_b, n * Lr);
    if (!rc) rc = s.reserve_dev(in_b, n * Lr);
    if (rc) return rc;
    parallel_copy({{s.h_in, data + sb * t0, in_b}});
    hipError_t e = in_b ? hipMemcpyAsync(s.d_in, s.h_in, in_b, hipMemcpyHostToDevice, s.stream) : hipSuccess;
    if (e != hipSuccess) return hip_status(e);
    std::vector<uint8_t *> douts(n);
    for (uint32_t i = 0; i < n; ++i) douts[i] = s.d_out + i * Lr;
    rc = encode_device(2, k, replicas, n, s.d_in, in_b, in_b, 1, douts.data(), 0,
                       last ? flags : (flags | VDS_EC_F_NO_TRAILER), s.stream);
    if (rc) return rc;
    if ((rc = s.push_out(n * Lr))) return rc;
    s.out_parts.resize(n);
    for (uint32_t i = 0; i < n; ++i) s.out_parts[i] = {outs[i] + 2 * t0, s.h_out + i * Lr, Lr};
    return VDS_EC_OK;
  });
}

int restore_host_split(uint32_t k, const uint16_t *nodes, const uint8_t *const *chunks, uint64_t chunk_size,
                       uint8_t *out, uint64_t *out_size, unsigned flags, int max_devices, uint32_t parts) {
  int rc = check_restore_args(k, nodes, chunks, chunk_size);
  if (rc) return rc;
  if (!out_size || (flags & VDS_EC_F_CELLS)) return VDS_EC_EINVAL;
  int ndev = 0;
  if ((rc = batch_devices(max_devices, &ndev))) return rc;
  const uint16_t padding = chunk_size < 2 ? 0 : (uint16_t)((chunks[0][chunk_size - 2] << 8) | chunks[0][chunk_size - 1]);
  uint64_t E = 0, nst = 0;
  if ((rc = range_restore_len(k, chunk_size, padding, flags, &E, &nst))) return rc;
  if (E > *out_size || (E && !out)) return VDS_EC_EINVAL;
  std::vector<uint16_t> m((size_t)k * k);
  if ((rc = inverse16(k, nodes, m.data()))) return rc;
  const uint64_t sb = 2ull * k;
  const auto ranges = stripe_ranges(nst, parts ? parts : (uint32_t)ndev);
  std::vector<Group> groups;
  for (uint32_t r = 0; r < ranges.size() && nst; ++r) groups.push_back({r, 1});
  rc = run_host_batch(groups, ndev, [&](BatchSlot &s, const Group &g) -> int {
    const auto [t0, t1] = ranges[g.o0];
    const uint64_t Lr = 2 * (t1 - t0), len = std::min(sb * t1, E) - sb * t0;
    int rc = s.reserve(k * Lr, len);
    if (!rc) rc = s.reserve_dev(k * Lr, len);
    if (rc) return rc;
    std::vector<Copy> in(k);
    std::vector<const uint8_t *> dchunks(k);
    for (uint32_t j = 0; j < k; ++j) {
      in[j] = {s.h_in + j * Lr, chunks[j] + 2 * t0, Lr};
      dchunks[j] = s.d_in + j * Lr;
    }
    parallel_copy(in);
    hipError_t e = hipMemcpyAsync(s.d_in, s.h_in, k * Lr, hipMemcpyHostToDevice, s.stream);
    if (e != hipSuccess) return hip_status(e);
    rc = restore_device(2, k, nodes, m.data(), dchunks.data(), Lr, 0, len, 1, s.d_out, 0, flags, s.stream);
    if (rc) return rc;
    if ((rc = s.push_out(len))) return rc;
    s.out_parts.assign(1, Copy{out + sb * t0, s.h_out, len});
    return VDS_EC_OK;
  });
  if (rc == VDS_EC_OK) *out_size = E;
  return rc;
}

}  // namespace

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
  rc = encode_device(2, k, replicas, n, c.d_in, size, size, 1, douts.data(), 0, flags, c.stream);
  if (rc) return rc;
  // the replica hashes of save_temp / save_data (dht_network_client.cpp:79, :593), on the device
  hipError_t e = launch_sha256(c.d_out, L, L, n, c.d_out + dig, c.stream);
  if (e != hipSuccess) return hip_status(e);
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
  HostCtx *cp = host_ctx();
  if (!cp) return VDS_EC_ENODEV;
  HostCtx &c = *cp;
  // replicas, then n digests at a 16-byte aligned offset: one push out
  const uint64_t dig = (L * n + 15) & ~15ull;
  rc = c.ensure(size ? size : 1, dig + 32ull * (n ? n : 1));
  if (!rc) rc = c.stage_in(data, size);
  if (rc) return rc;
  std::vector<Copy> parts;
  if (n) {
    std::vector<uint16_t> ids(n);
    std::vector<uint8_t *> douts(n);
    for (uint32_t i = 0; i < n; ++i) {
      ids[i] = (uint16_t)i;
      douts[i] = c.d_out + (uint64_t)i * L;
      parts.push_back({outs[i], c.h_out + (uint64_t)i * L, L});
    }
    rc = encode_device(2, k, ids.data(), n, c.d_in, size, size, 1, douts.data(), 0, 0, c.stream);
    if (rc) return rc;
    hipError_t e = launch_sha256(c.d_out, L, L, n, c.d_out + dig, c.stream);  // save_temp's replica names (:79)
    if (e != hipSuccess) return hip_status(e);
    e = launch_push(c.h_out_dev, c.d_out, dig + 32ull * n, c.stream);
    if (e != hipSuccess) return hip_status(e);
    parts.push_back({replica_digests, c.h_out + dig, 32ull * n});
  }
  // upload_data's hash of the body (server_api.cpp:16) on this thread while
  // the device works: one sequential chain, ~3 us a block in a GPU lane
  // (sha256_host.cpp)
  sha256_host(data, size, data_digest);
  if (n) {
    if ((rc = hip_status(hipStreamSynchronize(c.stream)))) return rc;
    parallel_copy(parts);
  }
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
