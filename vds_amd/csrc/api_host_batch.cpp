// api_host_batch.cpp -- caller-pinned slabs, the multi-GPU host batches
// and the stripe-range split of one object over several devices.
// (api_internal.hpp lists the host runtime's translation units.)
#include "api_internal.hpp"

namespace vds_ec {
namespace api {

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

// One persistent thread per device index >= 1 for the host batches (device 0
// runs on the caller's thread).  Never destroyed, as HostPool.
class DeviceWorkers {
 public:
  struct Task {
    std::function<void()> fn;
    std::mutex m;
    std::condition_variable cv;
    bool done = false;
    void wait() {
      std::unique_lock<std::mutex> g(m);
      cv.wait(g, [&] { return done; });
    }
  };
  static DeviceWorkers &get() {
    static DeviceWorkers *w = new DeviceWorkers();
    return *w;
  }
  std::shared_ptr<Task> post(int dev, std::function<void()> fn) {
    auto t = std::make_shared<Task>();
    t->fn = std::move(fn);
    Lane &l = lane(dev);
    {
      std::lock_guard<std::mutex> g(l.mu);
      l.q.push_back(t);
    }
    l.cv.notify_one();
    return t;
  }

 private:
  struct Lane {
    std::mutex mu;
    std::condition_variable cv;
    std::vector<std::shared_ptr<Task>> q;
  };
  Lane &lane(int dev) {
    std::lock_guard<std::mutex> g(mu_);
    auto &l = lanes_[dev];
    if (!l) {
      l = std::make_unique<Lane>();
      Lane *lp = l.get();
      std::thread([lp] {
        for (;;) {
          std::shared_ptr<Task> t;
          {
            std::unique_lock<std::mutex> g(lp->mu);
            lp->cv.wait(g, [&] { return !lp->q.empty(); });
            t = lp->q.front();
            lp->q.erase(lp->q.begin());
          }
          t->fn();
          std::lock_guard<std::mutex> g(t->m);
          t->done = true;
          t->cv.notify_all();
        }
      }).detach();
    }
    return *l;
  }
  std::mutex mu_;
  std::map<int, std::unique_ptr<Lane>> lanes_;
};

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
  // device 0 on the calling thread, the others on persistent per-device
  // workers: the thread-local planning tables (BatchScratch) and HIP thread
  // state survive from call to call instead of being rebuilt by a fresh
  // thread per group
  const int used = (int)std::min<size_t>((size_t)ndev, groups.size());
  std::vector<std::shared_ptr<DeviceWorkers::Task>> tasks;
  for (int d = 1; d < used; ++d) tasks.push_back(DeviceWorkers::get().post(d, [&worker, d] { worker(d); }));
  if (used > 0) {
    int cur = 0;
    const bool have = hipGetDevice(&cur) == hipSuccess;
    worker(0);
    if (have) (void)hipSetDevice(cur);  // (the caller's current device is left as it was)
  }
  for (auto &t : tasks) t->wait();
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
      return hip_status(((reinterpret_cast<uintptr_t>(out_dev) & 15u) == 0)
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
      return hip_status(((reinterpret_cast<uintptr_t>(out_dev) & 15u) == 0)
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

}  // namespace api
}  // namespace vds_ec
