// api_batch.cpp -- batched per-object-survivor restore and regenerate:
// routes, erased-set plans, tile pairing and the launches.
// (api_internal.hpp lists the host runtime's translation units.)
#include "api_internal.hpp"

namespace vds_ec {
namespace api {

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
  std::shared_mutex mu;  // (the batch planners look plans up from several threads at once)
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

// The store key of the erased set ~seen (k, n = k + k/4 compiled; or, ms >
// 0, the SMALL plan over 0..k+ms-1).
inline uint64_t syn_plan_key(uint32_t k, uint32_t n, uint64_t seen, uint32_t ms) {
  if (ms) n = k + ms;
  return (~seen & ((1ull << n) - 1)) | ((uint64_t)k << 56) | ((uint64_t)ms << 48);
}

// Solve the plan of that set: points and erased points ascending, the M x M
// solve as bit selections (or SMALL's masks).  No store access.
bool syn_plan_solve(uint32_t k, uint32_t n, uint64_t seen, SynBatchPlan *out, uint32_t ms) {
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
  static constexpr unsigned kMaxWorkers = 15;
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
    // the CPUs this process may run on (a GPU box's share of the host is 16;
    // hardware_concurrency counts the whole machine)
    unsigned hw = std::thread::hardware_concurrency();
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof set, &set) == 0) hw = std::min(hw ? hw : 1024u, (unsigned)CPU_COUNT(&set));
    nworkers_ = hw > 1 ? std::min(hw - 1, kMaxWorkers) : 0u;
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

// fn(part, o0, o1) over [0, count) in at most kMaxParts contiguous ranges of
// at least kMinPer objects; a call with the same count always makes the same
// ranges, so a later pass can continue from per-part totals of an earlier one.
constexpr unsigned kMaxParts = 16;
inline unsigned batch_parts(uint32_t count) {
  constexpr uint32_t kMinPer = 1024;
  return std::min<uint32_t>(kMaxParts, std::max<uint32_t>(1, count / kMinPer));
}
template <class F>
void parallel_parts(uint32_t count, F &&fn) {
  const unsigned parts = batch_parts(count);
  HostPool::get().run(parts, [&](unsigned p) {
    fn(p, (uint32_t)((uint64_t)count * p / parts), (uint32_t)((uint64_t)count * (p + 1) / parts));
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
  uint32_t plan;    // kRouteSyn: its plan's claim number (SynBatchBuild::plan_of)
};

// (BatchObjInfo::ms of the PERM regenerate: survivors exactly 0..k-1, one
// target in k..2k-1)
constexpr uint8_t kMsPerm = 3;

// The SMALL batch kernels (a -DVDS_BATCH_SMALL=0 build routes their objects
// to the N = k + k/4 syndrome kernel instead: A/B).
#ifndef VDS_BATCH_SMALL
#define VDS_BATCH_SMALL 1
#endif
constexpr bool small_enabled() { return VDS_BATCH_SMALL != 0; }
// Restore objects of the N = k + k/4 syndrome class at k = 32 (survivors
// within 0..39 beyond the SMALL sizes) through the RT batch instead
// (study switch, -DVDS_BATCH_N_TO_RT=1): at p = 0.25 those objects' erased
// sets are nearly all distinct, so their syndrome tiles run half empty, while
// RT tiles pair any two objects.  Same box, ABBA (profiles/round6/planner/
// ab_n40_to_rt.log): device time per live call 2.08-2.09 -> 2.03-2.05 ms at
// p = 0.25, unchanged at p = 0.02 -- within the rates' noise; off.
#ifndef VDS_BATCH_N_TO_RT
#define VDS_BATCH_N_TO_RT 0
#endif
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

// Dual syndrome tiles (restore_syn.hpp VDS_BATCH_DUAL; the host pairs only
// what the kernels were built with)
#ifndef VDS_BATCH_DUAL
#define VDS_BATCH_DUAL 1
#endif
constexpr bool dual_enabled() { return VDS_BATCH_DUAL != 0; }
// Tiles of unequal cost (the RT launch's, sorted by row count; a one-class
// syndrome launch's dual tiles) interleaved over the XCDs' ranges (A/B: 0 =
// in sorted order)
#ifndef VDS_BATCH_RT_SPREAD
#define VDS_BATCH_RT_SPREAD 1
#endif

// Host-side builder of one k_restore_syn batch launch, written straight into
// a pinned parameter slot: objs (and the empty object), then tiles, then
// plans.  plan_of() resolves survivor sets to plans and fill() writes
// descriptor i; both run on several threads at once (distinct i).
//
// Plans by class (rank: SMALL ms = 1, ms = 2, PERM, the N = k + k/4 syndrome
// kernel's), each class's plans contiguous in the slot so its tiles are too.
// In the first pass the first object of a new set claims it in a call-wide
// hash (CAS) and numbers it within its own (class, part) region, so the
// parts share no counter; numbered() then maps a claim to its dense slot
// index (class, then part, then claim order) in O(1).  In the second pass
// each part first fills the plans it claimed -- from the process-wide store
// under one lock hold, solving what the store lacks -- and then writes its
// descriptors with dense plan numbers.  (Claims through a shared counter and
// per-set store locking from eight threads made that pass 4x slower.)
inline uint32_t plan_class_rank(uint32_t ms) { return ms == 1 ? 0 : ms == 2 ? 1 : ms == kMsPerm ? 2 : 3; }
struct SynBatchBuild {
  static constexpr uint32_t kPending = 0xFFFFFFFFu;
  // claim = (class * kMaxParts + part) << kRegionShift | index within the
  // region (< the part's objects: < 2^26 for any count below 2^30)
  static constexpr int kRegionShift = 26;
  static_assert(4 * kMaxParts <= (1u << (32 - kRegionShift)), "claim regions fit in the claim's top bits");
  uint32_t k, n;
  bool regen = false;
  ParamSlot *slot = nullptr;
  size_t cap_objs = 0, cap_tiles = 0, o_tiles = 0, o_plans = 0;
  SynBatchObj *objs = nullptr;
  uint32_t nobj = 0;
  std::vector<uint32_t> obj_plan, obj_halves;
  struct PlanReq {
    uint64_t seen;
    uint32_t claim;
    uint8_t ms;
    uint16_t target;
  };
  // A part's cache of the keys it has looked up in this call, in front of the
  // shared table: a set that repeats within the part (most do at low loss
  // rates) is answered from the part's own cache lines.  Direct-mapped;
  // entries of an earlier call are told apart by the call's epoch.
  static constexpr uint32_t kLocal = 1024;
  struct LocalEntry {
    uint64_t key;
    uint32_t val, epoch;
  };
  struct alignas(64) PartPlans {  // (one cache line apart: the parts write them concurrently)
    std::vector<uint32_t> hused;  // table entries this part claimed (cleared one by one when the table is reused)
    std::vector<PlanReq> reqs, miss;
    std::vector<LocalEntry> local;
    uint32_t next[4];  // claims in each class
  };
  uint32_t epoch = 0;
  PartPlans pp[kMaxParts];
  uint32_t dense[4 * kMaxParts + 1];   // first slot plan of each (class, part) region
  uint32_t cls_end[4] = {0, 0, 0, 0};  // dense class ranges: [cls_end[c - 1], cls_end[c])
  // (survivor set, ms, PERM target) -> claim: open addressing, linear
  // probing, filled concurrently (a key is taken by CAS; its value reads
  // kPending until the claimer has numbered it)
  struct Entry {  // key and claim in one 16-byte entry: a claim moves one cache line between cores, not two
    uint64_t key;
    uint32_t val;
    uint32_t pad;
  };
  std::vector<Entry> ht;
  std::vector<uint64_t> first_, used_;
  unsigned hshift = 64;

  static size_t up16(size_t x) { return (x + 15) & ~size_t(15); }

  // A builder is per thread and reused (batch_scratch): the vectors keep
  // their capacity, so a steady stream of calls allocates nothing.  The
  // claim table is made ready for `count` objects.
  void reset(uint32_t k_, uint32_t n_, uint32_t count) {
    k = k_;
    n = n_;
    regen = false;
    slot = nullptr;
    cap_objs = cap_tiles = o_tiles = o_plans = 0;
    objs = nullptr;
    nobj = 0;
    unsigned bits = 4;
    while ((1ull << bits) < 2ull * count) ++bits;
    if (ht.size() != (1ull << bits)) {
      ht.assign(1ull << bits, Entry{0, kPending, 0});
      for (PartPlans &q : pp) q.hused.clear();
    }
    for (PartPlans &q : pp) {
      for (const uint32_t x : q.hused) {
        ht[x].key = 0;
        ht[x].val = kPending;
      }
      q.hused.clear();
      q.reqs.clear();
      for (uint32_t &x : q.next) x = 0;
      if (q.local.empty()) q.local.assign(kLocal, LocalEntry{0, 0, 0});
    }
    if (++epoch == 0) {  // (wrapped: forget every cached key)
      for (PartPlans &q : pp) q.local.assign(kLocal, LocalEntry{0, 0, 0});
      epoch = 1;
    }
    hshift = 64 - bits;
  }
  // The claim of survivor set `seen` (ms > 0: the SMALL plan over 0..k+ms-1,
  // or kMsPerm: survivors 0..k-1 and one target in k..2k-1; a set always
  // resolves to the same ms within a call: the route is a function of the
  // set), taken on first sight.  Thread-safe across parts (part: the
  // caller's parallel_parts range).
  uint32_t plan_of(unsigned part, uint64_t seen, uint32_t ms, uint32_t target) {
    // (keyed by set AND ms: a regenerate's route also depends on its targets,
    // so one set may meet two SMALL sizes in a call; PERM also by target)
    const uint64_t hk = seen | ((uint64_t)ms << 56) | (ms == kMsPerm ? (uint64_t)target << 48 : 0);
    const uint64_t hash = hk * 0x9E3779B97F4A7C15ull;
    LocalEntry &le = pp[part].local[(hash >> 54) & (kLocal - 1)];
    if (le.key == hk && le.epoch == epoch) return le.val;
    const uint32_t v = plan_of_shared(part, seen, ms, target, hk, hash);
    le = LocalEntry{hk, v, epoch};
    return v;
  }
  uint32_t plan_of_shared(unsigned part, uint64_t seen, uint32_t ms, uint32_t target, uint64_t hk, uint64_t hash) {
    const size_t mask = ht.size() - 1;
    size_t i = (size_t)(hash >> hshift);
    for (;;) {
      uint64_t cur = __atomic_load_n(&ht[i].key, __ATOMIC_ACQUIRE);
      if (cur == 0) {
        if (__atomic_compare_exchange_n(&ht[i].key, &cur, hk, false, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE)) {
          PartPlans &q = pp[part];
          const uint32_t c = plan_class_rank(ms);
          const uint32_t v = ((c * kMaxParts + part) << kRegionShift) | q.next[c]++;
          __atomic_store_n(&ht[i].val, v, __ATOMIC_RELEASE);
          q.hused.push_back((uint32_t)i);
          q.reqs.push_back(PlanReq{seen, v, (uint8_t)ms, (uint16_t)target});
          return v;
        }
        // (another thread claimed the entry first: cur holds its key)
      }
      if (cur == hk) {
        uint32_t v;
        while ((v = __atomic_load_n(&ht[i].val, __ATOMIC_ACQUIRE)) == kPending) {
        }  // (the claimer stores it right after numbering it)
        return v;
      }
      i = (i + 1) & mask;
    }
  }
  // After the first pass: the dense numbering of the claims.
  uint32_t number_plans(unsigned parts) {
    uint32_t at = 0;
    for (int c = 0; c < 4; ++c) {
      for (unsigned q = 0; q < kMaxParts; ++q) {
        dense[c * kMaxParts + q] = at;
        at += q < parts ? pp[q].next[c] : 0;
      }
      cls_end[c] = at;
    }
    dense[4 * kMaxParts] = at;
    return at;
  }
  uint32_t numbered(uint32_t claim) const {
    return dense[claim >> kRegionShift] + (claim & ((1u << kRegionShift) - 1));
  }
  // Part `part`'s claimed plans, into the slot (second pass, before its
  // descriptors); false when a set has no solve (not for distinct points).
  bool resolve_plans(unsigned part) {
    PartPlans &q = pp[part];
    SynBatchPlan *dst = reinterpret_cast<SynBatchPlan *>(slot->h + o_plans);
    SynPlanStore &st = syn_plan_store();
    bool ok = true;
    q.miss.clear();
    if (!q.reqs.empty()) {
      std::shared_lock<std::shared_mutex> g(st.mu);
      for (const PlanReq &r : q.reqs) {
        if (r.ms == kMsPerm) continue;
        auto it = st.map.find(syn_plan_key(k, n, r.seen, r.ms));
        if (it != st.map.end())
          dst[numbered(r.claim)] = it->second;
        else
          q.miss.push_back(r);
      }
    }
    size_t solved = 0;
    for (const PlanReq &r : q.miss) {
      if (syn_plan_solve(k, n, r.seen, &dst[numbered(r.claim)], r.ms))
        q.miss[solved++] = r;
      else
        ok = false;
    }
    if (solved) {
      std::unique_lock<std::shared_mutex> g(st.mu);
      if (st.map.size() + solved > SynPlanStore::kMax) st.map.clear();
      for (size_t x = 0; x < solved; ++x)
        st.map.emplace(syn_plan_key(k, n, q.miss[x].seen, q.miss[x].ms), dst[numbered(q.miss[x].claim)]);
    }
    for (const PlanReq &r : q.reqs) {
      SynBatchPlan &pl = dst[numbered(r.claim)];
      if (r.ms == kMsPerm) {
        pl = SynBatchPlan{};
        for (uint32_t j = 0; j < k; ++j) pl.point[j] = (uint8_t)j;
        for (uint32_t e = 0; e < kMaxFastK / 4; ++e) pl.erased[e] = (uint8_t)r.target;
        pl.cls = 3;  // (kClsPerm)
      } else {
        if (r.ms && regen) pl.nrec = r.ms;  // (regenerate: every erased point of A is a target candidate)
        pl.cls = r.ms;                      // (kClsSyn = 0, kClsSmall1 / 2 = ms)
      }
    }
    return ok;
  }

  // The slot bytes for `count` objects of `halves` half tiles and `plans`
  // distinct plans; then attach().
  size_t layout(uint32_t count, uint64_t halves, uint32_t plans) {
    nobj = count;
    cap_objs = (size_t)count + 1;
    cap_tiles = (size_t)((halves + count + 1) / 2 + 1);  // pairs within each plan: <= (halves + plans) / 2
    o_tiles = up16(cap_objs * sizeof(SynBatchObj));
    o_plans = up16(o_tiles + cap_tiles * sizeof(SynBatchTile));
    return o_plans + (size_t)plans * sizeof(SynBatchPlan);
  }
  void attach(ParamSlot *sl) {
    slot = sl;
    objs = reinterpret_cast<SynBatchObj *>(slot->h);
    obj_plan.resize(nobj);
    obj_halves.resize(nobj);
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
  // At k = 32 the odd half of each N-point syndrome plan (class 3)
  // goes into a dual tile with another plan's (kTileDual, after class 3's
  // own tiles) instead of a tile of its own beside the empty object.
  int launch(bool regen, hipStream_t s) {
    if (nobj == 0) return hip_status(param_release(slot, s));
    const uint32_t empty = nobj;
    std::memset(&objs[empty], 0, sizeof(SynBatchObj));
    const uint32_t np = cls_end[3];
    const uint32_t base[5] = {0, cls_end[0], cls_end[1], cls_end[2], cls_end[3]};
    const bool dual = dual_enabled() && k == 32;
    std::vector<uint64_t> &first = first_, &used = used_;
    first.assign(np + 1, 0);  // tile offset of each plan
    used.assign(np, 0);
    for (uint32_t o = 0; o < nobj; ++o) first[obj_plan[o] + 1] += obj_halves[o];
    uint64_t singles = 0;  // dual: class 3's odd halves
    for (size_t p = 0; p < np; ++p) {
      const uint64_t h = first[p + 1];
      const bool pair_out = dual && p >= base[3] && (h & 1u);
      singles += pair_out;
      first[p + 1] = first[p] + (pair_out ? h / 2 : (h + 1) / 2);
    }
    const uint64_t ndual = (singles + 1) / 2;
    const uint64_t ntiles = first[np] + ndual;
    if (ntiles > cap_tiles || ntiles > 0xFFFFFFFFull) {
      (void)param_release(slot, s);
      return VDS_EC_EINVAL;
    }
    // classes (contiguous plan and tile ranges; the dual tiles end class 3's)
    const uint32_t *bound = base + 1;
    auto cls_tiles = [&](int c) { return first[base[c + 1]] - first[base[c]] + (c == 3 ? ndual : 0); };
    int ncls = 0;
    for (int c = 0; c < 4; ++c) ncls += cls_tiles(c) > 0;
    // MULTI (ncls > 1): tile t goes to position pos(t), so that each XCD's
    // contiguous eighth of the launch (tile_range) gets every eighth tile --
    // the same mix of classes, whose tiles cost differently
    const uint64_t R = ntiles;
    auto pos = [&](uint64_t t) -> uint64_t {
      if (ncls <= 1 && (ndual == 0 || !VDS_BATCH_RT_SPREAD)) return t;  // (dual tiles cost more: spread them too)
      const uint64_t r = t % 8;
      return r * (R / 8) + std::min<uint64_t>(r, R % 8) + t / 8;
    };
    SynBatchTile *tiles = reinterpret_cast<SynBatchTile *>(slot->h + o_tiles);
    for (size_t p = 0; p < np; ++p)
      for (uint64_t t = first[p]; t < first[p + 1]; ++t)
        tiles[pos(t)] = SynBatchTile{{empty, empty}, {0, 0}, (uint32_t)p, 0, 0, 0};
    uint64_t si = 0;  // dual: singles placed
    for (uint32_t o = 0; o < nobj; ++o) {
      const uint32_t p = obj_plan[o];
      for (uint32_t h = 0; h < obj_halves[o]; ++h) {
        const uint64_t i = used[p]++;
        if (dual && p >= base[3] && i == 2 * (first[p + 1] - first[p])) {  // the plan's odd half
          SynBatchTile &t = tiles[pos(first[np] + si / 2)];
          if ((si & 1) == 0)
            t = SynBatchTile{{o, empty}, {h * kHalfStripes, 0}, p, 0, 0, 0};
          else
            t.obj[1] = o, t.stripe0[1] = h * kHalfStripes, t.mode = kTileDual;
          if (regen && h + 1 == obj_halves[o]) t.trailer |= 1u << (si & 1);
          ++si;
          continue;
        }
        SynBatchTile &t = tiles[pos(first[p] + i / 2)];
        t.obj[i & 1] = o;
        t.stripe0[i & 1] = h * kHalfStripes;
        if (regen && h + 1 == obj_halves[o]) t.trailer |= 1u << (i & 1);
      }
    }
    hipError_t e = param_commit(slot, o_plans + (size_t)np * sizeof(SynBatchPlan), s);
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
        const uint64_t t0 = first[p0], t1 = first[bound[c]] + (c == 3 ? ndual : 0);
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
// RT2 rows for the k = 32 restore's RT objects (a -DVDS_BATCH_RT2=0 build:
// every RT object takes the k-slot combination, A/B)
#ifndef VDS_BATCH_RT2
#define VDS_BATCH_RT2 1
#endif
constexpr bool rt2_enabled() { return VDS_BATCH_RT2 != 0; }

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
    // The tile count first (the mode boundary may leave a half empty), then
    // the tiles at interleaved positions: each XCD's contiguous eighth of the
    // launch (tile_range) gets every eighth tile of the sorted order, so every
    // XCD has the same mix of row counts (in sorted order the heaviest tiles
    // all landed on the last XCD, which then set the launch's length)
    uint64_t i = 0;
    uint32_t cur = 0;
    for (const uint32_t o : order) {
      if ((i & 1) && cur != objs[o].rt.mode) ++i;
      cur = objs[o].rt.mode;
      i += obj_halves[o];
    }
    const uint64_t R = (i + 1) / 2;
    auto pos = [&](uint64_t t) -> uint64_t {
      if (!VDS_BATCH_RT_SPREAD) return t;
      const uint64_t r = t % 8;
      return r * (R / 8) + std::min<uint64_t>(r, R % 8) + t / 8;
    };
    i = 0;
    for (const uint32_t o : order) {
      if ((i & 1) && tiles[pos(i / 2)].mode != objs[o].rt.mode) ++i;  // (the other mode starts a new tile)
      for (uint32_t h = 0; h < obj_halves[o]; ++h, ++i) {
        SynBatchTile &t = tiles[pos(i / 2)];
        if ((i & 1) == 0) t = SynBatchTile{{empty, empty}, {0, 0}, 0, 0, 0, objs[o].rt.mode};
        t.obj[i & 1] = o;
        t.stripe0[i & 1] = h * kHalfStripes;
        t.nm = std::max(t.nm, objs[o].rt.ne);
        if (regen && h + 1 == obj_halves[o]) t.trailer |= 1u << (i & 1);
      }
    }
    const uint64_t ntiles = R;
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

// Totals of the routed objects per part of a batch call (parallel_parts
// ranges): counted by the first pass, prefix-summed, then each part of the
// second pass numbers its own objects' descriptors and rows from its base.
struct PartTotals {
  uint32_t nsyn = 0, nrt = 0;
  uint64_t syn_halves = 0, rt_halves = 0, rt_rows = 0;
  void add(const BatchObjInfo &f) {
    if (f.route == kRouteSyn) {
      ++nsyn;
      syn_halves += f.halves;
    } else if (f.route == kRouteRt) {
      nrt += f.parts;
      rt_halves += (uint64_t)f.parts * f.halves;
      rt_rows += f.rows;
    }
  }
  void add(const PartTotals &t) {
    nsyn += t.nsyn;
    nrt += t.nrt;
    syn_halves += t.syn_halves;
    rt_halves += t.rt_halves;
    rt_rows += t.rt_rows;
  }
};
struct BatchIndex {
  PartTotals part[kMaxParts];  // the first pass's totals of each part
  PartTotals base[kMaxParts];  // each part's first descriptor / row (build())
  PartTotals all;
  unsigned parts = 0;
  void reset(uint32_t count) {
    parts = batch_parts(count);
    for (PartTotals &t : part) t = PartTotals{};
  }
  void build() {
    all = PartTotals{};
    for (unsigned p = 0; p < parts; ++p) {
      base[p] = all;
      all.add(part[p]);
    }
  }
};

// A -DVDS_HOST_TRACE=1 build: the batched calls print their host phases (us)
// to stderr (planning cost study, tools/host_trace.py).
#ifndef VDS_HOST_TRACE
#define VDS_HOST_TRACE 0
#endif
struct HostTrace {
  const char *name;
  bool on;
  std::chrono::steady_clock::time_point t0, last;
  char buf[256];
  int len = 0;
  explicit HostTrace(const char *n) : name(n), on(enabled()) {
    if (on) t0 = last = std::chrono::steady_clock::now();
  }
  static constexpr bool enabled() { return VDS_HOST_TRACE != 0; }
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

// The batch calls' per-object tables, per thread and reused: at 16K objects
// a call's fresh vectors came from mmap and paid their page faults every
// call (~100 us of the planning at loss 0.25).
struct BatchScratch {
  std::vector<uint64_t> lens;
  std::vector<BatchObjInfo> info;
  BatchIndex ix;
  SynBatchBuild bb;
  RtBatchBuild rb;
};
BatchScratch &batch_scratch() {
  thread_local BatchScratch sc;
  return sc;
}

// Acquire both builders' slots (together: see param_acquire_n).
int batch_begin(const BatchIndex &ix, SynBatchBuild &bb, RtBatchBuild &rb, HostTrace *ht) {
  size_t bytes[2];
  ParamSlot *sl[2] = {};
  int nb = 0;
  if (ix.all.nsyn) bytes[nb++] = bb.layout(ix.all.nsyn, ix.all.syn_halves, bb.number_plans(ix.parts));
  if (ix.all.nrt) bytes[nb++] = rb.layout(ix.all.nrt, ix.all.rt_halves, ix.all.rt_rows);
  const hipError_t e = param_acquire_n(nb, bytes, sl);
  if (e != hipSuccess) return hip_status(e);
  if (ht) ht->mark("acquire");
  nb = 0;
  if (ix.all.nsyn) bb.attach(sl[nb++]);
  if (ix.all.nrt) rb.attach(sl[nb++]);
  if (ht) ht->mark("attach");
  return VDS_EC_OK;
}

void batch_abandon(const BatchIndex &ix, SynBatchBuild &bb, RtBatchBuild &rb, hipStream_t s) {
  if (ix.all.nsyn) bb.abandon(s);
  if (ix.all.nrt) rb.abandon(s);
}

int batch_launch(const BatchIndex &ix, SynBatchBuild &bb, RtBatchBuild &rb, bool regen, hipStream_t s) {
  int rc = ix.all.nsyn ? bb.launch(regen, s) : VDS_EC_OK;
  if (rc) {
    if (ix.all.nrt) rb.abandon(s);
    return rc;
  }
  return ix.all.nrt ? rb.launch(regen, s) : VDS_EC_OK;
}

int restore_batch_device(uint32_t k, uint32_t count, const uint16_t *nodes, const uint8_t *const *chunks,
                         const uint64_t *chunk_sizes, const uint16_t *paddings, uint8_t *const *outs, unsigned flags,
                         hipStream_t s) {
  if (k == 0 || (count && (!nodes || !chunks || !chunk_sizes || !paddings || !outs))) return VDS_EC_EINVAL;
  if (count == 0) return VDS_EC_OK;
  if (count >= (1u << 30)) return VDS_EC_EINVAL;  // (the planner's claim numbers; a slot that size could not be pinned anyway)
  const uint32_t n = k + k / 4;
  const bool batch_ok = !(flags & VDS_EC_F_CELLS) && k % 4 == 0 && has_restore_syn(k, n);
  const bool syn = batch_ok && !restore_path_override_bs();
  HostTrace ht("restore_batch");
  // pass 1 (parallel): every object validated before anything is enqueued,
  // its route and sizes; per-part totals
  BatchScratch &sc = batch_scratch();
  std::vector<uint64_t> &lens = sc.lens;
  std::vector<BatchObjInfo> &info = sc.info;
  lens.resize(count);
  info.resize(count);
  BatchIndex &ix = sc.ix;
  ix.reset(count);
  SynBatchBuild &bb = sc.bb;
  bb.reset(k, n, count);
  FirstError err;
  parallel_parts(count, [&](unsigned part, uint32_t o0, uint32_t o1) {
    PartTotals tot;
    for (uint32_t o = o0; o < o1; ++o) {
      const uint16_t *nd = nodes + (uint64_t)o * k;
      lens[o] = 0;
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
        info[o] = f;
        return;
      }
      const uint64_t need = (lens[o] + 2ull * k - 1) / (2ull * k);  // stripes that produce output
      f.halves = (uint32_t)std::min<uint64_t>((need + kHalfStripes - 1) / kHalfStripes, UINT32_MAX);
      // (SynBatchTile::stripe0 is 32-bit: objects past 2^32 stripes take the per-object path)
      const bool fits = need <= 0xFFFFFFFFull - kHalfStripes;
      if (need == 0) {
        f.route = kRouteSkip;
      } else if (syn && fits && maxid < n && !(VDS_BATCH_N_TO_RT && k == 32 && small_ms_for(k, maxid) == 0)) {
        f.route = kRouteSyn;
        f.ms = small_ms_for(k, maxid);
        f.plan = bb.plan_of(part, f.seen, f.ms, 0);
      } else if (batch_ok && fits && maxid < 256) {
        f.route = kRouteRt;
        f.parts = 1;
        f.rows = (uint16_t)(k - __builtin_popcountll(f.seen & ((1ull << k) - 1)));  // erased points below k
      } else {
        f.route = kRouteOne;
      }
      info[o] = f;
      tot.add(f);
    }
    ix.part[part] = tot;
  });
  if (err.rc) return err.rc;
  int rc = device_ready();
  if (rc) return rc;
  ht.mark("pass1");
  ix.build();
  RtBatchBuild &rb = sc.rb;
  rb.reset(k, n);
  rb.rt2 = rt2_enabled();  // (restore only; RtBatchBuild::fill decides per object)
  if ((rc = batch_begin(ix, bb, rb, &ht))) return rc;
  ht.mark("begin");
  // pass 2 (parallel): the plans (resolved here, concurrently) and the
  // descriptors, numbered from each part's base
  parallel_parts(count, [&](unsigned part, uint32_t o0, uint32_t o1) {
    if (ix.all.nsyn && !bb.resolve_plans(part)) {  // (a set with no solve: not for distinct points)
      err.note(o0, VDS_EC_ESINGULAR);
      return;
    }
    uint32_t isyn = ix.base[part].nsyn, irt = ix.base[part].nrt;
    uint64_t row = ix.base[part].rt_rows;
    for (uint32_t o = o0; o < o1; ++o) {
      const BatchObjInfo &f = info[o];
      const uint16_t *nd = nodes + (uint64_t)o * k;
      const uint8_t *const *ch = chunks + (uint64_t)o * k;
      SynBatchObj *d;
      if (f.route == kRouteSyn) {
        d = &bb.fill(isyn++, f.seen, nd, ch, bb.numbered(f.plan), f.halves);
      } else if (f.route == kRouteRt) {
        uint8_t rowp[kMaxFastK];
        uint32_t ne = 0;
        for (uint64_t b = ~f.seen & ((1ull << k) - 1); b; b &= b - 1) rowp[ne++] = (uint8_t)__builtin_ctzll(b);
        d = &rb.fill(irt, nd, ch, rowp, ne, row, f.halves);
        irt += f.parts;
        row += f.rows;
      } else {
        continue;
      }
      d->out = outs[o];
      std::memset(d->regen, 0, sizeof d->regen);
      d->out_len = lens[o];
      d->chunk_len = chunk_sizes[o];
    }
  });
  if (err.rc) {
    batch_abandon(ix, bb, rb, s);
    return err.rc;
  }
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
  if (count >= (1u << 30)) return VDS_EC_EINVAL;  // (as restore_batch_device)
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
  info.resize(count);
  BatchIndex &ix = sc.ix;
  ix.reset(count);
  SynBatchBuild &bb = sc.bb;
  bb.reset(k, n, count);
  bb.regen = true;
  FirstError err;
  parallel_parts(count, [&](unsigned part, uint32_t o0, uint32_t o1) {
    PartTotals tot;
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
        info[o] = f;
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
      if (syn && small_enabled() && fits && nt == 1 && (k == 16 || k == 32) && maxid < k && tg[0] >= k &&
          tg[0] < 2 * k) {  // (syn: the restore-path override and has_restore_syn apply, as to SMALL)
        f.route = kRouteSyn;  // survivors exactly 0..k-1 (k distinct ids below k), one target in k..2k-1
        f.ms = kMsPerm;
        f.target = tg[0];
        f.plan = bb.plan_of(part, f.seen, f.ms, f.target);
      } else if (ok) {
        f.route = kRouteSyn;
        f.ms = small_ms_for(k, std::max(maxid, tmax));  // (every target an erased point of 0..k+ms-1)
        f.plan = bb.plan_of(part, f.seen, f.ms, 0);
      } else if (batch_ok && fits && maxid < 256 && tmax < 256) {
        f.route = kRouteRt;
        f.parts = (uint8_t)((nt + R - 1) / R);
        f.rows = (uint16_t)nt;
        // (RT descriptors per object: nt / (n - k) rounded up, < 256)
        if ((uint32_t)f.parts * R < nt) {
          err.note(o, VDS_EC_EINVAL);
          info[o] = BatchObjInfo{};
          return;
        }
      } else {
        f.route = kRouteOne;
      }
      info[o] = f;
      tot.add(f);
    }
    ix.part[part] = tot;
  });
  if (err.rc) return err.rc;
  int rc = device_ready();
  if (rc) return rc;
  ht.mark("pass1");
  ix.build();
  RtBatchBuild &rb = sc.rb;
  rb.reset(k, n);
  if ((rc = batch_begin(ix, bb, rb, &ht))) return rc;
  ht.mark("begin");
  parallel_parts(count, [&](unsigned part, uint32_t o0, uint32_t o1) {
    if (ix.all.nsyn && !bb.resolve_plans(part)) {  // (a set with no solve: not for distinct points)
      err.note(o0, VDS_EC_ESINGULAR);
      return;
    }
    uint32_t isyn = ix.base[part].nsyn, irt = ix.base[part].nrt;
    uint64_t row = ix.base[part].rt_rows;
    for (uint32_t o = o0; o < o1; ++o) {
      const BatchObjInfo &f = info[o];
      const uint16_t *nd = nodes + (uint64_t)o * k;
      const uint8_t *const *ch = chunks + (uint64_t)o * k;
      const uint16_t *tg = targets + (uint64_t)o * nt;
      uint8_t *const *os = outs + (uint64_t)o * nt;
      if (f.route == kRouteSyn) {
        SynBatchObj &d = bb.fill(isyn++, f.seen, nd, ch, bb.numbered(f.plan), f.halves);
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
        for (uint32_t p = 0, i0 = 0; p < f.parts; ++p, i0 += R) {
          const uint32_t cnt = std::min(R, nt - i0);
          uint8_t rowp[kMaxFastK / 4];
          for (uint32_t i = 0; i < cnt; ++i) rowp[i] = (uint8_t)tg[i0 + i];
          SynBatchObj &d = rb.fill(irt + p, nd, ch, rowp, cnt, row + i0, f.halves);
          std::memset(d.regen, 0, sizeof d.regen);
          for (uint32_t i = 0; i < cnt; ++i) d.regen[i] = os[i0 + i];
          d.out = nullptr;
          d.out_len = 0;
          d.chunk_len = chunk_sizes[o];
        }
        irt += f.parts;
        row += f.rows;
      }
    }
  });
  if (err.rc) {
    batch_abandon(ix, bb, rb, s);
    return err.rc;
  }
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

}  // namespace api
}  // namespace vds_ec
