// vds_ec_jit.cpp -- pattern-specific restore kernels compiled at run time.
//
// k_restore_syn (ec_restore_syn.hip) serves every survivor set of a compiled
// (k, n) with fixed syndrome programs plus a runtime M x M recovery walk
// (chunk_restore<uint16_t>::restore, chunk.h:290-444).  A repair pass meets
// few survivor sets -- the bench and a node-loss repair meet one -- so for a
// set seen on a non-batch restore this module generates the straight-line
// XOR programs of that set (xorprog.hpp: the value at each erased point below
// k as the Lagrange combination of the survivors, Paar-reduced) and compiles
// the same kernel body with them (hiprtc in the helper process vds_ec_jitc,
// gfx950), in place of the syndromes,
// the recovery walk and its LDS atomics.  Same bytes: the Lagrange
// combination is the unique polynomial through the survivors, as V_S^{-1} is.
//
// Compiles run on one background thread; until a set's kernel is loaded the
// restore keeps using k_restore_syn.  VDS_EC_JIT=0 disables the module,
// VDS_EC_JIT=sync compiles on the calling thread at the first use.  The kernel
// source includes the device headers and the generated interpolation programs,
// embedded in the helper compiler vds_ec_jitc at build time (vds_amd/build.py).
#include <dlfcn.h>
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <spawn.h>
#include <sys/stat.h>
#include <sys/wait.h>
#include <unistd.h>

#include <cerrno>

#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

#include "ec_internal.hpp"
#include "vds_ec.h"
#include "xorprog.hpp"

extern char **environ;

#ifndef VDS_GM2
#define VDS_GM2 1  // (restore_syn.hpp's defaults)
#endif
#ifndef VDS_GM2_PRIO
#define VDS_GM2_PRIO 9
#endif
#ifndef VDS_HALF_PRIO
#define VDS_HALF_PRIO 1
#endif
#ifndef VDS_FILL_REGS
#define VDS_FILL_REGS 1
#endif
#ifndef VDS_DIAG_STAMPS
#define VDS_DIAG_STAMPS 0
#endif
#ifndef VDS_EC_ARCH_STR
#define VDS_EC_ARCH_STR "gfx950"  // (build.py passes the library's architecture)
#endif

namespace vds_ec {
namespace {


constexpr int kJitMaxDev = 64;
constexpr size_t kJitMaxEntries = 256;  // distinct survivor sets kept (never evicted: kernels may be in flight)
// Points per Paar block of the fill programs, and whether a block's LDS reads
// are issued before the previous block's XORs.  k = 16, no spills up to 3
// with prefetch (4 spilled 91 VGPRs) and 4 without; same-box repair, 512 x
// 64 MiB: 2 14.62-14.72 ms, 3 14.52-14.60, 4 without prefetch 14.62
// (profiles/round3/ab/jit_knobs.log).  -DVDS_JIT_PB=n / -DVDS_JIT_PREFETCH=0
// builds override them (A/B).
#ifndef VDS_JIT_PB
#define VDS_JIT_PB 3
#endif
#ifndef VDS_JIT_PREFETCH
#define VDS_JIT_PREFETCH 1
#endif
static_assert(VDS_JIT_PB > 0 && VDS_JIT_PB <= 32, "fill block size");
constexpr int fill_block() { return VDS_JIT_PB; }
constexpr bool fill_prefetch() { return VDS_JIT_PREFETCH != 0; }
// Column-partitioned fill programs (xorprog.hpp emit_fill_scatter; default)
// or the row form (a -DVDS_JIT_SCATTER=0 build, A/B).
#ifndef VDS_JIT_SCATTER
#define VDS_JIT_SCATTER 1
#endif
constexpr bool fill_scatter() { return VDS_JIT_SCATTER != 0; }
// The own-group fill (xorprog.hpp emit_fill_own) for k = 16 sets with one
// erased point in each wave's interpolation group, e.g. the headline set
// {0, 5, 10, 15}: measured slower than the scatter fill and off by default
// (-DVDS_JIT_OWN=1 builds it).  Same box, ABBA, 512 x 64 MiB
// (profiles/round6/ab_own_fill.log): repair 13.15 ms (scatter) against 13.47
// (own, Paar blocks of 3), 13.34 (blocks of 2), 13.56 (no block prefetch);
// blocks of 4 spill 21 VGPRs.  Its 48 ds_read_b128 per lane of the other
// waves' survivors and ~25% more XORs cost more than the barrier and the 32
// ds_xor_b64 atomics per lane they replace.
#ifndef VDS_JIT_OWN
#define VDS_JIT_OWN 0
#endif

// JIT policy: 0 = off, 1 = background compile from a set's second use
// (default), 2 = compile on the calling thread at the first use.  Initially
// from VDS_EC_JIT (0 / off, sync), then vds_ec_jit_set_mode.
std::atomic<int> &jit_mode_ref() {
  static std::atomic<int> m{[] {
    const char *v = std::getenv("VDS_EC_JIT");
    if (!v) return 1;
    if (!std::strcmp(v, "0") || !std::strcmp(v, "off")) return 0;
    if (!std::strcmp(v, "sync")) return 2;
    return 1;
  }()};
  return m;
}
int jit_mode() { return jit_mode_ref().load(std::memory_order_relaxed); }
constexpr int kJitSightings = 2;         // async mode: uses of a set before its compile is queued
constexpr size_t kJitMaxSeen = 1 << 14;  // sighting counts kept (cleared when full)

struct Key {
  uint32_t k, n;
  uint64_t survivors;  // bit a: point a survives
  uint32_t regen = 0;  // 1: the regenerate kernel (targets: every erased point)
  bool operator<(const Key &o) const {
    return std::tie(k, n, survivors, regen) < std::tie(o.k, o.n, o.survivors, o.regen);
  }
};

struct Entry {
  enum State { kPending, kReady, kFailed };
  State state = kPending;  // (Jit::mu_)
  std::vector<char> code;
  std::string log;
  std::string cache_file;  // where `code` came from or went (removed if it fails to load)
  hipModule_t mod[kJitMaxDev] = {};  // (Jit::load_mu_)
  // published with release once loaded; read with acquire without load_mu_
  std::atomic<hipFunction_t> fn[kJitMaxDev] = {};
};

// The kernel's symbol: kind, (k, n) and the survivor mask, so that profiler
// summaries (rocprofv3 --stats) tell the instantiations apart, e.g.
// vds_ec_jit_restore_16_20_f7bde (survivors {1..4, 6..9, 11..14, 16..19}).
std::string kernel_name(const Key &key) {
  char b[96];
  std::snprintf(b, sizeof b, "vds_ec_jit_%s_%u_%u_%llx", key.regen ? "regen" : "restore", key.k, key.n,
                (unsigned long long)key.survivors);
  return b;
}

// The kernel source for one survivor set.
std::string kernel_source(const Key &key) {
  const int K = (int)key.k, N = (int)key.n, WV = K / 4;
  std::vector<int> sp;
  for (int a = 0; a < N; ++a)
    if ((key.survivors >> a) & 1u) sp.push_back(a);
  std::string s;
  xorgen::appendf(s,
                  "#define VDS_GM2 %d\n#define VDS_GM2_PRIO %d\n#define VDS_HALF_PRIO %d\n"
                  "#define VDS_FILL_REGS %d\n",
                  VDS_GM2, VDS_GM2_PRIO, VDS_HALF_PRIO, VDS_FILL_REGS);  // (the forms this library was built with)
#if VDS_DIAG_STAMPS
  xorgen::appendf(s, "#define VDS_DIAG_STAMPS 1\n");  // (phase stamps: vds_ec_diag_jit_stamps)
#endif
#if defined(VDS_DIAG_LOADS) && VDS_DIAG_LOADS
  xorgen::appendf(s, "#define VDS_DIAG_LOADS %d\n", VDS_DIAG_LOADS);  // (load study, restore_syn.hpp)
#endif
  xorgen::appendf(s, "#define VDS_SCHED_FENCE() __builtin_amdgcn_sched_barrier(0)\n#include \"restore_syn.hpp\"\n");
  xorgen::appendf(s, "namespace vds_ec {\n#include \"generated/restore_%d_%d_w%d.inc\"\n", K, N, WV);
  if (key.regen) {  // every erased point, in ascending order (= SynRestoreArgs::erased)
    std::vector<int> tg;
    for (int a = 0; a < N; ++a)
      if (!((key.survivors >> a) & 1u)) tg.push_back(a);
    xorgen::emit_fill_scatter(s, "JitFill", K, sp, &tg);
  } else if (VDS_JIT_OWN && xorgen::fill_own_eligible(K, sp)) {
    xorgen::emit_fill_own(s, "JitFill", K, sp, fill_block(), fill_prefetch());
  } else if (fill_scatter()) {
    xorgen::emit_fill_scatter(s, "JitFill", K, sp);
  } else {
    xorgen::emit_fill_programs(s, "JitFill", K, sp, fill_block(), fill_prefetch());
  }
  xorgen::appendf(s, "}  // namespace vds_ec\n");
  xorgen::appendf(s,
                  "extern \"C\" __global__ __launch_bounds__((vds_ec::SynShape<%d, %d, %d>::kThreads), "
                  "(vds_ec::SynShape<%d, %d, %d>::kWavesPerSimd))\n"
                  "void %s(vds_ec::SynRestoreArgs a) {\n"
                  "  vds_ec::restore_syn_body<%d, %d, %d, %s, false, false, vds_ec::JitFill>(a);\n}\n",
                  K, N, WV, K, N, WV, kernel_name(key).c_str(), K, N, WV, key.regen ? "true" : "false");
  return s;
}

// The helper compiler next to this library (vds_ec_jitc.cpp says why it is a
// separate process).
std::string helper_path() {
  Dl_info info{};
  if (!dladdr(reinterpret_cast<void *>(&helper_path), &info) || !info.dli_fname) return {};
  std::string p = info.dli_fname;
  const size_t slash = p.rfind('/');
  return (slash == std::string::npos ? std::string(".") : p.substr(0, slash)) + "/vds_ec_jitc";
}

std::string read_file(const std::string &path) {
  std::string out;
  if (FILE *f = std::fopen(path.c_str(), "rb")) {
    char buf[65536];
    size_t n;
    while ((n = std::fread(buf, 1, sizeof buf, f)) > 0) out.append(buf, n);
    std::fclose(f);
  }
  return out;
}

// On-disk cache of compiled kernels, shared by processes (e.g. the ranks of
// one node): $VDS_EC_JIT_CACHE, else $XDG_CACHE_HOME/vds_ec, else
// $HOME/.cache/vds_ec; VDS_EC_JIT_CACHE=0 disables it.  A file is named by a
// hash of the kernel source (which carries the programs and every build
// switch) and of the helper's size and mtime (which carries the embedded
// device headers); it is written to a temporary name and renamed, so readers
// never see a partial file.
std::string cache_dir() {
  static const std::string d = [] {
    const char *v = std::getenv("VDS_EC_JIT_CACHE");
    if (v && !std::strcmp(v, "0")) return std::string();
    std::string dir;
    if (v && *v) {
      dir = v;
    } else if (const char *x = std::getenv("XDG_CACHE_HOME"); x && *x) {
      dir = std::string(x) + "/vds_ec";
    } else if (const char *h = std::getenv("HOME"); h && *h) {
      dir = std::string(h) + "/.cache";
      (void)mkdir(dir.c_str(), 0700);
      dir += "/vds_ec";
    } else {
      return std::string();
    }
    (void)mkdir(dir.c_str(), 0700);
    return access(dir.c_str(), W_OK) == 0 ? dir : std::string();
  }();
  return d;
}

uint64_t fnv1a(const void *p, size_t n, uint64_t h = 1469598103934665603ull) {
  const unsigned char *b = static_cast<const unsigned char *>(p);
  for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 1099511628211ull;
  return h;
}

// The cache key: the kernel source, the target architecture and the helper's
// size and mtime.
uint64_t cache_key(const std::string &src, const std::string &helper) {
  struct stat st {};
  if (stat(helper.c_str(), &st) != 0) return 0;
  uint64_t h = fnv1a(src.data(), src.size());
  h = fnv1a(VDS_EC_ARCH_STR, sizeof VDS_EC_ARCH_STR, h);
  const int64_t id[2] = {(int64_t)st.st_size, (int64_t)st.st_mtime};
  return fnv1a(id, sizeof id, h) | 1u;  // (0: no key)
}

std::string cache_path(uint64_t key) {
  const std::string dir = cache_dir();
  if (dir.empty() || key == 0) return {};
  char name[64];
  std::snprintf(name, sizeof name, "/%016llx.co", (unsigned long long)key);
  return dir + name;
}

// A cache file is this header, then the code object.  A file whose header
// does not match (another key, a short or foreign file, damaged bytes) is a
// miss, and is removed: the cache directory may be shared, so nothing in it
// is trusted until its key, length and checksum agree.
struct CacheHeader {
  char magic[8];   // "VDSECJ1"
  uint64_t key;    // cache_key of the source it was compiled from
  uint64_t bytes;  // code object length
  uint64_t sum;    // fnv1a of the code object
};
constexpr char kCacheMagic[8] = "VDSECJ1";

bool cache_read(const std::string &path, uint64_t key, std::vector<char> &code) {
  const std::string f = read_file(path);
  if (f.empty()) return false;
  CacheHeader h{};
  bool ok = f.size() > sizeof h;
  if (ok) {
    std::memcpy(&h, f.data(), sizeof h);
    ok = !std::memcmp(h.magic, kCacheMagic, sizeof h.magic) && h.key == key && h.bytes == f.size() - sizeof h &&
         h.sum == fnv1a(f.data() + sizeof h, h.bytes);
  }
  if (!ok) {
    (void)std::remove(path.c_str());
    return false;
  }
  code.assign(f.begin() + sizeof h, f.end());
  return true;
}

// Written to a unique temporary name in the cache directory (mkstemp), then
// renamed: concurrent writers of one key never share a file, and readers see
// a whole file or none.
void cache_write(const std::string &path, uint64_t key, const std::vector<char> &code) {
  std::string tmp = path + ".XXXXXX";
  const int fd = mkstemp(&tmp[0]);
  if (fd < 0) return;
  CacheHeader h{};
  std::memcpy(h.magic, kCacheMagic, sizeof h.magic);
  h.key = key;
  h.bytes = code.size();
  h.sum = fnv1a(code.data(), code.size());
  bool ok = write(fd, &h, sizeof h) == (ssize_t)sizeof h;
  for (size_t at = 0; ok && at < code.size();) {
    const ssize_t w = write(fd, code.data() + at, code.size() - at);
    ok = w > 0;
    if (ok) at += (size_t)w;
  }
  ok = (close(fd) == 0) && ok;
  if (!ok || std::rename(tmp.c_str(), path.c_str()) != 0) (void)std::remove(tmp.c_str());
}

// Compile one survivor set's kernel with the helper (host only: no device
// needed): source and code object pass through a private temporary directory.
bool compile(const Key &key, std::vector<char> &code, std::string &log, std::string *cache_file = nullptr) {
  const std::string src = kernel_source(key);
  const std::string helper = helper_path();
  if (helper.empty() || access(helper.c_str(), X_OK) != 0) {
    log = "vds_ec_jitc not found next to libvds_ec.so";
    return false;
  }
  const uint64_t ckey = cache_key(src, helper);
  const std::string cached = cache_path(ckey);
  if (cache_file) *cache_file = cached;
  if (!cached.empty() && cache_read(cached, ckey, code)) return true;
  const char *tmpenv = std::getenv("TMPDIR");
  std::string dir = std::string(tmpenv && *tmpenv ? tmpenv : "/tmp") + "/vds_ec_jit_XXXXXX";
  if (!mkdtemp(&dir[0])) {
    log = "mkdtemp failed";
    return false;
  }
  const std::string in = dir + "/k.hip", out = dir + "/k.co", err = dir + "/log.txt";
  bool ok = false;
  if (FILE *f = std::fopen(in.c_str(), "w")) {
    ok = std::fwrite(src.data(), 1, src.size(), f) == src.size();
    ok = (std::fclose(f) == 0) && ok;
  }
  if (ok) {
    // a child process (posix_spawn), stderr into the log file
    posix_spawn_file_actions_t fa;
    posix_spawn_file_actions_init(&fa);
    posix_spawn_file_actions_addopen(&fa, 2, err.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0600);
    std::vector<char *> argv = {const_cast<char *>(helper.c_str()), const_cast<char *>(in.c_str()),
                                const_cast<char *>(out.c_str()), nullptr};
    pid_t pid = 0;
    ok = posix_spawn(&pid, helper.c_str(), &fa, nullptr, argv.data(), environ) == 0;
    posix_spawn_file_actions_destroy(&fa);
    int status = 0;
    if (ok) {
      while (waitpid(pid, &status, 0) < 0 && errno == EINTR) {
      }
      ok = WIFEXITED(status) && WEXITSTATUS(status) == 0;
    }
    log = read_file(err);
    if (ok) {
      const std::string bytes = read_file(out);
      code.assign(bytes.begin(), bytes.end());
      ok = !code.empty();
    }
  }
  std::remove(in.c_str());
  std::remove(out.c_str());
  std::remove(err.c_str());
  rmdir(dir.c_str());
  if (ok && !cached.empty()) cache_write(cached, ckey, code);  // (best effort)
  return ok;
}

// vds_ec_jit_dump16: the set's source and code object under `dir`.
bool dump(const Key &key, const char *dir) {
  std::vector<char> code;
  std::string log;
  if (!compile(key, code, log)) {
    std::fprintf(stderr, "vds_ec jit: compile failed:\n%s\n", log.c_str());
    return false;
  }
  const std::string src = kernel_source(key);
  char base[512];
  std::snprintf(base, sizeof base, "%s/jit_%u_%u_%llx%s", dir, key.k, key.n, (unsigned long long)key.survivors,
                key.regen ? "_regen" : "");
  bool ok = false;
  if (FILE *f = std::fopen((std::string(base) + ".hip").c_str(), "w")) {
    ok = std::fwrite(src.data(), 1, src.size(), f) == src.size();
    ok = (std::fclose(f) == 0) && ok;
  }
  if (FILE *f = std::fopen((std::string(base) + ".co").c_str(), "wb")) {
    ok = (std::fwrite(code.data(), 1, code.size(), f) == code.size()) && ok;
    ok = (std::fclose(f) == 0) && ok;
  } else {
    ok = false;
  }
  return ok;
}

class Jit {
 public:
  // Never destroyed (as HostPool): threads may still be inside function() at
  // exit, and the worker may be waiting on a helper compile; it is detached.
  static Jit &get() {
    static Jit *j = new Jit();
    return *j;
  }

  // The loaded kernel of `key` on the current device, or nullptr (not
  // compiled yet -- then queued -- or failed).
  hipFunction_t function(const Key &key) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kJitMaxDev) return nullptr;
    std::shared_ptr<Entry> e;
    {
      std::unique_lock<std::mutex> lk(mu_);
      auto it = map_.find(key);
      if (it == map_.end()) {
        if (map_.size() >= kJitMaxEntries) return nullptr;
        const bool sync = jit_mode() == 2;
        if (!sync) {  // one-off sets are not worth a compile
          if (seen_.size() >= kJitMaxSeen) seen_.clear();
          if (++seen_[key] < kJitSightings) return nullptr;
          seen_.erase(key);
        }
        e = std::make_shared<Entry>();
        map_.emplace(key, e);
        if (sync) {
          lk.unlock();
          run(key, e);
          lk.lock();
        } else {
          queue_.push_back(key);
          start_worker();
          cv_.notify_all();
          return nullptr;
        }
      } else {
        e = it->second;
      }
      if (e->state != Entry::kReady) return nullptr;
      if (hipFunction_t f = e->fn[dev].load(std::memory_order_acquire)) return f;
    }
    // first use on this device: load the code object (once per device)
    std::lock_guard<std::mutex> g(load_mu_);
    if (hipFunction_t f = e->fn[dev].load(std::memory_order_acquire)) return f;
    hipModule_t m = nullptr;
    hipFunction_t f = nullptr;
    if (hipModuleLoadData(&m, e->code.data()) != hipSuccess ||
        hipModuleGetFunction(&f, m, kernel_name(key).c_str()) != hipSuccess) {
      if (m) (void)hipModuleUnload(m);
      // remembered (the syndrome kernel serves the set from now on), and the
      // cached file that gave it is dropped so the next process recompiles
      std::lock_guard<std::mutex> lk(mu_);
      e->state = Entry::kFailed;
      if (!e->cache_file.empty()) (void)std::remove(e->cache_file.c_str());
      return nullptr;
    }
    e->mod[dev] = m;
    e->fn[dev].store(f, std::memory_order_release);
    return f;
  }

  bool ready(const Key &key) {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = map_.find(key);
    return it != map_.end() && it->second->state == Entry::kReady;
  }

  // Wait until no compile is queued or running.
  void wait() {
    std::unique_lock<std::mutex> lk(mu_);
    idle_cv_.wait(lk, [&] { return queue_.empty() && busy_ == 0; });
  }

#if VDS_DIAG_STAMPS
  // The module of `key` on the current device (diagnostic stamps readout).
  hipModule_t module(const Key &key) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kJitMaxDev) return nullptr;
    std::shared_ptr<Entry> e;
    {
      std::lock_guard<std::mutex> lk(mu_);
      auto it = map_.find(key);
      if (it == map_.end()) return nullptr;
      e = it->second;
    }
    std::lock_guard<std::mutex> g(load_mu_);
    return e->mod[dev];
  }
#endif

  // Compile-only (no device): the code object size of `key`'s kernel.
  bool build(const Key &key, size_t *bytes, std::string *log) {
    std::vector<char> code;
    std::string l;
    const bool ok = compile(key, code, l);
    if (bytes) *bytes = ok ? code.size() : 0;
    if (log) *log = l;
    return ok;
  }

 private:
  void run(const Key &key, const std::shared_ptr<Entry> &e) {
    std::vector<char> code;
    std::string log, file;
    const bool ok = compile(key, code, log, &file);
    std::lock_guard<std::mutex> lk(mu_);
    e->code.swap(code);
    e->log.swap(log);
    e->cache_file.swap(file);
    e->state = ok ? Entry::kReady : Entry::kFailed;
  }

  void start_worker() {  // (mu_ held)
    if (worker_started_) return;
    worker_ = std::thread([this] {
      std::unique_lock<std::mutex> lk(mu_);
      while (true) {
        cv_.wait(lk, [&] { return !queue_.empty(); });
        const Key key = queue_.front();
        queue_.pop_front();
        std::shared_ptr<Entry> e = map_[key];
        ++busy_;
        lk.unlock();
        run(key, e);
        lk.lock();
        --busy_;
        if (queue_.empty() && busy_ == 0) idle_cv_.notify_all();
      }
    });
    worker_.detach();
    worker_started_ = true;
  }

  std::mutex mu_, load_mu_;
  std::condition_variable cv_, idle_cv_;
  std::map<Key, std::shared_ptr<Entry>> map_;
  std::map<Key, int> seen_;
  std::deque<Key> queue_;
  std::thread worker_;
  bool worker_started_ = false;
  int busy_ = 0;
};

Key key_of(uint32_t k, uint32_t n, const uint8_t *points, bool regen) {
  Key key{k, n, 0, regen ? 1u : 0u};
  for (uint32_t j = 0; j < k; ++j) key.survivors |= 1ull << points[j];
  return key;
}

}  // namespace

bool jit_enabled() { return jit_mode() != 0; }

hipFunction_t jit_restore_function(uint32_t k, uint32_t n, const SynRestoreArgs &a, bool regen) {
  if (jit_mode() == 0 || !has_restore_syn(k, n)) return nullptr;
  return Jit::get().function(key_of(k, n, a.point, regen));
}

bool jit_ready(uint32_t k, uint32_t n, const SynRestoreArgs &a, bool regen) {
  return jit_mode() != 0 && has_restore_syn(k, n) && Jit::get().ready(key_of(k, n, a.point, regen));
}

}  // namespace vds_ec

using namespace vds_ec;

extern "C" {

int vds_ec_jit_set_mode(int mode) {
  if (mode < 0 || mode > 2) return VDS_EC_EINVAL;
  jit_mode_ref().store(mode, std::memory_order_relaxed);
  return VDS_EC_OK;
}

int vds_ec_jit_wait(void) {
  Jit::get().wait();
  return VDS_EC_OK;
}

// Survivors as replica ids; EINVAL unless they are k distinct points of
// 0..k+k/4-1 for a compiled (k, k + k/4).
static int jit_key(uint16_t k, const uint16_t *nodes, Key *key) {
  const uint32_t n = k + k / 4u;
  if (!nodes || k == 0 || k % 4 || !has_restore_syn(k, n)) return VDS_EC_EINVAL;
  *key = Key{k, n, 0};
  for (uint32_t j = 0; j < k; ++j) {
    if (nodes[j] >= n || ((key->survivors >> nodes[j]) & 1u)) return VDS_EC_EINVAL;
    key->survivors |= 1ull << nodes[j];
  }
  return VDS_EC_OK;
}

int vds_ec_jit_build16(uint16_t k, const uint16_t *nodes, uint64_t *code_bytes) {
  Key key;
  const int rc = jit_key(k, nodes, &key);
  if (rc) return rc;
  size_t bytes = 0;
  std::string log;
  if (!Jit::get().build(key, &bytes, &log)) {
    std::fprintf(stderr, "vds_ec jit: compile failed:\n%s\n", log.c_str());
    return VDS_EC_EHIP;
  }
  if (code_bytes) *code_bytes = bytes;
  return VDS_EC_OK;
}

#if VDS_DIAG_STAMPS
// Diagnostic build: the phase stamps (restore_syn.hpp Stamps) of survivor set
// `nodes`' run-time kernel, from its module's own g_syn_stamps.
int vds_ec_diag_jit_stamps(uint16_t k, const uint16_t *nodes, unsigned long long *host, size_t n) {
  Key key;
  if (jit_key(k, nodes, &key)) return VDS_EC_EINVAL;
  hipModule_t m = Jit::get().module(key);
  if (!m) return VDS_EC_EINVAL;
  hipDeviceptr_t d = nullptr;
  size_t bytes = 0;
  if (hipModuleGetGlobal(&d, &bytes, m, "_ZN6vds_ec12g_syn_stampsE") != hipSuccess) return VDS_EC_EHIP;
  if (n * sizeof(unsigned long long) > bytes) n = bytes / sizeof(unsigned long long);
  return hipMemcpyDtoH(host, d, n * sizeof(unsigned long long)) == hipSuccess ? VDS_EC_OK : VDS_EC_EHIP;
}
#endif

int vds_ec_jit_ready16(uint16_t k, const uint16_t *nodes) {
  Key key;
  if (jit_key(k, nodes, &key)) return 0;
  return Jit::get().ready(key) ? 1 : 0;
}

int vds_ec_jit_dump16(uint16_t k, const uint16_t *nodes, int regen, const char *dir) {
  Key key;
  if (!dir || jit_key(k, nodes, &key)) return VDS_EC_EINVAL;
  key.regen = regen ? 1u : 0u;
  return dump(key, dir) ? VDS_EC_OK : VDS_EC_EHIP;
}

}  // extern "C"
