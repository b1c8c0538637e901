// api_param_ring.cpp -- the stream-ordered parameter ring of the *_device entry points.
// (api_internal.hpp lists the host runtime's translation units.)
#include "api_internal.hpp"

namespace vds_ec {
namespace api {

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

}  // namespace api
}  // namespace vds_ec
