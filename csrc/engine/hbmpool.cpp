// HBM page pool (see hbmpool.h).
#include "hbmpool.h"

#include <c10/util/Exception.h>
#include <torch/csrc/cuda/CUDAPluggableAllocator.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <set>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <tuple>
#include <mutex>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "guard.h"
#include "guardalloc.h"

namespace mrh::hbm {

namespace {

constexpr int kMaxDev = 64;

// size classes: 512 B granules up to 4 KiB, then 8 classes per power of two
// (at most 12.5 % rounding) — a freed block is reused by any later request
// of its class on its stream
int64_t class_bytes(size_t size) {
  if (size <= 4096) return (int64_t)((size + 511) / 512 * 512);
  int b = 64 - __builtin_clzll((unsigned long long)(size - 1));  // 2^b >= size > 2^(b-1)
  const int64_t step = std::max<int64_t>(512, (int64_t(1) << (b - 1)) / 8);
  return ((int64_t)size + step - 1) / step * step;
}

struct Block {
  int64_t bytes = 0;
  int dev = 0;
  hipStream_t stream = nullptr;
  std::vector<hipStream_t> used_on;  // other streams that touched the block (record_stream)
  struct Seg* seg = nullptr;         // big blocks: the arena segment and offset they were cut from
  int64_t off = 0;
};

// an event recorded when a big block was freed, shared by the free ranges cut
// from or merged with it; a later user on any stream waits for it
struct Ev {
  hipEvent_t e = nullptr;
  ~Ev() {
    if (e) (void)hipEventDestroy(e);
  }
};
using EvP = std::shared_ptr<Ev>;

// Big blocks (>= kBigBlock) are cut best-fit from hipMalloc'd segments and
// coalesce with their free neighbours when freed, so the memory a job held
// at its peak serves any later mix of sizes (R-MAT-22's collate: 56, 28, 7 GB
// pieces) instead of growing the device allocation for every new size; fully
// free segments go back to the driver only when the pool holds much more
// than it uses (reserved > 1.5x in use).
struct FreeRange {
  int64_t size = 0;
  std::vector<EvP> evs;  // the frees this range's memory waits for
};
struct Seg {
  char* base = nullptr;
  int64_t size = 0;
  int64_t free_bytes = 0;
  std::map<int64_t, FreeRange> free;  // offset -> free range (coalesced)
};

// a freed block that other streams used: reusable once their events complete
struct Pending {
  void* p = nullptr;
  Block b;
  std::vector<hipEvent_t> evs;
};

struct Dev {
  hipMemPool_t pool = nullptr;
  int64_t in_use = 0, peak = 0, cap = 0, cached = 0, allocs = 0, frees = 0, failures = 0, cross = 0;
  int64_t grows = 0, releases = 0, oom_retries = 0;
  double grow_ms = 0;
  // blocks of >= kBigBlock come from hipMalloc'd segments, not the HIP pool:
  // re-growing the stream-ordered pool by tens of GB after its free memory
  // came back in other sizes took seconds (a 30 GB concat of tri_find_mr:
  // 4.5 s). They are cut best-fit from the segments and coalesce when freed.
  int64_t big_bytes = 0;     // held by the big-block segments (live + free): part of reserved
  int64_t big_peak = 0;
  std::vector<std::unique_ptr<Seg>> segs;
  std::set<std::tuple<int64_t, Seg*, int64_t>> by_size;  // (size, segment, offset) of every free range
  int64_t big_free = 0;                                   // free bytes inside the segments
  int64_t reserved_peak_true = 0;                         // hi-water of (HIP pool reserved + segments)
  int64_t total_mem = 0;     // device memory (hipMemGetInfo at the first growth)
  int64_t base_cap = 0;                   // set_cap's cap; cap = min(base_cap, active OpCaps)
  std::multiset<int64_t> op_caps;         // caps of the ops running now (any thread)
  std::map<std::pair<hipStream_t, int64_t>, std::vector<void*>> free;  // (stream, class) -> cached blocks
  std::vector<hipStream_t> streams;       // every stream with a cache entry
  std::vector<Pending> pending;
  // sticky: an event or stream wait of the pool failed (a device fault), so
  // no cached block can be trusted any more — every later allocation fails
  std::string fault;
};

void recompute_cap(Dev& d) {  // g_mu held
  int64_t c = d.base_cap;
  if (!d.op_caps.empty()) c = c > 0 ? std::min(c, *d.op_caps.begin()) : *d.op_caps.begin();
  d.cap = c;
}

// the pool cannot vouch for its blocks any more: record why (first fault
// wins), and the caller keeps the block out of every cache (leaked)
void set_fault(Dev& d, const std::string& why) {  // g_mu held
  if (d.fault.empty()) d.fault = why;
  ++d.failures;
}

void cache_put(Dev& d, hipStream_t s, int64_t bytes, void* p) {  // g_mu held
  d.free[{s, bytes}].push_back(p);
  if (std::find(d.streams.begin(), d.streams.end(), s) == d.streams.end()) d.streams.push_back(s);
}

int process_rank() {
  static const int r = [] {
    const char* e = std::getenv("RANK");
    return e && *e ? std::atoi(e) : 0;
  }();
  return r;
}

std::mutex g_mu;
Dev g_dev[kMaxDev];
std::unordered_map<void*, Block> g_blocks;
std::atomic<bool> g_installed{false};

std::string mib(int64_t b) {
  return b >= (int64_t(1) << 20) ? std::to_string(b >> 20) + " MiB" : std::to_string(b >> 10) + " KiB";
}

hipMemPool_t pool_of(int dev) {  // g_mu held
  Dev& d = g_dev[dev];
  if (d.pool) return d.pool;
  hipMemPoolProps p{};
  p.allocType = hipMemAllocationTypePinned;
  p.handleTypes = hipMemHandleTypeNone;
  p.location.type = hipMemLocationTypeDevice;
  p.location.id = dev;
  hipError_t e = hipMemPoolCreate(&d.pool, &p);
  TORCH_CHECK(e == hipSuccess, "mrhip page pool: hipMemPoolCreate failed on device ", dev, ": ", hipGetErrorString(e));
  // keep freed memory in the pool (pages are reused, not returned per op);
  // trim() gives it back
  uint64_t keep = UINT64_MAX;
  e = hipMemPoolSetAttribute(d.pool, hipMemPoolAttrReleaseThreshold, &keep);
  TORCH_CHECK(e == hipSuccess, "mrhip page pool: hipMemPoolSetAttribute failed: ", hipGetErrorString(e));
  return d.pool;
}

// pending blocks whose other-stream work is done go to their stream's cache;
// an event that reports an error (not "not ready") faults the pool and its
// block is never handed out again
void reap(Dev& d) {  // g_mu held
  for (size_t i = 0; i < d.pending.size();) {
    Pending& q = d.pending[i];
    bool done = true, bad = false;
    for (hipEvent_t e : q.evs) {
      const hipError_t r = hipEventQuery(e);
      if (r == hipErrorNotReady) {
        done = false;
        break;
      }
      if (r != hipSuccess) {
        (void)hipGetLastError();
        set_fault(d, std::string("event of a block used on another stream: ") + hipGetErrorString(r));
        bad = true;
      }
    }
    if (!done) {
      ++i;
      continue;
    }
    for (hipEvent_t e : q.evs) (void)hipEventDestroy(e);
    if (bad) d.cached -= q.b.bytes;  // leaked on purpose: other streams may still use it
    else cache_put(d, q.b.stream, q.b.bytes, q.p);
    q = std::move(d.pending.back());
    d.pending.pop_back();
  }
}

// every cached block back to the HIP pool (then the pool can hand the memory
// to any stream, or trim it to the driver)
constexpr int64_t kBigBlock = int64_t(256) << 20;

void release_cached(Dev& d) {  // g_mu held
  ++d.releases;
  for (Pending& q : d.pending) {
    bool ok = true;
    for (hipEvent_t e : q.evs) {
      // the block goes back to the HIP pool on its own stream behind the other
      // streams' events; a failed wait would free memory still in use
      const hipError_t r = hipStreamWaitEvent(q.b.stream, e, 0);
      if (r != hipSuccess) {
        (void)hipGetLastError();
        set_fault(d, std::string("stream wait before releasing a block: ") + hipGetErrorString(r));
        ok = false;
      }
      (void)hipEventDestroy(e);
    }
    if (ok) cache_put(d, q.b.stream, q.b.bytes, q.p);
  }
  d.pending.clear();
  for (auto& [k, v] : d.free)
    for (void* p : v) {
      if (hipFreeAsync(p, k.first) != hipSuccess) {
        (void)hipGetLastError();
        const hipError_t r = hipDeviceSynchronize();
        if (r != hipSuccess) {  // a sticky device fault: nothing can be freed safely
          (void)hipGetLastError();
          set_fault(d, std::string("device fault while releasing cached blocks: ") + hipGetErrorString(r));
          continue;
        }
        (void)hipFreeAsync(p, nullptr);
      }
    }
  d.free.clear();
  d.streams.clear();
  d.cached = 0;
}

// a cached block of this class on another stream, made safe for `stream` by
// an event of the stream it was freed on (bounds the reserved memory: blocks
// freed on the copy streams feed the compute stream and vice versa)
void* take_other_stream(Dev& d, hipStream_t stream, int64_t bytes) {  // g_mu held
  for (hipStream_t s : d.streams) {
    if (s == stream) continue;
    auto it = d.free.find({s, bytes});
    if (it == d.free.end() || it->second.empty()) continue;
    hipEvent_t ev = nullptr;
    hipError_t r = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    if (r == hipSuccess) r = hipEventRecord(ev, s);
    if (r == hipSuccess) r = hipStreamWaitEvent(stream, ev, 0);
    if (ev) (void)hipEventDestroy(ev);  // released once the wait no longer needs it
    if (r != hipSuccess) {
      (void)hipGetLastError();
      set_fault(d, std::string("cross-stream reuse event: ") + hipGetErrorString(r));
      return nullptr;
    }
    void* p = it->second.back();
    it->second.pop_back();
    ++d.cross;
    return p;
  }
  return nullptr;
}

constexpr int64_t kSegAlign = int64_t(2) << 20;   // big blocks: 2 MiB granules
constexpr int64_t kSegMin = int64_t(2) << 30;     // a new segment holds at least 2 GiB

int64_t pool_reserved(Dev& d) {  // g_mu held
  uint64_t r = 0;
  if (d.pool && hipMemPoolGetAttribute(d.pool, hipMemPoolAttrReservedMemCurrent, &r) != hipSuccess) {
    (void)hipGetLastError();
    r = 0;
  }
  return (int64_t)r + d.big_bytes;
}

void note_reserved(Dev& d) {  // g_mu held
  d.reserved_peak_true = std::max(d.reserved_peak_true, pool_reserved(d));
}

void range_add(Dev& d, Seg* sg, int64_t off, int64_t size, std::vector<EvP> evs) {  // g_mu held
  // coalesce with the free neighbours (their events join: a user waits for all)
  auto nx = sg->free.lower_bound(off);
  if (nx != sg->free.end() && nx->first == off + size) {
    d.by_size.erase({nx->second.size, sg, nx->first});
    size += nx->second.size;
    for (auto& e : nx->second.evs) evs.push_back(e);
    nx = sg->free.erase(nx);
  }
  if (nx != sg->free.begin()) {
    auto pv = std::prev(nx);
    if (pv->first + pv->second.size == off) {
      d.by_size.erase({pv->second.size, sg, pv->first});
      off = pv->first;
      size += pv->second.size;
      for (auto& e : pv->second.evs) evs.push_back(e);
      sg->free.erase(pv);
    }
  }
  // completed events need no wait; drop them (and duplicates) to keep lists short
  std::vector<EvP> live;
  for (auto& e : evs) {
    if (!e || std::find(live.begin(), live.end(), e) != live.end()) continue;
    const hipError_t r = hipEventQuery(e->e);
    if (r == hipSuccess) continue;
    if (r != hipErrorNotReady) (void)hipGetLastError();
    live.push_back(e);
  }
  sg->free[off] = FreeRange{size, std::move(live)};
  d.by_size.insert({size, sg, off});
}

// best fit among the free ranges; the rest of the range stays free
void* arena_take(Dev& d, int64_t bytes, hipStream_t stream, Seg** seg, int64_t* off) {  // g_mu held
  auto it = d.by_size.lower_bound({bytes, nullptr, 0});
  if (it == d.by_size.end()) return nullptr;
  auto [size, sg, o] = *it;
  d.by_size.erase(it);
  auto fr = sg->free.find(o);
  std::vector<EvP> evs = std::move(fr->second.evs);
  sg->free.erase(fr);
  for (auto& e : evs) {  // the block's earlier users (any stream) finish first
    if (hipStreamWaitEvent(stream, e->e, 0) != hipSuccess) {
      (void)hipGetLastError();
      set_fault(d, "stream wait on a freed big block");
      return nullptr;
    }
  }
  if (size > bytes) range_add(d, sg, o + bytes, size - bytes, evs);
  sg->free_bytes -= bytes;
  d.big_free -= bytes;
  *seg = sg;
  *off = o;
  return sg->base + o;
}

// segments with nothing in use leave the pool's books (g_mu held); the caller
// hands them back to the driver with free_segments() AFTER dropping g_mu: the
// waits for their last users and the synchronous hipFree would otherwise stall
// every allocation and free of every thread and stream behind them
std::vector<std::unique_ptr<Seg>> detach_free_segments(Dev& d) {  // g_mu held
  std::vector<std::unique_ptr<Seg>> out;
  for (size_t i = 0; i < d.segs.size();) {
    Seg* sg = d.segs[i].get();
    if (sg->free_bytes != sg->size) {
      ++i;
      continue;
    }
    for (auto& [o, fr] : sg->free) d.by_size.erase({fr.size, sg, o});
    d.big_bytes -= sg->size;
    d.big_free -= sg->size;
    out.push_back(std::move(d.segs[i]));
    d.segs.erase(d.segs.begin() + (std::ptrdiff_t)i);
    ++d.releases;
  }
  return out;
}

// g_mu NOT held: wait for each detached segment's last users, then free it
void free_segments(std::vector<std::unique_ptr<Seg>>& segs) {
  for (auto& sg : segs) {
    for (auto& [o, fr] : sg->free)
      for (auto& e : fr.evs)
        if (hipEventSynchronize(e->e) != hipSuccess) (void)hipGetLastError();
    if (hipFree(sg->base) != hipSuccess) (void)hipGetLastError();
  }
  segs.clear();
}

void* pool_alloc(size_t size, int dev, hipStream_t stream) {
  if (size == 0) return nullptr;
  TORCH_CHECK(dev >= 0 && dev < kMaxDev, "mrhip page pool: device index out of range");
  const int64_t bytes = class_bytes(size);
  static const bool fault_armed = [] {
    const char* e = std::getenv("MRH_FAULT");
    return e && std::strncmp(e, "hip:pool:", 9) == 0;
  }();
  hipMemPool_t pool;
  {
    std::unique_lock<std::mutex> l(g_mu);
    Dev& d = g_dev[dev];
    if (fault_armed) {  // MRH_FAULT=hip:pool:<rank>[:nth]: the nth allocation finds the pool faulted
      try {
        guard::hip_check(hipSuccess, "pool", process_rank());
      } catch (const std::exception& ex) {
        set_fault(d, ex.what());
      }
    }
    if (!d.fault.empty())
      TORCH_CHECK(false, "mrhip page pool: device ", dev, " is unusable after an earlier fault (", d.fault,
                  "); no allocation is served");
    if (d.cap > 0 && d.in_use + bytes > d.cap) {
      ++d.failures;
      TORCH_CHECK_WITH(OutOfMemoryError, false, "mrhip page pool: Cannot allocate page: ", mib(bytes),
                       " requested with ", mib(d.in_use), " in use of a cap of ", mib(d.cap),
                       " (maxpage x memsize / hbm_budget) on device ", dev, " in ", guard::current_op());
    }
    if (!d.pending.empty()) reap(d);
    if (bytes >= kBigBlock) {
      const int64_t bb = (bytes + kSegAlign - 1) / kSegAlign * kSegAlign;
      Seg* sg = nullptr;
      int64_t off = 0;
      void* p = arena_take(d, bb, stream, &sg, &off);
      if (!p && !d.fault.empty()) TORCH_CHECK(false, "mrhip page pool: device ", dev, " faulted: ", d.fault);
      if (!p) {
        // a new segment: first hand back what the pool holds beyond 1.5x its
        // use. The driver calls (waits for the freed segments' users,
        // hipFree, hipMalloc) run with g_mu dropped; the block's bytes are
        // counted in use meanwhile so concurrent allocations see them
        std::vector<std::unique_ptr<Seg>> drop;
        if (pool_reserved(d) + std::max(bb, kSegMin) > (d.in_use + bb) * 3 / 2) {
          drop = detach_free_segments(d);
          if (d.cached > (int64_t(1) << 30)) release_cached(d);
        }
        d.in_use += bb;
        const auto t0 = std::chrono::steady_clock::now();
        int64_t segsz = std::max(bb, kSegMin);
        char* base = nullptr;
        l.unlock();
        free_segments(drop);
        hipError_t e = hipMalloc((void**)&base, (size_t)segsz);
        if (e != hipSuccess && segsz > bb) {  // no room for the margin: exactly the block
          (void)hipGetLastError();
          segsz = bb;
          e = hipMalloc((void**)&base, (size_t)segsz);
        }
        if (e != hipSuccess) {  // everything idle back to the driver, then once more
          (void)hipGetLastError();
          l.lock();
          ++d.oom_retries;
          drop = detach_free_segments(d);
          release_cached(d);
          l.unlock();
          free_segments(drop);
          const hipError_t se = hipDeviceSynchronize();
          if (se != hipSuccess) {
            (void)hipGetLastError();
            l.lock();
            d.in_use -= bb;
            set_fault(d, std::string("device fault seen by an allocation retry: ") + hipGetErrorString(se));
            TORCH_CHECK(false, "mrhip page pool: device error on device ", dev, ": ", hipGetErrorString(se));
          }
          hipMemPool_t hp;
          {
            std::lock_guard<std::mutex> g(g_mu);
            hp = d.pool;
          }
          if (hp) (void)hipMemPoolTrimTo(hp, 0);
          e = hipMalloc((void**)&base, (size_t)segsz);
        }
        l.lock();
        d.in_use -= bb;  // counted again below, with the block
        ++d.grows;
        d.grow_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        if (e != hipSuccess || !base) {
          (void)hipGetLastError();
          ++d.failures;
          TORCH_CHECK_WITH(OutOfMemoryError, false, "mrhip page pool: HIP out of memory allocating ", mib(bb),
                           " on device ", dev, " (", mib(d.in_use), " in use): ", hipGetErrorString(e));
        }
        auto seg = std::make_unique<Seg>();
        seg->base = base;
        seg->size = segsz;
        seg->free_bytes = segsz;
        d.big_bytes += segsz;
        d.big_free += segsz;
        d.big_peak = std::max(d.big_peak, d.big_bytes);
        range_add(d, seg.get(), 0, segsz, {});
        d.segs.push_back(std::move(seg));
        note_reserved(d);
        p = arena_take(d, bb, stream, &sg, &off);
        TORCH_CHECK(p, "mrhip page pool: a fresh segment could not serve its block");
      }
      d.in_use += bb;
      d.peak = std::max(d.peak, d.in_use);
      ++d.allocs;
      Block b{bb, dev, stream, {}};
      b.seg = sg;
      b.off = off;
      g_blocks[p] = std::move(b);
      return p;
    }
    auto it = d.free.find({stream, bytes});
    void* p = nullptr;
    if (it != d.free.end() && !it->second.empty()) {  // stream-ordered reuse: no HIP call
      p = it->second.back();
      it->second.pop_back();
    } else {
      p = take_other_stream(d, stream, bytes);
      if (!d.fault.empty())
        TORCH_CHECK(false, "mrhip page pool: device ", dev, " faulted: ", d.fault);
    }
    if (p) {
      d.cached -= bytes;
      d.in_use += bytes;
      d.peak = std::max(d.peak, d.in_use);
      ++d.allocs;
      g_blocks[p] = Block{bytes, dev, stream, {}};
      return p;
    }
    // much idle memory cached in other classes and the device filling up:
    // hand it back before growing (the HIP pool reuses freed memory across
    // streams and sizes; big blocks go back to the driver)
    if (d.total_mem == 0) {
      size_t fr = 0, tot = 0;
      if (hipMemGetInfo(&fr, &tot) == hipSuccess) d.total_mem = (int64_t)tot;
      else (void)hipGetLastError();
    }
    const int64_t held = d.in_use + d.cached;
    if (d.cached > (int64_t(1) << 30) && d.cached > d.in_use / 4 &&
        (d.total_mem == 0 || held + bytes > d.total_mem / 10 * 7))
      release_cached(d);
    if (!d.fault.empty()) TORCH_CHECK(false, "mrhip page pool: device ", dev, " faulted: ", d.fault);
    pool = pool_of(dev);
    d.in_use += bytes;  // reserved before the call so concurrent allocations see it
    d.peak = std::max(d.peak, d.in_use);
    ++d.allocs;
  }
  void* p = nullptr;
  const auto t0 = std::chrono::steady_clock::now();
  auto grow = [&] { return hipMallocFromPoolAsync(&p, (size_t)bytes, pool, stream); };
  hipError_t e = grow();
  if (e != hipSuccess) {
    (void)hipGetLastError();
    {
      std::lock_guard<std::mutex> l(g_mu);
      ++g_dev[dev].oom_retries;
    }
    // memory held in the caches or freed on other streams: give it all back
    // to the pool / driver and retry once
    {
      std::lock_guard<std::mutex> l(g_mu);
      release_cached(g_dev[dev]);
    }
    const hipError_t se = hipDeviceSynchronize();
    if (se != hipSuccess) {  // not an out-of-memory: a device fault, which a retry must not hide
      (void)hipGetLastError();
      std::lock_guard<std::mutex> l(g_mu);
      g_dev[dev].in_use -= bytes;
      set_fault(g_dev[dev], std::string("device fault seen by an allocation retry: ") + hipGetErrorString(se));
      TORCH_CHECK(false, "mrhip page pool: device error on device ", dev, " while retrying an allocation of ",
                  mib(bytes), ": ", hipGetErrorString(se));
    }
    (void)hipMemPoolTrimTo(pool, 0);
    e = grow();
    if (e != hipSuccess) (void)hipGetLastError();
  }
  std::lock_guard<std::mutex> l(g_mu);
  ++g_dev[dev].grows;
  g_dev[dev].grow_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  if (e != hipSuccess || !p) {
    g_dev[dev].in_use -= bytes;
    ++g_dev[dev].failures;
    TORCH_CHECK_WITH(OutOfMemoryError, false, "mrhip page pool: HIP out of memory allocating ", mib(bytes),
                     " on device ", dev, " (", mib(g_dev[dev].in_use), " in use): ", hipGetErrorString(e));
  }
  note_reserved(g_dev[dev]);
  g_blocks[p] = Block{bytes, dev, stream, {}};
  return p;
}

void pool_free(void* ptr, size_t /*size*/, int /*dev*/, hipStream_t /*stream*/) {
  if (!ptr) return;
  std::lock_guard<std::mutex> l(g_mu);
  auto it = g_blocks.find(ptr);
  if (it == g_blocks.end()) return;  // not ours (cannot happen once installed)
  Block b = std::move(it->second);
  g_blocks.erase(it);
  Dev& d = g_dev[b.dev];
  d.in_use -= b.bytes;
  ++d.frees;
  if (b.seg) {
    // an event on every stream that used it: the next user, on any stream, waits
    std::vector<EvP> evs;
    std::vector<hipStream_t> ss = b.used_on;
    ss.push_back(b.stream);
    for (hipStream_t st : ss) {
      auto e = std::make_shared<Ev>();
      if (hipEventCreateWithFlags(&e->e, hipEventDisableTiming) != hipSuccess || hipEventRecord(e->e, st) != hipSuccess) {
        (void)hipGetLastError();
        const hipError_t r = hipStreamSynchronize(st);  // cannot order by event: drain instead
        if (r != hipSuccess) {
          (void)hipGetLastError();
          set_fault(d, std::string("freeing a big block: ") + hipGetErrorString(r));
          return;  // never reused
        }
        continue;
      }
      evs.push_back(std::move(e));
    }
    b.seg->free_bytes += b.bytes;
    d.big_free += b.bytes;
    range_add(d, b.seg, b.off, b.bytes, std::move(evs));
    return;
  }
  d.cached += b.bytes;
  if (b.used_on.empty()) {
    // later work on the allocating stream runs after every earlier use
    cache_put(d, b.stream, b.bytes, ptr);
    return;
  }
  // used on other streams too: reusable after an event of each of them
  Pending q;
  q.p = ptr;
  for (hipStream_t s : b.used_on) {
    hipEvent_t ev;
    if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess || hipEventRecord(ev, s) != hipSuccess) {
      (void)hipGetLastError();
      const hipError_t r = hipStreamSynchronize(s);
      if (r != hipSuccess) {  // cannot tell when the other stream is done with it: never reuse
        (void)hipGetLastError();
        set_fault(d, std::string("freeing a block used on another stream: ") + hipGetErrorString(r));
        d.cached -= b.bytes;
        return;
      }
      continue;
    }
    q.evs.push_back(ev);
  }
  q.b = std::move(b);
  d.pending.push_back(std::move(q));
}

// free_blocks = false (a stream that may never drain, e.g. an aborted RCCL
// stream): its cached blocks are dropped from the cache and leaked rather
// than freed behind work that may never finish
void forget_stream_locked(hipStream_t s, bool free_blocks = true) {  // g_mu held
  if (!s) return;
  for (Dev& d : g_dev) {
    for (auto it = d.free.begin(); it != d.free.end();) {
      if (it->first.first != s) {
        ++it;
        continue;
      }
      for (void* p : it->second) {
        if (free_blocks && hipFreeAsync(p, s) != hipSuccess) (void)hipGetLastError();
        d.cached -= it->first.second;
      }
      it = d.free.erase(it);
    }
    d.streams.erase(std::remove(d.streams.begin(), d.streams.end(), s), d.streams.end());
    for (Pending& q : d.pending) {
      if (q.b.stream == s) q.b.stream = nullptr;
      q.b.used_on.erase(std::remove(q.b.used_on.begin(), q.b.used_on.end(), s), q.b.used_on.end());
    }
  }
  for (auto& [p, b] : g_blocks) {
    if (b.stream == s) b.stream = nullptr;
    b.used_on.erase(std::remove(b.used_on.begin(), b.used_on.end(), s), b.used_on.end());
  }
}

void pool_record_stream(void* ptr, hipStream_t s) {
  std::lock_guard<std::mutex> l(g_mu);
  auto it = g_blocks.find(ptr);
  if (it == g_blocks.end() || s == it->second.stream) return;
  auto& v = it->second.used_on;
  if (std::find(v.begin(), v.end(), s) == v.end()) v.push_back(s);
}

void pool_reset() {  // torch.cuda.empty_cache() / emptyCache(): give cached memory back
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return;
  for (int d = 0; d < std::min(n, kMaxDev); ++d) trim(d, 0);
}

}  // namespace

bool install() {
  if (g_installed) return true;
  using torch::cuda::CUDAPluggableAllocator::CUDAPluggableAllocator;
  auto cur = torch::cuda::CUDAPluggableAllocator::getCurrentAllocator();
  if (cur && cur->initialized()) return false;  // device memory already handed out by another allocator
  auto a = std::make_shared<CUDAPluggableAllocator>(pool_alloc, pool_free);
  a->set_record_stream_fn(pool_record_stream);
  a->set_reset_fn(pool_reset);
  torch::cuda::CUDAPluggableAllocator::changeCurrentAllocator(a);
  g_installed = true;
  return true;
}

bool install_default() {
  const char* e = std::getenv("MRH_HBM_POOL");
  if (e && std::string(e) == "0") return false;
  return install();
}

bool installed() { return g_installed; }

PoolStats stats(int device) {
  PoolStats s;
  if (device < 0 || device >= kMaxDev) return s;
  std::lock_guard<std::mutex> l(g_mu);
  const Dev& d = g_dev[device];
  s.in_use = d.in_use;
  s.peak = d.peak;
  s.cap = d.cap;
  s.allocs = d.allocs;
  s.frees = d.frees;
  s.failures = d.failures;
  s.cached = d.cached;
  s.cross_stream_reuse = d.cross;
  s.faulted = !d.fault.empty();
  s.grows = d.grows;
  s.grow_ms = d.grow_ms;
  s.releases = d.releases;
  s.oom_retries = d.oom_retries;
  Dev& dm = const_cast<Dev&>(d);
  s.reserved = pool_reserved(dm);
  note_reserved(dm);
  s.reserved_peak = d.reserved_peak_true;  // hi-water of (HIP pool reserved + big-block segments)
  s.cached += d.big_free;
  return s;
}

void reset_peak(int device) {
  if (device < 0 || device >= kMaxDev) return;
  std::lock_guard<std::mutex> l(g_mu);
  g_dev[device].peak = g_dev[device].in_use;
}

void reset_reserved_peak(int device) {
  if (device < 0 || device >= kMaxDev) return;
  std::lock_guard<std::mutex> l(g_mu);
  g_dev[device].reserved_peak_true = pool_reserved(g_dev[device]);
}

int64_t set_cap(int device, int64_t cap) {
  if (device < 0 || device >= kMaxDev) return 0;
  std::lock_guard<std::mutex> l(g_mu);
  Dev& d = g_dev[device];
  const int64_t prev = d.base_cap;
  d.base_cap = std::max<int64_t>(0, cap);
  recompute_cap(d);
  return prev;
}

void trim(int device, int64_t keep_bytes) {
  if (device < 0 || device >= kMaxDev) return;
  hipMemPool_t p;
  std::vector<std::unique_ptr<Seg>> drop;
  {
    std::lock_guard<std::mutex> l(g_mu);
    p = g_dev[device].pool;
    if (p) release_cached(g_dev[device]);
    drop = detach_free_segments(g_dev[device]);
  }
  free_segments(drop);
  if (!p) return;
  // freed blocks are returned to the pool in stream order: let the device
  // drain so the trim sees them; a device fault here is the pool's too
  const hipError_t r = hipDeviceSynchronize();
  if (r != hipSuccess) {
    (void)hipGetLastError();
    std::lock_guard<std::mutex> l(g_mu);
    set_fault(g_dev[device], std::string("device fault seen by trim: ") + hipGetErrorString(r));
    return;
  }
  if (hipMemPoolTrimTo(p, (size_t)std::max<int64_t>(0, keep_bytes)) != hipSuccess) (void)hipGetLastError();
}

// every running op's cap is kept (a multiset: ops on one device may run on
// several threads, and their scopes need not nest); the cap in force is the
// tightest of them and set_cap's, so no exit order can leave a stale cap
OpCap::OpCap(int device, int64_t extra) {
  if (!g_installed || device < 0 || device >= kMaxDev || extra <= 0) return;
  std::lock_guard<std::mutex> l(g_mu);
  Dev& d = g_dev[device];
  dev_ = device;
  prev_ = d.in_use + extra;
  d.op_caps.insert(prev_);
  recompute_cap(d);
  on_ = true;
}

OpCap::~OpCap() {
  if (!on_) return;
  std::lock_guard<std::mutex> l(g_mu);
  Dev& d = g_dev[dev_];
  auto it = d.op_caps.find(prev_);
  if (it != d.op_caps.end()) d.op_caps.erase(it);
  recompute_cap(d);
}

void forget_stream(hipStream_t s) {
  if (!s) return;
  (void)hipStreamSynchronize(s);
  std::lock_guard<std::mutex> l(g_mu);
  forget_stream_locked(s);
}

void forget_stream_nosync(hipStream_t s) {
  if (!s) return;
  std::lock_guard<std::mutex> l(g_mu);
  forget_stream_locked(s, false);
}

}  // namespace mrh::hbm
