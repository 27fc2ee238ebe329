// HBM page pool (see hbmpool.h).
#include "hbmpool.h"

#include <c10/util/Exception.h>
#include <torch/csrc/cuda/CUDAPluggableAllocator.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

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
};

// a freed block that other streams used: reusable once their events complete
struct Pending {
  void* p = nullptr;
  Block b;
  std::vector<hipEvent_t> evs;
};

struct Dev {
  hipMemPool_t pool = nullptr;
  int64_t in_use = 0, peak = 0, cap = 0, cached = 0, allocs = 0, frees = 0, failures = 0;
  std::map<std::pair<hipStream_t, int64_t>, std::vector<void*>> free;  // (stream, class) -> cached blocks
  std::vector<Pending> pending;
};

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

// pending blocks whose other-stream work is done go to their stream's cache
void reap(Dev& d) {  // g_mu held
  for (size_t i = 0; i < d.pending.size();) {
    Pending& q = d.pending[i];
    bool done = true;
    for (hipEvent_t e : q.evs) {
      const hipError_t r = hipEventQuery(e);
      if (r == hipErrorNotReady) {
        done = false;
        break;
      }
      if (r != hipSuccess) (void)hipGetLastError();
    }
    if (!done) {
      ++i;
      continue;
    }
    for (hipEvent_t e : q.evs) (void)hipEventDestroy(e);
    d.free[{q.b.stream, q.b.bytes}].push_back(q.p);
    q = std::move(d.pending.back());
    d.pending.pop_back();
  }
}

// every cached block back to the HIP pool (then the pool can hand the memory
// to any stream, or trim it to the driver)
void release_cached(Dev& d) {  // g_mu held
  for (Pending& q : d.pending) {
    for (hipEvent_t e : q.evs) {
      (void)hipStreamWaitEvent(q.b.stream, e, 0);
      (void)hipEventDestroy(e);
    }
    d.free[{q.b.stream, q.b.bytes}].push_back(q.p);
  }
  d.pending.clear();
  for (auto& [k, v] : d.free)
    for (void* p : v)
      if (hipFreeAsync(p, k.first) != hipSuccess) {
        (void)hipGetLastError();
        (void)hipDeviceSynchronize();
        (void)hipFreeAsync(p, nullptr);
      }
  d.free.clear();
  d.cached = 0;
}

void* pool_alloc(size_t size, int dev, hipStream_t stream) {
  if (size == 0) return nullptr;
  TORCH_CHECK(dev >= 0 && dev < kMaxDev, "mrhip page pool: device index out of range");
  const int64_t bytes = class_bytes(size);
  hipMemPool_t pool;
  {
    std::lock_guard<std::mutex> l(g_mu);
    Dev& d = g_dev[dev];
    if (d.cap > 0 && d.in_use + bytes > d.cap) {
      ++d.failures;
      TORCH_CHECK_WITH(OutOfMemoryError, false, "mrhip page pool: Cannot allocate page: ", mib(bytes),
                       " requested with ", mib(d.in_use), " in use of a cap of ", mib(d.cap),
                       " (maxpage x memsize / hbm_budget) on device ", dev);
    }
    if (!d.pending.empty()) reap(d);
    auto it = d.free.find({stream, bytes});
    if (it != d.free.end() && !it->second.empty()) {  // stream-ordered reuse: no HIP call
      void* p = it->second.back();
      it->second.pop_back();
      d.cached -= bytes;
      d.in_use += bytes;
      d.peak = std::max(d.peak, d.in_use);
      ++d.allocs;
      g_blocks[p] = Block{bytes, dev, stream, {}};
      return p;
    }
    pool = pool_of(dev);
    d.in_use += bytes;  // reserved before the call so concurrent allocations see it
    d.peak = std::max(d.peak, d.in_use);
    ++d.allocs;
  }
  void* p = nullptr;
  hipError_t e = hipMallocFromPoolAsync(&p, (size_t)bytes, pool, stream);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    // memory held in the caches or freed on other streams: give it all back
    // to the pool / driver and retry once
    {
      std::lock_guard<std::mutex> l(g_mu);
      release_cached(g_dev[dev]);
    }
    (void)hipDeviceSynchronize();
    (void)hipMemPoolTrimTo(pool, 0);
    e = hipMallocFromPoolAsync(&p, (size_t)bytes, pool, stream);
    if (e != hipSuccess) (void)hipGetLastError();
  }
  std::lock_guard<std::mutex> l(g_mu);
  if (e != hipSuccess || !p) {
    g_dev[dev].in_use -= bytes;
    ++g_dev[dev].failures;
    TORCH_CHECK_WITH(OutOfMemoryError, false, "mrhip page pool: HIP out of memory allocating ", mib(bytes),
                     " on device ", dev, " (", mib(g_dev[dev].in_use), " in use): ", hipGetErrorString(e));
  }
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
  d.cached += b.bytes;
  ++d.frees;
  if (b.used_on.empty()) {
    // later work on the allocating stream runs after every earlier use
    d.free[{b.stream, b.bytes}].push_back(ptr);
    return;
  }
  // used on other streams too: reusable after an event of each of them
  Pending q;
  q.p = ptr;
  for (hipStream_t s : b.used_on) {
    hipEvent_t ev;
    if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess || hipEventRecord(ev, s) != hipSuccess) {
      (void)hipGetLastError();
      (void)hipStreamSynchronize(s);
      continue;
    }
    q.evs.push_back(ev);
  }
  q.b = std::move(b);
  d.pending.push_back(std::move(q));
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
  if (d.pool) {
    uint64_t r = 0;
    if (hipMemPoolGetAttribute(d.pool, hipMemPoolAttrReservedMemCurrent, &r) == hipSuccess) s.reserved = (int64_t)r;
  }
  return s;
}

void reset_peak(int device) {
  if (device < 0 || device >= kMaxDev) return;
  std::lock_guard<std::mutex> l(g_mu);
  g_dev[device].peak = g_dev[device].in_use;
}

int64_t set_cap(int device, int64_t cap) {
  if (device < 0 || device >= kMaxDev) return 0;
  std::lock_guard<std::mutex> l(g_mu);
  const int64_t prev = g_dev[device].cap;
  g_dev[device].cap = std::max<int64_t>(0, cap);
  return prev;
}

void trim(int device, int64_t keep_bytes) {
  if (device < 0 || device >= kMaxDev) return;
  hipMemPool_t p;
  {
    std::lock_guard<std::mutex> l(g_mu);
    p = g_dev[device].pool;
    if (p) release_cached(g_dev[device]);
  }
  if (!p) return;
  // freed blocks are returned to the pool in stream order: let the device
  // drain so the trim sees them
  (void)hipDeviceSynchronize();
  if (hipMemPoolTrimTo(p, (size_t)std::max<int64_t>(0, keep_bytes)) != hipSuccess) (void)hipGetLastError();
}

OpCap::OpCap(int device, int64_t extra) {
  if (!g_installed || device < 0 || device >= kMaxDev || extra <= 0) return;
  std::lock_guard<std::mutex> l(g_mu);
  Dev& d = g_dev[device];
  dev_ = device;
  prev_ = d.cap;
  const int64_t want = d.in_use + extra;
  d.cap = prev_ > 0 ? std::min(prev_, want) : want;  // never loosen an outer cap
  on_ = true;
}

OpCap::~OpCap() {
  if (!on_) return;
  std::lock_guard<std::mutex> l(g_mu);
  g_dev[dev_].cap = prev_;
}

}  // namespace mrh::hbm
