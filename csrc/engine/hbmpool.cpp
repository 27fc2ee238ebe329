// HBM page pool (see hbmpool.h).
#include "hbmpool.h"

#include <c10/util/Exception.h>
#include <torch/csrc/cuda/CUDAPluggableAllocator.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

namespace mrh::hbm {

namespace {

constexpr int kMaxDev = 64;
constexpr int64_t kGranule = 512;

struct Block {
  int64_t bytes = 0;  // accounted size (granules)
  int dev = 0;
  hipStream_t stream = nullptr;
  std::vector<hipStream_t> used_on;  // other streams that touched the block (record_stream)
};

struct Dev {
  hipMemPool_t pool = nullptr;
  int64_t in_use = 0, peak = 0, cap = 0, allocs = 0, frees = 0, failures = 0;
};

std::mutex g_mu;
Dev g_dev[kMaxDev];
std::unordered_map<void*, Block> g_blocks;
std::atomic<bool> g_installed{false};

std::string mib(int64_t b) { return std::to_string(b >> 20) + " MiB"; }

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

void* pool_alloc(size_t size, int dev, hipStream_t stream) {
  if (size == 0) return nullptr;
  TORCH_CHECK(dev >= 0 && dev < kMaxDev, "mrhip page pool: device index out of range");
  const int64_t bytes = ((int64_t)size + kGranule - 1) / kGranule * kGranule;
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
    pool = pool_of(dev);
    d.in_use += bytes;  // reserved before the call so concurrent allocations see it
    d.peak = std::max(d.peak, d.in_use);
    ++d.allocs;
  }
  void* p = nullptr;
  hipError_t e = hipMallocFromPoolAsync(&p, size, pool, stream);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    // cached free memory of the pool that this stream cannot reuse yet: give
    // it back to the driver and retry once
    (void)hipStreamSynchronize(stream);
    (void)hipMemPoolTrimTo(pool, 0);
    e = hipMallocFromPoolAsync(&p, size, pool, stream);
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
  Block b;
  {
    std::lock_guard<std::mutex> l(g_mu);
    auto it = g_blocks.find(ptr);
    if (it == g_blocks.end()) return;  // not ours (cannot happen once installed)
    b = std::move(it->second);
    g_blocks.erase(it);
    g_dev[b.dev].in_use -= b.bytes;
    ++g_dev[b.dev].frees;
  }
  // the block may only be reused after the work of every stream that used it:
  // the allocating stream waits for an event of each of the others, then frees
  for (hipStream_t s : b.used_on) {
    hipEvent_t ev;
    if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
      (void)hipGetLastError();
      (void)hipStreamSynchronize(s);
      continue;
    }
    if (hipEventRecord(ev, s) != hipSuccess || hipStreamWaitEvent(b.stream, ev, 0) != hipSuccess) {
      (void)hipGetLastError();
      (void)hipStreamSynchronize(s);
    }
    (void)hipEventDestroy(ev);
  }
  if (hipFreeAsync(ptr, b.stream) != hipSuccess) {
    // the allocating stream is gone: order against the whole device instead
    (void)hipGetLastError();
    (void)hipDeviceSynchronize();
    (void)hipFreeAsync(ptr, nullptr);
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
