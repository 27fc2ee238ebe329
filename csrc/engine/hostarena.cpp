// Pinned host arena (hostarena.h): one hipHostMalloc'd segment, best-fit
// blocks of 4 KiB granularity kept in an address-ordered free map (coalesced
// on free) plus a size-ordered index for the fit.
#include "hostarena.h"

#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <map>
#include <mutex>
#include <stdexcept>

namespace mrh {
namespace hostarena {
namespace {
constexpr int64_t kAlign = 4096;
struct Arena {
  std::mutex mu;
  uint8_t* base = nullptr;
  int64_t size = 0;
  std::map<int64_t, int64_t> free_by_off;            // offset -> bytes
  std::multimap<int64_t, int64_t> free_by_size;      // bytes -> offset
  Stats st;
  void insert(int64_t off, int64_t n) {
    free_by_off[off] = n;
    free_by_size.emplace(n, off);
  }
  void erase(int64_t off, int64_t n) {
    free_by_off.erase(off);
    auto r = free_by_size.equal_range(n);
    for (auto it = r.first; it != r.second; ++it)
      if (it->second == off) {
        free_by_size.erase(it);
        return;
      }
  }
  // -1: no fit
  int64_t take(int64_t n) {
    auto it = free_by_size.lower_bound(n);
    if (it == free_by_size.end()) return -1;
    const int64_t off = it->second, have = it->first;
    erase(off, have);
    if (have > n) insert(off + n, have - n);
    return off;
  }
  void give(int64_t off, int64_t n) {
    auto nx = free_by_off.find(off + n);
    if (nx != free_by_off.end()) {
      const int64_t m = nx->second;
      erase(off + n, m);
      n += m;
    }
    auto pv = free_by_off.lower_bound(off);
    if (pv != free_by_off.begin()) {
      --pv;
      if (pv->first + pv->second == off) {
        const int64_t o = pv->first, m = pv->second;
        erase(o, m);
        off = o;
        n += m;
      }
    }
    insert(off, n);
  }
};
Arena& arena() {
  static Arena* a = new Arena();  // never destroyed: blocks may be freed during static destruction
  return *a;
}
}  // namespace

double reserve(int64_t bytes) {
  Arena& a = arena();
  std::lock_guard<std::mutex> lk(a.mu);
  if (a.base || bytes <= 0) return 0.0;
  const int64_t n = (bytes + (int64_t(2) << 20) - 1) / (int64_t(2) << 20) * (int64_t(2) << 20);
  const auto t0 = std::chrono::steady_clock::now();
  void* p = nullptr;
  if (hipHostMalloc(&p, (size_t)n, hipHostMallocDefault) != hipSuccess || !p) {
    // no arena: every pinned allocation keeps using the caching host allocator
    (void)hipGetLastError();
    std::fprintf(stderr, "mrhip: pinned host arena of %lld bytes not available; continuing without it\n",
                 (long long)n);
    return -1.0;
  }
  a.base = static_cast<uint8_t*>(p);
  a.size = n;
  a.insert(0, n);
  a.st.reserved = n;
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

Stats stats() {
  Arena& a = arena();
  std::lock_guard<std::mutex> lk(a.mu);
  return a.st;
}

at::Tensor pinned_empty(at::IntArrayRef sizes, at::ScalarType dtype) {
  int64_t numel = 1;
  for (int64_t s : sizes) numel *= s;
  const int64_t bytes = numel * (int64_t)c10::elementSize(dtype);
  const at::TensorOptions o = at::TensorOptions().dtype(dtype).device(at::kCPU);
  Arena& a = arena();
  if (bytes > 0) {
    const int64_t n = (bytes + kAlign - 1) / kAlign * kAlign;
    int64_t off = -1;
    {
      std::lock_guard<std::mutex> lk(a.mu);
      if (a.base) {
        off = a.take(n);
        if (off >= 0) {
          ++a.st.hits;
          a.st.in_use += n;
          a.st.peak = std::max(a.st.peak, a.st.in_use);
        } else {
          ++a.st.misses;
        }
      }
    }
    if (off >= 0)
      return at::from_blob(
          a.base + off, sizes,
          [n, off](void*) {
            Arena& ar = arena();
            std::lock_guard<std::mutex> lk(ar.mu);
            ar.give(off, n);
            ar.st.in_use -= n;
          },
          o);
  }
  return at::empty(sizes, o.pinned_memory(true));
}
}  // namespace hostarena
}  // namespace mrh
