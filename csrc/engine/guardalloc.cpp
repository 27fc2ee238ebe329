// Guarded HBM allocator (guardalloc.h): canaried blocks behind ATen's
// pluggable allocator interface.
#include "guardalloc.h"

#include <hip/hip_runtime.h>
#include <torch/csrc/cuda/CUDAPluggableAllocator.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <unordered_map>

namespace mrh {
namespace guard {

namespace {

constexpr size_t kGuard = 4096;      // canary bytes on each side (keeps 256 B alignment)
constexpr uint8_t kCanary = 0xCB;
constexpr uint8_t kPoison = 0xA5;

struct Block {
  uint8_t* base = nullptr;
  size_t size = 0, padded = 0;
  std::string op;
};

std::mutex g_mu;
std::unordered_map<void*, Block>& blocks() {
  static auto* m = new std::unordered_map<void*, Block>();  // never destroyed: frees may run at exit
  return *m;
}
std::vector<GuardReport>& reports() {
  static auto* v = new std::vector<GuardReport>();
  return *v;
}
std::atomic<bool> g_active{false};
thread_local std::string t_op = "(outside any MapReduce op)";

size_t pad256(size_t x) { return (x + 255) & ~size_t(255); }

// corrupted canary bytes of one block (device synchronised by the caller)
void scan(const Block& b, int64_t* front, int64_t* back) {
  std::vector<uint8_t> h(kGuard + (b.padded - b.size) + kGuard);
  *front = *back = 0;
  if (hipMemcpy(h.data(), b.base, kGuard, hipMemcpyDeviceToHost) != hipSuccess) return;
  const size_t tail = b.padded - b.size + kGuard;
  if (hipMemcpy(h.data() + kGuard, b.base + kGuard + b.size, tail, hipMemcpyDeviceToHost) != hipSuccess) return;
  for (size_t i = 0; i < kGuard; ++i) *front += h[i] != kCanary;
  for (size_t i = 0; i < tail; ++i) *back += h[kGuard + i] != kCanary;
}

void report(void* user, const Block& b, int64_t front, int64_t back, const std::string& where) {
  GuardReport r;
  r.ptr = (uint64_t)(uintptr_t)user;
  r.size = (int64_t)b.size;
  r.front_bad = front;
  r.back_bad = back;
  r.alloc_op = b.op;
  r.found_op = where;
  std::fprintf(stderr,
               "mrhip guard: out-of-bounds device write on a %zu-byte block at %p (allocated in %s): %lld byte(s) "
               "before it, %lld past its end; detected %s\n",
               b.size, user, b.op.c_str(), (long long)front, (long long)back, where.c_str());
  reports().push_back(r);
}

// allocator callbacks cannot throw through ATen: a failed runtime call is
// printed and turned into "no memory" (alloc) or a logged error (free)
bool ok_or_log(hipError_t e, const char* what) {
  if (e == hipSuccess) return true;
  std::fprintf(stderr, "mrhip guard: %s failed: %s\n", what, hipGetErrorString(e));
  return false;
}

void* g_alloc(size_t size, int device, hipStream_t) {
  if (size == 0) return nullptr;
  if (!ok_or_log(hipSetDevice(device), "hipSetDevice")) return nullptr;
  Block b;
  b.size = size;
  b.padded = pad256(size);
  const size_t total = kGuard + b.padded + kGuard;
  if (hipMalloc(&b.base, total) != hipSuccess) {
    (void)hipGetLastError();  // clear the sticky OOM status; ATen reports it as out of memory
    return nullptr;
  }
  uint8_t* user = b.base + kGuard;
  const bool ok = ok_or_log(hipMemset(b.base, kCanary, kGuard), "hipMemset (front canary)") &&
                  ok_or_log(hipMemset(user, kPoison, size), "hipMemset (poison)") &&
                  ok_or_log(hipMemset(user + size, kCanary, b.padded - size + kGuard), "hipMemset (back canary)") &&
                  ok_or_log(hipDeviceSynchronize(), "hipDeviceSynchronize");
  if (!ok) {
    ok_or_log(hipFree(b.base), "hipFree");
    return nullptr;
  }
  b.op = t_op;
  std::lock_guard<std::mutex> lk(g_mu);
  blocks()[user] = std::move(b);
  return user;
}

void g_free(void* ptr, size_t, int device, hipStream_t) {
  if (!ptr) return;
  Block b;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = blocks().find(ptr);
    if (it == blocks().end()) return;
    b = std::move(it->second);
    blocks().erase(it);
  }
  ok_or_log(hipSetDevice(device), "hipSetDevice");
  // every kernel that may still write the block has finished
  ok_or_log(hipDeviceSynchronize(), "hipDeviceSynchronize (free)");
  int64_t f = 0, k = 0;
  scan(b, &f, &k);
  if (f || k) {
    std::lock_guard<std::mutex> lk(g_mu);
    report(ptr, b, f, k, "when the block was freed (during " + t_op + ")");
  }
  ok_or_log(hipFree(b.base), "hipFree");
}

}  // namespace

bool alloc_guard_enabled() {
  static const bool on = [] {
    const char* v = std::getenv("MRH_GUARD");
    return v && *v && *v != '0';
  }();
  return on;
}

bool install_alloc_guard() {
  static std::once_flag once;
  static std::string err;
  std::call_once(once, [] {
    if (!alloc_guard_enabled()) return;
    try {
      auto a = torch::cuda::CUDAPluggableAllocator::createCustomAllocator(g_alloc, g_free);
      torch::cuda::CUDAPluggableAllocator::changeCurrentAllocator(a);
      g_active = true;
    } catch (const std::exception& e) {
      err = e.what();
    }
  });
  if (alloc_guard_enabled() && !g_active)
    throw std::runtime_error("mrhip: MRH_GUARD=1 but the guarded allocator could not be installed (HBM was "
                             "already allocated through ATen?): " + err);
  return g_active;
}

bool alloc_guard_active() { return g_active; }

void set_current_op(const char* op) { t_op = op ? op : "(outside any MapReduce op)"; }
const char* current_op() { return t_op.c_str(); }

int check_all_blocks(const char* op) {
  if (!g_active) return 0;
  auto must = [](hipError_t e, const char* what) {
    if (e != hipSuccess) throw std::runtime_error(std::string("mrhip guard: ") + what + ": " + hipGetErrorString(e));
  };
  must(hipDeviceSynchronize(), "hipDeviceSynchronize");
  std::lock_guard<std::mutex> lk(g_mu);
  int bad = 0;
  for (auto& [user, b] : blocks()) {
    int64_t f = 0, k = 0;
    scan(b, &f, &k);
    if (!f && !k) continue;
    ++bad;
    report(user, b, f, k, std::string("at the end of ") + (op ? op : "a check"));
    // re-arm the canaries so one overrun is reported once
    must(hipMemset(b.base, kCanary, kGuard), "hipMemset (re-arm)");
    must(hipMemset(b.base + kGuard + b.size, kCanary, b.padded - b.size + kGuard), "hipMemset (re-arm)");
  }
  must(hipDeviceSynchronize(), "hipDeviceSynchronize");
  return bad;
}

std::vector<GuardReport> guard_reports() {
  std::lock_guard<std::mutex> lk(g_mu);
  return reports();
}

int64_t guarded_blocks_live() {
  std::lock_guard<std::mutex> lk(g_mu);
  return (int64_t)blocks().size();
}

}  // namespace guard
}  // namespace mrh
