// guard.h: bounded collectives, fault injection, spill-on-OOM registry,
// invariant checks.
#include "guard.h"

#include <c10/hip/HIPCachingAllocator.h>
#include <execinfo.h>
#include <signal.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <set>
#include <sstream>
#include <stdexcept>

#include "mapreduce.h"

namespace mrh::guard {

namespace {

int env_int(const char* k, int d) {
  const char* v = std::getenv(k);
  return v && *v ? std::atoi(v) : d;
}

struct Fault {
  std::string kind, op;
  int rank = -1, nth = 1;
  bool armed = false;
};

Fault parse_fault() {
  Fault f;
  const char* s = std::getenv("MRH_FAULT");
  if (!s || !*s) return f;
  std::stringstream ss(s);
  std::string tok;
  std::vector<std::string> p;
  while (std::getline(ss, tok, ':')) p.push_back(tok);
  if (p.size() < 3 || (p[0] != "abort" && p[0] != "throw" && p[0] != "oom" && p[0] != "hip"))
    throw std::runtime_error("MRH_FAULT must be kind:op:rank[:nth] with kind abort|throw|oom|hip, got '" +
                             std::string(s) + "'");
  f.kind = p[0];
  f.op = p[1];
  f.rank = std::atoi(p[2].c_str());
  if (p.size() > 3) f.nth = std::max(1, std::atoi(p[3].c_str()));
  f.armed = true;
  return f;
}

std::mutex g_mu;
Fault& fault() {
  static Fault f = parse_fault();
  return f;
}
std::map<std::string, int>& hits() {
  static std::map<std::string, int> h;
  return h;
}
std::set<MapReduce*>& live() {
  static std::set<MapReduce*> s;
  return s;
}

// does the armed fault fire at this entry of `op`? (counts the entry)
bool due(const char* op, int rank, const char* kind) {
  Fault& f = fault();
  if (!f.armed || f.kind != kind || f.op != op || (f.rank >= 0 && f.rank != rank)) return false;
  if (++hits()[op] != f.nth) return false;
  f.armed = false;
  return true;
}

void bad(const char* op, const std::string& what) {
  throw std::runtime_error(std::string("MRH_CHECK: invariant broken after ") + op + ": " + what);
}

void check_col(const at::Tensor& data, const at::Tensor& off, int w, int64_t n, const char* op, const char* col) {
  const int64_t bytes = data.defined() ? data.numel() : 0;
  if (w >= 0) {
    if (bytes < n * w) bad(op, std::string(col) + " arena smaller than n * width");
    return;
  }
  if (n == 0 && !off.defined()) return;  // empty variable column: offsets optional
  if (!off.defined() || off.numel() != n + 1) bad(op, std::string(col) + " offsets must have n+1 entries");
  at::Tensor o = off.to(at::kCPU);
  if (o.scalar_type() != at::kLong) bad(op, std::string(col) + " offsets must be int64");
  const int64_t* p = o.data_ptr<int64_t>();
  if (p[0] != 0) bad(op, std::string(col) + " offsets must start at 0");
  if (n > 0 && (o.narrow(0, 1, n) < o.narrow(0, 0, n)).any().item<bool>())
    bad(op, std::string(col) + " offsets are not monotone");
  if (p[n] > bytes) bad(op, std::string(col) + " offsets run past the arena");
}

// MRH_STACK_SIGNAL=1: SIGUSR2 prints the native backtrace of the thread that
// receives it (hang diagnosis without a debugger: `kill -USR2 <pid>`)
void on_usr2(int) {
  void* fr[64];
  const int n = backtrace(fr, 64);
  const char hdr[] = "mrhip: SIGUSR2 native backtrace:\n";
  (void)!write(2, hdr, sizeof(hdr) - 1);
  backtrace_symbols_fd(fr, n, 2);
}
struct StackSignal {
  StackSignal() {
    const char* v = std::getenv("MRH_STACK_SIGNAL");
    if (v && *v == '1') signal(SIGUSR2, on_usr2);
  }
} g_stack_signal;

}  // namespace

int comm_timeout_seconds() { return std::max(1, env_int("MRH_COMM_TIMEOUT", 600)); }

void fault_point(const char* op, int rank) {
  std::lock_guard<std::mutex> l(g_mu);
  if (due(op, rank, "abort")) {
    std::fprintf(stderr, "MRH_FAULT: rank %d aborts at %s\n", rank, op);
    std::fflush(nullptr);
    std::_Exit(3);
  }
  if (due(op, rank, "throw")) throw std::runtime_error(std::string("MRH_FAULT: injected failure in ") + op);
}

void hip_check(hipError_t e, const char* site, int rank) {
  {
    std::lock_guard<std::mutex> l(g_mu);
    if (e == hipSuccess && due(site, rank, "hip")) e = hipErrorUnknown;  // injected (MRH_FAULT=hip:site:rank)
  }
  if (e != hipSuccess)
    throw std::runtime_error(std::string("mrhip: HIP error at ") + site + " on rank " + std::to_string(rank) + ": " +
                             hipGetErrorString(e));
}

bool fault_oom(const char* op, int rank) {
  std::lock_guard<std::mutex> l(g_mu);
  return due(op, rank, "oom");
}

bool check_enabled() {
  static const bool on = env_int("MRH_CHECK", 0) != 0;
  return on;
}

void check_kv(const KV& kv, const char* op) {
  if (kv.n < 0) bad(op, "negative pair count");
  check_col(kv.kdata, kv.koff, kv.kw, kv.n, op, "key");
  check_col(kv.vdata, kv.voff, kv.vw, kv.n, op, "value");
}

void check_kmv(const KMV& kmv, const char* op) {
  check_kv(kmv.keys, op);
  if (kmv.keys.n != kmv.nkey) bad(op, "KMV key count != unique keys");
  if (!kmv.seg.defined() || kmv.seg.numel() != kmv.nkey + 1) bad(op, "KMV segments must have nkey+1 entries");
  at::Tensor s = kmv.seg.to(at::kCPU);
  const int64_t* p = s.data_ptr<int64_t>();
  if (p[0] != 0 || p[kmv.nkey] != kmv.nval) bad(op, "KMV segments must span [0, nval]");
  if (kmv.nkey > 0 && (s.narrow(0, 1, kmv.nkey) < s.narrow(0, 0, kmv.nkey)).any().item<bool>())
    bad(op, "KMV segments are not monotone");
  check_col(kmv.vdata, kmv.voff, kmv.vw, kmv.nval, op, "multivalue");
}

bool trace_enabled() {
  static const bool on = std::getenv("MRH_TRACE") && *std::getenv("MRH_TRACE");
  return on;
}

void trace_op(int rank, const char* op, int instance, int depth, double t0, double ms, int64_t nkv, int64_t nkmv,
              int64_t bytes, int64_t sent, int64_t recv) {
  static std::FILE* f = nullptr;
  static int frank = -1;
  std::lock_guard<std::mutex> l(g_mu);
  if (!f || frank != rank) {
    if (f) std::fclose(f);
    const std::string p = std::string(std::getenv("MRH_TRACE")) + "." + std::to_string(rank);
    f = std::fopen(p.c_str(), "a");
    frank = rank;
    if (!f) return;
  }
  std::fprintf(f,
               "{\"op\": \"%s\", \"instance\": %d, \"depth\": %d, \"t0\": %.6f, \"ms\": %.4f, \"kv\": %lld, "
               "\"kmv\": %lld, \"bytes\": %lld, \"sent\": %lld, \"recv\": %lld}\n",
               op, instance, depth, t0, ms, (long long)nkv, (long long)nkmv, (long long)bytes, (long long)sent,
               (long long)recv);
  std::fflush(f);
}

void register_mr(MapReduce* mr) {
  std::lock_guard<std::mutex> l(g_mu);
  live().insert(mr);
}

void unregister_mr(MapReduce* mr) {
  std::lock_guard<std::mutex> l(g_mu);
  live().erase(mr);
}

int spill_others(const MapReduce* keep, at::Device dev) {
  std::vector<MapReduce*> victims;
  {
    std::lock_guard<std::mutex> l(g_mu);
    for (MapReduce* m : live())
      if (m != keep && m->set.outofcore != -1 && m->device() == dev &&
          ((m->kv && m->kv->device() == dev) || (m->kmv && m->kmv->keys.device() == dev)))
        victims.push_back(m);
  }
  for (MapReduce* m : victims) {
    try {
      m->spill();  // pinned host DRAM
    } catch (const std::exception&) {
      m->spill_disk();  // host memory exhausted too: last tier
    }
  }
  if (dev.is_cuda()) c10::hip::HIPCachingAllocator::emptyCache();
  if (!victims.empty())
    std::fprintf(stderr, "mrhip: out of device memory; spilled %zu MapReduce object(s) to host and retrying\n",
                 victims.size());
  return (int)victims.size();
}

}  // namespace mrh::guard
