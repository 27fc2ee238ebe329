// Native RCCL transport + peer monitor (see rccl.h).
#include "rccl.h"
#include "hbmpool.h"

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <map>

#include "guard.h"

namespace mrh {

namespace {
double now_s() {
  using namespace std::chrono;
  return duration<double>(steady_clock::now().time_since_epoch()).count();
}
int env_int(const char* k, int d) {
  const char* v = std::getenv(k);
  return v && *v ? std::atoi(v) : d;
}
double env_f(const char* k, double d) {
  const char* v = std::getenv(k);
  return v && *v ? std::atof(v) : d;
}
void hip_ok(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("mrhip rccl: ") + what + ": " + hipGetErrorString(e));
}
constexpr int64_t kPoison = -(int64_t(1) << 40);
}  // namespace

// point-to-point piece size asked for by this process: MRH_RCCL_MAX_MSG bytes
// (default 256 MiB; <= 0: whole messages). A communicator uses rank 0's value
// (Rccl: sent with the unique id; Comm's process-group path: broadcast at
// construction), so ranks with different environments still cut every
// transfer into the same pieces.
int64_t max_msg_env() {
  const char* e = std::getenv("MRH_RCCL_MAX_MSG");
  const long long v = e && *e ? std::atoll(e) : (1LL << 28);
  return v > 0 ? (int64_t)v : std::numeric_limits<int64_t>::max();
}

RcclCounters& rccl_counters() {
  static RcclCounters c;
  return c;
}
void rccl_counters_reset() {
  RcclCounters& c = rccl_counters();
  c.all_reduce = 0;
  c.all_gather = 0;
  c.broadcast = 0;
  c.send = 0;
  c.recv = 0;
  c.group = 0;
}

// ====================================================================== Monitor

Monitor::Monitor(c10::intrusive_ptr<c10d::Store> root, int rank, int size)
    : store_(std::move(root)), rank_(rank), size_(size), last_val_(size, -1), last_change_(size, now_s()) {
  peer_timeout_ = env_f("MRH_PEER_TIMEOUT", 5.0);
  store_->add(hb_key(rank_), 1);  // exists before any peer checks it
  thread_ = std::thread([this] { beat_loop(); });
}

// No retire() here: a process that tears its communicator down without the
// end-of-job handshake (an exception that escaped, exit() from an error path)
// must look like a crash to its peers, not like a clean exit.
Monitor::~Monitor() {
  stop_ = true;
  if (thread_.joinable()) thread_.join();
}

void Monitor::beat_loop() {
  const int ms = std::max(10, env_int("MRH_HEARTBEAT_MS", 250));
  while (!stop_) {
    for (int t = 0; t < ms && !stop_; t += 10) std::this_thread::sleep_for(std::chrono::milliseconds(10));
    if (stop_ || poisoned_) break;
    try {
      store_->add(hb_key(rank_), 1);
    } catch (const std::exception&) {
      break;  // store server gone: the job is ending one way or another
    }
  }
}

void Monitor::retire() {
  if (poisoned_ || retired_.exchange(true)) return;
  try {
    store_->set("mrh/bye/" + std::to_string(rank_), std::vector<uint8_t>{1});
  } catch (const std::exception&) {
  }
}

void Monitor::poison(const std::string& why) {
  if (poisoned_.exchange(true)) return;
  failed_ = true;
  try {
    store_->set("mrh/why/" + std::to_string(rank_), std::vector<uint8_t>(why.begin(), why.end()));
    store_->add(hb_key(rank_), kPoison);
  } catch (const std::exception&) {
    // store unreachable: peers detect the silent counter instead
  }
}

void Monitor::check() {
  std::lock_guard<std::mutex> l(mu_);
  if (failed_ && !why_.empty()) throw PeerFailure(why_);
  const double t = now_s();
  static const double gap = env_int("MRH_MONITOR_MS", 50) * 1e-3;
  if (t - last_check_ < gap) return;
  last_check_ = t;
  std::vector<std::string> keys;
  for (int r = 0; r < size_; ++r) keys.push_back(hb_key(r));
  std::vector<std::vector<uint8_t>> vals;
  try {
    vals = store_->multiGet(keys);
  } catch (const std::exception& e) {
    failed_ = true;
    why_ = std::string("mrhip: rendezvous store unreachable (rank 0 gone?): ") + e.what();
    throw PeerFailure(why_);
  }
  for (int r = 0; r < size_; ++r) {
    if (r == rank_) continue;
    const int64_t v = std::atoll(std::string(vals[r].begin(), vals[r].end()).c_str());
    if (v < 0) {
      std::string why;
      try {
        auto w = store_->get("mrh/why/" + std::to_string(r));
        why.assign(w.begin(), w.end());
      } catch (const std::exception&) {
      }
      failed_ = true;
      why_ = "mrhip: rank " + std::to_string(r) + " failed: " + why;
      throw PeerFailure(why_);
    }
    if (v != last_val_[r]) {
      last_val_[r] = v;
      last_change_[r] = t;
    } else if (t - last_change_[r] > peer_timeout_) {
      bool bye = false;
      try {
        bye = store_->check({"mrh/bye/" + std::to_string(r)});
      } catch (const std::exception&) {
      }
      if (bye) continue;
      failed_ = true;
      why_ = "mrhip: rank " + std::to_string(r) + " stopped responding (no heartbeat for " +
             std::to_string((int)(t - last_change_[r])) + " s): process crashed or was killed";
      throw PeerFailure(why_);
    }
  }
}

// ====================================================================== id rendezvous

namespace {
std::string members_tag(const std::vector<int>& members) {
  uint64_t h = 1469598103934665603ull;  // FNV-1a over the member list
  for (int m : members) {
    h ^= (uint64_t)(uint32_t)m;
    h *= 1099511628211ull;
  }
  char buf[48];
  std::snprintf(buf, sizeof(buf), "n%zu-%016llx", members.size(), (unsigned long long)h);
  return buf;
}

// wait (polling, bounded) until `key` exists in the store
void wait_key(const c10::intrusive_ptr<c10d::Store>& store, const std::string& key, Monitor* mon, const char* what) {
  const double t0 = now_s(), limit = guard::comm_timeout_seconds();
  int sleep_us = 50;
  while (!store->check({key})) {
    if (mon) mon->check();
    if (now_s() - t0 > limit)
      throw PeerFailure(std::string("mrhip rccl: timed out after ") + std::to_string((int)limit) + " s waiting for " +
                        what + " (" + key + ")");
    std::this_thread::sleep_for(std::chrono::microseconds(sleep_us));
    sleep_us = std::min(sleep_us * 2, 5000);
  }
}
}  // namespace

IdRendezvous rendezvous_id(const c10::intrusive_ptr<c10d::Store>& store, const std::string& tag,
                           const std::vector<int>& members, int rank,
                           const std::function<std::vector<uint8_t>()>& make_id, Monitor* mon) {
  if (!store) throw std::runtime_error("mrhip rccl: multi-rank communicator needs the rendezvous store");
  // the n-th communicator this process creates over this member set; every
  // member creates the same communicators in the same order, so the numbers agree
  static std::mutex mu;
  static std::map<std::string, int64_t> seq;
  const std::string base = "mrh/rccl_id/" + tag + "/" + members_tag(members);
  int64_t n;
  {
    std::lock_guard<std::mutex> l(mu);
    n = seq[base]++;
  }
  IdRendezvous r;
  r.key = base + "/" + std::to_string(n);
  if (rank == 0) {
    r.id = make_id();
    store->set(r.key, r.id);
  } else {
    wait_key(store, r.key, mon, "the communicator's unique id");
    r.id = store->get(r.key);
    store->add(r.key + "/ack", 1);
  }
  return r;
}

void rendezvous_release(const c10::intrusive_ptr<c10d::Store>& store, const IdRendezvous& r, int nmembers,
                        Monitor* mon) {
  const double t0 = now_s(), limit = guard::comm_timeout_seconds();
  while (store->add(r.key + "/ack", 0) < nmembers - 1) {
    if (mon) mon->check();
    if (now_s() - t0 > limit) throw PeerFailure("mrhip rccl: timed out waiting for unique-id acknowledgements");
    std::this_thread::sleep_for(std::chrono::microseconds(200));
  }
  store->deleteKey(r.key);
  store->deleteKey(r.key + "/ack");
}

// ====================================================================== Rccl

void Rccl::check(ncclResult_t r, const char* what) {
  if (r == ncclSuccess || r == ncclInProgress) return;
  std::string msg = std::string("mrhip rccl: ") + what + " failed: " + ncclGetErrorString(r);
  if (comm_) {
    const char* last = ncclGetLastError(comm_);
    if (last && *last) msg += std::string(" (") + last + ")";
  }
  throw std::runtime_error(msg);
}

Rccl::Rccl(int rank, int size, int device, const c10::intrusive_ptr<c10d::Store>& store, const std::string& tag,
           const std::vector<int>& members_in, Monitor* mon)
    : rank_(rank), size_(size) {
  hip_ok(hipSetDevice(device), "hipSetDevice");
  ncclUniqueId id;
  IdRendezvous rv;
  max_msg_ = max_msg_env();
  if (size == 1) {
    check(ncclGetUniqueId(&id), "ncclGetUniqueId");
  } else {
    std::vector<int> members = members_in;
    if (members.empty())
      for (int r = 0; r < size; ++r) members.push_back(r);
    if ((int)members.size() != size) throw std::runtime_error("mrhip rccl: member list does not match the size");
    // the payload: the unique id, then rank 0's piece size
    rv = rendezvous_id(store, tag, members, rank, [&] {
      ncclUniqueId u;
      check(ncclGetUniqueId(&u), "ncclGetUniqueId");
      std::vector<uint8_t> b((uint8_t*)&u, (uint8_t*)&u + sizeof(u));
      b.resize(sizeof(u) + sizeof(int64_t));
      std::memcpy(b.data() + sizeof(u), &max_msg_, sizeof(int64_t));
      return b;
    }, mon);
    if (rv.id.size() != sizeof(id) + sizeof(int64_t)) throw std::runtime_error("mrhip rccl: bad unique id in store");
    std::memcpy(&id, rv.id.data(), sizeof(id));
    std::memcpy(&max_msg_, rv.id.data() + sizeof(id), sizeof(int64_t));
    id_key_ = rv.key;
  }
  check(ncclCommInitRank(&comm_, size, id, rank), "ncclCommInitRank");
  // ncclCommInitRank returns once every member joined, so every reader is done
  if (size > 1 && rank == 0) rendezvous_release(store, rv, size, mon);
  int lo = 0, hi = 0;
  hip_ok(hipDeviceGetStreamPriorityRange(&lo, &hi), "hipDeviceGetStreamPriorityRange");
  hip_ok(hipStreamCreateWithPriority(&stream_, hipStreamNonBlocking, hi), "hipStreamCreateWithPriority");
  ev_.resize(64);
  for (auto& e : ev_) hip_ok(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
}

// teardown cannot throw: statuses here are deliberately ignored (an aborted
// communicator's stream may report the abort)
Rccl::~Rccl() {
  if (stream_) {
    if (!aborted_) (void)hipStreamSynchronize(stream_);
  }
  if (comm_) {
    if (aborted_) {
      // already aborted: nothing left to release
    } else {
      (void)ncclCommDestroy(comm_);
    }
  }
  for (auto& e : ev_) (void)hipEventDestroy(e);
  if (stream_) {
    // an aborted communicator's stream may never drain: drop the pool's
    // references to it without waiting (a later event record on a destroyed
    // stream is the segfault class of hbm::forget_stream)
    if (aborted_) hbm::forget_stream_nosync(stream_);
    else hbm::forget_stream(stream_);
    (void)hipStreamDestroy(stream_);
  }
}

void Rccl::fence_in(hipStream_t s) {
  hipEvent_t e = ev_[ev_next_++ % ev_.size()];
  hip_ok(hipEventRecord(e, s), "hipEventRecord");
  hip_ok(hipStreamWaitEvent(stream_, e, 0), "hipStreamWaitEvent");
}

hipEvent_t Rccl::fence_out() {
  hipEvent_t e = ev_[ev_next_++ % ev_.size()];
  hip_ok(hipEventRecord(e, stream_), "hipEventRecord");
  return e;
}

hipEvent_t Rccl::sendrecv_async(const std::vector<Xfer>& sends, const std::vector<Xfer>& recvs, hipStream_t s) {
  if (aborted_) throw PeerFailure("mrhip rccl: communicator aborted");
  fence_in(s);
  // one transfer is posted as pieces of at most max_msg_ bytes (agreed at
  // init: both ends cut the same byte count the same way): on MI355X (RCCL
  // 2.26.6) a single point-to-point message of 1 GiB + 40 bytes came back
  // wrong from element 67141632 on (~512 MiB) while the same data in 1 GiB
  // pieces arrived intact up to 4 GiB (profiles/r4_rccl_big_messages.txt;
  // tests/test_rccl_gpu.py test_forced_rccl_large_transfers_bitwise)
  const int64_t max_msg = max_msg_;
  RcclCounters& cnt = rccl_counters();
  check(ncclGroupStart(), "ncclGroupStart");
  for (const Xfer& x : recvs)
    for (int64_t o = 0; o < x.bytes; o += max_msg) {
      check(ncclRecv((uint8_t*)x.ptr + o, (size_t)std::min(max_msg, x.bytes - o), ncclUint8, x.peer, comm_, stream_),
            "ncclRecv");
      ++cnt.recv;
    }
  for (const Xfer& x : sends)
    for (int64_t o = 0; o < x.bytes; o += max_msg) {
      check(ncclSend((uint8_t*)x.ptr + o, (size_t)std::min(max_msg, x.bytes - o), ncclUint8, x.peer, comm_, stream_),
            "ncclSend");
      ++cnt.send;
    }
  check(ncclGroupEnd(), "ncclGroupEnd");
  ++cnt.group;
  return fence_out();
}

void Rccl::sendrecv(const std::vector<Xfer>& sends, const std::vector<Xfer>& recvs, hipStream_t s) {
  hipEvent_t e = sendrecv_async(sends, recvs, s);
  hip_ok(hipStreamWaitEvent(s, e, 0), "hipStreamWaitEvent");
}

void Rccl::allreduce(void* buf, size_t count, ncclDataType_t dt, ncclRedOp_t op, hipStream_t s) {
  if (aborted_) throw PeerFailure("mrhip rccl: communicator aborted");
  fence_in(s);
  check(ncclAllReduce(buf, buf, count, dt, op, comm_, stream_), "ncclAllReduce");
  ++rccl_counters().all_reduce;
  hip_ok(hipStreamWaitEvent(s, fence_out(), 0), "hipStreamWaitEvent");
}

void Rccl::allgather(const void* send, void* recv, size_t bytes, hipStream_t s) {
  if (aborted_) throw PeerFailure("mrhip rccl: communicator aborted");
  fence_in(s);
  check(ncclAllGather(send, recv, bytes, ncclUint8, comm_, stream_), "ncclAllGather");
  ++rccl_counters().all_gather;
  hip_ok(hipStreamWaitEvent(s, fence_out(), 0), "hipStreamWaitEvent");
}

void Rccl::broadcast(void* buf, size_t bytes, int root, hipStream_t s) {
  if (aborted_) throw PeerFailure("mrhip rccl: communicator aborted");
  fence_in(s);
  check(ncclBroadcast(buf, buf, bytes, ncclUint8, root, comm_, stream_), "ncclBroadcast");
  ++rccl_counters().broadcast;
  hip_ok(hipStreamWaitEvent(s, fence_out(), 0), "hipStreamWaitEvent");
}

int Rccl::comm_count() {
  int n = 0;
  check(ncclCommCount(comm_, &n), "ncclCommCount");
  return n;
}
int Rccl::cu_device() {
  int d = -1;
  check(ncclCommCuDevice(comm_, &d), "ncclCommCuDevice");
  return d;
}
int Rccl::user_rank() {
  int r = -1;
  check(ncclCommUserRank(comm_, &r), "ncclCommUserRank");
  return r;
}

namespace {
std::mutex g_rccl_mu;
std::map<std::string, std::weak_ptr<Rccl>> g_rccl;
}  // namespace

std::shared_ptr<Rccl> shared_rccl(int rank, int size, int device, const c10::intrusive_ptr<c10d::Store>& store,
                                  const std::string& tag, const std::vector<int>& members, Monitor* mon) {
  std::string k = std::to_string((uintptr_t)store.get()) + "|" + tag + "|" + std::to_string(device) + "|" +
                  std::to_string(size) + "|" + std::to_string(rank);
  for (int m : members) k += "," + std::to_string(m);
  std::lock_guard<std::mutex> l(g_rccl_mu);
  auto& w = g_rccl[k];
  if (auto r = w.lock()) return r;
  auto r = std::make_shared<Rccl>(rank, size, device, store, tag, members, mon);
  w = r;
  return r;
}

int live_rccl_comms() {
  std::lock_guard<std::mutex> l(g_rccl_mu);
  int n = 0;
  for (auto& kv : g_rccl) n += kv.second.expired() ? 0 : 1;
  return n;
}

// Diagnostic: one RCCL operation on a one-rank communicator, eagerly and then
// captured into a HIP graph (ThreadLocal capture on a non-blocking stream, as
// the PageRank plan does) and replayed; each step is logged to stderr first
// so a crash names it. what: allreduce | allgather | broadcast | self (send to
// a second buffer) | self_inplace. Returns "ok" or the failed check.
std::string rccl_graph_probe(int device, const std::string& what, bool capture, int mode) {
  auto step = [](const char* m) {
    std::fprintf(stderr, "[rccl_graph_probe] %s\n", m);
    std::fflush(stderr);
  };
  hip_ok(hipSetDevice(device), "hipSetDevice");
  Rccl r(0, 1, device, c10::intrusive_ptr<c10d::Store>(), "gprobe");
  hipStream_t s = nullptr;
  hip_ok(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "hipStreamCreate");
  const size_t n = 1 << 16;
  std::vector<float> h(2 * n);
  for (size_t i = 0; i < 2 * n; ++i) h[i] = (float)(i % 977) + 0.5f;
  float* a = nullptr;
  hip_ok(hipMalloc((void**)&a, 2 * n * sizeof(float)), "hipMalloc");
  hip_ok(hipMemcpy(a, h.data(), 2 * n * sizeof(float), hipMemcpyHostToDevice), "hipMemcpy");
  const int64_t bytes = (int64_t)(n * sizeof(float));
  // "k_<op>": the op between two device copies of the second half onto
  // itself, so the captured graph is not empty (the PageRank iteration's
  // kernels around its RCCL rounds)
  const bool bracket = what.rfind("k_", 0) == 0;
  const std::string op = bracket ? what.substr(2) : what;
  auto touch = [&] {
    if (bracket) hip_ok(hipMemcpyAsync(a + n, a + n, (size_t)bytes, hipMemcpyDeviceToDevice, s), "hipMemcpyAsync");
  };
  auto enqueue = [&] {
    touch();
    if (op == "allreduce") r.allreduce(a, n, ncclFloat32, ncclSum, s);
    else if (op == "allgather") r.allgather(a, a, (size_t)bytes, s);
    else if (op == "broadcast") r.broadcast(a, (size_t)bytes, 0, s);
    else if (op == "self") r.sendrecv({Xfer{0, a, bytes}}, {Xfer{0, a + n, bytes}}, s);
    else if (op == "self_inplace") r.sendrecv({Xfer{0, a, bytes}}, {Xfer{0, a, bytes}}, s);
    else throw std::runtime_error("rccl_graph_probe: unknown op " + what);
    touch();
  };
  step("eager");
  enqueue();
  hip_ok(hipStreamSynchronize(s), "hipStreamSynchronize (eager)");
  if (capture) {
    hipGraph_t g = nullptr;
    hipGraphExec_t ge = nullptr;
    step("begin capture");
    const hipStreamCaptureMode cm = mode == 0 ? hipStreamCaptureModeGlobal
                                    : mode == 2 ? hipStreamCaptureModeRelaxed : hipStreamCaptureModeThreadLocal;
    hip_ok(hipStreamBeginCapture(s, cm), "hipStreamBeginCapture");
    step("enqueue under capture");
    enqueue();
    step("end capture");
    hip_ok(hipStreamEndCapture(s, &g), "hipStreamEndCapture");
    size_t nn = 0;
    hip_ok(hipGraphGetNodes(g, nullptr, &nn), "hipGraphGetNodes");
    std::fprintf(stderr, "[rccl_graph_probe] graph nodes: %zu\n", nn);
    step("instantiate");
    hip_ok(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0), "hipGraphInstantiate");
    for (int i = 0; i < 3; ++i) {
      step("launch");
      hip_ok(hipGraphLaunch(ge, s), "hipGraphLaunch");
    }
    hip_ok(hipStreamSynchronize(s), "hipStreamSynchronize (replay)");
    step("replayed");
    (void)hipGraphExecDestroy(ge);
    (void)hipGraphDestroy(g);
  }
  std::vector<float> o(2 * n);
  hip_ok(hipMemcpy(o.data(), a, 2 * n * sizeof(float), hipMemcpyDeviceToHost), "hipMemcpy back");
  (void)hipFree(a);
  (void)hipStreamDestroy(s);
  for (size_t i = 0; i < n; ++i) {
    const float want_hi = op == "self" ? h[i] : h[n + i];
    if (o[i] != h[i] || o[n + i] != want_hi) return "mismatch at " + std::to_string(i);
  }
  return "ok";
}

ncclResult_t Rccl::async_error() {
  if (!comm_ || aborted_) return ncclSuccess;
  ncclResult_t r = ncclSuccess;
  if (ncclCommGetAsyncError(comm_, &r) != ncclSuccess) return ncclSystemError;
  return r;
}

void Rccl::abort() {
  if (aborted_ || !comm_) return;
  aborted_ = true;
  (void)ncclCommAbort(comm_);
}

}  // namespace mrh
