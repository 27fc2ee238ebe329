// Native communicator (see comm.h).
#include "comm.h"

#include <numeric>
#include "guardalloc.h"
#include "hbmpool.h"

#include <ATen/hip/HIPContext.h>
#include <c10/hip/HIPFunctions.h>
#include <hip/hip_runtime.h>
#include <torch/csrc/distributed/c10d/PrefixStore.hpp>
#include <torch/csrc/distributed/c10d/TCPStore.hpp>
#include <torch/csrc/distributed/c10d/Types.hpp>

#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <stdexcept>
#include <thread>

#include "guard.h"
#include "storepg.h"

namespace mrh {

namespace {
int env_int(const char* k, int d) {
  const char* v = std::getenv(k);
  return v && *v ? std::atoi(v) : d;
}
// MRH_FORCE_RCCL: 0 = a one-rank job has no communicator; 1 = it gets a
// one-rank RCCL communicator whose data plane (send/recv rounds) runs through
// RCCL while the collectives stay the identity; 2 = every collective also
// calls its nccl* function (allreduce, all-gather, broadcast, the scalar
// allreduce / bcast), so each RCCL call site of the multi-GPU paths executes
// on one GPU (RCCL accepts nranks = 1)
int force_rccl_level() { return env_int("MRH_FORCE_RCCL", 0); }
bool force_rccl() { return force_rccl_level() != 0; }

c10d::ReduceOp::RedOpType red(Comm::Op op) {
  return op == Comm::SUM ? c10d::ReduceOp::SUM : op == Comm::MAX ? c10d::ReduceOp::MAX : c10d::ReduceOp::MIN;
}
ncclRedOp_t nred(Comm::Op op) { return op == Comm::SUM ? ncclSum : op == Comm::MAX ? ncclMax : ncclMin; }
ncclDataType_t ndt(at::ScalarType t) {
  switch (t) {
    case at::kLong: return ncclInt64;
    case at::kInt: return ncclInt32;
    case at::kDouble: return ncclFloat64;
    case at::kFloat: return ncclFloat32;
    case at::kByte: return ncclUint8;
    default: throw std::runtime_error("mrhip: unsupported allreduce dtype");
  }
}
void pg_allreduce(const PG& pg, at::Tensor& t, Comm::Op op) {
  std::vector<at::Tensor> v{t};
  c10d::AllreduceOptions o;
  o.reduceOp = c10d::ReduceOp(red(op));
  pg->allreduce(v, o)->wait();
  t = v[0];
}
hipStream_t cur(at::Device d) { return at::hip::getCurrentHIPStream(d.index()).stream(); }

// MRH_TRACE_COLL=1: one stderr line per collective (sequence, kind, bytes) to
// diff the collective order of ranks after a hang
void trace_coll(int rank, const char* kind, int64_t a, int64_t b) {
  static const bool on = env_int("MRH_TRACE_COLL", 0) != 0;
  if (!on) return;
  static std::atomic<int64_t> seq{0};
  std::fprintf(stderr, "[coll r%d #%lld] %s %lld %lld\n", rank, (long long)seq++, kind, (long long)a, (long long)b);
}

// one heartbeat monitor per (process, root store)
std::shared_ptr<Monitor> shared_monitor(const c10::intrusive_ptr<c10d::Store>& store, int rank, int size) {
  if (env_int("MRH_MONITOR", 1) == 0) return nullptr;  // no heartbeats / peer checks (debugging)
  static std::mutex mu;
  static std::map<c10d::Store*, std::weak_ptr<Monitor>> reg;
  std::lock_guard<std::mutex> l(mu);
  auto& w = reg[store.get()];
  if (auto m = w.lock()) return m;
  auto m = std::make_shared<Monitor>(store, rank, size);
  w = m;
  return m;
}

// bytes of a per-peer list of transfers, peer order, as one contiguous tensor
void copy_bytes(void* dst, const void* src, int64_t n, at::Device dev) {
  if (n <= 0) return;
  if (dev.is_cuda()) {
    if (hipMemcpyAsync(dst, src, (size_t)n, hipMemcpyDeviceToDevice, cur(dev)) != hipSuccess)
      throw std::runtime_error("mrhip: device copy failed");
  } else {
    std::memcpy(dst, src, (size_t)n);
  }
}
}  // namespace

// the job's device allocator, before its first HBM allocation: MRH_GUARD's
// canaried allocator, else the HBM page pool (hbmpool.h) unless MRH_HBM_POOL=0
// (a no-op when the process already allocated device memory)
static void install_allocator() {
  guard::install_alloc_guard();
  if (!guard::alloc_guard_active()) hbm::install_default();
}

Comm::Comm(at::Device dev) : dev_(dev) {
  if (dev_.is_cuda()) install_allocator();
  if (dev_.is_cuda() && force_rccl()) init_transport("", "self");
  loop_coll_ = rccl_ && force_rccl_level() >= 2;
  max_msg_ = rccl_ ? rccl_->max_msg() : max_msg_env();
}

Comm::Comm(PG pg, at::Device dev, c10::intrusive_ptr<c10d::Store> store, const std::string& transport,
           std::vector<int> members, int world_rank, int world_size)
    : dev_(dev), pg_(std::move(pg)), store_(std::move(store)) {
  if (dev_.is_cuda()) install_allocator();
  if (pg_) {
    rank_ = pg_->getRank();
    size_ = pg_->getSize();
  }
  if (members.empty())
    for (int r = 0; r < size_; ++r) members.push_back(r);
  if ((int)members.size() != size_) throw std::runtime_error("mrhip: member list does not match the group size");
  members_ = std::move(members);
  if (world_rank < 0) world_rank = members_[rank_];
  if (world_size < 0) world_size = size_;
  if (world_size > 1 && store_) mon_ = shared_monitor(store_, world_rank, world_size);
  if (size_ == 1) pg_.reset();
  // host scalars need a CPU backend on the group (gloo / the store
  // transport); an nccl-only group moves them as device tensors instead
  if (pg_) {
    try {
      host_pg_ = (bool)pg_->getBackend(c10::DeviceType::CPU);
    } catch (const std::exception&) {
      host_pg_ = false;
    }
  }
  init_transport(transport, "world");
  loop_coll_ = rccl_ && size_ == 1 && force_rccl_level() >= 2;
  // rank 0's piece size on every rank (a collective: every member constructs)
  if (rccl_) {
    max_msg_ = rccl_->max_msg();
  } else {
    const int64_t mine = max_msg_env();
    max_msg_ = size_ > 1 && pg_ ? allreduce(rank_ == 0 ? mine : 0, SUM) : mine;
  }
}

void Comm::init_transport(const std::string& transport, const std::string& tag) {
  if (!dev_.is_cuda() || transport == "pg") return;
  if (size_ == 1 && !force_rccl()) return;
  if (size_ > 1 && !store_) {
    if (pg_) return;  // no store to bootstrap from: keep the process group
    throw std::runtime_error("mrhip: multi-rank RCCL communicator needs a rendezvous store");
  }
  // one RCCL communicator per (member set, device) per process, shared by
  // every Comm over the same ranks
  // a device without an index ("cuda") means the current one
  rccl_ = shared_rccl(rank_, size_, rccl_device(), store_, tag, members_, mon_.get());
}

Comm::~Comm() = default;

int Comm::rccl_device() const { return dev_.has_index() ? dev_.index() : (int)c10::hip::current_device(); }

std::string Comm::transport() const {
  if (rccl_) return "rccl";
  if (pg_) return "pg:" + pg_->getBackendName();
  return "local";
}

std::shared_ptr<Comm> Comm::from_env() {
  const int ws = env_int("WORLD_SIZE", 1), rank = env_int("RANK", 0), local = env_int("LOCAL_RANK", 0);
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess) ndev = 0;
  at::Device dev(at::kCPU);
  if (ndev > 0) {
    const int d = local % ndev;
    c10::hip::set_device(d);
    dev = at::Device(at::kCUDA, d);
  }
  if (ws <= 1) return std::make_shared<Comm>(dev);
  const char* addr = std::getenv("MASTER_ADDR");
  c10d::TCPStoreOptions so;
  so.port = (uint16_t)env_int("MASTER_PORT", 29500);
  so.isServer = rank == 0;
  so.numWorkers = ws;
  so.timeout = std::chrono::milliseconds(1000LL * guard::comm_timeout_seconds());
  c10::intrusive_ptr<c10d::Store> store = c10::make_intrusive<c10d::TCPStore>(addr ? addr : "127.0.0.1", so);
  auto mon = shared_monitor(store, rank, ws);
  const bool pg_only = dev.is_cpu() || (std::getenv("MRH_TRANSPORT") && std::string(std::getenv("MRH_TRANSPORT")) == "pg");
  PG pg = make_host_pg(store, rank, ws, mon);
  return std::make_shared<Comm>(pg, dev, store, pg_only ? "pg" : "");
}

// the store transport (storepg.h): host tensors only
PG Comm::make_host_pg(const c10::intrusive_ptr<c10d::Store>& store, int rank, int size, std::shared_ptr<Monitor> mon) {
  auto pg = c10::make_intrusive<c10d::ProcessGroup>(store, rank, size);
  auto be = c10::make_intrusive<StoreBackend>(store, rank, size, std::move(mon));
  pg->setBackend(c10::DeviceType::CPU, c10d::ProcessGroup::BackendType::CUSTOM, be);
  pg->setDefaultBackend(c10d::ProcessGroup::BackendType::CUSTOM);
  return pg;
}

// ---------------------------------------------------------------- failure handling

void Comm::check_peers() const {
  if (mon_) mon_->check();
}

void Comm::fail_now(const std::string& why) const {
  if (mon_) mon_->poison(why);
  if (rccl_) rccl_->abort();
  throw PeerFailure(why);
}

void Comm::poison(const std::string& why) const {
  if (mon_) mon_->poison(why);
  if (rccl_) rccl_->abort();
}

void Comm::host_wait() const {
  if (!dev_.is_cuda()) return;
  hipEvent_t ev;
  if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess)
    throw std::runtime_error("mrhip: hipEventCreate failed");
  struct Drop {
    hipEvent_t e;
    ~Drop() { (void)hipEventDestroy(e); }  // destructor: cannot throw
  } drop{ev};
  if (hipEventRecord(ev, cur(dev_)) != hipSuccess) throw std::runtime_error("mrhip: hipEventRecord failed");
  // the deadline replaces the watchdog of a c10d RCCL group: a collective
  // whose peer never posts its half cannot block this rank forever
  const bool bounded = distributed() && size_ > 1;
  const double t0 = bounded ? wtime() : 0.0, limit = guard::comm_timeout_seconds();
  for (int spin = 0;; ++spin) {
    const hipError_t q = hipEventQuery(ev);
    if (q == hipSuccess) return;
    if (q != hipErrorNotReady) throw std::runtime_error(std::string("mrhip: device error: ") + hipGetErrorString(q));
    if (bounded && (spin & 255) == 0 && wtime() - t0 > limit)
      fail_now("mrhip: device work did not complete within MRH_COMM_TIMEOUT=" + std::to_string((int)limit) +
               " s (a collective whose peers never joined?)");
    if (rccl_) {
      const ncclResult_t r = rccl_->async_error();
      if (r != ncclSuccess && r != ncclInProgress)
        fail_now(std::string("mrhip: RCCL async error: ") + ncclGetErrorString(r));
    }
    if (mon_) {
      try {
        mon_->check();
      } catch (const PeerFailure& e) {
        fail_now(e.what());
      }
    }
    if (spin > 64) std::this_thread::sleep_for(std::chrono::microseconds(spin > 4096 ? 200 : 20));
  }
}

// ---------------------------------------------------------------- scalars

std::vector<int64_t> Comm::allreduce(std::vector<int64_t> v, Op op) const {
  // one rank (MRH_FORCE_RCCL=1 included): identity, no device round trip
  if (v.empty() || identity_coll()) return v;
  trace_coll(rank_, "allreduce_i64", (int64_t)v.size(), op);
  at::Tensor t = at::tensor(v, at::TensorOptions().dtype(at::kLong));
  if (host_scalars()) {
    pg_allreduce(pg_, t, op);
  } else if (rccl_) {
    t = t.to(dev_);
    rccl_->allreduce(t.data_ptr(), v.size(), ncclInt64, nred(op), cur(dev_));
    host_wait();
    t = t.to(at::kCPU);
  } else if (pg_) {  // a group without a CPU backend: device tensors through it
    t = t.to(dev_);
    pg_allreduce(pg_, t, op);
    t = t.to(at::kCPU);
  }
  std::memcpy(v.data(), t.data_ptr<int64_t>(), v.size() * sizeof(int64_t));
  return v;
}

std::vector<double> Comm::allreduce_f64(std::vector<double> v, Op op) const {
  if (v.empty() || identity_coll()) return v;
  trace_coll(rank_, "allreduce_f64", (int64_t)v.size(), op);
  at::Tensor t = at::tensor(v, at::TensorOptions().dtype(at::kDouble));
  if (host_scalars()) {
    pg_allreduce(pg_, t, op);
  } else if (rccl_) {
    t = t.to(dev_);
    rccl_->allreduce(t.data_ptr(), v.size(), ncclFloat64, nred(op), cur(dev_));
    host_wait();
    t = t.to(at::kCPU);
  } else if (pg_) {
    t = t.to(dev_);
    pg_allreduce(pg_, t, op);
    t = t.to(at::kCPU);
  }
  std::memcpy(v.data(), t.data_ptr<double>(), v.size() * sizeof(double));
  return v;
}

std::vector<double> Comm::allgather_f64(double x) const {
  std::vector<double> v(size_, 0.0);
  v[rank_] = x;
  return allreduce_f64(v, SUM);
}

std::string Comm::bcast(const std::string& s, int root) const {
  if (identity_coll()) return s;
  int64_t n = rank_ == root ? (int64_t)s.size() : 0;
  n = allreduce(n, SUM);
  at::Tensor t = at::zeros({std::max<int64_t>(n, 1)}, at::TensorOptions().dtype(at::kByte));
  if (rank_ == root && n) std::memcpy(t.data_ptr(), s.data(), n);
  if (host_scalars()) {
    std::vector<at::Tensor> v{t};
    c10d::BroadcastOptions bo;
    bo.rootRank = root;
    pg_->broadcast(v, bo)->wait();
    t = v[0];
  } else {
    t = t.to(dev_);
    broadcast_tensor(t, root);
    if (rccl_) host_wait();
    t = t.to(at::kCPU);
  }
  return std::string((const char*)t.data_ptr(), (size_t)n);
}

void Comm::barrier() const {
  if (!distributed()) return;
  allreduce((int64_t)0, SUM);
}

double Comm::wtime() {
  using namespace std::chrono;
  return duration<double>(steady_clock::now().time_since_epoch()).count();
}

// ---------------------------------------------------------------- data plane

void Comm::sendrecv(const std::vector<Xfer>& sends, const std::vector<Xfer>& recvs) const {
  {
    int64_t a = 0, b = 0;
    for (auto& x : sends) a += x.bytes;
    for (auto& x : recvs) b += x.bytes;
    trace_coll(rank_, "sendrecv", a, b);
  }
  if (rccl_) {
    rccl_->sendrecv(sends, recvs, cur(dev_));
    return;
  }
  if (!pg_) {  // world size 1: self copies, in order
    size_t j = 0;
    for (const Xfer& s : sends) {
      while (j < recvs.size() && recvs[j].bytes == 0) ++j;
      if (s.bytes == 0) continue;
      if (j >= recvs.size() || recvs[j].bytes != s.bytes) throw std::runtime_error("mrhip sendrecv: unmatched self transfer");
      copy_bytes(recvs[j].ptr, s.ptr, s.bytes, dev_);
      ++j;
    }
    return;
  }
  // process group: pack per peer in order, byte all-to-alls of at most
  // max_msg_ bytes per peer each (the round count agreed: a pair's bytes are
  // known to both ends, the longest pair sets it), unpack
  const int P = size_;
  std::vector<int64_t> sb(P, 0), rb(P, 0);
  for (const Xfer& x : sends) sb[x.peer] += x.bytes;
  for (const Xfer& x : recvs) rb[x.peer] += x.bytes;
  std::vector<int64_t> soff(P + 1, 0), roff(P + 1, 0);
  for (int p = 0; p < P; ++p) {
    soff[p + 1] = soff[p] + sb[p];
    roff[p + 1] = roff[p] + rb[p];
  }
  const int64_t st = soff[P], rt = roff[P];
  auto bo = at::TensorOptions().device(dev_).dtype(at::kByte);
  at::Tensor sbuf = at::empty({st}, bo), rbuf = at::empty({rt}, bo);
  std::vector<int64_t> fill = soff;
  for (const Xfer& x : sends) {
    copy_bytes((uint8_t*)sbuf.data_ptr() + fill[x.peer], x.ptr, x.bytes, dev_);
    fill[x.peer] += x.bytes;
  }
  const int64_t m = std::max<int64_t>(max_msg_, 1);
  // pieces of m bytes (no (b + m - 1) / m: m may be INT64_MAX, "no limit")
  auto npieces = [m](int64_t b) { return b <= 0 ? int64_t(0) : 1 + (b - 1) / m; };
  int64_t rounds = 1;
  for (int p = 0; p < P; ++p) rounds = std::max({rounds, npieces(sb[p]), npieces(rb[p])});
  rounds = allreduce(rounds, MAX);
  if (rounds == 1) {
    pg_->alltoall_base(rbuf, sbuf, rb, sb)->wait();
  } else {
    for (int64_t r = 0; r < rounds; ++r) {
      std::vector<int64_t> ps(P), pr(P);
      std::vector<at::Tensor> sp, rp;
      for (int p = 0; p < P; ++p) {
        const int64_t a = std::min(sb[p], r * m), b = std::min(sb[p], (r + 1) * m);
        const int64_t c = std::min(rb[p], r * m), d = std::min(rb[p], (r + 1) * m);
        ps[p] = b - a;
        pr[p] = d - c;
        sp.push_back(sbuf.narrow(0, soff[p] + a, b - a));
        rp.push_back(rbuf.narrow(0, roff[p] + c, d - c));
      }
      at::Tensor s1 = at::cat(sp), r1 = at::empty({std::accumulate(pr.begin(), pr.end(), int64_t(0))}, bo);
      pg_->alltoall_base(r1, s1, pr, ps)->wait();
      int64_t o = 0;
      for (int p = 0; p < P; ++p) {
        if (pr[p]) rp[p].copy_(r1.narrow(0, o, pr[p]));
        o += pr[p];
      }
    }
  }
  fill = roff;
  for (const Xfer& x : recvs) {
    copy_bytes(x.ptr, (uint8_t*)rbuf.data_ptr() + fill[x.peer], x.bytes, dev_);
    fill[x.peer] += x.bytes;
  }
  if (dev_.is_cuda()) host_wait();  // staging buffers die here
}

void Comm::allgather_bytes(const void* send, void* recv, int64_t bytes) const {
  trace_coll(rank_, "allgather", bytes, 0);
  if (size_ == 1 && !loop_coll_) {  // one rank (MRH_FORCE_RCCL=1): the identity, no collective kernel
    if (send != recv) copy_bytes(recv, send, bytes, dev_);
    return;
  }
  if (rccl_) {
    rccl_->allgather(send, recv, (size_t)bytes, cur(dev_));
    return;
  }
  if (!pg_) {
    copy_bytes(recv, send, bytes, dev_);
    return;
  }
  // process group: the block to every peer through the all-to-all (every
  // backend here implements it; gloo's and the store's allgather flavours differ)
  std::vector<Xfer> xs, xr;
  for (int p = 0; p < size_; ++p) {
    xs.push_back({p, const_cast<void*>(send), bytes});
    xr.push_back({p, (uint8_t*)recv + p * bytes, bytes});
  }
  sendrecv(xs, xr);
}

std::vector<int64_t> Comm::alltoall_counts(const std::vector<int64_t>& send) const {
  if (!distributed()) return send;
  auto lo = at::TensorOptions().dtype(at::kLong);
  at::Tensor s = at::tensor(send, lo).to(dev_);
  at::Tensor r = at::empty({size_}, lo.device(dev_));
  std::vector<Xfer> xs, xr;
  for (int p = 0; p < size_; ++p) {
    xs.push_back({p, s.data_ptr<int64_t>() + p, 8});
    xr.push_back({p, r.data_ptr<int64_t>() + p, 8});
  }
  sendrecv(xs, xr);
  host_wait();
  r = r.to(at::kCPU);
  return std::vector<int64_t>(r.data_ptr<int64_t>(), r.data_ptr<int64_t>() + size_);
}

at::Tensor Comm::alltoallv(const at::Tensor& in, const std::vector<int64_t>& send,
                           const std::vector<int64_t>& recv) const {
  if (!distributed()) return in;
  int64_t tot = 0;
  for (auto x : recv) tot += x;
  std::vector<int64_t> shape = in.sizes().vec();
  shape[0] = tot;
  at::Tensor out = at::empty(shape, in.options());
  at::Tensor src = in.contiguous();
  const int64_t row = (in.dim() > 1 ? src.numel() / std::max<int64_t>(1, in.size(0)) : 1) * in.element_size();
  std::vector<Xfer> xs, xr;
  int64_t so = 0, ro = 0;
  for (int p = 0; p < size_; ++p) {
    xs.push_back({p, (uint8_t*)src.data_ptr() + so * row, send[p] * row});
    xr.push_back({p, (uint8_t*)out.data_ptr() + ro * row, recv[p] * row});
    so += send[p];
    ro += recv[p];
  }
  sendrecv(xs, xr);
  return out;
}

at::Tensor Comm::allgather_var(const at::Tensor& in) const {
  if (!distributed()) return in;
  std::vector<double> sizes = allgather_f64((double)in.numel());
  int64_t tot = 0;
  for (double s : sizes) tot += (int64_t)s;
  at::Tensor src = in.contiguous().reshape({-1});
  at::Tensor out = at::empty({tot}, in.options());
  const int64_t es = in.element_size();
  std::vector<Xfer> xs, xr;
  int64_t o = 0;
  for (int p = 0; p < size_; ++p) {
    xs.push_back({p, src.data_ptr(), src.numel() * es});
    xr.push_back({p, (uint8_t*)out.data_ptr() + o * es, (int64_t)sizes[p] * es});
    o += (int64_t)sizes[p];
  }
  sendrecv(xs, xr);
  return out;
}

void Comm::allreduce_tensor(at::Tensor& t, Op op) const {
  if (identity_coll()) return;
  trace_coll(rank_, "allreduce_tensor", t.numel(), op);
  if (rccl_) {
    if (!t.is_contiguous()) t = t.contiguous();
    rccl_->allreduce(t.data_ptr(), (size_t)t.numel(), ndt(t.scalar_type()), nred(op), cur(dev_));
    return;
  }
  pg_allreduce(pg_, t, op);
}

void Comm::broadcast_tensor(at::Tensor& t, int root) const {
  if (identity_coll()) return;
  trace_coll(rank_, "broadcast", t.numel(), root);
  if (rccl_) {
    if (!t.is_contiguous()) t = t.contiguous();
    rccl_->broadcast(t.data_ptr(), (size_t)(t.numel() * t.element_size()), root, cur(dev_));
    return;
  }
  std::vector<at::Tensor> v{t};
  c10d::BroadcastOptions bo;
  bo.rootRank = root;
  pg_->broadcast(v, bo)->wait();
  t = v[0];
}

std::string gpu_pci_bus_id(int dev) {
  char buf[64] = {0};
  if (hipDeviceGetPCIBusId(buf, sizeof(buf), dev) != hipSuccess) return std::string();
  return std::string(buf);
}

std::shared_ptr<Comm> Comm::split(int color) const {
  if (size_ == 1) return std::make_shared<Comm>(dev_);
  static std::atomic<int> nsplit{0};
  const int id = nsplit++;  // every rank splits in the same sequence
  std::vector<double> colors = allgather_f64((double)color);
  int newrank = 0, newsize = 0;
  std::vector<int> members;
  for (int r = 0; r < size_; ++r)
    if (colors[r] == (double)color) {
      if (r == rank_) newrank = newsize;
      members.push_back(members_[r]);
      ++newsize;
    }
  if (newsize == 1) return std::make_shared<Comm>(dev_);
  if (!store_) throw std::runtime_error("mrhip: Comm::split needs the rendezvous store");
  // the subgroup's host transport gets its own key space; its RCCL id goes
  // through the root store under a key naming the member list
  auto pst = c10::make_intrusive<c10d::PrefixStore>("mrh_split_" + std::to_string(id) + "_" + std::to_string(color),
                                                    store_);
  auto c = std::make_shared<Comm>(dev_);
  c->rank_ = newrank;
  c->size_ = newsize;
  c->members_ = members;
  c->store_ = store_;
  c->mon_ = mon_;  // failure detection stays job-wide
  c->rccl_.reset();
  c->pg_ = make_host_pg(pst, newrank, newsize, mon_);
  c->host_pg_ = true;
  if (rccl_) c->rccl_ = shared_rccl(newrank, newsize, rccl_device(), store_, "split", members, mon_.get());
  c->max_msg_ = max_msg_;  // the parent's agreed value
  return c;
}

void Comm::shutdown() const {
  if (!store_ || size_ == 1) return;
  if (mon_ && mon_->failed()) return;  // a failed job has no orderly end
  if (mon_) mon_->retire();
  try {
    store_->add("mrh_shutdown", 1);
    if (rank_ != 0) return;
    const double t0 = wtime();
    while (store_->add("mrh_shutdown", 0) < size_ && wtime() - t0 < 60.0)
      std::this_thread::sleep_for(std::chrono::milliseconds(1));
  } catch (const std::exception&) {
    // a peer already tore the store down: nothing left to wait for
  }
}

int64_t Comm::next_task(const std::string& key) const {
  if (!store_) throw std::runtime_error("mrhip: mapstyle 2 needs a c10d store");
  check_peers();
  // scoped by the member list: concurrent worlds of one job share the root store
  std::string k = key + "@";
  for (int m : members_) k += std::to_string(m) + ",";
  return store_->add(k, 1) - 1;
}

RcclInfo Comm::rccl_info() const {
  RcclInfo i;
  i.live_comms = live_rccl_comms();
  if (!rccl_) return i;
  i.comm_count = rccl_->comm_count();
  i.cu_device = rccl_->cu_device();
  i.user_rank = rccl_->user_rank();
  i.id_key = rccl_->id_key();
  return i;
}

}  // namespace mrh
