// Native communicator (see comm.h). Scalar collectives run on the engine
// device: tiny RCCL all-reduces for the GPU engine (the same stream-ordered
// path as the shuffle), gloo for the CPU engine.
#define USE_C10D_NCCL 1
#include "comm.h"
#include "guard.h"
#include "storepg.h"

#include <ATen/hip/HIPContext.h>
#include <hip/hip_runtime.h>
#include <torch/csrc/distributed/c10d/PrefixStore.hpp>
#include <torch/csrc/distributed/c10d/ProcessGroupNCCL.hpp>
#include <torch/csrc/distributed/c10d/TCPStore.hpp>
#include <torch/csrc/distributed/c10d/Types.hpp>

#include <atomic>
#include <chrono>
#include <cstdlib>
#include <stdexcept>
#include <thread>

namespace mrh {

namespace {
int env_int(const char* k, int d) {
  const char* v = std::getenv(k);
  return v && *v ? std::atoi(v) : d;
}
c10d::ReduceOp::RedOpType red(Comm::Op op) {
  return op == Comm::SUM ? c10d::ReduceOp::SUM : op == Comm::MAX ? c10d::ReduceOp::MAX : c10d::ReduceOp::MIN;
}
void allreduce_t(const PG& pg, at::Tensor& t, Comm::Op op) {
  std::vector<at::Tensor> v{t};
  c10d::AllreduceOptions o;
  o.reduceOp = c10d::ReduceOp(red(op));
  pg->allreduce(v, o)->wait();
  t = v[0];
}
}  // namespace

Comm::Comm(at::Device dev) : dev_(dev) {}

Comm::Comm(PG pg, at::Device dev, c10::intrusive_ptr<c10d::Store> store)
    : dev_(dev), pg_(std::move(pg)), store_(std::move(store)) {
  if (pg_) {
    rank_ = pg_->getRank();
    size_ = pg_->getSize();
    if (size_ == 1) pg_.reset();
  }
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
  return std::make_shared<Comm>(make_pg(store, rank, ws, dev), dev, store);
}

// RCCL for the device engine; the store transport (storepg.h) for host engines
PG Comm::make_pg(const c10::intrusive_ptr<c10d::Store>& store, int rank, int size, at::Device dev) {
  auto pg = c10::make_intrusive<c10d::ProcessGroup>(store, rank, size);
  if (dev.is_cuda()) {
    auto opts = c10d::ProcessGroupNCCL::Options::create();
    opts->timeout = std::chrono::milliseconds(1000LL * guard::comm_timeout_seconds());  // watchdog bound
    auto be = c10::make_intrusive<c10d::ProcessGroupNCCL>(store, rank, size, opts);
    pg->setBackend(c10::DeviceType::CUDA, c10d::ProcessGroup::BackendType::NCCL, be);
    pg->setDefaultBackend(c10d::ProcessGroup::BackendType::NCCL);
  } else {
    auto be = c10::make_intrusive<StoreBackend>(store, rank, size);
    pg->setBackend(c10::DeviceType::CPU, c10d::ProcessGroup::BackendType::CUSTOM, be);
    pg->setDefaultBackend(c10d::ProcessGroup::BackendType::CUSTOM);
  }
  return pg;
}

std::vector<int64_t> Comm::allreduce(std::vector<int64_t> v, Op op) const {
  if (!pg_ || v.empty()) return v;
  at::Tensor t = at::tensor(v, at::TensorOptions().dtype(at::kLong)).to(dev_);
  allreduce_t(pg_, t, op);
  t = t.to(at::kCPU);
  std::memcpy(v.data(), t.data_ptr<int64_t>(), v.size() * sizeof(int64_t));
  return v;
}

std::vector<double> Comm::allreduce_f64(std::vector<double> v, Op op) const {
  if (!pg_ || v.empty()) return v;
  at::Tensor t = at::tensor(v, at::TensorOptions().dtype(at::kDouble)).to(dev_);
  allreduce_t(pg_, t, op);
  t = t.to(at::kCPU);
  std::memcpy(v.data(), t.data_ptr<double>(), v.size() * sizeof(double));
  return v;
}

std::vector<double> Comm::allgather_f64(double x) const {
  std::vector<double> v(size_, 0.0);
  v[rank_] = x;
  return allreduce_f64(v, SUM);
}

std::string Comm::bcast(const std::string& s, int root) const {
  if (!pg_) return s;
  int64_t n = rank_ == root ? (int64_t)s.size() : 0;
  n = allreduce(n, SUM);
  at::Tensor t = at::zeros({std::max<int64_t>(n, 1)}, at::TensorOptions().dtype(at::kByte));
  if (rank_ == root && n) std::memcpy(t.data_ptr(), s.data(), n);
  t = t.to(dev_);
  std::vector<at::Tensor> v{t};
  c10d::BroadcastOptions bo;
  bo.rootRank = root;
  pg_->broadcast(v, bo)->wait();
  t = v[0].to(at::kCPU);
  return std::string((const char*)t.data_ptr(), (size_t)n);
}

void Comm::barrier() const {
  if (!pg_) return;
  allreduce((int64_t)0, SUM);
}

double Comm::wtime() {
  using namespace std::chrono;
  return duration<double>(steady_clock::now().time_since_epoch()).count();
}

std::vector<int64_t> Comm::alltoall_counts(const std::vector<int64_t>& send) const {
  if (!pg_) return send;
  at::Tensor s = at::tensor(send, at::TensorOptions().dtype(at::kLong)).to(dev_);
  at::Tensor r = at::empty_like(s);
  std::vector<int64_t> eq(size_, 1);
  pg_->alltoall_base(r, s, eq, eq)->wait();
  r = r.to(at::kCPU);
  return std::vector<int64_t>(r.data_ptr<int64_t>(), r.data_ptr<int64_t>() + size_);
}

at::Tensor Comm::alltoallv(const at::Tensor& in, const std::vector<int64_t>& send,
                           const std::vector<int64_t>& recv) const {
  if (!pg_) return in;
  int64_t tot = 0;
  for (auto x : recv) tot += x;
  std::vector<int64_t> shape = in.sizes().vec();
  shape[0] = tot;
  at::Tensor out = at::empty(shape, in.options());
  at::Tensor src = in.contiguous();
  std::vector<int64_t> s = send, r = recv;
  pg_->alltoall_base(out, src, r, s)->wait();
  return out;
}

at::Tensor Comm::allgather_var(const at::Tensor& in) const {
  if (!pg_) return in;
  std::vector<double> sizes = allgather_f64((double)in.numel());
  int64_t mx = 0, tot = 0;
  for (double s : sizes) {
    mx = std::max<int64_t>(mx, (int64_t)s);
    tot += (int64_t)s;
  }
  at::Tensor buf = at::zeros({std::max<int64_t>(mx, 1)}, in.options());
  if (in.numel()) buf.narrow(0, 0, in.numel()).copy_(in.reshape({-1}));
  at::Tensor all = at::empty({buf.numel() * size_}, in.options());
  pg_->_allgather_base(all, buf)->wait();
  std::vector<at::Tensor> parts;
  for (int r = 0; r < size_; ++r) parts.push_back(all.narrow(0, r * buf.numel(), (int64_t)sizes[r]));
  return at::cat(parts);
}

void Comm::allreduce_tensor(at::Tensor& t, Op op) const {
  if (!pg_) return;
  allreduce_t(pg_, t, op);
}

std::string gpu_pci_bus_id(int dev) {
  char buf[64] = {0};
  if (hipDeviceGetPCIBusId(buf, sizeof(buf), dev) != hipSuccess) return std::string();
  return std::string(buf);
}

std::shared_ptr<Comm> Comm::split(int color) const {
  if (size_ == 1) return std::make_shared<Comm>(*this);
  static std::atomic<int> nsplit{0};
  const int id = nsplit++;  // every rank splits in the same sequence
  std::vector<double> colors = allgather_f64((double)color);
  int newrank = 0, newsize = 0;
  for (int r = 0; r < size_; ++r)
    if (colors[r] == (double)color) {
      if (r == rank_) newrank = newsize;
      ++newsize;
    }
  if (newsize == 1) return std::make_shared<Comm>(dev_);
  if (!store_) throw std::runtime_error("mrhip: Comm::split needs the rendezvous store");
  auto pst = c10::make_intrusive<c10d::PrefixStore>("mrh_split_" + std::to_string(id) + "_" + std::to_string(color),
                                                    store_);
  return std::make_shared<Comm>(make_pg(pst, newrank, newsize, dev_), dev_, pst);
}

void Comm::shutdown() const {
  if (!store_ || size_ == 1) return;
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
  return store_->add(key, 1) - 1;
}

}  // namespace mrh
