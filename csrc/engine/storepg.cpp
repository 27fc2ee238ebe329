// StoreBackend: see storepg.h.
#include "storepg.h"

#include <ATen/ATen.h>

#include <chrono>
#include <thread>

#include "guard.h"
#include "rccl.h"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>

namespace mrh {

namespace {

class DoneWork : public c10d::Work {
 public:
  DoneWork() { finish(); }
};

c10::intrusive_ptr<c10d::Work> done() { return c10::make_intrusive<DoneWork>(); }

std::vector<uint8_t> bytes_of(const at::Tensor& t) {
  if (t.device().type() != at::kCPU) throw std::runtime_error("mrh_store backend: host tensors only");
  at::Tensor c = t.contiguous();
  const size_t n = (size_t)c.numel() * c.element_size();
  std::vector<uint8_t> b(n);
  if (n) std::memcpy(b.data(), c.data_ptr(), n);
  return b;
}

void copy_into(at::Tensor& dst, const uint8_t* src, size_t nbytes) {
  if (dst.is_contiguous()) {
    if (nbytes) std::memcpy(dst.data_ptr(), src, nbytes);
    return;
  }
  at::Tensor tmp = at::empty(dst.sizes(), dst.options());
  if (nbytes) std::memcpy(tmp.data_ptr(), src, nbytes);
  dst.copy_(tmp);
}

}  // namespace

StoreBackend::StoreBackend(c10::intrusive_ptr<c10d::Store> store, int rank, int size, std::shared_ptr<Monitor> mon)
    : c10d::Backend(rank, size), store_(std::move(store)), mon_(std::move(mon)) {}

// blocking read of a peer's blob; with a monitor it polls (check + backoff up
// to 5 ms) so a peer that died before publishing fails the read in seconds
std::vector<uint8_t> StoreBackend::get(const std::string& k) {
  if (!mon_) return store_->get(k);  // bounded by the store's own timeout
  const auto t0 = std::chrono::steady_clock::now();
  const int limit = guard::comm_timeout_seconds();
  int sleep_us = 50;
  while (!store_->check({k})) {
    mon_->check();
    if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(limit)) {
      const std::string why = "mrh_store: no peer data for " + k + " within MRH_COMM_TIMEOUT=" +
                              std::to_string(limit) + " s";
      mon_->poison(why);
      throw PeerFailure(why);
    }
    std::this_thread::sleep_for(std::chrono::microseconds(sleep_us));
    sleep_us = std::min(sleep_us * 2, 5000);
  }
  return store_->get(k);
}

std::string StoreBackend::key(const char* op, int64_t seq, int a, int b) const {
  static const bool dbg = std::getenv("MRH_STORE_DEBUG") != nullptr;
  if (dbg) fprintf(stderr, "[mrh_store %d/%d] %s seq %lld %d %d\n", rank_, size_, op, (long long)seq, a, b);
  std::string k = std::string("mrhs/") + op + "/" + std::to_string(seq) + "/" + std::to_string(a);
  if (b >= 0) k += "/" + std::to_string(b);
  return k;
}

void StoreBackend::release(const std::string& done_key, const std::vector<std::string>& keys) {
  // the last of the size_ readers deletes the published blobs
  if (store_->add(done_key, 1) == size_) {
    for (const auto& k : keys) store_->deleteKey(k);
    store_->deleteKey(done_key);
  }
}

std::vector<std::vector<uint8_t>> StoreBackend::exchange_all(const char* op, const at::Tensor& mine) {
  const int64_t s = seq_++;
  store_->set(key(op, s, rank_), bytes_of(mine));
  std::vector<std::vector<uint8_t>> all(size_);
  std::vector<std::string> keys;
  for (int r = 0; r < size_; ++r) {
    keys.push_back(key(op, s, r));
    all[r] = get(keys.back());
  }
  release(key(op, s, -1) + "done", keys);
  return all;
}

c10::intrusive_ptr<c10d::Work> StoreBackend::allreduce(std::vector<at::Tensor>& tensors,
                                                       const c10d::AllreduceOptions& opts) {
  if (tensors.size() != 1) throw std::runtime_error("mrh_store allreduce: one tensor per call");
  at::Tensor& t = tensors[0];
  auto all = exchange_all("ar", t);
  std::vector<at::Tensor> parts;
  for (auto& b : all) {
    if ((int64_t)b.size() != t.numel() * t.element_size())
      throw std::runtime_error("mrh_store allreduce: size mismatch between ranks");
    at::Tensor p = at::empty({t.numel()}, t.options());
    copy_into(p, b.data(), b.size());
    parts.push_back(p);
  }
  at::Tensor st = at::stack(parts);
  at::Tensor r;
  switch (opts.reduceOp.op_) {
    case c10d::ReduceOp::SUM: r = st.sum(0); break;
    case c10d::ReduceOp::MAX: r = std::get<0>(st.max(0)); break;
    case c10d::ReduceOp::MIN: r = std::get<0>(st.min(0)); break;
    default: throw std::runtime_error("mrh_store allreduce: SUM/MAX/MIN only");
  }
  t.copy_(r.to(t.scalar_type()).view(t.sizes()));
  return done();
}

c10::intrusive_ptr<c10d::Work> StoreBackend::broadcast(std::vector<at::Tensor>& tensors,
                                                       const c10d::BroadcastOptions& opts) {
  if (tensors.size() != 1) throw std::runtime_error("mrh_store broadcast: one tensor per call");
  const int64_t s = seq_++;
  const std::string k = key("bc", s, (int)opts.rootRank);
  if (rank_ == opts.rootRank) store_->set(k, bytes_of(tensors[0]));
  auto b = get(k);
  if ((int64_t)b.size() != tensors[0].numel() * tensors[0].element_size())
    throw std::runtime_error("mrh_store broadcast: size mismatch between ranks");
  if (rank_ != opts.rootRank) copy_into(tensors[0], b.data(), b.size());
  release(key("bc", s, -1) + "done", {k});
  return done();
}

c10::intrusive_ptr<c10d::Work> StoreBackend::_allgather_base(at::Tensor& out, at::Tensor& in,
                                                             const c10d::AllgatherOptions&) {
  auto all = exchange_all("ag", in);
  const size_t nb = (size_t)in.numel() * in.element_size();
  std::vector<uint8_t> cat(nb * size_);
  for (int r = 0; r < size_; ++r) {
    if (all[r].size() != nb) throw std::runtime_error("mrh_store allgather: size mismatch between ranks");
    if (nb) std::memcpy(cat.data() + r * nb, all[r].data(), nb);
  }
  if ((size_t)out.numel() * out.element_size() != cat.size())
    throw std::runtime_error("mrh_store allgather: output size mismatch");
  copy_into(out, cat.data(), cat.size());
  return done();
}

c10::intrusive_ptr<c10d::Work> StoreBackend::alltoall_base(at::Tensor& out, at::Tensor& in,
                                                           std::vector<int64_t>& out_splits,
                                                           std::vector<int64_t>& in_splits,
                                                           const c10d::AllToAllOptions&) {
  const int64_t s = seq_++;
  at::Tensor src = in.contiguous();
  const int64_t row = in.dim() ? (in.size(0) ? src.numel() / in.size(0) : 0) * in.element_size() : in.element_size();
  auto split = [&](std::vector<int64_t>& sp, int64_t rows) {
    if (sp.empty()) sp.assign(size_, rows / size_);
    if ((int)sp.size() != size_) throw std::runtime_error("mrh_store alltoall: splits must have one entry per rank");
  };
  split(in_splits, in.dim() ? in.size(0) : 0);
  split(out_splits, out.dim() ? out.size(0) : 0);
  const int64_t orow = out.dim() ? (out.size(0) ? out.numel() / out.size(0) : 0) * out.element_size()
                                 : out.element_size();
  const uint8_t* sp = (const uint8_t*)src.data_ptr();
  int64_t off = 0;
  for (int p = 0; p < size_; ++p) {
    const int64_t nb = in_splits[p] * row;
    store_->set(key("a2a", s, rank_, p), std::vector<uint8_t>(sp + off, sp + off + nb));
    off += nb;
  }
  std::vector<uint8_t> recv;
  for (int p = 0; p < size_; ++p) {
    const std::string k = key("a2a", s, p, rank_);
    auto b = get(k);
    if ((int64_t)b.size() != out_splits[p] * orow)
      throw std::runtime_error("mrh_store alltoall: received size does not match the output split");
    recv.insert(recv.end(), b.begin(), b.end());
    store_->deleteKey(k);  // each blob has exactly one reader
  }
  if ((size_t)out.numel() * out.element_size() != recv.size())
    throw std::runtime_error("mrh_store alltoall: output size mismatch");
  copy_into(out, recv.data(), recv.size());
  return done();
}

c10::intrusive_ptr<c10d::Work> StoreBackend::barrier(const c10d::BarrierOptions&) {
  exchange_all("bar", at::zeros({1}, at::kByte));
  return done();
}

}  // namespace mrh
