// Host-tensor collectives over the c10d rendezvous store: the transport for
// native (C++ / C API / oink executable) multi-process runs of the CPU engine.
//
// The reference runs everything on one host through real MPI or through the
// serial mpistubs/ (mpistubs/mpi.cpp:42-395); its test
// strategy is "run the programs with mpirun -np N on one box" (SURVEY.md §4).
// The device engine's transport is RCCL over xGMI (ProcessGroupNCCL); torch's
// gloo is only reachable from Python in this image (no gloo headers), so
// native CPU processes use this backend instead: every collective is a set of
// keyed byte blobs in the TCPStore (one blob per (sender, receiver) for the
// all-to-all, one per rank for all-reduce / all-gather / broadcast), read by
// the peers and deleted by the last reader. It is a correctness transport for
// host tensors (tests, small jobs, CI without GPUs), not a data plane.
#pragma once
#include <torch/csrc/distributed/c10d/Backend.hpp>
#include <torch/csrc/distributed/c10d/Store.hpp>

#include <memory>
#include <string>

namespace mrh {

class Monitor;

class StoreBackend : public c10d::Backend {
 public:
  // mon (may be null): every blocking read polls it, so a dead or failed peer
  // ends the collective with PeerFailure instead of a store timeout
  StoreBackend(c10::intrusive_ptr<c10d::Store> store, int rank, int size, std::shared_ptr<Monitor> mon = {});

  const std::string getBackendName() const override { return "mrh_store"; }

  c10::intrusive_ptr<c10d::Work> broadcast(std::vector<at::Tensor>& tensors,
                                           const c10d::BroadcastOptions& opts) override;
  c10::intrusive_ptr<c10d::Work> allreduce(std::vector<at::Tensor>& tensors,
                                           const c10d::AllreduceOptions& opts) override;
  c10::intrusive_ptr<c10d::Work> _allgather_base(at::Tensor& out, at::Tensor& in,
                                                 const c10d::AllgatherOptions& opts) override;
  c10::intrusive_ptr<c10d::Work> alltoall_base(at::Tensor& out, at::Tensor& in, std::vector<int64_t>& out_splits,
                                               std::vector<int64_t>& in_splits,
                                               const c10d::AllToAllOptions& opts) override;
  c10::intrusive_ptr<c10d::Work> barrier(const c10d::BarrierOptions& opts) override;

 private:
  std::string key(const char* op, int64_t seq, int a, int b = -1) const;
  // publish this rank's blob, read every rank's, delete after the last reader
  std::vector<std::vector<uint8_t>> exchange_all(const char* op, const at::Tensor& mine);
  void release(const std::string& done_key, const std::vector<std::string>& keys);
  std::vector<uint8_t> get(const std::string& key);

  c10::intrusive_ptr<c10d::Store> store_;
  std::shared_ptr<Monitor> mon_;
  int64_t seq_ = 0;
};

}  // namespace mrh
