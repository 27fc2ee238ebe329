// Host-side view of the job's communicator for the native MapReduce object:
// rank/size, the engine device, the c10d ProcessGroup used by the shuffle
// (backend "nccl" = RCCL over xGMI for device tensors, "gloo" for host
// tensors), and the scalar collectives every MR op needs (the Allreduce SUM of
// pair counts that is each op's return value, stats MAX/MIN, barriers, file
// list broadcast). Replaces MR-MPI's direct MPI_Comm use and mpistubs/
// (world size 1 = no process group, identity collectives).
#pragma once
#include <torch/csrc/distributed/c10d/ProcessGroup.hpp>
#include <torch/csrc/distributed/c10d/Store.hpp>

#include <memory>
#include <string>
#include <vector>

namespace mrh {

using PG = c10::intrusive_ptr<c10d::ProcessGroup>;

class Comm {
 public:
  enum Op { SUM = 0, MAX = 1, MIN = 2 };

  // world size 1 on `dev`
  explicit Comm(at::Device dev = at::Device(at::kCPU));
  // an existing process group (e.g. created by torch.distributed)
  Comm(PG pg, at::Device dev, c10::intrusive_ptr<c10d::Store> store = {});

  // Bootstrap from torchrun-style env (RANK, WORLD_SIZE, LOCAL_RANK,
  // MASTER_ADDR, MASTER_PORT) without Python: binds the process to GPU
  // LOCAL_RANK when GPUs are visible, and for WORLD_SIZE > 1 creates a
  // TCPStore rendezvous and an RCCL process group (device engine) or the
  // store transport of storepg.h (host engine, e.g. CPU-only CI).
  static std::shared_ptr<Comm> from_env();
  // process group over `store`: RCCL for a cuda device, StoreBackend for cpu
  static PG make_pg(const c10::intrusive_ptr<c10d::Store>& store, int rank, int size, at::Device dev);

  int rank() const { return rank_; }
  int size() const { return size_; }
  at::Device device() const { return dev_; }
  const PG& pg() const { return pg_; }  // null when size == 1
  const c10::intrusive_ptr<c10d::Store>& store() const { return store_; }
  void set_store(c10::intrusive_ptr<c10d::Store> s) { store_ = std::move(s); }

  std::vector<int64_t> allreduce(std::vector<int64_t> v, Op op) const;
  int64_t allreduce(int64_t v, Op op) const { return allreduce(std::vector<int64_t>{v}, op)[0]; }
  std::vector<double> allreduce_f64(std::vector<double> v, Op op) const;
  double allreduce_f64(double v, Op op) const { return allreduce_f64(std::vector<double>{v}, op)[0]; }
  // every rank's value, in rank order
  std::vector<double> allgather_f64(double v) const;
  std::string bcast(const std::string& s, int root) const;
  void barrier() const;
  static double wtime();

  // MPI_Comm_split analog: a new communicator over the ranks with the same
  // color, ordered by rank (RCCL for device engines, the store transport for host ones);
  // every rank of this communicator must call it
  std::shared_ptr<Comm> split(int color) const;

  // end-of-job handshake: every rank checks in; rank 0, which serves the
  // rendezvous store, returns only when all ranks have (or after 60 s), so no
  // rank's last store operation races the server's exit
  void shutdown() const;

  // mapstyle 2 work queue: next global task index from a store counter
  int64_t next_task(const std::string& key) const;

  // device-data collectives on the engine device (RCCL over xGMI for cuda)
  // per-peer element counts -> counts received from every peer
  std::vector<int64_t> alltoall_counts(const std::vector<int64_t>& send) const;
  // variable all-to-all along dim 0 (splits in rows); identity when size == 1
  at::Tensor alltoallv(const at::Tensor& in, const std::vector<int64_t>& send, const std::vector<int64_t>& recv) const;
  // every rank's 1-D tensor concatenated in rank order
  at::Tensor allgather_var(const at::Tensor& in) const;
  // in-place sum/max/min allreduce of a device tensor
  void allreduce_tensor(at::Tensor& t, Op op) const;

 private:
  int rank_ = 0, size_ = 1;
  at::Device dev_;
  PG pg_;
  c10::intrusive_ptr<c10d::Store> store_;
};

using CommPtr = std::shared_ptr<Comm>;

// PCI bus id ("0000:05:00.0") of visible GPU `dev`, "" if unavailable
std::string gpu_pci_bus_id(int dev);

}  // namespace mrh
