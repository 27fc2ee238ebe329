// Host-side view of the job's communicator for the native MapReduce object:
// rank/size, the engine device, the data-plane transport, and the scalar
// collectives every MR op needs (the Allreduce SUM of pair counts that is each
// op's return value, stats MAX/MIN, barriers, file list broadcast). Replaces
// MR-MPI's direct MPI_Comm use and mpistubs/ (world size 1 = identity
// collectives).
//
// Transports (one per communicator, chosen at construction, no per-call
// dispatch):
//  * RCCL (device engine): the native RCCL communicator of rccl.h over xGMI,
//    bootstrapped through the job's rendezvous store. Used whenever the
//    engine device is a GPU and the job has more than one rank — and at world
//    size 1 too when MRH_FORCE_RCCL=1 (the send/recv data path runs through
//    RCCL, collectives are the identity) or MRH_FORCE_RCCL=2 (every
//    collective also calls its nccl* function on the one-rank communicator),
//    so the RCCL call sites run and are tested on a single GPU;
//  * PG (host engine / rehearsal): a c10d ProcessGroup — gloo from
//    torch.distributed, or the store transport of storepg.h for the native
//    programs on CPU — moving packed host (or staged device) buffers.
//
// Every host wait on communication is polled against the peer monitor
// (rccl.h): a failed or vanished peer turns into a PeerFailure on every rank
// within seconds (SURVEY.md §5 "failure detection"; reference Error::one ->
// MPI_Abort, src/error.cpp:47-57).
#pragma once
#include <hip/hip_runtime.h>
#include <torch/csrc/distributed/c10d/ProcessGroup.hpp>
#include <torch/csrc/distributed/c10d/Store.hpp>

#include <memory>
#include <string>
#include <vector>

#include "rccl.h"

namespace mrh {

using PG = c10::intrusive_ptr<c10d::ProcessGroup>;

struct RcclInfo {
  int comm_count = -1;   // ncclCommCount
  int cu_device = -1;    // ncclCommCuDevice
  int user_rank = -1;    // ncclCommUserRank
  int live_comms = 0;    // RCCL communicators this process holds
  std::string id_key;    // store key of the unique-id rendezvous
};

class Comm {
 public:
  enum Op { SUM = 0, MAX = 1, MIN = 2 };

  // world size 1 on `dev` (an RCCL loopback communicator if MRH_FORCE_RCCL=1)
  explicit Comm(at::Device dev = at::Device(at::kCPU));
  // an existing process group (e.g. created by torch.distributed) + the job's
  // root store; transport "" = automatic (RCCL for a GPU device), "pg" = stay
  // on the group. members = the group's ranks in world numbering (empty: the
  // group is the world); world_rank/world_size = this process in the world
  // (-1: the group's), for the job-wide peer monitor
  Comm(PG pg, at::Device dev, c10::intrusive_ptr<c10d::Store> store = {}, const std::string& transport = "",
       std::vector<int> members = {}, int world_rank = -1, int world_size = -1);
  ~Comm();

  // Bootstrap from torchrun-style env (RANK, WORLD_SIZE, LOCAL_RANK,
  // MASTER_ADDR, MASTER_PORT) without Python: binds the process to GPU
  // LOCAL_RANK when GPUs are visible, and for WORLD_SIZE > 1 creates a
  // TCPStore rendezvous plus the RCCL communicator (device engine) or the store
  // transport of storepg.h (host engine, e.g. CPU-only CI).
  static std::shared_ptr<Comm> from_env();
  // host process group over `store` (storepg.h)
  static PG make_host_pg(const c10::intrusive_ptr<c10d::Store>& store, int rank, int size,
                         std::shared_ptr<Monitor> mon);

  int rank() const { return rank_; }
  int size() const { return size_; }
  at::Device device() const { return dev_; }
  // true when ops must run the distributed code path (size > 1, or the forced
  // single-rank RCCL mode)
  bool distributed() const { return size_ > 1 || rccl_ != nullptr; }
  bool uses_rccl() const { return rccl_ != nullptr; }
  // MRH_FORCE_RCCL=2 on one rank: collectives call RCCL instead of the identity
  bool loopback_collectives() const { return loop_coll_; }
  std::string transport() const;
  const PG& pg() const { return pg_; }
  const std::shared_ptr<Rccl>& rccl() const { return rccl_; }
  const std::shared_ptr<Monitor>& monitor() const { return mon_; }
  const c10::intrusive_ptr<c10d::Store>& store() const { return store_; }
  // this communicator's ranks in world numbering
  const std::vector<int>& members() const { return members_; }

  // Host scalars (counts, stats, flags, the file list) travel over the host
  // process group when the communicator has one (gloo / the store transport):
  // no H2D/D2H staging and, above all, no device synchronisation, which an
  // RCCL scalar collective would force on every op's return value. Without a
  // host group they go through RCCL.
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
  // color, ordered by rank; every rank of this communicator must call it
  std::shared_ptr<Comm> split(int color) const;

  // end-of-job handshake: every rank checks in; rank 0, which serves the
  // rendezvous store, returns only when all ranks have (or after 60 s), so no
  // rank's last store operation races the server's exit
  void shutdown() const;

  // mapstyle 2 work queue: next global task index from a store counter
  int64_t next_task(const std::string& key) const;

  // what RCCL reports about this communicator (all -1 without RCCL)
  RcclInfo rccl_info() const;

  // ---------------------------------------------------------------- data plane
  // One grouped round of point-to-point byte transfers between this rank and
  // any peers (self included): RCCL send/recv on the comm stream fenced
  // against the current stream, or packed through the process group. Buffers
  // live on the engine device. Synchronous with respect to the current stream.
  void sendrecv(const std::vector<Xfer>& sends, const std::vector<Xfer>& recvs) const;
  // bytes per point-to-point piece (rank 0's MRH_RCCL_MAX_MSG, the same on
  // every rank: the RCCL path and the process-group path both cut transfers
  // into pieces of this size)
  int64_t max_msg() const { return max_msg_; }
  // all ranks' `bytes`-byte blocks concatenated in rank order into recv
  // (device buffers of the engine device)
  void allgather_bytes(const void* send, void* recv, int64_t bytes) const;
  // per-peer element counts -> counts received from every peer
  std::vector<int64_t> alltoall_counts(const std::vector<int64_t>& send) const;
  // variable all-to-all along dim 0 (splits in rows); identity when not distributed
  at::Tensor alltoallv(const at::Tensor& in, const std::vector<int64_t>& send, const std::vector<int64_t>& recv) const;
  // every rank's 1-D tensor concatenated in rank order
  at::Tensor allgather_var(const at::Tensor& in) const;
  // in-place sum/max/min allreduce of a device tensor
  void allreduce_tensor(at::Tensor& t, Op op) const;
  void broadcast_tensor(at::Tensor& t, int root) const;

  // Block the host until the work queued so far on the current stream is
  // done, polling for peer failure and RCCL async errors (throws PeerFailure
  // after aborting the communicator; on a multi-rank communicator also after
  // MRH_COMM_TIMEOUT seconds). Every host read of data that depends on
  // communication goes through here first.
  void host_wait() const;
  // fatal error on this rank: tell every peer and abort the communicator
  void poison(const std::string& why) const;
  // throws if a peer failed (cheap, rate limited)
  void check_peers() const;

 private:
  void init_transport(const std::string& transport, const std::string& tag);
  void fail_now(const std::string& why) const;
  bool host_scalars() const { return pg_ && host_pg_ && size_ > 1; }
  // a collective is the identity: not distributed, or one rank whose
  // communicator does not loop collectives through RCCL
  bool identity_coll() const { return !distributed() || (size_ == 1 && !loop_coll_); }
  bool loop_coll_ = false;  // MRH_FORCE_RCCL=2 (one rank)
  bool host_pg_ = false;  // pg_ has a CPU backend
  int64_t max_msg_ = 0;   // point-to-point piece size, agreed at construction
  int rccl_device() const;  // the device index (the current one for "cuda")

  int rank_ = 0, size_ = 1;
  at::Device dev_;
  std::vector<int> members_{0};
  PG pg_;
  c10::intrusive_ptr<c10d::Store> store_;
  std::shared_ptr<Rccl> rccl_;
  std::shared_ptr<Monitor> mon_;
};

using CommPtr = std::shared_ptr<Comm>;

// PCI bus id ("0000:05:00.0") of visible GPU `dev`, "" if unavailable
std::string gpu_pci_bus_id(int dev);

}  // namespace mrh
