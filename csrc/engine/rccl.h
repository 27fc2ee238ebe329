// Native RCCL transport and peer-failure monitor for the device engine.
//
// The reference moves every byte through MPI (src/irregular.cpp:269-363,
// src/mapreduce.cpp:569-623, 893-1036) and handles failure by MPI_Abort from
// the failing rank (src/error.cpp:47-57). On MI355X the data plane is RCCL
// over xGMI, driven directly (not through c10d), because the shuffle needs
// what c10d's all-to-all cannot give:
//
//  * grouped point-to-point rounds (ncclGroupStart / ncclSend / ncclRecv /
//    ncclGroupEnd) whose per-peer send and receive buffers are arbitrary device
//    pointers: a chunk of a bucket is sent from where it lies and received
//    straight into its final place in the output KV, so a chunked exchange
//    needs no per-round pack or unpack copies;
//  * a dedicated communication stream with event fences, so a round can be in
//    flight on the xGMI links while the compute stream works on the previous
//    one;
//  * fail-fast: every host wait on RCCL work is a polled wait that also checks
//    the communicator's async error and the peer monitor below, and calls
//    ncclCommAbort (which releases RCCL kernels spinning on a dead peer), so a
//    rank failure ends the job on every rank in seconds instead of at a
//    600 s watchdog.
//
// Bootstrap without MPI: rank 0 creates the ncclUniqueId and publishes it in
// the job's rendezvous store (the c10d TCPStore that torchrun / the native
// launcher already run); the other ranks read it and ncclCommInitRank. The
// store key names the communicator: its tag, a hash of its member list (world
// ranks) and a per-process sequence number of communicators created for that
// member set, so two communicators of one job never share a key (a second
// world communicator, MPI_Comm_split-style subgroups of different colours).
// Readers acknowledge; rank 0 deletes the key once every member has read it.
// A process keeps ONE RCCL communicator per member set and device: every
// Comm built over the same ranks shares it (shared_rccl).
//
// Monitor: each rank of a multi-rank job runs a heartbeat thread that adds 1
// to its store counter every MRH_HEARTBEAT_MS (default 250 ms). Any wait that
// polls checks all peers' counters in one multiGet: a counter that stops
// moving for MRH_PEER_TIMEOUT seconds (default 5) means that process is gone
// (crashed, killed, aborted); a counter driven negative means the peer hit a
// fatal error and poisoned the job (poison(), called when a MapReduce op
// throws on a multi-rank communicator), with the reason in a side key.
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <torch/csrc/distributed/c10d/Store.hpp>

#include <atomic>
#include <functional>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace mrh {

// a peer failed (or poisoned the job): the op that observed it cannot complete
struct PeerFailure : std::runtime_error {
  using std::runtime_error::runtime_error;
};

class Monitor {
 public:
  // root: the job's root store (never a per-split prefix store); rank/size in
  // the WORLD (every process of the job heartbeats exactly once)
  Monitor(c10::intrusive_ptr<c10d::Store> root, int rank, int size);
  ~Monitor();
  Monitor(const Monitor&) = delete;
  Monitor& operator=(const Monitor&) = delete;

  // throws PeerFailure if a peer poisoned the job or stopped heartbeating;
  // rate limited (at most one store round trip per MRH_MONITOR_MS, default 50 ms)
  void check();
  // tell every peer this rank hit a fatal error (idempotent)
  void poison(const std::string& why);
  bool failed() const { return failed_.load(); }
  // clean exit (Comm::shutdown only — never implied by teardown): peers stop
  // treating this rank's silent counter as a crash; no-op after poison()
  void retire();
  int rank() const { return rank_; }
  int size() const { return size_; }

 private:
  void beat_loop();
  std::string hb_key(int r) const { return "mrh/hb/" + std::to_string(r); }

  c10::intrusive_ptr<c10d::Store> store_;
  int rank_, size_;
  std::thread thread_;
  std::atomic<bool> stop_{false}, failed_{false}, poisoned_{false}, retired_{false};
  std::mutex mu_;
  std::vector<int64_t> last_val_;
  std::vector<double> last_change_;
  double last_check_ = 0;
  double peer_timeout_ = 5.0;
  std::string why_;
};

struct Xfer {
  int peer;
  void* ptr;
  int64_t bytes;
};

// ---- unique-id rendezvous (store only; the CPU tests drive it with fake ids)
struct IdRendezvous {
  std::string key;          // store key the id was published under
  std::vector<uint8_t> id;  // the id every member got
};
// Rank `rank` (0-based within `members`, the communicator's world ranks in
// order) obtains the id of the next communicator over `members`: rank 0 calls
// make_id() and publishes it, the others wait for it (polling `mon` for peer
// failure, bounded by MRH_COMM_TIMEOUT) and acknowledge.
IdRendezvous rendezvous_id(const c10::intrusive_ptr<c10d::Store>& store, const std::string& tag,
                           const std::vector<int>& members, int rank,
                           const std::function<std::vector<uint8_t>()>& make_id, Monitor* mon);
// rank 0, after the communicator is up: wait for every reader's
// acknowledgement, then delete the key (no stale id left for a later reader)
void rendezvous_release(const c10::intrusive_ptr<c10d::Store>& store, const IdRendezvous& r, int nmembers,
                        Monitor* mon);

class Rccl {
 public:
  // store may be null when size == 1 (the id is created locally); members =
  // the communicator's ranks in world numbering (empty = 0..size-1)
  Rccl(int rank, int size, int device, const c10::intrusive_ptr<c10d::Store>& store, const std::string& tag,
       const std::vector<int>& members = {}, Monitor* mon = nullptr);
  ~Rccl();
  Rccl(const Rccl&) = delete;
  Rccl& operator=(const Rccl&) = delete;

  int rank() const { return rank_; }
  int size() const { return size_; }
  hipStream_t stream() const { return stream_; }

  // ---- collectives enqueued on the communication stream, fenced against `s`:
  // they start after the work already queued on `s`, and work queued on `s`
  // afterwards sees their results (no host synchronisation)
  // one grouped round of point-to-point transfers (any peer, self included)
  void sendrecv(const std::vector<Xfer>& sends, const std::vector<Xfer>& recvs, hipStream_t s);
  // same, but the compute stream is NOT made to wait: returns an event that
  // completes with the round (the caller fences when it needs the data)
  hipEvent_t sendrecv_async(const std::vector<Xfer>& sends, const std::vector<Xfer>& recvs, hipStream_t s);
  void allreduce(void* buf, size_t count, ncclDataType_t dt, ncclRedOp_t op, hipStream_t s);
  void allgather(const void* send, void* recv, size_t bytes, hipStream_t s);
  void broadcast(void* buf, size_t bytes, int root, hipStream_t s);

  // what RCCL itself reports (ncclCommCount / ncclCommCuDevice / ncclCommUserRank)
  int comm_count();
  int cu_device();
  int user_rank();
  // the store key the id came through ("" for a local id)
  const std::string& id_key() const { return id_key_; }
  // bytes per point-to-point piece: rank 0's MRH_RCCL_MAX_MSG, agreed at init
  int64_t max_msg() const { return max_msg_; }

  // nccl async error (ncclSuccess / ncclInProgress when healthy)
  ncclResult_t async_error();
  // tear the communicator down (unblocks kernels waiting on a dead peer)
  void abort();
  bool aborted() const { return aborted_; }

 private:
  void fence_in(hipStream_t s);
  hipEvent_t fence_out();
  void check(ncclResult_t r, const char* what);

  int rank_, size_;
  ncclComm_t comm_ = nullptr;
  hipStream_t stream_ = nullptr;
  std::vector<hipEvent_t> ev_;  // ring of fence events
  size_t ev_next_ = 0;
  bool aborted_ = false;
  std::string id_key_;
  int64_t max_msg_ = 0;
};

// this process's MRH_RCCL_MAX_MSG (default 256 MiB; <= 0: no limit)
int64_t max_msg_env();

// Host-side calls per nccl* entry point made by this process's Rccl objects
// (enqueue count: a call captured into a HIP graph counts once, at capture).
// The forced one-rank modes and the tests read them to prove that a code path
// really went through RCCL rather than the one-rank identity.
struct RcclCounters {
  std::atomic<int64_t> all_reduce{0}, all_gather{0}, broadcast{0}, send{0}, recv{0}, group{0};
};
RcclCounters& rccl_counters();
// diagnostic (rccl.cpp): one RCCL op on a one-rank communicator, eager then
// captured into a HIP graph and replayed; "ok" or what failed
// (capture mode: 0 global, 1 thread-local, 2 relaxed)
std::string rccl_graph_probe(int device, const std::string& what, bool capture, int mode = 1);
void rccl_counters_reset();

// The process's communicator over (store, tag, members, device): an existing
// live one is shared, otherwise a new one is bootstrapped (collectively: every
// member must ask in the same order).
std::shared_ptr<Rccl> shared_rccl(int rank, int size, int device, const c10::intrusive_ptr<c10d::Store>& store,
                                  const std::string& tag, const std::vector<int>& members, Monitor* mon);
// number of live RCCL communicators this process holds (tests / bench record)
int live_rccl_comms();

}  // namespace mrh
