// Spool: the three-tier store of KV pieces behind every bounded op
// (MI355X-native replacement for MR-MPI's Spool and paged KeyValue files,
// reference src/spool.cpp:76-263, src/keyvalue.cpp:359-380, and the
// partition spools of src/keymultivalue.cpp:645-789).
//
// A piece is appended to the first tier with room:
//   HBM          while the spool's share of the HBM budget lasts (kept as is:
//                a device piece is not copied at all);
//   pinned host  while the host budget (Settings::host_budget) lasts — DMA-able
//                memory the next pass streams back at the PCIe rate;
//   disk         a file under fpath named like the reference's out-of-core
//                files (mrmpi.<kind>.<instance>.<counter>.<rank>,
//                src/mapreduce.cpp:3187-3205), memory-mapped read-only: its
//                columns are ordinary host tensors to every engine op (chunks
//                of them stream to HBM through the page cache), and the file
//                is deleted when the last tensor viewing it is freed.
// Budgets are shared by every spool of one op (SpoolBudget), so M partition
// spools together never exceed the op's host budget.
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <future>
#include <memory>
#include <utility>
#include <string>
#include <vector>

#include "kv.h"

namespace mrh {

// bytes the tiers may still take; < 0 = unlimited
struct SpoolBudget {
  int64_t hbm = -1;
  int64_t host = -1;
};

struct SpoolConfig {
  std::shared_ptr<SpoolBudget> budget = std::make_shared<SpoolBudget>();
  std::string dir = ".";
  std::string kind = "spool";  // file name: mrmpi.<kind>.<instance>.<counter>.<rank>
  int instance = 0, rank = 0;
  // host-emitted pairs (KeyValue::add) are flushed into the spool every
  // piece_bytes, so a map never holds more than one piece of them
  int64_t piece_bytes = int64_t(64) << 20;
};

struct SpoolStats {
  int64_t pieces = 0, hbm_bytes = 0, host_bytes = 0, disk_bytes = 0, files = 0;
  void add(const SpoolStats& o) {
    pieces += o.pieces;
    hbm_bytes += o.hbm_bytes;
    host_bytes += o.host_bytes;
    disk_bytes += o.disk_bytes;
    files += o.files;
  }
};

// process-wide totals (tests, cummulative_stats): files created / live on disk
// (a snapshot: background writers update them under a lock)
SpoolStats spool_totals();
int64_t spool_files_live();

// the process's disk-tier writer pool (spool.cpp DiskWriter): drained pinned
// bytes waiting for their file write (bounded by MRH_SPOOL_WRITE_INFLIGHT),
// the hi-water of that, threads started (at most MRH_SPOOL_WRITERS), jobs done
struct WriterStats {
  int64_t inflight_bytes = 0, peak_inflight_bytes = 0, cap_bytes = 0, jobs = 0;
  int threads = 0;
};
WriterStats spool_writer_stats();
void spool_writer_reset_peak();

// a device->host drain's completion event, shared by every spool holding a
// piece of the drained buffer (destroyed with the last holder)
struct DrainEvent {
  hipEvent_t e = nullptr;
  ~DrainEvent() {
    if (e) (void)hipEventDestroy(e);
  }
};
// the device KV `dev_kv` copied into one pinned host KV on stream `copy`,
// ordered after the work queued so far on the current stream; the returned
// event completes with the copy
std::shared_ptr<DrainEvent> drain_to_pinned(const KV& dev_kv, hipStream_t copy, KV* host_out);
// building blocks of asynchronous drains: `copy` waits for the work queued so
// far on the current stream; `t` (device) copied into new pinned memory on
// `copy` (the source kept alive until the copy ran); an event recorded on `s`
void fence_after_current(hipStream_t copy);
at::Tensor drain_tensor(const at::Tensor& t, hipStream_t copy);
std::shared_ptr<DrainEvent> record_event(hipStream_t s);

class Spool {
 public:
  Spool(at::Device dev, SpoolConfig cfg);
  ~Spool();
  Spool(const Spool&) = delete;
  Spool& operator=(const Spool&) = delete;
  Spool(Spool&&) = default;

  // append one piece (device or host tensors) to the first tier with room.
  // With `copy` set, a device piece bound for the host tier drains on that
  // stream (ordered after the work queued so far on the current stream) while
  // the caller goes on, and one bound for disk drains the same way into
  // pinned memory that a background thread writes to its file; every read of
  // the spool waits for the drains and writes first.
  void add(const KV& piece, hipStream_t copy = nullptr);
  // a piece of a host buffer still being drained (drain_to_pinned): host
  // tier, counted against the host budget, readable once `ev` completes
  void add_drained(const KV& host_piece, const std::shared_ptr<DrainEvent>& ev);
  // the same piece for the disk tier: a background thread waits for `ev`,
  // then writes and maps the file (no host budget taken)
  void add_drained_to_disk(const KV& host_piece, const std::shared_ptr<DrainEvent>& ev);
  // host budget bytes left to the spools sharing this one's budget (< 0: unlimited)
  int64_t host_room() const { return cfg_.budget->host; }
  // wait for the asynchronous drains
  void sync();
  int64_t n() const { return n_; }
  int64_t bytes() const { return bytes_; }
  bool empty() const { return pieces_.empty(); }
  const std::vector<KV>& pieces() {
    sync();
    return pieces_;
  }
  // every piece as one KV: in HBM if the total fits the HBM tier, else in
  // pinned host memory if it fits the host tier, else one memory-mapped file.
  // The spool is empty afterwards (its budget shares are returned).
  KV gather();
  // every piece as one HOST KV (pinned if it fits the host tier, else a file)
  KV gather_host();
  // every piece as it is (HBM / pinned host / file), in order, nothing
  // concatenated; the spool is empty afterwards (budget shares returned)
  std::vector<KV> take();
  void clear();
  const SpoolStats& stats() const { return st_; }

 private:
  std::string next_path() const;
  void release(const KV& piece, int tier);

  at::Device dev_;
  SpoolConfig cfg_;
  std::vector<KV> pieces_;
  std::vector<int> tier_;  // 0 HBM, 1 pinned host, 2 disk
  std::vector<std::shared_ptr<DrainEvent>> pending_;
  // disk-tier pieces being written by a background thread (index into
  // pieces_, the file-backed KV): the device piece drained into pinned
  // memory on the copy stream, then written and mapped off the caller's path
  std::vector<std::pair<size_t, std::future<KV>>> writing_;
  int64_t n_ = 0, bytes_ = 0;
  SpoolStats st_;
};

// host KV / KMV written to ONE file at `path` and memory-mapped back
// (read-only, pageable); the file is removed with the last view
KV kv_to_file(const std::vector<KV>& parts, const std::string& path);
KMV kmv_to_file(const std::vector<KMV>& parts, const std::string& path);
// next disk-tier path in `dir` with the reference's naming
std::string spool_path(const std::string& dir, const std::string& kind, int instance, int rank);

}  // namespace mrh
