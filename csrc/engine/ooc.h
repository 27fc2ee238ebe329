// Out-of-core convert / sort / builtin reduce (ooc.cpp): the KV or KMV lives
// in pinned host memory and HBM holds one budget-sized piece at a time.
#pragma once
#include <functional>
#include <string>

#include "kv.h"

namespace mrh {

struct OocStats {
  int64_t parts = 0;         // partitions (convert) / range buckets (sort)
  int64_t chunks = 0;        // budget-sized pieces streamed through HBM
  int64_t bytes_staged = 0;  // bytes moved host -> HBM in the partition pass
  int64_t files = 0;         // spool / result files written under fpath (disk tier)
  int64_t disk_bytes = 0;    // bytes those files held
  int64_t hot_keys = 0;      // convert: keys over a quarter budget grouped on the host, never in HBM whole
  int64_t split_keys = 0;    // reduce: keys whose values were cut into blocks across pieces
};

// where an out-of-core op may put its data (MapReduce settings)
struct OocEnv {
  int64_t hbm = 0;    // HBM budget (bytes)
  int64_t host = -1;  // pinned host bytes before the disk tier (< 0 unlimited)
  std::string dir = ".";
  int instance = 0, rank = 0;
  int streams = 0;  // 1: no copy/compute overlap (Settings::streams)
};

// does an op whose HBM working set is `factor` x `bytes` exceed the budget?
bool needs_ooc(int64_t bytes, int64_t budget, double factor);
// results are host-resident: pinned while they fit env.host, else one
// memory-mapped file under env.dir; inputs may be on the host (pinned,
// pageable or memory-mapped) or the device
// kvs: the KV as parts in order (a KV with appended parts, mapreduce.h); each
// is read where it lies
KMV ooc_convert(const std::vector<KV>& kvs, const OocEnv& env, at::Device dev, OocStats* st = nullptr);
// the same result as one host-resident KMV per partition (pinned while the
// host budget lasts, else a file each), not concatenated: the MapReduce
// object keeps them as its KMV's parts
std::vector<KMV> ooc_convert_parts(const std::vector<KV>& kvs, const OocEnv& env, at::Device dev,
                                   OocStats* st = nullptr);
KV ooc_sort(const KV& kv, int flag, bool by_value, const OocEnv& env, at::Device dev, OocStats* st = nullptr);
KV ooc_reduce_builtin(const KMV& kmv, const std::string& op, const std::string& dtype, const OocEnv& env,
                      at::Device dev, OocStats* st = nullptr);
// every key range of a (host-resident) KMV whose values fit a quarter of the
// budget, as a device KMV, to fn in key order (the reduce-family ops)
void ooc_for_each_kmv_piece(const KMV& kmv, const OocEnv& env, at::Device dev, const std::function<void(const KMV&)>& fn,
                            OocStats* st = nullptr);
// the same, and with `split` a key whose values exceed the piece size comes as
// several one-key pieces of consecutive value blocks (the reference's
// extended KMV pair, src/keymultivalue.cpp:1219-1350): fn's flags are 0 for
// whole keys, else kBlock | kFirst on its first block | kLast on its last
constexpr int kBlock = 1, kFirst = 2, kLast = 4;
void ooc_for_each_kmv_block(const KMV& kmv, const OocEnv& env, at::Device dev,
                            const std::function<void(const KMV&, int)>& fn, bool split, OocStats* st = nullptr);
// the shuffle of a KV larger than the budget (MR-MPI's paged aggregate,
// src/mapreduce.cpp:385-563: pages in lock-step up to the global page count,
// a two-page receive window): budget/4-byte chunks go to HBM one at a time,
// every rank the same number of rounds; each chunk's exchange receives in
// budget/4-byte rounds into pinned host memory, and the received pairs
// collect in pinned host memory up to env.host, in files beyond it.
// dest_host: one int32 destination per pair (undefined: hash partitioning)
KV ooc_exchange(const KV& kv, const at::Tensor& dest_host, const Comm& comm, const OocEnv& env, at::Device dev,
                int all2all = 1, OocStats* st = nullptr, ShuffleStats* sst = nullptr);

}  // namespace mrh
