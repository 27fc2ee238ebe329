// The native MapReduce object: MR-MPI's user API (reference src/mapreduce.h:28-126,
// src/mapreduce.cpp:93-3574) on the device-resident engine of kv.h.
//
// Same method names, settings (names, defaults, meaning), and return values
// (every data op returns the GLOBAL pair count, an Allreduce SUM). The MR owns
// one KV or one KMV (never both), as SoA tensors in HBM; all data-plane work
// (hash/partition, RCCL shuffle, group-by, sorts, segmented reduces, gathers)
// runs in the engine ops.
//
// Callbacks come in two tiers:
//  * host callbacks with the exact MR-MPI shapes (map task / file / chunk / mr,
//    reduce/compress, scan kv/kmv, hash, compare): the engine stages the data
//    to host once per op and the callback sees the reference's (key, kb, mv,
//    nvalues, valuebytes) views, including the multi-block protocol for keys
//    whose values exceed one page (nvalues == 0 + multivalue_block*());
//  * batch callbacks that receive the whole device KV/KMV and append device
//    KVs (kernels / ATen ops), which keep the data in HBM end to end.
#pragma once
#include <atomic>
#include <functional>
#include <memory>
#include <optional>
#include <string>
#include <vector>

#include "comm.h"
#include "keyvalue.h"
#include "kv.h"
#include "ooc.h"

namespace mrh {

class MapReduce;
struct OocStats;

using MapTaskFn = std::function<void(int itask, KeyValue& kv)>;
using MapFileFn = std::function<void(int itask, const char* fname, KeyValue& kv)>;
using MapChunkFn = std::function<void(int itask, char* str, int size, KeyValue& kv)>;
using MapKVFn = std::function<void(uint64_t itask, char* key, int kb, char* value, int vb, KeyValue& kv)>;
using ReduceFn = std::function<void(char* key, int kb, char* mv, int nvalues, int* valuebytes, KeyValue& kv)>;
using ScanKVFn = std::function<void(char* key, int kb, char* value, int vb)>;
using ScanKMVFn = std::function<void(char* key, int kb, char* mv, int nvalues, int* valuebytes)>;
using HashFn = std::function<int(char* key, int kb)>;
using CompareFn = std::function<int(char* a, int alen, char* b, int blen)>;
using MapBatchFn = std::function<void(const KV& src, KeyValue& kv)>;
using ReduceBatchFn = std::function<void(const KMV& src, KeyValue& kv)>;

struct Settings {
  int mapstyle = 0;    // 0 chunk, 1 stride, 2 dynamic work queue
  int all2all = 1;     // 1 grouped all-to-all rounds, 0 ring-ordered pairwise steps (shuffle.cpp)
  int verbosity = 0;   // 0 none, 1 totals, 2 per-proc histograms
  int timer = 0;       // 0 none, 1 barrier + rank-0 time, 2 per-proc histogram
  int memsize = 64;    // MB per page (negative: bytes); sets the host block size of long KMV values
  // minpage: pool pre-grown by minpage pages at the first op; maxpage: HBM
  // budget = maxpage pages (out-of-core beyond it); freepage: with a budget,
  // freed HBM returns to the driver after every op; zeropage: padding bytes of
  // aligned host-callback layouts are zeroed (reference src/mapreduce.cpp:3318-3547)
  int minpage = 0, maxpage = 0, freepage = 1, outofcore = 0, zeropage = 0;
  int keyalign = 4, valuealign = 4;
  std::string fpath = ".";
  // ---- MI355X-native settings
  // receive cap per shuffle round in bytes; 0 = the reference's 2 pages
  // (2 x memsize, src/mapreduce.cpp:418)
  int64_t chunk_bytes = 0;
  // HBM budget of this MR's data in bytes (0 = maxpage x memsize if maxpage
  // > 0, else unlimited): an aggregate whose received data would exceed it
  // lands in pinned host memory, and convert / sort_keys / sort_values /
  // builtin reduces run out of core over host spools (ooc.cpp)
  int64_t hbm_budget = 0;
  // pinned host bytes the spill tier may hold before it writes to disk (0 =
  // unlimited): map/reduce builders and the out-of-core spools put what
  // exceeds it in memory-mapped files under fpath (spool.h)
  int64_t host_budget = 0;
  // depth of the host -> HBM staging pipelines: the streaming apps
  // (InvertedIndex, wordfreq) keep streams - 1 input copies in flight on a
  // side stream while a chunk computes, and the out-of-core passes overlap
  // the next chunk's copy and the previous chunk's drain with compute
  // (streams >= 2); 1 = copy and compute one chunk at a time, on one stream;
  // 0 = each pipeline's tuned default (InvertedIndex 2, wordfreq 3, OOC 2)
  int streams = 0;
  // collate() groups each received shuffle round while the next one is on
  // the wire (1, default) or runs aggregate then convert (0); the env
  // MRH_PIPELINE_COLLATE=0 sets the default to 0
  int pipeline = -1;
};

class MapReduce {
 public:
  explicit MapReduce(CommPtr comm);
  ~MapReduce();
  MapReduce(const MapReduce&) = delete;
  MapReduce& operator=(const MapReduce&) = delete;

  Settings set;
  int mapfilecount = 0;

  // ---------------------------------------------------------------- data
  // The KV is `kv` followed by the parts appended to it and not yet
  // concatenated (add, an addflag map / close): appending is O(appended) —
  // the parts stay where they were made (HBM, pinned host, spool file). Ops
  // that stream their input (convert, collate and aggregate on one rank)
  // read the parts in place; every other op, and code reading `kv`
  // directly, flattens first (flatten(): one concatenation).
  std::optional<KV> kv;
  // The KMV likewise is `kmv` followed by parts: an out-of-core convert
  // leaves one host-resident KMV per partition (pinned, or a file) instead of
  // concatenating them on the host; the reduce family and scan walk the
  // parts, every other op (and code reading `kmv`) flattens first.
  std::optional<KMV> kmv;
  ConvertStats last_convert;
  void flatten();
  void flatten_kmv();
  // pairs of the KV including the appended parts
  int64_t kv_rows() const;
  const std::vector<KV>& kv_tail() const { return kv_tail_; }
  // keys of the KMV including its parts; its parts in order
  int64_t kmv_keys() const;
  std::vector<KMV> kmv_parts() const;
  size_t kmv_part_count() const { return kmv ? 1 + kmv_tail_.size() : 0; }

  // ---------------------------------------------------------------- object ops
  std::unique_ptr<MapReduce> copy() const;
  uint64_t add(MapReduce& other);
  uint64_t aggregate(const HashFn& hash = nullptr);
  uint64_t aggregate_dest(const at::Tensor& dest);  // explicit int32 destination per pair
  uint64_t broadcast(int root);
  uint64_t clone();
  uint64_t close();
  uint64_t collapse(const char* key, int kb);
  uint64_t collate(const HashFn& hash = nullptr);
  uint64_t compress(const ReduceFn& fn);
  uint64_t compress_builtin(const std::string& op, const std::string& dtype);
  uint64_t compress_batch(const ReduceBatchFn& fn);
  // device functors (devfn.h): user HIP device code compiled at run time
  uint64_t map_device(MapReduce& src, const std::string& code, int addflag = 0);
  uint64_t map_device_tasks(int64_t ntask, const std::string& code, int addflag = 0);
  uint64_t reduce_device(const std::string& code);
  uint64_t compress_device(const std::string& code);
  // sort by a device sort-key functor (mr_sortkey: key -> u64 in the wanted order), stable
  uint64_t sort_keys_device(const std::string& code, int bits = 64);
  uint64_t sort_values_device(const std::string& code, int bits = 64);
  uint64_t convert();
  // convert with the keys' hash64_keys() already computed by the producer
  uint64_t convert_prehashed(const at::Tensor& prehash);
  uint64_t gather(int nprocs);
  void open(int addflag = 0);
  KeyValue& kv_open();  // the builder other MRs' callbacks add into while open

  // map variants (reference :1044-1642); addflag 1 appends to the existing KV
  uint64_t map(int nmap, const MapTaskFn& fn, int addflag = 0);
  uint64_t map_file(const std::vector<std::string>& files, int selfflag, int recurse, int readflag,
                    const MapFileFn& fn, int addflag = 0);
  uint64_t map_file_char(int nmap, const std::vector<std::string>& files, int selfflag, int recurse, int readflag,
                         char sepchar, int delta, const MapChunkFn& fn, int addflag = 0);
  uint64_t map_file_str(int nmap, const std::vector<std::string>& files, int selfflag, int recurse, int readflag,
                        const std::string& sepstr, int delta, const MapChunkFn& fn, int addflag = 0);
  uint64_t map_mr(MapReduce& src, const MapKVFn& fn, int addflag = 0);
  uint64_t map_batch(int nmap, const MapTaskFn& fn, int addflag = 0) { return map(nmap, fn, addflag); }
  uint64_t map_mr_batch(MapReduce& src, const MapBatchFn& fn, int addflag = 0);

  uint64_t reduce(const ReduceFn& fn);
  uint64_t reduce_builtin(const std::string& op, const std::string& dtype);
  uint64_t reduce_batch(const ReduceBatchFn& fn);
  uint64_t scan_kv(const ScanKVFn& fn);
  uint64_t scan_kmv(const ScanKMVFn& fn);
  uint64_t scrunch(int nprocs, const char* key, int kb);

  // multi-block access to one long KMV value list from inside reduce/scan
  // callbacks (reference :1874-1925); `token` is the valuebytes pointer the
  // callback received with nvalues == 0
  uint64_t multivalue_blocks(int& nblock) const;
  void multivalue_block_select(int which) { block_select_ = which; }
  int multivalue_block(int iblock, char** mv, int** valuebytes);

  uint64_t sort_keys(int flag);
  uint64_t sort_keys(const CompareFn& fn);
  uint64_t sort_values(int flag);
  uint64_t sort_values(const CompareFn& fn);
  uint64_t sort_multivalues(int flag);
  uint64_t sort_multivalues(const CompareFn& fn);

  // print (reference :1671-1761): kflag/vflag 0 none,1 int,2 uint64,3 float,4 double,5 str,6 strn,7 raw bytes
  void print(int proc, int nstride, int kflag, int vflag);
  void print(const char* file, int fflag, int proc, int nstride, int kflag, int vflag);

  uint64_t kv_stats(int level);
  uint64_t kmv_stats(int level);
  void cummulative_stats(int level, int reset);
  void set_fpath(const std::string& p) { set.fpath = p; }

  // tiers the bounded builders of this MR's ops spooled to (spool.h), summed
  SpoolStats spool_stats;
  // out-of-core hot keys: grouped on the host (convert) / cut into value blocks (reduce)
  int64_t ooc_hot_keys = 0, ooc_split_keys = 0;

  // host spill tier: move the data to pinned host DRAM and back
  void spill();
  void unspill();
  // disk tier: write the data to fpath/mrmpi.<kv|kmv>.<instance>.<n>.<rank>
  // and free it; it is read back (and the file removed) on the next op
  void spill_disk();
  void ensure_resident();
  bool on_disk() const { return !disk_path_.empty(); }

  // checkpoint / restart of this rank's KV or KMV (binary SoA file, one per
  // rank: `path` gets ".<rank>" appended when nprocs > 1); load returns the
  // global pair count like every op
  void save(const std::string& path) const;
  uint64_t load(const std::string& path);

  const CommPtr& comm() const { return comm_; }
  int my_proc() const { return comm_->rank(); }
  int num_procs() const { return comm_->size(); }
  int instance() const { return instance_me_; }
  at::Device device() const { return comm_->device(); }

  // ---------------------------------------------------------------- static counters
  // (reference src/mapreduce.h:46-57)
  static std::atomic<int> instances_now, instances_ever;
  static std::atomic<int64_t> msize, msizemax, rsize, wsize, cssize, crsize;
  static double commtime;

  // file list expansion shared with the Python layer (reference :2812-2931)
  static std::vector<std::string> find_files(const Comm& comm, const std::vector<std::string>& files, int selfflag,
                                             int recurse, int readflag);

 private:
  void start();
  // parts_ok: the op reads the appended KV parts itself (else they are
  // flattened); kmv_parts_ok: the same for the KMV's parts
  void enter(const char* op, bool ooc_ok = false, bool parts_ok = false, bool kmv_parts_ok = false);
  void set_kmv_parts(std::vector<KMV> parts);
  void drop_kmv();
  // append `b` as a part: device parts past the HBM budget go through a
  // bounded builder (pinned host / spool files), nothing already held moves
  void append_part(const KV& b);
  // the KV and its appended parts, in order
  std::vector<KV> kv_parts() const;
  // the KV becomes `parts` (a builder's parts: no concatenation)
  void set_kv_parts(std::vector<KV> parts);
  int64_t data_bytes() const;
  void bound(KeyValue& b);
  KV concat_parts(const std::vector<KV>& parts);
 public:
  // the tiers and names an out-of-core op of this MR may use
  OocEnv ooc_env() const;
 private:
  void note_spool(const KeyValue& b);
  void note_ooc(const char* op, const OocStats& st);
  // out-of-core helpers: a shuffle past the budget, a user hash's owner ranks
  // (host), compress's group-by
  bool ooc_shuffle() const;
  at::Tensor host_dest(const HashFn& hash) const;
  KMV local_groups(const char* heading);
  void stats(const char* heading, int which);
  void need_kv(const char* what) const;
  void need_kmv(const char* what) const;
  void note_shuffle(const ShuffleStats& st);
  uint64_t count(int64_t n) const { return (uint64_t)comm_->allreduce(n, Comm::SUM); }
  std::vector<int> my_tasks(int nmap);
  uint64_t finish_map(KeyValue& kvb, int addflag, const char* heading = "Map");
  uint64_t map_chunks(int nmap, const std::vector<std::string>& files, int selfflag, int recurse, int readflag,
                      const std::string& sep, bool is_char, int delta, const MapChunkFn& fn, int addflag);
  void run_host_kmv(const KMV& kmv, const std::function<void(char*, int, char*, int, int*)>& fn);
  void histo(double v, const char* heading) const;
  int64_t block_bytes() const;
 public:
  // HBM budget of this object's data in bytes (0 = unlimited)
  int64_t budget() const;
  // memsize-sized pages a local KV/KMV of `bytes` spans (reference kv_stats
  // "N pages"; the out-of-core ops record their partition count too)
  int64_t pages(int64_t bytes) const { return std::max<int64_t>({int64_t(1), (bytes + block_bytes() - 1) / block_bytes(), pages_}); }
 private:
  // shuffle options from the settings
  ExchangeOpts xopts() const;

  void write_file(const std::string& p) const;
  int64_t read_file(const std::string& p);
  void drop_disk();
  // a map replacing the object's data (addflag 0, not reading its own KV)
  // drops the old KV/KMV up front instead of bringing them back to HBM
  void drop_for_map(int addflag, const MapReduce* src = nullptr);

  CommPtr comm_;
  std::vector<KV> kv_tail_;
  std::vector<KMV> kmv_tail_;
  std::string disk_path_;
  int disk_counter_ = 0;
  // group-by index of the KV built by the last map / close with grouping
  // enabled (keyvalue.h); convert() uses it while it still describes kv
  std::shared_ptr<GroupIndex> grouped_;
  std::unique_ptr<KeyValue> open_;
  int open_add_ = 0;
  double t0_ = 0;
  int64_t cs0_ = 0, cr0_ = 0;
  int instance_me_ = 0;
  // multi-block state of the key currently handed to a host callback
  struct Blocks {
    char* mv = nullptr;
    const int* sizes = nullptr;
    int64_t nval = 0;
    std::vector<int64_t> start;  // value index at the start of each block
    std::vector<int64_t> boff;   // byte offset of each block start relative to mv
  } blk_;
  int block_select_ = 0;
  int64_t pages_ = 0;
  bool started_ = false;
};

}  // namespace mrh
