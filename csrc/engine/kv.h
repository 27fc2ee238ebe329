// Device-resident KeyValue / KeyMultiValue containers (SoA) and the engine ops
// that transform them. This is the MI355X-native replacement for MR-MPI's
// paged byte stores (reference src/keyvalue.h:23-115, src/keymultivalue.h:23-196,
// src/spool.h:21-76): instead of fixed-size pages of interleaved
// [kb|vb|key|value] records, a KV is four flat tensors in HBM:
//
//   kdata : uint8  key bytes (packed)        koff : int64 [n+1]  (variable keys)
//   vdata : uint8  value bytes (packed)      voff : int64 [n+1]  (variable values)
//
// Fixed-width keys/values (the common graph case: uint64 vertex, EDGE{u64,u64},
// int count, double weight) carry kw/vw >= 0 and no offset array.
//
// A KMV is the same thing grouped: unique keys + values concatenated in group
// order + a CSR segment array seg[nkey+1]. A key with millions of values is
// just a long segment (the reference's multi-page "extended" KMV pair).
//
// All tensors live on the engine device: "cuda" (HIP on MI355X) for the real
// engine, "cpu" for the oracle / CPU test path. Every op dispatches on the
// tensor device; the CUDA branch always runs the hand-written HIP kernels.
#pragma once
#include <ATen/ATen.h>
#include <hip/hip_runtime.h>
#include <cstdint>
#include <functional>
#include <initializer_list>
#include <string>
#include <vector>

namespace mrh {

class Comm;

struct KV {
  at::Tensor kdata, koff, vdata, voff;
  int64_t n = 0;
  int kw = 0;  // >= 0 fixed key width in bytes, -1 variable
  int vw = 0;  // >= 0 fixed value width in bytes, -1 variable

  bool kfixed() const { return kw >= 0; }
  bool vfixed() const { return vw >= 0; }
  at::Device device() const { return kdata.defined() ? kdata.device() : at::Device(at::kCPU); }
  int64_t key_bytes() const { return kfixed() ? n * kw : (n ? koff[n].item<int64_t>() : 0); }
  int64_t value_bytes() const { return vfixed() ? n * vw : (n ? voff[n].item<int64_t>() : 0); }
  int64_t nbytes() const;  // total payload bytes incl. offsets
};

struct KMV {
  KV keys;                 // unique keys (values unused: vw == 0)
  at::Tensor vdata, voff;  // values in group order
  int vw = 0;
  at::Tensor seg;          // int64 [nkey+1]
  int64_t nkey = 0, nval = 0;
  int64_t nbytes() const;
};

// ------------------------------------------------------------------ construction
KV empty_kv(at::Device dev, int kw = 0, int vw = 0);
// from host/device tensors; widths inferred (offsets undefined => fixed width = numel/n)
KV make_kv(at::Tensor kdata, c10::optional<at::Tensor> koff, at::Tensor vdata,
           c10::optional<at::Tensor> voff, int64_t n, at::Device dev);
KV kv_to(const KV& kv, at::Device dev);
// pin: a CPU result goes straight into pinned host memory
KV concat(const std::vector<KV>& parts, at::Device dev, bool pin = false);
// KMVs one after the other (keys, values, rebased segments) on dev
KMV kmv_concat(const std::vector<KMV>& parts, at::Device dev, bool pin = false);
// the parts copied host -> device straight into one device KV (no host
// concatenation; fixed widths and offsets alike)
// (hold set: pinned sources are copied by hipMemcpyAsync on the current
// stream and appended to *hold, which the caller keeps until the stream passed
// the copies)
// device scalars read on the host with one synchronisation of stream s
// (pinned staging; no ATen kernels): {device src, host dst, bytes}
struct SmallRead {
  const void* src;
  void* dst;
  size_t bytes;
};
void read_small(hipStream_t s, std::initializer_list<SmallRead> items);
// MRH_OOC_TRACE=2: host seconds concat_upload spent allocating, issuing
// pinned copies and staging pageable ones (process totals)
struct UploadTimes {
  bool on = false;
  double alloc = 0, pinned = 0, staged = 0, stage_wait = 0, stage_memcpy = 0;
  int64_t pinned_calls = 0, staged_calls = 0;
};
UploadTimes& upload_times();
// a host tensor on the device, on the current stream: pinned by one async
// copy, pageable (a memory-mapped spool file) through the pinned staging ring
// with a multi-threaded memcpy (never HIP's on-the-fly pinning of pageable memory)
// (non_blocking: a pinned source may still be read by the copy when this returns)
at::Tensor to_device(const at::Tensor& t, at::Device dev, bool non_blocking = false);
KV concat_upload(const std::vector<KV>& parts, at::Device dev, std::vector<at::Tensor>* hold = nullptr);
KV to_var_keys(const KV& kv);
KV to_var_values(const KV& kv);
// offsets of a fixed-width column: [0, w, 2w, ...]
at::Tensor fixed_offsets(int64_t n, int w, at::Device dev);

// ------------------------------------------------------------------ primitives
// exclusive scan returning n+1 entries (int64 result for int32/int64 input, uint32 for uint32)
at::Tensor exclusive_scan(const at::Tensor& x);
// uint32 flags / counts (stored as kInt) -> exclusive scan, n + 1 uint32 (kInt)
at::Tensor scan_u32(const at::Tensor& x);
// stable sort of (u64 key, u32 val); returns (keys_sorted, vals_sorted, passes).
// skip_trivial: skip digit passes that are constant over all keys (costs one
// host sync); pass false when every digit in [begin_bit, end_bit) varies
std::tuple<at::Tensor, at::Tensor, int64_t> radix_sort_pairs(const at::Tensor& keys,
                                                              const at::Tensor& vals, int begin_bit,
                                                              int end_bit, bool skip_trivial = true);
// keys-only stable sort of int64 keys on bits [begin_bit, end_bit) (bits below
// begin_bit ride along as payload)
at::Tensor radix_sort_keys(const at::Tensor& keys, int begin_bit, int end_bit, bool skip_trivial = true);
at::Tensor hash32_keys(const KV& kv, uint32_t seed);   // lookup3 hashlittle
at::Tensor hash64_keys(const KV& kv);                  // lookup3 hashlittle2
// rows gathered by u32 permutation
KV gather(const KV& kv, const at::Tensor& perm);
at::Tensor gather_rows(const at::Tensor& data, const at::Tensor& off, int w, const at::Tensor& perm,
                       at::Tensor* new_off);

// ------------------------------------------------------------------ engine ops
struct ConvertStats {
  int64_t passes = 0;
  int64_t collisions = 0;
  bool exact = true;  // grouped on exact key bits (no hashing)
  // incremental group-by (grouper.h): 0 not used, 1 used, 2 a hash collision
  // sent it to the ordinary convert
  int grouped = 0;
  // hash-dictionary group-by of a whole KV (grouper.h convert_dict): 0 not
  // tried, 1 used, 2 tried and handed to the sort path (collision / too many
  // distinct keys)
  int dict = 0;
  int64_t dict_cap = 0;  // its final table capacity
};
// group-by (MR-MPI convert): KV -> KMV. Order of unique keys: sorted by key
// (fixed <= 8B keys) or by 64-bit hash (others).
// prehash (optional): hash64_keys(kv) already computed by the producer
KMV convert(const KV& kv, ConvertStats* st = nullptr, int force_hash_bits = 64, const at::Tensor& prehash = {});
// convert of a KV given as parts (in order), for the packed-pairs case
// (narrow fixed keys and 4- or 8-byte values); false = not applicable,
// nothing done and `parts` untouched. Otherwise `parts` is emptied: each
// part is released once packed, so a caller holding no other reference
// peaks at ~ the parts + 8 bytes a pair
bool convert_packed_parts(std::vector<KV>& parts, KMV* out, ConvertStats* st);
// one value per key (MR-MPI clone)
KMV clone(const KV& kv);
// whole KV -> one KMV pair key -> [k0,v0,k1,v1,...] (MR-MPI collapse)
KMV collapse(const KV& kv, const std::string& key);
// KMV -> KV of (key, reduced value); op in {count,sum,min,max,first,last}
KV reduce_builtin(const KMV& kmv, const std::string& op, const std::string& dtype);
// sort KV by key or value; flag as MR-MPI: 1 int,2 uint64,3 float,4 double,5 str,6 strn,
// negative = descending; extra: 7 int64, 8 uint32
KV sort_kv(const KV& kv, int flag, bool by_value);
// the unsigned 64-bit radix key sort_kv orders a column by (flag as sort_kv;
// flags 5/6: the big-endian 8-byte prefix) — the range-partition key of the
// out-of-core sort
at::Tensor column_sort_keys(const at::Tensor& data, const at::Tensor& off, int w, int64_t n, int flag);
// sort values inside each KMV segment
KMV sort_multivalues(const KMV& kmv, int flag);
// KMV -> KV with one (key, value) per value (inverse of convert)
KV expand(const KMV& kmv);

// ------------------------------------------------------------------ shuffle (shuffle.cpp)
struct ShuffleStats {
  int64_t send_bytes = 0, recv_bytes = 0, send_pairs = 0, recv_pairs = 0, rounds = 0;
  double seconds = 0;
};
struct ExchangeOpts {
  // receive cap per round in bytes (0 = one round): the exchange runs in
  // R = max_r ceil(recv_bytes_r / chunk_bytes) lock-step rounds
  int64_t chunk_bytes = 0;
  // received pairs land in pinned host memory through two HBM staging
  // buffers (out-of-core aggregate: HBM never holds the output)
  bool host_sink = false;
  // or choose the host sink by itself when this rank's received bytes exceed
  // this HBM budget (0 = unlimited)
  int64_t hbm_budget = 0;
  // 1: each round is one grouped all-to-all over every peer (RCCL group);
  // 0: the reference's custom exchange order (src/irregular.cpp:200-215,
  // 311-363): P pairwise steps per round, step j sends to me+j and receives
  // from me-j, one peer link busy at a time
  int all2all = 1;
  // pipelined consumer (collate): every round's received pairs are handed to
  // round_sink as a KV (views of a device staging buffer, valid until the
  // sink's work queued on the current stream has run; the sink must copy what
  // it keeps) while the next round is on the wire. exchange() then returns an
  // empty KV. Pairs reach the sink round by round, each round source-rank
  // major (with one round: exactly the order exchange() would return)
  std::function<void(const KV&)> round_sink;
};
// destination rank per pair: hashlittle(key, kb, P) % P (MR-MPI default)
at::Tensor partition_dest(const KV& kv, int P, at::Tensor* counts);
// all-to-all exchange of KV pairs to their destination ranks (dest: int32 per
// pair; undefined = hash partitioning fused into the partition kernel). The
// KV is consumed (its memory is released once packed).
KV exchange(KV kv, const at::Tensor& dest, const Comm& comm, const ExchangeOpts& o = {},
            ShuffleStats* st = nullptr);
// MR-MPI aggregate: hash partition + exchange
KV aggregate(KV kv, const Comm& comm, const ExchangeOpts& o = {}, ShuffleStats* st = nullptr);
// move everything to ranks 0..nprocs-1 (rank r sends to r % nprocs)
KV gather_to(KV kv, int nprocs, const Comm& comm, const ExchangeOpts& o = {}, ShuffleStats* st = nullptr);
// local stable partition of a KV into P contiguous buckets by dest (int32 in
// [0, P)): the exchange's partition kernels without the exchange (the
// out-of-core ops' spool partitioning, ooc.cpp)
struct Buckets {
  KV kv;                       // bucket-ordered pairs (bucket d is contiguous)
  std::vector<int64_t> count;  // pairs per bucket
};
Buckets bucket_local(const KV& kv, const at::Tensor& dest, int P);
// root's KV replicated on every rank
KV broadcast(const KV& kv, int root, const Comm& comm);

// ------------------------------------------------------------------ text / graph maps
// InvertedIndex map over one text buffer (padded by >= 32 bytes): KV(url+NUL, int32 doc)
KV map_urls(const at::Tensor& text, int64_t n, int32_t doc_id);
// wordfreq map: KV(word+NUL, NULL)
KV map_words(const at::Tensor& text, int64_t n);
// R-MAT: KV(EDGE{u64,u64}, NULL)
KV map_rmat(int64_t nedges, int nlevels, double a, double b, double c, double d, double fraction,
            uint64_t seed, uint64_t first_edge, at::Device dev);

// ------------------------------------------------------------------ graph iteration (graph.cpp)
void pr_contrib(const at::Tensor& seg, const at::Tensor& src, const at::Tensor& w, const at::Tensor& r,
                at::Tensor& out);
void pr_combine(const at::Tensor& seg, const at::Tensor& perm, const at::Tensor& recv, const at::Tensor& vid,
                at::Tensor& acc);
void scatter_f32(const at::Tensor& v, const at::Tensor& idx, at::Tensor& out);
at::Tensor pr_update(const at::Tensor& acc, const at::Tensor& r, at::Tensor& rn, const at::Tensor& dangling,
                     double base, double alpha, const at::Tensor& dmass, double invN, const at::Tensor& invdeg,
                     at::Tensor& cout);
void plan_gather_reduce(const at::Tensor& seg, const at::Tensor& src, const at::Tensor& x, const at::Tensor& w,
                        int64_t op, at::Tensor& out);
void plan_combine(const at::Tensor& seg, const at::Tensor& perm, const at::Tensor& recv, const at::Tensor& vid,
                  int64_t op, at::Tensor& acc);
// static-segment index for plans whose segments never change (CUDA only;
// csrc/kernels/wavesegred.h): per-iteration gather-reduce with no segment search
struct SegIndex {
  at::Tensor H, wbase, scratch;
  at::Tensor sched;  // optional XCD-pinned wave schedule (int32 [8, slen], -1 = none)
  int64_t nval = 0, slen = 0;
  bool defined() const { return H.defined(); }
};
SegIndex seg_index(const at::Tensor& seg, int64_t nval);
// the same over a head bitmap already built (k::ws_words(nval) words, e.g. by
// the unpack of a sorted plan): only the per-wave bases are computed
SegIndex seg_index(const at::Tensor& seg, int64_t nval, const at::Tensor& heads);
// out[s] = OP_{e in seg s} (x[src[e]] (+ w[e])), op 0 sum / 1 min / 2 max
void seg_gather_reduce(const SegIndex& ix, const at::Tensor& src, const at::Tensor& x, const at::Tensor& w, int64_t op,
                       at::Tensor& out);
std::pair<at::Tensor, at::Tensor> wedges(const at::Tensor& seg, const at::Tensor& nb, const at::Tensor& centre);
// the same wedges in chunks of at most max_w (<= 0: one chunk), handed to fn
// in wedge order: an emitter bounded by a page budget never holds the whole
// O(d^2) set (a hub of degree 20k alone makes 2e8 wedges, 4.8 GB)
void for_each_wedge_chunk(const at::Tensor& seg, const at::Tensor& nb, const at::Tensor& centre, int64_t max_w,
                          const std::function<void(const at::Tensor& edges, const at::Tensor& centre)>& fn);
// the same in the compact layout of large graphs: keys (min << vb | max)
// int64, centres int32 (12 bytes a wedge)
void for_each_wedge_chunk_compact(const at::Tensor& seg, const at::Tensor& nb, const at::Tensor& centre,
                                  int64_t max_w, int vb,
                                  const std::function<void(const at::Tensor& keys, const at::Tensor& centre)>& fn);
// segment id of every value of a CSR segment array (seg[nseg+1], nval values)
at::Tensor segment_ids(const at::Tensor& seg, int64_t nseg, int64_t nval);
// counts of each bin in [0, K) of an integer index column (device histogram)
at::Tensor bincount_dev(const at::Tensor& idx, int64_t K);
// positions of the true elements of a bool mask, in order (int64; the
// device path is flags + scan + scatter, not at::nonzero's rocPRIM partition)
at::Tensor mask_indices(const at::Tensor& mask);
// i repeated counts[i] times (the row index of every expanded element)
at::Tensor repeat_index(const at::Tensor& counts);
// segment boundaries of a sorted int64 key column: seg[nseg+1]
at::Tensor segments_sorted(const at::Tensor& sorted_keys);
// segment boundaries from u32 head flags (1 where a segment starts): seg[nseg+1]
at::Tensor segments_from_flags(const at::Tensor& flags);
// segment boundaries from a head bitmap over n values (int32 words, bit i of
// word i / 32 set where a segment starts; words past n zero): seg[nseg+1]
at::Tensor segments_from_bits(const at::Tensor& heads, int64_t n);

// K-means map with in-mapper combining (kmeans.cpp): KV(int32 cluster*(D+1)+j, double)
KV kmeans_map(const at::Tensor& points, const at::Tensor& centroids);

// ------------------------------------------------------------------ app epilogues
at::Tensor inverted_index_format(const KMV& kmv, const at::Tensor& names, const at::Tensor& name_off);

}  // namespace mrh
