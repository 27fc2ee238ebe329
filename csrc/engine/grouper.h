// GroupIndex: incremental, exact group-by of a KV while it is being built.
//
// MR-MPI groups a KV only when convert() runs (reference src/mapreduce.cpp:861-886,
// src/keymultivalue.cpp:645-789): every pair is hashed, bucketed and
// compared after the whole map has finished. On MI355X the map of a
// streaming job (InvertedIndex: part files arriving over PCIe) leaves the GPU
// idle between parts, so a KeyValue builder with grouping enabled does the
// group-by part by part in that shadow (csrc/kernels/group.hip):
//   add(part)  append the part to device arenas (no final concat), hash its
//              keys (lookup3 hashlittle2), claim / find each hash in an HBM
//              hash table, check every key's bytes against its group's first
//              key (exact);
//   finish()   the KMV in convert()'s order — unique keys by 64-bit hash
//              (fixed keys of <= 8 bytes: by raw value), values in append
//              order — from two short sorts (the groups by key order, the
//              pairs by group rank), no full-KV sort and no key
//              verification pass left for after the map.
// A 64-bit hash collision between different keys is detected by the byte
// check; finish() then reports failure and the caller runs the ordinary
// convert (exact regrouping) on kv().
#pragma once
#include <memory>

#include "kv.h"

namespace mrh {

// HashDict: the device hash dictionary of the distinct keys of a key column
// (csrc/kernels/group.hip k_dict_insert): one streaming pass over the pairs
// assigns every pair its group and checks every key's bytes against its
// group's first key (pairs per group: LDS histograms over the group ids). The table
// never takes more than half its slots; rows that found it full are left
// unassigned and counted, grow() rehashes into a larger table and a retry
// insert groups them (CUDA devices only).
class HashDict {
 public:
  HashDict(at::Device dev, int64_t cap);
  // rows [row0, row0 + n) of the key column (kd, koff | kw); h: optional
  // precomputed hash64 per row of the range; gid: int32 group per row
  // (-1: left unassigned by a full table)
  void insert(const at::Tensor& kd, const at::Tensor& koff, int kw, const at::Tensor& h, int64_t n, int64_t row0,
              int32_t* gid, bool retry);
  struct Status {
    int64_t groups = 0, collisions = 0, left = 0;
  };
  Status status() const;  // one host sync
  // rehash into a table of >= 2 * min_groups slots (group ids are kept); the
  // table takes new groups again
  void grow(int64_t min_groups);
  // group the rows [0, n) a full table left unassigned (gid -1)
  void retry(const at::Tensor& kd, const at::Tensor& koff, int kw, const at::Tensor& h, int64_t n, int32_t* gid);
  int64_t cap() const { return cap_; }
  const at::Tensor& rep() const { return rep_; }
  const at::Tensor& ghash() const { return ghash_; }
  // capacity for about `distinct` keys (power of two, >= 2x, >= 4096)
  static int64_t cap_for(int64_t distinct);
  // distinct hashes among a strided sample of up to `m` rows (a host sync)
  static int64_t sample_distinct(const KV& kv, int64_t m);

 private:
  void alloc(int64_t cap, int64_t keep_groups);
  at::Device dev_;
  int64_t cap_ = 0;
  at::Tensor slots_;  // k::DictSlot records
  at::Tensor rep_, ghash_, ctr_;
};

// convert() of a KV with few distinct keys per pair (words of a text, a hot
// key) on the hash dictionary: no full-KV sort. Keys come out in convert()'s
// order (by 64-bit hash), values in input order; with zero-width values the
// segments are the prefix sums of the group counts, no pair is moved.
// false (and nothing done) when the KV is not on the device, too small, has
// mostly distinct keys in a sample, or a 64-bit hash collision was found —
// the caller then runs the sort path (exact regrouping).
bool convert_dict(const KV& kv, KMV* out, ConvertStats* st, const at::Tensor& prehash);

class GroupIndex {
 public:
  explicit GroupIndex(at::Device dev);
  // can `part` be appended (same fixed widths / variable-ness as the parts so far)?
  bool accepts(const KV& part) const;
  void add(const KV& part);
  // capacity hint before (or between) adds: rows, key bytes and value bytes
  // the whole index will hold, so the arenas, the per-row arrays and the hash
  // table are sized once (no x1.5 regrow copies, no rehash) — the producer
  // knows its input size (InvertedIndex: part-file bytes). groups: distinct
  // keys to size the table for (< 0: rows, every key distinct at worst; 0:
  // from a sample of the first part; a full table grows at finish())
  void reserve(int64_t rows, int64_t key_bytes, int64_t value_bytes, int64_t groups = -1);
  int64_t size() const { return n_; }
  // the appended KV (views of the arenas)
  KV kv() const;
  // is `kv` still the KV this index describes (same tensors, no op in between)?
  bool describes(const KV& kv) const;
  // the grouped KMV; false if a hash collision needs the exact sort path
  bool finish(KMV* out, ConvertStats* st);
  // hash bits kept; 64 = all. MRH_GROUP_HASH_BITS=<b> narrows it so that
  // tests can force collisions through the exact fallback
  int hash_bits = 64;

 private:
  void reserve_rows(int64_t rows);
  void reserve_table(int64_t groups);
  void append_col(const at::Tensor& pd, const at::Tensor& poff, int w, int64_t n, at::Tensor* ad, at::Tensor* aoff,
                  int64_t* bytes);

  at::Device dev_;
  int kw_ = -2, vw_ = -2;  // -2: no part yet
  int64_t n_ = 0, rows_cap_ = 0;
  int64_t kbytes_ = 0, vbytes_ = 0;  // host upper bounds of the arena bytes in use
  at::Tensor kd_, koff_, vd_, voff_;  // arenas
  at::Tensor gid_;                    // int32 group id per row
  std::unique_ptr<HashDict> dict_;    // CUDA: the table (groups, counts)
  int64_t table_hint_ = 0;            // reserve(): groups to size the table for
  // CPU twin of the table
  at::Tensor rep_, ghash_;            // per group (capacity rows_cap_)
  at::Tensor slots_, sgid_;           // hash table
  at::Tensor ctr_;                    // int64 [ngroups, collisions]
  int64_t cap_ = 0;
  mutable KV view_;
};

}  // namespace mrh
