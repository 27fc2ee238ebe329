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

class GroupIndex {
 public:
  explicit GroupIndex(at::Device dev);
  // can `part` be appended (same fixed widths / variable-ness as the parts so far)?
  bool accepts(const KV& part) const;
  void add(const KV& part);
  // capacity hint before (or between) adds: rows, key bytes and value bytes
  // the whole index will hold, so the arenas, the per-row arrays and the hash
  // table are sized once (no x1.5 regrow copies, no rehash) — the producer
  // knows its input size (InvertedIndex: part-file bytes)
  void reserve(int64_t rows, int64_t key_bytes, int64_t value_bytes);
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
  at::Tensor rep_, ghash_;            // per group (capacity rows_cap_)
  at::Tensor slots_, sgid_;           // hash table
  at::Tensor ctr_;                    // int64 [ngroups, collisions]
  int64_t cap_ = 0;
  mutable KV view_;
};

}  // namespace mrh
