// Append-only KeyValue builder handed to map/reduce callbacks: the MR-MPI
// KeyValue::add API (reference src/keyvalue.h:55-57, src/keyvalue.cpp:343-643)
// over the device-resident SoA KV of kv.h.
//
// Host-emitted pairs accumulate in contiguous byte arrays (one memcpy per
// pair, no per-pair page/alignment bookkeeping); device batches (KV objects
// produced by kernels or ATen ops inside batch callbacks) are kept as chunks in
// emission order, so a callback can mix both without a host round trip for
// device data. finish() uploads the host part once and concatenates.
//
// set_spool() (a MapReduce object with an HBM or host budget): the builder is
// bounded — host-emitted pairs are flushed every SpoolConfig::piece_bytes and
// every chunk goes to a Spool (spool.h: HBM while the budget lasts, then
// pinned host, then memory-mapped files under fpath), and finish() returns
// the KV on the tier it fits (the reference pages a KeyValue to disk while
// the map is still emitting, src/keyvalue.cpp:359-380).
//
// enable_grouping() (before the first add): every chunk is instead appended
// to a GroupIndex (grouper.h), which groups it by key as it arrives, so a
// convert() right after the map finds the group-by already done; finish()
// then returns the index's arenas (no concat) and take_group() the index.
#pragma once
#include <memory>
#include <string>
#include <vector>

#include "grouper.h"
#include "kv.h"
#include "spool.h"

namespace mrh {

class KeyValue {
 public:
  explicit KeyValue(at::Device dev) : dev_(dev) { reset_host(); }

  // add(key, keybytes, value, valuebytes)
  void add(const char* k, int64_t kb, const char* v, int64_t vb) {
    if (kb) kd_.append(k, (size_t)kb);
    if (vb) vd_.append(v, (size_t)vb);
    note(kb, vb);
    koff_.push_back((int64_t)kd_.size());
    voff_.push_back((int64_t)vd_.size());
    ++nh_;
    if (spool_ && (int64_t)(kd_.size() + vd_.size()) + 16 * nh_ >= piece_bytes_) flush();
  }
  // add(n, keys, keybytes, values, valuebytes): n fixed-size pairs, packed
  void add(int64_t n, const char* ks, int64_t kb, const char* vs, int64_t vb) {
    for (int64_t i = 0; i < n; ++i) add(ks + i * kb, kb, vs + i * vb, vb);
  }
  // add(n, keys, keybytes[], values, valuebytes[]): n variable-size pairs, packed
  void add(int64_t n, const char* ks, const int* kb, const char* vs, const int* vb) {
    int64_t ka = 0, va = 0;
    for (int64_t i = 0; i < n; ++i) {
      add(ks + ka, kb[i], vs + va, vb[i]);
      ka += kb[i];
      va += vb[i];
    }
  }
  void add_kv(const KV& kv) {
    flush();
    if (kv.n) push(kv);
  }
  void enable_grouping() {
    // a bounded (spooled) builder does not group: the index keeps everything in HBM
    if (!grp_ && !spool_ && chunks_.empty() && nh_ == 0) grp_ = std::make_shared<GroupIndex>(dev_);
  }
  // bound this builder by the tiers of `cfg` (before the first add)
  void set_spool(const SpoolConfig& cfg) {
    if (spool_ || grp_ || !chunks_.empty() || nh_) return;
    spool_ = std::make_unique<Spool>(dev_, cfg);
    piece_bytes_ = std::max<int64_t>(cfg.piece_bytes, 4096);
  }
  // tiers the spooled pieces went to (empty stats without a spool)
  SpoolStats spool_stats() const { return spool_ ? spool_->stats() : last_spool_; }
  // bytes per spooled piece of a bounded builder (0: unbounded) — a batch
  // callback whose output can dwarf its input emits it in chunks of this size
  int64_t piece_bytes() const { return spool_ ? piece_bytes_ : 0; }
  bool grouping() const { return grp_ != nullptr; }
  // capacity hint for the grouped arenas (GroupIndex::reserve); no-op without grouping
  void reserve_grouping(int64_t rows, int64_t key_bytes, int64_t value_bytes, int64_t groups = -1) {
    if (grp_) grp_->reserve(rows, key_bytes, value_bytes, groups);
  }
  // the index of the KV the last finish() returned (null if not grouped)
  std::shared_ptr<GroupIndex> take_group() { return std::move(done_); }
  int64_t size() const {
    int64_t n = nh_ + (grp_ ? grp_->size() : 0) + (spool_ ? spool_->n() : 0);
    for (auto& c : chunks_) n += c.n;
    return n;
  }
  KV finish();
  // the same pairs as parts in order, nothing concatenated: the chunks as
  // added, a spool's pieces where they lie (HBM / pinned host / files), the
  // grouped arenas as one part. Never empty (one empty KV at least).
  std::vector<KV> finish_parts();
  at::Device device() const { return dev_; }

 private:
  void note(int64_t kb, int64_t vb) {
    if (kw_ == -2) kw_ = (int)kb;
    else if (kw_ != kb) kw_ = -1;
    if (vw_ == -2) vw_ = (int)vb;
    else if (vw_ != vb) vw_ = -1;
  }
  void reset_host() {
    kd_.clear();
    vd_.clear();
    koff_.assign(1, 0);
    voff_.assign(1, 0);
    nh_ = 0;
    kw_ = vw_ = -2;
  }
  void flush();
  void push(const KV& chunk);

  at::Device dev_;
  std::string kd_, vd_;
  std::vector<int64_t> koff_, voff_;
  int64_t nh_ = 0;
  int kw_ = -2, vw_ = -2;
  std::vector<KV> chunks_;
  std::shared_ptr<GroupIndex> grp_, done_;
  std::unique_ptr<Spool> spool_;
  int64_t piece_bytes_ = int64_t(64) << 20;
  SpoolStats last_spool_;
};

}  // namespace mrh
