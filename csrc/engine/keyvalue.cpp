// KeyValue builder (see keyvalue.h).
#include "keyvalue.h"

namespace mrh {

void KeyValue::flush() {
  if (nh_ == 0) return;
  KV kv;
  kv.n = nh_;
  auto bytes = [](const std::string& s) {
    return at::from_blob((void*)s.data(), {(int64_t)s.size()}, at::TensorOptions().dtype(at::kByte)).clone();
  };
  kv.kdata = bytes(kd_);
  kv.vdata = bytes(vd_);
  kv.kw = kw_ >= 0 ? kw_ : -1;
  kv.vw = vw_ >= 0 ? vw_ : -1;
  if (kv.kw < 0)
    kv.koff = at::from_blob(koff_.data(), {(int64_t)koff_.size()}, at::TensorOptions().dtype(at::kLong)).clone();
  if (kv.vw < 0)
    kv.voff = at::from_blob(voff_.data(), {(int64_t)voff_.size()}, at::TensorOptions().dtype(at::kLong)).clone();
  reset_host();
  if (spool_) {
    spool_->add(kv);  // the spool picks the tier (no detour through HBM)
    return;
  }
  push(kv_to(kv, dev_));
}

void KeyValue::push(const KV& c) {
  if (spool_) {
    spool_->add(c);
    return;
  }
  if (grp_) {
    if (grp_->accepts(c)) {
      grp_->add(c);
      return;
    }
    // a chunk of another layout: grouping stops, what it holds becomes a chunk
    if (grp_->size()) chunks_.push_back(grp_->kv());
    grp_.reset();
  }
  chunks_.push_back(c);
}

KV KeyValue::finish() {
  flush();
  done_.reset();
  if (spool_) {
    KV out = spool_->n() ? spool_->gather() : empty_kv(dev_, kw_ >= 0 ? kw_ : 0, vw_ >= 0 ? vw_ : 0);
    last_spool_ = spool_->stats();
    spool_.reset();
    return out;
  }
  if (grp_) {
    KV out = grp_->size() ? grp_->kv() : empty_kv(dev_, 0, 0);
    if (grp_->size()) done_ = std::move(grp_);
    grp_.reset();
    return out;
  }
  KV out = concat(chunks_, dev_);
  chunks_.clear();
  return out;
}

std::vector<KV> KeyValue::finish_parts() {
  flush();
  const KV none = empty_kv(dev_, kw_ >= 0 ? kw_ : 0, vw_ >= 0 ? vw_ : 0);
  if (spool_) {
    std::vector<KV> out = spool_->take();
    last_spool_ = spool_->stats();
    spool_.reset();
    done_.reset();
    if (out.empty()) out.push_back(none);
    return out;
  }
  if (grp_) return {finish()};
  done_.reset();
  std::vector<KV> out;
  for (const KV& c : chunks_)
    if (c.n) out.push_back(c);
  chunks_.clear();
  if (out.empty()) out.push_back(none);
  return out;
}

}  // namespace mrh
