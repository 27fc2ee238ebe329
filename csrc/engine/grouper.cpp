// GroupIndex (grouper.h): host driver of the incremental group-by kernels
// (csrc/kernels/group.hip) plus the CPU twin the CPU engine and the tests run.
#include "grouper.h"

#include <ATen/hip/HIPContext.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <stdexcept>

#include "../kernels/launch.h"

namespace mrh {

namespace {

at::TensorOptions opt(at::Device d, at::ScalarType t) { return at::TensorOptions().device(d).dtype(t); }
template <typename T>
T* P0(const at::Tensor& t) {
  return t.defined() ? reinterpret_cast<T*>(t.data_ptr()) : nullptr;
}
hipStream_t cur() { return at::hip::getCurrentHIPStream(); }
[[noreturn]] void fail(const std::string& m) { throw std::runtime_error("mrhip: GroupIndex: " + m); }
int64_t pow2_at_least(int64_t x) {
  int64_t p = 1;
  while (p < x) p <<= 1;
  return p;
}
constexpr uint32_t CLAIM = 0x80000000u;
// same slot function as group.hip
uint64_t home(uint64_t h, uint64_t mask) { return (h ^ (h >> 32)) & mask; }

// t grown to >= need elements (x1.5 headroom), keeping the first `keep`
void grow(at::Tensor* t, int64_t need, int64_t keep, at::ScalarType ty, at::Device dev) {
  if (t->defined() && t->numel() >= need) return;
  const int64_t cap = std::max<int64_t>({need, t->defined() ? t->numel() * 3 / 2 : 0, 1024});
  at::Tensor n = at::empty({cap}, opt(dev, ty));
  if (t->defined() && keep > 0) n.narrow(0, 0, keep).copy_(t->narrow(0, 0, keep));
  *t = n;
}

void copy_bytes(uint8_t* dst, const uint8_t* src, int64_t bytes, bool cuda) {
  if (bytes <= 0) return;
  if (cuda) {
    if (hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyDeviceToDevice, cur()) != hipSuccess)
      fail("device copy failed");
  } else {
    std::memcpy(dst, src, (size_t)bytes);
  }
}

}  // namespace

// ====================================================================== HashDict

HashDict::HashDict(at::Device dev, int64_t cap) : dev_(dev) {
  if (!dev.is_cuda()) fail("HashDict is a device table");
  alloc(pow2_at_least(std::max<int64_t>(cap, 4096)), 0);
  ctr_ = at::zeros({4}, opt(dev_, at::kLong));
}

int64_t HashDict::cap_for(int64_t distinct) { return pow2_at_least(std::max<int64_t>(2 * distinct + 1, 4096)); }

// (re)allocate the table at `cap` slots; the first `keep` groups' rep/ghash
// are carried over (the slots are rehashed by grow())
void HashDict::alloc(int64_t cap, int64_t keep) {
  if (cap > (int64_t(1) << 31)) fail("more than 2^30 groups in one hash dictionary");
  at::Tensor rep = at::full({cap}, -1, opt(dev_, at::kLong));
  at::Tensor gh = at::empty({cap}, opt(dev_, at::kLong));
  if (keep > 0) {
    rep.narrow(0, 0, keep).copy_(rep_.narrow(0, 0, keep));
    gh.narrow(0, 0, keep).copy_(ghash_.narrow(0, 0, keep));
  }
  rep_ = rep;
  ghash_ = gh;
  static_assert(sizeof(k::DictSlot) == 32, "slot records are 32 bytes");
  at::Tensor ns = at::zeros({cap * 4}, opt(dev_, at::kLong));  // all-zero records: empty, unpublished
  if (cap_ > 0) k::dict_rehash(P0<k::DictSlot>(slots_), cap_, P0<k::DictSlot>(ns), cap, cur());
  slots_ = ns;
  cap_ = cap;
}

void HashDict::insert(const at::Tensor& kd, const at::Tensor& koff, int kw, const at::Tensor& h, int64_t n,
                      int64_t row0, int32_t* gid, bool retry) {
  if (n <= 0) return;
  if (h.defined() && (h.numel() < n || h.scalar_type() != at::kLong)) fail("HashDict: one int64 hash per row");
  if (!gid) fail("HashDict: insert needs the group id column");
  k::DictTable t;
  t.slots = P0<k::DictSlot>(slots_);
  t.mask = (uint64_t)cap_ - 1;
  t.rep = P0<int64_t>(rep_);
  t.ghash = P0<uint64_t>(ghash_);
  t.ctr = P0<unsigned long long>(ctr_);
  t.limit = cap_ / 2;
  k::dict_insert(P0<uint8_t>(kd), kw < 0 ? P0<int64_t>(koff) : nullptr, kw, h.defined() ? P0<uint64_t>(h) : nullptr,
                 n, row0, t, gid, retry, cur());
}

HashDict::Status HashDict::status() const {
  at::Tensor c = ctr_.to(at::kCPU);
  const int64_t* p = c.data_ptr<int64_t>();
  return Status{p[0], p[1], p[2]};
}

void HashDict::grow(int64_t min_groups) {
  alloc(std::max(cap_for(min_groups), cap_ * 2), cap_);  // every old group entry: no host sync
  ctr_.narrow(0, 3, 1).zero_();  // the table takes claims again
}

void HashDict::retry(const at::Tensor& kd, const at::Tensor& koff, int kw, const at::Tensor& h, int64_t n, int32_t* gid) {
  ctr_.narrow(0, 2, 1).zero_();  // the rows left unassigned are counted again
  insert(kd, koff, kw, h, n, 0, gid, true);
}

int64_t HashDict::sample_distinct(const KV& kv, int64_t m) {
  m = std::min(m, kv.n);
  if (m <= 0) return 0;
  at::Tensor hs = at::empty({m}, opt(kv.device(), at::kLong));
  k::dict_sample(P0<uint8_t>(kv.kdata), kv.kfixed() ? nullptr : P0<int64_t>(kv.koff), kv.kw, kv.n, m,
                 P0<uint64_t>(hs), cur());
  at::Tensor h = hs.to(at::kCPU);
  int64_t* p = h.data_ptr<int64_t>();
  std::sort(p, p + m);
  return (int64_t)(std::unique(p, p + m) - p);
}

namespace {

// group order (by 64-bit hash) -> rank of every group, first row of every
// rank, pairs per rank; shared by convert_dict and GroupIndex::finish
struct Ranked {
  at::Tensor order, rank, heads, seg;
  int64_t passes = 0;
};
// pairs per group g < m of a group id column (LDS histograms, group.hip)
at::Tensor group_counts(const at::Tensor& gid, int64_t n, int64_t m) {
  at::Tensor cnt = at::empty({m}, opt(gid.device(), at::kLong));
  at::Tensor ws = at::empty({k::dict_counts_ws_elems()}, opt(gid.device(), at::kInt));
  k::dict_counts(P0<int32_t>(gid), n, m, P0<uint64_t>(cnt), P0<uint32_t>(ws), cur());
  return cnt;
}

Ranked rank_groups(const HashDict& d, int64_t m, const at::Tensor& gid, int64_t n, bool want_seg) {
  const at::Device dev = d.rep().device();
  Ranked r;
  at::Tensor iota = at::empty({m}, opt(dev, at::kInt));
  k::iota_u32(P0<uint32_t>(iota), m, cur());
  auto [gs, order, p] = radix_sort_pairs(d.ghash().narrow(0, 0, m), iota, 0, 64, false);
  r.order = order;
  r.passes = p;
  r.rank = at::empty({m}, opt(dev, at::kInt));
  r.heads = at::empty({m}, opt(dev, at::kInt));
  k::grp_rank(P0<uint32_t>(order), m, P0<int64_t>(d.rep()), P0<uint32_t>(r.rank), P0<uint32_t>(r.heads), cur());
  if (want_seg) {
    at::Tensor gc = group_counts(gid, n, m);
    at::Tensor cnt = at::empty({m}, opt(dev, at::kLong));
    k::dict_ranked_counts(P0<uint32_t>(order), m, P0<uint64_t>(gc), P0<int64_t>(cnt), cur());
    r.seg = exclusive_scan(cnt);
  }
  return r;
}

// values of the pairs in group-rank order (stable: input order inside a group)
at::Tensor pairs_by_rank(const at::Tensor& gid, int64_t n, int64_t m, const at::Tensor& rank, int64_t* passes) {
  const at::Device dev = gid.device();
  at::Tensor key = at::empty({n}, opt(dev, at::kLong));
  k::grp_pairkey(P0<int32_t>(gid), n, P0<uint32_t>(rank), P0<uint64_t>(key), cur());
  at::Tensor iota = at::empty({n}, opt(dev, at::kInt));
  k::iota_u32(P0<uint32_t>(iota), n, cur());
  int bits = 1;
  while (bits < 63 && (int64_t(1) << bits) < m) ++bits;
  auto [sk, perm, p] = radix_sort_pairs(key, iota, 0, bits, false);
  *passes += p;
  return perm;
}

// MRH_DICT_CAP=<slots>: the first table's capacity (tests force a full
// table and the grow + retry paths with a small one)
int64_t dict_cap_override() {
  static const int64_t c = [] {
    const char* e = std::getenv("MRH_DICT_CAP");
    return e && *e ? (int64_t)std::atoll(e) : (int64_t)0;
  }();
  return c;
}

bool dict_disabled() {
  static const bool off = [] {
    const char* e = std::getenv("MRH_DICT_CONVERT");
    return e && *e == '0';
  }();
  return off;
}

}  // namespace

bool convert_dict(const KV& kv, KMV* out, ConvertStats* st, const at::Tensor& prehash) {
  const at::Device dev = kv.device();
  const int64_t n = kv.n;
  if (!dev.is_cuda() || dict_disabled() || n < (int64_t(1) << 20) || n >= (int64_t(1) << 31)) return false;
  // a strided sample decides: keys repeating at least ~2x in the sample group
  // on the dictionary, mostly distinct ones (URLs) on the sort
  constexpr int64_t kSample = 1 << 16;
  const int64_t ds = HashDict::sample_distinct(kv, kSample);
  const int64_t ms = std::min(n, kSample);
  if (2 * ds > ms) return false;
  st->dict = 2;
  const bool need_perm = kv.vw != 0;  // values to move into group order
  at::Tensor gid = at::empty({n}, opt(dev, at::kInt));
  const at::Tensor h = prehash.defined() ? prehash.to(dev).contiguous() : at::Tensor();
  // distinct keys grow with n (a Zipf vocabulary keeps growing): 32x the
  // sample's, at least 2^20 slots, at most what n distinct keys need
  int64_t cap = std::min(HashDict::cap_for(std::max<int64_t>(32 * ds, int64_t(1) << 19)), HashDict::cap_for(n));
  if (dict_cap_override() > 0) cap = dict_cap_override();
  HashDict d(dev, cap);
  d.insert(kv.kdata, kv.koff, kv.kw, h, n, 0, P0<int32_t>(gid), false);
  HashDict::Status s = d.status();
  while (s.left && !s.collisions) {  // a full table: the rest grouped in a larger one
    d.grow(s.groups + s.left);
    d.retry(kv.kdata, kv.koff, kv.kw, h, n, P0<int32_t>(gid));
    s = d.status();
  }
  st->dict_cap = d.cap();
  if (s.collisions) {
    st->collisions = s.collisions;
    return false;
  }
  const int64_t m = s.groups;
  Ranked r = rank_groups(d, m, gid, n, true);
  st->exact = false;
  st->passes = r.passes;
  st->dict = 1;
  KMV& o = *out;
  o.keys.n = m;
  o.keys.kw = kv.kw;
  o.keys.vw = 0;
  o.keys.kdata = gather_rows(kv.kdata, kv.koff, kv.kw, r.heads, &o.keys.koff);
  o.keys.vdata = at::empty({0}, opt(dev, at::kByte));
  o.vw = kv.vw;
  if (need_perm) {
    at::Tensor perm = pairs_by_rank(gid, n, m, r.rank, &st->passes);
    o.vdata = gather_rows(kv.vdata, kv.voff, kv.vw, perm, &o.voff);
  } else {
    o.vdata = at::empty({0}, opt(dev, at::kByte));
  }
  o.seg = r.seg;
  o.nkey = m;
  o.nval = n;
  return true;
}

// ====================================================================== GroupIndex

GroupIndex::GroupIndex(at::Device dev) : dev_(dev) {
  if (const char* b = std::getenv("MRH_GROUP_HASH_BITS")) hash_bits = std::max(1, std::min(64, std::atoi(b)));
}

bool GroupIndex::accepts(const KV& p) const {
  if (kw_ == -2) return true;
  return p.kw == kw_ && p.vw == vw_;
}

void GroupIndex::reserve_rows(int64_t rows) {
  if (rows <= rows_cap_) return;
  const int64_t cap = std::max<int64_t>({rows, rows_cap_ * 3 / 2, 1024});
  grow(&gid_, cap, n_, at::kInt, dev_);
  if (!dev_.is_cuda()) {
    grow(&rep_, cap, rows_cap_, at::kLong, dev_);  // group count is device-side: keep the whole old array
    grow(&ghash_, cap, rows_cap_, at::kLong, dev_);
  }
  rows_cap_ = cap;
}

// CPU twin: an open-addressing table of <= 50 % load for `groups` groups
void GroupIndex::reserve_table(int64_t groups) {
  if (dev_.is_cuda()) return;  // the HashDict sizes and grows itself
  if (2 * groups <= cap_) return;
  const int64_t cap = pow2_at_least(std::max<int64_t>(4 * groups, 4096));
  if (cap > (int64_t(1) << 31)) fail("more than 2^30 groups in one KV");
  at::Tensor ns = at::zeros({cap}, opt(dev_, at::kLong));
  at::Tensor ng = at::empty({cap}, opt(dev_, at::kInt));
  if (cap_ > 0) {
    const uint64_t* os = P0<uint64_t>(slots_);
    const int32_t* og = P0<int32_t>(sgid_);
    uint64_t* sl = P0<uint64_t>(ns);
    int32_t* g = P0<int32_t>(ng);
    for (int64_t i = 0; i < cap_; ++i) {
      if (!os[i]) continue;
      uint64_t j = home(os[i], (uint64_t)cap - 1);
      while (sl[j]) j = (j + 1) & ((uint64_t)cap - 1);
      sl[j] = os[i];
      g[j] = og[i];
    }
  }
  slots_ = ns;
  sgid_ = ng;
  cap_ = cap;
}

void GroupIndex::reserve(int64_t rows, int64_t key_bytes, int64_t value_bytes, int64_t groups) {
  if (rows <= 0) return;
  reserve_rows(rows);
  const int64_t g = groups < 0 ? rows : groups;
  reserve_table(g);
  table_hint_ = std::max(table_hint_, g);  // 0: sampled from the first part
  // a hint after the first part: grow the table now (no retry at finish)
  if (dict_ && g > 0 && HashDict::cap_for(g) > dict_->cap()) dict_->grow(g);
  auto col = [&](int w, int64_t bytes, at::Tensor* ad, at::Tensor* aoff, int64_t used) {
    if (w == -2) return;  // layout unknown until the first part
    if (w >= 0) {
      grow(ad, std::max<int64_t>(rows * w, 1), n_ * w, at::kByte, dev_);
    } else {
      grow(ad, std::max<int64_t>(bytes, 1), used, at::kByte, dev_);
      grow(aoff, rows + 1, n_ + 1, at::kLong, dev_);
    }
  };
  col(kw_, key_bytes, &kd_, &koff_, kbytes_);
  col(vw_, value_bytes, &vd_, &voff_, vbytes_);
}

void GroupIndex::append_col(const at::Tensor& pd, const at::Tensor& poff, int w, int64_t n, at::Tensor* ad,
                            at::Tensor* aoff, int64_t* bytes) {
  const bool cuda = dev_.is_cuda();
  if (w >= 0) {
    grow(ad, std::max<int64_t>((n_ + n) * w, 1), n_ * w, at::kByte, dev_);
    copy_bytes(P0<uint8_t>(*ad) + n_ * w, P0<uint8_t>(pd), n * w, cuda);
    return;
  }
  const int64_t pb = pd.numel();  // parts carry no slack: koff[n] == numel (as concat())
  grow(ad, std::max<int64_t>(*bytes + pb, 1), *bytes, at::kByte, dev_);
  grow(aoff, n_ + n + 1, n_ + 1, at::kLong, dev_);
  copy_bytes(P0<uint8_t>(*ad) + *bytes, P0<uint8_t>(pd), pb, cuda);
  if (cuda) {
    k::grp_append_off(P0<int64_t>(poff), n, *bytes, P0<int64_t>(*aoff) + n_, cur());
  } else {
    const int64_t* s = P0<int64_t>(poff);
    int64_t* d = P0<int64_t>(*aoff) + n_;
    for (int64_t i = 0; i <= n; ++i) d[i] = s[i] + *bytes;
  }
  *bytes += pb;
}

void GroupIndex::add(const KV& part_in) {
  if (part_in.n == 0) return;
  if (!accepts(part_in)) fail("part layout differs from the grouped parts");
  const KV part = part_in.device() == dev_ ? part_in : kv_to(part_in, dev_);
  const int64_t n = part.n;
  if (n_ + n >= (int64_t(1) << 31)) fail("more than 2^31 - 1 pairs in one grouped KV");
  if (kw_ == -2) {
    kw_ = part.kw;
    vw_ = part.vw;
    ctr_ = at::zeros({2}, opt(dev_, at::kLong));
  }
  reserve_rows(n_ + n);
  reserve_table(n_ + n);
  append_col(part.kdata, part.koff, kw_, n, &kd_, &koff_, &kbytes_);
  append_col(part.vdata, part.voff, vw_, n, &vd_, &voff_, &vbytes_);
  if (dev_.is_cuda()) {
    if (!dict_) {
      // sized for the reserve() hint (every row a group: never full), else
      // for 32x the distinct keys of a sample of the first part; a table
      // that fills up leaves rows unassigned and finish() grows it and
      // groups them (no per-part host sync)
      const int64_t cap = dict_cap_override() > 0 ? dict_cap_override()
                          : table_hint_ > 0     ? HashDict::cap_for(table_hint_)
                                          : HashDict::cap_for(std::min<int64_t>(
                                                std::max<int64_t>(32 * HashDict::sample_distinct(part, 1 << 14),
                                                                  int64_t(1) << 16),
                                                int64_t(1) << 29));
      dict_ = std::make_unique<HashDict>(dev_, cap);
    }
    at::Tensor h;
    if (hash_bits < 64) h = at::bitwise_and(hash64_keys(part), (int64_t)((1ull << hash_bits) - 1));
    dict_->insert(kd_, koff_, kw_, h, n, n_, P0<int32_t>(gid_), false);
    n_ += n;
    return;
  }
  at::Tensor h = hash64_keys(part);
  if (hash_bits < 64) h = at::bitwise_and(h, (int64_t)((1ull << hash_bits) - 1));
  const uint64_t* hp = P0<uint64_t>(h);
  uint64_t* slots = P0<uint64_t>(slots_);
  int32_t* sgid = P0<int32_t>(sgid_);
  int64_t* ctr = P0<int64_t>(ctr_);
  int64_t* rep = P0<int64_t>(rep_);
  uint64_t* gh = P0<uint64_t>(ghash_);
  int32_t* gid = P0<int32_t>(gid_);
  const uint8_t* kd = P0<uint8_t>(kd_);
  const int64_t* ko = kw_ < 0 ? P0<int64_t>(koff_) : nullptr;
  auto kat = [&](int64_t r) { return ko ? kd + ko[r] : kd + r * kw_; };
  auto klen = [&](int64_t r) { return ko ? ko[r + 1] - ko[r] : (int64_t)kw_; };
  const uint64_t mask = (uint64_t)cap_ - 1;
  for (int64_t i = 0; i < n; ++i) {
    const uint64_t hv = hp[i] ? hp[i] : 1;
    uint64_t s = home(hv, mask);
    while (slots[s] && slots[s] != hv) s = (s + 1) & mask;
    const int64_t r = n_ + i;
    if (!slots[s]) {
      slots[s] = hv;
      const int32_t g = (int32_t)ctr[0]++;
      sgid[s] = g;
      rep[g] = r;
      gh[g] = hv;
      gid[r] = g;
      continue;
    }
    const int32_t g = sgid[s];
    gid[r] = g;
    const int64_t b = rep[g];
    if (klen(r) != klen(b) || std::memcmp(kat(r), kat(b), (size_t)klen(r))) ++ctr[1];
  }
  n_ += n;
}

KV GroupIndex::kv() const {
  if (kw_ == -2) return empty_kv(dev_, 0, 0);
  KV o;
  o.n = n_;
  o.kw = kw_;
  o.vw = vw_;
  o.kdata = kd_.narrow(0, 0, kw_ >= 0 ? n_ * kw_ : kbytes_);
  o.vdata = vd_.narrow(0, 0, vw_ >= 0 ? n_ * vw_ : vbytes_);
  if (kw_ < 0) o.koff = koff_.narrow(0, 0, n_ + 1);
  if (vw_ < 0) o.voff = voff_.narrow(0, 0, n_ + 1);
  return o;
}

bool GroupIndex::describes(const KV& kv) const {
  // same arena storage (data_ptr() of an empty view is null: zero-width values)
  auto same = [](const at::Tensor& t, const at::Tensor& a) {
    return t.defined() && a.defined() && t.has_storage() && t.storage().data() == a.storage().data();
  };
  return kw_ != -2 && n_ > 0 && kv.n == n_ && kv.kw == kw_ && kv.vw == vw_ && same(kv.kdata, kd_) &&
         same(kv.vdata, vd_);
}

bool GroupIndex::finish(KMV* out, ConvertStats* st) {
  if (!describes(kv())) fail("finish on an empty index");
  const bool cuda = dev_.is_cuda();
  int64_t m = 0, coll = 0;
  at::Tensor rep, ghash;
  if (cuda) {
    // the one host sync of the group-by: groups, collisions, rows a full
    // table left unassigned (grouped now in a larger table)
    HashDict::Status s = dict_->status();
    while (s.left && !s.collisions) {
      at::Tensor h;  // the hashes the parts were grouped on (narrowed in tests)
      if (hash_bits < 64) h = at::bitwise_and(hash64_keys(kv()), (int64_t)((1ull << hash_bits) - 1));
      dict_->grow(s.groups + s.left);
      dict_->retry(kd_, koff_, kw_, h, n_, P0<int32_t>(gid_));
      s = dict_->status();
    }
    m = s.groups;
    coll = s.collisions;
    rep = dict_->rep();
    ghash = dict_->ghash();
  } else {
    at::Tensor c = ctr_.to(at::kCPU);
    m = c.data_ptr<int64_t>()[0];
    coll = c.data_ptr<int64_t>()[1];
    rep = rep_;
    ghash = ghash_;
  }
  st->exact = false;
  st->collisions = coll;
  if (coll) return false;
  const int64_t n = n_;
  auto iota = [&](int64_t len) {
    at::Tensor t = at::empty({len}, opt(dev_, at::kInt));
    if (cuda) {
      k::iota_u32(P0<uint32_t>(t), len, cur());
    } else {
      std::iota(P0<int32_t>(t), P0<int32_t>(t) + len, 0);
    }
    return t;
  };
  // 1. groups in convert's key order: fixed keys of <= 8 bytes by their raw
  // little-endian value (exact), all others by 64-bit hash
  at::Tensor gkey;
  int gbits = 64;
  if (kw_ >= 0 && kw_ <= 8) {
    gbits = std::max(8, 8 * kw_);
    at::Tensor rep32 = rep.narrow(0, 0, m).to(at::kInt);
    at::Tensor uk = gather_rows(kd_, at::Tensor(), kw_, rep32, nullptr);
    gkey = at::empty({m}, opt(dev_, at::kLong));
    if (cuda) {
      at::Tensor scratch_idx = at::empty({m}, opt(dev_, at::kInt));
      k::make_sortkeys_fixed(P0<uint8_t>(uk), kw_, m, 0, false, P0<uint64_t>(gkey), P0<uint32_t>(scratch_idx), cur());
    } else {
      const uint8_t* d = P0<uint8_t>(uk);
      uint64_t* g = P0<uint64_t>(gkey);
      for (int64_t j = 0; j < m; ++j) {
        uint64_t raw = 0;
        for (int b = 0; b < kw_; ++b) raw |= (uint64_t)d[j * kw_ + b] << (8 * b);
        g[j] = raw;
      }
    }
  } else {
    gkey = ghash.narrow(0, 0, m);
  }
  auto [gsorted, order, p1] = radix_sort_pairs(gkey, iota(m), 0, gbits, false);
  at::Tensor rank = at::empty({m}, opt(dev_, at::kInt)), heads = at::empty({m}, opt(dev_, at::kInt));
  if (cuda) {
    k::grp_rank(P0<uint32_t>(order), m, P0<int64_t>(rep), P0<uint32_t>(rank), P0<uint32_t>(heads), cur());
  } else {
    const int32_t* o = P0<int32_t>(order);
    const int64_t* rp = P0<int64_t>(rep);
    int32_t* rk = P0<int32_t>(rank);
    int32_t* hd = P0<int32_t>(heads);
    for (int64_t j = 0; j < m; ++j) {
      rk[o[j]] = (int32_t)j;
      hd[j] = (int32_t)rp[o[j]];
    }
  }
  st->passes = p1;
  const KV all = kv();
  KMV& o = *out;
  o.keys.n = m;
  o.keys.kw = kw_;
  o.keys.vw = 0;
  o.keys.kdata = gather_rows(all.kdata, all.koff, kw_, heads, &o.keys.koff);
  o.keys.vdata = at::empty({0}, opt(dev_, at::kByte));
  o.vw = vw_;
  o.nkey = m;
  o.nval = n;
  if (cuda && vw_ == 0) {
    // 2. zero-width values: the segments are the prefix sums of the group
    // counts in rank order; no pair moves
    at::Tensor gc = group_counts(gid_, n, m);
    at::Tensor cnt = at::empty({m}, opt(dev_, at::kLong));
    k::dict_ranked_counts(P0<uint32_t>(order), m, P0<uint64_t>(gc), P0<int64_t>(cnt), cur());
    o.seg = exclusive_scan(cnt);
    o.vdata = at::empty({0}, opt(dev_, at::kByte));
    return true;
  }
  // 2. pairs by group rank: stable, so values keep their append order
  at::Tensor key = at::empty({n}, opt(dev_, at::kLong));
  if (cuda) {
    k::grp_pairkey(P0<int32_t>(gid_), n, P0<uint32_t>(rank), P0<uint64_t>(key), cur());
  } else {
    const int32_t* rk = P0<int32_t>(rank);
    const int32_t* g = P0<int32_t>(gid_);
    int64_t* kp = P0<int64_t>(key);
    for (int64_t i = 0; i < n; ++i) kp[i] = rk[g[i]];
  }
  int bits = 1;
  while (bits < 63 && (int64_t(1) << bits) < m) ++bits;
  auto [sk, perm, p2] = radix_sort_pairs(key, iota(n), 0, bits, false);
  at::Tensor seg = at::empty({m + 1}, opt(dev_, at::kLong));
  if (cuda) {
    k::grp_seg(P0<uint64_t>(sk), n, m, P0<int64_t>(seg), cur());
  } else {
    const int64_t* sv = P0<int64_t>(sk);
    int64_t* sg = P0<int64_t>(seg);
    for (int64_t i = 0; i < n; ++i)
      if (i == 0 || sv[i - 1] != sv[i]) sg[sv[i]] = i;
    sg[m] = n;
  }
  st->passes = p1 + p2;
  o.vdata = gather_rows(all.vdata, all.voff, vw_, perm, &o.voff);
  o.seg = seg;
  return true;
}

}  // namespace mrh
