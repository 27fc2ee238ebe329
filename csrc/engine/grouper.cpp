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
  grow(&rep_, cap, rows_cap_, at::kLong, dev_);  // group count is device-side: keep the whole old array
  grow(&ghash_, cap, rows_cap_, at::kLong, dev_);
  rows_cap_ = cap;
}

void GroupIndex::reserve_table(int64_t groups) {
  if (2 * groups <= cap_) return;  // load stays <= 50 %: every probe ends at a match or a free slot
  const int64_t cap = pow2_at_least(std::max<int64_t>(4 * groups, 4096));
  if (cap > (int64_t(1) << 31)) fail("more than 2^30 groups in one KV");
  at::Tensor ns = at::zeros({cap}, opt(dev_, at::kLong));
  at::Tensor ng = at::empty({cap}, opt(dev_, at::kInt));
  if (cap_ > 0) {
    if (dev_.is_cuda()) {
      k::grp_rehash(P0<uint64_t>(slots_), P0<int32_t>(sgid_), cap_, P0<uint64_t>(ns), P0<int32_t>(ng), cap, cur());
    } else {
      const uint64_t* os = P0<uint64_t>(slots_);
      const int32_t* og = P0<int32_t>(sgid_);
      uint64_t* s = P0<uint64_t>(ns);
      int32_t* g = P0<int32_t>(ng);
      for (int64_t i = 0; i < cap_; ++i) {
        if (!os[i]) continue;
        uint64_t j = home(os[i], (uint64_t)cap - 1);
        while (s[j]) j = (j + 1) & ((uint64_t)cap - 1);
        s[j] = os[i];
        g[j] = og[i];
      }
    }
  }
  slots_ = ns;
  sgid_ = ng;
  cap_ = cap;
}

void GroupIndex::reserve(int64_t rows, int64_t key_bytes, int64_t value_bytes) {
  if (rows <= 0) return;
  reserve_rows(rows);
  reserve_table(rows);
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
  at::Tensor h = hash64_keys(part);
  if (hash_bits < 64) h = at::bitwise_and(h, (int64_t)((1ull << hash_bits) - 1));
  if (dev_.is_cuda()) {
    at::Tensor code = at::empty({n}, opt(dev_, at::kInt));
    k::grp_insert(P0<uint64_t>(h), n, n_, P0<uint64_t>(slots_), P0<int32_t>(sgid_), cap_, P0<uint64_t>(ctr_),
                  P0<int64_t>(rep_), P0<uint64_t>(ghash_), P0<uint32_t>(code), cur());
    k::grp_resolve(P0<uint32_t>(code), n, n_, P0<int32_t>(sgid_), P0<int64_t>(rep_), P0<uint8_t>(kd_),
                   kw_ < 0 ? P0<int64_t>(koff_) : nullptr, kw_, P0<int32_t>(gid_), P0<uint64_t>(ctr_), cur());
  } else {
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
  at::Tensor c = ctr_.to(at::kCPU);  // the one host sync of the group-by: group count + collisions
  const int64_t m = c.data_ptr<int64_t>()[0], coll = c.data_ptr<int64_t>()[1];
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
    at::Tensor rep32 = rep_.narrow(0, 0, m).to(at::kInt);
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
    gkey = ghash_.narrow(0, 0, m);
  }
  auto [gsorted, order, p1] = radix_sort_pairs(gkey, iota(m), 0, gbits, false);
  at::Tensor rank = at::empty({m}, opt(dev_, at::kInt)), heads = at::empty({m}, opt(dev_, at::kInt));
  at::Tensor key = at::empty({n}, opt(dev_, at::kLong));
  if (cuda) {
    k::grp_rank(P0<uint32_t>(order), m, P0<int64_t>(rep_), P0<uint32_t>(rank), P0<uint32_t>(heads), cur());
    k::grp_pairkey(P0<int32_t>(gid_), n, P0<uint32_t>(rank), P0<uint64_t>(key), cur());
  } else {
    const int32_t* o = P0<int32_t>(order);
    const int64_t* rp = P0<int64_t>(rep_);
    int32_t* rk = P0<int32_t>(rank);
    int32_t* hd = P0<int32_t>(heads);
    for (int64_t j = 0; j < m; ++j) {
      rk[o[j]] = (int32_t)j;
      hd[j] = (int32_t)rp[o[j]];
    }
    const int32_t* g = P0<int32_t>(gid_);
    int64_t* kp = P0<int64_t>(key);
    for (int64_t i = 0; i < n; ++i) kp[i] = rk[g[i]];
  }
  // 2. pairs by group rank: stable, so values keep their append order
  int bits = 1;
  while (bits < 63 && (int64_t(1) << bits) < m) ++bits;
  auto [sk, perm, p2] = radix_sort_pairs(key, iota(n), 0, bits, false);
  at::Tensor seg = at::empty({m + 1}, opt(dev_, at::kLong));
  if (cuda) {
    k::grp_seg(P0<uint64_t>(sk), n, m, P0<int64_t>(seg), cur());
  } else {
    const int64_t* s = P0<int64_t>(sk);
    int64_t* sg = P0<int64_t>(seg);
    for (int64_t i = 0; i < n; ++i)
      if (i == 0 || s[i - 1] != s[i]) sg[s[i]] = i;
    sg[m] = n;
  }
  st->passes = p1 + p2;
  const KV all = kv();
  KMV& o = *out;
  o.keys.n = m;
  o.keys.kw = kw_;
  o.keys.vw = 0;
  o.keys.kdata = gather_rows(all.kdata, all.koff, kw_, heads, &o.keys.koff);
  o.keys.vdata = at::empty({0}, opt(dev_, at::kByte));
  o.vw = vw_;
  o.vdata = gather_rows(all.vdata, all.voff, vw_, perm, &o.voff);
  o.seg = seg;
  o.nkey = m;
  o.nval = n;
  return true;
}

}  // namespace mrh
