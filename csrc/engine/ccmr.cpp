// cc_find_mr callback ops (kernels: csrc/kernels/ccmr.hip) with host twins of
// identical semantics — including the salting RNG (splitmix64 of seed ^ pair
// index), so a CPU and a GPU run of the pipeline salt identically. The OINK
// command cc_find_mr (commands.cpp) runs the reference's zone pipeline
// (oink/cc_find.cpp:38-109) with these as its batch callbacks.
#include <ATen/hip/HIPContext.h>

#include <algorithm>
#include <cstring>
#include <limits>
#include <stdexcept>
#include <vector>

#include "../kernels/launch.h"
#include "ccmr.h"

namespace mrh {

namespace {
at::TensorOptions opt(at::Device d, at::ScalarType t) { return at::TensorOptions().device(d).dtype(t); }
template <typename T>
T* P0(const at::Tensor& t) {
  return t.defined() ? reinterpret_cast<T*>(t.data_ptr()) : nullptr;
}
hipStream_t cur() { return at::hip::getCurrentHIPStream(); }
void need(bool c, const char* m) {
  if (!c) throw std::runtime_error(std::string("mrhip: ") + m);
}
constexpr int64_t HIBIT = std::numeric_limits<int64_t>::min();
int64_t ld8(const uint8_t* p) {
  int64_t v;
  std::memcpy(&v, p, 8);
  return v;
}
uint64_t mix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
// value offsets of a KMV (fixed-width values get explicit ones)
at::Tensor value_offsets(const KMV& m) {
  return m.vw >= 0 ? fixed_offsets(m.nval, m.vw, m.seg.device()) : m.voff.contiguous();
}
// exclusive scan of int64 flags -> (pos[n+1], total)
std::pair<at::Tensor, int64_t> scan_count(const at::Tensor& f) {
  at::Tensor pos = exclusive_scan(f);
  return {pos, f.numel() ? pos[f.numel()].item<int64_t>() : 0};
}
}  // namespace

std::pair<at::Tensor, at::Tensor> ccmr_edge_zone(const KMV& m) {
  const at::Device dev = m.seg.device();
  at::Tensor voff = value_offsets(m);
  const int64_t* seg = P0<int64_t>(m.seg);
  if (dev.is_cuda()) {
    at::Tensor zone_of = at::zeros({std::max<int64_t>(m.nkey, 1)}, opt(dev, at::kLong));
    k::ccmr_edge_zone_of(seg, m.nkey, P0<int64_t>(voff), P0<uint8_t>(m.vdata), m.nval, P0<int64_t>(zone_of), cur());
    at::Tensor f = at::empty({m.nval}, opt(dev, at::kLong));
    k::ccmr_len_flags(P0<int64_t>(voff), m.nval, 16, P0<int64_t>(f), cur());
    auto [pos, ne] = scan_count(f);
    at::Tensor edge = at::empty({ne, 2}, opt(dev, at::kLong)), zone = at::empty({ne}, opt(dev, at::kLong));
    if (ne)
      k::ccmr_edge_zone_emit(seg, m.nkey, P0<int64_t>(voff), P0<uint8_t>(m.vdata), m.nval, P0<int64_t>(zone_of),
                             P0<int64_t>(pos), P0<int64_t>(edge), P0<int64_t>(zone), cur());
    return {edge, zone};
  }
  const int64_t* vo = P0<int64_t>(voff);
  const uint8_t* vd = P0<uint8_t>(m.vdata);
  std::vector<int64_t> e, z;
  for (int64_t s = 0; s < m.nkey; ++s) {
    int64_t zs = 0;
    for (int64_t j = seg[s]; j < seg[s + 1]; ++j)
      if (vo[j + 1] - vo[j] == 8) zs = ld8(vd + vo[j]);
    for (int64_t j = seg[s]; j < seg[s + 1]; ++j)
      if (vo[j + 1] - vo[j] == 16) {
        e.push_back(ld8(vd + vo[j]));
        e.push_back(ld8(vd + vo[j] + 8));
        z.push_back(zs);
      }
  }
  return {at::tensor(e, opt(at::kCPU, at::kLong)).view({-1, 2}), at::tensor(z, opt(at::kCPU, at::kLong))};
}

std::pair<at::Tensor, at::Tensor> ccmr_winner(const KMV& m) {
  need(m.vw == 8, "cc_find_mr winner: 8-byte zone values");
  const at::Device dev = m.seg.device();
  const int64_t* seg = P0<int64_t>(m.seg);
  const int64_t* z = P0<int64_t>(m.vdata);
  if (dev.is_cuda()) {
    at::Tensor f = at::empty({m.nkey}, opt(dev, at::kLong));
    k::ccmr_winner_flags(seg, m.nkey, z, m.nval, P0<int64_t>(f), cur());
    auto [pos, nw] = scan_count(f);
    at::Tensor big = at::empty({nw}, opt(dev, at::kLong)), pad = at::empty({nw, 2}, opt(dev, at::kLong));
    if (nw) k::ccmr_winner_emit(seg, m.nkey, z, m.nval, P0<int64_t>(pos), P0<int64_t>(big), P0<int64_t>(pad), cur());
    return {big, pad};
  }
  std::vector<int64_t> b, p;
  for (int64_t s = 0; s < m.nkey; ++s) {
    const int64_t h = seg[s], z0 = z[h], z1 = z[std::min<int64_t>(h + 1, m.nval - 1)];
    const int64_t s0 = z0 & ~HIBIT, s1 = z1 & ~HIBIT;
    if (s0 == s1) continue;
    b.push_back(s0 > s1 ? z0 : z1);
    p.push_back(s0 > s1 ? z1 : z0);
    p.push_back(0);
  }
  return {at::tensor(b, opt(at::kCPU, at::kLong)), at::tensor(p, opt(at::kCPU, at::kLong)).view({-1, 2})};
}

std::pair<at::Tensor, at::Tensor> ccmr_invert(const KV& kv, int P, int pshift, uint64_t seed) {
  need(kv.kw == 8 && kv.vw == 8, "cc_find_mr invert: (vertex, zone) pairs");
  const at::Device dev = kv.device();
  at::Tensor key = at::empty({kv.n}, opt(dev, at::kLong)), val = at::empty({kv.n}, opt(dev, at::kLong));
  const int64_t* v = P0<int64_t>(kv.kdata);
  const int64_t* zn = P0<int64_t>(kv.vdata);
  if (dev.is_cuda()) {
    k::ccmr_invert(v, zn, kv.n, P, pshift, seed, P0<int64_t>(key), P0<int64_t>(val), cur());
    return {key, val};
  }
  int64_t* ko = P0<int64_t>(key);
  int64_t* vo = P0<int64_t>(val);
  for (int64_t i = 0; i < kv.n; ++i) {
    const int64_t rp = (int64_t)(mix64(seed ^ (uint64_t)i) % (uint64_t)P);
    ko[i] = zn[i] < 0 ? (zn[i] | (rp << pshift)) : zn[i];
    vo[i] = v[i];
  }
  return {key, val};
}

std::pair<at::Tensor, at::Tensor> ccmr_zone_multi(const KV& kv, int P, int pshift) {
  need(kv.kw == 8 && kv.vw == 16, "cc_find_mr zone_multi: (zone, {zone, pad}) pairs");
  const at::Device dev = kv.device();
  const int64_t* zn = P0<int64_t>(kv.kdata);
  const int64_t* pad = P0<int64_t>(kv.vdata);
  if (dev.is_cuda()) {
    at::Tensor f = at::empty({kv.n}, opt(dev, at::kLong));
    k::ccmr_hot_flags(zn, kv.n, P0<int64_t>(f), cur());
    auto [pos, nhot] = scan_count(f);
    const int64_t n = kv.n + nhot * P;
    at::Tensor key = at::empty({n}, opt(dev, at::kLong)), val = at::empty({n, 2}, opt(dev, at::kLong));
    k::ccmr_zone_multi(zn, pad, kv.n, P, pshift, P0<int64_t>(pos), P0<int64_t>(key), P0<int64_t>(val), cur());
    return {key, val};
  }
  std::vector<int64_t> k, v, hk, hv;
  for (int64_t i = 0; i < kv.n; ++i) {
    const int64_t strip = zn[i] & ~HIBIT;
    k.push_back(strip);
    v.insert(v.end(), {pad[2 * i], pad[2 * i + 1]});
    if (zn[i] < 0)
      for (int r = 0; r < P; ++r) {
        hk.push_back(strip | ((int64_t)r << pshift) | HIBIT);
        hv.insert(hv.end(), {pad[2 * i], pad[2 * i + 1]});
      }
  }
  k.insert(k.end(), hk.begin(), hk.end());
  v.insert(v.end(), hv.begin(), hv.end());
  return {at::tensor(k, opt(at::kCPU, at::kLong)), at::tensor(v, opt(at::kCPU, at::kLong)).view({-1, 2})};
}

std::pair<at::Tensor, at::Tensor> ccmr_reassign(const KMV& m, int64_t lmask, int64_t nthresh) {
  need(m.keys.kw == 8, "cc_find_mr reassign: 8-byte zone keys");
  const at::Device dev = m.seg.device();
  at::Tensor voff = value_offsets(m);
  const int64_t* seg = P0<int64_t>(m.seg);
  const int64_t* keys = P0<int64_t>(m.keys.kdata);
  if (dev.is_cuda()) {
    at::Tensor zs = at::empty({std::max<int64_t>(m.nkey, 1)}, opt(dev, at::kLong));
    k::ccmr_reassign_seg(seg, m.nkey, keys, P0<int64_t>(voff), P0<uint8_t>(m.vdata), lmask, nthresh,
                         P0<int64_t>(zs), cur());
    at::Tensor f = at::empty({m.nval}, opt(dev, at::kLong));
    k::ccmr_len_flags(P0<int64_t>(voff), m.nval, 8, P0<int64_t>(f), cur());
    auto [pos, nv] = scan_count(f);
    at::Tensor v = at::empty({nv}, opt(dev, at::kLong)), zone = at::empty({nv}, opt(dev, at::kLong));
    if (nv)
      k::ccmr_reassign_emit(seg, m.nkey, P0<int64_t>(voff), P0<uint8_t>(m.vdata), m.nval, P0<int64_t>(zs),
                            P0<int64_t>(pos), P0<int64_t>(v), P0<int64_t>(zone), cur());
    return {v, zone};
  }
  const int64_t* vo = P0<int64_t>(voff);
  const uint8_t* vd = P0<uint8_t>(m.vdata);
  std::vector<int64_t> v, z;
  for (int64_t s = 0; s < m.nkey; ++s) {
    const int64_t key = keys[s], zone = key & lmask;
    int64_t best = zone, nvert = 0;
    for (int64_t j = seg[s]; j < seg[s + 1]; ++j) {
      const int64_t l = vo[j + 1] - vo[j];
      if (l == 8) ++nvert;
      else if (l == 16) best = std::min<int64_t>(best, ld8(vd + vo[j]) & ~HIBIT);
    }
    bool hwin = false;
    if (best < zone)
      for (int64_t j = seg[s]; j < seg[s + 1] && !hwin; ++j)
        if (vo[j + 1] - vo[j] == 16) {
          const int64_t pz = ld8(vd + vo[j]);
          hwin = pz < 0 && (pz & ~HIBIT) == best;
        }
    const int64_t zf = (key < 0 || hwin || nvert > nthresh) ? (best | HIBIT) : best;
    for (int64_t j = seg[s]; j < seg[s + 1]; ++j)
      if (vo[j + 1] - vo[j] == 8) {
        v.push_back(ld8(vd + vo[j]));
        z.push_back(zf);
      }
  }
  return {at::tensor(v, opt(at::kCPU, at::kLong)), at::tensor(z, opt(at::kCPU, at::kLong))};
}

}  // namespace mrh
