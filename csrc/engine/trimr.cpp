// tri_find_mr callback ops (kernels: csrc/kernels/trimr.hip) with CPU twins
// of identical semantics. The OINK command tri_find_mr (commands.cpp) runs
// the reference's 4-shuffle pipeline (oink/tri_find.cpp:43-82) with these
// as its batch map/reduce callbacks.
#include <ATen/hip/HIPContext.h>

#include <cstring>
#include <stdexcept>

#include "../kernels/launch.h"
#include "kv.h"
#include "tri.h"

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
// zero-filled byte array: a runtime memset on the device (no ATen fill kernel)
at::Tensor zeroed_bytes(int64_t n, at::Device dev) {
  at::Tensor t = at::empty({n}, opt(dev, at::kByte));
  if (dev.is_cuda()) {
    if (n && hipMemsetAsync(t.data_ptr(), 0, (size_t)n, at::hip::getCurrentHIPStream()) != hipSuccess)
      throw std::runtime_error("trimr: memset failed");
  } else {
    t.zero_();
  }
  return t;
}
}  // namespace

std::pair<at::Tensor, at::Tensor> trimr_first_degree(const KMV& m) {
  need(m.vw == 8 && m.keys.kw == 8, "tri_find_mr first degree: 8-byte vertex keys and values");
  const at::Device dev = m.seg.device();
  at::Tensor edge = at::empty({m.nval, 2}, opt(dev, at::kLong)), deg = at::empty({m.nval, 2}, opt(dev, at::kInt));
  if (!m.nval) return {edge, deg};
  const int64_t* seg = P0<int64_t>(m.seg);
  const int64_t* key = P0<int64_t>(m.keys.kdata);
  const int64_t* nbr = P0<int64_t>(m.vdata);
  if (dev.is_cuda()) {
    k::trimr_first_degree(seg, m.nkey, key, nbr, m.nval, P0<int64_t>(edge), P0<int32_t>(deg), cur());
    return {edge, deg};
  }
  int64_t* e = P0<int64_t>(edge);
  int32_t* d = P0<int32_t>(deg);
  for (int64_t s = 0; s < m.nkey; ++s) {
    const int32_t n = (int32_t)(seg[s + 1] - seg[s]);
    for (int64_t j = seg[s]; j < seg[s + 1]; ++j) {
      const int64_t vi = key[s], vj = nbr[j];
      const bool lt = vi < vj;
      e[2 * j] = lt ? vi : vj;
      e[2 * j + 1] = lt ? vj : vi;
      d[2 * j] = lt ? n : 0;
      d[2 * j + 1] = lt ? 0 : n;
    }
  }
  return {edge, deg};
}

at::Tensor trimr_second_degree(const KMV& m) {
  need(m.vw == 8, "tri_find_mr second degree: {int, int} values");
  const at::Device dev = m.seg.device();
  at::Tensor out = at::empty({m.nkey, 2}, opt(dev, at::kInt));
  if (!m.nkey) return out;
  const int64_t* seg = P0<int64_t>(m.seg);
  const int32_t* v = P0<int32_t>(m.vdata);
  if (dev.is_cuda()) {
    k::trimr_second_degree(seg, m.nkey, v, m.nval, P0<int32_t>(out), cur());
    return out;
  }
  int32_t* o = P0<int32_t>(out);
  for (int64_t s = 0; s < m.nkey; ++s) {
    const int64_t h = seg[s], h2 = h + 1 < m.nval ? h + 1 : m.nval - 1;
    const bool use1 = v[2 * h] != 0;
    o[2 * s] = use1 ? v[2 * h] : v[2 * h2];
    o[2 * s + 1] = use1 ? v[2 * h2 + 1] : v[2 * h + 1];
  }
  return out;
}

std::pair<at::Tensor, at::Tensor> trimr_low_degree(const KV& kv) {
  need(kv.kw == 16 && kv.vw == 8, "tri_find_mr low degree: EDGE keys, {int, int} values");
  const at::Device dev = kv.device();
  at::Tensor key = at::empty({kv.n}, opt(dev, at::kLong)), val = at::empty({kv.n}, opt(dev, at::kLong));
  if (!kv.n) return {key, val};
  const int64_t* e = P0<int64_t>(kv.kdata);
  const int32_t* dg = P0<int32_t>(kv.vdata);
  if (dev.is_cuda()) {
    k::trimr_low_degree(e, dg, kv.n, P0<int64_t>(key), P0<int64_t>(val), cur());
    return {key, val};
  }
  int64_t* k = P0<int64_t>(key);
  int64_t* v = P0<int64_t>(val);
  for (int64_t i = 0; i < kv.n; ++i) {
    const int64_t vi = e[2 * i], vj = e[2 * i + 1];
    const int32_t di = dg[2 * i], dj = dg[2 * i + 1];
    const bool fi = di < dj || (di == dj && vi < vj);
    k[i] = fi ? vi : vj;
    v[i] = fi ? vj : vi;
  }
  return {key, val};
}

// Compact layout (large graphs): keys are one packed word vi << vb | vj,
// values u32 centres; an edge carries vi as its marker (tri.h)
at::Tensor trimr_emit_compact(const KMV& m, int vb) {
  const at::Device dev = m.seg.device();
  if (!m.nkey || !m.nval) return at::empty({0, 3}, opt(dev, at::kLong));
  need(m.keys.kw == 8 && m.vw == 4, "tri_find_mr emit (compact): packed 8-byte edge keys, 4-byte centres");
  const int64_t* seg = P0<int64_t>(m.seg);
  const int64_t* ek = P0<int64_t>(m.keys.kdata);
  if (dev.is_cuda()) {
    const int64_t nval = m.nval;
    at::Tensor marked = zeroed_bytes(m.nkey, dev);
    const int64_t nt = k::trimr_emit_tiles(nval);
    at::Tensor tcount = at::empty({std::max<int64_t>(nt, 1)}, opt(dev, at::kLong));
    const void* vals = m.vdata.data_ptr();
    at::Tensor tk = at::empty({nt + 1}, opt(dev, at::kLong));
    const int64_t* tkp = P0<int64_t>(tk);
    k::trimr_emit_tile_keys(seg, m.nkey, nval, P0<int64_t>(tk), cur());
    k::trimr_emit_fixed(0, seg, m.nkey, nval, vals, P0<uint8_t>(marked), nullptr, nullptr, ek, nullptr, vb, tkp, cur());
    k::trimr_emit_fixed(1, seg, m.nkey, nval, vals, P0<uint8_t>(marked), P0<int64_t>(tcount), nullptr, ek, nullptr, vb,
                        tkp, cur());
    at::Tensor tbase = exclusive_scan(tcount.narrow(0, 0, nt).contiguous());
    const int64_t T = nt > 0 ? tbase[nt].item<int64_t>() : 0;
    at::Tensor out = at::empty({T, 3}, opt(dev, at::kLong));
    if (T)
      k::trimr_emit_fixed(2, seg, m.nkey, nval, vals, P0<uint8_t>(marked), nullptr, P0<int64_t>(tbase), ek,
                          P0<int64_t>(out), vb, tkp, cur());
    return out;
  }
  const uint32_t* v = P0<uint32_t>(m.vdata);
  const uint64_t mask = (1ull << vb) - 1;
  std::vector<int64_t> rows;
  for (int64_t s = 0; s < m.nkey; ++s) {
    const int64_t vi = (int64_t)((uint64_t)ek[s] >> vb), vj = (int64_t)((uint64_t)ek[s] & mask);
    bool marker = false;
    for (int64_t j = seg[s]; j < seg[s + 1]; ++j) marker |= (int64_t)v[j] == vi;
    if (!marker) continue;
    for (int64_t j = seg[s]; j < seg[s + 1]; ++j)
      if ((int64_t)v[j] != vi) rows.insert(rows.end(), {(int64_t)v[j], vi, vj});
  }
  return at::tensor(rows, opt(at::kCPU, at::kLong)).view({-1, 3});
}

// Edge markers: an empty value (the reference's NULL) or, with fixed 8-byte
// values, the key's first vertex (tri.h) — the pipeline marks its edges
// that way so that the last collate moves one narrow fixed-width value column
at::Tensor trimr_emit(const KMV& m, int compact_vb) {
  const at::Device dev = m.seg.device();
  if (compact_vb > 0) return trimr_emit_compact(m, compact_vb);
  // fixed widths other than 8: only markers (0) or no marker at all
  if (!m.nkey || (m.vw >= 0 && m.vw != 8)) return at::empty({0, 3}, opt(dev, at::kLong));
  need(m.keys.kw == 16, "tri_find_mr emit: EDGE keys");
  const bool fixed = m.vw == 8;
  const int64_t* seg = P0<int64_t>(m.seg);
  const int64_t* voff = fixed ? nullptr : P0<int64_t>(m.voff);
  const int64_t* ek = P0<int64_t>(m.keys.kdata);
  if (dev.is_cuda() && fixed) {
    const int64_t nval = m.nval;
    const int64_t* vals = P0<int64_t>(m.vdata);
    at::Tensor marked = zeroed_bytes(m.nkey, dev);
    const int64_t nt = k::trimr_emit_tiles(nval);
    at::Tensor tcount = at::empty({std::max<int64_t>(nt, 1)}, opt(dev, at::kLong));
    at::Tensor tk = at::empty({nt + 1}, opt(dev, at::kLong));
    const int64_t* tkp = P0<int64_t>(tk);
    k::trimr_emit_tile_keys(seg, m.nkey, nval, P0<int64_t>(tk), cur());
    k::trimr_emit_fixed(0, seg, m.nkey, nval, vals, P0<uint8_t>(marked), nullptr, nullptr, ek, nullptr, 0, tkp, cur());
    k::trimr_emit_fixed(1, seg, m.nkey, nval, vals, P0<uint8_t>(marked), P0<int64_t>(tcount), nullptr, ek, nullptr, 0,
                        tkp, cur());
    at::Tensor tbase = exclusive_scan(tcount.narrow(0, 0, nt).contiguous());
    const int64_t T = nt > 0 ? tbase[nt].item<int64_t>() : 0;
    at::Tensor out = at::empty({T, 3}, opt(dev, at::kLong));
    if (T)
      k::trimr_emit_fixed(2, seg, m.nkey, nval, vals, P0<uint8_t>(marked), nullptr, P0<int64_t>(tbase), ek,
                          P0<int64_t>(out), 0, tkp, cur());
    return out;
  }
  if (dev.is_cuda()) {
    at::Tensor cnt = at::empty({m.nkey}, opt(dev, at::kLong));
    k::trimr_emit_count(seg, m.nkey, voff, fixed ? P0<int64_t>(m.vdata) : nullptr, ek, P0<int64_t>(cnt), cur());
    at::Tensor pos = exclusive_scan(cnt);
    const int64_t T = pos[m.nkey].item<int64_t>();
    at::Tensor out = at::empty({T, 3}, opt(dev, at::kLong));
    if (T) k::trimr_emit_write(seg, m.nkey, voff, P0<uint8_t>(m.vdata), ek, P0<int64_t>(pos), P0<int64_t>(out), cur());
    return out;
  }
  const uint8_t* vd = P0<uint8_t>(m.vdata);
  std::vector<int64_t> rows;
  int64_t s = 0;
  auto value = [&](int64_t j, int64_t* c) {  // false: the edge marker
    if (fixed) {
      std::memcpy(c, vd + 8 * j, 8);
      return *c != ek[2 * s];
    }
    if (voff[j + 1] - voff[j] != 8) return false;
    std::memcpy(c, vd + voff[j], 8);
    return true;
  };
  for (s = 0; s < m.nkey; ++s) {
    bool marker = false;
    int64_t c;
    for (int64_t j = seg[s]; j < seg[s + 1]; ++j) marker |= !value(j, &c);
    if (!marker) continue;
    for (int64_t j = seg[s]; j < seg[s + 1]; ++j)
      if (value(j, &c)) rows.insert(rows.end(), {c, ek[2 * s], ek[2 * s + 1]});
  }
  return at::tensor(rows, opt(at::kCPU, at::kLong)).view({-1, 3});
}

}  // namespace mrh
