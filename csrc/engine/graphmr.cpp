// sssp_mr / luby_find_mr callback ops (kernels: csrc/kernels/graphmr.hip) with
// host twins of identical semantics. The OINK commands sssp_mr and
// luby_find_mr (commands.cpp) run the reference's MapReduce pipelines
// (oink/sssp.cpp:88-152, oink/luby_find.cpp:53-97) with these as their batch
// callbacks.
#include "graphmr.h"

#include <ATen/hip/HIPContext.h>

#include <cstring>
#include <stdexcept>
#include <vector>

#include "../kernels/launch.h"

namespace mrh {

namespace {
at::TensorOptions opt(at::Device d, at::ScalarType t) { return at::TensorOptions().device(d).dtype(t); }
template <typename T>
T* P0(const at::Tensor& t) {
  return t.defined() && t.numel() ? reinterpret_cast<T*>(t.data_ptr()) : nullptr;
}
hipStream_t cur() { return at::hip::getCurrentHIPStream(); }
void need(bool c, const char* m) {
  if (!c) throw std::runtime_error(std::string("mrhip: ") + m);
}
constexpr double FLTMAX = 3.4028234663852886e+38;  // (double)FLT_MAX, DISTANCE()'s weight
int64_t ld8(const uint8_t* p) {
  int64_t v;
  std::memcpy(&v, p, 8);
  return v;
}
double ldd(const uint8_t* p) {
  double v;
  std::memcpy(&v, p, 8);
  return v;
}
int64_t bits(double d) {
  int64_t b;
  std::memcpy(&b, &d, 8);
  return b;
}
double dbl(int64_t b) {
  double d;
  std::memcpy(&d, &b, 8);
  return d;
}
at::Tensor longs(const std::vector<int64_t>& v, int64_t w) {
  at::Tensor t = at::empty({(int64_t)v.size()}, opt(at::kCPU, at::kLong));
  if (!v.empty()) std::memcpy(t.data_ptr(), v.data(), v.size() * 8);
  return w > 1 ? t.view({-1, w}) : t;
}
// int64 [n] filled with a byte pattern (0 or 0xFF) by the copy engine, no ATen kernel
at::Tensor filled(int64_t n, at::Device dev, int byte) {
  at::Tensor t = at::empty({std::max<int64_t>(n, 1)}, opt(dev, at::kLong));
  if (n > 0 && hipMemsetAsync(t.data_ptr(), byte, (size_t)n * 8, cur()) != hipSuccess)
    throw std::runtime_error("mrhip: hipMemsetAsync failed");
  return t;
}
// totals of exclusive scans (pos[n]) read with one sync
int64_t total(const at::Tensor& pos, int64_t n) {
  int64_t v = 0;
  if (n > 0) read_small(cur(), {{P0<int64_t>(pos) + n, &v, 8}});
  return v;
}
std::pair<int64_t, int64_t> totals(const at::Tensor& a, int64_t na, const at::Tensor& b, int64_t nb) {
  int64_t x = 0, y = 0;
  if (na > 0 && nb > 0) read_small(cur(), {{P0<int64_t>(a) + na, &x, 8}, {P0<int64_t>(b) + nb, &y, 8}});
  else {
    x = total(a, na);
    y = total(b, nb);
  }
  return {x, y};
}
// a value's [offset, length) for a fixed (vw >= 0) or variable KMV
struct Vals {
  const int64_t* voff;
  int64_t vw;
  const uint8_t* vd;
  int64_t beg(int64_t j) const { return voff ? voff[j] : j * vw; }
  int64_t len(int64_t j) const { return voff ? voff[j + 1] - voff[j] : vw; }
  const uint8_t* at(int64_t j) const { return vd + beg(j); }
};
Vals vals_of(const KMV& m) {
  return Vals{m.vw >= 0 ? nullptr : P0<int64_t>(m.voff), m.vw >= 0 ? (int64_t)m.vw : 0, P0<uint8_t>(m.vdata)};
}
at::Tensor keys64(const KMV& m, int kw, const char* what) {
  need(m.keys.kw == kw, what);
  return m.keys.kdata.view(at::kLong);
}
}  // namespace

// ====================================================================== sssp_mr

SsspPick ssspmr_pick(const KMV& m) {
  need(m.vw == 24 || m.vw < 0, "sssp_mr pick: 24-byte DISTANCE values");
  const at::Device dev = m.seg.device();
  at::Tensor keys = keys64(m, 8, "sssp_mr pick: 8-byte vertex keys");
  const int64_t* seg = P0<int64_t>(m.seg);
  const Vals V = vals_of(m);
  SsspPick r;
  r.dist = at::empty({m.nkey, 3}, opt(dev, at::kLong));
  if (dev.is_cuda()) {
    at::Tensor ch = at::empty({std::max<int64_t>(m.nkey, 1)}, opt(dev, at::kLong));
    k::sssp_pick(seg, m.nkey, V.voff, V.vw, V.vd, P0<int64_t>(r.dist), P0<int64_t>(ch), cur());
    at::Tensor pos = exclusive_scan(ch.narrow(0, 0, m.nkey));
    const int64_t c = total(pos, m.nkey);
    r.ckeys = at::empty({c}, opt(dev, at::kLong));
    r.cdist = at::empty({c, 3}, opt(dev, at::kLong));
    if (c)
      k::sssp_pick_emit(P0<int64_t>(keys), m.nkey, P0<int64_t>(r.dist), P0<int64_t>(pos), P0<int64_t>(r.ckeys),
                        P0<int64_t>(r.cdist), cur());
    return r;
  }
  int64_t* out = P0<int64_t>(r.dist);
  const int64_t* kp = P0<int64_t>(keys);
  std::vector<int64_t> ck, cd;
  for (int64_t s = 0; s < m.nkey; ++s) {
    const int64_t j0 = seg[s], j1 = seg[s + 1];
    int64_t pp = 0, sp;
    double pw = FLTMAX, sw;
    for (int64_t j = j0; j < j1; ++j)
      if (ld8(V.at(j) + 16)) {
        pp = ld8(V.at(j));
        pw = ldd(V.at(j) + 8);
      }
    if (j1 - j0 == 1) {
      pp = sp = ld8(V.at(j0));
      pw = sw = ldd(V.at(j0) + 8);
    } else {
      sp = pw < FLTMAX ? pp : 0;
      sw = pw < FLTMAX ? pw : FLTMAX;
      for (int64_t j = j0; j < j1; ++j) {
        const double w = ldd(V.at(j) + 8);
        if (w < sw) {
          sw = w;
          sp = ld8(V.at(j));
        }
      }
    }
    out[3 * s] = sp;
    out[3 * s + 1] = bits(sw);
    out[3 * s + 2] = 1;
    if (pp != sp || pw != sw) {
      ck.push_back(kp[s]);
      cd.insert(cd.end(), {sp, bits(sw), 1});
    }
  }
  r.ckeys = longs(ck, 1);
  r.cdist = longs(cd, 3);
  return r;
}

SsspRelax ssspmr_relax(const KMV& m) {
  const at::Device dev = m.seg.device();
  at::Tensor keys = keys64(m, 8, "sssp_mr relax: 8-byte vertex keys");
  at::Tensor voff = m.vw >= 0 ? fixed_offsets(m.nval, m.vw, dev) : m.voff.contiguous();
  const int64_t* seg = P0<int64_t>(m.seg);
  const int64_t* vo = P0<int64_t>(voff);
  const uint8_t* vd = P0<uint8_t>(m.vdata);
  const int64_t* kp = P0<int64_t>(keys);
  SsspRelax r;
  if (dev.is_cuda()) {
    at::Tensor best = filled(m.nkey, dev, 0xFF), idx = filled(m.nkey, dev, 0xFF), found = filled(m.nkey, dev, 0);
    auto* bu = reinterpret_cast<unsigned long long*>(P0<int64_t>(best));
    auto* iu = reinterpret_cast<unsigned long long*>(P0<int64_t>(idx));
    k::sssp_best(seg, m.nkey, vo, vd, m.nval, bu, iu, P0<int64_t>(found), cur());
    at::Tensor fe = at::empty({m.nval}, opt(dev, at::kLong)), fp = at::empty({m.nval}, opt(dev, at::kLong));
    k::sssp_relax_flags(seg, m.nkey, kp, vo, vd, m.nval, iu, P0<int64_t>(found), P0<int64_t>(fe), P0<int64_t>(fp),
                        cur());
    at::Tensor pe = exclusive_scan(fe), pp = exclusive_scan(fp);
    auto [ne, np] = totals(pe, m.nval, pp, m.nval);
    r.ekeys = at::empty({ne}, opt(dev, at::kLong));
    r.edges = at::empty({ne, 2}, opt(dev, at::kLong));
    r.pkeys = at::empty({np}, opt(dev, at::kLong));
    r.paths = at::empty({np, 3}, opt(dev, at::kLong));
    if (ne)
      k::sssp_relax_emit(seg, m.nkey, kp, vo, vd, m.nval, iu, P0<int64_t>(found), P0<int64_t>(pe), P0<int64_t>(pp),
                         P0<int64_t>(r.ekeys), P0<int64_t>(r.edges), P0<int64_t>(r.pkeys), P0<int64_t>(r.paths),
                         cur());
    return r;
  }
  std::vector<int64_t> ek, ev, pk, pv;
  for (int64_t s = 0; s < m.nkey; ++s) {
    bool found = false;
    int64_t sp = 0;
    double sw = FLTMAX;
    for (int64_t j = seg[s]; j < seg[s + 1]; ++j)
      if (vo[j + 1] - vo[j] == 24) {
        found = true;
        const double w = ldd(vd + vo[j] + 8);
        if (w < sw) {
          sw = w;
          sp = ld8(vd + vo[j]);
        }
      }
    for (int64_t j = seg[s]; j < seg[s + 1]; ++j) {
      if (vo[j + 1] - vo[j] != 16) continue;
      const int64_t v = ld8(vd + vo[j]), wb = ld8(vd + vo[j] + 8);
      ek.push_back(kp[s]);
      ev.insert(ev.end(), {v, wb});
      if (found && sp != v && v != kp[s]) {
        pk.push_back(v);
        pv.insert(pv.end(), {kp[s], bits(sw + dbl(wb)), 0});
      }
    }
  }
  r.ekeys = longs(ek, 1);
  r.edges = longs(ev, 2);
  r.pkeys = longs(pk, 1);
  r.paths = longs(pv, 3);
  return r;
}

// ====================================================================== luby_find_mr

namespace {
double luby_rand(int64_t v, int64_t seed) {  // srand48(v + seed); drand48()
  const uint64_t x0 = ((uint64_t)(uint32_t)(v + seed) << 16) | 0x330Eull;
  const uint64_t x1 = (0x5DEECE66Dull * x0 + 0xBull) & ((1ull << 48) - 1);
  return (double)x1 * 0x1p-48;
}
// per-key marks (graphmr.hip k_luby_mark's modes)
std::vector<char> luby_marks(const KMV& m, int mode) {
  const int64_t* seg = P0<int64_t>(m.seg);
  const Vals V = vals_of(m);
  std::vector<char> mk((size_t)m.nkey, 0);
  for (int64_t s = 0; s < m.nkey; ++s)
    for (int64_t j = seg[s]; j < seg[s + 1] && !mk[s]; ++j) {
      const int64_t l = V.len(j);
      mk[s] = mode == 0 ? ld8(V.at(j) + 16) == 0 : mode == 1 ? l > 16 : mode == 2 ? l == 16 : l > 0;
    }
  return mk;
}
at::Tensor dev_marks(const KMV& m, int mode) {
  at::Tensor mark = filled(m.nkey, m.seg.device(), 0);
  const Vals V = vals_of(m);
  k::luby_mark(P0<int64_t>(m.seg), m.nkey, V.voff, V.vw, V.vd, m.nval, mode, P0<int64_t>(mark), cur());
  return mark;
}
}  // namespace

at::Tensor lubymr_random(const at::Tensor& edges, int64_t seed) {
  at::Tensor e = edges.reshape({-1, 2}).to(at::kLong).contiguous();
  const int64_t n = e.size(0);
  const at::Device dev = e.device();
  if (dev.is_cuda()) {
    at::Tensor f = at::empty({n}, opt(dev, at::kLong));
    k::luby_nonloop(P0<int64_t>(e), n, P0<int64_t>(f), cur());
    at::Tensor pos = exclusive_scan(f);
    const int64_t c = total(pos, n);
    at::Tensor out = at::empty({c, 4}, opt(dev, at::kLong));
    if (c) k::luby_random(P0<int64_t>(e), n, seed, P0<int64_t>(pos), P0<int64_t>(out), cur());
    return out;
  }
  const int64_t* ep = P0<int64_t>(e);
  std::vector<int64_t> o;
  for (int64_t i = 0; i < n; ++i) {
    const int64_t vi = ep[2 * i], vj = ep[2 * i + 1];
    if (vi == vj) continue;
    o.insert(o.end(), {vi, bits(luby_rand(vi, seed)), vj, bits(luby_rand(vj, seed))});
  }
  return longs(o, 4);
}

std::pair<at::Tensor, at::Tensor> lubymr_edge_winner(const KMV& m) {
  const at::Device dev = m.seg.device();
  at::Tensor keys = keys64(m, 32, "luby_find_mr edge_winner: 32-byte ERAND keys");
  const int64_t* kp = P0<int64_t>(keys);
  if (dev.is_cuda()) {
    at::Tensor mark = dev_marks(m, 3);
    at::Tensor f = at::empty({m.nkey}, opt(dev, at::kLong));
    k::luby_key_flags(P0<int64_t>(mark), m.nkey, 0, P0<int64_t>(f), cur());
    at::Tensor pos = exclusive_scan(f);
    const int64_t c = total(pos, m.nkey);
    at::Tensor okey = at::empty({2 * c, 2}, opt(dev, at::kLong)), oval = at::empty({2 * c, 3}, opt(dev, at::kLong));
    if (c) k::luby_edge_emit(kp, m.nkey, P0<int64_t>(pos), P0<int64_t>(okey), P0<int64_t>(oval), cur());
    return {okey, oval};
  }
  std::vector<char> dead = luby_marks(m, 3);
  std::vector<int64_t> ok, ov;
  for (int64_t s = 0; s < m.nkey; ++s) {
    if (dead[s]) continue;
    const int64_t vi = kp[4 * s], bi = kp[4 * s + 1], vj = kp[4 * s + 2], bj = kp[4 * s + 3];
    const double ri = dbl(bi), rj = dbl(bj);
    const bool first = ri < rj || (!(rj < ri) && (uint64_t)vi < (uint64_t)vj);
    const int64_t wv = first ? vi : vj, wb = first ? bi : bj, lv = first ? vj : vi, lb = first ? bj : bi;
    ok.insert(ok.end(), {wv, wb, lv, lb});
    ov.insert(ov.end(), {lv, lb, 1, wv, wb, 0});
  }
  return {longs(ok, 2), longs(ov, 3)};
}

LubyVert lubymr_vert(const KMV& m, bool loser) {
  const at::Device dev = m.seg.device();
  at::Tensor keys = keys64(m, 16, "luby_find_mr vert: 16-byte VRAND keys");
  if (!loser) need(m.vw == 24 || m.vw < 0, "luby_find_mr vert_winner: 24-byte VFLAG values");
  const int64_t* kp = P0<int64_t>(keys);
  const int64_t* seg = P0<int64_t>(m.seg);
  const Vals V = vals_of(m);
  const int64_t want = loser ? 1 : 0;  // the mark value that sends a VFLAG
  LubyVert r;
  if (dev.is_cuda()) {
    at::Tensor mark = dev_marks(m, loser ? 1 : 0);
    at::Tensor f = at::empty({m.nval}, opt(dev, at::kLong));
    k::luby_value_flags(seg, m.nkey, V.voff, V.vw, P0<int64_t>(mark), m.nval, want, P0<int64_t>(f), cur());
    at::Tensor p24 = exclusive_scan(f);
    const int64_t n24 = total(p24, m.nval), n16 = m.nval - n24;
    r.k24 = at::empty({n24, 2}, opt(dev, at::kLong));
    r.v24 = at::empty({n24, 3}, opt(dev, at::kLong));
    r.k16 = at::empty({n16, 2}, opt(dev, at::kLong));
    r.v16 = at::empty({n16, 2}, opt(dev, at::kLong));
    k::luby_vert_emit(seg, m.nkey, kp, V.voff, V.vw, V.vd, m.nval, P0<int64_t>(p24), P0<int64_t>(r.k24),
                      P0<int64_t>(r.v24), P0<int64_t>(r.k16), P0<int64_t>(r.v16), cur());
    return r;
  }
  std::vector<char> mk = luby_marks(m, loser ? 1 : 0);
  std::vector<int64_t> k24, v24, k16, v16;
  for (int64_t s = 0; s < m.nkey; ++s)
    for (int64_t j = seg[s]; j < seg[s + 1]; ++j) {
      const int64_t u = ld8(V.at(j)), ub = ld8(V.at(j) + 8);
      if (mk[s] == want) {
        k24.insert(k24.end(), {u, ub});
        v24.insert(v24.end(), {kp[2 * s], kp[2 * s + 1], 0});
      } else {
        k16.insert(k16.end(), {u, ub});
        v16.insert(v16.end(), {kp[2 * s], kp[2 * s + 1]});
      }
    }
  r.k24 = longs(k24, 2);
  r.v24 = longs(v24, 3);
  r.k16 = longs(k16, 2);
  r.v16 = longs(v16, 2);
  return r;
}

LubyEmit lubymr_emit(const KMV& m) {
  const at::Device dev = m.seg.device();
  at::Tensor keys = keys64(m, 16, "luby_find_mr vert_emit: 16-byte VRAND keys");
  const int64_t* kp = P0<int64_t>(keys);
  const int64_t* seg = P0<int64_t>(m.seg);
  const Vals V = vals_of(m);
  LubyEmit r;
  if (dev.is_cuda()) {
    at::Tensor mark = dev_marks(m, 2);
    at::Tensor fk = at::empty({m.nkey}, opt(dev, at::kLong)), fv = at::empty({m.nval}, opt(dev, at::kLong));
    k::luby_key_flags(P0<int64_t>(mark), m.nkey, 0, P0<int64_t>(fk), cur());
    k::luby_value_flags(seg, m.nkey, V.voff, V.vw, nullptr, m.nval, 0, P0<int64_t>(fv), cur());
    at::Tensor pk = exclusive_scan(fk), pf = exclusive_scan(fv);
    auto [nmis, nf] = totals(pk, m.nkey, pf, m.nval);
    r.mis = at::empty({nmis}, opt(dev, at::kLong));
    r.kflag = at::empty({nf, 4}, opt(dev, at::kLong));
    r.knull = at::empty({m.nval - nf, 4}, opt(dev, at::kLong));
    r.fval = at::empty({nf}, opt(dev, at::kInt));
    if (nf && hipMemsetAsync(r.fval.data_ptr(), 0, (size_t)nf * 4, cur()) != hipSuccess)
      throw std::runtime_error("mrhip: hipMemsetAsync failed");
    if (nmis) k::luby_mis_emit(kp, m.nkey, P0<int64_t>(pk), P0<int64_t>(r.mis), cur());
    k::luby_edges_emit(seg, m.nkey, kp, V.voff, V.vw, V.vd, m.nval, P0<int64_t>(pf), P0<int64_t>(r.kflag),
                       P0<int64_t>(r.knull), cur());
    return r;
  }
  std::vector<char> has16 = luby_marks(m, 2);
  std::vector<int64_t> mis, kf, kn;
  for (int64_t s = 0; s < m.nkey; ++s) {
    const int64_t v = kp[2 * s], vb = kp[2 * s + 1];
    if (!has16[s]) mis.push_back(v);
    for (int64_t j = seg[s]; j < seg[s + 1]; ++j) {
      const int64_t u = ld8(V.at(j)), ub = ld8(V.at(j) + 8);
      const bool vfirst = (uint64_t)v < (uint64_t)u;
      std::vector<int64_t>& o = V.len(j) != 16 ? kf : kn;
      o.insert(o.end(), {vfirst ? v : u, vfirst ? vb : ub, vfirst ? u : v, vfirst ? ub : vb});
    }
  }
  r.mis = longs(mis, 1);
  r.kflag = longs(kf, 4);
  r.fval = at::zeros({r.kflag.size(0)}, opt(at::kCPU, at::kInt));
  r.knull = longs(kn, 4);
  return r;
}

}  // namespace mrh
