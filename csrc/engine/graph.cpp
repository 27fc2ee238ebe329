// Graph-iteration engine ops (PageRank plan execution) with CPU twins.
#include <ATen/hip/HIPContext.h>

#include <algorithm>
#include <cmath>
#include <stdexcept>

#include "../kernels/launch.h"
#include "kv.h"

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
// a kernel operand: defined, contiguous, of dtype st, on device d (checked on
// the host before any launch; the kernels reinterpret raw pointers)
void operand(const at::Tensor& t, at::ScalarType st, const at::Device& d, const char* what) {
  if (!t.defined() || t.scalar_type() != st || t.device() != d || !t.is_contiguous())
    throw std::runtime_error(std::string("mrhip: ") + what + ": expected a contiguous " + c10::toString(st) +
                             " tensor on " + d.str() +
                             (t.defined() ? std::string(", got ") + c10::toString(t.scalar_type()) + " on " +
                                                t.device().str() + (t.is_contiguous() ? "" : " (strided)")
                                          : std::string(", got an undefined tensor")));
}
}  // namespace

// out[g] = sum_{e in seg g} r[src[e]] * w[e]
void pr_contrib(const at::Tensor& seg, const at::Tensor& src, const at::Tensor& w, const at::Tensor& r,
                at::Tensor& out) {
  const int64_t ng = seg.numel() - 1, ne = src.numel();
  const bool weighted = w.defined() && w.numel() > 0;
  need(src.scalar_type() == at::kInt && r.scalar_type() == at::kFloat && (!weighted || w.scalar_type() == at::kFloat),
       "pr_contrib dtypes");
  need(out.numel() >= ng, "pr_contrib out too small");
  if (ng <= 0) return;
  if (seg.is_cuda()) {
    at::Tensor scratch = at::empty({(int64_t)k::pr_scratch_bytes(ne)}, opt(seg.device(), at::kByte));
    k::pr_contrib(P0<int64_t>(seg), ng, ne, P0<int32_t>(src), weighted ? P0<float>(w) : nullptr, P0<float>(r),
                  P0<float>(out), P0<void>(scratch), cur());
    return;
  }
  const int64_t* sg = P0<int64_t>(seg);
  const int32_t* s = P0<int32_t>(src);
  const float* wp = weighted ? P0<float>(w) : nullptr;
  const float* rp = P0<float>(r);
  float* o = P0<float>(out);
  for (int64_t g = 0; g < ng; ++g) {
    float acc = 0.f;
    for (int64_t e = sg[g]; e < sg[g + 1]; ++e) acc += wp ? rp[s[e]] * wp[e] : rp[s[e]];
    o[g] = acc;
  }
}

// acc[vid[g]] = sum_{i in seg g} recv[perm[i]]   (acc must be pre-zeroed)
void pr_combine(const at::Tensor& seg, const at::Tensor& perm, const at::Tensor& recv, const at::Tensor& vid,
                at::Tensor& acc) {
  const int64_t ng = seg.numel() - 1, nr = perm.numel();
  const at::Device d = seg.device();
  operand(seg, at::kLong, d, "plan_combine seg");
  operand(perm, at::kInt, d, "plan_combine perm");
  operand(vid, at::kInt, d, "plan_combine vid");
  operand(recv, recv.scalar_type(), d, "plan_combine recv");
  operand(acc, recv.scalar_type(), d, "plan_combine acc (recv dtype)");
  need(ng <= 0 || vid.numel() >= ng, "plan_combine: one vid per group");
  if (ng <= 0) return;
  if (seg.is_cuda()) {
    at::Tensor grp = at::empty({ng}, opt(seg.device(), at::kFloat));
    at::Tensor scratch = at::empty({(int64_t)k::pr_scratch_bytes(nr)}, opt(seg.device(), at::kByte));
    k::pr_combine(P0<int64_t>(seg), ng, nr, P0<int32_t>(perm), P0<float>(recv), P0<int32_t>(vid), P0<float>(grp),
                  P0<float>(acc), P0<void>(scratch), cur());
    return;
  }
  const int64_t* sg = P0<int64_t>(seg);
  const int32_t* pp = P0<int32_t>(perm);
  const float* rv = P0<float>(recv);
  const int32_t* vp = P0<int32_t>(vid);
  float* a = P0<float>(acc);
  for (int64_t g = 0; g < ng; ++g) {
    float x = 0.f;
    for (int64_t i = sg[g]; i < sg[g + 1]; ++i) x += rv[pp[i]];
    a[vp[g]] = x;
  }
}

void scatter_f32(const at::Tensor& v, const at::Tensor& idx, at::Tensor& out) {
  const int64_t n = v.numel();
  if (v.is_cuda()) {
    k::scatter_f32(P0<float>(v), P0<int32_t>(idx), n, P0<float>(out), cur());
    return;
  }
  const float* vp = P0<float>(v);
  const int32_t* ip = P0<int32_t>(idx);
  float* o = P0<float>(out);
  for (int64_t i = 0; i < n; ++i) o[ip[i]] = vp[i];
}

// r_new = base + alpha*(acc + dmass/N); returns device double[2] = {sum|r_new - r|, dangling mass of r_new}
at::Tensor pr_update(const at::Tensor& acc, const at::Tensor& r, at::Tensor& rn, const at::Tensor& dangling,
                     double base, double alpha, const at::Tensor& dmass, double invN, const at::Tensor& invdeg,
                     at::Tensor& cout) {
  const int64_t n = r.numel();
  const bool wc = invdeg.defined() && invdeg.numel() > 0;
  if (r.is_cuda()) {
    // the kernel moves 16 bytes per access and zeroes acc behind its read
    auto al = [](const at::Tensor& t) { return reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0 && t.is_contiguous(); };
    need(acc.numel() >= n && rn.numel() >= n && dangling.numel() >= n && al(acc) && al(r) && al(rn) &&
             reinterpret_cast<uintptr_t>(dangling.data_ptr()) % 4 == 0 && (!wc || (al(invdeg) && al(cout))),
         "pr_update: contiguous 16-byte-aligned float columns of n entries (dangling 4-byte aligned)");
    int nb = k::pr_update_blocks(n);
    at::Tensor part = at::empty({nb, 2}, opt(r.device(), at::kDouble));
    k::pr_update(P0<float>(acc), P0<float>(r), P0<float>(rn), P0<uint8_t>(dangling), n, (float)base, (float)alpha,
                 P0<double>(dmass), invN, wc ? P0<float>(invdeg) : nullptr, wc ? P0<float>(cout) : nullptr,
                 P0<double>(part), cur());
    return part.sum(0);
  }
  const float* a = P0<float>(acc);
  const float* rp = P0<float>(r);
  float* o = P0<float>(rn);
  const uint8_t* dg = P0<uint8_t>(dangling);
  const float* idg = wc ? P0<float>(invdeg) : nullptr;
  float* co = wc ? P0<float>(cout) : nullptr;
  const float dterm = (float)(dmass.to(at::kCPU).item<double>() * invN);
  double d = 0, dm = 0;
  float* az = P0<float>(acc);
  for (int64_t i = 0; i < n; ++i) {
    float x = (float)base + (float)alpha * (a[i] + dterm);
    az[i] = 0.f;  // as the kernel: acc is zeroed behind its read
    o[i] = x;
    if (co) co[i] = x * idg[i];
    d += std::fabs((double)x - (double)rp[i]);
    if (dg[i]) dm += x;
  }
  return at::tensor({d, dm}, opt(at::kCPU, at::kDouble));
}

namespace {
int dcode(const at::Tensor& t) {
  switch (t.scalar_type()) {
    case at::kLong: return 1;
    case at::kFloat: return 2;
    case at::kDouble: return 3;
    default: throw std::runtime_error("mrhip plan: dtype must be int64, float32 or float64");
  }
}
template <typename T>
T red(int op, T a, T b) {
  return op == 0 ? a + b : op == 1 ? (b < a ? b : a) : (b > a ? b : a);
}
}  // namespace

// out[g] = OP_{e in seg g} (x[src[e]] (+ w[e]))
void plan_gather_reduce(const at::Tensor& seg, const at::Tensor& src, const at::Tensor& x, const at::Tensor& w,
                        int64_t op, at::Tensor& out) {
  const int64_t ng = seg.numel() - 1, ne = src.numel();
  const bool hw = w.defined() && w.numel() > 0;
  const at::Device d = seg.device();
  operand(seg, at::kLong, d, "plan_gather_reduce seg");
  operand(src, at::kInt, d, "plan_gather_reduce src");
  operand(x, x.scalar_type(), d, "plan_gather_reduce x");
  if (hw) operand(w, x.scalar_type(), d, "plan_gather_reduce weights (value dtype)");
  need(!hw || w.numel() == ne, "plan_gather_reduce: one weight per source id");
  operand(out, x.scalar_type(), d, "plan_gather_reduce out (value dtype)");
  need(out.numel() >= ng, "plan_gather_reduce: out smaller than the group count");
  if (ng <= 0) return;
  if (seg.is_cuda()) {
    at::Tensor scratch = at::empty({(int64_t)k::plan_scratch_bytes(ne)}, opt(seg.device(), at::kByte));
    k::plan_gather_reduce(dcode(x), P0<int64_t>(seg), ng, ne, P0<int32_t>(src), x.data_ptr(),
                          hw ? w.data_ptr() : nullptr, (int)op, out.data_ptr(), P0<void>(scratch), cur());
    return;
  }
  AT_DISPATCH_ALL_TYPES(x.scalar_type(), "plan_gather_reduce", [&] {
    const int64_t* sg = P0<int64_t>(seg);
    const int32_t* s = P0<int32_t>(src);
    const scalar_t* xp = x.data_ptr<scalar_t>();
    const scalar_t* wp = hw ? w.data_ptr<scalar_t>() : nullptr;
    scalar_t* o = out.data_ptr<scalar_t>();
    for (int64_t g = 0; g < ng; ++g) {
      scalar_t acc = xp[s[sg[g]]] + (wp ? wp[sg[g]] : scalar_t(0));
      for (int64_t e = sg[g] + 1; e < sg[g + 1]; ++e) acc = red<scalar_t>((int)op, acc, xp[s[e]] + (wp ? wp[e] : scalar_t(0)));
      o[g] = acc;
    }
  });
}

// acc[vid[g]] = OP_{i in seg g} recv[perm[i]]
void plan_combine(const at::Tensor& seg, const at::Tensor& perm, const at::Tensor& recv, const at::Tensor& vid,
                  int64_t op, at::Tensor& acc) {
  const int64_t ng = seg.numel() - 1, nr = perm.numel();
  if (ng <= 0) return;
  if (seg.is_cuda()) {
    at::Tensor grp = at::empty({ng}, recv.options());
    at::Tensor scratch = at::empty({(int64_t)k::plan_scratch_bytes(nr)}, opt(seg.device(), at::kByte));
    k::plan_combine(dcode(recv), P0<int64_t>(seg), ng, nr, P0<int32_t>(perm), recv.data_ptr(), P0<int32_t>(vid),
                    (int)op, grp.data_ptr(), acc.data_ptr(), P0<void>(scratch), cur());
    return;
  }
  AT_DISPATCH_ALL_TYPES(recv.scalar_type(), "plan_combine", [&] {
    const int64_t* sg = P0<int64_t>(seg);
    const int32_t* pp = P0<int32_t>(perm);
    const scalar_t* rv = recv.data_ptr<scalar_t>();
    const int32_t* vp = P0<int32_t>(vid);
    scalar_t* a = acc.data_ptr<scalar_t>();
    for (int64_t g = 0; g < ng; ++g) {
      scalar_t x = rv[pp[sg[g]]];
      for (int64_t i = sg[g] + 1; i < sg[g + 1]; ++i) x = red<scalar_t>((int)op, x, rv[pp[i]]);
      a[vp[g]] = x;
    }
  });
}

SegIndex seg_index(const at::Tensor& seg, int64_t nval) {
  SegIndex ix;
  need(seg.is_cuda(), "seg_index: device plans only");
  const at::Device d = seg.device();
  ix.nval = nval;
  ix.H = at::empty({k::ws_words(nval)}, opt(d, at::kInt));
  ix.wbase = at::empty({std::max<int64_t>(k::ws_waves(nval), 1)}, opt(d, at::kLong));
  ix.scratch = at::empty({(int64_t)k::ws_scratch_bytes(nval)}, opt(d, at::kByte));
  k::ws_index(P0<int64_t>(seg), seg.numel() - 1, nval, P0<uint32_t>(ix.H), P0<int64_t>(ix.wbase), cur());
  return ix;
}

SegIndex seg_index(const at::Tensor& seg, int64_t nval, const at::Tensor& heads) {
  SegIndex ix;
  need(seg.is_cuda() && heads.device() == seg.device(), "seg_index: device plans only");
  need(heads.scalar_type() == at::kInt && heads.numel() == k::ws_words(nval), "seg_index: heads must be ws_words(nval) words");
  const at::Device d = seg.device();
  ix.nval = nval;
  ix.H = heads;
  ix.wbase = at::empty({std::max<int64_t>(k::ws_waves(nval), 1)}, opt(d, at::kLong));
  ix.scratch = at::empty({(int64_t)k::ws_scratch_bytes(nval)}, opt(d, at::kByte));
  k::ws_bases(P0<int64_t>(seg), seg.numel() - 1, nval, P0<int64_t>(ix.wbase), cur());
  return ix;
}

void seg_gather_reduce(const SegIndex& ix, const at::Tensor& src, const at::Tensor& x, const at::Tensor& w, int64_t op,
                       at::Tensor& out) {
  const bool hw = w.defined() && w.numel() > 0;
  need(ix.defined() && src.numel() == ix.nval && src.scalar_type() == at::kInt && src.is_contiguous(),
       "seg_gather_reduce: src must be the plan's contiguous int32 source ids");
  need(reinterpret_cast<uintptr_t>(src.data_ptr()) % 16 == 0, "seg_gather_reduce: src must be 16-byte aligned");
  need(!hw || (w.scalar_type() == x.scalar_type() && w.numel() == ix.nval), "seg_gather_reduce: weights");
  need(out.scalar_type() == x.scalar_type() && x.is_contiguous() && out.is_contiguous(), "seg_gather_reduce: out");
  k::ws_gather_reduce(dcode(x), P0<uint32_t>(ix.H), P0<int64_t>(ix.wbase), ix.nval, P0<int32_t>(src), x.data_ptr(),
                      hw ? w.data_ptr() : nullptr, (int)op, out.data_ptr(), P0<void>(ix.scratch), cur(),
                      ix.sched.defined() ? P0<int32_t>(ix.sched) : nullptr, ix.slen, x.numel());
}

// all neighbour pairs per group: returns (edges [W,2] int64 (min,max), centre [W])
namespace {
struct WedgeScan {
  // exclusive scan of C(d,2): over every group (ng + 1 entries) on the CPU;
  // on the device over the groups with a wedge only (gidx, ngw + 1 entries)
  at::Tensor wscan, gidx;
  int64_t ng = 0, ngw = 0, nw = 0;
};
WedgeScan wedge_scan(const at::Tensor& seg, const at::Tensor& nb, const at::Tensor& centre) {
  WedgeScan w;
  w.ng = seg.numel() - 1;
  need(w.ng >= 0, "wedges: seg holds ngroups + 1 offsets");
  operand(seg, at::kLong, seg.device(), "wedges seg");
  operand(nb, at::kLong, seg.device(), "wedges neighbours");
  operand(centre, at::kLong, seg.device(), "wedges centre");
  need(centre.numel() >= w.ng, "wedges: one centre per group");
  at::Tensor d = seg.narrow(0, 1, w.ng) - seg.narrow(0, 0, w.ng);
  at::Tensor cnt = at::floor_divide(d * (d - 1), 2);
  if (seg.is_cuda()) {
    w.gidx = mask_indices(d >= 2);
    w.ngw = w.gidx.numel();
    cnt = cnt.index_select(0, w.gidx);
  }
  w.wscan = exclusive_scan(cnt.contiguous());
  const int64_t nscan = seg.is_cuda() ? w.ngw : w.ng;
  w.nw = nscan > 0 ? w.wscan[nscan].item<int64_t>() : 0;
  return w;
}
// wedges [w0, w1) of the scan
std::pair<at::Tensor, at::Tensor> wedge_range(const at::Tensor& seg, const WedgeScan& ws, const at::Tensor& nb,
                                              const at::Tensor& centre, int64_t w0, int64_t w1) {
  const int64_t n = w1 - w0;
  at::Tensor oe = at::empty({n, 2}, nb.options());
  at::Tensor oc = at::empty({n}, nb.options());
  if (n == 0) return {oe, oc};
  if (seg.is_cuda()) {
    at::Tensor tg = at::empty({k::wedge_tiles(n) + 1}, nb.options());
    k::wedges(P0<int64_t>(seg), P0<int64_t>(ws.gidx), P0<int64_t>(ws.wscan), ws.ngw, P0<int64_t>(nb),
              P0<int64_t>(centre), w0, n, P0<int64_t>(oe), P0<int64_t>(oc), P0<int64_t>(tg), cur());
    return {oe, oc};
  }
  const int64_t* sg = P0<int64_t>(seg);
  const int64_t* sc = P0<int64_t>(ws.wscan);
  const int64_t* nbp = P0<int64_t>(nb);
  const int64_t* c = P0<int64_t>(centre);
  int64_t* e = P0<int64_t>(oe);
  int64_t* co = P0<int64_t>(oc);
  // first wedge: its group, then (j, k) by walking the rows of its triangle
  int64_t g = std::upper_bound(sc, sc + ws.ng, w0) - sc - 1, t = w0 - sc[g], j = 0;
  int64_t d = sg[g + 1] - sg[g];
  while (t >= d - 1 - j) t -= d - 1 - j++;
  int64_t k2 = j + 1 + t;
  for (int64_t i = 0; i < n; ++i) {
    const uint64_t a = (uint64_t)nbp[sg[g] + j], b = (uint64_t)nbp[sg[g] + k2];
    e[2 * i] = (int64_t)(a < b ? a : b);
    e[2 * i + 1] = (int64_t)(a < b ? b : a);
    co[i] = c[g];
    if (++k2 < d) continue;
    k2 = ++j + 1;
    if (k2 < d) continue;
    do d = ++g < ws.ng ? sg[g + 1] - sg[g] : 2;  // next group with a wedge
    while (d < 2);
    j = 0, k2 = 1;
  }
  return {oe, oc};
}
}  // namespace

std::pair<at::Tensor, at::Tensor> wedges(const at::Tensor& seg, const at::Tensor& nb, const at::Tensor& centre) {
  const WedgeScan ws = wedge_scan(seg, nb, centre);
  return wedge_range(seg, ws, nb, centre, 0, ws.nw);
}

void for_each_wedge_chunk_compact(const at::Tensor& seg, const at::Tensor& nb, const at::Tensor& centre,
                                  int64_t max_w, int vb,
                                  const std::function<void(const at::Tensor&, const at::Tensor&)>& fn) {
  need(vb > 0 && vb <= 32, "wedges (compact): vertex bits in (0, 32]");
  const WedgeScan ws = wedge_scan(seg, nb, centre);
  const int64_t step = max_w > 0 ? max_w : std::max<int64_t>(ws.nw, 1);
  for (int64_t w0 = 0; w0 < ws.nw; w0 += step) {
    const int64_t n = std::min(ws.nw, w0 + step) - w0;
    if (seg.is_cuda()) {
      at::Tensor key = at::empty({n}, nb.options());
      at::Tensor c = at::empty({n}, nb.options().dtype(at::kInt));
      at::Tensor tg = at::empty({k::wedge_tiles(n) + 1}, nb.options());
      k::wedges_compact(P0<int64_t>(seg), P0<int64_t>(ws.gidx), P0<int64_t>(ws.wscan), ws.ngw, P0<int64_t>(nb),
                        P0<int64_t>(centre), w0, n, vb, P0<int64_t>(key), P0<uint32_t>(c), P0<int64_t>(tg), cur());
      fn(key, c);
    } else {
      auto r = wedge_range(seg, ws, nb, centre, w0, w0 + n);
      fn(at::bitwise_or(at::bitwise_left_shift(r.first.select(1, 0), vb), r.first.select(1, 1)), r.second.to(at::kInt));
    }
  }
}

void for_each_wedge_chunk(const at::Tensor& seg, const at::Tensor& nb, const at::Tensor& centre, int64_t max_w,
                          const std::function<void(const at::Tensor&, const at::Tensor&)>& fn) {
  const WedgeScan ws = wedge_scan(seg, nb, centre);
  const int64_t step = max_w > 0 ? max_w : std::max<int64_t>(ws.nw, 1);
  for (int64_t w0 = 0; w0 < ws.nw; w0 += step) {
    auto r = wedge_range(seg, ws, nb, centre, w0, std::min(ws.nw, w0 + step));
    fn(r.first, r.second);
  }
}

}  // namespace mrh
