// Graph-iteration engine ops (PageRank plan execution) with CPU twins.
#include <ATen/hip/HIPContext.h>

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
  for (int64_t i = 0; i < n; ++i) {
    float x = (float)base + (float)alpha * (a[i] + dterm);
    o[i] = x;
    if (co) co[i] = x * idg[i];
    d += std::fabs((double)x - (double)rp[i]);
    if (dg[i]) dm += x;
  }
  return at::tensor({d, dm}, opt(at::kCPU, at::kDouble));
}

}  // namespace mrh
