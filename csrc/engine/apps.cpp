// Application-level fused ops built on the engine (device epilogues).
#include <ATen/hip/HIPContext.h>

#include <cstring>
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
}  // namespace

// InvertedIndex reduce (reference cuda/InvertedIndex.cu:463-513): for every
// unique URL write "url\tname1 name2 ... \n" where names[i] is the file name
// of doc id i. Returns the formatted bytes (on the KMV's device).
at::Tensor inverted_index_format(const KMV& kmv, const at::Tensor& names, const at::Tensor& name_off) {
  const at::Device dev = kmv.keys.device();
  if (kmv.keys.kw >= 0) throw std::runtime_error("inverted_index_format: keys must be variable-length strings");
  if (kmv.vw != 4) throw std::runtime_error("inverted_index_format: values must be int32 doc ids");
  const int64_t nseg = kmv.nkey, nval = kmv.nval;
  at::Tensor nm = names.to(dev), no = name_off.to(dev, at::kLong);
  if (nseg == 0) return at::empty({0}, opt(dev, at::kByte));
  if (dev.is_cuda()) {
    hipStream_t s = at::hip::getCurrentHIPStream();
    at::Tensor lenv = at::empty({nval}, opt(dev, at::kInt));
    k::ii_value_len(P0<int32_t>(kmv.vdata), nval, P0<int64_t>(no), P0<int32_t>(lenv), s);
    at::Tensor cv = exclusive_scan(lenv);
    at::Tensor lens = at::empty({nseg}, opt(dev, at::kInt));
    k::ii_key_len(P0<int64_t>(kmv.keys.koff), nseg, P0<int32_t>(lens), s);
    at::Tensor cs = exclusive_scan(lens);
    int64_t total = cs[nseg].item<int64_t>() + cv[nval].item<int64_t>();
    at::Tensor out = at::empty({total}, opt(dev, at::kByte));
    k::ii_write(P0<uint8_t>(kmv.keys.kdata), P0<int64_t>(kmv.keys.koff), P0<int32_t>(kmv.vdata), nval,
                P0<int64_t>(kmv.seg), nseg, P0<int64_t>(cv), P0<int64_t>(cs), P0<uint8_t>(nm), P0<int64_t>(no),
                P0<uint8_t>(out), s);
    return out;
  }
  const uint8_t* kd = P0<uint8_t>(kmv.keys.kdata);
  const int64_t* ko = P0<int64_t>(kmv.keys.koff);
  const int32_t* v = P0<int32_t>(kmv.vdata);
  const int64_t* sg = P0<int64_t>(kmv.seg);
  const uint8_t* nmp = P0<uint8_t>(nm);
  const int64_t* nop = P0<int64_t>(no);
  std::string outs;
  for (int64_t s = 0; s < nseg; ++s) {
    outs.append((const char*)kd + ko[s], ko[s + 1] - ko[s] - 1);
    outs.push_back('\t');
    for (int64_t i = sg[s]; i < sg[s + 1]; ++i) {
      outs.append((const char*)nmp + nop[v[i]], nop[v[i] + 1] - nop[v[i]]);
      outs.push_back(' ');
    }
    outs.push_back('\n');
  }
  return at::from_blob((void*)outs.data(), {(int64_t)outs.size()}, opt(at::kCPU, at::kByte)).clone();
}

}  // namespace mrh
