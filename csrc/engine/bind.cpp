// Python bindings of the native engine (module gpu_mapreduce_amd._C).
//
// Exposes the device KV/KMV containers, the engine ops, the process-group
// shuffle, the native host-side KeyValue builder used by user callbacks
// (MR-MPI's KeyValue::add, reference src/keyvalue.cpp:343-643) and the
// host iteration loops that drive Python reduce/scan/map-over-MR callbacks
// (reference src/mapreduce.cpp:1769-1867,1933-2065,1560-1642).
#include <torch/extension.h>
#include <torch/csrc/distributed/c10d/ProcessGroup.hpp>

#include <cstring>
#include <string>

#include "kv.h"

namespace py = pybind11;
using namespace mrh;
using PG = c10::intrusive_ptr<c10d::ProcessGroup>;

namespace {

PG as_pg(py::object o) {
  if (o.is_none()) return PG();
  return o.cast<PG>();
}

// Native append-only builder behind the callback-facing KeyValue object.
// Host-emitted pairs accumulate in contiguous byte arrays; device batches
// (KV objects produced by kernels or torch ops) are kept as chunks, in order,
// so a map callback can mix both without a host round trip for device data.
class HostKV {
 public:
  explicit HostKV(std::string device) : dev_(device) { reset_host(); }

  void add(const std::string& k, const std::string& v) {
    kd_.append(k);
    vd_.append(v);
    note(k.size(), v.size());
    koff_.push_back((int64_t)kd_.size());
    voff_.push_back((int64_t)vd_.size());
    ++nh_;
  }
  // n fixed-size keys / values packed in two byte strings (MR-MPI add(n,k,kb,v,vb))
  void add_fixed(int64_t n, const std::string& ks, int64_t kb, const std::string& vs, int64_t vb) {
    if ((int64_t)ks.size() != n * kb || (int64_t)vs.size() != n * vb) throw std::runtime_error("add_multi: size mismatch");
    for (int64_t i = 0; i < n; ++i) {
      kd_.append(ks, i * kb, kb);
      vd_.append(vs, i * vb, vb);
      note(kb, vb);
      koff_.push_back((int64_t)kd_.size());
      voff_.push_back((int64_t)vd_.size());
    }
    nh_ += n;
  }
  // n variable-size keys/values with per-pair byte counts (MR-MPI add(n,k,kb[],v,vb[]))
  void add_var(const std::string& ks, const std::vector<int64_t>& kb, const std::string& vs,
               const std::vector<int64_t>& vb) {
    if (kb.size() != vb.size()) throw std::runtime_error("add_multi: length lists differ");
    int64_t ka = 0, va = 0;
    for (size_t i = 0; i < kb.size(); ++i) {
      kd_.append(ks, ka, kb[i]);
      vd_.append(vs, va, vb[i]);
      ka += kb[i];
      va += vb[i];
      note(kb[i], vb[i]);
      koff_.push_back((int64_t)kd_.size());
      voff_.push_back((int64_t)vd_.size());
    }
    nh_ += (int64_t)kb.size();
  }
  void add_kv(const KV& kv) {
    flush();
    chunks_.push_back(kv);
  }
  int64_t size() const {
    int64_t n = nh_;
    for (auto& c : chunks_) n += c.n;
    return n;
  }
  KV finish() {
    flush();
    at::Device d(dev_);
    KV out = concat(chunks_, d);
    chunks_.clear();
    return out;
  }

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
  void flush() {
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
    chunks_.push_back(kv_to(kv, at::Device(dev_)));
    reset_host();
  }
  std::string dev_;
  std::string kd_, vd_;
  std::vector<int64_t> koff_, voff_;
  int64_t nh_ = 0;
  int kw_ = -2, vw_ = -2;
  std::vector<KV> chunks_;
};

// ---------------------------------------------------------------- host iteration helpers
struct HostCol {
  at::Tensor data, off;
  int w;
  const uint8_t* d() const { return data.numel() ? data.data_ptr<uint8_t>() : nullptr; }
  int64_t a(int64_t i) const { return w >= 0 ? i * w : off.data_ptr<int64_t>()[i]; }
  int64_t len(int64_t i) const { return w >= 0 ? w : off.data_ptr<int64_t>()[i + 1] - off.data_ptr<int64_t>()[i]; }
  py::bytes get(int64_t i) const { return py::bytes((const char*)d() + a(i), (size_t)len(i)); }
};
HostCol host_col(const at::Tensor& data, const at::Tensor& off, int w) {
  HostCol c;
  c.data = data.to(at::kCPU).contiguous();
  c.off = (w < 0) ? off.to(at::kCPU).contiguous() : at::Tensor();
  c.w = w;
  return c;
}

// fn(i, key, value) for every pair
void kv_iter(const KV& kv, py::function fn) {
  HostCol k = host_col(kv.kdata, kv.koff, kv.kw), v = host_col(kv.vdata, kv.voff, kv.vw);
  for (int64_t i = 0; i < kv.n; ++i) fn(i, k.get(i), v.get(i));
}
// fn(key, [values]) for every KMV pair
void kmv_iter(const KMV& kmv, py::function fn) {
  HostCol k = host_col(kmv.keys.kdata, kmv.keys.koff, kmv.keys.kw), v = host_col(kmv.vdata, kmv.voff, kmv.vw);
  at::Tensor seg = kmv.seg.to(at::kCPU).contiguous();
  const int64_t* s = seg.data_ptr<int64_t>();
  for (int64_t i = 0; i < kmv.nkey; ++i) {
    py::list vals(s[i + 1] - s[i]);
    for (int64_t j = s[i]; j < s[i + 1]; ++j) vals[j - s[i]] = v.get(j);
    fn(k.get(i), vals);
  }
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "gpu_mapreduce_amd native engine (HIP/CDNA4 kernels + ATen + c10d)";

  py::class_<KV>(m, "KV")
      .def(py::init<>())
      .def_readwrite("kdata", &KV::kdata)
      .def_readwrite("koff", &KV::koff)
      .def_readwrite("vdata", &KV::vdata)
      .def_readwrite("voff", &KV::voff)
      .def_readwrite("n", &KV::n)
      .def_readwrite("kw", &KV::kw)
      .def_readwrite("vw", &KV::vw)
      .def("nbytes", &KV::nbytes)
      .def("key_bytes", &KV::key_bytes)
      .def("value_bytes", &KV::value_bytes)
      .def("to", [](const KV& kv, const std::string& d) { return kv_to(kv, at::Device(d)); });

  py::class_<KMV>(m, "KMV")
      .def(py::init<>())
      .def_readwrite("keys", &KMV::keys)
      .def_readwrite("vdata", &KMV::vdata)
      .def_readwrite("voff", &KMV::voff)
      .def_readwrite("vw", &KMV::vw)
      .def_readwrite("seg", &KMV::seg)
      .def_readwrite("nkey", &KMV::nkey)
      .def_readwrite("nval", &KMV::nval)
      .def("nbytes", &KMV::nbytes);

  py::class_<ConvertStats>(m, "ConvertStats")
      .def(py::init<>())
      .def_readonly("passes", &ConvertStats::passes)
      .def_readonly("collisions", &ConvertStats::collisions)
      .def_readonly("exact", &ConvertStats::exact);
  py::class_<ShuffleStats>(m, "ShuffleStats")
      .def(py::init<>())
      .def_readwrite("send_bytes", &ShuffleStats::send_bytes)
      .def_readwrite("recv_bytes", &ShuffleStats::recv_bytes)
      .def_readwrite("send_pairs", &ShuffleStats::send_pairs)
      .def_readwrite("recv_pairs", &ShuffleStats::recv_pairs)
      .def_readwrite("seconds", &ShuffleStats::seconds);

  py::class_<HostKV>(m, "HostKV")
      .def(py::init<std::string>())
      .def("add", &HostKV::add)
      .def("add_fixed", &HostKV::add_fixed)
      .def("add_var", &HostKV::add_var)
      .def("add_kv", &HostKV::add_kv)
      .def("size", &HostKV::size)
      .def("finish", &HostKV::finish);

  m.def("empty_kv", [](const std::string& d, int kw, int vw) { return empty_kv(at::Device(d), kw, vw); });
  m.def(
      "make_kv",
      [](at::Tensor kd, c10::optional<at::Tensor> ko, at::Tensor vd, c10::optional<at::Tensor> vo, int64_t n,
         const std::string& d) { return make_kv(kd, ko, vd, vo, n, at::Device(d)); },
      py::arg("kdata"), py::arg("koff"), py::arg("vdata"), py::arg("voff"), py::arg("n"), py::arg("device"));
  m.def("concat", [](const std::vector<KV>& parts, const std::string& d) { return concat(parts, at::Device(d)); });
  m.def("to_var_keys", &to_var_keys);
  m.def("to_var_values", &to_var_values);
  m.def("exclusive_scan", &exclusive_scan);
  m.def("radix_sort_pairs", &radix_sort_pairs);
  m.def("hash32_keys", &hash32_keys);
  m.def("hash64_keys", &hash64_keys);
  m.def("gather", &mrh::gather);
  m.def(
      "convert",
      [](const KV& kv, int force_hash_bits) {
        ConvertStats st;
        KMV r = convert(kv, &st, force_hash_bits);
        return std::make_pair(r, st);
      },
      py::arg("kv"), py::arg("force_hash_bits") = 64);
  m.def("clone", &mrh::clone);
  m.def("collapse", &mrh::collapse);
  m.def("reduce_builtin", &reduce_builtin);
  m.def("sort_kv", &sort_kv);
  m.def("sort_multivalues", &sort_multivalues);
  m.def("expand", &mrh::expand);
  m.def("partition_dest", [](const KV& kv, int P) {
    at::Tensor c;
    at::Tensor d = partition_dest(kv, P, &c);
    return std::make_pair(d, c);
  });
  m.def("exchange", [](const KV& kv, const at::Tensor& dest, py::object pg) {
    ShuffleStats st;
    KV r = exchange(kv, dest, as_pg(pg), &st);
    return std::make_pair(r, st);
  });
  m.def("aggregate", [](const KV& kv, py::object pg) {
    ShuffleStats st;
    KV r = aggregate(kv, as_pg(pg), &st);
    return std::make_pair(r, st);
  });
  m.def("gather_to", [](const KV& kv, int nprocs, py::object pg) {
    ShuffleStats st;
    KV r = gather_to(kv, nprocs, as_pg(pg), &st);
    return std::make_pair(r, st);
  });
  m.def("broadcast", [](const KV& kv, int root, py::object pg) { return broadcast(kv, root, as_pg(pg)); });
  m.def("map_urls", &map_urls);
  m.def("map_words", &map_words);
  m.def("map_rmat", [](int64_t ne, int nl, double a, double b, double c, double d, double f, uint64_t seed,
                       uint64_t first, const std::string& dev) {
    return map_rmat(ne, nl, a, b, c, d, f, seed, first, at::Device(dev));
  });
  m.def("inverted_index_format", &inverted_index_format);
  m.def("segments_sorted", &segments_sorted);
  m.def("pr_contrib", &mrh::pr_contrib);
  m.def("pr_combine", &mrh::pr_combine);
  m.def("scatter_f32", &mrh::scatter_f32);
  m.def("pr_update", &mrh::pr_update);
  m.def("plan_gather_reduce", &mrh::plan_gather_reduce);
  m.def("plan_combine", &mrh::plan_combine);
  m.def("wedges", &mrh::wedges);
  m.def("kv_iter", &kv_iter);
  m.def("kmv_iter", &kmv_iter);
  m.def("hip_compiled", []() { return true; });
}
