// Python bindings of the native engine (module gpu_mapreduce_amd._C).
//
// Exposes the device KV/KMV containers, the engine ops, the process-group
// shuffle, the native KeyValue builder, and the native MapReduce object
// (mapreduce.h) with Python callables adapted to its callback tiers: host
// callbacks receive bytes (and the reference's per-key value lists), batch
// callbacks receive the device KV/KMV. The engine itself lives in
// libmrhip.so, shared with the C API (csrc/capi).
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <c10/hip/HIPGuard.h>
#include <torch/csrc/distributed/c10d/ProcessGroup.hpp>

#include <csignal>
#include <cstring>
#include <execinfo.h>
#include <random>
#include <unistd.h>
#include <string>

#include "devfn.h"
#include "graphmr.h"
#include "hostarena.h"
#include "kv.h"
#include "graphplan.h"
#include "guardalloc.h"
#include "hbmpool.h"
#include "kernels/launch.h"
#include "mapreduce.h"
#include "tri.h"
#include "wordcount.h"
#include "oink/callbacks.h"
#include "oink/oink.h"
#include "oink/trifind_mr.h"

namespace py = pybind11;
using namespace mrh;

namespace mrh {
std::function<void(const std::string&)>& screen_sink();
}

namespace {

PG as_pg(py::object o) {
  if (o.is_none()) return PG();
  return o.cast<PG>();
}

// Run a collective native op (graph plans, their iterations); if it throws on
// a multi-rank communicator, poison the job before the error reaches Python,
// so peers blocked in the same collective fail within seconds instead of
// waiting on a rank that has moved on (MapReduce ops do this in OpTrace).
template <typename F>
auto poisoning(const CommPtr& c, const char* what, F&& f) -> decltype(f()) {
  try {
    return f();
  } catch (const std::exception& e) {
    if (c && c->size() > 1) c->poison(std::string(what) + " raised an error on rank " + std::to_string(c->rank()) +
                                      ": " + e.what());
    throw;
  }
}

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

py::object kvref(KeyValue& kv) { return py::cast(&kv, py::return_value_policy::reference); }

void append_block(py::list& out, char* p, int n, const int* sz) {
  for (int j = 0; j < n; ++j) {
    out.append(py::bytes(p, (size_t)sz[j]));
    p += sz[j];
  }
}

// A key whose values span several pages (the multi-block protocol, reference
// src/mapreduce.cpp:1828-1848, 1874-1925): handed to a Python callback
// instead of a list; block(i) materialises ONE page of values through the
// MR's multivalue_block, so a hot key is never one Python list. Valid only
// during the callback it was passed to.
struct ValueBlocks {
  MapReduce* mr = nullptr;
  int nb = 0;
  int64_t total = 0;
  bool valid = true;
  void check() const {
    if (!valid) throw std::runtime_error("multivalue blocks used after their reduce callback returned");
  }
  py::list block(int i) {
    check();
    if (i < 0 || i >= nb) throw py::index_error("multivalue block index out of range");
    char* p;
    int* sz;
    const int n = mr->multivalue_block(i, &p, &sz);
    py::list out;
    append_block(out, p, n, sz);
    return out;
  }
};

// the values of one key: a list of bytes, or (multi-block mode, mv ==
// nullptr) a ValueBlocks cursor; `live` gets the cursor to invalidate after
py::object value_arg(MapReduce& mr, char* mv, int nv, int* vb, std::shared_ptr<ValueBlocks>* live) {
  if (mv) {
    py::list out;
    append_block(out, mv, nv, vb);
    return out;
  }
  auto c = std::make_shared<ValueBlocks>();
  c->mr = &mr;
  c->total = (int64_t)mr.multivalue_blocks(c->nb);
  *live = c;
  return py::cast(c);
}

// every value of one key as one list (scan_kmv's read-only view)
py::list value_list(MapReduce& mr, char* mv, int nv, int* vb) {
  py::list out;
  if (mv) {
    append_block(out, mv, nv, vb);
  } else {
    int nb = 0;
    mr.multivalue_blocks(nb);
    for (int b = 0; b < nb; ++b) {
      char* p;
      int* sz;
      int n = mr.multivalue_block(b, &p, &sz);
      append_block(out, p, n, sz);
    }
  }
  return out;
}

HashFn py_hash(py::object h) {
  if (h.is_none()) return nullptr;
  return [h](char* k, int kb) {
    py::gil_scoped_acquire g;
    return h(py::bytes(k, (size_t)kb)).cast<int>();
  };
}
CompareFn py_cmp(py::object c) {
  return [c](char* a, int al, char* b, int bl) {
    py::gil_scoped_acquire g;
    return c(py::bytes(a, (size_t)al), py::bytes(b, (size_t)bl)).cast<int>();
  };
}

}  // namespace

namespace {
// MRH_SEGV_TRACE=1: a host segfault prints the native call stack to stderr
// before the default action (Python's faulthandler shows only Python frames)
void segv_trace(int sig) {
  void* fr[64];
  const int n = backtrace(fr, 64);
  const char msg[] = "mrhip: native stack at the fault:\n";
  (void)!write(2, msg, sizeof(msg) - 1);
  backtrace_symbols_fd(fr, n, 2);
  std::signal(sig, SIG_DFL);
  std::raise(sig);
}
}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  if (const char* v = std::getenv("MRH_SEGV_TRACE"); v && *v == '1') {
    std::signal(SIGSEGV, segv_trace);
    std::signal(SIGBUS, segv_trace);
  }
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
      .def_readonly("grouped", &ConvertStats::grouped)
      .def_readonly("dict", &ConvertStats::dict)
      .def_readonly("dict_cap", &ConvertStats::dict_cap)
      .def_readonly("exact", &ConvertStats::exact);
  py::class_<ShuffleStats>(m, "ShuffleStats")
      .def(py::init<>())
      .def_readwrite("send_bytes", &ShuffleStats::send_bytes)
      .def_readwrite("recv_bytes", &ShuffleStats::recv_bytes)
      .def_readwrite("send_pairs", &ShuffleStats::send_pairs)
      .def_readwrite("recv_pairs", &ShuffleStats::recv_pairs)
      .def_readwrite("seconds", &ShuffleStats::seconds)
      .def_readwrite("rounds", &ShuffleStats::rounds);

  // native KeyValue builder (MR-MPI KeyValue::add and its multi variants)
  py::class_<WordCounter>(m, "WordCounter")
      .def(py::init([](const std::string& d, int64_t init) { return new WordCounter(at::Device(d), init); }),
           py::arg("device"), py::arg("init_slots") = 1 << 20)
      .def("add", &WordCounter::add)
      .def("finish", &WordCounter::finish)
      .def_property_readonly("words", &WordCounter::words)
      .def_property_readonly("capacity", &WordCounter::capacity);
  py::class_<KeyValue>(m, "HostKV")
      .def(py::init([](const std::string& d) { return new KeyValue(at::Device(d)); }))
      .def("add", [](KeyValue& kv, const std::string& k,
                     const std::string& v) { kv.add(k.data(), (int64_t)k.size(), v.data(), (int64_t)v.size()); })
      .def("add_fixed",
           [](KeyValue& kv, int64_t n, const std::string& ks, int64_t kb, const std::string& vs, int64_t vb) {
             if ((int64_t)ks.size() != n * kb || (int64_t)vs.size() != n * vb)
               throw std::runtime_error("add_multi: size mismatch");
             kv.add(n, ks.data(), kb, vs.data(), vb);
           })
      .def("add_var",
           [](KeyValue& kv, const std::string& ks, const std::vector<int>& kb, const std::string& vs,
              const std::vector<int>& vb) {
             if (kb.size() != vb.size()) throw std::runtime_error("add_multi: length lists differ");
             kv.add((int64_t)kb.size(), ks.data(), kb.data(), vs.data(), vb.data());
           })
      .def("add_kv", &KeyValue::add_kv, py::call_guard<py::gil_scoped_release>())
      .def("enable_grouping", &KeyValue::enable_grouping)
      .def("reserve_grouping", &KeyValue::reserve_grouping, py::arg("rows"), py::arg("key_bytes"),
           py::arg("value_bytes"), py::arg("groups") = -1)
      .def_property_readonly("grouping", &KeyValue::grouping)
      .def("size", &KeyValue::size)
      .def("finish", &KeyValue::finish)
      .def_property_readonly("device", [](const KeyValue& kv) { return kv.device().str(); });

  py::class_<ValueBlocks, std::shared_ptr<ValueBlocks>>(m, "ValueBlocks")
      .def_readonly("nblocks", &ValueBlocks::nb)
      .def_readonly("nvalues", &ValueBlocks::total)
      .def("block", &ValueBlocks::block)
      .def("__len__", [](const ValueBlocks& b) { return b.total; });
  py::class_<Comm, std::shared_ptr<Comm>>(m, "NativeComm")
      .def(py::init([](py::object pg, const std::string& dev, py::object store, const std::string& transport,
                       std::vector<int> members, int world_rank, int world_size) {
             c10::intrusive_ptr<c10d::Store> st;
             if (!store.is_none()) st = store.cast<c10::intrusive_ptr<c10d::Store>>();
             PG p = as_pg(pg);
             py::gil_scoped_release nogil;  // RCCL bootstrap blocks until every rank arrives
             if (!p) return std::make_shared<Comm>(at::Device(dev));
             return std::make_shared<Comm>(p, at::Device(dev), st, transport, members, world_rank, world_size);
           }),
           py::arg("pg"), py::arg("device"), py::arg("store") = py::none(), py::arg("transport") = "",
           py::arg("members") = std::vector<int>{}, py::arg("world_rank") = -1, py::arg("world_size") = -1)
      .def_property_readonly("rank", &Comm::rank)
      .def_property_readonly("size", &Comm::size)
      .def_property_readonly("members", &Comm::members)
      .def_property_readonly("transport", &Comm::transport)
      .def_property_readonly("max_msg", &Comm::max_msg)
      .def_property_readonly("distributed", &Comm::distributed)
      .def_property_readonly("loopback_collectives", &Comm::loopback_collectives)
      .def_property_readonly("failed", [](const Comm& c) { return c.monitor() && c.monitor()->failed(); })
      .def("rccl_info",
           [](const Comm& c) {
             RcclInfo i = c.rccl_info();
             py::dict d;
             d["comm_count"] = i.comm_count;
             d["cu_device"] = i.cu_device;
             d["user_rank"] = i.user_rank;
             d["live_comms"] = i.live_comms;
             d["id_key"] = i.id_key;
             return d;
           })
      .def("barrier", &Comm::barrier, py::call_guard<py::gil_scoped_release>())
      .def("allreduce", [](const Comm& c, std::vector<int64_t> v, int op) { return c.allreduce(v, (Comm::Op)op); },
           py::call_guard<py::gil_scoped_release>())
      .def("allreduce_f64",
           [](const Comm& c, std::vector<double> v, int op) { return c.allreduce_f64(v, (Comm::Op)op); },
           py::call_guard<py::gil_scoped_release>())
      .def("bcast",
           [](const Comm& c, const std::string& s, int root) {
             std::string r;
             {
               py::gil_scoped_release nogil;
               r = c.bcast(s, root);
             }
             return py::bytes(r);
           })
      .def("alltoall_counts", &Comm::alltoall_counts, py::call_guard<py::gil_scoped_release>())
      .def("alltoallv", &Comm::alltoallv, py::call_guard<py::gil_scoped_release>())
      .def("allgather_var", &Comm::allgather_var, py::call_guard<py::gil_scoped_release>())
      .def("host_wait", &Comm::host_wait, py::call_guard<py::gil_scoped_release>())
      .def("check_peers", &Comm::check_peers)
      .def("poison", &Comm::poison)
      .def("shutdown", &Comm::shutdown, py::call_guard<py::gil_scoped_release>());

  using MR = MapReduce;
  py::class_<MR>(m, "NativeMapReduce")
      .def(py::init([](std::shared_ptr<Comm> c) { return new MR(c); }))
      .def_property("mapstyle", [](MR& r) { return r.set.mapstyle; }, [](MR& r, int v) { r.set.mapstyle = v; })
      .def_property("all2all", [](MR& r) { return r.set.all2all; }, [](MR& r, int v) { r.set.all2all = v; })
      .def_property("verbosity", [](MR& r) { return r.set.verbosity; }, [](MR& r, int v) { r.set.verbosity = v; })
      .def_property("timer", [](MR& r) { return r.set.timer; }, [](MR& r, int v) { r.set.timer = v; })
      .def_property("memsize", [](MR& r) { return r.set.memsize; }, [](MR& r, int v) { r.set.memsize = v; })
      .def_property("minpage", [](MR& r) { return r.set.minpage; }, [](MR& r, int v) { r.set.minpage = v; })
      .def_property("maxpage", [](MR& r) { return r.set.maxpage; }, [](MR& r, int v) { r.set.maxpage = v; })
      .def_property("freepage", [](MR& r) { return r.set.freepage; }, [](MR& r, int v) { r.set.freepage = v; })
      .def_property("outofcore", [](MR& r) { return r.set.outofcore; }, [](MR& r, int v) { r.set.outofcore = v; })
      .def_property("zeropage", [](MR& r) { return r.set.zeropage; }, [](MR& r, int v) { r.set.zeropage = v; })
      .def_property("keyalign", [](MR& r) { return r.set.keyalign; }, [](MR& r, int v) { r.set.keyalign = v; })
      .def_property("valuealign", [](MR& r) { return r.set.valuealign; },
                    [](MR& r, int v) { r.set.valuealign = v; })
      .def_property("fpath", [](MR& r) { return r.set.fpath; }, [](MR& r, const std::string& v) { r.set.fpath = v; })
      .def_property("chunk_bytes", [](MR& r) { return r.set.chunk_bytes; },
                    [](MR& r, int64_t v) { r.set.chunk_bytes = v; })
      .def_property("pipeline", [](MR& r) { return r.set.pipeline; }, [](MR& r, int v) { r.set.pipeline = v; })
      .def_property("hbm_budget", [](MR& r) { return r.set.hbm_budget; },
                    [](MR& r, int64_t v) { r.set.hbm_budget = v; })
      .def_property("host_budget", [](MR& r) { return r.set.host_budget; },
                    [](MR& r, int64_t v) { r.set.host_budget = v; })
      .def_property("streams", [](MR& r) { return r.set.streams; }, [](MR& r, int v) { r.set.streams = v; })
      .def_readwrite("mapfilecount", &MR::mapfilecount)
      .def_property_readonly("spool_stats",
                             [](MR& r) {
                               py::dict d;
                               d["pieces"] = r.spool_stats.pieces;
                               d["hbm_bytes"] = r.spool_stats.hbm_bytes;
                               d["host_bytes"] = r.spool_stats.host_bytes;
                               d["disk_bytes"] = r.spool_stats.disk_bytes;
                               d["files"] = r.spool_stats.files;
                               d["ooc_hot_keys"] = r.ooc_hot_keys;
                               d["ooc_split_keys"] = r.ooc_split_keys;
                               return d;
                             })
      .def_property(
          "kv", [](MR& r) -> py::object {
            r.ensure_resident();
            r.flatten();  // appended parts concatenated: the whole KV
            return r.kv ? py::cast(*r.kv) : py::none();
          },
          [](MR& r, py::object o) {
            r.flatten();
            if (o.is_none()) r.kv.reset();
            else r.kv = o.cast<KV>();
          })
      .def_property_readonly("kv_parts", [](MR& r) { return (int64_t)r.kv_tail().size() + (r.kv ? 1 : 0); })
      .def_property_readonly("kmv_parts", [](MR& r) { return (int64_t)r.kmv_part_count(); })
      .def_property(
          "kmv", [](MR& r) -> py::object {
            r.ensure_resident();
            r.flatten_kmv();
            return r.kmv ? py::cast(*r.kmv) : py::none();
          },
          [](MR& r, py::object o) {
            r.flatten_kmv();
            if (o.is_none()) r.kmv.reset();
            else r.kmv = o.cast<KMV>();
          })
      .def_property_readonly("last_convert", [](MR& r) { return r.last_convert; })
      .def("copy", [](MR& r) { return r.copy().release(); }, py::return_value_policy::take_ownership)
      .def("add", &MR::add, py::call_guard<py::gil_scoped_release>())
      .def("aggregate", [](MR& r, py::object h) {
        HashFn f = py_hash(h);
        py::gil_scoped_release nogil;
        return r.aggregate(f);
      })
      .def("aggregate_dest", &MR::aggregate_dest, py::call_guard<py::gil_scoped_release>())
      .def("broadcast", &MR::broadcast, py::call_guard<py::gil_scoped_release>())
      .def("clone", &MR::clone, py::call_guard<py::gil_scoped_release>())
      .def("close", &MR::close, py::call_guard<py::gil_scoped_release>())
      .def("collapse", [](MR& r, const std::string& k) { return r.collapse(k.data(), (int)k.size()); }, py::call_guard<py::gil_scoped_release>())
      .def("collate", [](MR& r, py::object h) {
        HashFn f = py_hash(h);
        py::gil_scoped_release nogil;
        return r.collate(f);
      })
      .def("convert", &MR::convert, py::call_guard<py::gil_scoped_release>())
      .def("convert_prehashed", &MR::convert_prehashed, py::call_guard<py::gil_scoped_release>())
      .def("gather", &MR::gather, py::call_guard<py::gil_scoped_release>())
      .def("open", &MR::open, py::call_guard<py::gil_scoped_release>())
      .def("kv_open", [](MR& r) { return kvref(r.kv_open()); })
      .def("map", [](MR& r, int nmap, py::function fn,
                     int add) {
        py::gil_scoped_release nogil;
        return r.map(nmap, [&](int t, KeyValue& kv) { py::gil_scoped_acquire g; fn(t, kvref(kv)); }, add);
      })
      .def("map_file",
           [](MR& r, std::vector<std::string> files, int self, int rec, int rd, py::function fn, int add) {
             py::gil_scoped_release nogil;
             return r.map_file(files, self, rec, rd, [&](int t, const char* f, KeyValue& kv) {
               py::gil_scoped_acquire g;
               fn(t, f, kvref(kv));
             }, add);
           })
      .def("map_file_chunks",
           [](MR& r, int nmap, std::vector<std::string> files, int self, int rec, int rd, const std::string& sep,
              bool is_char, int delta, py::function fn, int add) {
             MapChunkFn f = [&](int t, char* s, int n, KeyValue& kv) {
               py::gil_scoped_acquire g;
               fn(t, py::bytes(s, (size_t)n), kvref(kv));
             };
             py::gil_scoped_release nogil;
             if (is_char) return r.map_file_char(nmap, files, self, rec, rd, sep.empty() ? '\n' : sep[0], delta, f, add);
             return r.map_file_str(nmap, files, self, rec, rd, sep, delta, f, add);
           })
      .def("map_mr",
           [](MR& r, MR& src, py::function fn, int add) {
             py::gil_scoped_release nogil;
             return r.map_mr(
                 src,
                 [&](uint64_t i, char* k, int kb, char* v, int vb, KeyValue& kv) {
                   py::gil_scoped_acquire g;
                   fn(i, py::bytes(k, (size_t)kb), py::bytes(v, (size_t)vb), kvref(kv));
                 },
                 add);
           })
      .def("map_mr_batch",
           [](MR& r, MR& src, py::function fn, int add) {
             py::gil_scoped_release nogil;
             return r.map_mr_batch(src, [&](const KV& s, KeyValue& kv) { py::gil_scoped_acquire g; fn(s, kvref(kv)); }, add);
           })
      .def("reduce",
           [](MR& r, py::function fn) {
             py::gil_scoped_release nogil;
             return r.reduce([&](char* k, int kb, char* mv, int nv, int* vb, KeyValue& kv) {
               py::gil_scoped_acquire g;
               std::shared_ptr<ValueBlocks> live;
               struct Done {
                 std::shared_ptr<ValueBlocks>& c;
                 ~Done() {
                   if (c) c->valid = false;
                 }
               } done{live};
               fn(py::bytes(k, (size_t)kb), value_arg(r, mv, nv, vb, &live), kvref(kv));
             });
           })
      .def("compress",
           [](MR& r, py::function fn) {
             py::gil_scoped_release nogil;
             return r.compress([&](char* k, int kb, char* mv, int nv, int* vb, KeyValue& kv) {
               py::gil_scoped_acquire g;
               std::shared_ptr<ValueBlocks> live;
               struct Done {
                 std::shared_ptr<ValueBlocks>& c;
                 ~Done() {
                   if (c) c->valid = false;
                 }
               } done{live};
               fn(py::bytes(k, (size_t)kb), value_arg(r, mv, nv, vb, &live), kvref(kv));
             });
           })
      .def("reduce_builtin", &MR::reduce_builtin, py::call_guard<py::gil_scoped_release>())
      .def("compress_builtin", &MR::compress_builtin, py::call_guard<py::gil_scoped_release>())
      .def("reduce_batch",
           [](MR& r, py::function fn) {
             py::gil_scoped_release nogil;
             return r.reduce_batch([&](const KMV& s, KeyValue& kv) { py::gil_scoped_acquire g; fn(s, kvref(kv)); });
           })
      .def("map_device", &MR::map_device, py::arg("src"), py::arg("code"), py::arg("addflag") = 0,
           py::call_guard<py::gil_scoped_release>())
      .def("map_device_tasks", &MR::map_device_tasks, py::arg("ntask"), py::arg("code"), py::arg("addflag") = 0,
           py::call_guard<py::gil_scoped_release>())
      .def("reduce_device", &MR::reduce_device, py::call_guard<py::gil_scoped_release>())
      .def("compress_device", &MR::compress_device, py::call_guard<py::gil_scoped_release>())
      .def("sort_keys_device", &MR::sort_keys_device, py::arg("code"), py::arg("bits") = 64,
           py::call_guard<py::gil_scoped_release>())
      .def("sort_values_device", &MR::sort_values_device, py::arg("code"), py::arg("bits") = 64,
           py::call_guard<py::gil_scoped_release>())
      .def("compress_batch",
           [](MR& r, py::function fn) {
             py::gil_scoped_release nogil;
             return r.compress_batch([&](const KMV& s, KeyValue& kv) { py::gil_scoped_acquire g; fn(s, kvref(kv)); });
           })
      .def("scan_kv",
           [](MR& r, py::function fn) {
             py::gil_scoped_release nogil;
             return r.scan_kv([&](char* k, int kb, char* v, int vb) {
               py::gil_scoped_acquire g;
               fn(py::bytes(k, (size_t)kb), py::bytes(v, (size_t)vb));
             });
           })
      .def("scan_kmv",
           [](MR& r, py::function fn) {
             py::gil_scoped_release nogil;
             return r.scan_kmv([&](char* k, int kb, char* mv, int nv, int* vb) {
               py::gil_scoped_acquire g;
               fn(py::bytes(k, (size_t)kb), value_list(r, mv, nv, vb));
             });
           })
      .def("scrunch", [](MR& r, int n, const std::string& k) { return r.scrunch(n, k.data(), (int)k.size()); }, py::call_guard<py::gil_scoped_release>())
      .def("sort_keys", [](MR& r, int f) { return r.sort_keys(f); }, py::call_guard<py::gil_scoped_release>())
      .def("sort_keys_fn", [](MR& r, py::function c) { CompareFn f = py_cmp(c); py::gil_scoped_release nogil; return r.sort_keys(f); })
      .def("sort_values", [](MR& r, int f) { return r.sort_values(f); }, py::call_guard<py::gil_scoped_release>())
      .def("sort_values_fn", [](MR& r, py::function c) { CompareFn f = py_cmp(c); py::gil_scoped_release nogil; return r.sort_values(f); })
      .def("sort_multivalues", [](MR& r, int f) { return r.sort_multivalues(f); }, py::call_guard<py::gil_scoped_release>())
      .def("sort_multivalues_fn", [](MR& r, py::function c) { CompareFn f = py_cmp(c); py::gil_scoped_release nogil; return r.sort_multivalues(f); })
      .def("print",
           [](MR& r, int proc, int nstride, int kflag, int vflag, py::object file, int fflag) {
             const bool nofile = file.is_none();
             const std::string path = nofile ? std::string() : file.cast<std::string>();
             py::gil_scoped_release nogil;
             if (nofile) r.print(proc, nstride, kflag, vflag);
             else r.print(path.c_str(), fflag, proc, nstride, kflag, vflag);
           })
      .def("kv_stats", &MR::kv_stats, py::call_guard<py::gil_scoped_release>())
      .def("kmv_stats", &MR::kmv_stats, py::call_guard<py::gil_scoped_release>())
      .def("cummulative_stats", &MR::cummulative_stats, py::call_guard<py::gil_scoped_release>())
      .def("save", &MR::save, py::call_guard<py::gil_scoped_release>())
      .def("load", &MR::load, py::call_guard<py::gil_scoped_release>())
      .def("spill", &MR::spill, py::call_guard<py::gil_scoped_release>())
      .def("unspill", &MR::unspill, py::call_guard<py::gil_scoped_release>())
      .def("spill_disk", &MR::spill_disk, py::call_guard<py::gil_scoped_release>())
      .def("ensure_resident", &MR::ensure_resident, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("on_disk", &MR::on_disk)
      .def("my_proc", &MR::my_proc)
      .def("num_procs", &MR::num_procs)
      .def_property_readonly("device", [](MR& r) { return r.device().str(); });

  m.def("mr_counters", []() {
    py::dict d;
    d["instances_now"] = MapReduce::instances_now.load();
    d["instances_ever"] = MapReduce::instances_ever.load();
    d["msize"] = MapReduce::msize.load();
    d["msizemax"] = MapReduce::msizemax.load();
    d["rsize"] = MapReduce::rsize.load();
    d["wsize"] = MapReduce::wsize.load();
    d["cssize"] = MapReduce::cssize.load();
    d["crsize"] = MapReduce::crsize.load();
    d["commtime"] = MapReduce::commtime;
    return d;
  });
  m.def("mr_count_io", [](int64_t r, int64_t w) {
    MapReduce::rsize += r;
    MapReduce::wsize += w;
  });
  m.def("set_screen", [](py::object f) {
    if (f.is_none()) {
      screen_sink() = [](const std::string& s) {
        std::fwrite(s.data(), 1, s.size(), stdout);
        std::fflush(stdout);
      };
    } else {
      // deliberately leaked: the sink may outlive module teardown
      auto* h = new py::object(f);
      screen_sink() = [h](const std::string& s) {
        py::gil_scoped_acquire g;
        (*h)(s);
      };
    }
  });
  m.def("find_files", [](std::shared_ptr<Comm> c, std::vector<std::string> files, int self, int rec, int rd) {
    py::gil_scoped_release nogil;
    return MapReduce::find_files(*c, files, self, rec, rd);
  });

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
  // HBM page pool (hbmpool.h): the engine's device allocator with a hard cap
  m.def("hbm_pool_install", &hbm::install);
  m.def("hbm_pool_installed", &hbm::installed);
  // a block cached on a stream that is then destroyed (after forget_stream)
  // must not be reached through that stream again: allocate and free blocks of
  // one class on a private stream, retire the stream, then allocate the class
  // from the current stream (the cross-stream reuse path) and free it
  m.def("hbm_pool_stream_retire_check", [](int dev, int64_t bytes) {
    hipStream_t s = nullptr;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) throw std::runtime_error("hipStreamCreate");
    {
      c10::hip::HIPStreamGuard g(c10::hip::getStreamFromExternal(s, (c10::DeviceIndex)dev));
      at::Tensor a = at::empty({bytes}, at::TensorOptions().device(at::kCUDA, dev).dtype(at::kByte));
      a.fill_(1);
    }
    hbm::forget_stream(s);
    (void)hipStreamDestroy(s);
    at::Tensor b = at::empty({bytes}, at::TensorOptions().device(at::kCUDA, dev).dtype(at::kByte));
    b.fill_(2);
    return b.sum().item<int64_t>();
  });
  m.def("hbm_pool_stats", [](int dev) {
    const hbm::PoolStats s = hbm::stats(dev);
    py::dict d;
    d["in_use"] = s.in_use;
    d["peak"] = s.peak;
    d["reserved"] = s.reserved;
    d["reserved_peak"] = s.reserved_peak;
    d["cap"] = s.cap;
    d["allocs"] = s.allocs;
    d["frees"] = s.frees;
    d["failures"] = s.failures;
    d["cached"] = s.cached;
    d["cross_stream_reuse"] = s.cross_stream_reuse;
    d["faulted"] = s.faulted;
    d["grows"] = s.grows;
    d["grow_ms"] = s.grow_ms;
    d["releases"] = s.releases;
    d["oom_retries"] = s.oom_retries;
    return d;
  });
  m.def("hbm_pool_reset_peak", &hbm::reset_peak);
  m.def("hbm_pool_set_cap", &hbm::set_cap);
  m.def("hbm_pool_trim", &hbm::trim, py::call_guard<py::gil_scoped_release>());
  // MRH_GUARD device bounds-check mode (guardalloc.h)
  m.def("install_alloc_guard", &guard::install_alloc_guard);
  m.def("alloc_guard_active", &guard::alloc_guard_active);
  m.def("guard_check", [](const std::string& op) { return guard::check_all_blocks(op.c_str()); },
        py::call_guard<py::gil_scoped_release>());
  m.def("guard_blocks_live", &guard::guarded_blocks_live);
  m.def("guard_reports", [] {
    py::list out;
    for (const auto& r : guard::guard_reports()) {
      py::dict d;
      d["ptr"] = r.ptr;
      d["size"] = r.size;
      d["front_bad"] = r.front_bad;
      d["back_bad"] = r.back_bad;
      d["alloc_op"] = r.alloc_op;
      d["found_op"] = r.found_op;
      out.append(d);
    }
    return out;
  });
  // test hook: a deliberate overrun of `past` bytes past the end of a guarded
  // int32 device tensor (lands in its back canary; refused without the guard)
  m.def("_guard_selftest_overrun", [](at::Tensor t, int64_t past) {
    if (!guard::alloc_guard_active()) throw std::runtime_error("_guard_selftest_overrun needs MRH_GUARD=1");
    if (!t.is_cuda() || t.scalar_type() != at::kInt || !t.is_contiguous() || past < 4 || past > 4096 || past % 4)
      throw std::runtime_error("_guard_selftest_overrun: contiguous int32 HIP tensor, past in [4, 4096], multiple of 4");
    k::fill_i32(t.data_ptr<int32_t>(), t.numel() + past / 4, 7, at::hip::getCurrentHIPStream());
  });
  m.def("radix_sort_keys", &radix_sort_keys, py::arg("keys"), py::arg("begin_bit"), py::arg("end_bit"),
        py::arg("skip_trivial") = true);
  m.def("radix_sort_pairs", &radix_sort_pairs, py::arg("keys"), py::arg("vals"), py::arg("begin_bit"),
        py::arg("end_bit"), py::arg("skip_trivial") = true);
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
  m.def("reduce_builtin", &mrh::reduce_builtin);
  m.def("sort_kv", &sort_kv);
  m.def("sort_multivalues", &mrh::sort_multivalues);
  m.def("expand", &mrh::expand);
  m.def("partition_dest", [](const KV& kv, int P) {
    at::Tensor c;
    at::Tensor d = partition_dest(kv, P, &c);
    return std::make_pair(d, c);
  });
  auto xo = [](int64_t chunk, bool host_sink, int all2all) {
    ExchangeOpts o;
    o.chunk_bytes = chunk;
    o.host_sink = host_sink;
    o.all2all = all2all;
    return o;
  };
  m.def(
      "exchange",
      [xo](const KV& kv, c10::optional<at::Tensor> dest, std::shared_ptr<Comm> c, int64_t chunk, bool host_sink,
           int all2all) {
        ShuffleStats st;
        KV r = poisoning(c, "exchange", [&] { return exchange(kv, dest ? *dest : at::Tensor(), *c, xo(chunk, host_sink, all2all), &st); });
        return std::make_pair(r, st);
      },
      py::arg("kv"), py::arg("dest"), py::arg("comm"), py::arg("chunk_bytes") = 0, py::arg("host_sink") = false,
      py::arg("all2all") = 1, py::call_guard<py::gil_scoped_release>());
  m.def(
      "aggregate",
      [xo](const KV& kv, std::shared_ptr<Comm> c, int64_t chunk, bool host_sink, int all2all) {
        ShuffleStats st;
        KV r = poisoning(c, "aggregate", [&] { return mrh::aggregate(kv, *c, xo(chunk, host_sink, all2all), &st); });
        return std::make_pair(r, st);
      },
      py::arg("kv"), py::arg("comm"), py::arg("chunk_bytes") = 0, py::arg("host_sink") = false,
      py::arg("all2all") = 1, py::call_guard<py::gil_scoped_release>());
  m.def(
      "gather_to",
      [](const KV& kv, int nprocs, std::shared_ptr<Comm> c) {
        ShuffleStats st;
        KV r = poisoning(c, "gather_to", [&] { return gather_to(kv, nprocs, *c, ExchangeOpts(), &st); });
        return std::make_pair(r, st);
      },
      py::call_guard<py::gil_scoped_release>());
  m.def(
      "broadcast",
      [](const KV& kv, int root, std::shared_ptr<Comm> c) {
        return poisoning(c, "broadcast", [&] { return mrh::broadcast(kv, root, *c); });
      },
      py::call_guard<py::gil_scoped_release>());
  m.def("map_urls", &map_urls);
  m.def("kmeans_map", &kmeans_map);
  m.def("map_words", &map_words);
  m.def("map_rmat", [](int64_t ne, int nl, double a, double b, double c, double d, double f, uint64_t seed,
                       uint64_t first, const std::string& dev) {
    return map_rmat(ne, nl, a, b, c, d, f, seed, first, at::Device(dev));
  });
  m.def("inverted_index_format", &inverted_index_format);
  m.def("segments_sorted", &segments_sorted);
  m.def("segments_from_bits", &segments_from_bits);
  m.def("pr_contrib", &mrh::pr_contrib);
  m.def("pr_combine", &mrh::pr_combine);
  m.def("scatter_f32", &mrh::scatter_f32);
  m.def("pr_update", &mrh::pr_update);
  m.def("plan_gather_reduce", &mrh::plan_gather_reduce);
  m.def("plan_combine", &mrh::plan_combine);
  m.def("wedges", &mrh::wedges);
  m.def("wedge_chunks", [](const at::Tensor& seg, const at::Tensor& nb, const at::Tensor& centre, int64_t max_w) {
    std::vector<std::pair<at::Tensor, at::Tensor>> out;
    for_each_wedge_chunk(seg, nb, centre, max_w, [&](const at::Tensor& e, const at::Tensor& c) { out.emplace_back(e, c); });
    return out;
  });
  // the reference's 4-collate tri_find over this rank's [n,2] int64 edges,
  // each stage timed (oink/trifind_mr.h); budgets / fpath / memsize as the
  // MapReduce settings of the pipeline's object (0 / "": defaults)
  m.def(
      "tri_find_mr",
      [](std::shared_ptr<Comm> c, at::Tensor edges, int64_t hbm_budget, int64_t host_budget, std::string fpath,
         int memsize, bool upper) {
        oink::TriMRRun r;
        int64_t spool_files = 0, spool_host = 0, spool_disk = 0, in_vw = -2, in_n = -1;
        {
          py::gil_scoped_release nogil;
          r = poisoning(c, "tri_find_mr", [&] {
            MapReduce mre(c), mrt(c);
            at::Tensor e = edges.to(c->device()).to(at::kLong).reshape({-1, 2}).contiguous();
            mre.map(c->size(), [&](int, KeyValue& kv) {
              if (e.size(0)) oink::add_tensors(kv, e);
            });
            for (MapReduce* m : {&mre, &mrt}) {
              if (hbm_budget > 0) m->set.hbm_budget = hbm_budget;
              if (host_budget > 0) m->set.host_budget = host_budget;
              if (!fpath.empty()) m->set.fpath = fpath;
              if (memsize != 0) m->set.memsize = memsize;
            }
            oink::TriMRRun out = oink::tri_find_mr(mre, mrt, upper);
            mre.flatten();
            in_vw = mre.kv ? mre.kv->vw : -1;  // the edge MR as the pipeline left it
            in_n = mre.kv ? mre.kv->n : 0;
            spool_files = mrt.spool_stats.files + mre.spool_stats.files;
            spool_host = mrt.spool_stats.host_bytes + mre.spool_stats.host_bytes;
            spool_disk = mrt.spool_stats.disk_bytes + mre.spool_stats.disk_bytes;
            return out;
          });
        }
        py::list st;
        for (const auto& s : r.stages) {
          py::dict d;
          d["op"] = s.op;
          d["ms"] = s.seconds * 1e3;
          d["pairs_in"] = s.pairs_in;
          d["pairs_out"] = s.pairs_out;
          d["h2d_bytes"] = s.h2d_bytes;
          d["d2h_bytes"] = s.d2h_bytes;
          d["disk_bytes"] = s.disk_bytes;
          st.append(d);
        }
        py::dict d;
        d["triangles"] = r.triangles;
        d["stages"] = st;
        d["spool_files"] = spool_files;
        d["spool_host_bytes"] = spool_host;
        d["spool_disk_bytes"] = spool_disk;
        d["input_value_width_after"] = in_vw;
        d["compact_vb"] = r.compact_vb;
        d["input_pairs_after"] = in_n;
        return d;
      },
      py::arg("comm"), py::arg("edges"), py::arg("hbm_budget") = 0, py::arg("host_budget") = 0,
      py::arg("fpath") = "", py::arg("memsize") = 0, py::arg("upper") = true);
  // one-shot static-segment gather-reduce (builds the index each call; tests)
  m.def("seg_gather_reduce", [](const at::Tensor& seg, const at::Tensor& src, const at::Tensor& x,
                                c10::optional<at::Tensor> w, int64_t op) {
    const int64_t ng = seg.numel() - 1;
    at::Tensor out = at::empty({std::max<int64_t>(ng, 0)}, x.options());
    if (ng <= 0) return out;
    SegIndex ix = seg_index(seg, src.numel());
    seg_gather_reduce(ix, src.contiguous(), x.contiguous(), w ? *w : at::Tensor(), op, out);
    return out;
  });
  py::class_<EdgePlan>(m, "EdgePlan")
      .def(py::init([](std::shared_ptr<Comm> c, at::Tensor e, int64_t nvert, c10::optional<at::Tensor> w,
                       bool symmetric) {
             std::optional<at::Tensor> ww = w ? std::optional<at::Tensor>(*w) : std::nullopt;
             py::gil_scoped_release nogil;
             return poisoning(c, "EdgePlan", [&] { return new EdgePlan(c, e, nvert, ww, symmetric); });
           }),
           py::arg("comm"), py::arg("edges"), py::arg("nvert"), py::arg("weights") = py::none(),
           py::arg("symmetric") = false)
      .def("propagate",
           [](const EdgePlan& p, const at::Tensor& x, int op, double identity, bool use_weights) {
             return poisoning(p.comm, "EdgePlan.propagate", [&] { return p.propagate(x, op, identity, use_weights); });
           },
           py::call_guard<py::gil_scoped_release>())
      .def("count_global",
           [](const EdgePlan& p, const at::Tensor& mask) {
             return poisoning(p.comm, "EdgePlan.count_global", [&] { return p.count_global(mask); });
           },
           py::call_guard<py::gil_scoped_release>())
      .def_readonly("N", &EdgePlan::N)
      .def_readonly("nlocal", &EdgePlan::nlocal)
      .def_readonly("nedge", &EdgePlan::nedge)
      .def_readonly("ngrp", &EdgePlan::ngrp)
      .def_readonly("src", &EdgePlan::src)
      .def_readonly("w", &EdgePlan::w)
      .def_readonly("seg", &EdgePlan::seg)
      .def_readonly("local_ids", &EdgePlan::local_ids)
      .def_readonly("P", &EdgePlan::P)
      .def_readonly("me", &EdgePlan::me);
  m.def("connected_components",
        [](const EdgePlan& p, int mx) {
          return poisoning(p.comm, "connected_components", [&] { return connected_components(p, mx); });
        },
        py::arg("plan"), py::arg("max_iter") = 100000, py::call_guard<py::gil_scoped_release>());
  m.def(
      "luby_mis",
      [](const EdgePlan& p, int64_t seed, c10::optional<at::Tensor> act, int mx) {
        std::optional<at::Tensor> a = act ? std::optional<at::Tensor>(*act) : std::nullopt;
        py::gil_scoped_release nogil;
        return poisoning(p.comm, "luby_mis", [&] { return luby_mis(p, seed, a, mx); });
      },
      py::arg("plan"), py::arg("seed"), py::arg("active") = py::none(), py::arg("max_iter") = 100000);
  m.def("sssp",
        [](const EdgePlan& p, int64_t s, int mx) { return poisoning(p.comm, "sssp", [&] { return sssp(p, s, mx); }); },
        py::arg("plan"), py::arg("source"), py::arg("max_iter") = 1000000, py::call_guard<py::gil_scoped_release>());
  py::class_<PageRankPlan>(m, "PageRankPlan")
      .def(py::init([](std::shared_ptr<Comm> c, at::Tensor e, int64_t n, double a) {
        py::gil_scoped_release nogil;
        return poisoning(c, "PageRankPlan", [&] { return new PageRankPlan(c, e, n, a); });
      }))
      .def("reset", [](PageRankPlan& p) { poisoning(p.comm, "PageRankPlan.reset", [&] { p.reset(); }); },
           py::call_guard<py::gil_scoped_release>())
      .def("step", [](PageRankPlan& p) { poisoning(p.comm, "PageRankPlan.step", [&] { p.step(); }); },
           py::call_guard<py::gil_scoped_release>())
      .def("run",
           [](PageRankPlan& p, int maxiter, double tol) {
             return poisoning(p.comm, "PageRankPlan.run", [&] { return p.run(maxiter, tol); });
           },
           py::call_guard<py::gil_scoped_release>())
      .def("delta", [](const PageRankPlan& p) { return poisoning(p.comm, "PageRankPlan.delta", [&] { return p.delta(); }); },
           py::call_guard<py::gil_scoped_release>())
      .def("ids", &PageRankPlan::ids)
      .def("ranks", &PageRankPlan::ranks)
      .def_readonly("N", &PageRankPlan::N)
      .def_readonly("nlocal", &PageRankPlan::nlocal)
      .def_property_readonly("blocking", &PageRankPlan::blocking)
      .def_property_readonly("xcd_ranges", &PageRankPlan::xcd_ranges_count)
      .def_property_readonly("layout", &PageRankPlan::layout)
      .def_property_readonly("c_slice", &PageRankPlan::c_slice)
      .def_property_readonly("comm_bytes_per_iter", &PageRankPlan::comm_bytes_per_iter)
      .def_property_readonly("overlapped", &PageRankPlan::overlapped)
      .def_readwrite("use_graph", &PageRankPlan::use_graph)
      .def_property_readonly("graph_iterations", &PageRankPlan::graph_iterations)
      .def_readonly("nedge", &PageRankPlan::nedge)
      .def_readonly("ndangling", &PageRankPlan::ndangling);
  py::class_<TriangleGraph>(m, "TriangleGraph")
      .def(py::init([](std::shared_ptr<Comm> c, at::Tensor e, int64_t n) {
             py::gil_scoped_release nogil;
             return poisoning(c, "TriangleGraph", [&] { return new TriangleGraph(c, e, n); });
           }),
           py::arg("comm"), py::arg("edges"), py::arg("nvert") = -1)
      .def("count", [](const TriangleGraph& g) { return poisoning(g.comm, "TriangleGraph.count", [&] { return g.count(); }); },
           py::call_guard<py::gil_scoped_release>())
      .def("triangles",
           [](const TriangleGraph& g) {
             return poisoning(g.comm, "TriangleGraph.triangles", [&] { return g.triangles(); });
           },
           py::call_guard<py::gil_scoped_release>())
      .def_readonly("nvert", &TriangleGraph::nvert)
      .def_readonly("split", &TriangleGraph::split)
      .def_readonly("u0", &TriangleGraph::u0_)
      .def_readonly("u1", &TriangleGraph::u1_)
      .def_readonly("nedge", &TriangleGraph::nedge)
      .def_readonly("rowptr", &TriangleGraph::rowptr)
      .def_readonly("col", &TriangleGraph::col)
      .def_readonly("okeys", &TriangleGraph::okeys)
      .def_readonly("perm", &TriangleGraph::perm)
      .def_readonly("distributed", &TriangleGraph::distributed)
      .def_readonly("nlocal", &TriangleGraph::nlocal)
      .def_readonly("nrows", &TriangleGraph::nrows)
      .def_readonly("row_gid", &TriangleGraph::row_gid);
  m.def("tri_prepare", &mrh::tri_prepare);
  m.def("tri_count", &mrh::tri_count);
  m.def("tri_hub_size", &mrh::tri_hub_size);
  m.def("tri_last_hub_size", &mrh::tri_last_hub_size);
  m.def("tri_list", &mrh::tri_list);
  // sssp_mr / luby_find_mr callbacks (graphmr.h) for Python batch callbacks
  m.def("ssspmr_pick", [](const KMV& m) {
    SsspPick p = ssspmr_pick(m);
    return py::make_tuple(p.dist, p.ckeys, p.cdist);
  });
  m.def("ssspmr_relax", [](const KMV& m) {
    SsspRelax r = ssspmr_relax(m);
    return py::make_tuple(r.ekeys, r.edges, r.pkeys, r.paths);
  });
  m.def("lubymr_random", &lubymr_random);
  m.def("lubymr_edge_winner", &lubymr_edge_winner);
  m.def("lubymr_vert", [](const KMV& m, bool loser) {
    LubyVert r = lubymr_vert(m, loser);
    return py::make_tuple(r.k24, r.v24, r.k16, r.v16);
  });
  m.def("lubymr_emit", [](const KMV& m) {
    LubyEmit r = lubymr_emit(m);
    return py::make_tuple(r.mis, r.kflag, r.fval, r.knull);
  });
  m.def("device_functor_check", &devfn::compile_check, py::arg("code"), py::arg("reduce"),
        py::call_guard<py::gil_scoped_release>());
  m.def("device_functor_source", &devfn::full_source, py::arg("code"), py::arg("reduce"));
  m.def("device_sortkey_check", &devfn::compile_check_sortkey, py::arg("code"),
        py::call_guard<py::gil_scoped_release>());
  m.def("host_arena_reserve", &hostarena::reserve, py::call_guard<py::gil_scoped_release>());
  m.def("host_arena_stats", [] {
    hostarena::Stats s = hostarena::stats();
    py::dict d;
    d["reserved"] = s.reserved;
    d["in_use"] = s.in_use;
    d["peak"] = s.peak;
    d["hits"] = s.hits;
    d["misses"] = s.misses;
    return d;
  });
  m.def("kv_iter", &kv_iter);
  m.def("kmv_iter", &kmv_iter);
  // native OINK interpreter (csrc/oink)
  py::register_exception<mrh::oink::Error>(m, "OinkError", PyExc_RuntimeError);
  py::class_<mrh::oink::Oink>(m, "Oink")
      .def(py::init([](std::shared_ptr<Comm> u, std::vector<std::string> parts, py::object screen,
                       const std::string& logfile, std::vector<std::pair<std::string, std::vector<std::string>>> vars,
                       const std::string& echo, std::shared_ptr<Comm> world) {
             mrh::oink::Oink::Sink sink;
             if (!screen.is_none()) {
               std::shared_ptr<py::object> h(new py::object(screen), [](py::object* p) {
                 py::gil_scoped_acquire g;
                 delete p;
               });
               sink = [h](const std::string& s) {
                 py::gil_scoped_acquire g;
                 (*h)(s);
               };
             }
             return new mrh::oink::Oink(u, parts, sink, logfile, vars, echo, world);
           }),
           py::arg("comm"), py::arg("partitions"), py::arg("screen"), py::arg("logfile"), py::arg("variables"),
           py::arg("echo"), py::arg("world") = nullptr)
      .def("file", &mrh::oink::Oink::file, py::call_guard<py::gil_scoped_release>())
      .def("text", &mrh::oink::Oink::text, py::call_guard<py::gil_scoped_release>())
      .def("one", &mrh::oink::Oink::one, py::call_guard<py::gil_scoped_release>())
      .def("close", &mrh::oink::Oink::close)
      .def_readonly("deltatime", &mrh::oink::Oink::deltatime)
      .def_property_readonly("nworlds", [](mrh::oink::Oink& o) { return o.universe->nworlds; })
      .def_property_readonly("iworld", [](mrh::oink::Oink& o) { return o.universe->iworld; })
      .def("mr_names",
           [](mrh::oink::Oink& o) {
             std::vector<std::string> v;
             for (auto& e : o.obj->mrs)
               if (e.permanent) v.push_back(e.name);
             return v;
           })
      .def(
          "mr",
          [](mrh::oink::Oink& o, const std::string& name) -> MapReduce* {
            int i = o.obj->find_mr(name);
            if (i < 0) throw mrh::oink::Error("no MR object named " + name);
            return o.obj->mrs[i].mr.get();
          },
          py::return_value_policy::reference_internal);
  m.def("oink_main", [](std::shared_ptr<Comm> u, std::vector<std::string> argv) {
    py::gil_scoped_release nogil;
    return mrh::oink::main_args(u, argv);
  });
  // The RCCL unique-id rendezvous with a fake (random) id instead of
  // ncclGetUniqueId, so CPU multi-process tests drive the exact key protocol
  // of Rccl's constructor: returns (key, id bytes); rank 0 then waits for the
  // acknowledgements and deletes the key, as after ncclCommInitRank.
  m.def(
      "rccl_rendezvous_probe",
      [](py::object store, const std::string& tag, std::vector<int> members, int rank) {
        auto st = store.cast<c10::intrusive_ptr<c10d::Store>>();
        IdRendezvous r;
        {
          py::gil_scoped_release nogil;
          r = rendezvous_id(st, tag, members, rank, [] {
            std::vector<uint8_t> id(128);
            std::random_device rd;
            for (auto& b : id) b = (uint8_t)rd();
            return id;
          }, nullptr);
          if (rank == 0) rendezvous_release(st, r, (int)members.size(), nullptr);
        }
        return std::make_pair(r.key, py::bytes((const char*)r.id.data(), r.id.size()));
      },
      py::arg("store"), py::arg("tag"), py::arg("members"), py::arg("rank"));
  m.def("live_rccl_comms", &mrh::live_rccl_comms);
  // host-side calls per nccl* entry point so far in this process (rccl.h)
  m.def("rccl_counters", []() {
    const mrh::RcclCounters& c = mrh::rccl_counters();
    py::dict d;
    d["all_reduce"] = c.all_reduce.load();
    d["all_gather"] = c.all_gather.load();
    d["broadcast"] = c.broadcast.load();
    d["send"] = c.send.load();
    d["recv"] = c.recv.load();
    d["group"] = c.group.load();
    return d;
  });
  m.def("rccl_counters_reset", &mrh::rccl_counters_reset);
  m.def("rccl_graph_probe", &mrh::rccl_graph_probe, py::arg("device"), py::arg("what"), py::arg("capture"),
        py::arg("mode") = 1, py::call_guard<py::gil_scoped_release>());
  // spool files currently on disk in this process (disk tier, spool.h)
  m.def("spool_files_live", &mrh::spool_files_live);
  // the disk tier's background writer pool (spool.h WriterStats)
  m.def("spool_writer_stats", []() {
    const mrh::WriterStats w = mrh::spool_writer_stats();
    py::dict d;
    d["inflight_bytes"] = w.inflight_bytes;
    d["peak_inflight_bytes"] = w.peak_inflight_bytes;
    d["cap_bytes"] = w.cap_bytes;
    d["threads"] = w.threads;
    d["jobs"] = w.jobs;
    return d;
  });
  m.def("spool_writer_reset_peak", &mrh::spool_writer_reset_peak);
  // world size 1 runs the local transport (no communicator); this builds a
  // one-rank RCCL communicator on `device` and returns what RCCL reports
  m.def("rccl_self_probe", [](int device) {
    py::dict d;
    {
      Rccl r(0, 1, device, c10::intrusive_ptr<c10d::Store>(), "probe");
      d["comm_count"] = r.comm_count();
      d["cu_device"] = r.cu_device();
      d["user_rank"] = r.user_rank();
    }
    return d;
  });
  m.def("hip_compiled", []() { return true; });
  // PCI bus id of a visible GPU ("" if none), for NUMA-local CPU/memory binding
  m.def("gpu_pci_bus_id", &mrh::gpu_pci_bus_id);
}
