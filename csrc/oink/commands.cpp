// OINK named commands (reference oink/<name>.cpp, each registered by
// CommandStyle(name, Class) at <name>.h:11). Every command keeps the
// reference's params / -i inputs / -o outputs contract and its MapReduce op
// sequence; the per-pair callbacks become device-batch callbacks on the
// HBM-resident KV/KMV, and the iterative graph commands (cc_find, luby_find,
// sssp, pagerank) and tri_find run on the native plans of
// csrc/engine/graphplan.h instead of re-shuffling every edge each iteration.
#include <algorithm>
#include <chrono>
#include <cinttypes>
#include <cmath>
#include <cstdarg>
#include <cstdlib>
#include <cstring>
#include <filesystem>
#include <limits>
#include <random>

#include <ATen/CPUGeneratorImpl.h>

#include "callbacks.h"
#include "engine/ccmr.h"
#include "engine/graphmr.h"
#include "engine/graphplan.h"
#include "engine/tri.h"
#include "oink.h"
#include "trifind_mr.h"

namespace mrh {
namespace oink {

namespace {

std::string fmt(const char* f, ...) __attribute__((format(printf, 1, 2)));
std::string fmt(const char* f, ...) {
  char buf[2048];
  va_list ap;
  va_start(ap, f);
  vsnprintf(buf, sizeof(buf), f, ap);
  va_end(ap);
  return buf;
}
at::TensorOptions opt(at::Device d, at::ScalarType t) { return at::TensorOptions().device(d).dtype(t); }

long long lval(const std::string& s, const std::string& cmd) {
  char* e = nullptr;
  long long v = std::strtoll(s.c_str(), &e, 10);
  if (!e || *e || s.empty()) throw Error("Illegal " + cmd + " command");
  return v;
}
double dval(const std::string& s, const std::string& cmd) {
  char* e = nullptr;
  double v = std::strtod(s.c_str(), &e);
  if (!e || *e || s.empty()) throw Error("Illegal " + cmd + " command");
  return v;
}

MapFileFn rd(Parser p) { return file_reader(p); }
MapChunkFn rc(Parser p) { return chunk_reader(p); }

// per-value byte lengths / starts / owning key of a KMV
at::Tensor kmv_vlens(const KMV& m) {
  if (m.vw >= 0) return at::full({m.nval}, (int64_t)m.vw, opt(m.seg.device(), at::kLong));
  return m.voff.narrow(0, 1, m.nval) - m.voff.narrow(0, 0, m.nval);
}
at::Tensor kmv_vstart(const KMV& m) {
  if (m.vw >= 0) return at::arange(m.nval, opt(m.seg.device(), at::kLong)) * (int64_t)m.vw;
  return m.voff.narrow(0, 0, m.nval);
}
at::Tensor kmv_lens(const KMV& m) { return m.seg.narrow(0, 1, m.nkey) - m.seg.narrow(0, 0, m.nkey); }
at::Tensor kmv_sid(const KMV& m) {
  return segment_ids(m.seg, m.nkey, m.nval);
}
// w-byte items at byte offsets pos of vdata, as a [n, w] uint8 tensor
at::Tensor gather_bytes(const at::Tensor& vdata, const at::Tensor& pos, int w) {
  at::Tensor idx = pos.unsqueeze(1) + at::arange(w, opt(vdata.device(), at::kLong));
  return vdata.index({idx}).contiguous();
}

int64_t nvert_global(const Comm& comm, const at::Tensor& e) {
  const int64_t mx = e.numel() ? e.max().item<int64_t>() : -1;
  return comm.allreduce(mx, Comm::MAX) + 1;
}

// "  <b> ... <a> ..." lines of an (int key a, int value b) histogram on rank 0
void print_histo(Oink& o, MapReduce& mr, const char* f) {
  mr.flatten();
  if (o.me != 0 || !mr.kv || mr.kv->n == 0) return;
  at::Tensor k = mr.kv->kdata.to(at::kCPU).contiguous(), v = mr.kv->vdata.to(at::kCPU).contiguous();
  const int kw = mr.kv->kw > 0 ? mr.kv->kw : 4, vw = mr.kv->vw > 0 ? mr.kv->vw : 4;
  for (int64_t i = 0; i < mr.kv->n; ++i) {
    int32_t a, b;
    std::memcpy(&a, k.data_ptr<uint8_t>() + i * kw, 4);
    std::memcpy(&b, v.data_ptr<uint8_t>() + i * vw, 4);
    o.message(fmt(f, b, a));
  }
}

// ====================================================================== rmat / rmat2

struct RmatP {
  int nlevels = 0;
  int64_t nnz = 0, order = 0;
  double a = 0, b = 0, c = 0, d = 0, frac = 0;
  uint64_t seed = 0;
};
RmatP rmat_params(const Args& a, const std::string& name) {
  if (a.size() != 8) throw Error("Illegal " + name + " command");
  RmatP r;
  r.nlevels = (int)lval(a[0], name);
  r.nnz = lval(a[1], name);
  r.a = dval(a[2], name);
  r.b = dval(a[3], name);
  r.c = dval(a[4], name);
  r.d = dval(a[5], name);
  r.frac = dval(a[6], name);
  r.seed = (uint64_t)lval(a[7], name);
  if (std::fabs(r.a + r.b + r.c + r.d - 1.0) > 1e-12) throw Error("RMAT a,b,c,d must sum to 1");
  if (r.frac >= 1.0) throw Error("RMAT fraction must be < 1");
  if (r.nlevels < 1 || r.nlevels > 62) throw Error("RMAT levels must be in [1,62]");
  r.order = int64_t(1) << r.nlevels;  // 64-bit (reference oink/rmat.cpp:95 overflows an int)
  return r;
}

// map/task generator of this rank's share of new R-MAT edges (reference
// map_rmat_generate.cpp:14-67) on the GPU: edge ids continue across
// iterations, so every iteration draws fresh edges
class RmatGen {
 public:
  RmatGen(const RmatP& r, const Comm& c) : r_(r), P_(c.size()), me_(c.rank()) {}
  MapTaskFn gen(int64_t nremain) {
    const int64_t lo = base_ + me_ * (nremain / P_) + std::min<int64_t>(me_, nremain % P_);
    const int64_t n = nremain / P_ + (me_ < nremain % P_ ? 1 : 0);
    base_ += nremain;
    const RmatP r = r_;
    return [r, lo, n](int, KeyValue& kv) {
      if (n) kv.add_kv(map_rmat(n, r.nlevels, r.a, r.b, r.c, r.d, r.frac, r.seed, (uint64_t)lo, kv.device()));
    };
  }

 private:
  RmatP r_;
  int64_t P_, me_, base_ = 0;
};

// rmat N Nz a b c d frac seed -o file mr  (oink/rmat.cpp:37-71)
class RMAT : public Command {
 public:
  using Command::Command;
  RmatP r;
  void params(const Args& a) override {
    noutputs = 1;
    r = rmat_params(a, "rmat");
  }
  void run() override {
    MapReduce& mr = obj.create_mr();
    const int64_t ntotal = r.order * r.nnz;
    int64_t nremain = ntotal;
    int niter = 0;
    RmatGen g(r, *comm);
    while (nremain > 0) {
      ++niter;
      mr.map(nprocs, g.gen(nremain), 1);
      const int64_t nunique = (int64_t)mr.collate();
      mr.reduce_builtin("first", "");  // cull
      nremain = ntotal - nunique;
    }
    obj.output(1, mr, print_edge);
    message(fmt("RMAT: %" PRId64 " rows, %" PRId64 " non-zeroes, %d iterations", r.order, ntotal, niter));
    obj.cleanup();
  }
};

// rmat2: generate into a fresh MR, aggregate, add, convert (oink/rmat2.cpp:37-74)
class RMAT2 : public RMAT {
 public:
  using RMAT::RMAT;
  void params(const Args& a) override {
    noutputs = 1;
    r = rmat_params(a, "rmat2");
  }
  void run() override {
    MapReduce& mr = obj.create_mr();
    MapReduce& mrnew = obj.create_mr();
    const int64_t ntotal = r.order * r.nnz;
    int64_t nremain = ntotal;
    int niter = 0;
    RmatGen g(r, *comm);
    mr.map(nprocs, [](int, KeyValue&) {});
    while (nremain > 0) {
      ++niter;
      mrnew.map(nprocs, g.gen(nremain));
      mrnew.aggregate();
      mr.add(mrnew);
      const int64_t nunique = (int64_t)mr.convert();
      mr.reduce_builtin("first", "");
      nremain = ntotal - nunique;
    }
    obj.output(1, mr, print_edge);
    message(fmt("RMAT2: %" PRId64 " rows, %" PRId64 " non-zeroes, %d iterations", r.order, ntotal, niter));
    obj.cleanup();
  }
};

// ====================================================================== edge / vertex / degree commands

class EdgeUpper : public Command {  // oink/edge_upper.cpp:37-60
 public:
  EdgeUpper(Oink& o) : Command(o) { ninputs = noutputs = 1; }
  void run() override {
    MapReduce& mre = obj.input(1, rd(parse_edge), rc(parse_edge));
    MapReduce& mr = obj.create_mr();
    const uint64_t nedge = mre.kv_stats(0);
    mr.map_mr_batch(mre, edge_upper);
    mr.collate();
    const uint64_t unique = mr.reduce_builtin("first", "");
    obj.output(1, mr, print_edge);
    message(fmt("EdgeUpper: %" PRIu64 " original edges, %" PRIu64 " final edges", nedge, unique));
    obj.cleanup();
  }
};

class Degree : public Command {  // degree dup (oink/degree.cpp:36-59)
 public:
  Degree(Oink& o) : Command(o) { ninputs = noutputs = 1; }
  int dup = 0;
  void params(const Args& a) override {
    if (a.size() != 1) throw Error("Illegal degree command");
    dup = (int)lval(a[0], "degree");
  }
  void run() override {
    MapReduce& mre = obj.input(1, rd(parse_edge), rc(parse_edge));
    MapReduce& mrv = obj.create_mr();
    const uint64_t nedge = mre.kv_stats(0);
    mrv.map_mr_batch(mre, dup == 1 ? MapBatchFn(edge_to_vertex) : MapBatchFn(edge_to_vertices));
    mrv.collate();
    const uint64_t nvert = mrv.reduce_builtin("count", "");
    obj.output(1, mrv, print_vertex_int);
    message(fmt("Degree: %" PRIu64 " vertices, %" PRIu64 " edges", nvert, nedge));
    obj.cleanup();
  }
};

class DegreeStats : public Command {  // oink/degree_stats.cpp:35-64
 public:
  DegreeStats(Oink& o) : Command(o) { ninputs = 1; }
  int dup = 0;
  void params(const Args& a) override {
    if (a.size() != 1) throw Error("Illegal degree_stats command");
    dup = (int)lval(a[0], "degree_stats");
  }
  void run() override {
    MapReduce& mre = obj.input(1, rd(parse_edge), rc(parse_edge));
    MapReduce& mr = obj.create_mr();
    const uint64_t nedge = mre.kv_stats(0);
    mr.map_mr_batch(mre, dup == 1 ? MapBatchFn(edge_to_vertex) : MapBatchFn(edge_to_vertices));
    mr.collate();
    const uint64_t nvert = mr.reduce_builtin("count", "");
    mr.map_mr_batch(mr, invert);
    mr.collate();
    mr.reduce_builtin("count", "");
    mr.gather(1);
    mr.sort_keys(-1);
    message(fmt("DegreeStats: %" PRIu64 " vertices, %" PRIu64 " edges", nvert, nedge));
    print_histo(oink, mr, "  %d vertices with %d edges");
    obj.cleanup();
  }
};

class Histo : public Command {  // oink/histo.cpp:36-73
 public:
  Histo(Oink& o) : Command(o) { ninputs = noutputs = 1; }
  void run() override {
    MapReduce* mr = &obj.input(1);
    const uint64_t ntotal = mr->kv_stats(0);
    if (obj.permanent(*mr)) mr = &obj.copy_mr(*mr);
    mr->collate();
    const uint64_t nunique = mr->reduce_builtin("count", "");
    obj.output(1, *mr);
    if (obj.permanent(*mr)) mr = &obj.copy_mr(*mr);
    mr->map_mr_batch(*mr, invert);
    mr->collate();
    mr->reduce_builtin("count", "");
    mr->gather(1);
    mr->sort_keys(-1);
    message(fmt("Histo: %" PRIu64 " total keys, %" PRIu64 " unique", ntotal, nunique));
    print_histo(oink, *mr, "  %d keys appear %d times");
    obj.cleanup();
  }
};

// edges + (vertex, int degree) -> (edge, 1/degree(vi)) (oink/degree_weight.cpp:35-125)
class DegreeWeight : public Command {
 public:
  DegreeWeight(Oink& o) : Command(o) {
    ninputs = 2;
    noutputs = 1;
  }
  void run() override {
    MapReduce& mre = obj.input(1, rd(parse_edge), rc(parse_edge));
    MapReduce& mrd = obj.input(2, rd(parse_vertex_label), rc(parse_vertex_label));
    MapReduce& mrewt = obj.create_mr();
    const uint64_t nvert = mrd.kv_stats(0);
    mrewt.map_mr_batch(mre, edge_to_vertex_pair);
    mrewt.add(mrd);
    mrewt.collate();
    const uint64_t nedge = mrewt.reduce_batch([](const KMV& m, KeyValue& kv) {
      if (!m.nval) return;
      const at::Device d = m.seg.device();
      at::Tensor vl = kmv_vlens(m), vs = kmv_vstart(m), sid = kmv_sid(m);
      at::Tensor is_deg = vl == 4, is_e = vl == 8;
      at::Tensor deg = at::zeros({m.nkey}, opt(d, at::kDouble));
      at::Tensor dv = gather_bytes(m.vdata, vs.index({is_deg}), 4).view(at::kInt).reshape({-1}).to(at::kDouble);
      deg.index_put_({sid.index({is_deg})}, dv);
      at::Tensor se = sid.index({is_e});
      at::Tensor vj = gather_bytes(m.vdata, vs.index({is_e}), 8).view(at::kLong).reshape({-1});
      at::Tensor vi = m.keys.kdata.view(at::kLong).index({se});
      add_tensors(kv, at::stack({vi, vj}, 1), 1.0 / deg.index({se}));
    });
    obj.output(1, mrewt, print_edge_weight);
    message(fmt("DegreeWeight: %" PRIu64 " vertices, %" PRIu64 " edges", nvert, nedge));
    obj.cleanup();
  }
};

// wordfreq ntop -i files -o file mr (oink/wordfreq.cpp:40-90)
class WordFreq : public Command {
 public:
  WordFreq(Oink& o) : Command(o) { ninputs = noutputs = 1; }
  int ntop = 0;
  void params(const Args& a) override {
    if (a.size() != 1) throw Error("Illegal wordfreq command");
    ntop = (int)lval(a[0], "wordfreq");
  }
  void run() override {
    int64_t nfiles = 0;
    MapReduce* mr = &obj.input(1, file_reader(parse_words, &nfiles), rc(parse_words));
    const uint64_t nwords = mr->kv_stats(0);
    const int64_t nfiles_all = comm->allreduce(nfiles, Comm::SUM);
    if (obj.permanent(*mr)) mr = &obj.copy_mr(*mr);
    mr->collate();
    const uint64_t nunique = mr->reduce_builtin("count", "");
    obj.output(1, *mr, print_string_int);
    if (ntop) {
      if (obj.permanent(*mr)) mr = &obj.copy_mr(*mr);
      mr->sort_values(-1);
      mr->map_mr_batch(*mr, [](const KV& src, KeyValue& kv) {  // local top 10
        const int64_t n = std::min<int64_t>(10, src.n);
        if (n) kv.add_kv(gather(src, at::arange(n, opt(src.device(), at::kInt))));
      });
      mr->gather(1);
      mr->sort_values(-1);
      mr->flatten();
      if (me == 0 && mr->kv) {
        const KV& kv = *mr->kv;
        at::Tensor kd = kv.kdata.to(at::kCPU).contiguous(), ko = kv.koff.to(at::kCPU).contiguous();
        at::Tensor vd = kv.vdata.to(at::kCPU).contiguous();
        for (int64_t i = 0; i < std::min<int64_t>(ntop, kv.n); ++i) {
          const int64_t a = ko.data_ptr<int64_t>()[i], b = ko.data_ptr<int64_t>()[i + 1];
          const char* w = (const char*)kd.data_ptr<uint8_t>() + a;
          int32_t c;
          std::memcpy(&c, vd.data_ptr<uint8_t>() + 4 * i, 4);
          message(fmt("%d %s", c, std::string(w, strnlen(w, (size_t)(b - a))).c_str()));
        }
      }
    }
    message(fmt("WordFreq: %" PRId64 " files, %" PRIu64 " words, %" PRIu64 " unique", nfiles_all, nwords, nunique));
    obj.cleanup();
  }
};

class VertexExtract : public Command {  // oink/vertex_extract.cpp:36-55
 public:
  VertexExtract(Oink& o) : Command(o) { ninputs = noutputs = 1; }
  void run() override {
    MapReduce& mre = obj.input(1, rd(parse_edge_weight), rc(parse_edge_weight));
    MapReduce& mrv = obj.create_mr();
    mrv.map_mr_batch(mre, edge_to_vertices);
    mrv.collate();
    mrv.reduce_builtin("first", "");
    obj.output(1, mrv, print_vertex);
    obj.cleanup();
  }
};

// (v, [neighbours]) adjacency lists (oink/neighbor.cpp:34-51)
class Neighbor : public Command {
 public:
  Neighbor(Oink& o) : Command(o) { ninputs = noutputs = 1; }
  void run() override {
    MapReduce& mre = obj.input(1, rd(parse_edge), rc(parse_edge));
    MapReduce& mrn = obj.create_mr();
    mrn.map_mr_batch(mre, [](const KV& src, KeyValue& kv) {
      if (!src.n) return;
      at::Tensor e = edges_of(src);
      add_tensors(kv, at::cat({e.select(1, 0), e.select(1, 1)}), at::cat({e.select(1, 1), e.select(1, 0)}));
    });
    mrn.collate();
    mrn.reduce_batch([](const KMV& m, KeyValue& kv) {
      if (m.nkey) add_tensors(kv, m.keys.kdata.view(at::kLong), m.vdata, m.seg * 8);
    });
    obj.output(1, mrn, print_neighbors);
    obj.cleanup();
  }
};

// neigh_tri dir -i neighbors triangles: one file per vertex with its
// neighbour edges and the triangles it belongs to (oink/neigh_tri.cpp:39-60)
class NeighTri : public Command {
 public:
  NeighTri(Oink& o) : Command(o) {
    ninputs = 2;
    noutputs = 1;
  }
  std::string dir;
  void params(const Args& a) override {
    if (a.size() != 1) throw Error("Illegal neigh_tri command");
    dir = a[0];
  }
  void run() override {
    MapReduce& mrn = obj.input(1, rd(parse_neighbors), rc(parse_neighbors));
    MapReduce& mrt = obj.input(2, rd(parse_tri), rc(parse_tri));
    MapReduce& mrnplus = obj.create_mr();
    mrnplus.map_mr_batch(mrn, [](const KV& src, KeyValue& kv) {  // (v, packed list) -> (v, vj) pairs
      if (!src.n) return;
      if (src.vw == 8) {
        kv.add_kv(src);
        return;
      }
      if (src.vw >= 0 && src.vw % 8) throw Error("neighbor values must be lists of vertices");
      at::Tensor cnt = src.vw >= 0 ? at::full({src.n}, (int64_t)(src.vw / 8), opt(src.device(), at::kLong))
                                   : at::floor_divide(src.voff.narrow(0, 1, src.n) - src.voff.narrow(0, 0, src.n), 8);
      add_tensors(kv, src.kdata.view(at::kLong).index_select(0, repeat_index(cnt)), src.vdata.view(at::kLong));
    });
    mrnplus.map_mr_batch(
        mrt,
        [](const KV& src, KeyValue& kv) {
          if (!src.n) return;
          at::Tensor t = src.kdata.view(at::kLong).view({-1, 3});
          at::Tensor vi = t.select(1, 0), vj = t.select(1, 1), vk = t.select(1, 2);
          add_tensors(kv, at::cat({vi, vj, vk}),
                      at::cat({at::stack({vj, vk}, 1), at::stack({vi, vk}, 1), at::stack({vi, vj}, 1)}));
        },
        1);
    mrnplus.collate();
    std::filesystem::create_directories(dir);
    const std::string d = dir;
    mrnplus.scan_kmv([&mrnplus, d](char* k, int, char* mv, int nv, int* vb) {
      uint64_t vi;
      std::memcpy(&vi, k, 8);
      std::FILE* f = std::fopen((d + "/" + std::to_string(vi)).c_str(), "w");
      if (!f) throw Error("Could not open neigh_tri output file");
      auto walk = [&](char* p, int cnt, int* sz) {
        for (int i = 0; i < cnt; ++i) {
          uint64_t x[2] = {0, 0};
          std::memcpy(x, p, std::min(sz[i], 16));
          if (sz[i] == 8) std::fprintf(f, "%" PRIu64 " %" PRIu64 "\n", vi, x[0]);
          else std::fprintf(f, "%" PRIu64 " %" PRIu64 "\n", x[0], x[1]);
          p += sz[i];
        }
      };
      if (mv) {
        walk(mv, nv, vb);
      } else {
        int nb = 0;
        mrnplus.multivalue_blocks(nb);
        for (int b = 0; b < nb; ++b) {
          char* p;
          int* sz;
          int c = mrnplus.multivalue_block(b, &p, &sz);
          walk(p, c, sz);
        }
      }
      std::fclose(f);
    });
    obj.output(1, mrnplus);
    obj.cleanup();
  }
};

// ====================================================================== triangles

// tri_find -i edges -o file mr: every triangle once, (vi, vj, vk) with
// vi < vj < vk, on the replicated degree-oriented CSR (graphplan.h
// TriangleGraph); same result as the reference's 4-shuffle pipeline
// (oink/tri_find.cpp:43-82), available as tri_find_mr
class TriFind : public Command {
 public:
  TriFind(Oink& o) : Command(o) { ninputs = noutputs = 1; }
  void run() override {
    MapReduce& mre = obj.input(1, rd(parse_edge), rc(parse_edge));
    mre.flatten();
    at::Tensor e = mre.kv ? edges_of(*mre.kv) : at::empty({0, 2}, opt(comm->device(), at::kLong));
    TriangleGraph g(comm, e, -1);
    at::Tensor tri = g.triangles();
    const int64_t ntri = comm->allreduce(tri.numel() ? tri.size(0) : 0, Comm::SUM);
    MapReduce& mrt = obj.create_mr();
    mrt.map(nprocs, [&](int, KeyValue& kv) {
      if (tri.numel()) add_tensors(kv, tri.contiguous());
    });
    obj.output(1, mrt, print_tri);
    message(fmt("Tri_find: %" PRId64 " triangles", ntri));
    obj.cleanup();
  }
};

// the reference's 4-shuffle pipeline; the O(d^2) wedge generation is the
// load-balanced wedges kernel (oink/tri_find.cpp:43-82, callbacks :104-325)
class TriFindMR : public Command {
 public:
  TriFindMR(Oink& o) : Command(o) { ninputs = noutputs = 1; }
  void run() override {
    MapReduce& mre = obj.input(1, rd(parse_edge), rc(parse_edge));
    MapReduce& mrt = obj.create_mr();
    const uint64_t ntri = tri_find_mr(mre, mrt).triangles;
    obj.output(1, mrt, print_tri);
    message(fmt("Tri_find: %" PRIu64 " triangles", ntri));
    obj.cleanup();
  }
};

// ====================================================================== iterative graph commands

at::Tensor present(const EdgePlan& p) {  // local vertices that appear in any edge
  if (p.nlocal == 0) return at::zeros({0}, opt(p.dev, at::kBool));
  return bincount_dev(p.src, p.nlocal) > 0;
}

// cc_find nthresh: (vertex, component id = min vertex id) (oink/cc_find.cpp:38-109).
// nthresh (hot-zone splitting) is accepted and unused here: on the edge plan
// a vertex is one key and a hub's in-edges are one load-balanced segment, so
// no zone ever gathers on one rank. cc_find_mr runs the reference's zone
// pipeline, where nthresh does split hot zones over ranks.
class CCFind : public Command {
 public:
  CCFind(Oink& o) : Command(o) { ninputs = noutputs = 1; }
  void params(const Args& a) override {
    if (a.size() != 1) throw Error("Illegal cc_find command");
    lval(a[0], "cc_find");
  }
  void run() override {
    MapReduce& mre = obj.input(1, rd(parse_edge), rc(parse_edge));
    mre.flatten();
    at::Tensor e = mre.kv ? edges_of(*mre.kv) : at::empty({0, 2}, opt(comm->device(), at::kLong));
    const int64_t N = nvert_global(*comm, e);
    EdgePlan plan(comm, e, N, std::nullopt, true);
    auto [lab, niter] = connected_components(plan);
    at::Tensor pres = present(plan);
    at::Tensor ids = plan.local_ids.index({pres}), zl = lab.index({pres});
    MapReduce& mrv = obj.create_mr();
    mrv.map(nprocs, [&](int, KeyValue& kv) {
      if (ids.numel()) add_tensors(kv, ids, zl);
    });
    obj.output(1, mrv, print_vertex_u64);
    const int64_t ncc = comm->allreduce(ids.numel() ? (zl == ids).sum().item<int64_t>() : 0, Comm::SUM);
    message(fmt("CC_find: %" PRId64 " components in %d iterations", ncc, niter));
    obj.cleanup();
  }
};

// cc_find_mr nthresh: the reference's MapReduce formulation of connected
// components (oink/cc_find.cpp:38-109) with its hot-zone splitting: a zone
// holding more than nthresh vertices is marked with the high bit, and from
// then on its vertices are scattered over random ranks (a random rank id in
// the bits under the high bit of the key, :224-234) while zone-change records
// for it are replicated to every such salted key (:240-265) — so no single
// rank has to reduce a giant zone. Per iteration: 2 collates to attach the
// current zone to both ends of every edge, a winner reduce that emits
// (loser zone -> winner zone) pairs, and a salted collate + reassign reduce.
// Every callback is a batch callback on device tensors.
class CCFindMR : public Command {
 public:
  CCFindMR(Oink& o) : Command(o) { ninputs = noutputs = 1; }
  int64_t nthresh = 0;
  void params(const Args& a) override {
    if (a.size() != 1) throw Error("Illegal cc_find_mr command");
    nthresh = lval(a[0], "cc_find_mr");
  }
  void run() override {
    constexpr int64_t HIBIT = std::numeric_limits<int64_t>::min();  // bit 63
    const int64_t P = nprocs;
    int pbits = 0;
    while ((int64_t(1) << pbits) < P) ++pbits;
    const int pshift = 63 - pbits;                         // rank id sits just under the high bit
    const int64_t lmask = (int64_t)(~0ull >> (pbits + 1));  // strips the high bit and the rank id
    MapReduce& mre = obj.input(1, rd(parse_edge), rc(parse_edge));
    MapReduce& mrv = obj.create_mr();
    MapReduce& mrz = obj.create_mr();
    const at::Device dev = comm->device();
    // every vertex starts in its own zone
    mrv.map_mr_batch(mre, [](const KV& src, KeyValue& kv) {
      if (!src.n) return;
      at::Tensor e = edges_of(src);
      add_tensors(kv, at::cat({e.select(1, 0), e.select(1, 1)}));
    });
    mrv.collate();
    mrv.reduce_batch([](const KMV& m, KeyValue& kv) {
      if (m.nkey) add_tensors(kv, m.keys.kdata.view(at::kLong), m.keys.kdata.view(at::kLong));
    });
    int niter = 0;
    while (true) {
      ++niter;
      // (v, edge) for both ends + (v, zone): the zone rides along to every edge
      mrz.map_mr_batch(mre, [](const KV& src, KeyValue& kv) {
        if (!src.n) return;
        at::Tensor e = edges_of(src);
        add_tensors(kv, at::cat({e.select(1, 0), e.select(1, 1)}), at::cat({e, e}));
      });
      mrz.add(mrv);
      mrz.collate();
      mrz.reduce_batch([](const KMV& m, KeyValue& kv) {  // reduce_edge_zone: (edge, zone of this end)
        if (!m.nval) return;
        auto [ed, zn] = ccmr_edge_zone(m);
        if (ed.numel()) add_tensors(kv, ed, zn);
      });
      mrz.collate();
      int64_t changed = 0;
      mrz.reduce_batch([&](const KMV& m, KeyValue& kv) {  // reduce_zone_winner
        if (!m.nkey) return;
        auto [big, pad] = ccmr_winner(m);  // value = PAD {winner zone, 0}: 16 bytes tell it apart from a vertex
        changed += big.numel();
        if (big.numel()) add_tensors(kv, big, pad);
      });
      if (comm->allreduce(changed, Comm::SUM) == 0) break;
      // vertices of hot zones go to a random salted copy of their zone key
      const uint64_t seed = 0x9E3779B97F4A7C15ull * (uint64_t)(niter + 1) ^ (123456789ull + (uint64_t)me);
      mrv.map_mr_batch(mrv, [&](const KV& src, KeyValue& kv) {  // map_invert_multi
        if (!src.n) return;
        auto [key, v] = ccmr_invert(src, (int)P, pshift, seed);
        add_tensors(kv, key, v);
      });
      mrv.map_mr_batch(mrz, [&](const KV& src, KeyValue& kv) {  // map_zone_multi: replicate to every salted key
        if (!src.n) return;
        auto [key, pad] = ccmr_zone_multi(src, (int)P, pshift);
        add_tensors(kv, key, pad);
      }, 1);
      mrv.collate();
      mrv.reduce_batch([&](const KMV& m, KeyValue& kv) {  // reduce_zone_reassign
        if (!m.nkey) return;
        auto [v, zone] = ccmr_reassign(m, lmask, nthresh);
        if (v.numel()) add_tensors(kv, v, zone);
      });
    }
    mrv.map_mr_batch(mrv, [&](const KV& src, KeyValue& kv) {  // map_strip
      if (src.n) add_tensors(kv, src.kdata.view(at::kLong), at::bitwise_and(src.vdata.view(at::kLong), ~HIBIT));
    });
    obj.output(1, mrv, print_vertex_u64);
    uint64_t ncc = 0;
    {
      MapReduce& mrc = obj.create_mr();
      mrc.map_mr_batch(mrv, [](const KV& src, KeyValue& kv) {
        if (src.n) add_tensors(kv, src.vdata.view(at::kLong), src.kdata.view(at::kLong));
      });
      ncc = mrc.collate();
    }
    (void)dev;
    message(fmt("CC_find: %" PRIu64 " components in %d iterations", ncc, niter));
    obj.cleanup();
  }
};

class CCStats : public Command {  // oink/cc_stats.cpp:37-62
 public:
  CCStats(Oink& o) : Command(o) { ninputs = 1; }
  void run() override {
    MapReduce& mrv = obj.input(1, rd(parse_vertex_vertex), rc(parse_vertex_vertex));
    MapReduce& mr = obj.create_mr();
    const uint64_t nvert = mr.map_mr_batch(mrv, invert);
    const uint64_t ncc = mr.collate();
    mr.reduce_builtin("count", "");
    mr.map_mr_batch(mr, invert);
    mr.collate();
    mr.reduce_builtin("count", "");
    mr.gather(1);
    mr.sort_keys(-1);
    message(fmt("CCStats: %" PRIu64 " components, %" PRIu64 " vertices", ncc, nvert));
    print_histo(oink, mr, "  %d CCs with %d vertices");
    obj.cleanup();
  }
};

// luby_find seed: maximal independent set (oink/luby_find.cpp:53-97)
class LubyFind : public Command {
 public:
  LubyFind(Oink& o) : Command(o) { ninputs = noutputs = 1; }
  int64_t seed = 0;
  void params(const Args& a) override {
    if (a.size() != 1) throw Error("Illegal luby_find command");
    seed = lval(a[0], "luby_find");
  }
  void run() override {
    MapReduce& mre = obj.input(1, rd(parse_edge), rc(parse_edge));
    mre.flatten();
    at::Tensor e = mre.kv ? edges_of(*mre.kv) : at::empty({0, 2}, opt(comm->device(), at::kLong));
    e = e.index({e.select(1, 0) != e.select(1, 1)});
    const int64_t N = nvert_global(*comm, e);
    EdgePlan plan(comm, e, N, std::nullopt, true);
    at::Tensor pres = present(plan);
    auto [mis, niter] = luby_mis(plan, seed, pres);
    at::Tensor ids = plan.local_ids.index({mis});
    MapReduce& mrv = obj.create_mr();
    mrv.open();  // winners are added from outside any map (reference :314)
    if (ids.numel()) add_tensors(mrv.kv_open(), ids);
    const uint64_t nset = mrv.close();
    obj.output(1, mrv, print_vertex);
    message(fmt("Luby_find: %" PRIu64 " MIS vertices in %d iterations", nset, niter));
    obj.cleanup();
  }
};

// sssp ncnt seed -i weighted-edges -o file mr: single-source shortest paths
// from ncnt random sources with out-edges (oink/sssp.cpp:49-184). Output
// lines are "v distance predecessor" as the reference prints them
// (oink/sssp.cpp:405-411); the source's predecessor is 0 (DISTANCE()).
class SSSP : public Command {
 public:
  SSSP(Oink& o) : Command(o) { ninputs = noutputs = 1; }
  int64_t ncnt = 0, seed = 0;
  void params(const Args& a) override {
    if (a.size() != 2) throw Error("Illegal sssp command");
    ncnt = lval(a[0], "sssp");
    seed = lval(a[1], "sssp");
  }
  void run() override {
    MapReduce& mre = obj.input(1, rd(parse_edge_weight), rc(parse_edge_weight));
    const at::Device dev = comm->device();
    mre.flatten();
    at::Tensor e = mre.kv ? edges_of(*mre.kv) : at::empty({0, 2}, opt(dev, at::kLong));
    at::Tensor w = (mre.kv && mre.kv->vw == 8) ? mre.kv->vdata.view(at::kDouble)
                                               : at::ones({e.size(0)}, opt(dev, at::kDouble));
    const int64_t N = nvert_global(*comm, e);
    EdgePlan plan(comm, e, N, w, false);
    at::Tensor outdeg = bincount_dev(plan.src, plan.nlocal);
    at::Tensor cand = plan.local_ids.index({outdeg > 0}).contiguous();
    at::Tensor all = comm->allgather_var(cand).to(at::kCPU);
    std::vector<int64_t> c(all.data_ptr<int64_t>(), all.data_ptr<int64_t>() + all.numel());
    std::sort(c.begin(), c.end());
    std::mt19937_64 rng((uint64_t)seed);
    std::shuffle(c.begin(), c.end(), rng);
    if ((int64_t)c.size() > ncnt) c.resize((size_t)ncnt);
    MapReduce& mr = obj.create_mr();
    for (size_t i = 0; i < c.size(); ++i) {
      const int64_t s = c[i];
      auto [d, niter] = sssp(plan, s);
      at::Tensor ok = at::isfinite(d);
      const int64_t nlab = comm->allreduce(ok.sum().item<int64_t>(), Comm::SUM);
      message(fmt("%zu:  Source = %" PRId64 "; Iterations = %d; Num Vtx Labeled = %" PRId64, i, s, niter, nlab));
      at::Tensor pred = sssp_predecessors(plan, e, w, d, s);
      at::Tensor ids = plan.local_ids.index({ok}), dd = d.index({ok});
      at::Tensor vals = at::stack({dd.view(at::kLong), pred.index({ok})}, 1);
      mr.map(
          nprocs,
          [&](int, KeyValue& kv) {
            if (ids.numel()) add_tensors(kv, ids, vals);
          },
          1);
    }
    obj.output(1, mr, print_sssp);
    obj.cleanup();
  }
};

// sssp_mr ncnt seed -i weighted-edges -o file mr: the reference's MapReduce
// formulation of SSSP (oink/sssp.cpp:49-184), the one pipeline that puts in
// one loop an aggregate, cross-MR appends (kv->append/complete: open(1) /
// kv_open / close here), compress as the combiner and an Allreduce
// termination. Per iteration: aggregate the candidate distances (mrpath) to
// their vertices' ranks; move them into mrvert; compress mrvert with
// pick_shortest_distances, which emits every vertex's winner back and the
// changed ones into mrpath; stop when no rank changed any (close() counts
// over all ranks); else move mrpath into mredge (aggregated by source vertex)
// and compress it with update_adjacent_distances, which re-emits the edges
// and emits relaxed distances of the changed vertices' neighbours into mrpath.
// Both compress callbacks are batch callbacks on device tensors
// (graphmr.hip). Sources are picked as by `sssp` (vertices with out-edges,
// shuffled by seed), so the two commands' outputs line up; the output is the
// labelled vertices' "v distance predecessor" lines (the reference prints its
// last mrpath, which is empty when the loop ends, oink/sssp.cpp:170-173).
double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

class SSSPMR : public Command {
 public:
  SSSPMR(Oink& o) : Command(o) { ninputs = noutputs = 1; }
  int64_t ncnt = 0, seed = 0;
  void params(const Args& a) override {
    if (a.size() != 2) throw Error("Illegal sssp_mr command");
    ncnt = lval(a[0], "sssp_mr");
    seed = lval(a[1], "sssp_mr");
  }
  void run() override {
    constexpr double FLTMAX = 3.4028234663852886e+38;  // DISTANCE()'s weight (oink/sssp.h:50-54)
    const at::Device dev = comm->device();
    MapReduce& mre = obj.input(1, rd(parse_edge_weight), rc(parse_edge_weight));
    // vertices from the edges (edge_to_vertices + collate + cull, :63-66)
    MapReduce& mrvert = obj.create_mr();
    mrvert.map_mr_batch(mre, [](const KV& src, KeyValue& kv) {
      if (!src.n) return;
      at::Tensor e = edges_of(src);
      add_tensors(kv, at::cat({e.select(1, 0), e.select(1, 1)}));
    });
    mrvert.collate();
    mrvert.reduce_batch([](const KMV& m, KeyValue& kv) {
      if (m.nkey) add_tensors(kv, m.keys.kdata.view(at::kLong));
    });
    // edges by source vertex: Vi -> EDGEVALUE {Vj, wt} (reorganize_edges + aggregate, :75-76)
    MapReduce& mredge = obj.create_mr();
    mredge.map_mr_batch(mre, [](const KV& src, KeyValue& kv) {
      if (!src.n) return;
      at::Tensor e = edges_of(src);
      at::Tensor w = src.vw == 8 ? src.vdata.view(at::kLong)
                                 : at::full({src.n}, (double)1.0, src.kdata.options().dtype(at::kDouble)).view(at::kLong);
      add_tensors(kv, e.select(1, 0), at::stack({e.select(1, 1), w}, 1));
    });
    mredge.aggregate();
    // sources: the distinct source vertices of the edges, every rank's, shuffled by seed
    std::vector<int64_t> c;
    {
      MapReduce& mrs = obj.create_mr();
      mrs.map_mr_batch(mredge, [](const KV& src, KeyValue& kv) {
        if (src.n) add_tensors(kv, src.kdata.view(at::kLong));
      });
      at::Tensor mine = at::empty({0}, opt(dev, at::kLong));
      mrs.compress_batch([&](const KMV& m, KeyValue&) {
        if (m.nkey) mine = at::cat({mine, m.keys.kdata.view(at::kLong).to(dev)});
      });
      at::Tensor all = comm->allgather_var(mine.contiguous()).to(at::kCPU);
      c.assign(all.data_ptr<int64_t>(), all.data_ptr<int64_t>() + all.numel());
      std::sort(c.begin(), c.end());
      std::mt19937_64 rng((uint64_t)seed);
      std::shuffle(c.begin(), c.end(), rng);
      if ((int64_t)c.size() > ncnt) c.resize((size_t)ncnt);
    }
    MapReduce& mrpath = obj.create_mr();
    MapReduce& mrout = obj.create_mr();
    const int64_t inf_bits = [&] {
      int64_t b;
      std::memcpy(&b, &FLTMAX, 8);
      return b;
    }();
    double tcompute = 0;
    for (size_t i = 0; i < c.size(); ++i) {
      const int64_t source = c[i];
      const double t0 = now_s();
      // every vertex unreached, current (initialize_vertex_distances, :94)
      mrvert.map_mr_batch(mrvert, [&](const KV& src, KeyValue& kv) {
        if (!src.n) return;
        at::Tensor d = at::empty({src.n, 3}, src.kdata.options().dtype(at::kLong));
        d.select(1, 0).fill_(0);
        d.select(1, 1).fill_(inf_bits);
        d.select(1, 2).fill_(1);
        add_tensors(kv, src.kdata.view(at::kLong), d);
      });
      // the source at distance 0, not yet current (add_source, :100)
      mrpath.map(1, [&](int, KeyValue& kv) {
        double z = 0.0;
        int64_t d[3] = {0, 0, 0};
        std::memcpy(&d[1], &z, 8);
        kv.add((const char*)&source, 8, (const char*)d, 24);
      });
      int iter = 0;
      while (true) {
        ++iter;
        mrpath.aggregate();
        mrvert.open(1);  // mrvert->kv->append(); mrpath->map(move_to_new_mr) (:112-114)
        mrpath.map_mr_batch(mrpath, [&](const KV& src, KeyValue&) {
          if (src.n) mrvert.kv_open().add_kv(src);
        });
        mrvert.close();
        mrpath.open();
        mrvert.compress_batch([&](const KMV& m, KeyValue& kv) {  // pick_shortest_distances (:120-122)
          if (!m.nkey) return;
          SsspPick p = ssspmr_pick(m);
          add_tensors(kv, m.keys.kdata.view(at::kLong), p.dist);
          if (p.ckeys.numel()) add_tensors(mrpath.kv_open(), p.ckeys, p.cdist);
        });
        const uint64_t nchanged = mrpath.close();  // summed over ranks (:124-126)
        if (nchanged == 0) break;
        mredge.open(1);  // mredge->kv->append(); mrpath->map(move_to_new_mr) (:131-133)
        mrpath.map_mr_batch(mrpath, [&](const KV& src, KeyValue&) {
          if (src.n) mredge.kv_open().add_kv(src);
        });
        mredge.close();
        mrpath.open();
        mredge.compress_batch([&](const KMV& m, KeyValue& kv) {  // update_adjacent_distances (:135-137)
          if (!m.nkey) return;
          SsspRelax r = ssspmr_relax(m);
          if (r.ekeys.numel()) add_tensors(kv, r.ekeys, r.edges);
          if (r.pkeys.numel()) add_tensors(mrpath.kv_open(), r.pkeys, r.paths);
        });
        mrpath.close();
      }
      tcompute += now_s() - t0;
      // labelled vertices -> (v, {distance, predecessor}) (print, :405-411)
      int64_t nlab = 0;
      mrout.map_mr_batch(
          mrvert,
          [&](const KV& src, KeyValue& kv) {
            if (!src.n) return;
            at::Tensor d = src.vdata.view(at::kLong).view({-1, 3});
            at::Tensor w = d.select(1, 1).contiguous().view(at::kDouble);
            at::Tensor ok = w < FLTMAX;
            at::Tensor ids = src.kdata.view(at::kLong).index({ok});
            nlab += ids.numel();
            if (ids.numel()) add_tensors(kv, ids, at::stack({d.select(1, 1).index({ok}), d.select(1, 0).index({ok})}, 1));
          },
          1);
      nlab = comm->allreduce(nlab, Comm::SUM);
      message(fmt("%zu:  Source = %" PRId64 "; Iterations = %d; Num Vtx Labeled = %" PRId64, i, source, iter, nlab));
    }
    message(fmt("Total time in SSSP: %g", tcompute));
    obj.output(1, mrout, print_sssp);
    obj.cleanup();
  }
};

// luby_find_mr seed -i edges -o file mr: the reference's MapReduce formulation
// of Luby's maximal independent set (oink/luby_find.cpp:53-97). Every vertex
// gets the reference's random number (drand48() after srand48(v + seed)),
// edges become ERAND keys; per iteration four reduce + collate rounds: edge
// winners (the end with the smaller (r, v)), vertices that won all their
// edges, their neighbours (losers), and the emit round that adds the winners
// to mrv — a second MR kept open across the whole loop (mrv->open() ...
// close(), :73/:88) — and sends the edges back, flagged when an end was
// removed. The loop ends when no live edge is left (reduce's global count).
// The result is the greedy MIS in (r, v) order, so it is the reference's set
// for the same seed. Self loops are dropped (the reference can loop forever on
// one); an edge is deleted when any of its values is a flag (the reference
// checks the first two only).
class LubyFindMR : public Command {
 public:
  LubyFindMR(Oink& o) : Command(o) { ninputs = noutputs = 1; }
  int64_t seed = 0;
  void params(const Args& a) override {
    if (a.size() != 1) throw Error("Illegal luby_find_mr command");
    seed = lval(a[0], "luby_find_mr");
  }
  void run() override {
    MapReduce& mre = obj.input(1, rd(parse_edge), rc(parse_edge));
    MapReduce& mrv = obj.create_mr();
    MapReduce& mrw = obj.create_mr();
    mrw.map_mr_batch(mre, [&](const KV& src, KeyValue& kv) {  // map_vert_random (:120-136)
      if (!src.n) return;
      at::Tensor er = lubymr_random(edges_of(src), seed);
      if (er.size(0)) add_tensors(kv, er);
    });
    mrw.clone();
    int niter = 0;
    mrv.open();
    while (true) {
      const uint64_t n = mrw.reduce_batch([](const KMV& m, KeyValue& kv) {  // reduce_edge_winner
        if (!m.nkey) return;
        auto [k, v] = lubymr_edge_winner(m);
        if (k.size(0)) add_tensors(kv, k, v);
      });
      if (n == 0) break;
      for (bool loser : {false, true}) {  // reduce_vert_winner, reduce_vert_loser
        mrw.collate();
        mrw.reduce_batch([&](const KMV& m, KeyValue& kv) {
          if (!m.nkey) return;
          LubyVert r = lubymr_vert(m, loser);
          if (r.k24.size(0)) add_tensors(kv, r.k24, r.v24);
          if (r.k16.size(0)) add_tensors(kv, r.k16, r.v16);
        });
      }
      mrw.collate();
      mrw.reduce_batch([&](const KMV& m, KeyValue& kv) {  // reduce_vert_emit
        if (!m.nkey) return;
        LubyEmit r = lubymr_emit(m);
        if (r.mis.numel()) add_tensors(mrv.kv_open(), r.mis);
        if (r.kflag.size(0)) add_tensors(kv, r.kflag, r.fval);
        if (r.knull.size(0)) add_tensors(kv, r.knull);
      });
      mrw.collate();
      ++niter;
    }
    const uint64_t nset = mrv.close();
    obj.output(1, mrv, print_vertex);
    message(fmt("Luby_find: %" PRIu64 " MIS vertices in %d iterations", nset, niter));
    obj.cleanup();
  }
};

// pagerank tol maxiter alpha -i edges -o file mr (the reference command is a
// stub, oink/pagerank.cpp:54-56; implemented per oinkdoc/pagerank.txt)
class PageRankCmd : public Command {
 public:
  PageRankCmd(Oink& o) : Command(o) { ninputs = noutputs = 1; }
  double tol = 0, alpha = 0.85;
  int maxiter = 0;
  void params(const Args& a) override {
    if (a.size() != 3) throw Error("Illegal pagerank command");
    tol = dval(a[0], "pagerank");
    maxiter = (int)lval(a[1], "pagerank");
    alpha = dval(a[2], "pagerank");
  }
  void run() override {
    MapReduce& mre = obj.input(1, rd(parse_edge), rc(parse_edge));
    mre.flatten();
    at::Tensor e = mre.kv ? edges_of(*mre.kv) : at::empty({0, 2}, opt(comm->device(), at::kLong));
    const int64_t N = nvert_global(*comm, e);
    PageRankPlan pr(comm, e, N, alpha);
    const int niter = pr.run(maxiter, tol);
    at::Tensor ids = pr.ids(), r = pr.ranks().to(at::kDouble);
    MapReduce& mrr = obj.create_mr();
    mrr.map(nprocs, [&](int, KeyValue& kv) {
      if (ids.numel()) add_tensors(kv, ids, r);
    });
    obj.output(1, mrr, print_vertex_double);
    message(fmt("PageRank: %" PRId64 " vertices, %d iterations, L1 delta %g", N, niter, pr.delta()));
    obj.cleanup();
  }
};

template <typename T>
CommandFactory factory() {
  return [](Oink& o) { return std::unique_ptr<Command>(new T(o)); };
}

struct Registrar {
  Registrar() {
    auto& r = command_registry();
    r["rmat"] = factory<RMAT>();
    r["rmat2"] = factory<RMAT2>();
    r["edge_upper"] = factory<EdgeUpper>();
    r["degree"] = factory<Degree>();
    r["degree_stats"] = factory<DegreeStats>();
    r["degree_weight"] = factory<DegreeWeight>();
    r["histo"] = factory<Histo>();
    r["wordfreq"] = factory<WordFreq>();
    r["vertex_extract"] = factory<VertexExtract>();
    r["neighbor"] = factory<Neighbor>();
    r["neigh_tri"] = factory<NeighTri>();
    r["tri_find"] = factory<TriFind>();
    r["tri_find_mr"] = factory<TriFindMR>();
    r["cc_find"] = factory<CCFind>();
    r["cc_find_mr"] = factory<CCFindMR>();
    r["cc_stats"] = factory<CCStats>();
    r["luby_find"] = factory<LubyFind>();
    r["sssp"] = factory<SSSP>();
    r["sssp_mr"] = factory<SSSPMR>();
    r["luby_find_mr"] = factory<LubyFindMR>();
    r["pagerank"] = factory<PageRankCmd>();
  }
} registrar;

}  // namespace
}  // namespace oink
}  // namespace mrh
