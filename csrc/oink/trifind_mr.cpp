// MapReduce triangle finder (see trifind_mr.h).
#include "trifind_mr.h"

#include <cstdlib>

#include "callbacks.h"
#include "engine/comm.h"
#include "engine/tri.h"
#include "engine/spool.h"
#include "engine/xfer.h"
#include "kernels/launch.h"

#include <ATen/hip/HIPContext.h>

namespace mrh {
namespace oink {

namespace {
hipStream_t stream() { return at::hip::getCurrentHIPStream(); }
at::TensorOptions like(const at::Tensor& t, at::ScalarType ty) { return at::TensorOptions().device(t.device()).dtype(ty); }
}  // namespace

TriMRRun tri_find_mr(MapReduce& mre, MapReduce& mrt, bool upper) {
  TriMRRun run;
  const Comm& comm = *mrt.comm();
  auto npairs = [&](MapReduce& m) -> int64_t {
    const int64_t n = m.kv ? m.kv_rows() : m.kmv ? m.kmv_keys() : 0;
    return comm.allreduce(n, Comm::SUM);
  };
  // one stage: the op, then a device sync so its kernels count in its time
  auto stage = [&](const char* name, MapReduce& m, const std::function<void()>& op) {
    TriMRStage s;
    s.op = name;
    s.pairs_in = npairs(m);
    comm.host_wait();
    comm.barrier();
    const XferCount x0 = xfer_count();
    const int64_t d0 = spool_totals().disk_bytes;
    const double t0 = Comm::wtime();
    op();
    comm.host_wait();
    comm.barrier();
    s.seconds = Comm::wtime() - t0;
    const XferCount x1 = xfer_count();
    s.h2d_bytes = x1.h2d - x0.h2d;
    s.d2h_bytes = x1.d2h - x0.d2h;
    s.disk_bytes = spool_totals().disk_bytes - d0;
    s.pairs_out = npairs(m);
    run.stages.push_back(s);
  };
  if (upper) {
    stage("map edge_upper", mre, [&] { mre.map_mr_batch(mre, edge_upper); });
    stage("collate 0", mre, [&] { mre.collate(); });
    stage("reduce cull", mre, [&] { mre.reduce_builtin("first", ""); });
  }
  stage("map_edge_vert", mrt, [&] {
    mrt.map_mr_batch(mre, [](const KV& src, KeyValue& kv) {  // (vi, vj) and (vj, vi)
      if (!src.n) return;
      at::Tensor e = edges_of(src);
      if (e.is_cuda() && e.is_contiguous()) {  // one kernel (util.hip), not two ATen cats of strided columns
        at::Tensor key = at::empty({2 * src.n}, like(e, at::kLong)), val = at::empty({2 * src.n}, like(e, at::kLong));
        k::edge_both_ways(e.data_ptr<int64_t>(), src.n, key.data_ptr<int64_t>(), val.data_ptr<int64_t>(), stream());
        add_tensors(kv, key, val);
        return;
      }
      add_tensors(kv, at::cat({e.select(1, 0), e.select(1, 1)}), at::cat({e.select(1, 1), e.select(1, 0)}));
    });
  });
  stage("collate 1", mrt, [&] { mrt.collate(); });
  stage("reduce first_degree", mrt, [&] {
    mrt.reduce_batch([](const KMV& m, KeyValue& kv) {  // edge -> {deg, 0} / {0, deg}
      if (!m.nval) return;
      auto [edge, deg] = trimr_first_degree(m);
      add_tensors(kv, edge, deg);
    });
  });
  stage("collate 2", mrt, [&] { mrt.collate(); });
  stage("reduce second_degree", mrt, [&] {
    mrt.reduce_batch([](const KMV& m, KeyValue& kv) {  // edge -> {di, dj}
      if (!m.nkey) return;
      add_tensors(kv, m.keys.kdata.view(at::kLong).view({-1, 2}), trimr_second_degree(m));
    });
  });
  stage("map low_degree", mrt, [&] {
    mrt.map_mr_batch(mrt, [](const KV& src, KeyValue& kv) {  // (lower-degree end, other end)
      if (!src.n) return;
      auto [key, val] = trimr_low_degree(src);
      add_tensors(kv, key, val);
    });
  });
  stage("collate 3", mrt, [&] { mrt.collate(); });
  // Edge markers and the layout of the last collate, decided on every rank
  // alike (allreduced). An upper edge (vi < vj) carries vi as its marker, not
  // an empty value: every pair of collate 4 then has one narrow value and the
  // collate groups them as packed (edge, vertex) words. A wedge centre is
  // never vi then (the centre of wedge (vi, vj) is a third vertex), but it
  // can be when some edge is not upper (self-loops, vi > vj): then edges
  // carry the reference's empty value instead. Compact layout (upper edges,
  // vertex ids below 2^32): an edge key is one word vi << vb | vj (vb = the
  // bits of the largest id) and a centre 4 bytes — a wedge is 12 bytes, not
  // 24 (R-MAT-22's ~6 G wedges fit in HBM); MRH_TRIMR_COMPACT=0 turns it off.
  int64_t bad = 0, vmax = 0;
  if (mre.kv_rows()) {
    mre.flatten();
    at::Tensor e = edges_of(*mre.kv);
    if (e.is_cuda() && e.is_contiguous()) {  // one pass, one small read (util.hip edge_probe)
      const int64_t n = std::min<int64_t>(e.size(0), mre.kv->n);
      at::Tensor tmp = at::empty({k::minmax_scratch_words(n, 3) + 3}, like(e, at::kLong));
      int64_t* res = tmp.data_ptr<int64_t>() + k::minmax_scratch_words(n, 3);
      k::edge_probe(e.data_ptr<int64_t>(), n, tmp.data_ptr<int64_t>(), res, stream());
      int64_t r[3];
      read_small(stream(), {{res, r, 24}});
      bad = (r[1] != 0 || r[0] < 0) ? 1 : 0;
      vmax = r[2];
    } else {
      bad = (e.select(1, 0) >= e.select(1, 1)).any().item<bool>() ? 1 : 0;
      bad = std::max<int64_t>(bad, (e.min().item<int64_t>() < 0) ? 1 : 0);
      vmax = e.max().item<int64_t>();
    }
  }
  const bool marked_by_vertex = comm.allreduce(bad, Comm::MAX) == 0;
  vmax = comm.allreduce(vmax, Comm::MAX);
  int vb = 1;
  while (vb < 63 && (vmax >> vb) != 0) ++vb;
  static const bool compact_env = [] {
    const char* e = std::getenv("MRH_TRIMR_COMPACT");
    return !(e && *e == '0');
  }();
  const bool compact = compact_env && marked_by_vertex && vb <= 32;
  run.compact_vb = compact ? vb : 0;
  stage("reduce nsq_angles", mrt, [&] {
    mrt.reduce_batch([&](const KMV& m, KeyValue& kv) {  // O(d^2) wedges, load-balanced kernel
      if (!m.nkey) return;
      // wedges are generated in bounded chunks (24 B a wedge while generated):
      // spool pieces under a page budget, 2^28 wedges otherwise
      if (compact) {  // 12 bytes a wedge, written so by the wedge kernel
        const int64_t chunk = kv.piece_bytes() ? kv.piece_bytes() / 12 : int64_t(1) << 29;
        for_each_wedge_chunk_compact(m.seg, m.vdata.view(at::kLong), m.keys.kdata.view(at::kLong), chunk, vb,
                                     [&](const at::Tensor& key, const at::Tensor& c) { add_tensors(kv, key, c); });
        return;
      }
      const int64_t chunk = kv.piece_bytes() / 24;
      for_each_wedge_chunk(m.seg, m.vdata.view(at::kLong), m.keys.kdata.view(at::kLong), chunk,
                           [&](const at::Tensor& e, const at::Tensor& c) { add_tensors(kv, e, c); });
    });
  });
  stage("add edges", mrt, [&] {
    // the reference adds the edge MR unchanged (oink/tri_find.cpp:71): the
    // marked copies go through a temporary MR, the input is left as it was
    MapReduce marked(mre.comm());
    marked.set = mre.set;
    marked.map_mr_batch(mre, [&](const KV& src, KeyValue& kv) {
      if (!src.n) return;
      at::Tensor e = edges_of(src);
      const bool dev = e.is_cuda() && e.is_contiguous();
      if (compact && dev) {  // key vi << vb | vj and the vi marker in one kernel
        at::Tensor key = at::empty({src.n}, like(e, at::kLong)), val = at::empty({src.n}, like(e, at::kInt));
        k::edge_pack(e.data_ptr<int64_t>(), src.n, vb, reinterpret_cast<uint64_t*>(key.data_ptr<int64_t>()),
                     val.data_ptr<int32_t>(), stream());
        add_tensors(kv, key, val);
      } else if (compact) {
        at::Tensor key = at::bitwise_or(at::bitwise_left_shift(e.select(1, 0), vb), e.select(1, 1));
        add_tensors(kv, key, e.select(1, 0).to(at::kInt));
      } else if (marked_by_vertex && dev) {
        at::Tensor val = at::empty({src.n}, like(e, at::kLong));
        k::edge_first(e.data_ptr<int64_t>(), src.n, val.data_ptr<int64_t>(), stream());
        add_tensors(kv, e, val);
      } else if (marked_by_vertex) {
        add_tensors(kv, e, e.select(1, 0).contiguous());
      } else {
        KV x = make_kv(e.contiguous().view(at::kByte).view({-1}), c10::nullopt,
                       at::empty({0}, at::TensorOptions().device(e.device()).dtype(at::kByte)),
                       at::zeros({src.n + 1}, at::TensorOptions().device(e.device()).dtype(at::kLong)), src.n,
                       e.device());
        kv.add_kv(x);
      }
    });
    mrt.add(marked);
  });
  stage("collate 4", mrt, [&] { mrt.collate(); });
  stage("reduce emit_triangles", mrt, [&] {
    run.triangles = mrt.reduce_batch([&](const KMV& m, KeyValue& kv) {
      at::Tensor tri = trimr_emit(m, compact ? vb : 0);
      if (tri.size(0)) add_tensors(kv, tri);
    });
  });
  return run;
}

}  // namespace oink
}  // namespace mrh
