// MapReduce triangle finder (see trifind_mr.h).
#include "trifind_mr.h"

#include "callbacks.h"
#include "engine/comm.h"
#include "engine/tri.h"

namespace mrh {
namespace oink {

TriMRRun tri_find_mr(MapReduce& mre, MapReduce& mrt, bool upper) {
  TriMRRun run;
  const Comm& comm = *mrt.comm();
  auto npairs = [&](MapReduce& m) -> int64_t {
    const int64_t n = m.kv ? m.kv_rows() : m.kmv ? m.kmv->nkey : 0;
    return comm.allreduce(n, Comm::SUM);
  };
  // one stage: the op, then a device sync so its kernels count in its time
  auto stage = [&](const char* name, MapReduce& m, const std::function<void()>& op) {
    TriMRStage s;
    s.op = name;
    s.pairs_in = npairs(m);
    comm.host_wait();
    comm.barrier();
    const double t0 = Comm::wtime();
    op();
    comm.host_wait();
    comm.barrier();
    s.seconds = Comm::wtime() - t0;
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
  stage("reduce nsq_angles", mrt, [&] {
    mrt.reduce_batch([](const KMV& m, KeyValue& kv) {  // O(d^2) wedges, load-balanced kernel
      if (!m.nkey) return;
      // under a page budget the wedges go out in spool pieces (24 B a wedge)
      const int64_t chunk = kv.piece_bytes() / 24;
      for_each_wedge_chunk(m.seg, m.vdata.view(at::kLong), m.keys.kdata.view(at::kLong), chunk,
                           [&](const at::Tensor& e, const at::Tensor& c) { add_tensors(kv, e, c); });
    });
  });
  stage("add edges", mrt, [&] {
    // the reference adds the edge MR unchanged (oink/tri_find.cpp:71): the
    // marked copies go through a temporary MR, the input is left as it was.
    // An upper edge (vi < vj) carries vi as its marker, not an empty value:
    // every pair of collate 4 then has one narrow 8-byte value and the
    // collate groups them as packed (edge, vertex) words. A wedge centre is
    // never vi then (the centre of wedge (vi, vj) is a third vertex), but it
    // can be when some edge is not upper (self-loops, vi > vj): then, on
    // every rank alike, edges carry the reference's empty value instead.
    int64_t bad = 0;
    if (mre.kv && mre.kv->n) {
      mre.flatten();
      at::Tensor e = edges_of(*mre.kv);
      bad = (e.select(1, 0) >= e.select(1, 1)).any().item<bool>() ? 1 : 0;
    }
    const bool marked_by_vertex = comm.allreduce(bad, Comm::MAX) == 0;
    MapReduce marked(mre.comm());
    marked.set = mre.set;
    marked.map_mr_batch(mre, [&](const KV& src, KeyValue& kv) {
      if (!src.n) return;
      at::Tensor e = edges_of(src);
      if (marked_by_vertex) {
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
    run.triangles = mrt.reduce_batch([](const KMV& m, KeyValue& kv) {
      at::Tensor tri = trimr_emit(m);
      if (tri.size(0)) add_tensors(kv, tri);
    });
  });
  return run;
}

}  // namespace oink
}  // namespace mrh
