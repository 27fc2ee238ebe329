// Native graph engines on top of the MapReduce primitives: the reusable
// "edge plan" for iterative propagation (CC, Luby MIS, SSSP), PageRank, and
// the replicated-CSR triangle finder. Used by the OINK commands (csrc/oink)
// and, through the bindings, by the Python models.
//
// Edge plan = the MapReduce dataflow of one propagation step
//     map      edge (i -> j)  ->  (j, f(x_i, w_ij))
//     combine  OP per j on the sender           (MR-MPI compress)
//     shuffle  to owner(j) = j % P               (RCCL all-to-all over xGMI)
//     reduce   OP per j on the owner
// whose keys never change between iterations: the sort / group / routing is
// built once, and each iteration moves only values (one fused gather +
// segmented-reduce kernel, one all-to-all, one combine kernel). The
// reference re-shuffles every edge 2-4 times per iteration
// (oink/cc_find.cpp:73-92, oink/sssp.cpp:49-184, oink/luby_find.cpp:53-97).
#pragma once
#include <hip/hip_runtime.h>
#include <ATen/ATen.h>

#include <optional>
#include <utility>
#include <vector>

#include "comm.h"
#include "kv.h"

namespace mrh {

enum PlanOp { PLAN_SUM = 0, PLAN_MIN = 1, PLAN_MAX = 2 };

class EdgePlan {
 public:
  // edges: this rank's [n,2] int64 (vi, vj), any distribution; weights: optional
  // per-edge values in the dtype of the propagated vectors
  EdgePlan(CommPtr comm, const at::Tensor& edges, int64_t nvert, const std::optional<at::Tensor>& weights,
           bool symmetric);
  // acc[v] = OP over in-edges (i -> v) of x[i] (+ w); vertices without in-edges get `identity`
  at::Tensor propagate(const at::Tensor& x, int op, double identity, bool use_weights) const;
  int64_t count_global(const at::Tensor& mask) const;

  CommPtr comm;
  int P, me;
  at::Device dev;
  int64_t N, nlocal, nedge = 0, ngrp = 0;
  at::Tensor src;        // int32 local source id per planned edge
  at::Tensor w;          // planned per-edge weights (undefined if none)
  at::Tensor seg;        // int64 [ngrp+1] groups of edges with the same destination
  at::Tensor local_ids;  // int64 global ids of this rank's vertices (v = i*P + me)

 private:
  at::Tensor vid_, rseg_, rperm_, rvid_;
  SegIndex six_;  // static-segment index of `seg` (device plans)
  std::vector<int64_t> send_splits_, recv_splits_;
};

// true when device plans should use the static-segment wave kernel
// (wavesegred.h); MRH_PLAN_KERNEL=tiles selects the generic segred kernel
bool use_seg_index(const at::Device& d);

// label(v) = min vertex id of v's component; returns (labels, iterations)
std::pair<at::Tensor, int> connected_components(const EdgePlan& plan, int max_iter = 100000);
// Luby's maximal independent set; returns (in_set bool, rounds)
std::pair<at::Tensor, int> luby_mis(const EdgePlan& plan, int64_t seed, const std::optional<at::Tensor>& active,
                                    int max_iter = 100000);
// Bellman-Ford from `source` over float64 weights; returns (dist with +inf, iterations)
std::pair<at::Tensor, int> sssp(const EdgePlan& plan, int64_t source, int max_iter = 1000000);

// predecessor of every local vertex on a shortest path from `source` (the
// reference's DISTANCE e.v, oink/sssp.cpp:405-411): the smallest u with an
// edge u -> v and d[u] + w(u,v) == d[v]; 0 for the source, -1 if unreached
at::Tensor sssp_predecessors(const EdgePlan& plan, const at::Tensor& edges, const at::Tensor& weights,
                             const at::Tensor& dist, int64_t source);

// PageRank on edges partitioned by source (oinkdoc/pagerank.txt; the
// reference command is a stub, oink/pagerank.cpp:54-56)
class PageRankPlan {
 public:
  PageRankPlan(CommPtr comm, const at::Tensor& edges, int64_t nvert, double alpha);
  ~PageRankPlan();
  PageRankPlan(const PageRankPlan&) = delete;
  PageRankPlan& operator=(const PageRankPlan&) = delete;
  void reset();
  void step();
  int run(int maxiter, double tol);
  double delta() const;
  at::Tensor ids() const;  // global ids of this rank's vertices, same order as ranks()
  at::Tensor ranks() const { return r_; }

  CommPtr comm;
  int P, me;
  at::Device dev;
  int64_t N, nlocal, nedge = 0, ndangling = 0;
  double alpha;

 private:
  at::Tensor order_, src_, w_, seg_, send_, recv_, rseg_, rperm_, rvid_, vid_, dangling_, invdeg_, acc_;
  at::Tensor r_, rn_, c_, dmass_, stats_;
  SegIndex six_;
  std::vector<int64_t> send_splits_, recv_splits_;
  // XCD source ranges (one GPU): R = xr_ ranges, combine tiles, (range, tile)
  // group offsets, destination (new id) per group, gather schedule
  int64_t xr_ = 0, xtile_ = 0, xslen_ = 0;
  at::Tensor xoff_, ghi_, xsched_, part_;
  // one XCD-path iteration from r into rn (no host work, no allocation)
  void launch_iter(const at::Tensor& r, at::Tensor& rn);
  // HIP graph of two iterations (r_ -> rn_ -> r_), replayed by run() for a
  // fixed iteration count; rebuilt if the buffers it captured moved
  bool graph_ok() const;
  void graph_build();
  void graph_free();
  hipGraphExec_t gexec_ = nullptr;
  hipStream_t gstream_ = nullptr;
  hipEvent_t gev_[2] = {nullptr, nullptr};
  std::vector<const void*> gkey_;
  int64_t graph_iters_ = 0;
  // maxr_cap: at most this many ranges (hot + cold)
  void xcd_ranges(const at::Tensor& degn, int64_t nactive, int dbits, std::vector<int64_t>& rb,
                  std::vector<int64_t>& redge, int maxr_cap = 64);
  void xcd_schedule(const std::vector<int64_t>& redge);
  // the 8 x slen wave schedule of n edges whose ranges start at redge
  // (redge.back() = n): hot range r on XCD slot (r_base + r) % 8, then (if
  // last_cold) the cold range's waves round-robin
  std::pair<at::Tensor, int64_t> wave_schedule(const std::vector<int64_t>& redge, int64_t n, int r_base = 0,
                                               bool last_cold = true) const;
  // the plan from this rank's edges (source-owned): device kernels, or the
  // tensor-op twin on the CPU engine
  void build_device(const at::Tensor& e);
  void build_host(const at::Tensor& e);
  // out-degrees (partitioned count, or run lengths of a source sort) and the
  // degree relabel (both device builds); relabel returns the local dangling count
  at::Tensor out_degrees(at::Tensor& packed, bool sorted_by_source);
  static bool degrees_by_sort();
  // sorted (group key << 32 | source) -> src_, seg_ and the head bitmap heads_
  void unpack_sorted(const at::Tensor& sorted);
  at::Tensor heads_;  // until the segment index takes it
  int64_t relabel_by_degree(at::Tensor deg, bool want_degn, at::Tensor& nid, at::Tensor& degn);
  // several GPUs: destination-owned edges, replicated c vector (graphplan.cpp)
  void build_device_dist(const at::Tensor& e);
  void launch_iter_dist(const at::Tensor& r, at::Tensor& rn);
  bool dist_dev_ = false, mix_ = false;
  int64_t S_ = 0;      // c slice length per rank
  at::Tensor cfull_;   // the replicated c vector, P slices of S_ (+ slack)
  // several GPUs: the edges cut into K pieces by source chunk (chunk j = new
  // ids [chunk_b_[j], chunk_b_[j + 1]) of every rank, about equal edge
  // counts: consecutive XCD ranges of the one-GPU plan), each with its own
  // segment index, schedule and 16-byte aligned source stream; the c exchange runs on side_ in K rounds (round j: chunk j of
  // every slice, to and from every peer at once) and piece j is gathered as
  // soon as round j has landed (MRH_PR_OVERLAP=0: one all-gather after the
  // tile step, then one gather)
  struct Piece {
    SegIndex six;
    at::Tensor src;
    int64_t g0 = 0, ng = 0, n = 0;  // first group, groups, edges
  };
  std::vector<Piece> pieces_;
  std::vector<int64_t> chunk_b_;
  at::Tensor srcp_;
  bool c_fresh_ = true;  // cfull_ holds every rank's slice of the last tile step
  bool dist_warm_ = false, dist_graph_failed_ = false;  // eager exchange rounds ran (RCCL connections exist)
  std::vector<const void*> graph_key() const;
  hipStream_t side_ = nullptr;
  std::vector<hipEvent_t> ring_ev_;
  void build_pieces(const std::vector<int>& piece_nr);
  void ring_start();
  void ring_free();
  // several ranks: the destination-owner side of the exchange from the
  // group destinations ujv (global ids) and the new id of every old local id
  void build_exchange(const at::Tensor& ujv, const at::Tensor& new_of_old);
  // propagation blocking (one GPU; pbpr.hip): phase-1 sources and slots,
  // phase-2 16-bit destinations, contributions, work units
  void build_blocking(const at::Tensor& dst_new);
  bool pb_ = false;
  at::Tensor pb_src_, pb_out_, pb_dst_, pb_vals_, pb_ub_, pb_ue0_, pb_ue1_, pb_uex_;
  int64_t pb_nunit_ = 0;

 public:
  bool blocking() const { return pb_; }
  // "replicated" (multi-GPU: destination-owned edges + all-gathered c),
  // "partials" (source-owned + all-to-all of partial sums), "local"
  std::string layout() const { return dist_dev_ ? "replicated" : comm->distributed() ? "partials" : "local"; }
  int64_t c_slice() const { return S_; }
  // bytes this rank receives per iteration (the c slices of the other ranks
  // and the 16-byte stats allreduce; 0 on one rank)
  int64_t comm_bytes_per_iter() const { return dist_dev_ && P > 1 ? (int64_t)(P - 1) * S_ * 4 + 16 : 0; }
  bool overlapped() const { return !pieces_.empty(); }
  int64_t xcd_ranges_count() const { return xr_; }
  // fixed-count run() replays a captured HIP graph (MRH_PR_GRAPH=0: off)
  bool use_graph = true;
  int64_t graph_iterations() const { return graph_iters_; }
};

// Triangle finder on a degree-oriented CSR (tri.cpp kernels). Multi-rank jobs
// build it distributed (owned rows + fetched halo rows, O(E/P + halo) per
// rank); MRH_TRI_REPLICATED=1 (or a single rank) replicates the whole graph.
class TriangleGraph {
 public:
  TriangleGraph(CommPtr comm, const at::Tensor& edges, int64_t nvert = -1);
  int64_t count() const;          // global triangle count
  at::Tensor triangles() const;   // this rank's triangles [T,3] int64 original ids, rows ascending

  CommPtr comm;
  int64_t nvert = 0, nedge = 0, e0 = 0, e1 = 0;
  bool distributed = false;
  int64_t nlocal = 0, nrows = 0;  // distributed: owned rows, owned + halo rows
  at::Tensor rowptr, col, okeys, perm, row_gid;
  // split build: the CSR is whole on every rank, okeys holds this rank's rows
  // [u0_, u1_) only
  bool split = false;
  int64_t u0_ = 0, u1_ = 0;

 private:
  void build_distributed(const at::Tensor& lo, const at::Tensor& hi);
  void build_split(const at::Tensor& packed);
  static std::vector<int64_t> work_split(const at::Tensor& d, int64_t P);
};

}  // namespace mrh
