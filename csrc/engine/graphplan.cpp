// Native graph engines (see graphplan.h).
#include "graphplan.h"
#include "hbmpool.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <stdexcept>

#include <ATen/hip/HIPContext.h>
#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPStream.h>

#include "../kernels/launch.h"
#include "tri.h"

namespace mrh {

namespace {
constexpr int64_t VMASK = (int64_t(1) << 40) - 1;
at::TensorOptions opt(at::Device d, at::ScalarType t) { return at::TensorOptions().device(d).dtype(t); }

// MRH_PR_STAGES=1: device-synchronised wall time of every plan-build stage on
// stderr (the setup breakdown of profiles/r4_pagerank_setup_stages.txt)
struct StageClock {
  bool on = false;
  double t = 0;
  StageClock() {
    const char* e = std::getenv("MRH_PR_STAGES");
    on = e && *e == '1';
    if (on) {
      (void)hipDeviceSynchronize();
      t = Comm::wtime();
    }
  }
  void operator()(const char* what) {
    if (!on) return;
    (void)hipDeviceSynchronize();
    const double now = Comm::wtime();
    std::fprintf(stderr, "mrhip PageRankPlan stage %-22s %8.2f ms\n", what, 1e3 * (now - t));
    t = now;
  }
};

at::Tensor iota32(int64_t n, at::Device d) { return at::arange(n, opt(d, at::kInt)); }

// stable (keys, perm) sort; tolerates n == 0
std::pair<at::Tensor, at::Tensor> sort_with_perm(const at::Tensor& key, int end_bit = 64) {
  const int64_t n = key.numel();
  if (n == 0) return {key, at::empty({0}, key.options().dtype(at::kInt))};
  auto r = radix_sort_pairs(key.contiguous(), iota32(n, key.device()), 0, end_bit);
  return {std::get<0>(r), std::get<1>(r)};
}

// pairs per owner rank (v % P) of an int64 id column, on the engine device
at::Tensor owner_counts(const at::Tensor& ids, int P) {
  at::Tensor c = at::zeros({P}, ids.options().dtype(at::kLong));
  if (ids.numel() == 0) return c;
  if (ids.is_cuda()) {
    k::count_mod(reinterpret_cast<const int64_t*>(ids.data_ptr()), ids.numel(), P,
                 reinterpret_cast<int64_t*>(c.data_ptr()), at::hip::getCurrentHIPStream());
  } else {
    at::Tensor h = ids.contiguous();
    const int64_t* p = h.data_ptr<int64_t>();
    int64_t* o = c.data_ptr<int64_t>();
    for (int64_t i = 0; i < h.numel(); ++i) o[p[i] % P]++;
  }
  return c;
}

at::Tensor segments(const at::Tensor& sorted) {
  if (sorted.numel() == 0) return at::zeros({1}, sorted.options().dtype(at::kLong));
  return segments_sorted(sorted);
}

std::vector<int64_t> to_vec(const at::Tensor& t) {
  at::Tensor c = t.to(at::kCPU).to(at::kLong).contiguous();
  return std::vector<int64_t>(c.data_ptr<int64_t>(), c.data_ptr<int64_t>() + c.numel());
}

// route edges to the owner of their source (engine shuffle), keeping weights
void to_source_owner(const Comm& comm, at::Tensor& e, at::Tensor& w) {
  const int P = comm.size();
  if (!comm.distributed()) return;
  const at::Device dev = e.device();
  const int64_t n = e.size(0);
  at::Tensor vb = w.defined() ? w.contiguous().view(at::kByte) : at::empty({0}, opt(dev, at::kByte));
  KV kv = make_kv(e.contiguous().view(at::kByte), std::nullopt, vb, std::nullopt, n, dev);
  at::Tensor dest = at::remainder(e.select(1, 0), P).to(at::kInt);
  KV out = exchange(std::move(kv), dest, comm);
  e = out.kdata.view(at::kLong).view({-1, 2});
  if (w.defined()) w = out.vdata.view(w.scalar_type());
}
}  // namespace

bool use_seg_index(const at::Device& d) {
  const char* e = std::getenv("MRH_PLAN_KERNEL");
  return d.is_cuda() && !(e && std::strcmp(e, "tiles") == 0);
}

// ====================================================================== EdgePlan

EdgePlan::EdgePlan(CommPtr c, const at::Tensor& edges, int64_t nvert, const std::optional<at::Tensor>& weights,
                   bool symmetric)
    : comm(std::move(c)), P(comm->size()), me(comm->rank()), dev(comm->device()), N(nvert) {
  nlocal = std::max<int64_t>(0, (N - me + P - 1) / P);
  at::Tensor e = edges.to(dev).to(at::kLong).reshape({-1, 2});
  at::Tensor wt = weights ? weights->to(dev) : at::Tensor();
  if (symmetric) {
    e = at::cat({e, e.flip(1)});
    if (wt.defined()) wt = at::cat({wt, wt});
  }
  to_source_owner(*comm, e, wt);
  nedge = e.size(0);
  at::Tensor src_local = at::floor_divide(e.select(1, 0), P).to(at::kInt);
  at::Tensor vj = e.select(1, 1).contiguous();
  const bool dist = comm->distributed();
  at::Tensor key = dist ? at::bitwise_or(at::bitwise_left_shift(at::remainder(vj, P), 40), vj) : vj;
  auto [ks, perm] = sort_with_perm(key);
  at::Tensor pl = perm.to(at::kLong);
  src = src_local.index_select(0, pl).contiguous();
  if (wt.defined()) w = wt.index_select(0, pl).contiguous();
  seg = segments(ks);
  ngrp = seg.numel() - 1;
  at::Tensor ujv = at::bitwise_and(ks.index_select(0, seg.narrow(0, 0, ngrp)), VMASK);
  if (dist) {
    send_splits_ = to_vec(owner_counts(ujv, P));
    recv_splits_ = comm->alltoall_counts(send_splits_);
    at::Tensor rids = comm->alltoallv(ujv.contiguous(), send_splits_, recv_splits_);
    auto [rs, rperm] = sort_with_perm(at::floor_divide(rids, P));
    rseg_ = segments(rs);
    rperm_ = rperm;
    rvid_ = rs.index_select(0, rseg_.narrow(0, 0, rseg_.numel() - 1)).to(at::kInt);
  } else {
    vid_ = at::floor_divide(ujv, P).to(at::kLong);
  }
  local_ids = at::arange(nlocal, opt(dev, at::kLong)) * P + me;
  if (ngrp > 0 && use_seg_index(dev)) six_ = seg_index(seg, nedge);
}

at::Tensor EdgePlan::propagate(const at::Tensor& x, int op, double identity, bool use_weights) const {
  at::Tensor send = at::empty({ngrp}, x.options());
  at::Tensor wv = (use_weights && w.defined()) ? w : at::empty({0}, x.options());
  if (ngrp > 0) {
    if (six_.defined()) seg_gather_reduce(six_, src, x.contiguous(), wv, op, send);
    else plan_gather_reduce(seg, src, x.contiguous(), wv, op, send);
  }
  at::Tensor acc = at::full({nlocal}, identity, x.options());
  if (comm->distributed()) {
    at::Tensor recv = comm->alltoallv(send, send_splits_, recv_splits_);
    if (recv.numel()) plan_combine(rseg_, rperm_, recv, rvid_, op, acc);
  } else if (ngrp > 0) {
    acc.index_put_({vid_}, send);
  }
  return acc;
}

int64_t EdgePlan::count_global(const at::Tensor& mask) const {
  return comm->allreduce(mask.numel() ? mask.sum().item<int64_t>() : 0, Comm::SUM);
}

std::pair<at::Tensor, int> connected_components(const EdgePlan& plan, int max_iter) {
  at::Tensor lab = plan.local_ids.clone();
  const double big = (double)(int64_t(1) << 62);
  int it = 0;
  while (it < max_iter) {
    ++it;
    at::Tensor m = plan.propagate(lab, PLAN_MIN, big, false);
    at::Tensor nw = at::minimum(lab, m);
    const int64_t changed = plan.count_global(nw != lab);
    lab = nw;
    if (!changed) break;
  }
  return {lab, it};
}

std::pair<at::Tensor, int> luby_mis(const EdgePlan& plan, int64_t seed, const std::optional<at::Tensor>& active,
                                    int max_iter) {
  const at::Tensor& ids = plan.local_ids;
  at::Tensor act = active ? active->to(plan.dev).to(at::kBool).clone() : at::ones({plan.nlocal}, opt(plan.dev, at::kBool));
  at::Tensor mis = at::zeros({plan.nlocal}, opt(plan.dev, at::kBool));
  int it = 0;
  while (it < max_iter && plan.count_global(act) > 0) {
    ++it;
    // priority = (23 hashed bits of (vertex, seed, round), vertex id): unique per round
    const uint64_t salt = (uint64_t)(seed + 1) * 0x632BE59BD9B4E019ull + (uint64_t)it * 0x8CB92BA72F3D8DD7ull;
    at::Tensor h = ids * (int64_t)0x9E3779B97F4A7C15ull + (int64_t)salt;
    h = at::bitwise_xor(h, at::bitwise_right_shift(h, 31)) * (int64_t)0x94D049BB133111EBull;
    h = at::bitwise_xor(h, at::bitwise_right_shift(h, 29));
    at::Tensor r = at::bitwise_or(at::bitwise_left_shift(at::bitwise_and(at::bitwise_right_shift(h, 40),
                                                                          (int64_t)((1 << 23) - 1)),
                                                         40),
                                  at::bitwise_and(ids, VMASK));
    at::Tensor pri = at::where(act, r, at::full_like(r, -1));
    at::Tensor m = plan.propagate(pri, PLAN_MAX, -1.0, false);
    at::Tensor join = at::logical_and(act, pri > m);
    mis = at::logical_or(mis, join);
    at::Tensor nb = plan.propagate(join.to(at::kLong), PLAN_MAX, 0.0, false);
    act = at::logical_and(act, at::logical_not(at::logical_or(join, nb > 0)));
  }
  return {mis, it};
}

std::pair<at::Tensor, int> sssp(const EdgePlan& plan, int64_t source, int max_iter) {
  const double inf = std::numeric_limits<double>::infinity();
  at::Tensor d = at::full({plan.nlocal}, inf, opt(plan.dev, at::kDouble));
  if (source % plan.P == plan.me) d.index_put_({source / plan.P}, 0.0);
  int it = 0;
  while (it < max_iter) {
    ++it;
    at::Tensor m = plan.propagate(d, PLAN_MIN, inf, true);
    at::Tensor nw = at::minimum(d, m);
    const int64_t changed = plan.count_global(nw != d);
    d = nw;
    if (!changed) break;
  }
  return {d, it};
}

at::Tensor sssp_predecessors(const EdgePlan& plan, const at::Tensor& edges, const at::Tensor& weights,
                             const at::Tensor& dist, int64_t source) {
  const Comm& comm = *plan.comm;
  const int P = plan.P;
  const at::Device dev = plan.dev;
  at::Tensor e = edges.to(dev).to(at::kLong).reshape({-1, 2}).contiguous();
  at::Tensor w = weights.to(dev).to(at::kDouble).contiguous();
  // 1. every edge u -> v to the owner of u, where d[u] lives: candidate d[u] + w
  KV kv = make_kv(e.select(1, 0).contiguous().view(at::kByte), std::nullopt,
                  at::stack({e.select(1, 1), w.view(at::kLong)}, 1).contiguous().view(at::kByte), std::nullopt,
                  e.size(0), dev);
  kv = exchange(std::move(kv), at::remainder(e.select(1, 0), P).to(at::kInt), comm);
  at::Tensor u = kv.kdata.view(at::kLong), vw = kv.vdata.view(at::kLong).view({-1, 2});
  at::Tensor cand = dist.index_select(0, at::floor_divide(u, P)) + vw.select(1, 1).contiguous().view(at::kDouble);
  // 2. (v, candidate, u) to the owner of v: u is a predecessor iff its candidate
  //    equals d[v] (the same double sum the relaxation computed)
  KV kv2 = make_kv(vw.select(1, 0).contiguous().view(at::kByte), std::nullopt,
                   at::stack({cand.view(at::kLong), u}, 1).contiguous().view(at::kByte), std::nullopt, u.numel(), dev);
  kv2 = exchange(std::move(kv2), at::remainder(vw.select(1, 0), P).to(at::kInt), comm);
  at::Tensor v = kv2.kdata.view(at::kLong), cu = kv2.vdata.view(at::kLong).view({-1, 2});
  at::Tensor lv = at::floor_divide(v, P);
  at::Tensor ok = at::logical_and(cu.select(1, 0).contiguous().view(at::kDouble) == dist.index_select(0, lv),
                                  at::isfinite(dist.index_select(0, lv)));
  // deterministic tie-break across equal-length paths: the smallest predecessor id
  at::Tensor pred = at::full({plan.nlocal}, std::numeric_limits<int64_t>::max(), at::TensorOptions().device(dev).dtype(at::kLong));
  at::Tensor oki = mask_indices(ok);
  if (oki.numel()) pred.scatter_reduce_(0, lv.index_select(0, oki), cu.select(1, 1).index_select(0, oki), "amin", true);
  pred.masked_fill_(pred == std::numeric_limits<int64_t>::max(), -1);
  if (source % P == plan.me) pred.index_put_({source / P}, 0);  // the source: DISTANCE() default, e.v = 0
  return pred;
}

// ====================================================================== PageRank

PageRankPlan::PageRankPlan(CommPtr c, const at::Tensor& edges, int64_t nvert, double a)
    : comm(std::move(c)), P(comm->size()), me(comm->rank()), dev(comm->device()), N(nvert), alpha(a) {
  nlocal = std::max<int64_t>(0, (N - me + P - 1) / P);
  StageClock clk;
  at::Tensor e = edges.to(dev).to(at::kLong).reshape({-1, 2});
  clk("edges to device");
  // several GPUs (or the forced-RCCL rank): destination-owned edges and a
  // replicated c vector (build_device_dist); MRH_PR_DIST=partials keeps the
  // source-owned plan with an all-to-all of per-destination partial sums
  const char* dmode = std::getenv("MRH_PR_DIST");
  const bool partials = dmode && std::strcmp(dmode, "partials") == 0;
  if (dev.is_cuda() && comm->distributed() && !partials && N < (int64_t(1) << 31)) {
    build_device_dist(e.contiguous());
  } else {
    at::Tensor none;
    to_source_owner(*comm, e, none);
    nedge = e.size(0);
    if (dev.is_cuda() && nedge < (int64_t(1) << 32) && N < (int64_t(1) << 31)) build_device(e.contiguous());
    else build_host(e);
  }
  clk("plan (total)");
  e = at::Tensor();
  const int64_t ngrp = seg_.numel() - 1;
  // one GPU, opt-in (MRH_PR_BLOCKING=1): propagation blocking (pbpr.hip).
  // Measured on RMAT-26 at 8.9 ms per iteration (phase 1 3.5 + phase 2 5.4)
  // vs 7.9 ms for the pull kernel, whose 60 % L2 hit rate on the
  // degree-sorted gathers already beats two streaming passes
  // (profiles/r2_pagerank_blocking.txt); kept for graphs without hub locality
  {
    const char* env = std::getenv("MRH_PR_BLOCKING");
    const bool want = env && *env == '1';
    if (want && !comm->distributed() && dev.is_cuda() && nedge > 0 && nedge < (int64_t(1) << 31) && ngrp > 0)
      build_blocking(vid_.index_select(0, segment_ids(seg_, ngrp, nedge)));
  }
  // the fused tile step (XCD ranges) needs no accumulator array, only its
  // per-tile partials
  acc_ = at::empty({xr_ > 0 ? 0 : nlocal}, opt(dev, at::kFloat));
  if (xr_ > 0) part_ = at::empty({std::max<int64_t>(xtile_, 1), 2}, opt(dev, at::kDouble));
  {
    const char* g = std::getenv("MRH_PR_GRAPH");
    use_graph = !(g && *g == '0');
  }
  if (ngrp > 0 && use_seg_index(dev) && !pb_) {
    six_ = heads_.defined() ? seg_index(seg_, nedge, heads_) : seg_index(seg_, nedge);
    heads_ = at::Tensor();
    if (xsched_.defined()) {
      six_.sched = xsched_;
      six_.slen = xslen_;
    }
  }
  clk("segment index");
  reset();
  clk("reset");
}

// Device build: two keys-only sorts of packed edges, no group-by, no
// payload arrays, no permutation gathers.
//  1. edges packed as (local source << 32 | destination) and sorted on the
//     source bits: every out-degree is a run length (a histogram of random
//     global atomics ran 5x slower — they execute at the memory side);
//  2. the nlocal vertices sorted by degree, descending and stable (R-MAT hubs
//     are spread over ids with few 1-bits; clustering them keeps the hot part
//     of the gathered rank array cache-resident); k_pr_relabel writes the new
//     id of every vertex, the dangling flags and 1/outdeg in the same pass;
//  3. the source-sorted edges repacked as (destination group << 32 | new
//     source id) — the source ids are monotone, so the relabel is a
//     sequential walk — and sorted on the destination bits;
//  4. unpack: the int32 source stream + group head flags -> CSR segments.
namespace {
void pr_chk(hipError_t r, const char* what) {
  if (r != hipSuccess) throw std::runtime_error(std::string("PageRankPlan: ") + what + ": " + hipGetErrorString(r));
}
// smallest b >= 1 with maxval < 2^b (capped at 31)
int pr_bits_for(int64_t maxval) {
  int b = 1;
  while (b < 31 && (int64_t(1) << b) <= maxval) ++b;
  return b;
}
// route packed u64 keys to ranks `dest` (engine shuffle, fixed 8-byte keys)
at::Tensor route_u64(const Comm& comm, const at::Tensor& keys, const at::Tensor& dest) {
  KV kv;
  kv.n = keys.numel();
  kv.kw = 8;
  kv.vw = 0;
  kv.kdata = keys.contiguous().view(at::kByte).reshape({-1});
  kv.vdata = at::empty({0}, opt(comm.device(), at::kByte));
  kv = exchange(std::move(kv), dest, comm);
  return kv.kdata.view(at::kLong).reshape({-1});
}
}  // namespace

// out-degrees of this rank's out-edges. packed (destination << 32 | local
// source) in any order: by default it is sorted on the source bits above 10
// (runs of 1024 sources contiguous: 2 passes at RMAT-26, packed is replaced
// by the sorted array) and counted tile by tile in LDS windows — the
// source-run order also turns the later new-id reads of the sources into
// near-sequential ones; MRH_PR_DEGREES=partition counts the unsorted edges
// (count_low_words: bucket scatter + LDS histograms). The older build,
// MRH_PR_DEGREES=sort: (local source << 32 | destination) fully sorted on
// the source bits, whose run lengths are the degrees.
at::Tensor PageRankPlan::out_degrees(at::Tensor& packed, bool sorted_by_source) {
  const hipStream_t s = at::hip::getCurrentHIPStream();
  const int64_t ne = packed.numel();
  at::Tensor deg = at::empty({std::max<int64_t>(nlocal, 1)}, opt(dev, at::kInt));
  pr_chk(hipMemsetAsync(deg.data_ptr(), 0, deg.numel() * 4, s), "hipMemsetAsync");
  if (ne == 0) return deg;
  if (!sorted_by_source) {
    const char* e = std::getenv("MRH_PR_DEGREES");
    if (e && std::strcmp(e, "partition") == 0) {
      count_low_words(packed, deg);
      return deg;
    }
    constexpr int kRun = 10;
    const int sbits = pr_bits_for(std::max<int64_t>(nlocal - 1, 0));
    if (sbits > kRun) packed = radix_sort_keys(packed, kRun, sbits, false);
    k::pr_deg_window(reinterpret_cast<const uint64_t*>(packed.data_ptr()), ne, kRun,
                     reinterpret_cast<uint32_t*>(deg.data_ptr()), s);
    return deg;
  }
  at::Tensor flags = at::empty({ne}, opt(dev, at::kInt));
  k::pr_heads(reinterpret_cast<const uint64_t*>(packed.data_ptr()), ne, reinterpret_cast<uint32_t*>(flags.data_ptr()),
              s);
  at::Tensor useg = segments_from_flags(flags);
  flags = at::Tensor();
  k::pr_run_degree(reinterpret_cast<const uint64_t*>(packed.data_ptr()), useg.data_ptr<int64_t>(), useg.numel() - 1,
                   reinterpret_cast<uint32_t*>(deg.data_ptr()), s);
  return deg;
}

// sorted (group key << 32 | new source id) -> src_, the groups seg_ and
// their head bitmap heads_ (the gather's segment index, no per-edge flags)
void PageRankPlan::unpack_sorted(const at::Tensor& sorted) {
  const hipStream_t s = at::hip::getCurrentHIPStream();
  src_ = at::empty({nedge}, opt(dev, at::kInt));
  heads_ = at::empty({k::ws_words(nedge)}, opt(dev, at::kInt));
  pr_chk(hipMemsetAsync(heads_.data_ptr(), 0, heads_.numel() * 4, s), "hipMemsetAsync");
  k::pr_unpack_bits(reinterpret_cast<const uint64_t*>(sorted.data_ptr()), nedge, src_.data_ptr<int32_t>(),
                    reinterpret_cast<uint32_t*>(heads_.data_ptr()), s);
  seg_ = segments_from_bits(heads_, nedge);
}

bool PageRankPlan::degrees_by_sort() {
  const char* e = std::getenv("MRH_PR_DEGREES");
  return e && std::strcmp(e, "sort") == 0;
}

// Step 2 of both device builds: deg = out-degree of every local vertex (int32
// [max(nlocal, 1)], out_degrees). Sorts the nlocal vertices by degree
// (descending, stable) and writes the new id of every old local id (nid),
// order_, dangling_, invdeg_; degn (if want_degn): the degree of every new id.
// Returns the number of dangling (out-degree 0) local vertices.
int64_t PageRankPlan::relabel_by_degree(at::Tensor deg, bool want_degn, at::Tensor& nid, at::Tensor& degn) {
  const hipStream_t s = at::hip::getCurrentHIPStream();
  nid = at::empty({std::max<int64_t>(nlocal, 1)}, opt(dev, at::kInt));
  order_ = at::empty({nlocal}, opt(dev, at::kLong));
  dangling_ = at::empty({nlocal}, opt(dev, at::kByte));
  invdeg_ = at::empty({nlocal}, opt(dev, at::kFloat));
  at::Tensor nd = at::empty({1}, opt(dev, at::kLong));
  pr_chk(hipMemsetAsync(nd.data_ptr(), 0, 8, s), "hipMemsetAsync");
  degn = at::Tensor();
  if (nlocal > 0) {
    at::Tensor dkey = at::empty({nlocal}, opt(dev, at::kLong)), io = at::empty({nlocal}, opt(dev, at::kInt));
    k::pr_degkey(reinterpret_cast<const uint32_t*>(deg.data_ptr()), nlocal, reinterpret_cast<uint64_t*>(dkey.data_ptr()),
                 reinterpret_cast<uint32_t*>(io.data_ptr()), s);
    // 32-bit key; constant high digits (every degree < 2^24) are skipped
    at::Tensor ord = std::get<1>(radix_sort_pairs(dkey, io, 0, 32, true));
    dkey = io = at::Tensor();
    if (want_degn) degn = at::empty({nlocal}, opt(dev, at::kInt));
    k::pr_relabel(reinterpret_cast<const uint32_t*>(ord.data_ptr()), reinterpret_cast<const uint32_t*>(deg.data_ptr()),
                  nlocal, nid.data_ptr<int32_t>(), order_.data_ptr<int64_t>(), dangling_.data_ptr<uint8_t>(),
                  invdeg_.data_ptr<float>(), reinterpret_cast<unsigned long long*>(nd.data_ptr()),
                  degn.defined() ? degn.data_ptr<int32_t>() : nullptr, s);
  }
  return nd.item<int64_t>();
}

void PageRankPlan::build_device(const at::Tensor& e) {
  StageClock clk;
  const hipStream_t s = at::hip::getCurrentHIPStream();
  const bool dist = comm->distributed();
  const int64_t nlmax = (N + P - 1) / P;
  auto bits_for = pr_bits_for;
  // 1. out-degrees over (destination << 32 | source), su left in source-run
  // order (out_degrees; MRH_PR_DEGREES=sort: sort (source << 32 |
  // destination) on the source bits, degrees = run lengths)
  const bool bysort = degrees_by_sort() || dist;
  at::Tensor su, deg;
  {
    at::Tensor packed = at::empty({nedge}, opt(dev, at::kLong));
    k::pr_pack_src(e.data_ptr<int64_t>(), nedge, P, !bysort, reinterpret_cast<uint64_t*>(packed.data_ptr()), s);
    su = bysort ? radix_sort_keys(packed, 32, 32 + bits_for(std::max<int64_t>(nlocal - 1, 0)), false) : packed;
    deg = out_degrees(su, bysort);
  }
  clk("pack + out-degrees");
  // 2. vertices by degree; XCD source ranges (one GPU; MRH_PR_XCD=0
  // disables): see xcd_ranges()
  const char* xenv = std::getenv("MRH_PR_XCD");
  const char* benv = std::getenv("MRH_PR_BLOCKING");  // propagation blocking needs the plain layout
  const bool want_xcd = !dist && !(xenv && *xenv == '0') && !(benv && *benv == '1');
  at::Tensor nid, degn;
  const int64_t ndl = relabel_by_degree(deg, want_xcd, nid, degn);
  deg = at::Tensor();
  const int64_t nactive = std::max<int64_t>(nlocal - ndl, 0);
  clk("relabel");
  // 3. by destination group, new source ids in the low word; with XCD source
  // ranges the groups are (range, destination)
  const int64_t himax = !dist ? std::max<int64_t>(N - 1, 0) : P * nlmax - 1;
  const int dbits = bits_for(himax);
  std::vector<int64_t> rb, redge;  // hot range boundaries (new ids) and their first edges
  if (degn.defined() && nactive > 0) xcd_ranges(degn, nactive, dbits, rb, redge);
  degn = at::Tensor();
  clk("xcd ranges");
  const int nhot = rb.empty() ? 0 : (int)rb.size() - 1;
  at::Tensor rbd;
  if (nhot > 0) {
    std::vector<int32_t> rb32(rb.begin(), rb.end());
    rbd = at::from_blob(rb32.data(), {(int64_t)rb32.size()}, opt(at::kCPU, at::kInt)).to(dev);
  }
  int rbits = 0;
  while ((1 << rbits) < nhot + 1) ++rbits;
  if (nhot == 0) rbits = 0;
  at::Tensor sorted;
  {
    at::Tensor packed = at::empty({nedge}, opt(dev, at::kLong));
    k::pr_pack(reinterpret_cast<const uint64_t*>(su.data_ptr()), nedge, P, nlmax, !dist, !bysort, nid.data_ptr<int32_t>(),
               nhot > 0 ? rbd.data_ptr<int32_t>() : nullptr, nhot, dbits, reinterpret_cast<uint64_t*>(packed.data_ptr()),
               s);
    clk("pack");
    su = at::Tensor();
    // MRH_PR_SRC_ORDER=1: the sources of every group in ascending new id too
    // (the sort also runs over the low word: 4 more passes at RMAT-26) — an
    // experiment on the gather's request rate
    const char* so = std::getenv("MRH_PR_SRC_ORDER");
    const int lo_bit = so && *so == '1' ? 0 : 32;
    sorted = radix_sort_keys(packed, lo_bit, 32 + dbits + rbits, false);
  }
  clk("sort by destination");
  // 4. unpack
  unpack_sorted(sorted);
  const int64_t ngrp = seg_.numel() - 1;
  at::Tensor hi = at::empty({ngrp}, opt(dev, at::kLong));
  k::pr_group_hi(reinterpret_cast<const uint64_t*>(sorted.data_ptr()), seg_.data_ptr<int64_t>(), ngrp,
                 hi.data_ptr<int64_t>(), s);
  sorted = at::Tensor();
  w_ = at::empty({0}, opt(dev, at::kFloat));  // weights folded into c = r / outdeg
  send_ = at::empty({ngrp}, opt(dev, at::kFloat));
  if (dist) {
    // hi = owner * nlmax + local id at the owner -> global destination id
    at::Tensor ujv = at::remainder(hi, nlmax) * P + at::floor_divide(hi, nlmax);
    build_exchange(ujv, nid.narrow(0, 0, nlocal));
  } else if (nhot > 0 && ngrp > 0) {
    // partial sums per (range, destination): the fused tile step reads each
    // tile's R runs of (new destination id, partial) and updates the tile's ranks
    xr_ = nhot + 1;
    xtile_ = (nlocal + (int64_t(1) << k::pr_tile_bits()) - 1) >> k::pr_tile_bits();
    ghi_ = at::empty({ngrp}, opt(dev, at::kInt));
    k::pr_group_vid(hi.data_ptr<int64_t>(), ngrp, nullptr, (int64_t(1) << dbits) - 1, ghi_.data_ptr<int32_t>(), s);
    xoff_ = at::empty({xr_ * (xtile_ + 1)}, opt(dev, at::kLong));
    k::pr_range_offsets(hi.data_ptr<int64_t>(), ngrp, dbits, xr_, xtile_, xoff_.data_ptr<int64_t>(), s);
    xcd_schedule(redge);
  } else {
    vid_ = at::empty({ngrp}, opt(dev, at::kInt));  // the group's destination (packed as its new id)
    k::pr_group_vid(hi.data_ptr<int64_t>(), ngrp, nullptr, (int64_t(1) << dbits) - 1, vid_.data_ptr<int32_t>(), s);
  }
  ndangling = comm->allreduce(ndl, Comm::SUM);
  clk("unpack + groups");
}

// Multi-GPU device build: destination-owned edges, replicated c vector.
// Every rank keeps the in-edges of the vertices it owns and gathers c = r /
// outdeg of their sources from a full copy of c, which one in-place RCCL
// all-gather of the ranks' c slices refreshes per iteration — the one
// collective of an iteration besides the 16-byte (L1 delta, dangling mass)
// allreduce. Each rank then runs exactly the one-GPU iteration: XCD source
// ranges over the gathered vector, the fused tile step over its own
// destinations, no combine of received partial sums. With 288 GB of HBM per
// GPU the replicated vector costs nothing (RMAT-26: 256 MB), and the
// all-gather moves only the active (out-degree > 0) sources: each rank's
// slice is its first S new ids (degree-descending; the dangling ids are last
// and contribute c = 0), S = the largest active count.
//   1. edges -> the source owner, vertices owned by sigma(v) % P (vmix.h:
//      balanced for R-MAT, whose v % P is not); out-degrees + degree relabel
//      (relabel_by_degree);
//   2. edges -> the destination owner as (sigma(v), slot of the source in c);
//   3. XCD source ranges on the interleaved order gid = new id * P + rank
//      (every rank's hot sources first), from the all-gathered degrees;
//   4. sort by (range, new destination id); unpack as build_device.
// One rank (the forced-RCCL mode) uses sigma = identity: the plan and its
// results are then bitwise those of build_device.
void PageRankPlan::build_device_dist(const at::Tensor& e) {
  StageClock clk;
  const hipStream_t s = at::hip::getCurrentHIPStream();
  dist_dev_ = true;
  mix_ = P > 1;
  {
    const char* m = std::getenv("MRH_PR_MIX");  // 0: owner = v % P (the edge plan's rule; for comparison)
    if (m && *m == '0') mix_ = false;
  }
  const int64_t nlmax = (N + P - 1) / P;
  // 1. to the source owner; out-degrees and relabel
  at::Tensor su;
  {
    const int64_t n0 = e.size(0);
    at::Tensor packed = at::empty({n0}, opt(dev, at::kLong)), dest = at::empty({n0}, opt(dev, at::kInt));
    k::pr_mix_pack(e.data_ptr<int64_t>(), n0, P, N, mix_, reinterpret_cast<uint64_t*>(packed.data_ptr()),
                   dest.data_ptr<int32_t>(), s);
    packed = route_u64(*comm, packed, dest);
    dest = at::Tensor();
    clk("exchange to source owner");
    k::pr_localize(reinterpret_cast<uint64_t*>(packed.data_ptr()), packed.numel(), P, s);
    su = packed;  // (sv << 32 | local source), in arrival order
  }
  at::Tensor deg = out_degrees(su, false);
  clk("out-degrees");
  const char* xenv = std::getenv("MRH_PR_XCD");
  const bool want_xcd = !(xenv && *xenv == '0');
  at::Tensor nid, degn;
  const int64_t ndl = relabel_by_degree(deg, want_xcd, nid, degn);
  deg = at::Tensor();
  const int64_t nactive = std::max<int64_t>(nlocal - ndl, 0);
  ndangling = comm->allreduce(ndl, Comm::SUM);
  // slice length: the largest active count, a multiple of 16 (64-byte aligned slices)
  int64_t S = comm->allreduce(nactive, Comm::MAX);
  S = (std::max<int64_t>(S, 1) + 15) / 16 * 16;
  if (P * S >= (int64_t(1) << 31)) throw std::runtime_error("PageRankPlan: replicated c vector needs P * S < 2^31");
  S_ = S;
  clk("degrees + relabel");
  // 2. to the destination owner
  at::Tensor pk;
  {
    const int64_t n1 = su.numel();
    pk = at::empty({n1}, opt(dev, at::kLong));
    at::Tensor dest = at::empty({n1}, opt(dev, at::kInt));
    k::pr_pack_dst(reinterpret_cast<const uint64_t*>(su.data_ptr()), n1, P, (int64_t)me * S, nid.data_ptr<int32_t>(),
                   reinterpret_cast<uint64_t*>(pk.data_ptr()), dest.data_ptr<int32_t>(), s);
    su = at::Tensor();
    pk = route_u64(*comm, pk, dest);
  }
  nedge = pk.numel();
  if (nedge >= (int64_t(1) << 32)) throw std::runtime_error("PageRankPlan: >= 2^32 in-edges on one rank");
  clk("exchange to dest owner");
  // 3. XCD source ranges over the interleaved global order gid = new id * P +
  // rank (the degree of every gid: the all-gathered degree array read
  // column-major). Several ranks (MRH_PR_OVERLAP != 0): first cut into K
  // source chunks of equal edge count (MRH_PR_PIECES, default 4) — chunk j =
  // new ids [b_j, b_j+1) of every rank, a contiguous run of gids — each with
  // its own ranges, so that chunk j's edges are one contiguous run the gather
  // can take on as soon as round j of the c exchange has landed.
  const int dbits = pr_bits_for(std::max<int64_t>(nlocal - 1, 0));
  // MRH_PR_OVERLAP=0: off; =2: also on one rank (the forced-RCCL mode:
  // chunked gathers, side-stream rounds and their events without peers)
  const char* oenv = std::getenv("MRH_PR_OVERLAP");
  // (MRH_FORCE_RCCL=2 on one rank takes the multi-rank default: pieces on)
  const bool multi = P > 1 || comm->loopback_collectives();
  const bool by_piece = (multi && !(oenv && *oenv == '0')) || (oenv && *oenv == '2');
  std::vector<int64_t> rb, redge;
  std::vector<int> piece_nr;  // ranges of every chunk (by_piece)
  at::Tensor dg;
  {
    at::Tensor dl = at::zeros({S}, opt(dev, at::kInt));
    const int64_t k0 = degn.defined() ? std::min(S, nlocal) : 0;
    if (k0 > 0) dl.narrow(0, 0, k0).copy_(degn.narrow(0, 0, k0));
    if (degn.defined() || by_piece) {
      at::Tensor dall = at::empty({P * S}, opt(dev, at::kInt));
      comm->allgather_bytes(dl.data_ptr(), dall.data_ptr(), S * 4);
      dg = dall.view({P, S}).t().contiguous().view({-1});
    }
  }
  const bool want_ranges = degn.defined();
  degn = at::Tensor();
  if (by_piece) {
    int K = 4;
    if (const char* e = std::getenv("MRH_PR_PIECES")) K = std::max(1, std::min(64, std::atoi(e)));
    // the one-GPU ranges over the interleaved order, then grouped into at
    // most K chunks of whole layers (8 ranges) near the edge-count quantiles:
    // a chunk ends at a range boundary moved to a multiple of 16 P (so it is new id b_j of every rank, b_j a
    // multiple of 16: 64-byte aligned transfers); no range is added
    std::vector<int64_t> grb, gre;
    if (want_ranges) xcd_ranges(dg, P * S, dbits, grb, gre);
    if (grb.empty()) {
      grb = {0};
      gre = {0, dg.defined() && S > 0 ? dg.sum().item<int64_t>() : 0};
    }
    const int nr = (int)grb.size();  // ranges: nr - 1 hot, then the cold one
    const int64_t total = gre.back();
    std::vector<int> cut{0};  // first range of every chunk
    std::vector<int64_t> b{0};
    for (int j = 1; j < K && total > 0; ++j) {
      const int64_t target = total * j / K;
      int r = (int)(std::lower_bound(gre.begin(), gre.begin() + nr, target) - gre.begin());
      // whole layers only: a layer's 8 ranges run side by side on the 8
      // XCDs, a chunk holding part of one would leave XCDs idle
      r = (r + 4) / 8 * 8;
      if (r <= cut.back() || r >= nr) continue;
      const int64_t id = (grb[r] / P + 8) / 16 * 16;  // nearest multiple of 16 new ids
      const int64_t g = id * P;
      if (id <= b.back() || g <= grb[r - 1] || (r + 1 < nr && g >= grb[r + 1]) || id >= S) continue;
      grb[r] = g;
      cut.push_back(r);
      b.push_back(id);
    }
    b.push_back(S);
    chunk_b_ = b;
    for (size_t j = 0; j + 1 < cut.size(); ++j) piece_nr.push_back(cut[j + 1] - cut[j]);
    piece_nr.push_back(nr - cut.back());
    rb = grb;
    if (rb.size() == 1) rb.clear();  // one cold range: no range ids at all
  } else if (want_ranges) {
    xcd_ranges(dg, P * S, dbits, rb, redge);
  }
  dg = at::Tensor();
  // nhot: range boundaries past the first (ranges = nhot + 1)
  const int nhot = rb.empty() ? 0 : (int)rb.size() - 1;
  at::Tensor rbd;
  if (nhot > 0) {
    std::vector<int32_t> rb32(rb.begin(), rb.end());
    rbd = at::from_blob(rb32.data(), {(int64_t)rb32.size()}, opt(at::kCPU, at::kInt)).to(dev);
  }
  int rbits = 0;
  while ((1 << rbits) < nhot + 1) ++rbits;
  if (nhot == 0) rbits = 0;
  if (dbits + rbits > 32) throw std::runtime_error("PageRankPlan: range and destination bits exceed 32");
  // 4. sort by (range, destination), unpack
  at::Tensor sorted;
  {
    at::Tensor key = at::empty({nedge}, opt(dev, at::kLong));
    k::pr_pack_gather(reinterpret_cast<const uint64_t*>(pk.data_ptr()), nedge, P, S, nid.data_ptr<int32_t>(),
                      nhot > 0 ? rbd.data_ptr<int32_t>() : nullptr, nhot, dbits,
                      reinterpret_cast<uint64_t*>(key.data_ptr()), s);
    pk = at::Tensor();
    clk("xcd ranges + pack");
    sorted = radix_sort_keys(key, 32, 32 + dbits + rbits, false);
  }
  clk("sort by destination");
  unpack_sorted(sorted);
  const int64_t ngrp = seg_.numel() - 1;
  at::Tensor hi = at::empty({std::max<int64_t>(ngrp, 1)}, opt(dev, at::kLong));
  k::pr_group_hi(reinterpret_cast<const uint64_t*>(sorted.data_ptr()), seg_.data_ptr<int64_t>(), ngrp,
                 hi.data_ptr<int64_t>(), s);
  sorted = at::Tensor();
  w_ = at::empty({0}, opt(dev, at::kFloat));
  send_ = at::empty({ngrp}, opt(dev, at::kFloat));
  // the fused tile step always (R = 1: no hot ranges)
  xr_ = nhot + 1;
  xtile_ = (nlocal + (int64_t(1) << k::pr_tile_bits()) - 1) >> k::pr_tile_bits();
  ghi_ = at::empty({std::max<int64_t>(ngrp, 1)}, opt(dev, at::kInt));
  k::pr_group_vid(hi.data_ptr<int64_t>(), ngrp, nullptr, (int64_t(1) << dbits) - 1, ghi_.data_ptr<int32_t>(), s);
  xoff_ = at::empty({xr_ * (xtile_ + 1)}, opt(dev, at::kLong));
  k::pr_range_offsets(hi.data_ptr<int64_t>(), ngrp, dbits, xr_, xtile_, xoff_.data_ptr<int64_t>(), s);
  if (by_piece) {
    build_pieces(piece_nr);
  } else if (nhot > 0 && ngrp > 0) {
    // exact first edge of every range on this rank (the gather's wave
    // schedule); the ranges themselves came from the global degrees
    at::Tensor first = xoff_.view({xr_, xtile_ + 1}).select(1, 0).clamp_max(ngrp).contiguous();
    std::vector<int64_t> re = to_vec(seg_.index_select(0, first));  // xr_ entries, not the whole seg_
    redge.assign(re.begin(), re.end());
    redge.push_back(nedge);
    xcd_schedule(redge);
  }
  // the replicated c vector: P slices of S; the tile step writes this rank's
  // nlocal entries at me * S (entries past S are dangling, c = 0, and land in
  // the next slice, which the all-gather then overwrites), hence the slack
  cfull_ = at::zeros({P * S + nlmax + 64}, opt(dev, at::kFloat));
  c_ = cfull_.narrow(0, (int64_t)me * S, nlocal);
  clk("unpack + groups");
}

// the source pieces of the overlapped iteration (see graphplan.h): the first
// group / edge of every range from the plan, each piece's run of source ids
// copied to a 16-byte aligned slot of srcp_, its segment index and schedule
void PageRankPlan::build_pieces(const std::vector<int>& piece_nr) {
  pieces_.clear();
  const int K = (int)piece_nr.size();
  const int64_t ngrp = seg_.numel() - 1;
  std::vector<int64_t> fg = to_vec(xoff_.view({xr_, xtile_ + 1}).select(1, 0).clamp_max(ngrp).contiguous());
  fg.push_back(ngrp);
  at::Tensor fgd = at::from_blob(fg.data(), {(int64_t)fg.size()}, opt(at::kCPU, at::kLong)).to(dev);
  std::vector<int64_t> fe = to_vec(seg_.index_select(0, fgd));  // first edge of every range, then nedge
  std::vector<int64_t> R0(K + 1, 0);                           // first range of every piece
  for (int q = 0; q < K; ++q) R0[q + 1] = R0[q] + piece_nr[q];
  if (R0[K] != xr_) throw std::runtime_error("PageRankPlan: piece ranges do not add up");
  std::vector<int64_t> off(K + 1, 0);
  for (int q = 0; q < K; ++q) off[q + 1] = off[q] + (fe[R0[q + 1]] - fe[R0[q]] + 3) / 4 * 4;
  srcp_ = at::empty({std::max<int64_t>(off[K], 4)}, opt(dev, at::kInt));
  for (int q = 0; q < K; ++q) {
    Piece pc;
    const int64_t e0 = fe[R0[q]];
    pc.g0 = fg[R0[q]];
    pc.ng = fg[R0[q + 1]] - pc.g0;
    pc.n = fe[R0[q + 1]] - e0;
    if (pc.n > 0 && pc.ng > 0) {
      pc.src = srcp_.narrow(0, off[q], pc.n);
      pc.src.copy_(src_.narrow(0, e0, pc.n));
      pc.six = seg_index(seg_.narrow(0, pc.g0, pc.ng + 1) - e0, pc.n);
      // hot range r on XCD slot r % 8 as in the one-GPU schedule; only the
      // last chunk ends with the cold range (dealt round-robin)
      const bool last = q + 1 == K;
      if (piece_nr[q] > 1 || !last) {
        std::vector<int64_t> re;
        for (int64_t r = R0[q]; r < R0[q + 1]; ++r) re.push_back(fe[r] - e0);
        re.push_back(pc.n);
        auto [sc, sl] = wave_schedule(re, pc.n, (int)R0[q], last);
        pc.six.sched = sc;
        pc.six.slen = sl;
      }
    }
    pieces_.push_back(std::move(pc));
  }
  pr_chk(hipStreamCreateWithFlags(&side_, hipStreamNonBlocking), "hipStreamCreate");
  ring_ev_.assign(K + 1, nullptr);
  for (auto& e : ring_ev_) pr_chk(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
}

void PageRankPlan::ring_free() {
  for (auto& e : ring_ev_)
    if (e) (void)hipEventDestroy(e);
  ring_ev_.clear();
  if (side_) {
    hbm::forget_stream(side_);  // the pg transport allocates on it
    (void)hipStreamDestroy(side_);
  }
  side_ = nullptr;
}

// the c exchange on side_, behind the work queued so far on the current
// stream (the last tile step): round j sends chunk j of this rank's slice to
// every peer and receives theirs — one grouped round over all xGMI links at
// once, not a ring over one — and records ring_ev_[j + 1]
void PageRankPlan::ring_start() {
  const hipStream_t cs = at::hip::getCurrentHIPStream();
  pr_chk(hipEventRecord(ring_ev_[0], cs), "hipEventRecord");
  pr_chk(hipStreamWaitEvent(side_, ring_ev_[0], 0), "hipStreamWaitEvent");
  const c10::DeviceIndex di = dev.has_index() ? dev.index() : c10::hip::current_device();
  c10::hip::HIPStreamGuard guard(c10::hip::getStreamFromExternal(side_, di));
  uint8_t* base = reinterpret_cast<uint8_t*>(cfull_.data_ptr());
  // MRH_FORCE_RCCL=2 on one rank: the slice goes to this rank itself (in
  // place, the identity), so the eager rounds hold real RCCL send/recv
  // operations. Not under HIP-graph capture: RCCL 2.26.6 segfaults in
  // hipStreamEndCapture on a captured self send/recv, while a captured
  // ncclAllReduce replays correctly (tools/rccl_graph_probe.py,
  // profiles/r6_rccl_graph_probe.txt) — the captured iteration keeps its
  // stats allreduce as the RCCL operation inside the graph
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  pr_chk(hipStreamIsCapturing(cs, &cap), "hipStreamIsCapturing");
  const bool self = P == 1 && comm->loopback_collectives() && cap == hipStreamCaptureStatusNone;
  for (size_t j = 0; j + 1 < chunk_b_.size(); ++j) {
    const int64_t a = chunk_b_[j] * 4, len = (chunk_b_[j + 1] - chunk_b_[j]) * 4;
    std::vector<Xfer> xs, xr;
    for (int p = 0; p < P; ++p) {
      if (p == me && !self) continue;
      xs.push_back(Xfer{p, base + (int64_t)me * S_ * 4 + a, len});
      xr.push_back(Xfer{p, base + (int64_t)p * S_ * 4 + a, len});
    }
    if (!xs.empty()) comm->sendrecv(xs, xr);
    pr_chk(hipEventRecord(ring_ev_[j + 1], side_), "hipEventRecord");
  }
}

// one multi-GPU iteration from r into rn: gather from the replicated c,
// fused tile step (writes this rank's c slice in place), (L1, dangling)
// partials -> allreduce; then the c slices go to every rank. With source
// pieces the exchange of the previous tile step's slices runs on side_ in
// chunk rounds, and piece j is gathered right after round j landed (while
// round j + 1 is in flight); the tile step waits for every piece. Else one
// all-gather after the tile step.
void PageRankPlan::launch_iter_dist(const at::Tensor& r, at::Tensor& rn) {
  const hipStream_t s = at::hip::getCurrentHIPStream();
  const bool pieces = !pieces_.empty();
  if (pieces) {
    const bool ring = !c_fresh_;
    if (ring) ring_start();
    for (size_t q = 0; q < pieces_.size(); ++q) {
      // every round is waited for, even by an empty piece: the tile step
      // below writes past this rank's slice into the next rank's chunk 0
      if (ring) pr_chk(hipStreamWaitEvent(s, ring_ev_[q + 1], 0), "hipStreamWaitEvent");
      Piece& pc = pieces_[q];
      if (pc.n > 0 && pc.ng > 0) {
        at::Tensor o = send_.narrow(0, pc.g0, pc.ng);
        seg_gather_reduce(pc.six, pc.src, cfull_, at::Tensor(), 0, o);
      }
    }
  } else if (six_.defined()) {
    seg_gather_reduce(six_, src_, cfull_, at::Tensor(), 0, send_);
  }
  const double base = (1.0 - alpha) / (double)N;
  k::pr_tile_step(send_.data_ptr<float>(), ghi_.data_ptr<int32_t>(), xoff_.data_ptr<int64_t>(), (int)xr_, xtile_,
                  nlocal, r.data_ptr<float>(), rn.data_ptr<float>(), dangling_.data_ptr<uint8_t>(), (float)base,
                  (float)alpha, stats_.data_ptr<double>() + 1, 1.0 / (double)N, invdeg_.data_ptr<float>(),
                  c_.data_ptr<float>(), part_.data_ptr<double>(), s);
  k::pr_partials_sum(part_.data_ptr<double>(), xtile_, stats_.data_ptr<double>(), s);
  comm->allreduce_tensor(stats_, Comm::SUM);
  if (pieces) c_fresh_ = false;  // the next iteration starts the ring
  else comm->allgather_bytes(c_.data_ptr(), cfull_.data_ptr(), S_ * 4);
}

// XCD source ranges. Each XCD has its own 4 MiB L2; the pull gather reads
// x[src] for every edge, and the degree-sorted new ids put the hot sources
// first. The sources [0, T) are cut into layers of 8 ranges of equal edge
// count whose widest range still fits one L2 (MRH_PR_L2_BYTES, 85 % of it);
// range r of every layer runs on XCD slot r % 8 (xcd_schedule), so each XCD
// streams its edges against an L2-resident slice of x. Layers are added until
// less than 2 % of the edges are left (the cold tail, spread over all XCDs)
// or the range ids run out of bits above the destination bits.
// rb: the hot range boundaries (nhot + 1 new ids), redge: the first edge of
// every range, hot and cold (nhot + 2 entries, redge.back() = nedge).
void PageRankPlan::xcd_ranges(const at::Tensor& degn, int64_t nactive, int dbits, std::vector<int64_t>& rb,
                              std::vector<int64_t>& redge, int maxr_cap) {
  // the widest range's slice of x is 85 % of l2: 3 MiB of each XCD's 4 MiB L2
  // measured best with the fused tile step — RMAT-26 x20 at 2 / 3 / 4 / 5 /
  // 6 MiB: 124.4 / 122.8 / 125.1 / 138.6 / 143.6 ms (profiles/r3_pagerank_sweep.txt)
  int64_t l2 = int64_t(3) << 20;
  if (const char* e = std::getenv("MRH_PR_L2_BYTES")) l2 = std::max<int64_t>(4096, std::atoll(e));
  const int64_t cap = l2 / 4 * 85 / 100;
  if (nactive <= cap) return;  // the whole active rank vector fits one L2
  const int maxr = std::min(std::min(64, maxr_cap), 1 << std::max(0, std::min(6, 32 - dbits)));
  int maxl = (maxr - 1) / 8;
  if (const char* e = std::getenv("MRH_PR_XCD_LAYERS")) maxl = std::max(0, std::min(maxl, std::atoi(e)));
  if (maxl <= 0) return;
  // edges of the ids below i, sampled every `st` ids (boundaries are multiples
  // of st, where the sample is exact)
  at::Tensor cum = exclusive_scan(degn.narrow(0, 0, nactive));
  const int64_t st = std::max<int64_t>(1, nactive >> 20);
  const int64_t ns = nactive / st + 1;
  at::Tensor smp = at::empty({ns}, opt(dev, at::kLong));
  k::sample_i64(cum.data_ptr<int64_t>(), nactive + 1, st, ns, smp.data_ptr<int64_t>(),
                at::hip::getCurrentHIPStream());
  std::vector<int64_t> c = to_vec(smp);
  const int64_t total = cum[nactive].item<int64_t>();
  cum = smp = at::Tensor();
  auto id_of = [&](int64_t k) { return std::min(k * st, nactive); };
  // first sample k in [a, b] with c[k] >= v
  auto first_ge = [&](int64_t a, int64_t b, int64_t v) {
    return std::lower_bound(c.begin() + a, c.begin() + b + 1, v) - c.begin();
  };
  // width (ids) of the last of 8 equal-edge ranges of samples [a, b)
  auto last_width = [&](int64_t a, int64_t b) {
    const int64_t k7 = first_ge(a, b, c[a] + (c[b] - c[a]) * 7 / 8);
    return id_of(b) - id_of(k7);
  };
  std::vector<int64_t> ks{0};
  int64_t a = 0;
  for (int l = 0; l < maxl; ++l) {
    if (c[a] >= total - total / 50 || ns - 1 - a < 8) break;
    int64_t lo = a + 8, hi = ns - 1;  // largest b with last_width(a, b) <= cap
    if (last_width(a, lo) > cap) break;
    while (lo < hi) {
      const int64_t mid = (lo + hi + 1) / 2;
      if (last_width(a, mid) <= cap) lo = mid;
      else hi = mid - 1;
    }
    const int64_t b = lo;
    for (int r = 1; r < 8; ++r) ks.push_back(first_ge(a, b, c[a] + (c[b] - c[a]) * r / 8));
    ks.push_back(b);
    a = b;
  }
  if (ks.size() < 9) return;
  rb.clear();
  redge.clear();
  for (int64_t k : ks) {
    rb.push_back(id_of(k));
    redge.push_back(c[k]);
  }
  redge.push_back(total);
}

// the 8 x slen wave schedule of the gather: wave w (edges [1024 w, 1024 w +
// 1024)) belongs to the range holding its first edge; hot range r runs on
// slot r % 8 in layer order, the cold waves are dealt round-robin after them
std::pair<at::Tensor, int64_t> PageRankPlan::wave_schedule(const std::vector<int64_t>& redge, int64_t n, int r_base,
                                                           bool last_cold) const {
  const int64_t T = 1024;  // wavesegred.h WS_TILE
  const int64_t nw = (n + T - 1) / T;
  const int nhot = (int)redge.size() - (last_cold ? 2 : 1);
  std::vector<std::vector<int32_t>> rows(8);
  auto wave_of = [&](int64_t e) { return std::min(nw, (e + T - 1) / T); };
  for (int r = 0; r < nhot; ++r)
    for (int64_t w = wave_of(redge[r]); w < wave_of(redge[r + 1]); ++w) rows[(r_base + r) % 8].push_back((int32_t)w);
  int64_t c = 0;
  for (int64_t w = wave_of(redge[std::max(nhot, 0)]); w < nw; ++w, ++c) rows[c % 8].push_back((int32_t)w);
  size_t slen = 0;
  for (auto& r : rows) slen = std::max(slen, r.size());
  std::vector<int32_t> flat(8 * slen, -1);
  for (int x = 0; x < 8; ++x) std::copy(rows[x].begin(), rows[x].end(), flat.begin() + x * slen);
  return {at::from_blob(flat.data(), {8, (int64_t)slen}, opt(at::kCPU, at::kInt)).to(dev), (int64_t)slen};
}

void PageRankPlan::xcd_schedule(const std::vector<int64_t>& redge) {
  auto [sc, slen] = wave_schedule(redge, nedge);
  xsched_ = sc;
  xslen_ = slen;
}

void PageRankPlan::build_exchange(const at::Tensor& ujv, const at::Tensor& new_of_old) {
  send_splits_ = to_vec(owner_counts(ujv, P));
  recv_splits_ = comm->alltoall_counts(send_splits_);
  at::Tensor rids = comm->alltoallv(ujv.contiguous(), send_splits_, recv_splits_);
  auto [rs, rperm] = sort_with_perm(at::floor_divide(rids, P));
  rseg_ = segments(rs);
  rperm_ = rperm;
  rvid_ = new_of_old.index_select(0, rs.index_select(0, rseg_.narrow(0, 0, rseg_.numel() - 1))).contiguous();
  recv_ = at::empty({rids.numel()}, opt(dev, at::kFloat));
}

// CPU engine: the same plan from tensor ops (group-by source for the degrees)
void PageRankPlan::build_host(const at::Tensor& e) {
  KV kv = make_kv(e.select(1, 0).contiguous().view(at::kByte), std::nullopt, e.select(1, 1).contiguous().view(at::kByte),
                  std::nullopt, nedge, dev);
  at::Tensor vi, deg, vj;
  if (nedge) {
    KMV kmv = convert(kv);
    vi = kmv.keys.kdata.view(at::kLong);
    deg = kmv.seg.narrow(0, 1, kmv.nkey) - kmv.seg.narrow(0, 0, kmv.nkey);
    vj = kmv.vdata.view(at::kLong);
  } else {
    vi = deg = vj = at::empty({0}, opt(dev, at::kLong));
  }
  at::Tensor outdeg = at::zeros({nlocal}, opt(dev, at::kLong));
  if (vi.numel()) outdeg.index_put_({at::floor_divide(vi, P)}, deg);
  at::Tensor dkey = (int64_t(1) << 40) - outdeg;
  order_ = sort_with_perm(dkey, 48).second.to(at::kLong);
  at::Tensor new_of_old = at::empty({nlocal}, opt(dev, at::kInt));
  new_of_old.index_put_({order_}, iota32(nlocal, dev));
  at::Tensor src_local = nedge ? new_of_old.index_select(0, at::floor_divide(vi, P)).index_select(0, repeat_index(deg))
                               : at::empty({0}, opt(dev, at::kInt));
  const bool dist = comm->distributed();
  at::Tensor key = dist ? at::bitwise_or(at::bitwise_left_shift(at::remainder(vj, P), 40), vj) : vj.clone();
  auto [ks, perm] = sort_with_perm(key);
  src_ = src_local.index_select(0, perm.to(at::kLong)).contiguous();
  w_ = at::empty({0}, opt(dev, at::kFloat));
  seg_ = segments(ks);
  const int64_t ngrp = seg_.numel() - 1;
  at::Tensor gk = ks.index_select(0, seg_.narrow(0, 0, ngrp));
  send_ = at::empty({ngrp}, opt(dev, at::kFloat));
  if (dist) build_exchange(at::bitwise_and(gk, VMASK), new_of_old);
  else vid_ = new_of_old.index_select(0, at::floor_divide(gk, P)).contiguous();
  at::Tensor deg_new = outdeg.index_select(0, order_);
  dangling_ = (deg_new == 0).to(at::kByte);
  invdeg_ = at::where(deg_new > 0, 1.0 / deg_new.clamp_min(1).to(at::kDouble), at::zeros_like(deg_new, at::kDouble))
                .to(at::kFloat);
  ndangling = comm->allreduce(dangling_.sum().item<int64_t>(), Comm::SUM);
}

// Static layout of the propagation-blocked iteration (pbpr.hip): phase-1
// order = (source chunk of 2^18 sources, destination), phase-2 order = the
// same edges stably re-sorted by destination bin of 2^14; work
// units = bins cut into slices of <= 2^18 edges (hub bins get many slices).
void PageRankPlan::build_blocking(const at::Tensor& dst_new) {
  const int64_t m = nedge;
  const int CS = 18, BS = 14;
  if (k::pb_bin_size() != (1 << BS)) throw std::runtime_error("PageRank blocking: bin size mismatch");
  int nb = 1;
  while (nb < 32 && (int64_t(1) << nb) < nlocal) ++nb;
  nb = std::max(nb, BS + 1);
  const int cbits = std::max(nb - CS, 0), bbits = nb - BS;
  // phase-1 key (source chunk, destination bin, source): a chunk's sources
  // share a small window of c and a hub's out-edges into one bin are adjacent
  // (broadcast gathers). Sorting each run by destination instead made the
  // phase-2 atomics cheaper (5.4 -> 3.2 ms) but the gathers random (3.5 ->
  // 9.0 ms) on RMAT-26.
  at::Tensor s64 = src_.to(at::kLong), d64 = dst_new.to(at::kLong);
  at::Tensor key1 = at::bitwise_or(
      at::bitwise_or(at::bitwise_left_shift(at::bitwise_right_shift(s64, CS), (int64_t)(bbits + nb)),
                     at::bitwise_left_shift(at::bitwise_right_shift(d64, BS), (int64_t)nb)),
      s64);
  s64 = d64 = at::Tensor();
  auto [k1s, perm1] = sort_with_perm(key1, cbits + bbits + nb);
  key1 = k1s = at::Tensor();
  const at::Tensor p1 = perm1.to(at::kLong);
  pb_src_ = src_.index_select(0, p1).contiguous();
  at::Tensor dst1 = dst_new.index_select(0, p1).contiguous();
  perm1 = at::Tensor();
  at::Tensor bin1 = at::bitwise_right_shift(dst1.to(at::kLong), BS);
  auto [bins, perm2] = sort_with_perm(bin1, std::max(bbits, 1));
  bin1 = at::Tensor();
  pb_out_ = at::empty({m}, opt(dev, at::kInt));
  pb_dst_ = at::empty({m}, opt(dev, at::kShort));
  k::pb_layout(perm2.data_ptr<int32_t>(), dst1.data_ptr<int32_t>(), m, pb_out_.data_ptr<int32_t>(),
               reinterpret_cast<uint16_t*>(pb_dst_.data_ptr()), at::hip::getCurrentHIPStream());
  perm2 = dst1 = at::Tensor();
  // work units from the bin boundaries (one host copy of ~nlocal/2^14 entries)
  at::Tensor bseg = segments(bins);
  const int64_t nbin = bseg.numel() - 1;
  std::vector<int64_t> hs = to_vec(bseg);
  std::vector<int64_t> hb = to_vec(bins.index_select(0, bseg.narrow(0, 0, nbin)));
  bins = at::Tensor();
  constexpr int64_t SL = int64_t(1) << 18;
  std::vector<int32_t> ub;
  std::vector<int64_t> e0, e1;
  std::vector<uint8_t> ex;
  for (int64_t i = 0; i < nbin; ++i) {
    const int64_t a = hs[i], b = hs[i + 1], ns = (b - a + SL - 1) / SL;
    for (int64_t j = 0; j < ns; ++j) {
      ub.push_back((int32_t)hb[i]);
      e0.push_back(a + (b - a) * j / ns);
      e1.push_back(a + (b - a) * (j + 1) / ns);
      ex.push_back(ns == 1 ? 1 : 0);
    }
  }
  pb_nunit_ = (int64_t)ub.size();
  auto up = [&](const void* p, int64_t n, at::ScalarType t) {
    return at::from_blob(const_cast<void*>(p), {n}, opt(at::kCPU, t)).clone().to(dev);
  };
  pb_ub_ = up(ub.data(), pb_nunit_, at::kInt);
  pb_ue0_ = up(e0.data(), pb_nunit_, at::kLong);
  pb_ue1_ = up(e1.data(), pb_nunit_, at::kLong);
  pb_uex_ = up(ex.data(), pb_nunit_, at::kByte);
  pb_vals_ = at::empty({m}, opt(dev, at::kFloat));
  src_ = at::Tensor();  // the pull layout is not needed any more
  pb_ = true;
}

// in place once the buffers exist: a captured iteration graph keeps its
// pointers valid across runs
void PageRankPlan::reset() {
  if (!r_.defined() || r_.numel() != nlocal) {
    r_ = at::empty({nlocal}, opt(dev, at::kFloat));
    rn_ = at::empty_like(r_);
    if (!dist_dev_) c_ = at::empty_like(r_);  // dist: c_ is this rank's slice of cfull_
  }
  r_.fill_(1.0 / (double)N);
  at::mul_out(c_, r_, invdeg_);
  if (!stats_.defined() || stats_.numel() != 2) stats_ = at::empty({2}, opt(dev, at::kDouble));
  stats_.narrow(0, 0, 1).zero_();
  stats_.narrow(0, 1, 1).fill_((double)ndangling / (double)N);
  dmass_ = stats_.narrow(0, 1, 1);  // the dangling mass of the previous iteration
  acc_.zero_();
  if (dist_dev_) comm->allgather_bytes(c_.data_ptr(), cfull_.data_ptr(), S_ * 4);
  c_fresh_ = true;
}

// one XCD-path iteration: gather + segmented reduce of c into send_, then
// the fused tile step (combine, r -> rn, c = rn / outdeg, partials) and the
// partials' sum into stats_ (stats_[1] is the next iteration's dmass)
void PageRankPlan::launch_iter(const at::Tensor& r, at::Tensor& rn) {
  seg_gather_reduce(six_, src_, c_, at::Tensor(), 0, send_);
  const double base = (1.0 - alpha) / (double)N;
  const hipStream_t s = at::hip::getCurrentHIPStream();
  k::pr_tile_step(send_.data_ptr<float>(), ghi_.data_ptr<int32_t>(), xoff_.data_ptr<int64_t>(), (int)xr_, xtile_,
                  nlocal, r.data_ptr<float>(), rn.data_ptr<float>(), dangling_.data_ptr<uint8_t>(), (float)base,
                  (float)alpha, stats_.data_ptr<double>() + 1, 1.0 / (double)N, invdeg_.data_ptr<float>(),
                  c_.data_ptr<float>(), part_.data_ptr<double>(), s);
  k::pr_partials_sum(part_.data_ptr<double>(), xtile_, stats_.data_ptr<double>(), s);
}

PageRankPlan::~PageRankPlan() {
  graph_free();
  ring_free();
}

void PageRankPlan::graph_free() {
  if (gexec_) (void)hipGraphExecDestroy(gexec_);
  gexec_ = nullptr;
  for (auto& e : gev_) {
    if (e) (void)hipEventDestroy(e);
    e = nullptr;
  }
  if (gstream_) {
    hbm::forget_stream(gstream_);
    (void)hipStreamDestroy(gstream_);
  }
  gstream_ = nullptr;
  gkey_.clear();
}

// graph replay: the XCD tile-step path, a fixed iteration count, no
// serialising diagnostic mode. One GPU; or the replicated multi-GPU plan over
// the native RCCL communicator, whose exchange rounds (side_), allreduce and
// the RCCL stream join the capture through their events. MRH_PR_DIST_GRAPH:
// 0 = the multi-GPU iteration stays eager, 1 = replay at any P; unset =
// replay on a one-rank communicator only (validated on the 1-GPU box; a
// multi-rank capture of RCCL peers has not run on an 8-GPU node yet)
bool PageRankPlan::graph_ok() const {
  static const bool sync = [] {
    const char* v = std::getenv("MRH_SYNC");
    return v && *v && *v != '0';
  }();
  static const int dist_graph = [] {
    const char* v = std::getenv("MRH_PR_DIST_GRAPH");
    return v && *v ? std::atoi(v) : -1;
  }();
  if (!use_graph || sync || !dev.is_cuda() || pb_ || xr_ <= 0 || send_.numel() == 0) return false;
  if (dist_dev_) {
    const bool on = dist_graph > 0 || (dist_graph < 0 && P == 1);
    return on && !dist_graph_failed_ && comm->uses_rccl() && !pieces_.empty();
  }
  return !comm->distributed() && six_.defined();
}

// capture two iterations (r_ -> rn_, rn_ -> r_) on a private stream: every
// launch of them becomes a graph node, so a 20-iteration run is 10 graph
// launches instead of ~100 kernel / memset launches from the host
void PageRankPlan::graph_build() {
  graph_free();
  auto chk = [](hipError_t e, const char* what) {
    if (e != hipSuccess) throw std::runtime_error(std::string("PageRank graph: ") + what + ": " + hipGetErrorString(e));
  };
  chk(hipStreamCreateWithFlags(&gstream_, hipStreamNonBlocking), "hipStreamCreate");
  for (auto& e : gev_) chk(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
  // the buffers are ready when the caller's stream gets here
  chk(hipEventRecord(gev_[0], at::hip::getCurrentHIPStream()), "hipEventRecord");
  chk(hipStreamWaitEvent(gstream_, gev_[0], 0), "hipStreamWaitEvent");
  hipGraph_t g = nullptr;
  {
    // the plan's device may be "cuda" without an index: the stream guard needs the real one
    const c10::DeviceIndex di = dev.has_index() ? dev.index() : c10::hip::current_device();
    c10::hip::HIPStreamGuard guard(c10::hip::getStreamFromExternal(gstream_, di));
    if (at::hip::getCurrentHIPStream().stream() != gstream_)
      throw std::runtime_error("PageRank graph: the capture stream is not current");
    chk(hipStreamBeginCapture(gstream_, hipStreamCaptureModeThreadLocal), "hipStreamBeginCapture");
    try {
      if (dist_dev_) {  // ring on in both (run() made c_fresh_ false first)
        launch_iter_dist(r_, rn_);
        launch_iter_dist(rn_, r_);
      } else {
        launch_iter(r_, rn_);
        launch_iter(rn_, r_);
      }
    } catch (...) {
      hipGraph_t bad = nullptr;
      (void)hipStreamEndCapture(gstream_, &bad);
      if (bad) (void)hipGraphDestroy(bad);
      throw;
    }
    chk(hipStreamEndCapture(gstream_, &g), "hipStreamEndCapture");
  }
  const hipError_t e = hipGraphInstantiate(&gexec_, g, nullptr, nullptr, 0);
  (void)hipGraphDestroy(g);
  chk(e, "hipGraphInstantiate");
  gkey_ = graph_key();
}

std::vector<const void*> PageRankPlan::graph_key() const {
  return {r_.data_ptr(), rn_.data_ptr(), c_.data_ptr(), stats_.data_ptr(), send_.data_ptr(), part_.data_ptr(),
          cfull_.defined() ? cfull_.data_ptr() : nullptr};
}

void PageRankPlan::step() {
  if (dist_dev_) {
    launch_iter_dist(r_, rn_);
    dmass_ = stats_.narrow(0, 1, 1);
    std::swap(r_, rn_);
    return;
  }
  if (pb_) {
    const hipStream_t s = at::hip::getCurrentHIPStream();
    k::pb_phase1(pb_src_.data_ptr<int32_t>(), pb_out_.data_ptr<int32_t>(), nedge, c_.data_ptr<float>(),
                 pb_vals_.data_ptr<float>(), s);
    acc_.zero_();
    k::pb_phase2(pb_vals_.data_ptr<float>(), reinterpret_cast<const uint16_t*>(pb_dst_.data_ptr()),
                 pb_ub_.data_ptr<int32_t>(), pb_ue0_.data_ptr<int64_t>(), pb_ue1_.data_ptr<int64_t>(),
                 pb_uex_.data_ptr<uint8_t>(), pb_nunit_, nlocal, acc_.data_ptr<float>(), s);
  } else {
    // acc_ is zero here: reset() and every pr_update leave it so
    if (six_.defined()) seg_gather_reduce(six_, src_, c_, at::Tensor(), 0, send_);
    else if (send_.numel()) pr_contrib(seg_, src_, w_, c_, send_);
  }
  if (pb_) {
  } else if (comm->distributed()) {
    at::Tensor recv = comm->alltoallv(send_, send_splits_, recv_splits_);
    if (recv.numel()) pr_combine(rseg_, rperm_, recv, rvid_, acc_);
  } else if (send_.numel() && xr_ > 0) {
    // combine and update fused per destination tile (no acc round trip);
    // the gather above already ran: only the tile step and the partials here
    const double base = (1.0 - alpha) / (double)N;
    const hipStream_t s = at::hip::getCurrentHIPStream();
    k::pr_tile_step(send_.data_ptr<float>(), ghi_.data_ptr<int32_t>(), xoff_.data_ptr<int64_t>(), (int)xr_, xtile_,
                    nlocal, r_.data_ptr<float>(), rn_.data_ptr<float>(), dangling_.data_ptr<uint8_t>(), (float)base,
                    (float)alpha, stats_.data_ptr<double>() + 1, 1.0 / (double)N, invdeg_.data_ptr<float>(),
                    c_.data_ptr<float>(), part_.data_ptr<double>(), s);
    k::pr_partials_sum(part_.data_ptr<double>(), xtile_, stats_.data_ptr<double>(), s);
    dmass_ = stats_.narrow(0, 1, 1);
    std::swap(r_, rn_);
    return;
  } else if (send_.numel()) {
    scatter_f32(send_, vid_, acc_);
  }
  const double base = (1.0 - alpha) / (double)N;
  at::Tensor st = pr_update(acc_, r_, rn_, dangling_, base, alpha, dmass_, 1.0 / (double)N, invdeg_, c_);
  st = st.to(dev);
  comm->allreduce_tensor(st, Comm::SUM);
  dmass_ = st.narrow(0, 1, 1);
  stats_ = st;
  std::swap(r_, rn_);
}

int PageRankPlan::run(int maxiter, double tol) {
  if (tol <= 0 && maxiter >= 2 && graph_ok()) {
    int eager = 0;
    if (dist_dev_) {
      // the captured pair has the exchange ring on: the first iteration after
      // reset() runs eagerly (c is fresh), and eager iterations come first
      // until RCCL's peer connections exist (they are made on first use,
      // which capture does not allow)
      const int need = dist_warm_ ? 0 : 2;
      while (eager < maxiter && (c_fresh_ || eager < need)) {
        step();
        ++eager;
      }
      dist_warm_ = true;
      if (maxiter - eager < 2) {
        for (; eager < maxiter; ++eager) step();
        return maxiter;
      }
    }
    const int todo = maxiter - eager;
    if (!gexec_ || graph_key() != gkey_) {
      bool built = true;
      try {
        graph_build();
      } catch (const std::exception&) {
        if (!dist_dev_) throw;
        graph_free();
        built = false;
      }
      if (dist_dev_) {
        // every rank replays or none does: a rank whose capture failed would
        // leave its peers' captured rounds without a partner
        at::Tensor f = at::full({1}, built ? 1 : 0, opt(dev, at::kInt));
        comm->allreduce_tensor(f, Comm::MIN);
        if (f.item<int>() == 0) {
          graph_free();
          dist_graph_failed_ = true;
          for (; eager < maxiter; ++eager) step();
          return maxiter;
        }
      }
    }
    const hipStream_t cs = at::hip::getCurrentHIPStream();
    auto chk = [](hipError_t e, const char* what) {
      if (e != hipSuccess) throw std::runtime_error(std::string("PageRank graph: ") + what + ": " + hipGetErrorString(e));
    };
    chk(hipEventRecord(gev_[0], cs), "hipEventRecord");
    chk(hipStreamWaitEvent(gstream_, gev_[0], 0), "hipStreamWaitEvent");
    for (int p = 0; p < todo / 2; ++p) chk(hipGraphLaunch(gexec_, gstream_), "hipGraphLaunch");
    chk(hipEventRecord(gev_[1], gstream_), "hipEventRecord");
    chk(hipStreamWaitEvent(cs, gev_[1], 0), "hipStreamWaitEvent");
    graph_iters_ += 2 * (todo / 2);
    dmass_ = stats_.narrow(0, 1, 1);  // r_ holds the latest ranks after every pair
    if (todo % 2) step();
    return maxiter;
  }
  int it = 0;
  for (it = 1; it <= maxiter; ++it) {
    step();
    if (tol > 0 && delta() < tol) break;
  }
  return std::min(it, maxiter);
}

double PageRankPlan::delta() const { return stats_[0].item<double>(); }

at::Tensor PageRankPlan::ids() const {
  if (!dist_dev_) return order_ * P + me;
  at::Tensor out = at::empty({nlocal}, opt(dev, at::kLong));
  k::pr_unmix_ids(order_.data_ptr<int64_t>(), nlocal, P, me, N, mix_, out.data_ptr<int64_t>(),
                  at::hip::getCurrentHIPStream());
  return out;
}

// ====================================================================== triangles

namespace {
// route the int64 rows of a [n, k] tensor to ranks `dest` (engine shuffle)
at::Tensor route_rows(const Comm& comm, const at::Tensor& rows, const at::Tensor& dest, int k) {
  const at::Device dev = comm.device();
  const int64_t n = rows.size(0);
  KV kv;
  kv.n = n;
  kv.kw = 8 * k;
  kv.vw = 0;
  kv.kdata = rows.contiguous().view(at::kByte).reshape({-1});
  kv.vdata = at::empty({0}, opt(dev, at::kByte));
  kv = exchange(std::move(kv), dest.to(at::kInt), comm);
  return kv.kdata.view(at::kLong).view({-1, k});
}

// position of every query in sorted unique keys, -1 if absent
at::Tensor lookup(const at::Tensor& keys, const at::Tensor& q) {
  at::Tensor out = at::empty({q.numel()}, q.options().dtype(at::kLong));
  if (!q.numel()) return out;
  if (q.is_cuda()) {
    k::lookup_sorted(keys.data_ptr<int64_t>(), keys.numel(), q.data_ptr<int64_t>(), q.numel(), out.data_ptr<int64_t>(),
                     at::hip::getCurrentHIPStream());
    return out;
  }
  const int64_t* kp = keys.data_ptr<int64_t>();
  const int64_t* qp = q.data_ptr<int64_t>();
  int64_t* o = out.data_ptr<int64_t>();
  for (int64_t j = 0; j < q.numel(); ++j) {
    const int64_t* it = std::lower_bound(kp, kp + keys.numel(), qp[j]);
    o[j] = (it != kp + keys.numel() && *it == qp[j]) ? it - kp : -1;
  }
  return out;
}

// MRH_TRI_ONESORT=1: rank vertices by their degree counted over the raw
// edges, duplicates included, so the one-rank build sorts once (orient, sort,
// then drop duplicates) instead of twice. Measured slower on RMAT-24: 157.9
// vs 124.2 ms per step — the duplicate-inflated order makes the hub rows'
// counting costlier than the saved sort (profiles/r4_trifind_onesort.txt);
// the default ranks by the unique edges' degrees
bool tri_raw_degrees() {
  const char* e = std::getenv("MRH_TRI_ONESORT");
  return e && *e == '1';
}

// sorted unique values of an int64 column
at::Tensor unique_sorted(const at::Tensor& x) {
  if (x.numel() == 0) return x.contiguous();
  at::Tensor s = x.is_cuda() && x.scalar_type() == at::kLong ? radix_sort_keys(x, 0, 64) : sort_with_perm(x.contiguous()).first;
  at::Tensor sg = segments(s);
  return s.index_select(0, sg.narrow(0, 0, sg.numel() - 1)).contiguous();
}

// a spread of the packed edge bits (the owner of an undirected edge)
at::Tensor edge_owner(const at::Tensor& p, int P) {
  at::Tensor h = at::bitwise_xor(p, at::bitwise_right_shift(p, 29)) * (int64_t)0x9E3779B97F4A7C15ull;
  return at::remainder(at::bitwise_and(at::bitwise_right_shift(h, 24), (int64_t(1) << 39) - 1), P);
}
}  // namespace

TriangleGraph::TriangleGraph(CommPtr c, const at::Tensor& edges, int64_t nv) : comm(std::move(c)) {
  const at::Device dev = comm->device();
  at::Tensor e = edges.to(dev).to(at::kLong).reshape({-1, 2}).contiguous();
  // Build modes for several ranks (MRH_TRI_BUILD = split | halo | replicated;
  // the older MRH_TRI_REPLICATED=1 / 0 = replicated / halo):
  //  * split (GPU default when the whole graph's CSR fits a quarter of the
  //    free HBM — RMAT-24: ~13 GB of 288 GB): the edges are deduplicated,
  //    degree-ranked and sorted by key-range and row-range owners (build_split),
  //    only the finished column array is all-gathered; every rank holds the
  //    CSR and counts its share of the rows (split by estimated work);
  //  * halo (CPU default, and graphs too large to replicate): O(E/P + halo)
  //    memory per rank (build_distributed);
  //  * replicated: every rank all-gathers the raw edge list and builds the
  //    whole CSR itself (the round-3 path, kept for comparison).
  std::string mode = "split";
  if (const char* bm = std::getenv("MRH_TRI_BUILD")) {
    if (*bm) mode = bm;
  } else if (const char* rep = std::getenv("MRH_TRI_REPLICATED")) {
    if (*rep) mode = *rep == '1' ? "replicated" : "halo";
  } else if (comm->distributed()) {
    const int64_t mall = comm->allreduce(e.size(0), Comm::SUM);
    size_t free_b = 0, total_b = 0;
    int fits = 0;
    if (dev.is_cuda() && hipMemGetInfo(&free_b, &total_b) == hipSuccess)
      fits = (double)mall * 48.0 < (double)free_b / 4.0 ? 1 : 0;
    mode = comm->allreduce((int64_t)fits, Comm::MIN) == 1 ? "split" : "halo";  // every rank takes the same path
  }
  if (mode != "split" && mode != "halo" && mode != "replicated")
    throw std::runtime_error("MRH_TRI_BUILD must be split, halo or replicated");
  if (!comm->distributed()) mode = "replicated";  // one rank: the whole graph is local anyway
  at::Tensor p;
  if (mode != "halo" && dev.is_cuda() && nv >= 0) {
    // one pass: packed min << 32 | max, a self loop packed as edge (0, 0) —
    // it sorts first, keeps every key byte that is constant over the real
    // edges constant (the radix sort still skips those passes), and is
    // dropped after the dedup
    nvert = nv;
    if (nvert >= (int64_t(1) << 31)) throw std::runtime_error("mrhip: triangle path needs vertex ids < 2^31");
    p = at::empty({e.size(0)}, opt(dev, at::kLong));
    at::Tensor bad = at::zeros({1}, opt(dev, at::kInt));
    k::tri_pack(e.data_ptr<int64_t>(), e.size(0), nvert, reinterpret_cast<uint64_t*>(p.data_ptr()),
                reinterpret_cast<unsigned int*>(bad.data_ptr()), at::hip::getCurrentHIPStream());
    if (bad.item<int32_t>())
      throw std::runtime_error("TriangleGraph: an edge has a vertex id outside [0, nvert = " + std::to_string(nvert) + ")");
  } else {
    at::Tensor lo = at::minimum(e.select(1, 0), e.select(1, 1)), hi = at::maximum(e.select(1, 0), e.select(1, 1));
    at::Tensor keep = mask_indices(lo != hi);  // no self loops
    lo = lo.index_select(0, keep);
    hi = hi.index_select(0, keep);
    if (nv < 0) nv = comm->allreduce(hi.numel() ? hi.max().item<int64_t>() : -1, Comm::MAX) + 1;
    nvert = nv;
    if (nvert >= (int64_t(1) << 31)) throw std::runtime_error("mrhip: triangle path needs vertex ids < 2^31");
    if (mode == "halo") {
      build_distributed(lo, hi);
      return;
    }
    p = at::bitwise_or(at::bitwise_left_shift(lo, 32), hi).contiguous();
  }
  e = at::Tensor();
  if (mode == "split") {
    build_split(p);
    return;
  }
  // replicated degree-oriented CSR: every rank holds the whole graph and
  // counts its share of the rows
  static const bool dbg = std::getenv("MRH_TRI_DEBUG") != nullptr;
  auto stage = [&](const char* what) {
    if (!dbg) return;
    if (dev.is_cuda()) (void)hipDeviceSynchronize();
    std::fprintf(stderr, "mrhip TriangleGraph: %s done\n", what);
  };
  stage("pack");
  distributed = false;
  if (comm->distributed()) p = comm->allgather_var(p);
  if (tri_raw_degrees()) {
    // one sort instead of two: rank the vertices by their degree counted with
    // the duplicate edges (any total order orients correctly; duplicates only
    // nudge the order), orient the raw edges, sort once and drop the
    // duplicates and self loops (packed (0, 0) -> equal halves) afterwards —
    // the dedup sort of the raw edges before the orientation sort is gone
    at::Tensor deg = tri_degrees(p, std::max<int64_t>(nvert, 1));
    auto [rank, pm] = tri_rank_perm(deg);
    deg = at::Tensor();
    at::Tensor o = tri_orient_keys(p, rank);
    p = at::Tensor();
    rank = at::Tensor();
    at::Tensor srt = o.numel() ? radix_sort_keys(o, 0, 64) : o;
    o = at::Tensor();
    stage("orient + sort");
    const int64_t n = srt.numel();
    if (n > 0) {
      at::Tensor keep = at::ne(at::bitwise_right_shift(srt, 32), at::bitwise_and(srt, (int64_t)0xffffffff));
      if (n > 1) keep.narrow(0, 1, n - 1).logical_and_(at::ne(srt.narrow(0, 1, n - 1), srt.narrow(0, 0, n - 1)));
      srt = srt.index_select(0, mask_indices(keep)).contiguous();
    }
    okeys = srt;
    nedge = okeys.numel();
    rowptr = tri_rowptr_of(okeys, std::max<int64_t>(nvert, 1));
    col = tri_col_of(okeys);
    perm = pm;
    stage("CSR");
  } else {
    at::Tensor uniq = unique_sorted(p);
    stage("dedup");
    p = at::Tensor();
    if (uniq.numel() > 0 && uniq[0].item<int64_t>() == 0) uniq = uniq.narrow(0, 1, uniq.numel() - 1);  // (0, 0): self loops
    stage("drop self loops");
    nedge = uniq.numel();
    std::tie(rowptr, col, okeys, perm) = tri_prepare(uniq, std::max<int64_t>(nvert, 1));
    stage("CSR");
  }
  const int64_t m = okeys.numel(), P = comm->size(), me = comm->rank();
  e0 = 0;
  e1 = m;
  if (P > 1 && m > 0) {
    const int64_t nr = rowptr.numel() - 1;
    at::Tensor d = rowptr.narrow(0, 1, nr) - rowptr.narrow(0, 0, nr);
    std::vector<int64_t> rb = work_split(d, P);
    e0 = rowptr[rb[me]].item<int64_t>();
    e1 = rowptr[rb[me + 1]].item<int64_t>();
  }
}

// row boundaries (P + 1, identical on every rank given the same d) cutting
// the rows into P ranges of equal estimated work d+(u)^2 + d+(u) — the wedges
// the hash and hub-bitmap kernels walk — not equal edge counts: the top-ranked
// rows hold most of the work in few edges
std::vector<int64_t> TriangleGraph::work_split(const at::Tensor& d_in, int64_t P) {
  const int64_t nr = d_in.numel();
  at::Tensor d = d_in.to(at::kLong);
  at::Tensor cost = exclusive_scan((d * d + d).contiguous());  // nr + 1 entries
  const int64_t total = cost[nr].item<int64_t>();
  std::vector<int64_t> tg(P - 1);
  for (int64_t r = 1; r < P; ++r) tg[r - 1] = total / P * r + (total % P) * r / P;
  std::vector<int64_t> rb{0};
  if (P > 1) {
    at::Tensor targets = at::from_blob(tg.data(), {P - 1}, at::TensorOptions().dtype(at::kLong)).to(cost.device());
    at::Tensor ub = at::searchsorted(cost, targets).clamp(0, nr).to(at::kCPU);
    for (int64_t r = 0; r < P - 1; ++r) rb.push_back(ub[r].item<int64_t>());
  }
  rb.push_back(nr);
  for (size_t i = 1; i < rb.size(); ++i) rb[i] = std::max(rb[i], rb[i - 1]);
  return rb;
}

// Multi-rank build of the replicated CSR without replicating the work
// (sample sort by key range, then by row range):
//  1. every packed edge to the owner of its key range (splitters from an
//     all-gathered sample), sort + dedup there: the ranks hold disjoint sets
//     of unique edges;
//  2. degrees: a partial count per rank, allreduced (nvert int32); every
//     rank derives the same (degree, id) ranks;
//  3. the local unique edges oriented to the higher rank and sorted; local
//     out-degrees d+ from the sorted runs, allreduced -> the global rowptr
//     and the row split by estimated work (work_split);
//  4. the oriented edges to their row owner, merged there (another local
//     sort of the P received sorted runs): this rank's rows, in order;
//  5. the column arrays all-gathered in rank order = the global CSR order.
// Per rank that is O(E/P) sorting, two all-to-alls of E/P keys and one
// all-gather of the 4-byte columns, instead of the whole raw edge list
// all-gathered and sorted on every rank.
// owner of every key: the number of sorted splitters <= key (searchsorted
// side right) — the engine's LDS binary-search kernel on the device (keys
// and splitters non-negative int64: unsigned order = signed order)
static at::Tensor owners_right(const at::Tensor& split, const at::Tensor& keys) {
  if (!keys.is_cuda() || split.numel() > 4096) return at::searchsorted(split, keys, /*out_int32=*/true, /*right=*/true);
  at::Tensor sp = split.contiguous(), k = keys.contiguous();
  at::Tensor out = at::empty({k.numel()}, k.options().dtype(at::kInt));
  if (k.numel())
    k::bucket_by_splitters(reinterpret_cast<const uint64_t*>(k.data_ptr<int64_t>()), k.numel(),
                           reinterpret_cast<const uint64_t*>(sp.data_ptr<int64_t>()), (int)sp.numel(),
                           out.data_ptr<int32_t>(), at::hip::getCurrentHIPStream(), /*right=*/true);
  return out;
}

void TriangleGraph::build_split(const at::Tensor& p_in) {
  const Comm& cm = *comm;
  const int P = cm.size(), me = cm.rank();
  const at::Device dev = cm.device();
  auto L = at::TensorOptions().device(dev).dtype(at::kLong);
  split = true;
  distributed = false;
  at::Tensor p = p_in.contiguous();
  const int64_t nv = std::max<int64_t>(nvert, 1);
  // the degree order: counted over the raw edges, duplicates included, like
  // the one-rank build (tri_raw_degrees), so both orient and count alike
  at::Tensor deg;
  if (tri_raw_degrees()) deg = tri_degrees(p, nv);
  // 1. key-range owners from NS strided samples per rank
  {
    constexpr int64_t NS = 4096;
    const int64_t n = p.numel();
    at::Tensor smp = at::full({NS}, std::numeric_limits<int64_t>::max(), L);
    if (n > 0) smp = p.index_select(0, at::floor_divide(at::arange(NS, L) * n, NS));
    at::Tensor all = at::empty({P * NS}, L);
    cm.allgather_bytes(smp.data_ptr(), all.data_ptr(), NS * 8);
    at::Tensor srt = std::get<0>(at::sort(all));
    at::Tensor spl = srt.index_select(0, at::arange(1, P, L) * NS).contiguous();  // P - 1 splitters
    at::Tensor dest = P > 1 ? owners_right(spl, p) : at::zeros({n}, L.dtype(at::kInt));
    p = route_u64(cm, p, dest);
  }
  at::Tensor uniq = unique_sorted(p);
  p = at::Tensor();
  if (uniq.numel() > 0 && uniq[0].item<int64_t>() == 0) uniq = uniq.narrow(0, 1, uniq.numel() - 1);  // self loops
  nedge = cm.allreduce(uniq.numel(), Comm::SUM);
  // 2. global degrees -> ranks
  at::Tensor rank;
  {
    if (!deg.defined()) deg = tri_degrees(uniq, nv);
    cm.allreduce_tensor(deg, Comm::SUM);
    std::tie(rank, perm) = tri_rank_perm(deg);
    deg = at::Tensor();
  }
  // 3. oriented + sorted locally; d+ allreduced -> rowptr, row split
  at::Tensor os = tri_orient_keys(uniq, rank);
  uniq = rank = at::Tensor();
  if (os.numel()) os = radix_sort_keys(os, 0, 64);
  std::vector<int64_t> rb;
  {
    at::Tensor lrp = tri_rowptr_of(os, nv);
    at::Tensor dp = (lrp.narrow(0, 1, nv) - lrp.narrow(0, 0, nv)).to(at::kInt).contiguous();
    lrp = at::Tensor();
    cm.allreduce_tensor(dp, Comm::SUM);
    rowptr = exclusive_scan(dp.to(at::kLong).contiguous());
    rb = work_split(dp, P);
  }
  u0_ = rb[me];
  u1_ = rb[me + 1];
  // 4. to the row owners; P sorted runs -> one
  if (P > 1) {
    std::vector<int64_t> bk;
    for (int r = 1; r < P; ++r) bk.push_back(rb[r] << 32);
    at::Tensor b = at::from_blob(bk.data(), {P - 1}, at::TensorOptions().dtype(at::kLong)).to(dev);
    at::Tensor dest = owners_right(b, os);
    os = route_u64(cm, os, dest);
    if (os.numel()) os = radix_sort_keys(os, 0, 64);
  }
  okeys = os;
  // 5. the columns of every rank's rows, in rank (= row) order
  col = cm.allgather_var(tri_col_of(okeys));
  const int64_t m = rowptr[nv].item<int64_t>();
  if (col.numel() != m || m != nedge)
    throw std::runtime_error("TriangleGraph split build: " + std::to_string(col.numel()) + " columns gathered, rowptr says " +
                             std::to_string(m) + ", " + std::to_string(nedge) + " unique edges");
  e0 = 0;
  e1 = okeys.numel();
}

// Distributed build (reference tri_find shuffles every edge 4 times,
// oink/tri_find.cpp:43-82): memory per rank is O(E/P + halo), never the
// whole graph.
//  1. dedup: every undirected edge to a hashed owner, sort + unique;
//  2. degrees at the vertex owners (v % P);
//  3. orientation u -> v by (degree, id): the edge visits the owners of both
//     ends to pick up their degrees, then lands at the owner of u;
//  4. local CSR of the owned rows N+(u), u % P == me;
//  5. halo: the owners of the remote targets v return N+(v) (one request /
//     response all-to-all pair), keeping only entries that are rows here
//     (any w of a triangle u, v, w lies in N+(u), so nothing else can match);
//  6. rows relabelled into one local id space (owned u -> u / P, halo -> nlocal
//     + index) with every row sorted, so the LDS-hash / merge kernels of the
//     replicated path count the owned rows unchanged.
void TriangleGraph::build_distributed(const at::Tensor& lo_in, const at::Tensor& hi_in) {
  distributed = true;
  const Comm& cm = *comm;
  const int P = cm.size(), me = cm.rank();
  const at::Device dev = cm.device();
  auto L = at::TensorOptions().device(dev).dtype(at::kLong);
  nlocal = std::max<int64_t>(0, (nvert - me + P - 1) / P);
  // 1. dedup at hashed owners
  at::Tensor p = at::bitwise_or(at::bitwise_left_shift(lo_in, 32), hi_in).contiguous();
  p = route_rows(cm, p.view({-1, 1}), edge_owner(p, P), 1).reshape({-1});
  p = unique_sorted(p);
  nedge = cm.allreduce(p.numel(), Comm::SUM);
  at::Tensor lo = at::bitwise_right_shift(p, 32), hi = at::bitwise_and(p, (int64_t)0xffffffff);
  // 2. degrees at the owners
  at::Tensor ends = at::cat({lo, hi}).view({-1, 1});
  at::Tensor got = route_rows(cm, ends, at::remainder(ends.reshape({-1}), P), 1).reshape({-1});
  at::Tensor deg = bincount_dev(at::floor_divide(got, P), nlocal);
  // 3. orientation: pick up deg(lo) at owner(lo), deg(hi) at owner(hi)
  at::Tensor r = route_rows(cm, at::stack({lo, hi}, 1), at::remainder(lo, P), 2);
  r = at::stack({r.select(1, 0), r.select(1, 1), deg.index_select(0, at::floor_divide(r.select(1, 0), P))}, 1);
  r = route_rows(cm, r, at::remainder(r.select(1, 1), P), 3);
  at::Tensor a = r.select(1, 0), b = r.select(1, 1), da = r.select(1, 2);
  at::Tensor db = deg.index_select(0, at::floor_divide(b, P));
  at::Tensor a_first = at::logical_or(da < db, at::logical_and(da == db, a < b));
  at::Tensor u = at::where(a_first, a, b), v = at::where(a_first, b, a);
  at::Tensor uv = route_rows(cm, at::stack({u, v}, 1), at::remainder(u, P), 2);
  u = uv.select(1, 0).contiguous();
  v = uv.select(1, 1).contiguous();
  // 4. owned rows, sorted by (local row, target id)
  at::Tensor lu = at::floor_divide(u, P);
  {
    auto sp = sort_with_perm(at::bitwise_or(at::bitwise_left_shift(lu, 32), v));
    at::Tensor pl = sp.second.to(at::kLong);
    u = u.index_select(0, pl);
    v = v.index_select(0, pl);
    lu = lu.index_select(0, pl);
  }
  at::Tensor own_rp = exclusive_scan(bincount_dev(lu, nlocal));
  // 5. halo rows: request N+(v) for remote targets
  at::Tensor remote = at::remainder(v, P) != me;
  at::Tensor hids = unique_sorted(v.index_select(0, mask_indices(remote)));
  at::Tensor req = route_rows(cm, at::stack({hids, at::full_like(hids, me)}, 1), at::remainder(hids, P), 2);
  at::Tensor rv = req.select(1, 0).contiguous(), rq = req.select(1, 1).contiguous();
  at::Tensor rrow = at::floor_divide(rv, P);
  at::Tensor rcnt = own_rp.index_select(0, rrow + 1) - own_rp.index_select(0, rrow);
  at::Tensor rep = repeat_index(rcnt);                       // request of every response entry
  at::Tensor pos = own_rp.index_select(0, rrow).index_select(0, rep) +
                   (at::arange(rep.numel(), L) - exclusive_scan(rcnt).narrow(0, 0, rcnt.numel()).index_select(0, rep));
  at::Tensor resp = at::stack({rv.index_select(0, rep), v.index_select(0, pos)}, 1);
  resp = route_rows(cm, resp, rq.index_select(0, rep), 2);
  at::Tensor hv = resp.select(1, 0).contiguous(), hw = resp.select(1, 1).contiguous();
  // keep only entries that are rows here (owned, or a requested halo id)
  at::Tensor hw_halo = lookup(hids, hw);
  at::Tensor keep = at::logical_or(at::remainder(hw, P) == me, hw_halo >= 0);
  at::Tensor ki = mask_indices(keep);
  hv = hv.index_select(0, ki);
  hw = hw.index_select(0, ki);
  hw_halo = hw_halo.index_select(0, ki);
  // 6. one local id space, rows sorted by local id
  const int64_t nh = hids.numel();
  nrows = nlocal + nh;
  auto relabel = [&](const at::Tensor& x, const at::Tensor& halo_idx) {
    return at::where(at::remainder(x, P) == me, at::floor_divide(x, P), halo_idx + nlocal);
  };
  at::Tensor own_col = relabel(v, lookup(hids, v));
  at::Tensor h_row = lookup(hids, hv) + nlocal;
  at::Tensor h_col = relabel(hw, hw_halo);
  at::Tensor rows_all = at::cat({lu, h_row}), cols_all = at::cat({own_col, h_col});
  auto sp = sort_with_perm(at::bitwise_or(at::bitwise_left_shift(rows_all, 32), cols_all));
  at::Tensor keys = sp.first;
  col = at::bitwise_and(keys, (int64_t)0xffffffff).to(at::kInt).contiguous();
  rowptr = exclusive_scan(bincount_dev(at::bitwise_right_shift(keys, 32), nrows));
  // owned oriented edges in the local space (row < nlocal), for counting and listing
  at::Tensor owned = at::bitwise_right_shift(keys, 32) < nlocal;
  okeys = keys.index_select(0, mask_indices(owned)).contiguous();
  e0 = 0;
  e1 = okeys.numel();
  // global id of every local row
  row_gid = at::cat({at::arange(nlocal, L) * P + me, hids});
}

int64_t TriangleGraph::count() const {
  if (split) return comm->allreduce(tri_count_range(rowptr, col, u0_, u1_), Comm::SUM);
  if (!distributed) return comm->allreduce(tri_count(rowptr, col, okeys, e0, e1), Comm::SUM);
  return comm->allreduce(tri_count_rows(rowptr, col, 0, nlocal), Comm::SUM);
}

at::Tensor TriangleGraph::triangles() const {
  at::Tensor t = tri_list(rowptr, col, okeys, e0, e1);
  if (!t.numel()) return t;
  const at::Tensor& ids = distributed ? row_gid : perm;
  return std::get<0>(at::sort(ids.index_select(0, t.reshape({-1})).view({-1, 3}), 1));
}

}  // namespace mrh
