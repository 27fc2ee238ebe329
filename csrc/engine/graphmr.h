// sssp_mr and luby_find_mr callback ops (graphmr.cpp; kernels
// csrc/kernels/graphmr.hip), for the OINK commands that run the reference's
// MapReduce formulations (oink/sssp.cpp:88-152, oink/luby_find.cpp:53-97).
// Records are int64 words: DISTANCE {pred, wt bits, current}, EDGEVALUE
// {v, wt bits}, ERAND {vi, ri bits, vj, rj bits}, VRAND {v, r bits}, VFLAG
// {v, r bits, flag}. Each op has a host twin of identical semantics.
#pragma once
#include <ATen/ATen.h>

#include <utility>

#include "kv.h"

namespace mrh {
// pick_shortest_distances (oink/sssp.cpp:244-293) over vertex -> DISTANCE
// groups: dist [nkey,3] (every key's winner, current set) and the keys whose
// distance changed with their new distance (ckeys [c], cdist [c,3])
struct SsspPick {
  at::Tensor dist, ckeys, cdist;
};
SsspPick ssspmr_pick(const KMV& m);
// update_adjacent_distances (oink/sssp.cpp:299-360) over vertex -> {EDGEVALUE
// (16 B), DISTANCE (24 B)} groups: the edges re-emitted (ekeys [e], edges
// [e,2]) and the relaxed distances of the out-neighbours of every key that
// holds a distance (pkeys [p], paths [p,3])
struct SsspRelax {
  at::Tensor ekeys, edges, pkeys, paths;
};
SsspRelax ssspmr_relax(const KMV& m);

// map_vert_random (oink/luby_find.cpp:120-136): edges [n,2] -> ERAND [m,4]
// with drand48() after srand48(v + seed) per end; self loops dropped
at::Tensor lubymr_random(const at::Tensor& edges, int64_t seed);
// reduce_edge_winner (:140-182): live edge keys (no non-empty value) ->
// (VRAND keys [2m,2], VFLAG values [2m,3]), winner then loser
std::pair<at::Tensor, at::Tensor> lubymr_edge_winner(const KMV& m);
// reduce_vert_winner (:186-234, loser = false) / reduce_vert_loser (:238-285):
// per value, key = the neighbour's VRAND; value = this key's VRAND as a
// VFLAG (k24, v24 [.,3]) when the key won all its edges / has a winner
// neighbour, else as a VRAND (k16, v16 [.,2])
struct LubyVert {
  at::Tensor k24, v24, k16, v16;
};
LubyVert lubymr_vert(const KMV& m, bool loser);
// reduce_vert_emit (:289-344): MIS vertices (keys without a 16-byte value)
// and the edges back as ERAND keys, with an int 0 flag (kflag, its values
// fval) or without a value (knull)
struct LubyEmit {
  at::Tensor mis, kflag, fval, knull;
};
LubyEmit lubymr_emit(const KMV& m);
}  // namespace mrh
