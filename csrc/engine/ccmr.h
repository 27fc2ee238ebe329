// cc_find_mr callback ops (ccmr.cpp; reference oink/cc_find.cpp:119-330).
// Zones are int64: bit 63 marks a hot zone, the bits under it (from pshift)
// carry the rank a hot zone's vertex was salted to.
#pragma once
#include <ATen/ATen.h>

#include <utility>

#include "kv.h"

namespace mrh {
// vertex -> {zone (8 B), edges (16 B)}: (edge [E,2], zone of the vertex [E])
std::pair<at::Tensor, at::Tensor> ccmr_edge_zone(const KMV& m);
// edge -> its two end zones: (larger zone, {smaller zone, 0}) where they differ
std::pair<at::Tensor, at::Tensor> ccmr_winner(const KMV& m);
// KV(vertex, zone) -> (zone, vertex); hot zones get a random rank (splitmix64
// of seed ^ pair index, mod P) in the bits at pshift
std::pair<at::Tensor, at::Tensor> ccmr_invert(const KV& kv, int P, int pshift, uint64_t seed);
// KV(zone, {zone, 0}) -> (zone without the hot bit, pad), plus one copy per
// salted key (r << pshift | hot bit, r < P) of every hot zone's record
std::pair<at::Tensor, at::Tensor> ccmr_zone_multi(const KV& kv, int P, int pshift);
// zone key -> {vertices (8 B), change records (16 B)}: (vertex, new zone)
std::pair<at::Tensor, at::Tensor> ccmr_reassign(const KMV& m, int64_t lmask, int64_t nthresh);
}  // namespace mrh
