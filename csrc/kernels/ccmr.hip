// cc_find_mr: the reference's zone-based connected components pipeline
// (oink/cc_find.cpp:38-109, callbacks :119-330) — its map/reduce callbacks as
// device kernels on the KMV / KV columns (the zone key's bit 63 marks a hot
// zone, the bits under it carry the salting rank):
//
//  edge_zone    reduce_edge_zone: a vertex's zone (its 8-byte value) rides
//               along to each of its edges (16-byte values)
//  winner       reduce_zone_winner: an edge whose two ends are in different
//               zones emits (larger zone -> {smaller zone, 0})
//  invert       map_invert_multi: (v, zone) -> (zone, v); a hot zone's
//               vertices go to a random salted copy of the zone key
//  zone_multi   map_zone_multi: zone-change records, replicated to every
//               salted copy of a hot zone
//  reassign     reduce_zone_reassign: a zone key's vertices take the smallest
//               winning zone (its hot bit comes along), and the zone turns
//               hot above nthresh vertices
//
// Items are values (segment found by binary search: a hub's segment may hold
// millions of values) or keys; every emitting kernel writes at the offsets of
// an exclusive scan of its flags, so the output order is the input order.
#include <algorithm>

#include "common.h"
#include "launch.h"

namespace mrh {
namespace k {
namespace {

constexpr int NT = 256;
constexpr int64_t HIBIT = (int64_t)(1ull << 63);
inline unsigned blocks(int64_t n) { return (unsigned)std::min<int64_t>((n + NT - 1) / NT, 1 << 20); }

__device__ inline int64_t seg_of(const int64_t* __restrict__ seg, int64_t nseg, int64_t j) {
  int64_t lo = 0, hi = nseg;
  while (hi - lo > 1) {
    const int64_t mid = (lo + hi) >> 1;
    if (seg[mid] <= j) lo = mid;
    else hi = mid;
  }
  return lo;
}

__device__ inline int64_t load8(const uint8_t* p) {
  int64_t v;
  __builtin_memcpy(&v, p, 8);
  return v;
}

#define GRID_LOOP(i, n) for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < (n); i += (int64_t)gridDim.x * NT)

// value lengths == w -> int64 flags
__global__ __launch_bounds__(NT) void k_len_flags(const int64_t* __restrict__ voff, int64_t nval, int64_t w,
                                                 int64_t* __restrict__ f) {
  GRID_LOOP(j, nval) f[j] = (voff[j + 1] - voff[j]) == w;
}

__global__ __launch_bounds__(NT) void k_edge_zone_of(const int64_t* __restrict__ seg, int64_t nkey,
                                                    const int64_t* __restrict__ voff, const uint8_t* __restrict__ vd,
                                                    int64_t nval, int64_t* __restrict__ zone_of) {
  GRID_LOOP(j, nval) {
    if (voff[j + 1] - voff[j] == 8) zone_of[seg_of(seg, nkey, j)] = load8(vd + voff[j]);
  }
}

__global__ __launch_bounds__(NT) void k_edge_zone_emit(const int64_t* __restrict__ seg, int64_t nkey,
                                                      const int64_t* __restrict__ voff,
                                                      const uint8_t* __restrict__ vd, int64_t nval,
                                                      const int64_t* __restrict__ zone_of,
                                                      const int64_t* __restrict__ pos, int64_t* __restrict__ edge,
                                                      int64_t* __restrict__ zone) {
  GRID_LOOP(j, nval) {
    const int64_t b = voff[j];
    if (voff[j + 1] - b != 16) continue;
    const int64_t p = pos[j];
    edge[2 * p] = load8(vd + b);
    edge[2 * p + 1] = load8(vd + b + 8);
    zone[p] = zone_of[seg_of(seg, nkey, j)];
  }
}

__global__ __launch_bounds__(NT) void k_winner_flags(const int64_t* __restrict__ seg, int64_t nkey,
                                                    const int64_t* __restrict__ z, int64_t nval,
                                                    int64_t* __restrict__ f) {
  GRID_LOOP(s, nkey) {
    const int64_t h = seg[s];
    const int64_t z0 = z[h], z1 = z[h + 1 < nval ? h + 1 : nval - 1];
    f[s] = (z0 & ~HIBIT) != (z1 & ~HIBIT);
  }
}

__global__ __launch_bounds__(NT) void k_winner_emit(const int64_t* __restrict__ seg, int64_t nkey,
                                                   const int64_t* __restrict__ z, int64_t nval,
                                                   const int64_t* __restrict__ pos, int64_t* __restrict__ big,
                                                   int64_t* __restrict__ pad) {
  GRID_LOOP(s, nkey) {
    if (pos[s + 1] == pos[s]) continue;
    const int64_t h = seg[s];
    const int64_t z0 = z[h], z1 = z[h + 1 < nval ? h + 1 : nval - 1];
    const bool first = (z0 & ~HIBIT) > (z1 & ~HIBIT);
    const int64_t p = pos[s];
    big[p] = first ? z0 : z1;
    pad[2 * p] = first ? z1 : z0;
    pad[2 * p + 1] = 0;
  }
}

__device__ inline uint64_t mix64(uint64_t x) {  // splitmix64 finaliser
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

__global__ __launch_bounds__(NT) void k_invert(const int64_t* __restrict__ v, const int64_t* __restrict__ zn,
                                              int64_t n, int P, int pshift, uint64_t seed,
                                              int64_t* __restrict__ key, int64_t* __restrict__ val) {
  GRID_LOOP(i, n) {
    const int64_t z = zn[i];
    const int64_t rp = (int64_t)(mix64(seed ^ (uint64_t)i) % (uint64_t)P);
    key[i] = z < 0 ? (z | (rp << pshift)) : z;
    val[i] = v[i];
  }
}

__global__ __launch_bounds__(NT) void k_hot_flags(const int64_t* __restrict__ zn, int64_t n, int64_t* __restrict__ f) {
  GRID_LOOP(i, n) f[i] = zn[i] < 0;
}

__global__ __launch_bounds__(NT) void k_zone_multi(const int64_t* __restrict__ zn, const int64_t* __restrict__ pad,
                                                  int64_t n, int P, int pshift, const int64_t* __restrict__ pos,
                                                  int64_t* __restrict__ key, int64_t* __restrict__ val) {
  GRID_LOOP(i, n) {
    const int64_t z = zn[i], strip = z & ~HIBIT, p0 = pad[2 * i], p1 = pad[2 * i + 1];
    key[i] = strip;
    val[2 * i] = p0;
    val[2 * i + 1] = p1;
    if (z < 0) {
      const int64_t o = n + pos[i] * P;
      for (int r = 0; r < P; ++r) {
        key[o + r] = strip | ((int64_t)r << pshift) | HIBIT;
        val[2 * (o + r)] = p0;
        val[2 * (o + r) + 1] = p1;
      }
    }
  }
}

// per zone key: the smallest zone among the key's own and its change records
// (8-byte values: vertices, 16-byte: {zone, 0} records), hot when the key was,
// when a record carrying the hot bit wins, or above nthresh vertices
__global__ __launch_bounds__(NT) void k_reassign_seg(const int64_t* __restrict__ seg, int64_t nkey,
                                                    const int64_t* __restrict__ keys,
                                                    const int64_t* __restrict__ voff,
                                                    const uint8_t* __restrict__ vd, int64_t lmask, int64_t nthresh,
                                                    int64_t* __restrict__ zone_out) {
  GRID_LOOP(s, nkey) {
    const int64_t key = keys[s], zone = key & lmask;
    int64_t best = zone, nvert = 0;
    for (int64_t j = seg[s]; j < seg[s + 1]; ++j) {
      const int64_t l = voff[j + 1] - voff[j];
      if (l == 8) ++nvert;
      else if (l == 16) best = std::min<int64_t>(best, load8(vd + voff[j]) & ~HIBIT);
    }
    bool hwin = false;
    if (best < zone)
      for (int64_t j = seg[s]; j < seg[s + 1] && !hwin; ++j) {
        if (voff[j + 1] - voff[j] != 16) continue;
        const int64_t pz = load8(vd + voff[j]);
        hwin = pz < 0 && (pz & ~HIBIT) == best;
      }
    const bool hot = key < 0 || hwin || nvert > nthresh;
    zone_out[s] = hot ? (best | HIBIT) : best;
  }
}

__global__ __launch_bounds__(NT) void k_reassign_emit(const int64_t* __restrict__ seg, int64_t nkey,
                                                     const int64_t* __restrict__ voff,
                                                     const uint8_t* __restrict__ vd, int64_t nval,
                                                     const int64_t* __restrict__ zone_seg,
                                                     const int64_t* __restrict__ pos, int64_t* __restrict__ v,
                                                     int64_t* __restrict__ zone) {
  GRID_LOOP(j, nval) {
    if (voff[j + 1] - voff[j] != 8) continue;
    const int64_t p = pos[j];
    v[p] = load8(vd + voff[j]);
    zone[p] = zone_seg[seg_of(seg, nkey, j)];
  }
}

}  // namespace

#define LAUNCH(kern, n, ...)                                                          \
  do {                                                                                \
    if ((n) > 0) {                                                                    \
      hipLaunchKernelGGL(kern, dim3(blocks(n)), dim3(NT), 0, s, __VA_ARGS__);        \
      MRH_CHECK_LAUNCH();                                                             \
    }                                                                                 \
  } while (0)

void ccmr_len_flags(const int64_t* voff, int64_t nval, int64_t w, int64_t* f, hipStream_t s) {
  LAUNCH(k_len_flags, nval, voff, nval, w, f);
}
void ccmr_edge_zone_of(const int64_t* seg, int64_t nkey, const int64_t* voff, const uint8_t* vd, int64_t nval,
                       int64_t* zone_of, hipStream_t s) {
  if (nkey > 0) LAUNCH(k_edge_zone_of, nval, seg, nkey, voff, vd, nval, zone_of);
}
void ccmr_edge_zone_emit(const int64_t* seg, int64_t nkey, const int64_t* voff, const uint8_t* vd, int64_t nval,
                         const int64_t* zone_of, const int64_t* pos, int64_t* edge, int64_t* zone, hipStream_t s) {
  if (nkey > 0) LAUNCH(k_edge_zone_emit, nval, seg, nkey, voff, vd, nval, zone_of, pos, edge, zone);
}
void ccmr_winner_flags(const int64_t* seg, int64_t nkey, const int64_t* z, int64_t nval, int64_t* f, hipStream_t s) {
  if (nval > 0) LAUNCH(k_winner_flags, nkey, seg, nkey, z, nval, f);
}
void ccmr_winner_emit(const int64_t* seg, int64_t nkey, const int64_t* z, int64_t nval, const int64_t* pos,
                      int64_t* big, int64_t* pad, hipStream_t s) {
  if (nval > 0) LAUNCH(k_winner_emit, nkey, seg, nkey, z, nval, pos, big, pad);
}
void ccmr_invert(const int64_t* v, const int64_t* zn, int64_t n, int P, int pshift, uint64_t seed, int64_t* key,
                 int64_t* val, hipStream_t s) {
  LAUNCH(k_invert, n, v, zn, n, P, pshift, seed, key, val);
}
void ccmr_hot_flags(const int64_t* zn, int64_t n, int64_t* f, hipStream_t s) { LAUNCH(k_hot_flags, n, zn, n, f); }
void ccmr_zone_multi(const int64_t* zn, const int64_t* pad, int64_t n, int P, int pshift, const int64_t* pos,
                     int64_t* key, int64_t* val, hipStream_t s) {
  LAUNCH(k_zone_multi, n, zn, pad, n, P, pshift, pos, key, val);
}
void ccmr_reassign_seg(const int64_t* seg, int64_t nkey, const int64_t* keys, const int64_t* voff, const uint8_t* vd,
                       int64_t lmask, int64_t nthresh, int64_t* zone_out, hipStream_t s) {
  LAUNCH(k_reassign_seg, nkey, seg, nkey, keys, voff, vd, lmask, nthresh, zone_out);
}
void ccmr_reassign_emit(const int64_t* seg, int64_t nkey, const int64_t* voff, const uint8_t* vd, int64_t nval,
                        const int64_t* zone_seg, const int64_t* pos, int64_t* v, int64_t* zone, hipStream_t s) {
  if (nkey > 0) LAUNCH(k_reassign_emit, nval, seg, nkey, voff, vd, nval, zone_seg, pos, v, zone);
}

}  // namespace k
}  // namespace mrh
