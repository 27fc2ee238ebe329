// sssp_mr and luby_find_mr: the reference's MapReduce formulations of single-
// source shortest paths (oink/sssp.cpp:88-152, callbacks :187-360) and of
// Luby's maximal independent set (oink/luby_find.cpp:53-97, callbacks
// :120-344) — their reduce / compress callbacks as device kernels on the KMV
// columns. Records are 8-byte words:
//
//   DISTANCE  {pred, wt (double), current}  24 B  (sssp.h:47-67)
//   EDGEVALUE {v, wt (double)}              16 B  (sssp.h:34-45)
//   ERAND     {vi, ri, vj, rj}              32 B key (luby_find.cpp:36-41)
//   VRAND     {v, r}                        16 B
//   VFLAG     {v, r, flag}                  24 B  (the reference's struct pads to 24)
//
// Mixed values (edges and distances in one key's multivalue; VRAND and VFLAG)
// are told apart by their length, as the reference does. Per-key decisions
// that scan a whole multivalue (a hub can hold millions of values) are made by
// value-parallel kernels (segment by binary search) with benign-race stores or
// 64-bit atomics into per-key words; every emitting kernel writes at the
// offsets of an exclusive scan of its flags, so output order is input order.
#include <algorithm>

#include "common.h"
#include "launch.h"

namespace mrh {
namespace k {
namespace {

constexpr int NT = 256;
constexpr double FLTMAX = 3.4028234663852886e+38;  // (double)FLT_MAX: DISTANCE()'s "unreached"
inline unsigned blocks(int64_t n) { return (unsigned)std::min<int64_t>((n + NT - 1) / NT, 1 << 20); }

#define GRID_LOOP(i, n) for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < (n); i += (int64_t)gridDim.x * NT)

__device__ inline int64_t seg_of(const int64_t* __restrict__ seg, int64_t nseg, int64_t j) {
  int64_t lo = 0, hi = nseg;
  while (hi - lo > 1) {
    const int64_t mid = (lo + hi) >> 1;
    if (seg[mid] <= j) lo = mid;
    else hi = mid;
  }
  return lo;
}
__device__ inline int64_t ld8(const uint8_t* p) {
  int64_t v;
  __builtin_memcpy(&v, p, 8);
  return v;
}
__device__ inline double ldd(const uint8_t* p) {
  double v;
  __builtin_memcpy(&v, p, 8);
  return v;
}
__device__ inline double as_d(int64_t b) { return __longlong_as_double(b); }
__device__ inline int64_t as_l(double d) { return __double_as_longlong(d); }
// doubles -> unsigned keys in numeric order (negative ones flipped)
__device__ inline unsigned long long dkey(double d) {
  const unsigned long long b = (unsigned long long)as_l(d);
  return (b >> 63) ? ~b : (b | (1ull << 63));
}
__device__ inline int64_t vlen(const int64_t* __restrict__ voff, int64_t vw, int64_t j) {
  return voff ? voff[j + 1] - voff[j] : vw;
}
__device__ inline int64_t vbeg(const int64_t* __restrict__ voff, int64_t vw, int64_t j) {
  return voff ? voff[j] : j * vw;
}

// ------------------------------------------------------------------ sssp_mr

// pick_shortest_distances (sssp.cpp:244-293), one key per thread: previous =
// the last current record, shortest = previous unless a record is strictly
// shorter (the first such in value order) — the reference's scan with the
// vertex's own record first, as its kv order puts it. A single value is both.
__global__ __launch_bounds__(NT) void k_sssp_pick(const int64_t* __restrict__ seg, int64_t nkey,
                                                 const int64_t* __restrict__ voff, int64_t vw,
                                                 const uint8_t* __restrict__ vd, int64_t* __restrict__ out,
                                                 int64_t* __restrict__ changed) {
  GRID_LOOP(s, nkey) {
    const int64_t j0 = seg[s], j1 = seg[s + 1];
    int64_t pp = 0, sp;
    double pw = FLTMAX, sw;
    for (int64_t j = j0; j < j1; ++j) {
      const uint8_t* r = vd + vbeg(voff, vw, j);
      if (ld8(r + 16)) {
        pp = ld8(r);
        pw = ldd(r + 8);
      }
    }
    if (j1 - j0 == 1) {
      const uint8_t* r = vd + vbeg(voff, vw, j0);
      pp = sp = ld8(r);
      pw = sw = ldd(r + 8);
    } else {
      sp = pw < FLTMAX ? pp : 0;
      sw = pw < FLTMAX ? pw : FLTMAX;
      for (int64_t j = j0; j < j1; ++j) {
        const uint8_t* r = vd + vbeg(voff, vw, j);
        const double w = ldd(r + 8);
        if (w < sw) {
          sw = w;
          sp = ld8(r);
        }
      }
    }
    out[3 * s] = sp;
    out[3 * s + 1] = as_l(sw);
    out[3 * s + 2] = 1;
    changed[s] = (pp != sp) || (pw != sw);
  }
}

__global__ __launch_bounds__(NT) void k_sssp_pick_emit(const int64_t* __restrict__ keys, int64_t nkey,
                                                      const int64_t* __restrict__ dist,
                                                      const int64_t* __restrict__ pos, int64_t* __restrict__ okey,
                                                      int64_t* __restrict__ odist) {
  GRID_LOOP(s, nkey) {
    const int64_t p = pos[s];
    if (pos[s + 1] == p) continue;
    okey[p] = keys[s];
    odist[3 * p] = dist[3 * s];
    odist[3 * p + 1] = dist[3 * s + 1];
    odist[3 * p + 2] = dist[3 * s + 2];
  }
}

// update_adjacent_distances (sssp.cpp:299-360), value-parallel. Pass 1: every
// distance record marks its key found and min-reduces its weight key.
__global__ __launch_bounds__(NT) void k_sssp_best_wt(const int64_t* __restrict__ seg, int64_t nkey,
                                                    const int64_t* __restrict__ voff, const uint8_t* __restrict__ vd,
                                                    int64_t nval, unsigned long long* __restrict__ best,
                                                    int64_t* __restrict__ found) {
  GRID_LOOP(j, nval) {
    if (voff[j + 1] - voff[j] != 24) continue;
    const int64_t s = seg_of(seg, nkey, j);
    found[s] = 1;
    const double w = ldd(vd + voff[j] + 8);
    if (w < FLTMAX) atomicMin(best + s, dkey(w));
  }
}
// pass 2: the first record in value order with the minimum weight
__global__ __launch_bounds__(NT) void k_sssp_best_idx(const int64_t* __restrict__ seg, int64_t nkey,
                                                     const int64_t* __restrict__ voff, const uint8_t* __restrict__ vd,
                                                     int64_t nval, const unsigned long long* __restrict__ best,
                                                     unsigned long long* __restrict__ idx) {
  GRID_LOOP(j, nval) {
    if (voff[j + 1] - voff[j] != 24) continue;
    const int64_t s = seg_of(seg, nkey, j);
    const double w = ldd(vd + voff[j] + 8);
    if (w < FLTMAX && dkey(w) == best[s]) atomicMin(idx + s, (unsigned long long)j);
  }
}
// the shortest distance of value j's key: {pred, wt}; found = a distance was there
__device__ inline bool sssp_shortest(const int64_t* __restrict__ voff, const uint8_t* __restrict__ vd,
                                     const unsigned long long* __restrict__ idx,
                                     const int64_t* __restrict__ found, int64_t s, int64_t& sp, double& sw) {
  const unsigned long long b = idx[s];
  if (b != ~0ull) {
    sp = ld8(vd + voff[b]);
    sw = ldd(vd + voff[b] + 8);
  } else {
    sp = 0;
    sw = FLTMAX;
  }
  return found[s] != 0;
}
// fe: an edge (re-emitted into mredge); fp: an edge that relaxes (not back to
// the predecessor, not a self loop) from a key whose distance changed
__global__ __launch_bounds__(NT) void k_sssp_relax_flags(const int64_t* __restrict__ seg, int64_t nkey,
                                                        const int64_t* __restrict__ keys,
                                                        const int64_t* __restrict__ voff,
                                                        const uint8_t* __restrict__ vd, int64_t nval,
                                                        const unsigned long long* __restrict__ idx,
                                                        const int64_t* __restrict__ found, int64_t* __restrict__ fe,
                                                        int64_t* __restrict__ fp) {
  GRID_LOOP(j, nval) {
    const bool edge = voff[j + 1] - voff[j] == 16;
    fe[j] = edge;
    int64_t f = 0;
    if (edge) {
      const int64_t s = seg_of(seg, nkey, j);
      int64_t sp;
      double sw;
      if (sssp_shortest(voff, vd, idx, found, s, sp, sw)) {
        const int64_t v = ld8(vd + voff[j]);
        f = (sp != v) && (v != keys[s]);
      }
    }
    fp[j] = f;
  }
}
__global__ __launch_bounds__(NT) void k_sssp_relax_emit(const int64_t* __restrict__ seg, int64_t nkey,
                                                       const int64_t* __restrict__ keys,
                                                       const int64_t* __restrict__ voff,
                                                       const uint8_t* __restrict__ vd, int64_t nval,
                                                       const unsigned long long* __restrict__ idx,
                                                       const int64_t* __restrict__ found,
                                                       const int64_t* __restrict__ pe, const int64_t* __restrict__ pp,
                                                       int64_t* __restrict__ ekey, int64_t* __restrict__ eval,
                                                       int64_t* __restrict__ pkey, int64_t* __restrict__ pval) {
  GRID_LOOP(j, nval) {
    if (pe[j + 1] == pe[j]) continue;
    const int64_t s = seg_of(seg, nkey, j);
    const uint8_t* r = vd + voff[j];
    const int64_t v = ld8(r), wb = ld8(r + 8), key = keys[s];
    const int64_t e = pe[j];
    ekey[e] = key;
    eval[2 * e] = v;
    eval[2 * e + 1] = wb;
    if (pp[j + 1] == pp[j]) continue;
    int64_t sp;
    double sw;
    sssp_shortest(voff, vd, idx, found, s, sp, sw);
    const int64_t p = pp[j];
    pkey[p] = v;
    pval[3 * p] = key;
    pval[3 * p + 1] = as_l(sw + as_d(wb));
    pval[3 * p + 2] = 0;
  }
}

// ------------------------------------------------------------------ luby_find_mr

// srand48(v + seed); drand48() (map_vert_random, luby_find.cpp:120-136): the
// 48-bit LCG state seeded with the low 32 bits << 16 | 0x330E, one step, / 2^48
__device__ inline double luby_rand(int64_t v, int64_t seed) {
  const uint64_t x0 = ((uint64_t)(uint32_t)(v + seed) << 16) | 0x330Eull;
  const uint64_t x1 = (0x5DEECE66Dull * x0 + 0xBull) & ((1ull << 48) - 1);
  return (double)x1 * 0x1p-48;
}
__global__ __launch_bounds__(NT) void k_luby_nonloop(const int64_t* __restrict__ e, int64_t n, int64_t* __restrict__ f) {
  GRID_LOOP(i, n) f[i] = e[2 * i] != e[2 * i + 1];
}
__global__ __launch_bounds__(NT) void k_luby_random(const int64_t* __restrict__ e, int64_t n, int64_t seed,
                                                   const int64_t* __restrict__ pos, int64_t* __restrict__ out) {
  GRID_LOOP(i, n) {
    const int64_t p = pos[i];
    if (pos[i + 1] == p) continue;
    const int64_t vi = e[2 * i], vj = e[2 * i + 1];
    out[4 * p] = vi;
    out[4 * p + 1] = as_l(luby_rand(vi, seed));
    out[4 * p + 2] = vj;
    out[4 * p + 3] = as_l(luby_rand(vj, seed));
  }
}
// per-key marks from the values (benign races: every writer stores 1).
//   mode 0 (reduce_vert_winner :186-208): a VFLAG with flag 0 (lost an edge)
//   mode 1 (reduce_vert_loser  :238-258): a value longer than 16 B (a winner's VFLAG)
//   mode 2 (reduce_vert_emit   :289-309): a 16-byte value (a neighbour that stays)
//   mode 3 (reduce_edge_winner :140-144): any non-empty value (an end was removed)
__global__ __launch_bounds__(NT) void k_luby_mark(const int64_t* __restrict__ seg, int64_t nkey,
                                                 const int64_t* __restrict__ voff, int64_t vw,
                                                 const uint8_t* __restrict__ vd, int64_t nval, int mode,
                                                 int64_t* __restrict__ mark) {
  GRID_LOOP(j, nval) {
    const int64_t l = vlen(voff, vw, j);
    bool m;
    if (mode == 0) m = ld8(vd + vbeg(voff, vw, j) + 16) == 0;
    else if (mode == 1) m = l > 16;
    else if (mode == 2) m = l == 16;
    else m = l > 0;
    if (m) mark[seg_of(seg, nkey, j)] = 1;
  }
}
// per key: f = (mark == want)
__global__ __launch_bounds__(NT) void k_luby_key_flags(const int64_t* __restrict__ mark, int64_t nkey, int64_t want,
                                                      int64_t* __restrict__ f) {
  GRID_LOOP(s, nkey) f[s] = mark[s] == want;
}
// live edge keys emit (winner VRAND, VFLAG{loser, 1}) and (loser VRAND, VFLAG{winner, 0})
__global__ __launch_bounds__(NT) void k_luby_edge_emit(const int64_t* __restrict__ keys, int64_t nkey,
                                                      const int64_t* __restrict__ pos, int64_t* __restrict__ okey,
                                                      int64_t* __restrict__ oval) {
  GRID_LOOP(s, nkey) {
    const int64_t p = pos[s];
    if (pos[s + 1] == p) continue;
    const int64_t vi = keys[4 * s], bi = keys[4 * s + 1], vj = keys[4 * s + 2], bj = keys[4 * s + 3];
    const double ri = as_d(bi), rj = as_d(bj);
    const bool first = ri < rj || (!(rj < ri) && (uint64_t)vi < (uint64_t)vj);
    const int64_t wv = first ? vi : vj, wb = first ? bi : bj, lv = first ? vj : vi, lb = first ? bj : bi;
    int64_t* k0 = okey + 4 * p;
    int64_t* v0 = oval + 6 * p;
    k0[0] = wv;
    k0[1] = wb;
    v0[0] = lv;
    v0[1] = lb;
    v0[2] = 1;
    k0[2] = lv;
    k0[3] = lb;
    v0[3] = wv;
    v0[4] = wb;
    v0[5] = 0;
  }
}
// per value: f = the key's mark selects the 24-byte record (want) / the value
// is not a 16-byte VRAND (mode 2's edges with a flag)
__global__ __launch_bounds__(NT) void k_luby_value_flags(const int64_t* __restrict__ seg, int64_t nkey,
                                                        const int64_t* __restrict__ voff, int64_t vw,
                                                        const int64_t* __restrict__ mark, int64_t nval, int64_t want,
                                                        int64_t* __restrict__ f) {
  GRID_LOOP(j, nval) {
    if (mark) f[j] = mark[seg_of(seg, nkey, j)] == want;
    else f[j] = vlen(voff, vw, j) != 16;
  }
}
// reduce_vert_winner / _loser emit: for each value (a neighbour u), key =
// VRAND of u, value = this key's VRAND, with flag 0 when f24 says so
__global__ __launch_bounds__(NT) void k_luby_vert_emit(const int64_t* __restrict__ seg, int64_t nkey,
                                                      const int64_t* __restrict__ keys,
                                                      const int64_t* __restrict__ voff, int64_t vw,
                                                      const uint8_t* __restrict__ vd, int64_t nval,
                                                      const int64_t* __restrict__ p24, int64_t* __restrict__ k24,
                                                      int64_t* __restrict__ v24, int64_t* __restrict__ k16,
                                                      int64_t* __restrict__ v16) {
  GRID_LOOP(j, nval) {
    const int64_t s = seg_of(seg, nkey, j);
    const uint8_t* r = vd + vbeg(voff, vw, j);
    const int64_t u = ld8(r), ub = ld8(r + 8);
    const int64_t p = p24[j];
    if (p24[j + 1] != p) {
      k24[2 * p] = u;
      k24[2 * p + 1] = ub;
      v24[3 * p] = keys[2 * s];
      v24[3 * p + 1] = keys[2 * s + 1];
      v24[3 * p + 2] = 0;
    } else {
      const int64_t q = j - p;
      k16[2 * q] = u;
      k16[2 * q + 1] = ub;
      v16[2 * q] = keys[2 * s];
      v16[2 * q + 1] = keys[2 * s + 1];
    }
  }
}
// reduce_vert_emit's edges: ERAND with the smaller vertex first; flagged (the
// neighbour's value was a VFLAG) edges carry an int 0, the others no value
__global__ __launch_bounds__(NT) void k_luby_edges_emit(const int64_t* __restrict__ seg, int64_t nkey,
                                                       const int64_t* __restrict__ keys,
                                                       const int64_t* __restrict__ voff, int64_t vw,
                                                       const uint8_t* __restrict__ vd, int64_t nval,
                                                       const int64_t* __restrict__ pf, int64_t* __restrict__ kf,
                                                       int64_t* __restrict__ kn) {
  GRID_LOOP(j, nval) {
    const int64_t s = seg_of(seg, nkey, j);
    const uint8_t* r = vd + vbeg(voff, vw, j);
    const int64_t u = ld8(r), ub = ld8(r + 8), v = keys[2 * s], vb = keys[2 * s + 1];
    const bool vfirst = (uint64_t)v < (uint64_t)u;
    const int64_t p = pf[j];
    int64_t* o = (pf[j + 1] != p) ? kf + 4 * p : kn + 4 * (j - p);
    o[0] = vfirst ? v : u;
    o[1] = vfirst ? vb : ub;
    o[2] = vfirst ? u : v;
    o[3] = vfirst ? ub : vb;
  }
}
__global__ __launch_bounds__(NT) void k_luby_mis_emit(const int64_t* __restrict__ keys, int64_t nkey,
                                                     const int64_t* __restrict__ pos, int64_t* __restrict__ out) {
  GRID_LOOP(s, nkey) {
    if (pos[s + 1] != pos[s]) out[pos[s]] = keys[2 * s];
  }
}

}  // namespace

#define LAUNCH(kern, n, ...)                                                   \
  do {                                                                         \
    if ((n) > 0) {                                                             \
      hipLaunchKernelGGL(kern, dim3(blocks(n)), dim3(NT), 0, s, __VA_ARGS__); \
      MRH_CHECK_LAUNCH();                                                      \
    }                                                                          \
  } while (0)

void sssp_pick(const int64_t* seg, int64_t nkey, const int64_t* voff, int64_t vw, const uint8_t* vd, int64_t* out,
               int64_t* changed, hipStream_t s) {
  LAUNCH(k_sssp_pick, nkey, seg, nkey, voff, vw, vd, out, changed);
}
void sssp_pick_emit(const int64_t* keys, int64_t nkey, const int64_t* dist, const int64_t* pos, int64_t* okey,
                    int64_t* odist, hipStream_t s) {
  LAUNCH(k_sssp_pick_emit, nkey, keys, nkey, dist, pos, okey, odist);
}
void sssp_best(const int64_t* seg, int64_t nkey, const int64_t* voff, const uint8_t* vd, int64_t nval,
               unsigned long long* best, unsigned long long* idx, int64_t* found, hipStream_t s) {
  if (nkey <= 0) return;
  LAUNCH(k_sssp_best_wt, nval, seg, nkey, voff, vd, nval, best, found);
  LAUNCH(k_sssp_best_idx, nval, seg, nkey, voff, vd, nval, best, idx);
}
void sssp_relax_flags(const int64_t* seg, int64_t nkey, const int64_t* keys, const int64_t* voff, const uint8_t* vd,
                      int64_t nval, const unsigned long long* idx, const int64_t* found, int64_t* fe, int64_t* fp,
                      hipStream_t s) {
  if (nkey > 0) LAUNCH(k_sssp_relax_flags, nval, seg, nkey, keys, voff, vd, nval, idx, found, fe, fp);
}
void sssp_relax_emit(const int64_t* seg, int64_t nkey, const int64_t* keys, const int64_t* voff, const uint8_t* vd,
                     int64_t nval, const unsigned long long* idx, const int64_t* found, const int64_t* pe,
                     const int64_t* pp, int64_t* ekey, int64_t* eval, int64_t* pkey, int64_t* pval, hipStream_t s) {
  if (nkey > 0)
    LAUNCH(k_sssp_relax_emit, nval, seg, nkey, keys, voff, vd, nval, idx, found, pe, pp, ekey, eval, pkey, pval);
}
void luby_nonloop(const int64_t* e, int64_t n, int64_t* f, hipStream_t s) { LAUNCH(k_luby_nonloop, n, e, n, f); }
void luby_random(const int64_t* e, int64_t n, int64_t seed, const int64_t* pos, int64_t* out, hipStream_t s) {
  LAUNCH(k_luby_random, n, e, n, seed, pos, out);
}
void luby_mark(const int64_t* seg, int64_t nkey, const int64_t* voff, int64_t vw, const uint8_t* vd, int64_t nval,
               int mode, int64_t* mark, hipStream_t s) {
  if (nkey > 0) LAUNCH(k_luby_mark, nval, seg, nkey, voff, vw, vd, nval, mode, mark);
}
void luby_key_flags(const int64_t* mark, int64_t nkey, int64_t want, int64_t* f, hipStream_t s) {
  LAUNCH(k_luby_key_flags, nkey, mark, nkey, want, f);
}
void luby_edge_emit(const int64_t* keys, int64_t nkey, const int64_t* pos, int64_t* okey, int64_t* oval,
                    hipStream_t s) {
  LAUNCH(k_luby_edge_emit, nkey, keys, nkey, pos, okey, oval);
}
void luby_value_flags(const int64_t* seg, int64_t nkey, const int64_t* voff, int64_t vw, const int64_t* mark,
                      int64_t nval, int64_t want, int64_t* f, hipStream_t s) {
  if (nkey > 0) LAUNCH(k_luby_value_flags, nval, seg, nkey, voff, vw, mark, nval, want, f);
}
void luby_vert_emit(const int64_t* seg, int64_t nkey, const int64_t* keys, const int64_t* voff, int64_t vw,
                    const uint8_t* vd, int64_t nval, const int64_t* p24, int64_t* k24, int64_t* v24, int64_t* k16,
                    int64_t* v16, hipStream_t s) {
  if (nkey > 0) LAUNCH(k_luby_vert_emit, nval, seg, nkey, keys, voff, vw, vd, nval, p24, k24, v24, k16, v16);
}
void luby_edges_emit(const int64_t* seg, int64_t nkey, const int64_t* keys, const int64_t* voff, int64_t vw,
                     const uint8_t* vd, int64_t nval, const int64_t* pf, int64_t* kf, int64_t* kn, hipStream_t s) {
  if (nkey > 0) LAUNCH(k_luby_edges_emit, nval, seg, nkey, keys, voff, vw, vd, nval, pf, kf, kn);
}
void luby_mis_emit(const int64_t* keys, int64_t nkey, const int64_t* pos, int64_t* out, hipStream_t s) {
  LAUNCH(k_luby_mis_emit, nkey, keys, nkey, pos, out);
}

}  // namespace k
}  // namespace mrh
