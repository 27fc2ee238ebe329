// Triangle enumeration kernels (the tri_find workload, reference
// oink/tri_find.cpp:43-82, re-designed for one GPU holding the whole graph).
//
// The reference finds triangles with 4 MapReduce shuffles and materialises
// every wedge (O(sum d^2) KVs, :207-276). Here the deduplicated edge list is
// replicated in HBM (RMAT-24 x16 is ~2 GB, 288 GB per GPU), oriented from the
// lower to the higher (degree, id) endpoint — the same low-degree rule as the
// reference's map_low_degree — and stored as CSR with sorted rows. Every
// triangle a<b<c (in that order) is then found exactly once, on edge (a,b),
// as the element c of N+(a) ∩ N+(b): a sorted-list intersection per edge, no
// wedge ever materialised. Ranks split the oriented edge range.
//
//   k_tri_degree : deg[v] += 1 for both endpoints of every edge
//   k_tri_orient : packed (lo<<32|hi) -> packed (src<<32|dst), src = lower (deg,id)
//   k_tri_count  : per oriented edge |N+(u) ∩ N+(v)| (merge intersection,
//                  galloping when the lists are unbalanced); optional per-edge
//                  counts; wave-reduced total
//   k_tri_emit   : the triangles (u, v, w) at exclusive-scan offsets
#include "common.h"
#include "launch.h"
#include <algorithm>
#include <cstdlib>
#include <string>

namespace mrh {
namespace k {
namespace {

constexpr int NT = 256;

// the edges are sorted by their low endpoint: a wave counts each run of equal
// low endpoints with one atomic (R-MAT hubs would otherwise serialise 64
// lanes on one address); the high endpoints are scattered, one atomic each
__global__ __launch_bounds__(NT) void k_tri_degree(const uint64_t* __restrict__ e, int64_t m,
                                                  uint32_t* __restrict__ deg) {
  const int lane = dev::lane_id();
  const int64_t stride = (int64_t)gridDim.x * NT;
  for (int64_t base = (int64_t)blockIdx.x * NT + (threadIdx.x & ~(MRH_WAVE - 1)); base < m; base += stride) {
    const int64_t i = base + lane;
    const bool ok = i < m;
    const uint64_t x = ok ? e[i] : ~0ull;
    const uint32_t lo = (uint32_t)(x >> 32);
    const uint32_t prev = __shfl_up(lo, 1, MRH_WAVE);
    const uint64_t heads = __ballot(ok && (lane == 0 || lo != prev));
    const uint64_t okm = __ballot(ok);
    if (ok && ((heads >> lane) & 1ull)) {
      const uint64_t above = heads & ~((2ull << lane) - 1ull);  // heads after this lane
      const int end = above ? __ffsll((long long)above) - 1 : 64 - __clzll(okm);
      atomicAdd(deg + lo, (uint32_t)(end - lane));
    }
    if (ok) atomicAdd(deg + (uint32_t)x, 1u);
  }
}

// Degrees without scattered atomics for the high endpoints: k_tri_degree's
// one random atomic per edge ran at ~14 G/s (19 ms for RMAT-24's 268 M edges,
// contended or not). Instead:
//   k_deg_lo      : the low endpoints (sorted runs): one atomic per run per wave;
//   k_deg_count   : bucket = hi >> DEG_RB (32768 vertices): LDS histogram per
//                   block, one global add per bucket per block;
//   k_deg_scatter : the same blocks reserve their bucket ranges (one atomic per
//                   bucket per block) and write hi & 32767 as u16 into them;
//   k_deg_hist    : one block per (bucket, piece) counts its u16 ids in a
//                   32768-bin LDS histogram and adds it to deg — plain stores
//                   when the block holds the whole bucket.
constexpr int DEG_RB = 15;
constexpr int DEG_BINS = 1 << DEG_RB;
constexpr int DEG_MAXB = 4096;   // buckets (nvert <= 2^27 on this path)
constexpr int DEG_SMALLB = 1024; // the kernels' LDS tables for up to 2^25 vertices (higher occupancy)
constexpr int DEG_NT = 1024;

__global__ __launch_bounds__(NT) void k_deg_lo(const uint64_t* __restrict__ e, int64_t m, uint32_t* __restrict__ deg) {
  const int lane = dev::lane_id();
  const int64_t stride = (int64_t)gridDim.x * NT;
  for (int64_t base = (int64_t)blockIdx.x * NT + (threadIdx.x & ~(MRH_WAVE - 1)); base < m; base += stride) {
    const int64_t i = base + lane;
    const bool ok = i < m;
    const uint32_t lo = ok ? (uint32_t)(e[i] >> 32) : 0xffffffffu;
    const uint32_t prev = __shfl_up(lo, 1, MRH_WAVE);
    const uint64_t heads = __ballot(ok && (lane == 0 || lo != prev));
    const uint64_t okm = __ballot(ok);
    if (ok && ((heads >> lane) & 1ull)) {
      const uint64_t above = heads & ~((2ull << lane) - 1ull);
      const int end = above ? __ffsll((long long)above) - 1 : 64 - __clzll(okm);
      atomicAdd(deg + lo, (uint32_t)(end - lane));
    }
  }
}

template <int MAXB>
__global__ __launch_bounds__(NT) void k_deg_count(const uint64_t* __restrict__ e, int64_t m, int nb,
                                                 unsigned int* __restrict__ bcount) {
  __shared__ uint32_t h[MAXB];
  for (int i = threadIdx.x; i < nb; i += NT) h[i] = 0;
  __syncthreads();
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < m; i += (int64_t)gridDim.x * NT)
    atomicAdd(&h[(uint32_t)e[i] >> DEG_RB], 1u);
  __syncthreads();
  for (int i = threadIdx.x; i < nb; i += NT)
    if (h[i]) atomicAdd(bcount + i, h[i]);
}

// the same grid and element order as k_deg_count: every block counts its
// elements per bucket again, reserves that many slots of each bucket, then
// places its elements
template <int MAXB>
__global__ __launch_bounds__(NT) void k_deg_scatter(const uint64_t* __restrict__ e, int64_t m, int nb,
                                                   unsigned long long* __restrict__ cursor,
                                                   uint16_t* __restrict__ out) {
  __shared__ uint32_t h[MAXB];
  __shared__ unsigned long long base[MAXB];
  for (int i = threadIdx.x; i < nb; i += NT) h[i] = 0;
  __syncthreads();
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < m; i += (int64_t)gridDim.x * NT)
    atomicAdd(&h[(uint32_t)e[i] >> DEG_RB], 1u);
  __syncthreads();
  for (int i = threadIdx.x; i < nb; i += NT) {
    base[i] = h[i] ? atomicAdd(cursor + i, (unsigned long long)h[i]) : 0ull;
    h[i] = 0;
  }
  __syncthreads();
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < m; i += (int64_t)gridDim.x * NT) {
    const uint32_t hi = (uint32_t)e[i];
    const uint32_t b = hi >> DEG_RB;
    const uint32_t o = atomicAdd(&h[b], 1u);
    out[base[b] + o] = (uint16_t)(hi & (DEG_BINS - 1));
  }
}

// item = (bucket << 40 | piece start offset within the bucket, 40 bits);
// len per item in ilen; whole = the item covers its bucket (plain stores)
__global__ __launch_bounds__(DEG_NT) void k_deg_hist(const uint16_t* __restrict__ ids,
                                                    const unsigned long long* __restrict__ bstart,
                                                    const uint64_t* __restrict__ items,
                                                    const uint32_t* __restrict__ ilen,
                                                    const uint8_t* __restrict__ whole, int64_t nitems,
                                                    int64_t nvert, uint32_t* __restrict__ deg) {
  __shared__ uint32_t h[DEG_BINS];
  for (int64_t it = blockIdx.x; it < nitems; it += gridDim.x) {
    for (int i = threadIdx.x; i < DEG_BINS; i += DEG_NT) h[i] = 0;
    __syncthreads();
    const uint64_t item = items[it];
    const int64_t b = (int64_t)(item >> 40);
    const int64_t s0 = (int64_t)bstart[b] + (int64_t)(item & ((1ull << 40) - 1));
    const int64_t n = ilen[it];
    for (int64_t i = threadIdx.x; i < n; i += DEG_NT) atomicAdd(&h[ids[s0 + i]], 1u);
    __syncthreads();
    const int64_t v0 = b << DEG_RB;
    const bool w = whole[it] != 0;
    for (int i = threadIdx.x; i < DEG_BINS && v0 + i < nvert; i += DEG_NT) {
      const uint32_t c = h[i];
      if (!c) continue;
      if (w) deg[v0 + i] += c;  // this block owns the bucket's vertices
      else atomicAdd(deg + v0 + i, c);
    }
    __syncthreads();
  }
}

// [n, 2] int64 edges -> packed min << 32 | max; a self loop becomes edge
// (0, 0), i.e. key 0 (sorts first, dropped after the dedup; any other
// sentinel would make constant key bytes vary and cost radix passes) — one
// pass instead of the minimum / maximum / mask / compaction / shift / or chain
// an id outside [0, nvert) sets *bad (and packs as 0): the host checks it
// before any kernel indexes a per-vertex array with the ids
__global__ __launch_bounds__(NT) void k_tri_pack(const int64_t* __restrict__ e, int64_t n, int64_t nvert,
                                                uint64_t* __restrict__ out, unsigned int* __restrict__ bad) {
  bool oob = false;
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) {
    const uint64_t a = (uint64_t)e[2 * i], b = (uint64_t)e[2 * i + 1];
    const uint64_t lo = a < b ? a : b, hi = a < b ? b : a;
    const bool ok = hi < (uint64_t)nvert;  // unsigned: negative ids are huge
    oob |= !ok;
    out[i] = (!ok || lo == hi) ? 0ull : (lo << 32) | hi;
  }
  if (__ballot(oob) && dev::lane_id() == 0) atomicOr(bad, 1u);
}

// col[i] = low word of okeys[i]; rank[perm[r]] = r
__global__ __launch_bounds__(NT) void k_tri_col(const uint64_t* __restrict__ okeys, int64_t m,
                                               uint32_t* __restrict__ col) {
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < m; i += (int64_t)gridDim.x * NT)
    col[i] = (uint32_t)okeys[i];
}
__global__ __launch_bounds__(NT) void k_tri_rank(const int32_t* __restrict__ perm, int64_t n,
                                                int32_t* __restrict__ rank) {
  for (int64_t r = (int64_t)blockIdx.x * NT + threadIdx.x; r < n; r += (int64_t)gridDim.x * NT) rank[perm[r]] = (int32_t)r;
}

// rank[v] = position of v in (degree, id) order; the edge points from the
// lower to the higher rank and is stored in rank ids, so every row holds only
// higher ids and sorted rows can be cut at any id bound
__global__ __launch_bounds__(NT) void k_tri_orient(const uint64_t* __restrict__ e, int64_t m,
                                                  const uint32_t* __restrict__ rank, uint64_t* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < m; i += (int64_t)gridDim.x * NT) {
    const uint64_t x = e[i];
    const uint32_t ra = rank[(uint32_t)(x >> 32)], rb = rank[(uint32_t)x];
    out[i] = ra < rb ? ((uint64_t)ra << 32 | rb) : ((uint64_t)rb << 32 | ra);
  }
}

// first index in [lo, hi) with col[idx] >= x
__device__ __forceinline__ int64_t lower_bound(const uint32_t* __restrict__ c, int64_t lo, int64_t hi, uint32_t x) {
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (c[mid] < x) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// |L(u) ∩ L(v)| for sorted rows; writes the common elements when `w` != null
template <bool EMIT>
__device__ __forceinline__ uint32_t intersect(const uint32_t* __restrict__ col, int64_t a0, int64_t a1, int64_t b0,
                                              int64_t b1, uint64_t* __restrict__ w, uint64_t u, uint64_t v) {
  uint32_t n = 0;
  int64_t la = a1 - a0, lb = b1 - b0;
  if (la == 0 || lb == 0) return 0;
  if (la > lb) {  // iterate the shorter list
    int64_t t0 = a0, t1 = a1;
    a0 = b0;
    a1 = b1;
    b0 = t0;
    b1 = t1;
    const int64_t t = la;
    la = lb;
    lb = t;
  }
  if (lb > 32 * la) {  // unbalanced: binary search each element of the short list
    int64_t p = b0;
    for (int64_t i = a0; i < a1 && p < b1; ++i) {
      const uint32_t x = col[i];
      p = lower_bound(col, p, b1, x);
      if (p < b1 && col[p] == x) {
        if (EMIT) {
          w[3 * n] = u;
          w[3 * n + 1] = v;
          w[3 * n + 2] = x;
        }
        ++n;
        ++p;
      }
    }
    return n;
  }
  int64_t i = a0, j = b0;
  uint32_t x = col[i], y = col[j];
  while (true) {
    if (x < y) {
      if (++i == a1) break;
      x = col[i];
    } else if (y < x) {
      if (++j == b1) break;
      y = col[j];
    } else {
      if (EMIT) {
        w[3 * n] = u;
        w[3 * n + 1] = v;
        w[3 * n + 2] = x;
      }
      ++n;
      if (++i == a1 || ++j == b1) break;
      x = col[i];
      y = col[j];
    }
  }
  return n;
}

__global__ __launch_bounds__(NT) void k_tri_count(const int64_t* __restrict__ rowptr, const uint32_t* __restrict__ col,
                                                 const uint64_t* __restrict__ okeys, int64_t e0, int64_t e1,
                                                 uint32_t* __restrict__ cnt, unsigned long long* __restrict__ total) {
  unsigned long long mine = 0;
  for (int64_t e = e0 + (int64_t)blockIdx.x * NT + threadIdx.x; e < e1; e += (int64_t)gridDim.x * NT) {
    const uint64_t k = okeys[e];
    const uint32_t u = (uint32_t)(k >> 32), v = (uint32_t)k;
    const uint32_t c = intersect<false>(col, rowptr[u], rowptr[u + 1], rowptr[v], rowptr[v + 1], nullptr, u, v);
    if (cnt) cnt[e - e0] = c;
    mine += c;
  }
  mine = dev::wave_sum(mine);
  if ((threadIdx.x & (MRH_WAVE - 1)) == 0 && mine) atomicAdd(total, mine);
}

__global__ __launch_bounds__(NT) void k_tri_emit(const int64_t* __restrict__ rowptr, const uint32_t* __restrict__ col,
                                                const uint64_t* __restrict__ okeys, int64_t e0, int64_t e1,
                                                const int64_t* __restrict__ off, uint64_t* __restrict__ out) {
  for (int64_t e = e0 + (int64_t)blockIdx.x * NT + threadIdx.x; e < e1; e += (int64_t)gridDim.x * NT) {
    const int64_t o = off[e - e0];
    if (off[e - e0 + 1] == o) continue;
    const uint64_t k = okeys[e];
    const uint32_t u = (uint32_t)(k >> 32), v = (uint32_t)k;
    intersect<true>(col, rowptr[u], rowptr[u + 1], rowptr[v], rowptr[v + 1], out + 3 * o, u, v);
  }
}

// ---------------------------------------------------------------- hash-based vertex-centric count
// For every vertex u, the triangles found on its out-edges (u,v) are
// |N+(u) ∩ N+(v)| summed over v ∈ N+(u). N+(u) goes into an LDS hash table
// once; then the flattened (v, w ∈ N+(v)) pairs of all v are spread evenly
// over the 64 lanes of the wave (a prefix sum of the out-degrees of 64 v's at
// a time), so the work is Σ_e d+(v) coalesced reads + LDS probes instead of a
// divergent per-edge merge of d+(u) + d+(v).
constexpr uint32_t EMPTY = 0xffffffffu;
constexpr int TW = 2048;          // per-wave table slots in the small kernel: d+(u) <= 1024
constexpr int BIG_NT = 1024;      // one block per big vertex
constexpr int BIG_TAB = 32768;    // 128 KB table: d+(u) <= 16384
constexpr int HASH_NW = NT / MRH_WAVE;

// murmur3 finaliser: R-MAT vertex ids share low-bit patterns, so the low
// bits of a plain multiplicative hash would chain badly
__device__ __forceinline__ uint32_t hslot(uint32_t x, uint32_t mask) {
  x ^= x >> 16;
  x *= 0x85EBCA6Bu;
  x ^= x >> 13;
  x *= 0xC2B2AE35u;
  x ^= x >> 16;
  return x & mask;
}

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ void tab_insert(uint32_t* tab, uint32_t mask, uint32_t x) {
  uint32_t s = hslot(x, mask);
  while (true) {
    const uint32_t old = atomicCAS(tab + s, EMPTY, x);
    if (old == EMPTY || old == x) return;
    s = (s + 1) & mask;
  }
}

__device__ __forceinline__ bool tab_has(const uint32_t* tab, uint32_t mask, uint32_t x) {
  uint32_t s = hslot(x, mask);
  while (true) {
    const uint32_t y = tab[s];
    if (y == x) return true;
    if (y == EMPTY) return false;
    s = (s + 1) & mask;
  }
}

// hub bitmaps for the probe walk (k_tri_hub_count's H; H == null: none)
struct Hubs {
  const unsigned long long* H;
  int64_t hb, W;
};

// one wave walks the v's of N+(u) in chunks of 64: returns the number of w ∈ N+(v) found in tab
// rows hold rank ids in increasing order, so only the prefix of N+(v) up to
// max N+(u) can match: cut each row there (binary search) before probing.
// A hub v (rank >= hb) has its out-neighbours in bitmap row H[v]: instead of
// walking N+(v) (long for hubs) the wave tests the elements of N+(u) after v
// (all hubs, since they rank above v) against that row — |N+(u)| - pos(v) - 1
// bit tests
__device__ __forceinline__ uint64_t probe_chunks(const int64_t* __restrict__ rowptr, const uint32_t* __restrict__ col,
                                                 int64_t c0, int64_t b, int64_t cstep, const uint32_t* tab,
                                                 uint32_t mask, uint32_t maxu, int64_t* pre, int64_t* st,
                                                 int64_t* hv, const Hubs& hubs) {
  const int l = dev::lane_id();
  uint64_t cnt = 0;
  for (int64_t c = c0; c < b; c += cstep) {
    int64_t len = 0, vs = 0, hrow = -1;
    if (c + l < b) {
      const uint32_t v = col[c + l];
      if (hubs.H && (int64_t)v >= hubs.hb) {
        hrow = ((int64_t)v - hubs.hb) * hubs.W;
        vs = c + l + 1;  // the rest of N+(u): hubs above v
        len = b - vs;
      } else {
        vs = rowptr[v];
        len = lower_bound(col, vs, rowptr[v + 1], maxu + 1u) - vs;
      }
    }
    const int64_t inc = dev::wave_incl_scan(len);
    const int64_t tot = __shfl(inc, MRH_WAVE - 1, MRH_WAVE);
    pre[l + 1] = inc;
    if (l == 0) pre[0] = 0;
    st[l] = vs;
    hv[l] = hrow;
    wave_sync();
    // lane l takes flat items l, l+64, ...: its owning v only moves forward, so
    // a short monotone walk replaces a binary search; two items per trip keep
    // two independent global loads in flight
    int j = 0;
    for (int64_t t = l; t < tot; t += 2 * MRH_WAVE) {
      while (pre[j + 1] <= t) ++j;
      const uint32_t x0 = col[st[j] + (t - pre[j])];
      const int64_t h0 = hv[j];
      const int64_t t1 = t + MRH_WAVE;
      uint32_t x1 = EMPTY;
      int64_t h1 = -1;
      if (t1 < tot) {
        while (pre[j + 1] <= t1) ++j;
        x1 = col[st[j] + (t1 - pre[j])];
        h1 = hv[j];
      }
      if (h0 >= 0) {
        const int64_t bit = (int64_t)x0 - hubs.hb;
        cnt += (hubs.H[h0 + (bit >> 6)] >> (bit & 63)) & 1ull;
      } else {
        cnt += tab_has(tab, mask, x0) ? 1u : 0u;
      }
      if (x1 != EMPTY) {
        if (h1 >= 0) {
          const int64_t bit = (int64_t)x1 - hubs.hb;
          cnt += (hubs.H[h1 + (bit >> 6)] >> (bit & 63)) & 1ull;
        } else {
          cnt += tab_has(tab, mask, x1) ? 1u : 0u;
        }
      }
    }
    wave_sync();
  }
  return cnt;
}

// wave per vertex with a per-wave LDS table of TWN slots (d+(u) <= TWN/2);
// larger vertices go to the next tier's list. Tier 1 walks the vertex range
// [u0,u1) (list == null), later tiers the list filled by the previous one.
// Small tables keep LDS per block low, so tier 1 (nearly every vertex) runs
// at high occupancy to hide the dependent global loads.
template <int TWN>
__global__ __launch_bounds__(NT) void k_tri_hash_wave(const int64_t* __restrict__ rowptr,
                                                     const uint32_t* __restrict__ col, int64_t u0, int64_t u1,
                                                     const uint32_t* __restrict__ list,
                                                     const uint32_t* __restrict__ nlist,
                                                     uint32_t* __restrict__ next, uint32_t* __restrict__ nnext,
                                                     unsigned long long* __restrict__ total, Hubs hubs) {
  __shared__ uint32_t tab[HASH_NW][TWN];
  __shared__ int64_t pre[HASH_NW][MRH_WAVE + 1];
  __shared__ int64_t st[HASH_NW][MRH_WAVE];
  __shared__ int64_t hv[HASH_NW][MRH_WAVE];
  const int w = dev::wave_id(), l = dev::lane_id();
  uint64_t cnt = 0;
  const int64_t nw = (int64_t)gridDim.x * HASH_NW;
  const int64_t nitems = list ? (int64_t)*nlist : u1 - u0;
  for (int64_t it = (int64_t)blockIdx.x * HASH_NW + w; it < nitems; it += nw) {
    const int64_t u = list ? (int64_t)list[it] : u0 + it;
    const int64_t a = rowptr[u], b = rowptr[u + 1], d = b - a;
    if (d < 2) continue;
    if (d > TWN / 2) {
      if (l == 0) next[atomicAdd(nnext, 1u)] = (uint32_t)u;
      continue;
    }
    uint32_t size = 64;
    while (size < 2 * d) size <<= 1;
    const uint32_t mask = size - 1;
    for (uint32_t i = l; i < size; i += MRH_WAVE) tab[w][i] = EMPTY;
    wave_sync();
    for (int64_t i = a + l; i < b; i += MRH_WAVE) tab_insert(tab[w], mask, col[i]);
    wave_sync();
    cnt += probe_chunks(rowptr, col, a, b, MRH_WAVE, tab[w], mask, col[b - 1], pre[w], st[w], hv[w], hubs);
  }
  cnt = dev::wave_sum(cnt);
  if (l == 0 && cnt) atomicAdd(total, (unsigned long long)cnt);
}

// one block per big vertex (d+(u) > 1024); beyond the LDS table a per-edge merge
__global__ __launch_bounds__(BIG_NT) void k_tri_hash_big(const int64_t* __restrict__ rowptr,
                                                        const uint32_t* __restrict__ col,
                                                        const uint32_t* __restrict__ big,
                                                        const uint32_t* __restrict__ nbig,
                                                        unsigned long long* __restrict__ total, Hubs hubs) {
  __shared__ uint32_t tab[BIG_TAB];
  __shared__ int64_t pre[BIG_NT / MRH_WAVE][MRH_WAVE + 1];
  __shared__ int64_t st[BIG_NT / MRH_WAVE][MRH_WAVE];
  __shared__ int64_t hv[BIG_NT / MRH_WAVE][MRH_WAVE];
  const int w = dev::wave_id(), l = dev::lane_id();
  const uint32_t n = *nbig;
  uint64_t cnt = 0;
  for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) {
    const uint32_t u = big[i];
    const int64_t a = rowptr[u], b = rowptr[u + 1], d = b - a;
    if (2 * d > BIG_TAB) {
      for (int64_t e = a + threadIdx.x; e < b; e += BIG_NT) {
        const uint32_t v = col[e];
        cnt += intersect<false>(col, a, b, rowptr[v], rowptr[v + 1], nullptr, u, v);
      }
      continue;
    }
    uint32_t size = 64;
    while (size < 2 * d) size <<= 1;
    const uint32_t mask = size - 1;
    for (uint32_t j = threadIdx.x; j < size; j += BIG_NT) tab[j] = EMPTY;
    __syncthreads();
    for (int64_t j = a + threadIdx.x; j < b; j += BIG_NT) tab_insert(tab, mask, col[j]);
    __syncthreads();
    cnt += probe_chunks(rowptr, col, a + (int64_t)w * MRH_WAVE, b, (int64_t)BIG_NT, tab, mask, col[b - 1], pre[w],
                        st[w], hv[w], hubs);
    __syncthreads();
  }
  cnt = dev::wave_sum(cnt);
  if (l == 0 && cnt) atomicAdd(total, (unsigned long long)cnt);
}

// ---------------------------------------------------------------- hub bitmaps
// The K highest-ranked vertices ("hubs", ranks [hb, nvert) with hb = nvert-K)
// only have out-neighbours among themselves (edges point to higher ranks),
// so every triangle whose lowest vertex is a hub lies inside the hub
// subgraph. Its oriented adjacency is a dense K x K bit matrix H (row u:
// bit w-hb set for w in N+(u)); the triangles found on edge (u, v) are then
// popcount(H[u] & H[v]) — 64 candidate vertices per AND instead of one hash
// probe per element of N+(v). The hash kernels keep the vertices below hb.
// (A dense int8 MFMA product H.H^T would do K^3 multiply-adds regardless of
// the ~1 % density of the hub subgraph: 100x the AND/popcount work.)
__global__ __launch_bounds__(NT) void k_tri_hub_build(const int64_t* __restrict__ rowptr,
                                                     const uint32_t* __restrict__ col, int64_t hb, int64_t K,
                                                     unsigned long long* __restrict__ H) {
  const int64_t W = K / 64;
  const int64_t nw = (int64_t)gridDim.x * HASH_NW;
  for (int64_t r = (int64_t)blockIdx.x * HASH_NW + dev::wave_id(); r < K; r += nw) {
    const int64_t u = hb + r;
    for (int64_t e = rowptr[u] + dev::lane_id(); e < rowptr[u + 1]; e += MRH_WAVE) {
      const int64_t b = (int64_t)col[e] - hb;  // >= 1: N+(u) holds higher ranks only
      atomicOr(&H[r * W + (b >> 6)], 1ull << (b & 63));
    }
  }
}

// dense core: the top T ranks as a 0/1 int8 matrix (row u - cb: 1 at w - cb
// for w in N+(u)); the triangles whose lowest vertex is in the core are then
// sum(A .* (A A^T)), an int8 matrix-core GEMM instead of AND/popcount walks
__global__ __launch_bounds__(NT) void k_tri_core_build(const int64_t* __restrict__ rowptr,
                                                      const uint32_t* __restrict__ col, int64_t cb, int64_t T,
                                                      int8_t* __restrict__ A) {
  const int64_t nw = (int64_t)gridDim.x * HASH_NW;
  for (int64_t r = (int64_t)blockIdx.x * HASH_NW + dev::wave_id(); r < T; r += nw) {
    const int64_t u = cb + r;
    for (int64_t e = rowptr[u] + dev::lane_id(); e < rowptr[u + 1]; e += MRH_WAVE)
      A[r * T + ((int64_t)col[e] - cb)] = 1;  // N+(u) holds higher ranks only: inside the core
  }
}

// one workgroup per hub u in [r0, r1) (rows relative to hb); each thread
// keeps HUB_WPT words of H[u] in registers and ANDs them with the same words
// of H[v] for every v in N+(u) (coalesced row reads, words below v skipped)
constexpr int HUB_NT = 256;
constexpr int HUB_LIST = 2048;   // LDS list of a sparse hub row's non-zero words (24 KB)
constexpr int HUB_SPARSE = 8;    // sparse when fewer than W / 8 words are non-zero
template <int WPT>
__global__ __launch_bounds__(HUB_NT) void k_tri_hub_count(const int64_t* __restrict__ rowptr,
                                                         const uint32_t* __restrict__ col, int64_t hb, int64_t K,
                                                         int64_t r0, int64_t r1,
                                                         const unsigned long long* __restrict__ H,
                                                         unsigned long long* __restrict__ total) {
  constexpr int NWV = HUB_NT / MRH_WAVE;
  __shared__ int s_scan[HUB_NT / MRH_WAVE + 1];
  __shared__ int32_t s_idx[HUB_LIST];
  __shared__ unsigned long long s_val[HUB_LIST];
  __shared__ int s_jw[WPT * NWV + 1];          // non-zero words per (register j, wave), then their offsets
  __shared__ int s_vr[HUB_NT], s_lb[HUB_NT], s_off[HUB_NT + 1];
  const int64_t W = K / 64;
  const int wv = dev::wave_id(), ln = dev::lane_id();
  const uint64_t lt = dev::lanemask_lt();
  uint64_t cnt = 0;
  for (int64_t r = r0 + blockIdx.x; r < r1; r += gridDim.x) {
    const int64_t u = hb + r;
    const int64_t a = rowptr[u], b = rowptr[u + 1];
    if (b - a < 2) continue;  // uniform over the block: no barrier is skipped unevenly
    const unsigned long long* hu = H + r * W;
    unsigned long long mine[WPT];
#pragma unroll
    for (int j = 0; j < WPT; ++j) {
      const int64_t w = threadIdx.x + (int64_t)j * HUB_NT;
      mine[j] = w < W ? hu[w] : 0ull;
    }
    // the row's non-zero words in ascending word order (word = j * HUB_NT +
    // thread, i.e. (j, wave, lane) order): per-(j, wave) ballot counts, one
    // scan over them, then every thread places its words
#pragma unroll
    for (int j = 0; j < WPT; ++j) {
      const uint64_t bm = __ballot(mine[j] != 0ull);
      if (ln == 0) s_jw[j * NWV + wv] = __popcll(bm);
    }
    __syncthreads();
    if (threadIdx.x < MRH_WAVE) {  // exclusive scan of the WPT * NWV (<= 128) counts, two per lane
      const int i0 = 2 * ln, i1 = 2 * ln + 1;
      const int x0 = i0 < WPT * NWV ? s_jw[i0] : 0, x1 = i1 < WPT * NWV ? s_jw[i1] : 0;
      const int incl = dev::wave_incl_scan(x0 + x1);
      if (i0 < WPT * NWV) s_jw[i0] = incl - x0 - x1;
      if (i1 < WPT * NWV) s_jw[i1] = incl - x1;
      if (ln == MRH_WAVE - 1) s_jw[WPT * NWV] = incl;
    }
    __syncthreads();
    const int total_nz = s_jw[WPT * NWV];
    // sparse rows (the lower hubs: few of W words set) AND only their
    // non-zero words against each H[v]: d+(u) x nnz word loads instead of
    // d+(u) x W, and only the words at or above v's own column (H[v] has no
    // bits below it): with the words sorted, each edge's valid words are a
    // suffix [lb, nz), and the (edge, word) pairs of 256 edges at a time are
    // flattened over the block — every lane loads a word that can match
    if ((int64_t)total_nz * HUB_SPARSE < W && total_nz <= HUB_LIST) {
#pragma unroll
      for (int j = 0; j < WPT; ++j) {
        const uint64_t bm = __ballot(mine[j] != 0ull);
        if (mine[j]) {
          const int o = s_jw[j * NWV + wv] + __popcll(bm & lt);
          s_idx[o] = (int32_t)(threadIdx.x + j * HUB_NT);
          s_val[o] = mine[j];
        }
      }
      __syncthreads();
      const int nz = total_nz;
      for (int64_t eb = a; eb < b; eb += HUB_NT) {
        const int64_t e = eb + threadIdx.x;
        int c = 0, vr = 0, lb = 0;
        if (e < b) {
          vr = (int)((int64_t)col[e] - hb);
          const int w0 = vr >> 6;
          int lo = 0, hi = nz;
          while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (s_idx[mid] < w0) lo = mid + 1;
            else hi = mid;
          }
          lb = lo;
          c = nz - lo;
        }
        int tot;
        const int off = dev::block_excl_scan<int, HUB_NT>(c, s_scan, &tot);
        s_vr[threadIdx.x] = vr;
        s_lb[threadIdx.x] = lb;
        s_off[threadIdx.x] = off;
        if (threadIdx.x == 0) s_off[HUB_NT] = tot;
        __syncthreads();
        // pair p = (edge j, word s_lb[j] + p - s_off[j]); a thread's pairs
        // are HUB_NT apart, so its edge index only moves forward; four pairs
        // per trip keep four independent loads of H in flight
        int j = 0;
        for (int p = threadIdx.x; p < tot; p += 4 * HUB_NT) {
          int64_t addr[4];
          unsigned long long mv[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int q = p + k * HUB_NT;
            addr[k] = -1;
            mv[k] = 0ull;
            if (q < tot) {
              while (s_off[j + 1] <= q) ++j;
              const int li = s_lb[j] + (q - s_off[j]);
              addr[k] = (int64_t)s_vr[j] * W + s_idx[li];
              mv[k] = s_val[li];
            }
          }
          unsigned long long hv[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) hv[k] = addr[k] >= 0 ? H[addr[k]] : 0ull;
#pragma unroll
          for (int k = 0; k < 4; ++k) cnt += __popcll(mv[k] & hv[k]);
        }
        __syncthreads();
      }
      continue;
    }
    for (int64_t e = a; e < b; ++e) {
      const int64_t vr = (int64_t)col[e] - hb;
      const unsigned long long* hv = H + vr * W;
      const int64_t w0 = vr >> 6;  // H[v] has no bits at or below column vr
#pragma unroll
      for (int j = 0; j < WPT; ++j) {
        const int64_t w = threadIdx.x + (int64_t)j * HUB_NT;
        if (w >= w0 && w < W && mine[j]) cnt += __popcll(mine[j] & hv[w]);
      }
    }
  }
  cnt = dev::wave_sum(cnt);
  if (dev::lane_id() == 0 && cnt) atomicAdd(total, (unsigned long long)cnt);
}

// LDS-bitmap hub kernel: one workgroup per hub u at a time; N+(u) (hub
// ranks, relative to hb) is set as bits of a K-bit bitmap in LDS (64 KiB at
// K = 524288), then every wave takes a v of N+(u) and its 64 lanes stream
// N+(v) from the CSR column array — coalesced 4-byte reads — testing each w
// against the LDS bitmap: |N+(u) ∩ N+(v)| costs d+(v) coalesced loads and LDS
// bit tests instead of nnz(H[u]) scattered 8-byte loads of H[v] (the bitmap
// kernel above, whose sparse lower-hub rows made it 67 % of tri_find). The
// bits of N+(u) are cleared again behind the count (O(d+(u)), not O(K)).
constexpr int HUBL_NT = 256;
constexpr int HUBL_WORDS = 8192;  // K <= 524288
__global__ __launch_bounds__(HUBL_NT) void k_tri_hub_lds(const int64_t* __restrict__ rowptr,
                                                        const uint32_t* __restrict__ col, int64_t hb, int64_t r0,
                                                        int64_t r1, unsigned long long* __restrict__ total) {
  __shared__ unsigned long long bm[HUBL_WORDS];
  for (int i = threadIdx.x; i < HUBL_WORDS; i += HUBL_NT) bm[i] = 0ull;
  __syncthreads();
  const int lane = dev::lane_id(), wv = dev::wave_id();
  constexpr int NWV = HUBL_NT / MRH_WAVE;
  uint64_t cnt = 0;
  for (int64_t r = r0 + blockIdx.x; r < r1; r += gridDim.x) {
    const int64_t u = hb + r;
    const int64_t a = rowptr[u], b = rowptr[u + 1];
    if (b - a < 2) continue;  // uniform over the block
    for (int64_t e = a + threadIdx.x; e < b; e += HUBL_NT) {
      const uint32_t c = (uint32_t)((int64_t)col[e] - hb);
      atomicOr(&bm[c >> 6], 1ull << (c & 63));
    }
    __syncthreads();
    // each wave takes 64 v's of N+(u) at a time and flattens their N+(v)
    // lists (wave prefix sum of d+(v)): lane l tests element s*64 + l of the
    // concatenation, so all 64 lanes work whatever the d+(v) mix
    for (int64_t i0 = a + (int64_t)wv * MRH_WAVE; i0 < b; i0 += (int64_t)NWV * MRH_WAVE) {
      const int64_t i = i0 + lane;
      int64_t s0 = 0;
      int dv = 0;
      if (i < b) {
        const int64_t v = col[i];
        s0 = rowptr[v];
        dv = (int)(rowptr[v + 1] - s0);
      }
      int incl = dv;
#pragma unroll
      for (int o = 1; o < MRH_WAVE; o <<= 1) {
        const int y = __shfl_up(incl, o, MRH_WAVE);
        if (lane >= o) incl += y;
      }
      const int tot = __shfl(incl, MRH_WAVE - 1, MRH_WAVE);
      for (int k0 = 0; k0 < tot; k0 += MRH_WAVE) {
        const int k = k0 + lane;
        // owner lane j of element k: the first lane whose inclusive sum > k
        int lo = 0, hi = MRH_WAVE - 1;
#pragma unroll
        for (int st = 0; st < 6; ++st) {
          const int mid = (lo + hi) >> 1;
          const int im = __shfl(incl, mid, MRH_WAVE);
          if (im > k) hi = mid;
          else lo = mid + 1;
        }
        const int j = lo;
        const int ex = __shfl(incl - dv, j, MRH_WAVE);
        const int64_t sj = __shfl(s0, j, MRH_WAVE);
        if (k < tot) {
          const uint32_t w = (uint32_t)((int64_t)col[sj + (k - ex)] - hb);
          cnt += (bm[w >> 6] >> (w & 63)) & 1ull;
        }
      }
    }
    __syncthreads();
    for (int64_t e = a + threadIdx.x; e < b; e += HUBL_NT) {
      const uint32_t c = (uint32_t)((int64_t)col[e] - hb);
      bm[c >> 6] = 0ull;
    }
    __syncthreads();
  }
  cnt = dev::wave_sum(cnt);
  if (lane == 0 && cnt) atomicAdd(total, (unsigned long long)cnt);
}

// ---------------------------------------------------------------- hub rows, v-major ("pull")
// The hub rows counted grouped by the MIDDLE vertex v instead of the low
// vertex u: every hub edge (u, v) contributes |N+(u) ∩ N+(v)|, and the
// candidates w are the elements of N+(u) after v (rows are sorted). Grouped by
// v, one wave (or block) holds N+(v) in an LDS hash table and streams, for
// every in-edge (u, v), the tail of u's row past v — coalesced 4-byte reads of
// the CSR column array, each tested in LDS — so the bitmap kernel's d+(u) x
// nnz(H[u]) scattered 8-byte loads of other hubs' bitmap rows (3.9 G L2
// misses on RMAT-24, profiles/r3_trifind_pmc.txt) become streaming reads plus
// LDS probes. The in-edges of v are the hub edges sorted by destination
// (keys-only radix sort of (v - hb) << 32 | edge index); a hub with many
// in-edges is cut into pieces of PULL_PIECE in-edges (each piece rebuilds the
// small table of N+(v)), so the top hubs do not serialise on one wave.
constexpr int64_t PULL_PIECE = 2048;

__global__ __launch_bounds__(NT) void k_tri_tpack(const uint32_t* __restrict__ col, int64_t ea, int64_t n, int64_t hb,
                                                 uint64_t* __restrict__ tk) {
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT)
    tk[i] = ((uint64_t)((int64_t)col[ea + i] - hb) << 32) | (uint64_t)i;
}

// endx[i] = end of the row of edge ea + i's source, relative to ea
__global__ __launch_bounds__(NT) void k_tri_hub_end(const uint64_t* __restrict__ okeys,
                                                   const int64_t* __restrict__ rowptr, int64_t ea, int64_t n,
                                                   uint32_t* __restrict__ endx) {
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT)
    endx[i] = (uint32_t)(rowptr[(int64_t)(okeys[ea + i] >> 32) + 1] - ea);
}

// pieces per hub v: ceil(in-edges / PULL_PIECE), none when N+(v) is empty
__global__ __launch_bounds__(NT) void k_tri_pull_npieces(const int64_t* __restrict__ tptr,
                                                        const int64_t* __restrict__ rowptr, int64_t hb, int64_t K,
                                                        int64_t* __restrict__ np) {
  for (int64_t r = (int64_t)blockIdx.x * NT + threadIdx.x; r < K; r += (int64_t)gridDim.x * NT) {
    const int64_t din = tptr[r + 1] - tptr[r], dout = rowptr[hb + r + 1] - rowptr[hb + r];
    np[r] = (din > 0 && dout > 0) ? (din + PULL_PIECE - 1) / PULL_PIECE : 0;
  }
}

// work items (r << 32 | piece) at the exclusive-scan offsets off
__global__ __launch_bounds__(NT) void k_tri_pull_items(const int64_t* __restrict__ off, int64_t K,
                                                      uint64_t* __restrict__ items) {
  for (int64_t r = (int64_t)blockIdx.x * NT + threadIdx.x; r < K; r += (int64_t)gridDim.x * NT)
    for (int64_t p = off[r]; p < off[r + 1]; ++p) items[p] = ((uint64_t)r << 32) | (uint64_t)(p - off[r]);
}

struct TabTest {
  const uint32_t* tab;
  uint32_t mask;
  __device__ __forceinline__ bool operator()(uint32_t x) const { return tab_has(tab, mask, x); }
};
// N+(v) too long for an LDS table: its bitmap row in H
struct RowTest {
  const unsigned long long* row;
  int64_t hb;
  __device__ __forceinline__ bool operator()(uint32_t x) const {
    const int64_t b = (int64_t)x - hb;
    return (row[b >> 6] >> (b & 63)) & 1ull;
  }
};

// one wave streams the row tails of in-edge items [c0, p1) (step cstep, 64 at
// a time): item x = edge ea + x = (u, v), tail = col[ea + x + 1, ea + endx[x])
// cut at max N+(v); every element is tested against N+(v)
template <class Test>
__device__ __forceinline__ uint64_t pull_chunks(const uint32_t* __restrict__ col, int64_t ea,
                                                const uint64_t* __restrict__ tks, const uint32_t* __restrict__ endx,
                                                int64_t c0, int64_t p1, int64_t cstep, const Test& test, uint32_t maxv,
                                                int64_t* pre, int64_t* st) {
  const int l = dev::lane_id();
  uint64_t cnt = 0;
  for (int64_t c = c0; c < p1; c += cstep) {
    int64_t len = 0, vs = 0;
    if (c + l < p1) {
      const uint32_t x = (uint32_t)tks[c + l];
      vs = ea + (int64_t)x + 1;
      len = lower_bound(col, vs, ea + (int64_t)endx[x], maxv + 1u) - vs;
    }
    const int64_t inc = dev::wave_incl_scan(len);
    const int64_t tot = __shfl(inc, MRH_WAVE - 1, MRH_WAVE);
    pre[l + 1] = inc;
    if (l == 0) pre[0] = 0;
    st[l] = vs;
    wave_sync();
    int j = 0;
    for (int64_t t = l; t < tot; t += 2 * MRH_WAVE) {
      while (pre[j + 1] <= t) ++j;
      const uint32_t x0 = col[st[j] + (t - pre[j])];
      const int64_t t1 = t + MRH_WAVE;
      uint32_t x1 = 0;
      const bool has1 = t1 < tot;
      if (has1) {
        while (pre[j + 1] <= t1) ++j;
        x1 = col[st[j] + (t1 - pre[j])];
      }
      cnt += test(x0) ? 1u : 0u;
      if (has1) cnt += test(x1) ? 1u : 0u;
    }
    wave_sync();
  }
  return cnt;
}

template <int TWN>
__global__ __launch_bounds__(NT) void k_tri_hub_pull(const int64_t* __restrict__ rowptr,
                                                    const uint32_t* __restrict__ col, int64_t hb, int64_t ea,
                                                    const uint64_t* __restrict__ tks, const int64_t* __restrict__ tptr,
                                                    const uint32_t* __restrict__ endx,
                                                    const uint64_t* __restrict__ items,
                                                    const int64_t* __restrict__ nitems, uint64_t* __restrict__ big,
                                                    unsigned int* __restrict__ nbig,
                                                    unsigned long long* __restrict__ total) {
  __shared__ uint32_t tab[HASH_NW][TWN];
  __shared__ int64_t pre[HASH_NW][MRH_WAVE + 1];
  __shared__ int64_t st[HASH_NW][MRH_WAVE];
  const int w = dev::wave_id(), l = dev::lane_id();
  uint64_t cnt = 0;
  const int64_t nw = (int64_t)gridDim.x * HASH_NW, ni = *nitems;
  for (int64_t it = (int64_t)blockIdx.x * HASH_NW + w; it < ni; it += nw) {
    const uint64_t item = items[it];
    const int64_t r = (int64_t)(item >> 32), piece = (int64_t)(uint32_t)item;
    const int64_t a = rowptr[hb + r], b = rowptr[hb + r + 1], d = b - a;
    if (d > TWN / 2) {
      if (l == 0) big[atomicAdd(nbig, 1u)] = item;
      continue;
    }
    uint32_t size = 64;
    while (size < 2 * d) size <<= 1;
    const uint32_t mask = size - 1;
    for (uint32_t i = l; i < size; i += MRH_WAVE) tab[w][i] = EMPTY;
    wave_sync();
    for (int64_t i = a + l; i < b; i += MRH_WAVE) tab_insert(tab[w], mask, col[i]);
    wave_sync();
    const int64_t p0 = tptr[r] + piece * PULL_PIECE, p1 = tptr[r + 1] < p0 + PULL_PIECE ? tptr[r + 1] : p0 + PULL_PIECE;
    cnt += pull_chunks(col, ea, tks, endx, p0, p1, MRH_WAVE, TabTest{tab[w], mask}, col[b - 1], pre[w], st[w]);
  }
  cnt = dev::wave_sum(cnt);
  if (l == 0 && cnt) atomicAdd(total, (unsigned long long)cnt);
}

// one block per big item (N+(v) beyond the wave table): a 32768-slot LDS
// table, or v's bitmap row in H when N+(v) is longer still
__global__ __launch_bounds__(BIG_NT) void k_tri_hub_pull_big(const int64_t* __restrict__ rowptr,
                                                            const uint32_t* __restrict__ col, int64_t hb, int64_t ea,
                                                            const uint64_t* __restrict__ tks,
                                                            const int64_t* __restrict__ tptr,
                                                            const uint32_t* __restrict__ endx,
                                                            const uint64_t* __restrict__ big,
                                                            const unsigned int* __restrict__ nbig,
                                                            const unsigned long long* __restrict__ H, int64_t W,
                                                            unsigned long long* __restrict__ total) {
  __shared__ uint32_t tab[BIG_TAB];
  __shared__ int64_t pre[BIG_NT / MRH_WAVE][MRH_WAVE + 1];
  __shared__ int64_t st[BIG_NT / MRH_WAVE][MRH_WAVE];
  const int w = dev::wave_id(), l = dev::lane_id();
  const unsigned int n = *nbig;
  uint64_t cnt = 0;
  for (unsigned int i = blockIdx.x; i < n; i += gridDim.x) {
    const uint64_t item = big[i];
    const int64_t r = (int64_t)(item >> 32), piece = (int64_t)(uint32_t)item;
    const int64_t a = rowptr[hb + r], b = rowptr[hb + r + 1], d = b - a;
    const int64_t p0 = tptr[r] + piece * PULL_PIECE, p1 = tptr[r + 1] < p0 + PULL_PIECE ? tptr[r + 1] : p0 + PULL_PIECE;
    const int64_t c0 = p0 + (int64_t)w * MRH_WAVE;
    if (2 * d > BIG_TAB) {  // uniform over the block
      cnt += pull_chunks(col, ea, tks, endx, c0, p1, (int64_t)BIG_NT, RowTest{H + r * W, hb}, col[b - 1], pre[w], st[w]);
      __syncthreads();
      continue;
    }
    uint32_t size = 64;
    while (size < 2 * d) size <<= 1;
    const uint32_t mask = size - 1;
    for (uint32_t j = threadIdx.x; j < size; j += BIG_NT) tab[j] = EMPTY;
    __syncthreads();
    for (int64_t j = a + threadIdx.x; j < b; j += BIG_NT) tab_insert(tab, mask, col[j]);
    __syncthreads();
    cnt += pull_chunks(col, ea, tks, endx, c0, p1, (int64_t)BIG_NT, TabTest{tab, mask}, col[b - 1], pre[w], st[w]);
    __syncthreads();
  }
  cnt = dev::wave_sum(cnt);
  if (l == 0 && cnt) atomicAdd(total, (unsigned long long)cnt);
}

// rowptr[v] = first index of src v in the sorted oriented keys (rowptr[nvert] = m)
// one thread per vertex: binary search (the top ranks have no out-edges, so a
// per-edge gap fill would leave one thread walking millions of vertices)
__global__ __launch_bounds__(NT) void k_rowptr(const uint64_t* __restrict__ okeys, int64_t m, int64_t nvert,
                                              int64_t* __restrict__ rowptr) {
  for (int64_t v = (int64_t)blockIdx.x * NT + threadIdx.x; v <= nvert; v += (int64_t)gridDim.x * NT) {
    const uint64_t key = (uint64_t)v << 32;
    int64_t lo = 0, hi = m;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (okeys[mid] < key) lo = mid + 1;
      else hi = mid;
    }
    rowptr[v] = lo;
  }
}

unsigned grid_for(int64_t n) {
  int64_t b = (n + NT - 1) / NT;
  return (unsigned)(b < 1 ? 1 : (b > 65536 ? 65536 : b));
}

}  // namespace

void tri_degree(const uint64_t* e, int64_t m, uint32_t* deg, hipStream_t s) {
  if (m <= 0) return;
  hipLaunchKernelGGL(k_tri_degree, dim3(grid_for(m)), dim3(NT), 0, s, e, m, deg);
  MRH_CHECK_LAUNCH();
}

__global__ __launch_bounds__(NT) void k_count_low(const uint64_t* __restrict__ e, int64_t m, uint32_t* __restrict__ deg) {
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < m; i += (int64_t)gridDim.x * NT)
    atomicAdd(deg + (uint32_t)e[i], 1u);
}
void count_low_atomic(const uint64_t* e, int64_t m, uint32_t* deg, hipStream_t s) {
  if (m <= 0) return;
  hipLaunchKernelGGL(k_count_low, dim3(grid_for(m)), dim3(NT), 0, s, e, m, deg);
  MRH_CHECK_LAUNCH();
}

int tri_deg_buckets(int64_t nvert) {
  const int64_t nb = (nvert + DEG_BINS - 1) >> DEG_RB;
  return nb <= DEG_MAXB ? (int)nb : -1;
}
int tri_deg_bucket_bits() { return DEG_RB; }
unsigned tri_deg_grid(int64_t m) { return (unsigned)std::min<int64_t>(std::max<int64_t>((m + NT * 64 - 1) / (NT * 64), 1), 4096); }

void tri_deg_lo(const uint64_t* e, int64_t m, uint32_t* deg, hipStream_t s) {
  if (m <= 0) return;
  hipLaunchKernelGGL(k_deg_lo, dim3(grid_for(m)), dim3(NT), 0, s, e, m, deg);
  MRH_CHECK_LAUNCH();
}

void tri_deg_count(const uint64_t* e, int64_t m, int nb, unsigned int* bcount, hipStream_t s) {
  if (m <= 0) return;
  check_arg(nb >= 1 && nb <= DEG_MAXB, "tri_deg_count: bucket count out of range");
  if (nb <= DEG_SMALLB)
    hipLaunchKernelGGL(k_deg_count<DEG_SMALLB>, dim3(tri_deg_grid(m)), dim3(NT), 0, s, e, m, nb, bcount);
  else
    hipLaunchKernelGGL(k_deg_count<DEG_MAXB>, dim3(tri_deg_grid(m)), dim3(NT), 0, s, e, m, nb, bcount);
  MRH_CHECK_LAUNCH();
}

void tri_deg_scatter(const uint64_t* e, int64_t m, int nb, unsigned long long* cursor, uint16_t* out, hipStream_t s) {
  if (m <= 0) return;
  check_arg(nb >= 1 && nb <= DEG_MAXB, "tri_deg_scatter: bucket count out of range");
  if (nb <= DEG_SMALLB)
    hipLaunchKernelGGL(k_deg_scatter<DEG_SMALLB>, dim3(tri_deg_grid(m)), dim3(NT), 0, s, e, m, nb, cursor, out);
  else
    hipLaunchKernelGGL(k_deg_scatter<DEG_MAXB>, dim3(tri_deg_grid(m)), dim3(NT), 0, s, e, m, nb, cursor, out);
  MRH_CHECK_LAUNCH();
}

void tri_deg_hist(const uint16_t* ids, const unsigned long long* bstart, const uint64_t* items, const uint32_t* ilen,
                  const uint8_t* whole, int64_t nitems, int64_t nvert, uint32_t* deg, hipStream_t s) {
  if (nitems <= 0) return;
  hipLaunchKernelGGL(k_deg_hist, dim3((unsigned)std::min<int64_t>(nitems, 2048)), dim3(DEG_NT), 0, s, ids, bstart,
                     items, ilen, whole, nitems, nvert, deg);
  MRH_CHECK_LAUNCH();
}

void tri_pack(const int64_t* e, int64_t n, int64_t nvert, uint64_t* out, unsigned int* bad, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_tri_pack, dim3(grid_for(n)), dim3(NT), 0, s, e, n, nvert, out, bad);
  MRH_CHECK_LAUNCH();
}
void tri_col(const uint64_t* okeys, int64_t m, uint32_t* col, hipStream_t s) {
  if (m <= 0) return;
  hipLaunchKernelGGL(k_tri_col, dim3(grid_for(m)), dim3(NT), 0, s, okeys, m, col);
  MRH_CHECK_LAUNCH();
}
void tri_rank(const int32_t* perm, int64_t n, int32_t* rank, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_tri_rank, dim3(grid_for(n)), dim3(NT), 0, s, perm, n, rank);
  MRH_CHECK_LAUNCH();
}

void tri_orient(const uint64_t* e, int64_t m, const uint32_t* rank, uint64_t* out, hipStream_t s) {
  if (m <= 0) return;
  hipLaunchKernelGGL(k_tri_orient, dim3(grid_for(m)), dim3(NT), 0, s, e, m, rank, out);
  MRH_CHECK_LAUNCH();
}

void tri_count(const int64_t* rowptr, const uint32_t* col, const uint64_t* okeys, int64_t e0, int64_t e1,
               uint32_t* cnt, unsigned long long* total, hipStream_t s) {
  if (e1 <= e0) return;
  hipLaunchKernelGGL(k_tri_count, dim3(grid_for(e1 - e0)), dim3(NT), 0, s, rowptr, col, okeys, e0, e1, cnt, total);
  MRH_CHECK_LAUNCH();
}

void tri_count_hash(const int64_t* rowptr, const uint32_t* col, int64_t u0, int64_t u1, uint32_t* big,
                    uint32_t* nbig, unsigned long long* total, hipStream_t s, const uint64_t* H, int64_t hb,
                    int64_t K) {
  const Hubs hubs{(const unsigned long long*)H, hb, K / 64};
  if (u1 <= u0) return;
  // scratch: big = [mid list | big list] each u1-u0 entries; nbig = [nmid, nbig]
  const int64_t nv = u1 - u0;
  uint32_t* mid = big;
  uint32_t* bigl = big + nv;
  int64_t blocks = (nv + HASH_NW - 1) / HASH_NW;
  if (blocks > 16384) blocks = 16384;  // waves grid-stride over the vertices
  hipLaunchKernelGGL(k_tri_hash_wave<256>, dim3((unsigned)blocks), dim3(NT), 0, s, rowptr, col, u0, u1,
                     (const uint32_t*)nullptr, (const uint32_t*)nullptr, mid, nbig, total, hubs);
  MRH_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_tri_hash_wave<TW>, dim3(2048), dim3(NT), 0, s, rowptr, col, u0, u1, (const uint32_t*)mid,
                     (const uint32_t*)nbig, bigl, nbig + 1, total, hubs);
  MRH_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_tri_hash_big, dim3(512), dim3(BIG_NT), 0, s, rowptr, col, bigl, nbig + 1, total, hubs);
  MRH_CHECK_LAUNCH();
}

void tri_hub_count(const int64_t* rowptr, const uint32_t* col, int64_t hb, int64_t K, int64_t u0, int64_t u1,
                   uint64_t* H, unsigned long long* total, hipStream_t s) {
  check_arg(K > 0 && K % 64 == 0 && K <= HUB_NT * 64 * 32, "tri_hub_count: K must be a multiple of 64, <= 524288");
  const int64_t r0 = std::max<int64_t>(u0 - hb, 0), r1 = std::min<int64_t>(u1 - hb, K);
  // the bitmaps are always built: the hash kernels' hub probes read them too
  MRH_HIP(hipMemsetAsync(H, 0, (size_t)K * (K / 64) * 8, s));
  hipLaunchKernelGGL(k_tri_hub_build, dim3((unsigned)std::min<int64_t>((K + HASH_NW - 1) / HASH_NW, 16384)), dim3(NT),
                     0, s, rowptr, col, hb, K, (unsigned long long*)H);
  MRH_CHECK_LAUNCH();
  if (r1 <= r0) return;
  const int64_t W = K / 64;
  const unsigned long long* Hc = (const unsigned long long*)H;
  // MRH_TRI_HUB_KERNEL=lds selects the LDS-bitmap kernel: on RMAT-24 it ran
  // 1081 ms per tri_find against 350 with the global bitmap rows
  // (profiles/r3_trifind_hub_kernels.txt), so the bitmap kernel is the default
  static const int hub_kernel = [] {
    const char* e = std::getenv("MRH_TRI_HUB_KERNEL");
    return (e && std::string(e) == "lds") ? 1 : 0;
  }();
  if (hub_kernel == 1 && W <= HUBL_WORDS) {
    const unsigned g = (unsigned)std::min<int64_t>(r1 - r0, 4096);
    hipLaunchKernelGGL(k_tri_hub_lds, dim3(g), dim3(HUBL_NT), 0, s, rowptr, col, hb, r0, r1, total);
    MRH_CHECK_LAUNCH();
    return;
  }
  // MRH_TRI_HUB_CHUNKS=n: n dispatches over equal row ranges (a per-range
  // kernel trace of the hub work; one dispatch by default)
  static const int chunks = [] {
    const char* e = std::getenv("MRH_TRI_HUB_CHUNKS");
    return e ? std::max(1, std::min(64, std::atoi(e))) : 1;
  }();
  for (int c = 0; c < chunks; ++c) {
    const int64_t c0 = r0 + (r1 - r0) * c / chunks, c1 = r0 + (r1 - r0) * (c + 1) / chunks;
    if (c1 <= c0) continue;
    const unsigned grid = (unsigned)std::min<int64_t>(c1 - c0, 65536);
    if (W <= HUB_NT * 2)
      hipLaunchKernelGGL(k_tri_hub_count<2>, dim3(grid), dim3(HUB_NT), 0, s, rowptr, col, hb, K, c0, c1, Hc, total);
    else if (W <= HUB_NT * 4)
      hipLaunchKernelGGL(k_tri_hub_count<4>, dim3(grid), dim3(HUB_NT), 0, s, rowptr, col, hb, K, c0, c1, Hc, total);
    else if (W <= HUB_NT * 8)
      hipLaunchKernelGGL(k_tri_hub_count<8>, dim3(grid), dim3(HUB_NT), 0, s, rowptr, col, hb, K, c0, c1, Hc, total);
    else if (W <= HUB_NT * 16)
      hipLaunchKernelGGL(k_tri_hub_count<16>, dim3(grid), dim3(HUB_NT), 0, s, rowptr, col, hb, K, c0, c1, Hc, total);
    else
      hipLaunchKernelGGL(k_tri_hub_count<32>, dim3(grid), dim3(HUB_NT), 0, s, rowptr, col, hb, K, c0, c1, Hc, total);
    MRH_CHECK_LAUNCH();
  }
}

void tri_hub_pull_prep(const uint32_t* col, const uint64_t* okeys, const int64_t* rowptr, int64_t hb, int64_t ea,
                       int64_t n, uint64_t* tk, uint32_t* endx, hipStream_t s) {
  if (n <= 0) return;
  check_arg(n < (int64_t(1) << 32), "tri_hub_pull: more than 2^32 hub edges on one rank");
  hipLaunchKernelGGL(k_tri_tpack, dim3(grid_for(n)), dim3(NT), 0, s, col, ea, n, hb, tk);
  MRH_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_tri_hub_end, dim3(grid_for(n)), dim3(NT), 0, s, okeys, rowptr, ea, n, endx);
  MRH_CHECK_LAUNCH();
}

void tri_hub_pull_npieces(const int64_t* tptr, const int64_t* rowptr, int64_t hb, int64_t K, int64_t* np,
                          hipStream_t s) {
  if (K <= 0) return;
  hipLaunchKernelGGL(k_tri_pull_npieces, dim3(grid_for(K)), dim3(NT), 0, s, tptr, rowptr, hb, K, np);
  MRH_CHECK_LAUNCH();
}

int64_t tri_hub_pull_max_items(int64_t n, int64_t K) { return n / PULL_PIECE + K + 1; }

void tri_hub_pull(const int64_t* rowptr, const uint32_t* col, int64_t hb, int64_t K, int64_t ea, const uint64_t* tks,
                  const int64_t* tptr, const uint32_t* endx, const int64_t* off, uint64_t* items, uint64_t* big,
                  unsigned int* nbig, const uint64_t* H, unsigned long long* total, hipStream_t s) {
  if (K <= 0) return;
  hipLaunchKernelGGL(k_tri_pull_items, dim3(grid_for(K)), dim3(NT), 0, s, off, K, items);
  MRH_CHECK_LAUNCH();
  MRH_HIP(hipMemsetAsync(nbig, 0, sizeof(unsigned int), s));
  // off[K] = the item count, read on the device (no host round trip)
  hipLaunchKernelGGL(k_tri_hub_pull<TW>, dim3(4096), dim3(NT), 0, s, rowptr, col, hb, ea, tks, tptr, endx,
                     (const uint64_t*)items, off + K, big, nbig, total);
  MRH_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_tri_hub_pull_big, dim3(512), dim3(BIG_NT), 0, s, rowptr, col, hb, ea, tks, tptr, endx,
                     (const uint64_t*)big, (const unsigned int*)nbig, (const unsigned long long*)H, K / 64, total);
  MRH_CHECK_LAUNCH();
}

void tri_core_build(const int64_t* rowptr, const uint32_t* col, int64_t cb, int64_t T, int8_t* A, hipStream_t s) {
  if (T <= 0) return;
  MRH_HIP(hipMemsetAsync(A, 0, (size_t)T * (size_t)T, s));
  hipLaunchKernelGGL(k_tri_core_build, dim3((unsigned)std::min<int64_t>((T + HASH_NW - 1) / HASH_NW, 16384)), dim3(NT),
                     0, s, rowptr, col, cb, T, A);
  MRH_CHECK_LAUNCH();
}

void tri_rowptr(const uint64_t* okeys, int64_t m, int64_t nvert, int64_t* rowptr, hipStream_t s) {
  hipLaunchKernelGGL(k_rowptr, dim3(grid_for(nvert + 1)), dim3(NT), 0, s, okeys, m, nvert, rowptr);
  MRH_CHECK_LAUNCH();
}

void tri_emit(const int64_t* rowptr, const uint32_t* col, const uint64_t* okeys, int64_t e0, int64_t e1,
              const int64_t* off, uint64_t* out, hipStream_t s) {
  if (e1 <= e0) return;
  hipLaunchKernelGGL(k_tri_emit, dim3(grid_for(e1 - e0)), dim3(NT), 0, s, rowptr, col, okeys, e0, e1, off, out);
  MRH_CHECK_LAUNCH();
}

}  // namespace k
}  // namespace mrh
