// Iterative-graph kernels (PageRank over the MapReduce plan of pagerank.py).
//
// The reference's pagerank command is a stub (oink/pagerank.cpp:54-56); the
// algorithm follows oinkdoc/pagerank.txt: weights 1/outdeg (degree_weight),
// r' = (1-alpha)/N + alpha * (sum_in w*r + dangling/N).
//
//  pr_contrib : map+combine of one iteration, fused: for every destination
//               vertex group g (edges pre-sorted by (owner(dst), dst)),
//               send[g] = sum_e r[src_local[e]] * w[e]   (balanced segred)
//  pr_combine : reduce side: acc[vid[g]] = sum of received partials of g
//  pr_update  : r_new = base + alpha*(acc + dangling/N); per-block |r_new-r|
//               and dangling-mass partials for the convergence allreduce
#include "common.h"
#include "launch.h"
#include "segred.h"
#include "vmix.h"
#include "wavesegred.h"

namespace mrh {
namespace k {
namespace {

constexpr int NT = 256;

struct ContribGet {
  const int32_t* src;
  const float* w;
  const float* r;
  __device__ __forceinline__ float operator()(int64_t i) const { return r[src[i]] * w[i]; }
};

// unweighted form: r already holds r_i / outdeg_i (written by pr_update), so
// the per-edge weight stream is not read at all
struct ContribGetC {
  const int32_t* src;
  const float* c;
  // the index stream is read once: non-temporal, so it does not evict the
  // gathered rank array from L2 / Infinity Cache
  __device__ __forceinline__ float operator()(int64_t i) const { return c[__builtin_nontemporal_load(src + i)]; }
};

// ---------------------------------------------------------------- plan build
// The PageRank plan of one rank built without a group-by or a payload array:
// the edges are sorted twice as packed u64 keys (by source: out-degrees are
// run lengths; then by destination group with the new source id in the low
// word), the degree relabel sorts the nlocal vertices.

// packed (local source << 32 | destination) of every edge: sorting it on
// the source bits makes the out-degrees segment lengths (random-address
// global atomics run at the memory side, ~17x below their coalesced rate:
// a degree histogram by atomics cost 98 ms on RMAT-26, this sort ~20)
// swap: (destination << 32 | local source) instead — the out-degrees then
// come from a partitioned count of the low words (count_low_words), no sort
__global__ __launch_bounds__(NT) void k_pr_pack_src(const int64_t* __restrict__ e, int64_t n, int P, int swap,
                                                    uint64_t* __restrict__ out) {
  const int64_t stride = (int64_t)gridDim.x * NT;
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += stride) {
    const int64_t u = __builtin_nontemporal_load(e + 2 * i), v = __builtin_nontemporal_load(e + 2 * i + 1);
    const uint64_t lu = (uint64_t)(P == 1 ? u : u / P);
    out[i] = swap ? (((uint64_t)v << 32) | (uint32_t)lu) : ((lu << 32) | (uint32_t)v);
  }
}

// out-degrees from edges sorted on the source's bits above `shift` (the low
// word is the source; runs of 2^shift sources are contiguous): one block per
// tile of DW_TILE edges counts them in an LDS window of DW_BINS sources from
// its first edge's run, then adds the window to deg (lane-contiguous atomics);
// an edge past the window (a tile spanning more than DW_BINS sources, i.e.
// average degree < 0.5 there) adds to deg directly
constexpr int DW_TILE = 8192, DW_BINS = 16384;
__global__ __launch_bounds__(NT) void k_pr_deg_window(const uint64_t* __restrict__ e, int64_t m, int shift,
                                                      uint32_t* __restrict__ deg) {
  __shared__ uint32_t h[DW_BINS];
  const int64_t t0 = (int64_t)blockIdx.x * DW_TILE;
  const int tn = (int)(m - t0 < DW_TILE ? m - t0 : DW_TILE);
  const uint32_t vbase = ((uint32_t)e[t0] >> shift) << shift;
  for (int i = threadIdx.x; i < DW_BINS; i += NT) h[i] = 0;
  __syncthreads();
  const int lane = dev::lane_id();
  for (int i = threadIdx.x; i < DW_TILE; i += NT) {
    const bool valid = i < tn;
    const uint32_t v = valid ? (uint32_t)e[t0 + i] : 0u;
    const uint64_t active = __ballot(valid);
    if (!active) break;
    // a hub's run: every lane on one source is one add (same-address LDS
    // atomics from 64 lanes serialise)
    const int first = __ffsll((long long)active) - 1;
    const uint32_t v0 = (uint32_t)__shfl((int)v, first, MRH_WAVE);
    if (__ballot(valid && v == v0) == active) {
      if (lane == first) {
        if (v0 - vbase < (uint32_t)DW_BINS) atomicAdd(&h[v0 - vbase], (uint32_t)__popcll(active));
        else atomicAdd(deg + v0, (uint32_t)__popcll(active));
      }
    } else if (valid) {
      if (v - vbase < (uint32_t)DW_BINS) atomicAdd(&h[v - vbase], 1u);
      else atomicAdd(deg + v, 1u);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < DW_BINS; i += NT) {
    const uint32_t c = h[i];
    if (c) atomicAdd(deg + vbase + i, c);
  }
}

// head flag of every run of equal high words in a sorted packed array
__global__ __launch_bounds__(NT) void k_pr_heads(const uint64_t* __restrict__ s, int64_t n,
                                                 uint32_t* __restrict__ flags) {
  const int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (i < n) flags[i] = (i == 0 || (s[i - 1] >> 32) != (s[i] >> 32)) ? 1u : 0u;
}

// deg[source of run g] = length of run g (deg zeroed before)
__global__ __launch_bounds__(NT) void k_pr_run_degree(const uint64_t* __restrict__ s, const int64_t* __restrict__ seg,
                                                      int64_t nrun, uint32_t* __restrict__ deg) {
  const int64_t g = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (g < nrun) deg[s[seg[g]] >> 32] = (uint32_t)(seg[g + 1] - seg[g]);
}

// vertex sort key: descending degree, ties by id (stable sort of ~deg)
__global__ __launch_bounds__(NT) void k_pr_degkey(const uint32_t* __restrict__ deg, int64_t n,
                                                  uint64_t* __restrict__ key, uint32_t* __restrict__ iota) {
  const int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (i < n) {
    key[i] = (uint64_t)(0xFFFFFFFFu - deg[i]);
    iota[i] = (uint32_t)i;
  }
}

// new id i of old vertex order[i]: nid[order[i]] = i; the per-new-id
// dangling flag and 1/outdeg; the dangling count (one atomic per wave);
// degn (nullable): the out-degree of every new id (degree-descending)
__global__ __launch_bounds__(NT) void k_pr_relabel(const uint32_t* __restrict__ order, const uint32_t* __restrict__ deg,
                                                   int64_t n, int32_t* __restrict__ nid, int64_t* __restrict__ order64,
                                                   uint8_t* __restrict__ dangling, float* __restrict__ invdeg,
                                                   unsigned long long* __restrict__ ndangling,
                                                   int32_t* __restrict__ degn) {
  const int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x;
  bool dg = false;
  if (i < n) {
    const uint32_t o = order[i];
    nid[o] = (int32_t)i;
    order64[i] = o;
    const uint32_t d = deg[o];
    dg = d == 0;
    dangling[i] = dg ? 1 : 0;
    invdeg[i] = dg ? 0.f : (float)(1.0 / (double)d);
    if (degn) degn[i] = (int32_t)d;
  }
  // degrees descend, so the dangling vertices are the tail: the first of
  // them records the count (one store, no per-wave atomics on one word)
  if (i < n && dg) {
    const bool prev_dg = i > 0 && deg[order[i - 1]] == 0;
    if (!prev_dg) *ndangling = (unsigned long long)(n - i);
  }
}

// out[k] = in[min(k * stride, n - 1)], k < ns (a host-sized sample of a scan)
__global__ __launch_bounds__(NT) void k_sample_i64(const int64_t* __restrict__ in, int64_t n, int64_t stride,
                                                   int64_t ns, int64_t* __restrict__ out) {
  const int64_t k = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (k < ns) out[k] = in[k * stride < n ? k * stride : n - 1];
}

// source range of a new source id: hot ranges [rb[r], rb[r+1]) for r < nr,
// every id >= rb[nr] is the cold range nr
__device__ __forceinline__ uint32_t pr_range_of(uint32_t src, const int32_t* __restrict__ rb, int nr) {
  int lo = 0, hi = nr;  // number of rb[1..nr] <= src
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if ((uint32_t)rb[mid] <= src) lo = mid;
    else hi = mid - 1;
  }
  return (uint32_t)lo;
}

// the gather's sort key of every source-sorted edge (u << 32 | v): hi =
// destination group (one rank, no exchange: v; otherwise (v % P) * nlmax +
// v / P, owner-major), lo = new id of u (u is monotone here: the nid reads
// are a sequential walk)
__global__ __launch_bounds__(NT) void k_pr_pack(const uint64_t* __restrict__ su, int64_t n, int P, int64_t nlmax,
                                                int local, int swapped, const int32_t* __restrict__ nid,
                                                const int32_t* __restrict__ rb, int nr, int dbits,
                                                uint64_t* __restrict__ out) {
  const int64_t stride = (int64_t)gridDim.x * NT;
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += stride) {
    uint64_t x = __builtin_nontemporal_load(su + i);
    if (swapped) x = (x << 32) | (x >> 32);  // (v << 32 | u) input: unsorted, nid[u] is a random read
    const int64_t v = (int64_t)(uint32_t)x;
    // one GPU: the destination as its NEW id (the relabelled id space of the
    // rank vector), so the combine writes each tile of new ids contiguously;
    // P > 1: the owner-major global destination
    uint64_t hi = local ? (uint64_t)(uint32_t)nid[v] : (uint64_t)((v % P) * nlmax + v / P);
    const uint32_t src = (uint32_t)nid[x >> 32];
    // XCD source ranges: the range of the new source id above the
    // destination bits (groups = (range, destination))
    if (rb) hi |= (uint64_t)pr_range_of(src, rb, nr) << dbits;
    out[i] = (hi << 32) | src;
  }
}

// ---- multi-GPU plan (graphplan.cpp build_device_dist): vertex v is owned by
// rank sigma(v) % P as local id sigma(v) / P (vmix.h; sigma = identity when
// mix == 0). Edges move twice: to the source owner (out-degrees, relabel) and
// to the destination owner, which gathers c = r / outdeg from the replicated
// (all-gathered) c vector.

// q = x / d for x, d < 2^31 without an integer divide (none in hardware):
// a double product (exact to well under one unit) and one correction step
__device__ __forceinline__ uint32_t pr_udiv(uint32_t x, uint32_t d, double inv) {
  uint32_t q = (uint32_t)((double)x * inv);
  if (q * d > x) --q;
  else if ((q + 1) * d <= x) ++q;
  return q;
}

// edge (u, v) -> packed (sigma(u) << 32 | sigma(v)), destination rank
// sigma(u) % P
__global__ __launch_bounds__(NT) void k_pr_mix_pack(const int64_t* __restrict__ e, int64_t n, int P, int64_t N, int b,
                                                    int mix, uint64_t* __restrict__ out, int32_t* __restrict__ dest) {
  const int64_t stride = (int64_t)gridDim.x * NT;
  const double invP = 1.0 / (double)P;
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += stride) {
    uint64_t u = (uint64_t)__builtin_nontemporal_load(e + 2 * i), v = (uint64_t)__builtin_nontemporal_load(e + 2 * i + 1);
    if (mix) {
      u = dev::vmix(u, N, b);
      v = dev::vmix(v, N, b);
    }
    out[i] = (v << 32) | u;  // the source in the low word: out-degrees by count_low_words
    dest[i] = (int32_t)((uint32_t)u - pr_udiv((uint32_t)u, (uint32_t)P, invP) * (uint32_t)P);
  }
}

// at the source owner: (su << 32 | sv) -> (su / P << 32 | sv), in place
__global__ __launch_bounds__(NT) void k_pr_localize(uint64_t* __restrict__ p, int64_t n, int P) {
  const int64_t stride = (int64_t)gridDim.x * NT;
  const double invP = 1.0 / (double)P;
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += stride) {
    const uint64_t x = p[i];
    p[i] = (x & 0xffffffff00000000ull) | (uint64_t)pr_udiv((uint32_t)x, (uint32_t)P, invP);
  }
}

// source-sorted (lu << 32 | sv) -> (sv << 32 | pos), pos = me * S + nid[lu]:
// the source's slot in the all-gathered c vector (rank-major slices of S
// entries); destination rank sv % P
__global__ __launch_bounds__(NT) void k_pr_pack_dst(const uint64_t* __restrict__ su, int64_t n, int P, int64_t base,
                                                    const int32_t* __restrict__ nid, uint64_t* __restrict__ out,
                                                    int32_t* __restrict__ dest) {
  const int64_t stride = (int64_t)gridDim.x * NT;
  const double invP = 1.0 / (double)P;
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += stride) {
    const uint64_t x = __builtin_nontemporal_load(su + i);
    const uint64_t sv = x >> 32;
    const uint64_t pos = (uint64_t)(base + nid[(uint32_t)x]);
    out[i] = (sv << 32) | pos;
    dest[i] = (int32_t)((uint32_t)sv - pr_udiv((uint32_t)sv, (uint32_t)P, invP) * (uint32_t)P);
  }
}

// at the destination owner: (sv << 32 | pos) -> the gather's sort key:
// hi = (source range << dbits) | new destination id nid[sv / P], lo = pos.
// The source range is found on the interleaved global order gid = (pos % S)
// * P + pos / S (every rank's hottest sources first), so a range's sources
// are P contiguous pieces of the c vector whose total fits one XCD's L2
__global__ __launch_bounds__(NT) void k_pr_pack_gather(const uint64_t* __restrict__ in, int64_t n, int P, int64_t S,
                                                       const int32_t* __restrict__ nid, const int32_t* __restrict__ rb,
                                                       int nr, int dbits, uint64_t* __restrict__ out) {
  const int64_t stride = (int64_t)gridDim.x * NT;
  const double invP = 1.0 / (double)P, invS = 1.0 / (double)S;
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += stride) {
    const uint64_t x = __builtin_nontemporal_load(in + i);
    const uint32_t pos = (uint32_t)x;
    uint64_t hi = (uint64_t)(uint32_t)nid[pr_udiv((uint32_t)(x >> 32), (uint32_t)P, invP)];
    if (rb) {
      const uint32_t q = pr_udiv(pos, (uint32_t)S, invS);
      const uint32_t gid = (pos - q * (uint32_t)S) * (uint32_t)P + q;
      hi |= (uint64_t)pr_range_of(gid, rb, nr) << dbits;
    }
    out[i] = (hi << 32) | pos;
  }
}

// global ids of the owned vertices: ids[i] = sigma^-1(order[i] * P + me)
__global__ __launch_bounds__(NT) void k_pr_unmix_ids(const int64_t* __restrict__ order, int64_t n, int P, int me,
                                                     int64_t N, int b, int mix, int64_t* __restrict__ ids) {
  const int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (i >= n) return;
  const uint64_t y = (uint64_t)order[i] * (uint64_t)P + (uint64_t)me;
  ids[i] = (int64_t)(mix ? dev::vunmix(y, N, b) : y);
}

// sorted packed keys -> the int32 source stream of the gather and the u32
// head flag of every destination group
__global__ __launch_bounds__(NT) void k_pr_unpack(const uint64_t* __restrict__ s, int64_t n, int32_t* __restrict__ src,
                                                  uint32_t* __restrict__ flags) {
  const int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (i >= n) return;
  const uint64_t k = s[i];
  src[i] = (int32_t)(uint32_t)k;
  flags[i] = (i == 0 || (s[i - 1] >> 32) != (k >> 32)) ? 1u : 0u;
}

// the same split, the heads as a bitmap (bit i of u32 word i / 32; one
// ballot per wave, written as one 8-byte store by lane 0 — waves start at
// multiples of 64) instead of a u32 flag per edge: the gather's segment index
// (wavesegred.h H) directly, 1/32 of the bytes; words past n stay as zeroed
__global__ __launch_bounds__(NT) void k_pr_unpack_bits(const uint64_t* __restrict__ s, int64_t n,
                                                       int32_t* __restrict__ src, uint2* __restrict__ H) {
  const int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x;
  bool head = false;
  if (i < n) {
    const uint64_t k = s[i];
    src[i] = (int32_t)(uint32_t)k;
    head = i == 0 || (s[i - 1] >> 32) != (k >> 32);
  }
  const uint64_t b = __ballot(head);
  if (dev::lane_id() == 0 && i < n) H[i >> 6] = make_uint2((uint32_t)b, (uint32_t)(b >> 32));
}

// per destination group: its hi word (the group's destination)
__global__ __launch_bounds__(NT) void k_pr_group_hi(const uint64_t* __restrict__ s, const int64_t* __restrict__ seg,
                                                    int64_t ngrp, int64_t* __restrict__ hi) {
  const int64_t g = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (g < ngrp) hi[g] = (int64_t)(s[seg[g]] >> 32);
}

// target row of group g: nid[hi] (hi an old id), or hi itself (nid == null);
// the bits at and above dmask's width are the source block
__global__ __launch_bounds__(NT) void k_pr_group_vid(const int64_t* __restrict__ hi, int64_t ngrp,
                                                     const int32_t* __restrict__ nid, int64_t dmask,
                                                     int32_t* __restrict__ vid) {
  const int64_t g = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (g < ngrp) {
    const int64_t h = hi[g] & dmask;
    vid[g] = nid ? nid[h] : (int32_t)h;
  }
}

// first group of every (range r, destination tile t) of the (range,
// destination)-sorted group keys hi: off[r * (ntile + 1) + t]; t == ntile is
// the end of range r
__global__ __launch_bounds__(NT) void k_pr_range_offsets(const int64_t* __restrict__ hi, int64_t ngrp, int dbits,
                                                         int R, int64_t ntile, int tile_bits,
                                                         int64_t* __restrict__ off) {
  const int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (i >= (int64_t)R * (ntile + 1)) return;
  const int64_t r = i / (ntile + 1), t = i - r * (ntile + 1);
  const int64_t key = t < ntile ? (r << dbits) + (t << tile_bits) : ((r + 1) << dbits);
  int64_t lo = 0, h = ngrp;
  while (lo < h) {
    const int64_t mid = (lo + h) >> 1;
    if (hi[mid] < key) lo = mid + 1;
    else h = mid;
  }
  off[i] = lo;
}

// One PageRank step's combine + update per tile of 2^PR_TILE_BITS
// destinations (new ids d0 .. d0 + TILE): the sum over the source ranges of
// the partial sums of each destination, then r_new = base + alpha * (sum +
// dangling / N), c = r_new / outdeg, and the block's L1 delta and dangling
// mass as fp64 partials — the rank vector is read and written once per
// iteration, no acc array round trip. The tile's R runs of (destination,
// partial) are read as one flattened index space (no per-range barrier, no
// dependent load chain) and added into LDS as 62-bit fixed point with integer
// atomics — integer adds commute, so the result does not depend on their
// order (bitwise reproducible). Every partial is in [0, 1] (r sums to 1 and
// c = r / outdeg), so 2^62 * sum fits int64; values >= 2^-39 convert exactly.
constexpr int PR_TILE_BITS = 12;
constexpr int PR_MAX_RANGES = 64;

__device__ __forceinline__ void pr_one(float a, float rv, float idg, bool dg, float base, float alpha, float dterm,
                                       float& x, float& c, double& d, double& dm) {
  x = base + alpha * (a + dterm);
  c = x * idg;
  d += fabs((double)x - (double)rv);
  if (dg) dm += x;
}

__device__ __forceinline__ float fx_to_f(unsigned long long v) { return (float)((double)(long long)v * 0x1p-62); }

__global__ __launch_bounds__(NT) void k_pr_tile_step(const float* __restrict__ send, const int32_t* __restrict__ ghi,
                                                     const int64_t* __restrict__ off, int R, int64_t ntile,
                                                     int64_t ndst, const float* __restrict__ r,
                                                     float* __restrict__ rn, const uint8_t* __restrict__ dangling,
                                                     float base, float alpha, const double* __restrict__ dmass,
                                                     double invN, const float* __restrict__ invdeg,
                                                     float* __restrict__ cout, double* __restrict__ partial) {
  constexpr int TILE = 1 << PR_TILE_BITS;
  __shared__ unsigned long long sum[TILE];
  __shared__ int64_t s_b[PR_MAX_RANGES];
  __shared__ int s_pre[PR_MAX_RANGES + 1];
  __shared__ double sh[2][NT / MRH_WAVE];
  const int64_t t = blockIdx.x;
  const int64_t d0 = t << PR_TILE_BITS;
  for (int i = threadIdx.x; i < TILE; i += NT) sum[i] = 0ull;
  if (threadIdx.x < MRH_WAVE) {  // range starts and a wave scan of the run lengths (R <= 64)
    const int q = threadIdx.x;
    int64_t g0 = 0, g1 = 0;
    if (q < R) {
      g0 = off[(int64_t)q * (ntile + 1) + t];
      g1 = off[(int64_t)q * (ntile + 1) + t + 1];
      s_b[q] = g0;
    }
    int len = (int)(g1 - g0), incl = len;
#pragma unroll
    for (int d = 1; d < MRH_WAVE; d <<= 1) {
      const int y = __shfl_up(incl, d, MRH_WAVE);
      if (q >= d) incl += y;
    }
    if (q < R) s_pre[q] = incl - len;
    if (q == R - 1) s_pre[R] = incl;
  }
  __syncthreads();
  const int total = s_pre[R];
  for (int j = threadIdx.x; j < total; j += NT) {
    int lo = 0, hi = R - 1;  // the range holding flattened pair j: last range with s_pre <= j
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (s_pre[mid] <= j) lo = mid;
      else hi = mid - 1;
    }
    const int64_t g = s_b[lo] + (j - s_pre[lo]);
    const int d = (int)(ghi[g] - d0);
    atomicAdd(&sum[d], (unsigned long long)(long long)((double)send[g] * 0x1p62));
  }
  __syncthreads();
  const float dterm = (float)(dmass[0] * invN);
  double dd = 0.0, dm = 0.0;
  const int64_t nd = ndst - d0 < TILE ? ndst - d0 : TILE;
  if (nd == TILE) {  // full tile: 16-byte accesses (d0 is a multiple of TILE)
    for (int q = threadIdx.x; q < TILE / 4; q += NT) {
      const int64_t v4 = (d0 >> 2) + q;
      const float4 rv = reinterpret_cast<const float4*>(r)[v4];
      const float4 ig = reinterpret_cast<const float4*>(invdeg)[v4];
      const uint32_t dg = reinterpret_cast<const uint32_t*>(dangling)[v4];
      float4 x, c;
      pr_one(fx_to_f(sum[4 * q]), rv.x, ig.x, dg & 0xffu, base, alpha, dterm, x.x, c.x, dd, dm);
      pr_one(fx_to_f(sum[4 * q + 1]), rv.y, ig.y, (dg >> 8) & 0xffu, base, alpha, dterm, x.y, c.y, dd, dm);
      pr_one(fx_to_f(sum[4 * q + 2]), rv.z, ig.z, (dg >> 16) & 0xffu, base, alpha, dterm, x.z, c.z, dd, dm);
      pr_one(fx_to_f(sum[4 * q + 3]), rv.w, ig.w, dg >> 24, base, alpha, dterm, x.w, c.w, dd, dm);
      reinterpret_cast<float4*>(rn)[v4] = x;
      reinterpret_cast<float4*>(cout)[v4] = c;
    }
  } else {
    for (int i = threadIdx.x; i < nd; i += NT) {
      const int64_t v = d0 + i;
      float x, c;
      pr_one(fx_to_f(sum[i]), r[v], invdeg[v], dangling[v] != 0, base, alpha, dterm, x, c, dd, dm);
      rn[v] = x;
      cout[v] = c;
    }
  }
  for (int o = MRH_WAVE / 2; o > 0; o >>= 1) {
    dd += __shfl_xor(dd, o, MRH_WAVE);
    dm += __shfl_xor(dm, o, MRH_WAVE);
  }
  if (dev::lane_id() == 0) {
    sh[0][dev::wave_id()] = dd;
    sh[1][dev::wave_id()] = dm;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double a = 0, b = 0;
    for (int w = 0; w < NT / MRH_WAVE; ++w) {
      a += sh[0][w];
      b += sh[1][w];
    }
    partial[2 * t] = a;
    partial[2 * t + 1] = b;
  }
}

// stats[0..1] = the sums of the per-tile (L1 delta, dangling mass) partials
// of k_pr_tile_step, in a fixed order (one block: bitwise reproducible, and
// no allocation — the iteration can be replayed from a captured graph)
__global__ __launch_bounds__(NT) void k_pr_partials_sum(const double* __restrict__ part, int64_t ntile,
                                                        double* __restrict__ stats) {
  __shared__ double sh[2][NT / MRH_WAVE];
  double a = 0.0, b = 0.0;
  for (int64_t t = threadIdx.x; t < ntile; t += NT) {
    a += part[2 * t];
    b += part[2 * t + 1];
  }
  for (int o = MRH_WAVE / 2; o > 0; o >>= 1) {
    a += __shfl_xor(a, o, MRH_WAVE);
    b += __shfl_xor(b, o, MRH_WAVE);
  }
  if (dev::lane_id() == 0) {
    sh[0][dev::wave_id()] = a;
    sh[1][dev::wave_id()] = b;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double x = 0.0, y = 0.0;
    for (int w = 0; w < NT / MRH_WAVE; ++w) {
      x += sh[0][w];
      y += sh[1][w];
    }
    stats[0] = x;
    stats[1] = y;
  }
}

struct PermGet {
  const int32_t* perm;
  const float* v;
  __device__ __forceinline__ float operator()(int64_t i) const { return v[perm[i]]; }
};

__global__ __launch_bounds__(NT) void k_scatter_f32(const float* __restrict__ v, const int32_t* __restrict__ idx,
                                                   int64_t n, float* __restrict__ out) {
  int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (i < n) out[idx[i]] = v[i];
}

// one PageRank update over the local vertices, 4 per thread per trip
// (16-byte loads/stores of acc, r, invdeg, rn, c; the bytes of dangling as
// one u32), plus the L1 delta and the dangling mass as fp64 block partials.
// acc is zeroed behind its read, so the next iteration's combine starts
// from a clean array without a separate fill pass.
__global__ __launch_bounds__(NT) void k_pr_update(float* __restrict__ acc, const float* __restrict__ r,
                                                 float* __restrict__ rn, const uint8_t* __restrict__ dangling,
                                                 int64_t n, float base, float alpha,
                                                 const double* __restrict__ dmass, double invN,
                                                 const float* __restrict__ invdeg, float* __restrict__ cout,
                                                 double* __restrict__ partial) {
  __shared__ double sh[2][NT / MRH_WAVE];
  const float dterm = (float)(dmass[0] * invN);
  double d = 0.0, dm = 0.0;
  const int64_t n4 = n / 4;
  const int64_t stride = (int64_t)gridDim.x * NT;
  for (int64_t q = (int64_t)blockIdx.x * NT + threadIdx.x; q < n4; q += stride) {
    const float4 a = reinterpret_cast<const float4*>(acc)[q];
    const float4 rv = reinterpret_cast<const float4*>(r)[q];
    const float4 ig = cout ? reinterpret_cast<const float4*>(invdeg)[q] : make_float4(0.f, 0.f, 0.f, 0.f);
    const uint32_t dg = reinterpret_cast<const uint32_t*>(dangling)[q];
    reinterpret_cast<float4*>(acc)[q] = make_float4(0.f, 0.f, 0.f, 0.f);
    float4 x, c;
    pr_one(a.x, rv.x, ig.x, dg & 0xffu, base, alpha, dterm, x.x, c.x, d, dm);
    pr_one(a.y, rv.y, ig.y, (dg >> 8) & 0xffu, base, alpha, dterm, x.y, c.y, d, dm);
    pr_one(a.z, rv.z, ig.z, (dg >> 16) & 0xffu, base, alpha, dterm, x.z, c.z, d, dm);
    pr_one(a.w, rv.w, ig.w, dg >> 24, base, alpha, dterm, x.w, c.w, d, dm);
    reinterpret_cast<float4*>(rn)[q] = x;
    if (cout) reinterpret_cast<float4*>(cout)[q] = c;
  }
  for (int64_t i = 4 * n4 + (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += stride) {
    float x, c;
    pr_one(acc[i], r[i], cout ? invdeg[i] : 0.f, dangling[i] != 0, base, alpha, dterm, x, c, d, dm);
    acc[i] = 0.f;
    rn[i] = x;
    if (cout) cout[i] = c;
  }
  for (int o = MRH_WAVE / 2; o > 0; o >>= 1) {
    d += __shfl_xor(d, o, MRH_WAVE);
    dm += __shfl_xor(dm, o, MRH_WAVE);
  }
  if (dev::lane_id() == 0) {
    sh[0][dev::wave_id()] = d;
    sh[1][dev::wave_id()] = dm;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double a = 0, b = 0;
    for (int w = 0; w < NT / MRH_WAVE; ++w) {
      a += sh[0][w];
      b += sh[1][w];
    }
    partial[2 * blockIdx.x] = a;
    partial[2 * blockIdx.x + 1] = b;
  }
}

// generic plan getters: value carried by edge e = x[src[e]] (+ w[e])
template <typename T>
struct XWGet {
  const int32_t* src;
  const T* x;
  const T* w;
  __device__ __forceinline__ T operator()(int64_t i) const {
    T v = x[__builtin_nontemporal_load(src + i)];
    return w ? v + w[i] : v;
  }
};
template <typename T>
struct PermGetT {
  const int32_t* perm;
  const T* v;
  __device__ __forceinline__ T operator()(int64_t i) const { return v[perm[i]]; }
};
template <typename T>
__global__ __launch_bounds__(NT) void k_scatter_t(const T* __restrict__ v, const int32_t* __restrict__ idx, int64_t n,
                                                 T* __restrict__ out) {
  int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (i < n) out[idx[i]] = v[i];
}

// Wedges of tri_find (reference oink/tri_find.cpp:207-276, O(d^2) per vertex):
// for group g with neighbour list nb[seg[g]..seg[g+1]) emit every pair
// (min, max) with value = centre key[g]. Only groups with a wedge (d >= 2)
// take part: gidx lists them and wscan is the exclusive scan of their C(d,2).
// One block per tile of WG_TILE consecutive wedge ids: the tile's first group
// comes from tg (k_wedge_tile_groups, one pass over the groups per call —
// a per-block global binary search cost ~40 us of latency per tile), the
// block stages the scan entries and ids of its groups in LDS (at most
// WG_TILE + 1: each has a wedge), and every wedge finds its group in an LDS
// map (each group's index written at its first wedge, then a max-scan). The
// pair (j, k) comes from the triangular index; thread t writes wedges t,
// t + NT, ... of the tile (coalesced stores).
constexpr int WG_IT = 16;
constexpr int WG_TILE = NT * WG_IT;

// tg[t] = the group of wedge w0 + t * WG_TILE; tg[ntile] = the group of the
// call's last wedge (grid-stride over the groups)
__global__ __launch_bounds__(NT) void k_wedge_tile_groups(const int64_t* __restrict__ wscan, int64_t ngw, int64_t w0,
                                                          int64_t nwedge, int64_t ntile, int64_t* __restrict__ tg) {
  const int64_t w1 = w0 + nwedge;
  for (int64_t g = (int64_t)blockIdx.x * NT + threadIdx.x; g < ngw; g += (int64_t)gridDim.x * NT) {
    const int64_t a = wscan[g] > w0 ? wscan[g] : w0, b = wscan[g + 1] < w1 ? wscan[g + 1] : w1;
    if (a >= b) continue;
    for (int64_t t = (a - w0 + WG_TILE - 1) / WG_TILE; w0 + t * WG_TILE < b; ++t) tg[t] = g;
    if (b == w1) tg[ntile] = g;
  }
}

// CMP: the compact layout of large graphs — one word (min << vb | max) per
// wedge and a 4-byte centre (12 bytes a wedge instead of 24)
template <int CMP>
__global__ __launch_bounds__(NT) void k_wedges(const int64_t* __restrict__ seg, const int64_t* __restrict__ gidx,
                                              const int64_t* __restrict__ wscan, const int64_t* __restrict__ tg,
                                              const int64_t* __restrict__ nb, const int64_t* __restrict__ centre,
                                              int64_t w0, int64_t nwedge, int64_t* __restrict__ out_edge,
                                              void* __restrict__ out_centre, int vb) {
  __shared__ int64_t s_scan[WG_TILE + 2];
  __shared__ int64_t s_gi[WG_TILE + 2];
  __shared__ uint16_t s_map[WG_TILE];
  __shared__ int32_t s_run[NT];
  const int64_t t0 = (int64_t)blockIdx.x * WG_TILE;  // tile offset in this call's output
  const int tn = (int)(nwedge - t0 < WG_TILE ? nwedge - t0 : WG_TILE);
  // groups g0 .. g0 + ng - 1: the tile's first wedge's group to the next
  // tile's (one more than the tile's last group when a group starts it)
  const int64_t g0 = tg[blockIdx.x];
  const int ng = (int)(tg[blockIdx.x + 1] - g0 + 1);
  for (int i = threadIdx.x; i < WG_TILE; i += NT) s_map[i] = 0;
  __syncthreads();
  for (int i = threadIdx.x; i <= ng; i += NT) {
    const int64_t sc = wscan[g0 + i];
    s_scan[i] = sc;
    if (i < ng) {
      s_gi[i] = gidx[g0 + i];
      const int64_t pos = sc - (w0 + t0);
      if (pos > 0 && pos < tn) s_map[pos] = (uint16_t)i;
    }
  }
  __syncthreads();
  {  // inclusive max-scan of the map: thread t owns entries [WG_IT t, WG_IT t + WG_IT)
    const int b0 = threadIdx.x * WG_IT;
    int m = 0;
#pragma unroll
    for (int q = 0; q < WG_IT; ++q) m = max(m, (int)s_map[b0 + q]);
    s_run[threadIdx.x] = m;
    __syncthreads();
    for (int o = 1; o < NT; o <<= 1) {
      const int v = threadIdx.x >= o ? s_run[threadIdx.x - o] : 0;
      __syncthreads();
      s_run[threadIdx.x] = max(s_run[threadIdx.x], v);
      __syncthreads();
    }
    int run = threadIdx.x ? s_run[threadIdx.x - 1] : 0;
#pragma unroll
    for (int q = 0; q < WG_IT; ++q) {
      run = max(run, (int)s_map[b0 + q]);
      s_map[b0 + q] = (uint16_t)run;
    }
  }
  __syncthreads();
#pragma unroll 4
  for (int it = 0; it < WG_IT; ++it) {
    const int o = it * NT + threadIdx.x;
    if (o >= tn) break;
    const int64_t w = w0 + t0 + o;
    const int lo = s_map[o];
    const int64_t g = s_gi[lo];
    const int64_t t = w - s_scan[lo];
    const int64_t base = seg[g];
    const int64_t d = seg[g + 1] - base;
    // row j has (d-1-j) pairs; find j with S(j) <= t < S(j+1), S(j) = j*(2d-j-1)/2
    const double dd = (double)(2 * d - 1);
    int64_t j = (int64_t)floor((dd - sqrt(dd * dd - 8.0 * (double)t)) * 0.5);
    if (j < 0) j = 0;
    while (j > 0 && j * (2 * d - j - 1) / 2 > t) --j;
    while ((j + 1) * (2 * d - j - 2) / 2 <= t) ++j;
    const int64_t k = j + 1 + (t - j * (2 * d - j - 1) / 2);
    const int64_t a = nb[base + j], b = nb[base + k];
    const bool lt = (uint64_t)a < (uint64_t)b;
    if (CMP) {
      out_edge[t0 + o] = (int64_t)(((uint64_t)(lt ? a : b) << vb) | (uint64_t)(lt ? b : a));
      static_cast<uint32_t*>(out_centre)[t0 + o] = (uint32_t)centre[g];
    } else {
      out_edge[2 * (t0 + o)] = lt ? a : b;
      out_edge[2 * (t0 + o) + 1] = lt ? b : a;
      static_cast<int64_t*>(out_centre)[t0 + o] = centre[g];
    }
  }
}

}  // namespace

template <typename T>
void plan_gather_reduce_t(const int64_t* seg, int64_t nseg, int64_t ne, const int32_t* src, const T* x, const T* w,
                          int op, T* out, void* scratch, hipStream_t s) {
  size_t nc = dev::segred_carry_entries(ne);
  int64_t* cs = reinterpret_cast<int64_t*>(scratch);
  T* cv = reinterpret_cast<T*>(reinterpret_cast<char*>(scratch) + nc * sizeof(int64_t));
  XWGet<T> g{src, x, w};
  if (op == 0) dev::segred_launch<T, 0>(g, seg, nseg, ne, out, cs, cv, s);
  else if (op == 1) dev::segred_launch<T, 1>(g, seg, nseg, ne, out, cs, cv, s);
  else dev::segred_launch<T, 2>(g, seg, nseg, ne, out, cs, cv, s);
}
template <typename T>
void plan_combine_t(const int64_t* seg, int64_t ngrp, int64_t nrecv, const int32_t* perm, const T* recv,
                    const int32_t* vid, int op, T* grp, T* acc, void* scratch, hipStream_t s) {
  size_t nc = dev::segred_carry_entries(nrecv);
  int64_t* cs = reinterpret_cast<int64_t*>(scratch);
  T* cv = reinterpret_cast<T*>(reinterpret_cast<char*>(scratch) + nc * sizeof(int64_t));
  PermGetT<T> g{perm, recv};
  if (op == 0) dev::segred_launch<T, 0>(g, seg, ngrp, nrecv, grp, cs, cv, s);
  else if (op == 1) dev::segred_launch<T, 1>(g, seg, ngrp, nrecv, grp, cs, cv, s);
  else dev::segred_launch<T, 2>(g, seg, ngrp, nrecv, grp, cs, cv, s);
  if (ngrp > 0)
    hipLaunchKernelGGL(k_scatter_t<T>, dim3((unsigned)((ngrp + NT - 1) / NT)), dim3(NT), 0, s, grp, vid, ngrp, acc);
  MRH_CHECK_LAUNCH();
}

size_t plan_scratch_bytes(int64_t n) { return dev::segred_carry_entries(n) * 16 + 64; }

void plan_gather_reduce(int dtype, const int64_t* seg, int64_t nseg, int64_t ne, const int32_t* src, const void* x,
                        const void* w, int op, void* out, void* scratch, hipStream_t s) {
  if (nseg <= 0) return;
  switch (dtype) {
    case 1: plan_gather_reduce_t<int64_t>(seg, nseg, ne, src, (const int64_t*)x, (const int64_t*)w, op, (int64_t*)out, scratch, s); break;
    case 2: plan_gather_reduce_t<float>(seg, nseg, ne, src, (const float*)x, (const float*)w, op, (float*)out, scratch, s); break;
    default: plan_gather_reduce_t<double>(seg, nseg, ne, src, (const double*)x, (const double*)w, op, (double*)out, scratch, s); break;
  }
}
void plan_combine(int dtype, const int64_t* seg, int64_t ngrp, int64_t nrecv, const int32_t* perm, const void* recv,
                  const int32_t* vid, int op, void* grp, void* acc, void* scratch, hipStream_t s) {
  if (ngrp <= 0) return;
  switch (dtype) {
    case 1: plan_combine_t<int64_t>(seg, ngrp, nrecv, perm, (const int64_t*)recv, vid, op, (int64_t*)grp, (int64_t*)acc, scratch, s); break;
    case 2: plan_combine_t<float>(seg, ngrp, nrecv, perm, (const float*)recv, vid, op, (float*)grp, (float*)acc, scratch, s); break;
    default: plan_combine_t<double>(seg, ngrp, nrecv, perm, (const double*)recv, vid, op, (double*)grp, (double*)acc, scratch, s); break;
  }
}
int64_t ws_words(int64_t nval) { return dev::ws_head_words(nval); }
int64_t ws_waves(int64_t nval) { return dev::ws_nwave(nval); }
size_t ws_scratch_bytes(int64_t nval) {
  const int64_t nc = dev::ws_nwave(nval) * 2, nc2 = 2 * ((nc + 63) / 64);
  return (size_t)nc * 16 + (size_t)nc2 * 16 + 64;
}

void ws_bases(const int64_t* seg, int64_t nseg, int64_t nval, int64_t* wbase, hipStream_t s) {
  const int64_t nw = dev::ws_nwave(nval);
  if (nw > 0)
    hipLaunchKernelGGL(dev::k_ws_base, dim3((unsigned)((nw + 255) / 256)), dim3(256), 0, s, seg, nseg, nw, wbase);
  MRH_CHECK_LAUNCH();
}
void ws_index(const int64_t* seg, int64_t nseg, int64_t nval, uint32_t* H, int64_t* wbase, hipStream_t s) {
  const int64_t nw = dev::ws_nwave(nval);
  MRH_HIP(hipMemsetAsync(H, 0, sizeof(uint32_t) * dev::ws_head_words(nval), s));
  if (nseg > 0)
    hipLaunchKernelGGL(dev::k_ws_heads, dim3((unsigned)((nseg + 255) / 256)), dim3(256), 0, s, seg, nseg, H);
  if (nw > 0)
    hipLaunchKernelGGL(dev::k_ws_base, dim3((unsigned)((nw + 255) / 256)), dim3(256), 0, s, seg, nseg, nw, wbase);
  MRH_CHECK_LAUNCH();
}

template <typename T>
static void ws_gr_t(const uint32_t* H, const int64_t* wbase, int64_t nval, const int32_t* src, const T* x, const T* w,
                    int op, T* out, void* scratch, hipStream_t s, const int32_t* sched, int64_t slen, int64_t nx) {
  // scratch: carry (2 nw) ids + values, then the level-2 carry (2 ceil(2 nw / 64)) ids + values
  const int64_t nc = dev::ws_nwave(nval) * 2, nc2 = 2 * ((nc + 63) / 64);
  char* p = reinterpret_cast<char*>(scratch);
  int64_t* cs = reinterpret_cast<int64_t*>(p);
  T* cv = reinterpret_cast<T*>(p + (size_t)nc * sizeof(int64_t));
  int64_t* cs2 = reinterpret_cast<int64_t*>(p + (size_t)nc * 16);
  T* cv2 = reinterpret_cast<T*>(p + (size_t)nc * 16 + (size_t)nc2 * sizeof(int64_t));
  if (op == 0) dev::ws_gather_reduce<T, 0>(H, wbase, nval, src, x, w, out, cs, cv, s, cs2, cv2, sched, slen, nx);
  else if (op == 1) dev::ws_gather_reduce<T, 1>(H, wbase, nval, src, x, w, out, cs, cv, s, cs2, cv2, sched, slen, nx);
  else dev::ws_gather_reduce<T, 2>(H, wbase, nval, src, x, w, out, cs, cv, s, cs2, cv2, sched, slen, nx);
}

void ws_gather_reduce(int dtype, const uint32_t* H, const int64_t* wbase, int64_t nval, const int32_t* src,
                      const void* x, const void* w, int op, void* out, void* scratch, hipStream_t s,
                      const int32_t* sched, int64_t slen, int64_t nx) {
  if (nval <= 0) return;
  switch (dtype) {
    case 1: ws_gr_t<int64_t>(H, wbase, nval, src, (const int64_t*)x, (const int64_t*)w, op, (int64_t*)out, scratch, s, sched, slen, nx); break;
    case 2: ws_gr_t<float>(H, wbase, nval, src, (const float*)x, (const float*)w, op, (float*)out, scratch, s, sched, slen, nx); break;
    default: ws_gr_t<double>(H, wbase, nval, src, (const double*)x, (const double*)w, op, (double*)out, scratch, s, sched, slen, nx); break;
  }
}

int64_t wedge_tiles(int64_t nwedge) { return (nwedge + WG_TILE - 1) / WG_TILE; }

static void wedge_tile_groups(const int64_t* wscan, int64_t ngw, int64_t w0, int64_t nwedge, int64_t* tg,
                              hipStream_t s) {
  const unsigned g = (unsigned)std::max<int64_t>(1, std::min<int64_t>((ngw + NT - 1) / NT, 1 << 16));
  hipLaunchKernelGGL(k_wedge_tile_groups, dim3(g), dim3(NT), 0, s, wscan, ngw, w0, nwedge, wedge_tiles(nwedge), tg);
  MRH_CHECK_LAUNCH();
}

void wedges(const int64_t* seg, const int64_t* gidx, const int64_t* wscan, int64_t ngw, const int64_t* nb,
            const int64_t* centre, int64_t w0, int64_t nwedge, int64_t* out_edge, int64_t* out_centre, int64_t* tg,
            hipStream_t s) {
  if (nwedge <= 0 || ngw <= 0) return;
  wedge_tile_groups(wscan, ngw, w0, nwedge, tg, s);
  hipLaunchKernelGGL(k_wedges<0>, dim3((unsigned)wedge_tiles(nwedge)), dim3(NT), 0, s, seg, gidx, wscan, tg, nb,
                     centre, w0, nwedge, out_edge, (void*)out_centre, 0);
  MRH_CHECK_LAUNCH();
}

void wedges_compact(const int64_t* seg, const int64_t* gidx, const int64_t* wscan, int64_t ngw, const int64_t* nb,
                    const int64_t* centre, int64_t w0, int64_t nwedge, int vb, int64_t* out_key, uint32_t* out_centre,
                    int64_t* tg, hipStream_t s) {
  if (nwedge <= 0 || ngw <= 0) return;
  check_arg(vb > 0 && vb <= 32, "wedges_compact: vertex bits in (0, 32]");
  wedge_tile_groups(wscan, ngw, w0, nwedge, tg, s);
  hipLaunchKernelGGL(k_wedges<1>, dim3((unsigned)wedge_tiles(nwedge)), dim3(NT), 0, s, seg, gidx, wscan, tg, nb,
                     centre, w0, nwedge, out_key, (void*)out_centre, vb);
  MRH_CHECK_LAUNCH();
}

size_t pr_scratch_bytes(int64_t nval) { return dev::segred_carry_entries(nval) * (sizeof(int64_t) + sizeof(float)) + 64; }

void pr_contrib(const int64_t* seg, int64_t nseg, int64_t nedge, const int32_t* src, const float* w, const float* r,
                float* out, void* scratch, hipStream_t s) {
  size_t nc = dev::segred_carry_entries(nedge);
  int64_t* cs = reinterpret_cast<int64_t*>(scratch);
  float* cv = reinterpret_cast<float*>(reinterpret_cast<char*>(scratch) + nc * sizeof(int64_t));
  if (w)
    dev::segred_launch<float, 0>(ContribGet{src, w, r}, seg, nseg, nedge, out, cs, cv, s);
  else
    dev::segred_launch<float, 0>(ContribGetC{src, r}, seg, nseg, nedge, out, cs, cv, s);
}

void pr_combine(const int64_t* seg, int64_t ngrp, int64_t nrecv, const int32_t* perm, const float* recv,
                const int32_t* vid, float* grp, float* acc, void* scratch, hipStream_t s) {
  size_t nc = dev::segred_carry_entries(nrecv);
  int64_t* cs = reinterpret_cast<int64_t*>(scratch);
  float* cv = reinterpret_cast<float*>(reinterpret_cast<char*>(scratch) + nc * sizeof(int64_t));
  dev::segred_launch<float, 0>(PermGet{perm, recv}, seg, ngrp, nrecv, grp, cs, cv, s);
  if (ngrp > 0)
    hipLaunchKernelGGL(k_scatter_f32, dim3((unsigned)((ngrp + NT - 1) / NT)), dim3(NT), 0, s, grp, vid, ngrp, acc);
  MRH_CHECK_LAUNCH();
}

void scatter_f32(const float* v, const int32_t* idx, int64_t n, float* out, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_scatter_f32, dim3((unsigned)((n + NT - 1) / NT)), dim3(NT), 0, s, v, idx, n, out);
  MRH_CHECK_LAUNCH();
}

static unsigned pr_grid(int64_t n) {
  const int64_t b = (n + NT - 1) / NT;
  return (unsigned)(b < 1 ? 1 : b);
}
static unsigned pr_grid_stride(int64_t n) {
  const int64_t b = (n + NT - 1) / NT;
  return (unsigned)(b < 1 ? 1 : (b > 65536 ? 65536 : b));
}

void pr_pack_src(const int64_t* e, int64_t n, int P, bool swap, uint64_t* out, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_pr_pack_src, dim3(pr_grid_stride(n)), dim3(NT), 0, s, e, n, P, swap ? 1 : 0, out);
  MRH_CHECK_LAUNCH();
}
void pr_heads(const uint64_t* sorted, int64_t n, uint32_t* flags, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_pr_heads, dim3(pr_grid(n)), dim3(NT), 0, s, sorted, n, flags);
  MRH_CHECK_LAUNCH();
}
void pr_run_degree(const uint64_t* sorted, const int64_t* seg, int64_t nrun, uint32_t* deg, hipStream_t s) {
  if (nrun <= 0) return;
  hipLaunchKernelGGL(k_pr_run_degree, dim3(pr_grid(nrun)), dim3(NT), 0, s, sorted, seg, nrun, deg);
  MRH_CHECK_LAUNCH();
}
void pr_degkey(const uint32_t* deg, int64_t n, uint64_t* key, uint32_t* iota, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_pr_degkey, dim3(pr_grid(n)), dim3(NT), 0, s, deg, n, key, iota);
  MRH_CHECK_LAUNCH();
}
void pr_relabel(const uint32_t* order, const uint32_t* deg, int64_t n, int32_t* nid, int64_t* order64,
                uint8_t* dangling, float* invdeg, unsigned long long* ndangling, int32_t* degn, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_pr_relabel, dim3(pr_grid(n)), dim3(NT), 0, s, order, deg, n, nid, order64, dangling, invdeg,
                     ndangling, degn);
  MRH_CHECK_LAUNCH();
}
void sample_i64(const int64_t* in, int64_t n, int64_t stride, int64_t ns, int64_t* out, hipStream_t s) {
  if (ns <= 0 || n <= 0) return;
  hipLaunchKernelGGL(k_sample_i64, dim3(pr_grid(ns)), dim3(NT), 0, s, in, n, stride, ns, out);
  MRH_CHECK_LAUNCH();
}
void pr_pack(const uint64_t* su, int64_t n, int P, int64_t nlmax, bool local, bool swapped, const int32_t* nid,
             const int32_t* rb, int nr, int dbits, uint64_t* out, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_pr_pack, dim3(pr_grid_stride(n)), dim3(NT), 0, s, su, n, P, nlmax, local ? 1 : 0,
                     swapped ? 1 : 0, nid, rb, nr, dbits, out);
  MRH_CHECK_LAUNCH();
}
void pr_mix_pack(const int64_t* e, int64_t n, int P, int64_t N, bool mix, uint64_t* out, int32_t* dest, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_pr_mix_pack, dim3(pr_grid_stride(n)), dim3(NT), 0, s, e, n, P, N, dev::vmix_bits(N), mix ? 1 : 0,
                     out, dest);
  MRH_CHECK_LAUNCH();
}
void pr_localize(uint64_t* p, int64_t n, int P, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_pr_localize, dim3(pr_grid_stride(n)), dim3(NT), 0, s, p, n, P);
  MRH_CHECK_LAUNCH();
}
void pr_pack_dst(const uint64_t* su, int64_t n, int P, int64_t base, const int32_t* nid, uint64_t* out, int32_t* dest,
                 hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_pr_pack_dst, dim3(pr_grid_stride(n)), dim3(NT), 0, s, su, n, P, base, nid, out, dest);
  MRH_CHECK_LAUNCH();
}
void pr_pack_gather(const uint64_t* in, int64_t n, int P, int64_t S, const int32_t* nid, const int32_t* rb, int nr,
                    int dbits, uint64_t* out, hipStream_t s) {
  if (n <= 0) return;
  check_arg(S > 0 && P * S < (int64_t(1) << 31), "pr_pack_gather: 0 < P * S < 2^31");
  hipLaunchKernelGGL(k_pr_pack_gather, dim3(pr_grid_stride(n)), dim3(NT), 0, s, in, n, P, S, nid, rb, nr, dbits, out);
  MRH_CHECK_LAUNCH();
}
void pr_unmix_ids(const int64_t* order, int64_t n, int P, int me, int64_t N, bool mix, int64_t* ids, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_pr_unmix_ids, dim3(pr_grid(n)), dim3(NT), 0, s, order, n, P, me, N, dev::vmix_bits(N),
                     mix ? 1 : 0, ids);
  MRH_CHECK_LAUNCH();
}
void pr_unpack(const uint64_t* sorted, int64_t n, int32_t* src, uint32_t* flags, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_pr_unpack, dim3(pr_grid(n)), dim3(NT), 0, s, sorted, n, src, flags);
  MRH_CHECK_LAUNCH();
}
void pr_deg_window(const uint64_t* e, int64_t m, int shift, uint32_t* deg, hipStream_t s) {
  if (m <= 0) return;
  hipLaunchKernelGGL(k_pr_deg_window, dim3((unsigned)((m + DW_TILE - 1) / DW_TILE)), dim3(NT), 0, s, e, m, shift, deg);
  MRH_CHECK_LAUNCH();
}
void pr_unpack_bits(const uint64_t* sorted, int64_t n, int32_t* src, uint32_t* H, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_pr_unpack_bits, dim3(pr_grid(n)), dim3(NT), 0, s, sorted, n, src, reinterpret_cast<uint2*>(H));
  MRH_CHECK_LAUNCH();
}
void pr_group_hi(const uint64_t* sorted, const int64_t* seg, int64_t ngrp, int64_t* hi, hipStream_t s) {
  if (ngrp <= 0) return;
  hipLaunchKernelGGL(k_pr_group_hi, dim3(pr_grid(ngrp)), dim3(NT), 0, s, sorted, seg, ngrp, hi);
  MRH_CHECK_LAUNCH();
}
void pr_group_vid(const int64_t* hi, int64_t ngrp, const int32_t* nid, int64_t dmask, int32_t* vid, hipStream_t s) {
  if (ngrp <= 0) return;
  hipLaunchKernelGGL(k_pr_group_vid, dim3(pr_grid(ngrp)), dim3(NT), 0, s, hi, ngrp, nid, dmask, vid);
  MRH_CHECK_LAUNCH();
}
int pr_tile_bits() { return PR_TILE_BITS; }
void pr_range_offsets(const int64_t* hi, int64_t ngrp, int dbits, int R, int64_t ntile, int64_t* off, hipStream_t s) {
  const int64_t n = (int64_t)R * (ntile + 1);
  if (n <= 0) return;
  hipLaunchKernelGGL(k_pr_range_offsets, dim3(pr_grid(n)), dim3(NT), 0, s, hi, ngrp, dbits, R, ntile, PR_TILE_BITS,
                     off);
  MRH_CHECK_LAUNCH();
}
void pr_tile_step(const float* send, const int32_t* ghi, const int64_t* off, int R, int64_t ntile, int64_t ndst,
                  const float* r, float* rn, const uint8_t* dangling, float base, float alpha, const double* dmass,
                  double invN, const float* invdeg, float* cout, double* partial, hipStream_t s) {
  if (ntile <= 0) return;
  check_arg(R >= 1 && R <= PR_MAX_RANGES, "pr_tile_step: 1 <= R <= 64 source ranges");
  check_arg(ntile == (ndst + (1 << PR_TILE_BITS) - 1) >> PR_TILE_BITS, "pr_tile_step: ntile must cover ndst");
  check_arg(((uintptr_t)r | (uintptr_t)rn | (uintptr_t)invdeg | (uintptr_t)cout) % 16 == 0 && (uintptr_t)dangling % 4 == 0,
            "pr_tile_step: 16-byte aligned float columns, 4-byte aligned dangling flags");
  hipLaunchKernelGGL(k_pr_tile_step, dim3((unsigned)ntile), dim3(NT), 0, s, send, ghi, off, R, ntile, ndst, r, rn,
                     dangling, base, alpha, dmass, invN, invdeg, cout, partial);
  MRH_CHECK_LAUNCH();
}

void pr_partials_sum(const double* part, int64_t ntile, double* stats, hipStream_t s) {
  hipLaunchKernelGGL(k_pr_partials_sum, dim3(1), dim3(NT), 0, s, part, ntile, stats);
  MRH_CHECK_LAUNCH();
}

int pr_update_blocks(int64_t n) {
  int64_t b = (n / 4 + NT - 1) / NT;
  return (int)(b < 4096 ? (b < 1 ? 1 : b) : 4096);
}

void pr_update(float* acc, const float* r, float* rn, const uint8_t* dangling, int64_t n, float base,
               float alpha, const double* dmass, double invN, const float* invdeg, float* cout, double* partial,
               hipStream_t s) {
  hipLaunchKernelGGL(k_pr_update, dim3(pr_update_blocks(n)), dim3(NT), 0, s, acc, r, rn, dangling, n, base, alpha,
                     dmass, invN, invdeg, cout, partial);
  MRH_CHECK_LAUNCH();
}

}  // namespace k
}  // namespace mrh
