// Static-segment gather-reduce for iterated plans (PageRank, CC, SSSP, Luby):
//
//     out[s] = OP over e in [seg[s], seg[s+1]) of  x[src[e]] (+ w[e])
//
// The segments never change between iterations, so instead of searching the
// segment array every launch (segred.h) the plan precomputes, once,
//   * a head bitmap H (bit e set <=> an edge e starts a segment), and
//   * wbase[w] = number of segments starting before wave w's first edge.
// Each wave64 owns WS_TILE = 64 x WS_IT consecutive edges; lane l owns WS_IT
// consecutive edges, loads their source ids with 16-byte vector loads and
// issues WS_IT independent gathers at once. Runs are reduced in registers;
// partial runs crossing lanes are joined by a 6-step segmented shuffle scan;
// runs crossing waves go to a 2-slot carry per wave folded by
// k_segred_carry (segred.h). No LDS and no barriers: occupancy is bounded only
// by VGPRs, which is what a latency-bound random gather needs (the LDS-staged
// segred kernel ran at 2 waves/SIMD). Every fold has a fixed order, so the
// result is bitwise reproducible.
#pragma once
#include "common.h"
#include "segred.h"

namespace mrh {
namespace dev {

constexpr int WS_IT = 16;
constexpr int WS_TILE = 64 * WS_IT;
constexpr int WS_NT = 256;

typedef int v4i32 __attribute__((ext_vector_type(4)));

// bits for segment heads; H must be zeroed and hold ws_head_words(nval) words
__global__ __launch_bounds__(256) inline void k_ws_heads(const int64_t* __restrict__ seg, int64_t nseg,
                                                         uint32_t* __restrict__ H) {
  int64_t s = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (s < nseg) {
    int64_t e = seg[s];
    atomicOr(&H[e >> 5], 1u << (e & 31));
  }
}

__global__ __launch_bounds__(256) inline void k_ws_base(const int64_t* __restrict__ seg, int64_t nseg, int64_t nwave,
                                                        int64_t* __restrict__ wbase) {
  int64_t w = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (w >= nwave) return;
  const int64_t e0 = w * WS_TILE;
  int64_t lo = 0, hi = nseg;  // first s with seg[s] >= e0
  while (lo < hi) {
    int64_t mid = (lo + hi) >> 1;
    if (seg[mid] < e0) lo = mid + 1;
    else hi = mid;
  }
  wbase[w] = lo;
}

inline int64_t ws_nwave(int64_t nval) { return (nval + WS_TILE - 1) / WS_TILE; }
inline int64_t ws_head_words(int64_t nval) { return ws_nwave(nval) * (WS_TILE / 32) + 2; }

// gathers of x[src]: straight from memory, or — the hot-prefix kernel — the
// hottest sources (ids [0, hn): the degree-sorted new ids put them first)
// from an LDS copy
template <typename T>
struct GatherMem {
  const T* __restrict__ x;
  __device__ __forceinline__ T operator()(int32_t id) const { return x[id]; }
};
template <typename T>
struct GatherHot {
  const T* __restrict__ x;
  const T* xs;  // LDS copy of x[0, hn)
  int32_t hn;
  __device__ __forceinline__ T operator()(int32_t id) const { return (uint32_t)id < (uint32_t)hn ? xs[id] : x[id]; }
};

// one wave's tile of WS_TILE edges (wave-uniform wv)
template <typename T, int OP, typename G>
__device__ __forceinline__ void ws_tile(int64_t wv, const uint32_t* __restrict__ H, const int64_t* __restrict__ wbase,
                                        int64_t nval, const int32_t* __restrict__ src, const G& gx,
                                        const T* __restrict__ w, T* __restrict__ out, int64_t* __restrict__ carry_seg,
                                        T* __restrict__ carry_val) {
  using R = RedOp<T, OP>;
  const int lane = threadIdx.x & 63;
  const int64_t E0 = wv * WS_TILE;
  const int64_t L0 = E0 + (int64_t)lane * WS_IT;
  const int64_t nv = nval - L0;  // valid edges of this lane (may be <= 0)

  uint32_t f = (__builtin_nontemporal_load(H + (L0 >> 5)) >> (L0 & 31)) & 0xffffu;
  T v[WS_IT];
  if (nv >= WS_IT) {
    const v4i32* p = reinterpret_cast<const v4i32*>(src + L0);
#pragma unroll
    for (int q = 0; q < WS_IT / 4; ++q) {
      v4i32 id = __builtin_nontemporal_load(p + q);
      v[4 * q + 0] = gx(id.x);
      v[4 * q + 1] = gx(id.y);
      v[4 * q + 2] = gx(id.z);
      v[4 * q + 3] = gx(id.w);
    }
    if (w) {
#pragma unroll
      for (int j = 0; j < WS_IT; ++j) v[j] = v[j] + w[L0 + j];
    }
  } else {
    f = nv > 0 ? (f & ((1u << nv) - 1u)) : 0u;
#pragma unroll
    for (int j = 0; j < WS_IT; ++j) {
      if (j < nv) {
        T a = gx(src[L0 + j]);
        v[j] = w ? a + w[L0 + j] : a;
      } else {
        v[j] = R::ident();
      }
    }
  }
  // heads before this lane (wave exclusive prefix of popcounts)
  const int cnt = __popc(f);
  int incl = cnt;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    int y = __shfl_up(incl, d, 64);
    if (lane >= d) incl += y;
  }
  const int pre = incl - cnt;
  const int64_t base = wbase[wv];
  // sid(edge) = base + #heads in [E0, edge] - 1
  int64_t sid = base + pre + (int)(f & 1u) - 1;
  T acc = R::ident(), headpart = R::ident();
  bool first = true;
#pragma unroll
  for (int j = 0; j < WS_IT; ++j) {
    if (j > 0 && ((f >> j) & 1u)) {
      if (first && !(f & 1u)) headpart = acc;  // first run began before this lane
      else out[sid] = acc;                     // run began and ended inside the lane
      first = false;
      ++sid;
      acc = R::ident();
    }
    acc = R::f(acc, v[j]);
  }
  // segmented inclusive scan of the tail runs across lanes
  T S = acc;
  int F = f != 0u;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    T ys = __shfl_up(S, d, 64);
    int yf = __shfl_up(F, d, 64);
    if (lane >= d) {
      if (!F) S = R::f(ys, S);
      F |= yf;
    }
  }
  T Sprev = __shfl_up(S, 1, 64);
  if (lane == 0) Sprev = R::ident();
  // a lane holding a head closes the run containing edge L0-1
  if (f != 0u && nv > 0 && (lane > 0 || !(f & 1u))) {
    const T tot = R::f(Sprev, headpart);
    if (pre == 0) {  // that run began before the wave: cross-wave partial
      carry_seg[2 * wv] = base - 1;
      carry_val[2 * wv] = tot;
    } else {
      out[base + pre - 1] = tot;
    }
  }
  if (lane == 63) {
    const int total_heads = incl;
    const int64_t E1 = E0 + WS_TILE;
    const bool complete = E1 >= nval || ((H[E1 >> 5] >> (E1 & 31)) & 1u);
    const int64_t s_last = base + total_heads - 1;
    if (total_heads == 0) {
      carry_seg[2 * wv] = s_last;
      carry_val[2 * wv] = S;
    } else if (complete) {
      out[s_last] = S;
    } else {
      carry_seg[2 * wv + 1] = s_last;
      carry_val[2 * wv + 1] = S;
    }
  }
}

template <typename T, int OP>
__global__ __launch_bounds__(WS_NT) void k_ws_gather_reduce(const uint32_t* __restrict__ H,
                                                            const int64_t* __restrict__ wbase, int64_t nval,
                                                            int64_t nwave, const int32_t* __restrict__ src,
                                                            const T* __restrict__ x, const T* __restrict__ w,
                                                            T* __restrict__ out, int64_t* __restrict__ carry_seg,
                                                            T* __restrict__ carry_val,
                                                            const int32_t* __restrict__ sched, int64_t slen) {
  int64_t wv = (int64_t)blockIdx.x * (WS_NT / 64) + (threadIdx.x >> 6);
  if (sched) {
    // XCD-pinned schedule: blocks b and b + 8 run on one XCD, so slot b % 8
    // walks row b % 8 of the schedule (its own source ranges: their slice of
    // x stays in that XCD's L2)
    const int64_t lw = (int64_t)(blockIdx.x >> 3) * (WS_NT / 64) + (threadIdx.x >> 6);
    if (lw >= slen) return;
    wv = sched[(int64_t)(blockIdx.x & 7) * slen + lw];
    if (wv < 0) return;
  }
  if (wv >= nwave) return;  // uniform per wave
  ws_tile<T, OP>(wv, H, wbase, nval, src, GatherMem<T>{x}, w, out, carry_seg, carry_val);
}

// Hot-prefix variant: persistent blocks (WSH_NT threads, one per CU) stage
// x[0, hn) — the hottest sources, degree-sorted first — in LDS once and walk
// their XCD slot's schedule row (or every tile, without a schedule): gathers
// of hot sources are LDS reads, so the L2 serves only the others (the pull
// gather is bound by L2 requests, one per edge). Same per-tile fold order as
// k_ws_gather_reduce: bitwise the same result.
constexpr int WSH_NT = 1024;
template <typename T, int OP>
__global__ __launch_bounds__(WSH_NT) void k_ws_gather_reduce_hot(const uint32_t* __restrict__ H,
                                                                 const int64_t* __restrict__ wbase, int64_t nval,
                                                                 int64_t nwave, const int32_t* __restrict__ src,
                                                                 const T* __restrict__ x, const T* __restrict__ w,
                                                                 T* __restrict__ out, int64_t* __restrict__ carry_seg,
                                                                 T* __restrict__ carry_val,
                                                                 const int32_t* __restrict__ sched, int64_t slen,
                                                                 int32_t hn) {
  extern __shared__ unsigned char ws_smem[];
  T* xs = reinterpret_cast<T*>(ws_smem);
  for (int32_t i = threadIdx.x; i < hn; i += WSH_NT) xs[i] = x[i];
  __syncthreads();
  const GatherHot<T> gx{x, xs, hn};
  constexpr int WPB = WSH_NT / 64;
  const int wave = threadIdx.x >> 6;
  if (sched) {
    const int64_t per_slot = gridDim.x >> 3;  // blocks per XCD slot (grid: a multiple of 8)
    const int64_t j = blockIdx.x >> 3;
    const int32_t* row = sched + (int64_t)(blockIdx.x & 7) * slen;
    for (int64_t lw = j * WPB + wave; lw < slen; lw += per_slot * WPB) {
      const int64_t wv = row[lw];
      if (wv < 0 || wv >= nwave) continue;  // uniform per wave
      ws_tile<T, OP>(wv, H, wbase, nval, src, gx, w, out, carry_seg, carry_val);
    }
  } else {
    for (int64_t wv = (int64_t)blockIdx.x * WPB + wave; wv < nwave; wv += (int64_t)gridDim.x * WPB)
      ws_tile<T, OP>(wv, H, wbase, nval, src, gx, w, out, carry_seg, carry_val);
  }
}

// carry slots reset to -1 by a kernel, not hipMemsetAsync: the gather is
// captured into PageRank's HIP graph, and kernel nodes are the graph node
// type every ROCm release replays as launched
__global__ __launch_bounds__(256) inline void k_ws_fill_neg1(int64_t* __restrict__ p, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) p[i] = -1;
}
inline void ws_fill_neg1(int64_t* p, int64_t n, hipStream_t s) {
  if (n <= 0) return;
  const int64_t b = (n + 255) / 256;
  hipLaunchKernelGGL(k_ws_fill_neg1, dim3((unsigned)(b < 4096 ? b : 4096)), dim3(256), 0, s, p, n);
  MRH_CHECK_LAUNCH();
}

// ids of the hot prefix the persistent kernel keeps in LDS: MRH_PR_HOT (ids,
// at most the 128 KiB of LDS a 1024-thread block holds next to nothing else:
// 32 k floats; -1 = that cap). Off by default: on RMAT-26 it cut the L2
// requests of the gather by only 8% (hot sources already hit in the vL1D) and
// the one-block-per-CU persistent grid ran 6.09 ms against 5.38 ms per
// iteration (profiles/r5_pagerank_hot_prefix.txt)
template <typename T>
inline int64_t ws_hot_ids(int64_t nx) {
  static const int64_t env = [] {
    const char* e = std::getenv("MRH_PR_HOT");
    return e && *e ? (int64_t)std::atoll(e) : (int64_t)0;
  }();
  if (env == 0) return 0;
  const int64_t cap = (int64_t(128) << 10) / (int64_t)sizeof(T);
  const int64_t want = env < 0 ? cap : std::min(env, cap);
  return std::min(want, nx);
}
inline int ws_num_cus() {
  static int cus[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (cus[dev] == 0 && hipDeviceGetAttribute(&cus[dev], hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    cus[dev] = 256;
  return cus[dev];
}

// launcher; carry buffers need 2*ws_nwave(nval) entries each; nx: entries of
// x (0: unknown, no hot-prefix kernel)
template <typename T, int OP>
inline void ws_gather_reduce(const uint32_t* H, const int64_t* wbase, int64_t nval, const int32_t* src, const T* x,
                             const T* w, T* out, int64_t* carry_seg, T* carry_val, hipStream_t s,
                             int64_t* carry2_seg = nullptr, T* carry2_val = nullptr,
                             const int32_t* sched = nullptr, int64_t slen = 0, int64_t nx = 0) {
  if (nval <= 0) return;
  const int64_t nw = ws_nwave(nval);
  ws_fill_neg1(carry_seg, 2 * nw, s);
  const int64_t hot = ws_hot_ids<T>(nx);
  if (hot >= 1024 && nval >= (int64_t(1) << 22)) {
    static bool attr = false;
    const size_t lds = (size_t)hot * sizeof(T);
    if (!attr) {
      MRH_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_ws_gather_reduce_hot<T, OP>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)(int64_t(160) << 10)));
      attr = true;
    }
    const int grid = std::max(8, ws_num_cus() / 8 * 8);  // one block per CU, a multiple of 8 (XCD slots)
    hipLaunchKernelGGL((k_ws_gather_reduce_hot<T, OP>), dim3((unsigned)grid), dim3(WSH_NT), lds, s, H, wbase, nval,
                       nw, src, x, w, out, carry_seg, carry_val, sched, slen, (int32_t)hot);
  } else {
    const int64_t nb = sched ? 8 * ((slen + (WS_NT / 64) - 1) / (WS_NT / 64)) : (nw + (WS_NT / 64) - 1) / (WS_NT / 64);
    hipLaunchKernelGGL((k_ws_gather_reduce<T, OP>), dim3((unsigned)nb), dim3(WS_NT), 0, s, H, wbase, nval, nw, src, x,
                       w, out, carry_seg, carry_val, sched, slen);
  }
  MRH_CHECK_LAUNCH();
  const int64_t nc = 2 * nw;
  if (carry2_seg && nc > 4096) {  // two-level fold (k_carry_fold): long runs in parallel
    const int64_t nw1 = (nc + 63) / 64;
    ws_fill_neg1(carry2_seg, 2 * nw1, s);
    hipLaunchKernelGGL((k_carry_fold<T, OP>), dim3((unsigned)((nc + 255) / 256)), dim3(256), 0, s, carry_seg,
                       carry_val, nc, out, carry2_seg, carry2_val);
    MRH_CHECK_LAUNCH();
    hipLaunchKernelGGL((k_segred_carry<T, OP>), dim3((unsigned)((2 * nw1 + SR_NT - 1) / SR_NT)), dim3(SR_NT), 0, s,
                       carry2_seg, carry2_val, 2 * nw1, out);
    MRH_CHECK_LAUNCH();
    return;
  }
  hipLaunchKernelGGL((k_segred_carry<T, OP>), dim3((unsigned)((nc + SR_NT - 1) / SR_NT)), dim3(SR_NT), 0, s, carry_seg,
                     carry_val, nc, out);
  MRH_CHECK_LAUNCH();
}

}  // namespace dev
}  // namespace mrh
