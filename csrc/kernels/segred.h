// Load-balanced, deterministic segmented reduction (device template).
//
// out[s] = OP over i in [seg[s], seg[s+1]) of get(i)
//
// Work is split by VALUES, not by segments: block b owns values
// [b*TILE, (b+1)*TILE) whatever the segment lengths, so a 3M-value R-MAT hub
// and a million 1-value segments cost the same per value (SURVEY §7.5 skew).
//   pass 1 (k_segred_tiles): each thread reduces IT consecutive values; runs
//     that are complete inside the thread are written directly; incomplete
//     head/tail partials go to an LDS list in thread order, which the block
//     folds per segment; segments complete inside the block are written, the
//     block's first/last partial go to a carry array (2 per block);
//   pass 2 (k_segred_carry): per segment crossing block boundaries, carries
//     are folded in block order.
// Every fold happens in a fixed order, so results are bitwise reproducible.
// Segments must be non-empty (true for every KMV and CSR built by the engine).
#pragma once
#include "common.h"

namespace mrh {
namespace dev {

constexpr int SR_NT = 256;
constexpr int SR_IT = 16;
constexpr int SR_TILE = SR_NT * SR_IT;

template <typename T, int OP>
struct RedOp;
template <typename T>
struct RedOp<T, 0> {
  __device__ static T ident() { return T(0); }
  __device__ static T f(T a, T b) { return a + b; }
};
template <typename T>
struct RedOp<T, 1> {
  __device__ static T ident();
  __device__ static T f(T a, T b) { return b < a ? b : a; }
};
template <typename T>
struct RedOp<T, 2> {
  __device__ static T ident();
  __device__ static T f(T a, T b) { return b > a ? b : a; }
};
template <> __device__ inline int32_t RedOp<int32_t, 1>::ident() { return 0x7fffffff; }
template <> __device__ inline int32_t RedOp<int32_t, 2>::ident() { return (int32_t)0x80000000; }
template <> __device__ inline int64_t RedOp<int64_t, 1>::ident() { return 0x7fffffffffffffffll; }
template <> __device__ inline int64_t RedOp<int64_t, 2>::ident() { return (int64_t)0x8000000000000000ull; }
template <> __device__ inline float RedOp<float, 1>::ident() { return __builtin_huge_valf(); }
template <> __device__ inline float RedOp<float, 2>::ident() { return -__builtin_huge_valf(); }
template <> __device__ inline double RedOp<double, 1>::ident() { return __builtin_huge_val(); }
template <> __device__ inline double RedOp<double, 2>::ident() { return -__builtin_huge_val(); }

// largest s in [0, nseg) with seg[s] <= i
__device__ __forceinline__ int64_t seg_upper(const int64_t* __restrict__ seg, int64_t nseg, int64_t i) {
  int64_t lo = 0, hi = nseg - 1;
  while (lo < hi) {
    int64_t mid = (lo + hi + 1) >> 1;
    if (seg[mid] <= i) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// Block layout: values are fetched STRIPED (value b0 + j*NT + t by thread t:
// coalesced index loads, 16 independent gathers in flight per thread) into
// LDS, then reduced BLOCKED (IT consecutive values per thread). The segment
// boundaries overlapping the block are staged in LDS once (two global binary
// searches per block instead of one per thread).
__device__ __forceinline__ int lpad(int i) { return i + (i >> 4); }

template <typename T, int OP, typename G>
__global__ __launch_bounds__(SR_NT) void k_segred_tiles(G get, const int64_t* __restrict__ seg, int64_t nseg,
                                                        int64_t nval, T* __restrict__ out,
                                                        int64_t* __restrict__ carry_seg, T* __restrict__ carry_val) {
  using R = RedOp<T, OP>;
  // segment bounds relative to b0, clamped to [-1, TILE + 1] (int32: half
  // the LDS of absolute offsets, so more blocks fit a CU); values padded one
  // slot per 16 so the blocked reads (16 consecutive per thread) spread over
  // the banks
  __shared__ int32_t lseg[SR_TILE + 2];
  __shared__ T lval[SR_TILE + SR_TILE / 16];
  __shared__ int64_t ls[2 * SR_NT];
  __shared__ T lv[2 * SR_NT];
  __shared__ int64_t eseg[2 * (2 * SR_NT / 64)];  // the 8 chunks' first / last runs
  __shared__ T eval[2 * (2 * SR_NT / 64)];
  __shared__ int64_t sb_sh, ns_sh;
  const int t = threadIdx.x;
  const int64_t b0 = (int64_t)blockIdx.x * SR_TILE;
  const int64_t b1 = min(b0 + (int64_t)SR_TILE, nval);
  if (t == 0) {
    int64_t sb = seg_upper(seg, nseg, b0);
    int64_t se = seg_upper(seg, nseg, b1 - 1);
    sb_sh = sb;
    ns_sh = se - sb + 1;  // segments overlapping the block
  }
  // striped fetch of the block's values
  T v[SR_IT];
#pragma unroll
  for (int j = 0; j < SR_IT; ++j) {
    int64_t e = b0 + (int64_t)j * SR_NT + t;
    v[j] = e < b1 ? get(e) : R::ident();
  }
#pragma unroll
  for (int j = 0; j < SR_IT; ++j) lval[lpad(j * SR_NT + t)] = v[j];
  __syncthreads();
  const int64_t sb = sb_sh, ns = ns_sh;
  if (ns == 1) {
    // the whole tile lies in one segment (a hot key's values): a block
    // reduction of the registers in a fixed order, no partial lists — the
    // general path below folds 2 x 256 partials serially in one thread
    __shared__ T wred[SR_NT / 64];
    T acc = v[0];
#pragma unroll
    for (int j = 1; j < SR_IT; ++j) acc = R::f(acc, v[j]);
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) acc = R::f(acc, __shfl_xor(acc, d, 64));
    if ((t & 63) == 0) wred[t >> 6] = acc;
    __syncthreads();
    if (t == 0) {
      T a = wred[0];
#pragma unroll
      for (int w = 1; w < SR_NT / 64; ++w) a = R::f(a, wred[w]);
      const int64_t s0 = seg[sb], s1 = seg[sb + 1];
      if (s0 >= b0 && s1 <= b1) {
        out[sb] = a;
      } else {
        const int slot = s0 < b0 ? 0 : 1;
        carry_seg[2 * blockIdx.x + slot] = sb;
        carry_val[2 * blockIdx.x + slot] = a;
      }
    }
    return;
  }
  for (int64_t j = t; j <= ns; j += SR_NT) {
    const int64_t r = seg[sb + j] - b0;
    lseg[j] = (int32_t)(r < 0 ? -1 : r > SR_TILE ? SR_TILE + 1 : r);
  }
  ls[2 * t] = -1;
  ls[2 * t + 1] = -1;
  if (t < 2 * (2 * SR_NT / 64)) eseg[t] = -1;
  __syncthreads();

  // thread range [t0, t1) relative to b0
  const int32_t t0 = t * SR_IT;
  const int32_t t1 = (int32_t)min((int64_t)t0 + SR_IT, b1 - b0);
  if (t0 < t1) {
    // local segment of t0: largest q in [0, ns) with lseg[q] <= t0
    int64_t lo = 0, hi = ns - 1;
    while (lo < hi) {
      int64_t mid = (lo + hi + 1) >> 1;
      if (lseg[mid] <= t0) lo = mid;
      else hi = mid - 1;
    }
    int64_t q = lo;
    int32_t s_end = lseg[q + 1];
    T acc = R::ident();
    bool first_run = true;
    for (int32_t i = t0; i < t1; ++i) {
      while (i >= s_end) {  // close run of segment sb+q
        if (lseg[q] >= t0) out[sb + q] = acc;  // started inside the thread: complete
        else { ls[2 * t] = sb + q; lv[2 * t] = acc; }
        first_run = false;
        ++q;
        s_end = lseg[q + 1];
        acc = R::ident();
      }
      acc = R::f(acc, lval[lpad(i)]);
    }
    // last run of the thread ends at t1
    const bool starts_inside = lseg[q] >= t0;
    const bool ends_inside = s_end <= t1;
    if (starts_inside && ends_inside) {
      out[sb + q] = acc;
    } else if (!starts_inside && first_run) {
      ls[2 * t] = sb + q;  // one run covering the whole thread range
      lv[2 * t] = acc;
    } else {
      ls[2 * t + 1] = sb + q;
      lv[2 * t + 1] = acc;
    }
  }
  __syncthreads();
  // fold the incomplete partials per segment: the 2 x 256 entries (thread
  // order, segment ids non-decreasing, -1 = none) in 8 chunks of 64, two per
  // wave, by a segmented wave scan; a run inside a chunk is the segment's
  // whole block total; each chunk's first and last runs (which may continue
  // in the neighbouring chunk) go to 16 edge slots that thread 0 folds in
  // order. (A serial fold of up to 512 entries in one thread made a tile
  // holding a segment boundary cost ~10x an interior one.)
  auto finish = [&](int64_t s, T acc) {
    const int64_t s0 = seg[s], s1 = seg[s + 1];
    if (s0 >= b0 && s1 <= b1) {
      out[s] = acc;
    } else {  // the block's first partial (segment started before b0) -> slot 0, else slot 1
      const int slot = s0 < b0 ? 0 : 1;
      carry_seg[2 * blockIdx.x + slot] = s;
      carry_val[2 * blockIdx.x + slot] = acc;
    }
  };
  const int lane = t & 63;
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    const int j = t + pass * SR_NT, c = j >> 6;
    int64_t sj = ls[j];
    T v = sj >= 0 ? lv[j] : R::ident();
    const uint64_t valid = __ballot(sj >= 0);
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {  // invalid entries join the run before them
      const int64_t y = __shfl_up(sj, d, 64);
      if (lane >= d && y > sj) sj = y;
    }
    const int64_t sp = __shfl_up(sj, 1, 64), sn = __shfl_down(sj, 1, 64);
    const bool head = lane == 0 || sj != sp;
    const uint64_t heads = __ballot(head);
    T S = v;
    int F = head;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const T ys = __shfl_up(S, d, 64);
      const int yf = __shfl_up(F, d, 64);
      if (lane >= d) {
        if (!F) S = R::f(ys, S);
        F |= yf;
      }
    }
    const bool tail = lane == 63 || sj != sn;
    if (tail && sj >= 0) {
      const int fv = __ffsll((long long)valid) - 1;
      const uint64_t upto = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);
      const uint64_t after_fv = ~((2ull << fv) - 1ull);
      const bool first = (heads & upto & after_fv) == 0ull;
      if (first || lane == 63) {
        eseg[2 * c + (first ? 0 : 1)] = sj;
        eval[2 * c + (first ? 0 : 1)] = S;
      } else {
        finish(sj, S);
      }
    }
  }
  __syncthreads();
  if (t == 0) {
    int64_t cur = -1;
    T acc = R::ident();
    for (int e = 0; e < 2 * (2 * SR_NT / 64); ++e) {
      const int64_t se = eseg[e];
      if (se < 0) continue;
      if (se != cur) {
        if (cur >= 0) finish(cur, acc);
        cur = se;
        acc = eval[e];
      } else {
        acc = R::f(acc, eval[e]);
      }
    }
    if (cur >= 0) finish(cur, acc);
  }
}

template <typename T, int OP>
__global__ __launch_bounds__(SR_NT) void k_segred_carry(const int64_t* __restrict__ carry_seg,
                                                        const T* __restrict__ carry_val, int64_t ncarry,
                                                        T* __restrict__ out) {
  using R = RedOp<T, OP>;
  int64_t j = (int64_t)blockIdx.x * SR_NT + threadIdx.x;
  if (j >= ncarry) return;
  int64_t s = carry_seg[j];
  if (s < 0) return;
  int64_t jp = j - 1;
  while (jp >= 0 && carry_seg[jp] < 0) --jp;
  if (jp >= 0 && carry_seg[jp] == s) return;
  T acc = carry_val[j];
  for (int64_t k = j + 1; k < ncarry; ++k) {
    int64_t sk = carry_seg[k];
    if (sk < 0) continue;
    if (sk != s) break;
    acc = R::f(acc, carry_val[k]);
  }
  out[s] = acc;
}

// Two-level carry fold for long carry arrays (k_segred_carry folds a run of
// equal segment ids serially in one thread, so one segment spanning
// thousands of tiles — an R-MAT hub's in-edges — serialises the launch).
// Level 1: one wave per 64 carry entries; invalid (-1) entries join the run
// before them with the identity (valid ids are non-decreasing); a segmented
// wave scan reduces every run in entry order; runs that start and end inside
// the wave are final, the wave's first and last runs go to slots 0 / 1 of
// the level-2 carry (cs2 = -1 initialised), which k_segred_carry folds.
// The fold order is fixed: results are bitwise reproducible.
template <typename T, int OP>
__global__ __launch_bounds__(256) void k_carry_fold(const int64_t* __restrict__ cs, const T* __restrict__ cv,
                                                   int64_t nc, T* __restrict__ out, int64_t* __restrict__ cs2,
                                                   T* __restrict__ cv2) {
  using R = RedOp<T, OP>;
  const int lane = threadIdx.x & 63;
  const int64_t wv = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  const int64_t j = wv * 64 + lane;
  int64_t s = -1;
  T v = R::ident();
  if (j < nc) {
    s = cs[j];
    if (s >= 0) v = cv[j];
  }
  const uint64_t valid = __ballot(s >= 0);
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int64_t y = __shfl_up(s, d, 64);
    if (lane >= d && y > s) s = y;
  }
  const int64_t sp = __shfl_up(s, 1, 64), sn = __shfl_down(s, 1, 64);
  const bool head = lane == 0 || s != sp;
  const uint64_t heads = __ballot(head);
  T S = v;
  int F = head;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const T ys = __shfl_up(S, d, 64);
    const int yf = __shfl_up(F, d, 64);
    if (lane >= d) {
      if (!F) S = R::f(ys, S);
      F |= yf;
    }
  }
  const bool tail = lane == 63 || s != sn;
  if (!tail || s < 0) return;
  // the wave's first run is the one holding its first valid entry fv (it may
  // continue a run of the previous wave across invalid entries): no head in
  // lanes (fv, lane]; the last run reaches lane 63
  const int fv = __ffsll((long long)valid) - 1;  // valid != 0: a tail with s >= 0 exists
  const uint64_t upto = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);
  const uint64_t after_fv = ~((2ull << fv) - 1ull);
  const bool first = (heads & upto & after_fv) == 0ull;
  const bool last = lane == 63;
  if (first || last) {
    const int slot = first ? 0 : 1;
    cs2[2 * wv + slot] = s;
    cv2[2 * wv + slot] = S;
  } else {
    out[s] = S;
  }
}

// host launcher: carry buffers need 2*nblocks entries each
template <typename T, int OP, typename G>
inline void segred_launch(G get, const int64_t* seg, int64_t nseg, int64_t nval, T* out, int64_t* carry_seg,
                          T* carry_val, hipStream_t s) {
  if (nseg <= 0 || nval <= 0) return;
  int64_t nb = (nval + SR_TILE - 1) / SR_TILE;
  MRH_HIP(hipMemsetAsync(carry_seg, 0xff, sizeof(int64_t) * 2 * nb, s));  // -1
  hipLaunchKernelGGL((k_segred_tiles<T, OP, G>), dim3((unsigned)nb), dim3(SR_NT), 0, s, get, seg, nseg, nval, out,
                     carry_seg, carry_val);
  MRH_CHECK_LAUNCH();
  // carries folded in levels of k_carry_fold (64 entries per wave) until at
  // most 64 are left for k_segred_carry's serial fold: one hot segment over
  // thousands of tiles is never folded entry by entry in one thread
  int64_t nc = 2 * nb;
  int64_t* cs = carry_seg;
  T* cv = carry_val;
  while (nc > 64) {
    const int64_t nw1 = (nc + 63) / 64;
    int64_t* cs2 = cs + nc;  // the next level sits behind this one (segred_carry_entries)
    T* cv2 = cv + nc;
    MRH_HIP(hipMemsetAsync(cs2, 0xff, sizeof(int64_t) * 2 * nw1, s));
    hipLaunchKernelGGL((k_carry_fold<T, OP>), dim3((unsigned)((nc + 255) / 256)), dim3(256), 0, s, cs, cv, nc, out,
                       cs2, cv2);
    MRH_CHECK_LAUNCH();
    cs = cs2;
    cv = cv2;
    nc = 2 * nw1;
  }
  hipLaunchKernelGGL((k_segred_carry<T, OP>), dim3((unsigned)((nc + SR_NT - 1) / SR_NT)), dim3(SR_NT), 0, s, cs, cv,
                     nc, out);
  MRH_CHECK_LAUNCH();
}

// carry entries a segred_launch needs per array: 2 per tile, plus every
// further level of the carry fold (2 per 64 entries of the level before)
inline size_t segred_carry_entries(int64_t nval) {
  size_t nc = 2 * (size_t)((nval + SR_TILE - 1) / SR_TILE), total = nc;
  while (nc > 64) {
    nc = 2 * ((nc + 63) / 64);
    total += nc;
  }
  return total + 2;
}

}  // namespace dev
}  // namespace mrh
