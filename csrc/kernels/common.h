// Device helpers shared by the CDNA4 kernels: wave64 scans/reductions and
// block-level scans. Everything here assumes a 64-lane wavefront (gfx950).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include "hashfn.h"

#define MRH_WAVE 64

#define MRH_CHECK_LAUNCH()                                                       \
  do {                                                                           \
    hipError_t e__ = hipGetLastError();                                          \
    if (e__ != hipSuccess) {                                                     \
      fprintf(stderr, "mrhip kernel launch failed: %s at %s:%d\n",               \
              hipGetErrorString(e__), __FILE__, __LINE__);                       \
      abort();                                                                   \
    }                                                                            \
  } while (0)

namespace mrh {
namespace dev {

__device__ __forceinline__ int lane_id() { return threadIdx.x & (MRH_WAVE - 1); }
__device__ __forceinline__ int wave_id() { return threadIdx.x / MRH_WAVE; }
__device__ __forceinline__ uint64_t lanemask_lt() {
  return (lane_id() == 0) ? 0ull : (~0ull >> (64 - lane_id()));
}

// inclusive wave scan (64 lanes) via DPP-friendly shfl_up
template <typename T>
__device__ __forceinline__ T wave_incl_scan(T v) {
  const int l = lane_id();
#pragma unroll
  for (int o = 1; o < MRH_WAVE; o <<= 1) {
    T u = __shfl_up(v, o, MRH_WAVE);
    if (l >= o) v += u;
  }
  return v;
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int o = MRH_WAVE / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, MRH_WAVE);
  return v;
}

// Block exclusive scan of one value per thread; returns exclusive prefix,
// writes block total to *total. `sh` needs (blockDim/64 + 1) T entries.
template <typename T, int NT>
__device__ __forceinline__ T block_excl_scan(T v, T* sh, T* total) {
  constexpr int NW = NT / MRH_WAVE;
  const int l = lane_id(), w = wave_id();
  T incl = wave_incl_scan(v);
  if (l == MRH_WAVE - 1) sh[w] = incl;
  __syncthreads();
  if (w == 0) {
    T x = (l < NW) ? sh[l] : T(0);
    T xs = wave_incl_scan(x);
    if (l < NW) sh[l] = xs - x;
    if (l == NW - 1) sh[NW] = xs;
  }
  __syncthreads();
  T res = incl - v + sh[w];
  *total = sh[NW];
  __syncthreads();
  return res;
}

}  // namespace dev
}  // namespace mrh
