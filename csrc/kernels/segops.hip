// Small segment / histogram / compaction kernels that replace ATen library
// kernels (at::searchsorted, at::repeat_interleave, at::bincount,
// at::nonzero -> rocPRIM) on the engine's paths.
//
//  k_seg_marks   marks[seg[s]] += 1 for every segment start s >= 1 inside
//                [0, nval); the inclusive scan of marks is then the segment id
//                of every value (empty segments are counted, so ids match
//                searchsorted(seg, i, right) - 1 exactly);
//  k_histogram   counts[idx[i]]++ with one global atomic per element (for
//                wide histograms; narrow ones use the LDS count_mod kernel);
//  k_compact_nz  indices of the non-zero u64 slots of a hash table, in
//                order, from the exclusive scan of the non-zero flags;
//  k_mask_flags / k_compact_mask  the same for a bool mask (the engine's
//                boolean-mask selections: at::nonzero would run rocPRIM's
//                partition kernel).
#include <algorithm>

#include "common.h"
#include "launch.h"

namespace mrh {
namespace k {
namespace {

constexpr int NT = 256;
inline unsigned blocks(int64_t n) { return (unsigned)std::min<int64_t>((n + NT - 1) / NT, 1 << 20); }

__global__ __launch_bounds__(NT) void k_seg_marks(const int64_t* __restrict__ seg, int64_t nseg, int64_t nval,
                                                 int64_t* __restrict__ marks) {
  for (int64_t s = (int64_t)blockIdx.x * NT + threadIdx.x + 1; s < nseg; s += (int64_t)gridDim.x * NT) {
    const int64_t p = seg[s];
    if (p < nval) atomicAdd((unsigned long long*)&marks[p], 1ull);
  }
}

__global__ __launch_bounds__(NT) void k_histogram(const int64_t* __restrict__ idx, int64_t n, int64_t K,
                                                 int64_t* __restrict__ counts) {
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) {
    const int64_t b = idx[i];
    if (b >= 0 && b < K) atomicAdd((unsigned long long*)&counts[b], 1ull);
  }
}

__global__ __launch_bounds__(NT) void k_nz_flags(const uint64_t* __restrict__ v, int64_t n, int32_t* __restrict__ f) {
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) f[i] = v[i] != 0;
}

__global__ __launch_bounds__(NT) void k_compact_nz(const uint64_t* __restrict__ v, const int64_t* __restrict__ pos,
                                                  int64_t n, int64_t* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT)
    if (v[i]) out[pos[i]] = i;
}

// idx[j] = position of q[j] in the sorted unique keys, or -1
__global__ __launch_bounds__(NT) void k_lookup_sorted(const int64_t* __restrict__ keys, int64_t n,
                                                     const int64_t* __restrict__ q, int64_t m,
                                                     int64_t* __restrict__ idx) {
  for (int64_t j = (int64_t)blockIdx.x * NT + threadIdx.x; j < m; j += (int64_t)gridDim.x * NT) {
    const int64_t x = q[j];
    int64_t lo = 0, hi = n;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (keys[mid] < x) lo = mid + 1;
      else hi = mid;
    }
    idx[j] = (lo < n && keys[lo] == x) ? lo : -1;
  }
}

__global__ __launch_bounds__(NT) void k_mask_flags(const uint8_t* __restrict__ m, int64_t n, int64_t* __restrict__ f) {
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) f[i] = m[i] != 0;
}

__global__ __launch_bounds__(NT) void k_compact_mask(const uint8_t* __restrict__ m, const int64_t* __restrict__ pos,
                                                    int64_t n, int64_t* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT)
    if (m[i]) out[pos[i]] = i;
}

}  // namespace

void mask_flags(const uint8_t* m, int64_t n, int64_t* f, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_mask_flags, dim3(blocks(n)), dim3(NT), 0, s, m, n, f);
  MRH_CHECK_LAUNCH();
}

void compact_mask(const uint8_t* m, const int64_t* pos, int64_t n, int64_t* out, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_compact_mask, dim3(blocks(n)), dim3(NT), 0, s, m, pos, n, out);
  MRH_CHECK_LAUNCH();
}

void lookup_sorted(const int64_t* keys, int64_t n, const int64_t* q, int64_t m, int64_t* idx, hipStream_t s) {
  if (m <= 0) return;
  hipLaunchKernelGGL(k_lookup_sorted, dim3(blocks(m)), dim3(NT), 0, s, keys, n, q, m, idx);
  MRH_CHECK_LAUNCH();
}

void seg_marks(const int64_t* seg, int64_t nseg, int64_t nval, int64_t* marks, hipStream_t s) {
  MRH_HIP(hipMemsetAsync(marks, 0, sizeof(int64_t) * std::max<int64_t>(nval, 1), s));
  if (nseg <= 1 || nval <= 0) return;
  hipLaunchKernelGGL(k_seg_marks, dim3(blocks(nseg)), dim3(NT), 0, s, seg, nseg, nval, marks);
  MRH_CHECK_LAUNCH();
}

void histogram(const int64_t* idx, int64_t n, int64_t K, int64_t* counts, hipStream_t s) {
  MRH_HIP(hipMemsetAsync(counts, 0, sizeof(int64_t) * std::max<int64_t>(K, 1), s));
  if (n <= 0) return;
  hipLaunchKernelGGL(k_histogram, dim3(blocks(n)), dim3(NT), 0, s, idx, n, K, counts);
  MRH_CHECK_LAUNCH();
}

void nz_flags(const uint64_t* v, int64_t n, int32_t* f, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_nz_flags, dim3(blocks(n)), dim3(NT), 0, s, v, n, f);
  MRH_CHECK_LAUNCH();
}

void compact_nz(const uint64_t* v, const int64_t* pos, int64_t n, int64_t* out, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_compact_nz, dim3(blocks(n)), dim3(NT), 0, s, v, pos, n, out);
  MRH_CHECK_LAUNCH();
}

}  // namespace k
}  // namespace mrh
