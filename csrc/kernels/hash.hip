// Key hashing and hash partitioning (aggregate's per-KV owner computation,
// reference src/mapreduce.cpp:453-473: owner = hashlittle(key,kb,nprocs) % nprocs).
//
// Fixed-width keys: one thread per key. Variable-width keys: one thread per key
// reading its bytes through L1/L2 (keys are packed back to back, so a wave's 64
// keys share a few cache lines).
#include "common.h"
#include "launch.h"
#include <cstdio>
#include <cstdlib>

namespace mrh {
namespace k {
namespace {

constexpr int H_NT = 256;

__global__ __launch_bounds__(H_NT) void k_hash32_fixed(const uint8_t* __restrict__ kd, int kw, int64_t n,
                                                      uint32_t seed, uint32_t* __restrict__ out) {
  int64_t i = (int64_t)blockIdx.x * H_NT + threadIdx.x;
  if (i >= n) return;
  out[i] = dev::hashlittle(kd + i * kw, kw, seed);
}

__global__ __launch_bounds__(H_NT) void k_hash32_var(const uint8_t* __restrict__ kd,
                                                    const int64_t* __restrict__ off, int64_t n,
                                                    uint32_t seed, uint32_t* __restrict__ out) {
  int64_t i = (int64_t)blockIdx.x * H_NT + threadIdx.x;
  if (i >= n) return;
  int64_t a = off[i], b = off[i + 1];
  uint32_t c = seed, bb = 0;
  dev::lookup3_wide(kd + a, b - a, &c, &bb);
  out[i] = c;
}

__global__ __launch_bounds__(H_NT) void k_hash64_fixed(const uint8_t* __restrict__ kd, int kw, int64_t n,
                                                      uint64_t* __restrict__ out) {
  int64_t i = (int64_t)blockIdx.x * H_NT + threadIdx.x;
  if (i >= n) return;
  out[i] = dev::hash64(kd + i * kw, kw);
}

__global__ __launch_bounds__(H_NT) void k_hash64_var(const uint8_t* __restrict__ kd,
                                                    const int64_t* __restrict__ off, int64_t n,
                                                    uint64_t* __restrict__ out) {
  int64_t i = (int64_t)blockIdx.x * H_NT + threadIdx.x;
  if (i >= n) return;
  int64_t a = off[i], b = off[i + 1];
  uint32_t c = 0x9e3779b9u, bb = 0x7f4a7c15u;
  dev::lookup3_wide(kd + a, b - a, &c, &bb);
  out[i] = ((uint64_t)c << 32) | bb;
}

// dest = h % P with an LDS histogram per block (P <= 1024), one global atomic per bin per block.
__global__ __launch_bounds__(H_NT) void k_partition(const uint32_t* __restrict__ h, int64_t n, int P,
                                                   int32_t* __restrict__ dest,
                                                   int64_t* __restrict__ counts) {
  __shared__ uint32_t hist[1024];
  for (int i = threadIdx.x; i < P; i += H_NT) hist[i] = 0;
  __syncthreads();
  for (int64_t i = (int64_t)blockIdx.x * H_NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * H_NT) {
    int d = (int)(h[i] % (uint32_t)P);
    dest[i] = d;
    atomicAdd(&hist[d], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < P; i += H_NT)
    if (hist[i]) atomicAdd((unsigned long long*)&counts[i], (unsigned long long)hist[i]);
}

inline unsigned nblk(int64_t n) { return (unsigned)((n + H_NT - 1) / H_NT); }

}  // namespace

void hash32_fixed(const uint8_t* kdata, int kw, int64_t n, uint32_t seed, uint32_t* out, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_hash32_fixed, dim3(nblk(n)), dim3(H_NT), 0, s, kdata, kw, n, seed, out);
  MRH_CHECK_LAUNCH();
}
void hash32_var(const uint8_t* kdata, const int64_t* koff, int64_t n, uint32_t seed, uint32_t* out,
                hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_hash32_var, dim3(nblk(n)), dim3(H_NT), 0, s, kdata, koff, n, seed, out);
  MRH_CHECK_LAUNCH();
}
void hash64_fixed(const uint8_t* kdata, int kw, int64_t n, uint64_t* out, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_hash64_fixed, dim3(nblk(n)), dim3(H_NT), 0, s, kdata, kw, n, out);
  MRH_CHECK_LAUNCH();
}
void hash64_var(const uint8_t* kdata, const int64_t* koff, int64_t n, uint64_t* out, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_hash64_var, dim3(nblk(n)), dim3(H_NT), 0, s, kdata, koff, n, out);
  MRH_CHECK_LAUNCH();
}
void partition_dest(const uint32_t* h, int64_t n, int P, int32_t* dest, int64_t* counts, hipStream_t s) {
  MRH_HIP(hipMemsetAsync(counts, 0, sizeof(int64_t) * P, s));
  if (n <= 0) return;
  check_arg(P <= 1024, "partition: more than 1024 ranks unsupported");
  unsigned g = nblk(n);
  if (g > 2048) g = 2048;
  hipLaunchKernelGGL(k_partition, dim3(g), dim3(H_NT), 0, s, h, n, P, dest, counts);
  MRH_CHECK_LAUNCH();
}

}  // namespace k
}  // namespace mrh
