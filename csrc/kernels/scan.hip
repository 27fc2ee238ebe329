// Device-wide exclusive prefix sums (reduce-then-scan, 3 launches, recursive
// on the block partials). Used for histogram offsets, compaction positions and
// variable-length KV offsets. Tile = 256 threads x 8 items = 2048 elements.
#include "common.h"
#include "launch.h"
#include <cstdio>
#include <cstdlib>

namespace mrh {
namespace k {
namespace {

constexpr int SCAN_NT = 256;
constexpr int SCAN_IT = 8;
constexpr int SCAN_TILE = SCAN_NT * SCAN_IT;

template <typename Tin, typename Tacc>
__global__ __launch_bounds__(SCAN_NT) void k_tile_reduce(const Tin* __restrict__ in, int64_t n,
                                                        Tacc* __restrict__ partial) {
  __shared__ Tacc sh[SCAN_NT / MRH_WAVE];
  const int64_t base = (int64_t)blockIdx.x * SCAN_TILE;
  Tacc s = 0;
#pragma unroll
  for (int i = 0; i < SCAN_IT; ++i) {
    int64_t j = base + (int64_t)i * SCAN_NT + threadIdx.x;
    if (j < n) s += (Tacc)in[j];
  }
  s = dev::wave_sum(s);
  if (dev::lane_id() == 0) sh[dev::wave_id()] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    Tacc t = 0;
#pragma unroll
    for (int w = 0; w < SCAN_NT / MRH_WAVE; ++w) t += sh[w];
    partial[blockIdx.x] = t;
  }
}

// each thread owns SCAN_IT consecutive elements (blocked arrangement)
template <typename Tin, typename Tacc>
__global__ __launch_bounds__(SCAN_NT) void k_tile_scan(const Tin* __restrict__ in, int64_t n,
                                                      const Tacc* __restrict__ block_off,
                                                      Tacc* __restrict__ out, bool write_total) {
  __shared__ Tacc sh[SCAN_NT / MRH_WAVE + 1];
  const int64_t base = (int64_t)blockIdx.x * SCAN_TILE + (int64_t)threadIdx.x * SCAN_IT;
  Tacc v[SCAN_IT];
  Tacc s = 0;
#pragma unroll
  for (int i = 0; i < SCAN_IT; ++i) {
    int64_t j = base + i;
    v[i] = (j < n) ? (Tacc)in[j] : Tacc(0);
    s += v[i];
  }
  Tacc total;
  Tacc pre = dev::block_excl_scan<Tacc, SCAN_NT>(s, sh, &total);
  pre += block_off ? block_off[blockIdx.x] : Tacc(0);
#pragma unroll
  for (int i = 0; i < SCAN_IT; ++i) {
    int64_t j = base + i;
    if (j < n) out[j] = pre;
    pre += v[i];
  }
  if (write_total && blockIdx.x == gridDim.x - 1 && threadIdx.x == SCAN_NT - 1) out[n] = pre;
}

template <typename Tin, typename Tacc>
void scan_impl(const Tin* in, Tacc* out, int64_t n, char* temp, hipStream_t s) {
  if (n <= 0) {
    MRH_HIP(hipMemsetAsync(out, 0, sizeof(Tacc), s));
    return;
  }
  int64_t nb = (n + SCAN_TILE - 1) / SCAN_TILE;
  if (nb == 1) {
    hipLaunchKernelGGL((k_tile_scan<Tin, Tacc>), dim3(1), dim3(SCAN_NT), 0, s, in, n,
                       (const Tacc*)nullptr, out, true);
    MRH_CHECK_LAUNCH();
    return;
  }
  Tacc* partial = reinterpret_cast<Tacc*>(temp);
  Tacc* partial_scan = partial + nb;
  char* next = reinterpret_cast<char*>(partial_scan + nb + 1);
  // keep 256-byte alignment for the recursive level
  next = reinterpret_cast<char*>((reinterpret_cast<uintptr_t>(next) + 255) & ~uintptr_t(255));
  hipLaunchKernelGGL((k_tile_reduce<Tin, Tacc>), dim3(nb), dim3(SCAN_NT), 0, s, in, n, partial);
  MRH_CHECK_LAUNCH();
  scan_impl<Tacc, Tacc>(partial, partial_scan, nb, next, s);
  hipLaunchKernelGGL((k_tile_scan<Tin, Tacc>), dim3(nb), dim3(SCAN_NT), 0, s, in, n,
                     (const Tacc*)partial_scan, out, true);
  MRH_CHECK_LAUNCH();
}

}  // namespace

size_t scan_temp_bytes(int64_t n) {
  size_t total = 256;
  while (n > SCAN_TILE) {
    int64_t nb = (n + SCAN_TILE - 1) / SCAN_TILE;
    total += (size_t)(2 * nb + 1) * 8 + 512;
    n = nb;
  }
  return total;
}

void exclusive_scan_u32(const uint32_t* in, uint32_t* out, int64_t n, void* temp, hipStream_t s) {
  scan_impl<uint32_t, uint32_t>(in, out, n, reinterpret_cast<char*>(temp), s);
}
void exclusive_scan_i64(const int64_t* in, int64_t* out, int64_t n, void* temp, hipStream_t s) {
  scan_impl<int64_t, int64_t>(in, out, n, reinterpret_cast<char*>(temp), s);
}
void lengths_to_offsets(const int32_t* len, int64_t* off, int64_t n, void* temp, hipStream_t s) {
  scan_impl<int32_t, int64_t>(len, off, n, reinterpret_cast<char*>(temp), s);
}

}  // namespace k
}  // namespace mrh
