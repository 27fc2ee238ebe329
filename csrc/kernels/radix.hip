// Stable LSD radix sort of (uint64 key, uint32 value) pairs for CDNA4.
//
// Replaces MR-MPI's qsort()+2-way spool merge (reference src/mapreduce.cpp:2462-2633)
// and the hash-table group-by of KeyMultiValue::convert (src/keymultivalue.cpp:645-789).
//
// Per 8-bit digit pass:
//   upsweep   : per-block digit histogram in LDS -> hist[digit][block]
//   scan      : device exclusive scan over the digit-major histogram
//   downsweep : wave64 multi-split ranking (8 x __ballot match + popcount, one
//               LDS counter row per wave), block-local reorder through LDS,
//               then coalesced-by-digit-run scatter to global memory.
// A single global histogram of all 8 digit positions (one read of the keys)
// lets the host skip passes whose digit is constant (e.g. the zero high bits of
// vertex ids), so a 2^26-vertex key costs 4 passes, not 8.
#include "common.h"
#include "launch.h"
#include <cstdio>
#include <cstdlib>
#include <vector>

namespace mrh {
namespace k {
namespace {

constexpr int RX_NT = 256;
constexpr int RX_NW = RX_NT / MRH_WAVE;
constexpr int RX_IT = 8;
constexpr int RX_TILE = RX_NT * RX_IT;   // 2048 pairs per block
constexpr int RX_BINS = 256;

__global__ __launch_bounds__(RX_NT) void k_global_hist(const uint64_t* __restrict__ keys, int64_t n,
                                                      uint32_t* __restrict__ counts /*[8][256]*/) {
  __shared__ uint32_t h[8][RX_BINS];
  for (int i = threadIdx.x; i < 8 * RX_BINS; i += RX_NT) (&h[0][0])[i] = 0;
  __syncthreads();
  for (int64_t i = (int64_t)blockIdx.x * RX_NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * RX_NT) {
    uint64_t k = keys[i];
#pragma unroll
    for (int p = 0; p < 8; ++p) atomicAdd(&h[p][(k >> (8 * p)) & 255], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 8 * RX_BINS; i += RX_NT) {
    uint32_t v = (&h[0][0])[i];
    if (v) atomicAdd(&counts[i], v);
  }
}

__global__ __launch_bounds__(RX_NT) void k_upsweep(const uint64_t* __restrict__ keys, int64_t n, int shift,
                                                  uint32_t* __restrict__ hist, int nb) {
  __shared__ uint32_t cnt[RX_BINS];
  cnt[threadIdx.x] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * RX_TILE;
#pragma unroll
  for (int i = 0; i < RX_IT; ++i) {
    int64_t j = base + (int64_t)i * RX_NT + threadIdx.x;
    if (j < n) atomicAdd(&cnt[(keys[j] >> shift) & 255], 1u);
  }
  __syncthreads();
  hist[(int64_t)threadIdx.x * nb + blockIdx.x] = cnt[threadIdx.x];
}

__global__ __launch_bounds__(RX_NT) void k_downsweep(const uint64_t* __restrict__ kin,
                                                    const uint32_t* __restrict__ vin,
                                                    uint64_t* __restrict__ kout,
                                                    uint32_t* __restrict__ vout, int64_t n, int shift,
                                                    const uint32_t* __restrict__ hist_scan, int nb) {
  __shared__ uint64_t skeys[RX_TILE];
  __shared__ uint32_t svals[RX_TILE];
  __shared__ uint32_t wcnt[RX_NW][RX_BINS];
  __shared__ uint32_t bdig[RX_BINS];
  __shared__ uint32_t gofs[RX_BINS];
  __shared__ uint32_t scan_sh[RX_NW + 1];

  const int lane = dev::lane_id();
  const int w = dev::wave_id();
  const int64_t base = (int64_t)blockIdx.x * RX_TILE;
  const int64_t wbase = base + (int64_t)w * (MRH_WAVE * RX_IT);
  const int tilecount = (int)((n - base) < RX_TILE ? (n - base) : RX_TILE);

  for (int i = threadIdx.x; i < RX_NW * RX_BINS; i += RX_NT) (&wcnt[0][0])[i] = 0;

  uint64_t kk[RX_IT];
  uint32_t vv[RX_IT];
  uint32_t lr[RX_IT];
#pragma unroll
  for (int j = 0; j < RX_IT; ++j) {
    int64_t idx = wbase + (int64_t)j * MRH_WAVE + lane;
    bool valid = idx < n;
    kk[j] = valid ? kin[idx] : 0ull;
    vv[j] = valid ? vin[idx] : 0u;
  }
  __syncthreads();

  const uint64_t lt = dev::lanemask_lt();
#pragma unroll
  for (int j = 0; j < RX_IT; ++j) {
    int64_t idx = wbase + (int64_t)j * MRH_WAVE + lane;
    bool valid = idx < n;
    uint32_t d = (uint32_t)(kk[j] >> shift) & 255u;
    uint64_t peers = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      bool bit = (d >> b) & 1u;
      uint64_t bb = __ballot(bit);
      peers &= bit ? bb : ~bb;
    }
    uint32_t before = 0;
    if (valid) before = wcnt[w][d];
    bool leader = valid && ((peers & lt) == 0);
    if (leader) wcnt[w][d] = before + (uint32_t)__popcll(peers);
    lr[j] = before + (uint32_t)__popcll(peers & lt);
  }
  __syncthreads();

  {  // digit t = threadIdx.x : wave prefixes, block-local digit offsets, global offsets
    const int t = threadIdx.x;
    uint32_t run = 0;
#pragma unroll
    for (int ww = 0; ww < RX_NW; ++ww) {
      uint32_t c = wcnt[ww][t];
      wcnt[ww][t] = run;
      run += c;
    }
    uint32_t total;
    uint32_t ex = dev::block_excl_scan<uint32_t, RX_NT>(run, scan_sh, &total);
    bdig[t] = ex;
    gofs[t] = hist_scan[(int64_t)t * nb + blockIdx.x];
  }
  __syncthreads();

#pragma unroll
  for (int j = 0; j < RX_IT; ++j) {
    int64_t idx = wbase + (int64_t)j * MRH_WAVE + lane;
    if (idx < n) {
      uint32_t d = (uint32_t)(kk[j] >> shift) & 255u;
      uint32_t pos = bdig[d] + wcnt[w][d] + lr[j];
      skeys[pos] = kk[j];
      svals[pos] = vv[j];
    }
  }
  __syncthreads();

  for (int i = threadIdx.x; i < tilecount; i += RX_NT) {
    uint64_t key = skeys[i];
    uint32_t d = (uint32_t)(key >> shift) & 255u;
    uint32_t g = gofs[d] + (uint32_t)i - bdig[d];
    kout[g] = key;
    vout[g] = svals[i];
  }
}

}  // namespace

size_t radix_temp_bytes(int64_t n) {
  int64_t nb = (n + RX_TILE - 1) / RX_TILE;
  size_t hist = ((size_t)RX_BINS * nb + 1) * sizeof(uint32_t);
  size_t a = (hist + 255) & ~size_t(255);
  return 2 * a + scan_temp_bytes((int64_t)RX_BINS * nb) + 8 * RX_BINS * 4 + 1024;
}

void radix_sort_u64_u32(const uint64_t* keys_in, const uint32_t* vals_in, uint64_t* keys_out,
                        uint32_t* vals_out, uint64_t* keys_alt, uint32_t* vals_alt, int64_t n,
                        int begin_bit, int end_bit, void* temp, hipStream_t s, int* passes_run) {
  if (passes_run) *passes_run = 0;
  if (n <= 0) return;
  check_arg(n <= 0xFFFFFFFFll, "radix sort: more than 2^32-1 pairs per call (the out-of-core sort splits larger inputs)");
  const int64_t nb = (n + RX_TILE - 1) / RX_TILE;
  char* t = reinterpret_cast<char*>(temp);
  size_t hist_bytes = ((((size_t)RX_BINS * nb + 1) * sizeof(uint32_t)) + 255) & ~size_t(255);
  uint32_t* hist = reinterpret_cast<uint32_t*>(t);
  uint32_t* hist_scan = reinterpret_cast<uint32_t*>(t + hist_bytes);
  uint32_t* gcounts = reinterpret_cast<uint32_t*>(t + 2 * hist_bytes);
  char* scan_tmp = t + 2 * hist_bytes + 8 * RX_BINS * 4 + 256;
  scan_tmp = reinterpret_cast<char*>((reinterpret_cast<uintptr_t>(scan_tmp) + 255) & ~uintptr_t(255));

  // which digit positions actually vary?
  hipMemsetAsync(gcounts, 0, 8 * RX_BINS * 4, s);
  int ghist_blocks = (int)((n + RX_NT - 1) / RX_NT);
  if (ghist_blocks > 2048) ghist_blocks = 2048;
  hipLaunchKernelGGL(k_global_hist, dim3(ghist_blocks), dim3(RX_NT), 0, s, keys_in, n, gcounts);
  MRH_CHECK_LAUNCH();
  std::vector<uint32_t> hc(8 * RX_BINS);
  hipMemcpyAsync(hc.data(), gcounts, 8 * RX_BINS * 4, hipMemcpyDeviceToHost, s);
  hipStreamSynchronize(s);
  std::vector<int> passes;
  for (int p = begin_bit / 8; p * 8 < end_bit && p < 8; ++p) {
    bool trivial = false;
    for (int b = 0; b < RX_BINS; ++b)
      if (hc[p * RX_BINS + b] == (uint32_t)n) { trivial = true; break; }
    if (!trivial) passes.push_back(p);
  }
  const int np = (int)passes.size();
  if (passes_run) *passes_run = np;
  if (np == 0) {
    hipMemcpyAsync(keys_out, keys_in, n * 8, hipMemcpyDeviceToDevice, s);
    hipMemcpyAsync(vals_out, vals_in, n * 4, hipMemcpyDeviceToDevice, s);
    return;
  }
  const uint64_t* ki = keys_in;
  const uint32_t* vi = vals_in;
  for (int q = 0; q < np; ++q) {
    // ping-pong so that the final pass lands in *_out
    bool to_out = ((np - 1 - q) % 2) == 0;
    uint64_t* ko = to_out ? keys_out : keys_alt;
    uint32_t* vo = to_out ? vals_out : vals_alt;
    int shift = passes[q] * 8;
    hipLaunchKernelGGL(k_upsweep, dim3(nb), dim3(RX_NT), 0, s, ki, n, shift, hist, (int)nb);
    MRH_CHECK_LAUNCH();
    exclusive_scan_u32(hist, hist_scan, (int64_t)RX_BINS * nb, scan_tmp, s);
    hipLaunchKernelGGL(k_downsweep, dim3(nb), dim3(RX_NT), 0, s, ki, vi, ko, vo, n, shift,
                       (const uint32_t*)hist_scan, (int)nb);
    MRH_CHECK_LAUNCH();
    ki = ko;
    vi = vo;
  }
}

}  // namespace k
}  // namespace mrh
