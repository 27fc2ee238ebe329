// Stable LSD radix sort of (uint64 key, uint32 value) pairs — or of uint64 keys
// alone (vals_in == nullptr; payload bits packed below the sorted range) — for CDNA4:
// one-sweep passes with decoupled look-back (Adinets & Merrill, "Onesweep",
// 2022), re-built for 64-lane wavefronts.
//
// Replaces MR-MPI's qsort()+2-way spool merge (reference src/mapreduce.cpp:2462-2633)
// and the hash-table group-by of KeyMultiValue::convert (src/keymultivalue.cpp:645-789).
//
//   k_global_hist : one read of the keys -> the digit histograms of all eight
//                   8-bit digit positions (LDS atomics into lane-striped
//                   copies, one per wave for a digit uniform over the wave;
//                   one global atomic per bin)
//   k_digit_base  : per digit position, the exclusive scan of its 256 counts =
//                   the global start of every digit (no host round trip)
//   k_onesweep    : one kernel per pass. A workgroup takes the next 4096-pair
//                   tile from an atomic ticket (so every earlier tile is already
//                   resident: the look-back below always makes progress), ranks
//                   its pairs with the wave64 multi-split (8 ballots + popcount
//                   per pair, one LDS counter row per wave), publishes its
//                   per-digit counts, looks back over earlier tiles for its
//                   exclusive prefix (stopping at the first tile that already
//                   published an inclusive one), publishes that, reorders the
//                   tile through LDS and scatters coalesced runs per digit.
// Keys are read once per pass (the upsweep/scan/downsweep design read them
// twice and needed three launches per pass).
//
// Look-back words (u64, one per tile and digit): bits 0-47 count, 48-55 the
// pass epoch (1..8), 56-57 state (1 tile aggregate, 2 inclusive prefix). The
// epoch lets all passes of one sort share one status array, zeroed once.
//
// Passes whose digit is constant over all keys can be skipped (skip_trivial):
// that needs the histogram on the host (one sync); callers that know every
// digit varies (hashes, dense ranks) sort without any host synchronisation.
#include "common.h"
#include "launch.h"
#include <cstdio>
#include <algorithm>
#include <cstdlib>
#include <vector>

namespace mrh {
namespace k {
namespace {

constexpr int RX_NT = 256;
constexpr int RX_NW = RX_NT / MRH_WAVE;
constexpr int RX_IT = 8;
constexpr int RX_TILE = RX_NT * RX_IT;   // smallest tile (2048 pairs): sizes the look-back array
constexpr int RX_BINS = 256;
constexpr uint64_t LB_COUNT = (1ull << 48) - 1;
constexpr uint64_t LB_AGG = 1ull << 56, LB_PRE = 2ull << 56;

// the npos digits of the sorted bit range only (digit q at bit sh0 + 8q, the
// last one lastbits wide): bits outside it are constant-heavy (zero high
// bytes) and would serialise on one LDS bin. Skewed digits (the zero high
// bytes of small ids, hub ids) still put many lanes of a wave on one bin:
// RX_HREP copies of the histograms, lane l adding to copy l % RX_HREP, cut
// those same-address LDS atomics RX_HREP-fold; a digit uniform over the wave
// is one add of the lane count.
constexpr int RX_HREP = 4;
__global__ __launch_bounds__(RX_NT) void k_global_hist(const uint64_t* __restrict__ keys, int64_t n, int sh0, int npos,
                                                      int lastbits, uint32_t* __restrict__ counts /*[8][256]*/) {
  __shared__ uint32_t h[8][RX_BINS][RX_HREP];  // copies of a bin side by side: different banks
  for (int i = threadIdx.x; i < RX_HREP * 8 * RX_BINS; i += RX_NT) (&h[0][0][0])[i] = 0;
  __syncthreads();
  const int lane = dev::lane_id();
  const int rep = lane % RX_HREP;
  auto add = [&](uint64_t k) {
    const uint64_t active = __ballot(1);
    const int first = __ffsll((long long)active) - 1;
#pragma unroll
    for (int p = 0; p < 8; ++p)
      if (p < npos) {
        const uint32_t d = (uint32_t)(k >> (sh0 + 8 * p)) & (p == npos - 1 ? (1u << lastbits) - 1u : 255u);
        const uint32_t d0 = (uint32_t)__shfl((int)d, first, MRH_WAVE);
        if (__ballot(d == d0) == active) {
          if (lane == first) atomicAdd(&h[p][d0][0], (uint32_t)__popcll(active));
        } else {
          atomicAdd(&h[p][d][rep], 1u);
        }
      }
  };
  // four loads in flight per thread, then their digits
  const int64_t stride = (int64_t)gridDim.x * RX_NT;
  int64_t i = (int64_t)blockIdx.x * RX_NT + threadIdx.x;
  for (; i + 3 * stride < n; i += 4 * stride) {
    const uint64_t k0 = keys[i], k1 = keys[i + stride], k2 = keys[i + 2 * stride], k3 = keys[i + 3 * stride];
    add(k0);
    add(k1);
    add(k2);
    add(k3);
  }
  for (; i < n; i += stride) add(keys[i]);
  __syncthreads();
  for (int i = threadIdx.x; i < 8 * RX_BINS; i += RX_NT) {
    uint32_t v = 0;
#pragma unroll
    for (int r = 0; r < RX_HREP; ++r) v += (&h[0][0][0])[i * RX_HREP + r];
    if (v) atomicAdd(&counts[i], v);
  }
}

// block p: base[p][d] = sum of counts[p][0..d)
__global__ __launch_bounds__(RX_BINS) void k_digit_base(const uint32_t* __restrict__ counts,
                                                       uint64_t* __restrict__ base) {
  __shared__ uint64_t sh[RX_BINS / MRH_WAVE + 1];
  const int p = blockIdx.x, t = threadIdx.x;
  uint64_t total;
  const uint64_t ex = dev::block_excl_scan<uint64_t, RX_BINS>((uint64_t)counts[p * RX_BINS + t], sh, &total);
  base[p * RX_BINS + t] = ex;
}

template <int RX_IT, bool VALS>
__global__ __launch_bounds__(RX_NT) void k_onesweep(const uint64_t* __restrict__ kin, const uint32_t* __restrict__ vin,
                                                   uint64_t* __restrict__ kout, uint32_t* __restrict__ vout,
                                                   int64_t n, int shift, uint32_t dmask,
                                                   const uint64_t* __restrict__ dbase,
                                                   unsigned long long* __restrict__ status, uint64_t epoch,
                                                   unsigned int* __restrict__ ticket) {
  constexpr int RX_TILE = RX_NT * RX_IT;
  __shared__ uint64_t skeys[RX_TILE];
  __shared__ uint32_t svals[VALS ? RX_TILE : 1];  // keys-only: the LDS goes to bigger tiles
  __shared__ uint32_t wcnt[RX_NW][RX_BINS];
  __shared__ uint32_t bdig[RX_BINS];
  __shared__ uint64_t gofs[RX_BINS];
  __shared__ uint32_t scan_sh[RX_NW + 1];
  __shared__ uint32_t s_tile;

  if (threadIdx.x == 0) s_tile = atomicAdd(ticket, 1u);
  for (int i = threadIdx.x; i < RX_NW * RX_BINS; i += RX_NT) (&wcnt[0][0])[i] = 0;
  __syncthreads();
  const int64_t tile = s_tile;
  const int lane = dev::lane_id();
  const int w = dev::wave_id();
  const int64_t base = tile * RX_TILE;
  const int64_t wbase = base + (int64_t)w * (MRH_WAVE * RX_IT);
  const int tilecount = (int)((n - base) < RX_TILE ? (n - base) : RX_TILE);

  uint64_t kk[RX_IT];
  uint32_t vv[RX_IT];
  uint32_t lr[RX_IT];
#pragma unroll
  for (int j = 0; j < RX_IT; ++j) {
    int64_t idx = wbase + (int64_t)j * MRH_WAVE + lane;
    bool valid = idx < n;
    kk[j] = valid ? kin[idx] : 0ull;
    vv[j] = (VALS && valid) ? vin[idx] : 0u;
  }

  // wave multi-split: rank of each pair among equal digits of its wave
  const uint64_t lt = dev::lanemask_lt();
#pragma unroll
  for (int j = 0; j < RX_IT; ++j) {
    int64_t idx = wbase + (int64_t)j * MRH_WAVE + lane;
    bool valid = idx < n;
    uint32_t d = (uint32_t)(kk[j] >> shift) & dmask;
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

  {  // digit t = threadIdx.x: wave prefixes, block-local digit offsets, tile count
    const int t = threadIdx.x;
    uint32_t run = 0;
#pragma unroll
    for (int ww = 0; ww < RX_NW; ++ww) {
      uint32_t c = wcnt[ww][t];
      wcnt[ww][t] = run;
      run += c;
    }
    uint32_t total;
    bdig[t] = dev::block_excl_scan<uint32_t, RX_NT>(run, scan_sh, &total);
    // decoupled look-back for digit t
    unsigned long long* st = status + tile * RX_BINS + t;
    uint64_t excl = 0;
    if (tile == 0) {
      __hip_atomic_store(st, (unsigned long long)(LB_PRE | (epoch << 48) | run), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    } else {
      __hip_atomic_store(st, (unsigned long long)(LB_AGG | (epoch << 48) | run), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
      for (int64_t p = tile - 1; p >= 0;) {
        const uint64_t v = __hip_atomic_load(status + p * RX_BINS + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (((v >> 48) & 255) != epoch) {  // tile p has not published yet (it is resident: spin)
          __builtin_amdgcn_s_sleep(1);
          continue;
        }
        excl += v & LB_COUNT;
        if (v & LB_PRE) break;
        --p;
      }
      __hip_atomic_store(st, (unsigned long long)(LB_PRE | (epoch << 48) | (excl + run)), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
    gofs[t] = dbase[t] + excl;
  }
  __syncthreads();

#pragma unroll
  for (int j = 0; j < RX_IT; ++j) {
    int64_t idx = wbase + (int64_t)j * MRH_WAVE + lane;
    if (idx < n) {
      uint32_t d = (uint32_t)(kk[j] >> shift) & dmask;
      uint32_t pos = bdig[d] + wcnt[w][d] + lr[j];
      skeys[pos] = kk[j];
      if (VALS) svals[pos] = vv[j];
    }
  }
  __syncthreads();

  for (int i = threadIdx.x; i < tilecount; i += RX_NT) {
    uint64_t key = skeys[i];
    uint32_t d = (uint32_t)(key >> shift) & dmask;
    uint64_t g = gofs[d] + (uint64_t)i - bdig[d];
    kout[g] = key;
    if (VALS) vout[g] = svals[i];
  }
}

size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

// pairs per thread of a one-sweep tile: 16 (4096-pair tiles) by default —
// on MI355X it beats 8 at every size (half the look-back chain, 16-key runs
// per digit in the scatter: 5.4 M keys 90 -> 78 us/pass, 200 M keys
// 2.74 -> 2.22 ms/pass, profiles/r2_radix_onesweep_bench.txt); MRH_RX_IT=8
// selects 2048-pair tiles. Keys-only sorts have no value column in LDS and
// take MRH_RX_KIT keys per thread (default 32: 8192-key tiles, 32-key runs)
int rx_items() {
  static const int it = [] {
    const char* v = std::getenv("MRH_RX_IT");
    return (v && std::atoi(v) == 8) ? 8 : 16;
  }();
  return it;
}
int rx_key_items() {
  static const int it = [] {
    const char* v = std::getenv("MRH_RX_KIT");
    const int k = v ? std::atoi(v) : 32;
    return k == 8 || k == 16 || k == 24 ? k : 32;
  }();
  return it;
}

}  // namespace

size_t radix_temp_bytes(int64_t n) {
  const int64_t nb = (n + RX_TILE - 1) / RX_TILE;
  return align256((size_t)nb * RX_BINS * 8) + align256(8 * RX_BINS * 8) + align256(8 * RX_BINS * 4) + 256 + 256;
}

void radix_sort_u64_u32(const uint64_t* keys_in, const uint32_t* vals_in, uint64_t* keys_out,
                        uint32_t* vals_out, uint64_t* keys_alt, uint32_t* vals_alt, int64_t n,
                        int begin_bit, int end_bit, void* temp, hipStream_t s, int* passes_run, bool skip_trivial) {
  if (passes_run) *passes_run = 0;
  if (n <= 0) return;
  check_arg(n <= 0xFFFFFFFFll, "radix sort: more than 2^32-1 pairs per call (the out-of-core sort splits larger inputs)");
  const int64_t nb = (n + RX_TILE - 1) / RX_TILE;  // status rows sized for the smallest tile
  const int items = vals_in ? rx_items() : rx_key_items();
  const int64_t ntile = (n + (int64_t)RX_NT * items - 1) / ((int64_t)RX_NT * items);
  char* t = reinterpret_cast<char*>(temp);
  t = reinterpret_cast<char*>((reinterpret_cast<uintptr_t>(t) + 255) & ~uintptr_t(255));
  const size_t st_bytes = align256((size_t)nb * RX_BINS * 8);
  unsigned long long* status = reinterpret_cast<unsigned long long*>(t);
  uint64_t* dbase = reinterpret_cast<uint64_t*>(t + st_bytes);
  uint32_t* gcounts = reinterpret_cast<uint32_t*>(t + st_bytes + align256(8 * RX_BINS * 8));
  unsigned int* tickets = reinterpret_cast<unsigned int*>(t + st_bytes + align256(8 * RX_BINS * 8) +
                                                          align256(8 * RX_BINS * 4));

  // zero the look-back words, the histogram and the 8 tickets in one memset
  // (they are contiguous apart from dbase, which k_digit_base overwrites)
  MRH_HIP(hipMemsetAsync(status, 0, st_bytes, s));
  MRH_HIP(hipMemsetAsync(gcounts, 0, align256(8 * RX_BINS * 4) + 8 * sizeof(unsigned int), s));
  int ghist_blocks = (int)((n + RX_NT - 1) / RX_NT);
  if (ghist_blocks > 2048) ghist_blocks = 2048;
  // digits of at most 8 bits from begin_bit up (any bit offset; the last one
  // narrower when the range is not a multiple of 8 bits)
  const int npos = std::min(8, (end_bit - begin_bit + 7) / 8);
  const int lastbits = end_bit - begin_bit - 8 * (npos - 1);
  hipLaunchKernelGGL(k_global_hist, dim3(ghist_blocks), dim3(RX_NT), 0, s, keys_in, n, begin_bit, npos, lastbits,
                     gcounts);
  MRH_CHECK_LAUNCH();
  std::vector<int> passes;
  if (skip_trivial) {  // which digit positions actually vary? (one host sync)
    std::vector<uint32_t> hc(8 * RX_BINS);
    MRH_HIP(hipMemcpyAsync(hc.data(), gcounts, 8 * RX_BINS * 4, hipMemcpyDeviceToHost, s));
    MRH_HIP(hipStreamSynchronize(s));
    for (int p = 0; p < npos; ++p) {
      bool trivial = false;
      for (int b = 0; b < RX_BINS; ++b)
        if (hc[p * RX_BINS + b] == (uint32_t)n) {
          trivial = true;
          break;
        }
      if (!trivial) passes.push_back(p);
    }
  } else {
    for (int p = 0; p < npos; ++p) passes.push_back(p);
  }
  const int np = (int)passes.size();
  if (passes_run) *passes_run = np;
  if (np == 0) {
    MRH_HIP(hipMemcpyAsync(keys_out, keys_in, n * 8, hipMemcpyDeviceToDevice, s));
    if (vals_in) MRH_HIP(hipMemcpyAsync(vals_out, vals_in, n * 4, hipMemcpyDeviceToDevice, s));
    return;
  }
  hipLaunchKernelGGL(k_digit_base, dim3(8), dim3(RX_BINS), 0, s, (const uint32_t*)gcounts, dbase);
  MRH_CHECK_LAUNCH();
  const uint64_t* ki = keys_in;
  const uint32_t* vi = vals_in;
  for (int q = 0; q < np; ++q) {
    // ping-pong so that the final pass lands in *_out
    bool to_out = ((np - 1 - q) % 2) == 0;
    uint64_t* ko = to_out ? keys_out : keys_alt;
    uint32_t* vo = vals_in ? (to_out ? vals_out : vals_alt) : nullptr;
    const int p = passes[q];
    const uint64_t* db = dbase + p * RX_BINS;
    const uint64_t ep = (uint64_t)(q + 1);
    const int shift = begin_bit + 8 * p;
    const uint32_t dmask = p == npos - 1 ? (1u << lastbits) - 1u : 255u;
#define MRH_ONESWEEP(IT, V)                                                                                        \
  hipLaunchKernelGGL((k_onesweep<IT, V>), dim3((unsigned)ntile), dim3(RX_NT), 0, s, ki, vi, ko, vo, n, shift, dmask, \
                     db, status, ep, tickets + q)
    if (vals_in) {
      if (items == 16) MRH_ONESWEEP(16, true);
      else MRH_ONESWEEP(8, true);
    } else {
      switch (items) {
        case 8: MRH_ONESWEEP(8, false); break;
        case 16: MRH_ONESWEEP(16, false); break;
        case 24: MRH_ONESWEEP(24, false); break;
        default: MRH_ONESWEEP(32, false); break;
      }
    }
#undef MRH_ONESWEEP
    MRH_CHECK_LAUNCH();
    ki = ko;
    vi = vo;
  }
}

}  // namespace k
}  // namespace mrh
