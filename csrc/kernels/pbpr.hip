// Propagation-blocked PageRank iteration for one GPU (PageRankPlan with
// blocking, csrc/engine/graphplan.cpp). The pull iteration (gather c[src] per
// in-edge, wavesegred.h) is bound by its random 4-byte gathers: at RMAT-26,
// 461 M L2 misses x 64 B per iteration (profiles/r1_pagerank_pmc.txt).
// Propagation blocking (Beamer, Asanovic, Patterson, IPDPS 2017) turns them
// into two streaming passes over a static edge layout:
//
//   phase 1  edges in (source chunk, destination bin, source) order: each
//            edge's contribution c[src] — read from a source window that stays
//            in L2 — is written to its slot in the phase-2 order (p1_out);
//            the slots of one (chunk, bin) run are consecutive, so the writes
//            are coalesced runs;
//   phase 2  edges in (destination bin, chunk, source) order: one workgroup
//            per (bin, edge slice); each wave sums its 64 edges per run of
//            equal destinations (segmented wave scan), one LDS atomic per run
//            into a 16 K-entry accumulator indexed by the 16-bit offset, then
//            writes (exclusive bin) or atomically adds (bin split over
//            several slices) its sums into the rank accumulator.
//
// Per edge: 4 B src + 4 B slot + 4 B value written, then 4 B value + 2 B
// destination read — all streamed. LDS float atomics make the summation
// order inside a bin run-to-run dependent (fp32 rounding only).
// Opt-in (MRH_PR_BLOCKING=1): on RMAT-26 the two passes take 8.9 ms per
// iteration against 7.9 ms for the pull kernel (profiles/r2_pagerank_blocking.txt).
#include "common.h"
#include "launch.h"

namespace mrh {
namespace k {
namespace {

constexpr int P1_NT = 256;
constexpr int P2_NT = 1024;
constexpr int BIN = 1 << 14;  // destinations per bin (64 KB of LDS)

__global__ __launch_bounds__(P1_NT) void k_pb_phase1(const int32_t* __restrict__ src, const int32_t* __restrict__ out_pos,
                                                    int64_t m, const float* __restrict__ c, float* __restrict__ vals) {
  for (int64_t j = (int64_t)blockIdx.x * P1_NT + threadIdx.x; j < m; j += (int64_t)gridDim.x * P1_NT)
    vals[out_pos[j]] = c[src[j]];
}

// unit u: bin ub[u], edges [ue0[u], ue1[u]) of the phase-2 order; uex[u] != 0
// when it is the bin's only unit (plain stores) else atomics
__global__ __launch_bounds__(P2_NT) void k_pb_phase2(const float* __restrict__ vals, const uint16_t* __restrict__ dst,
                                                    const int32_t* __restrict__ ub, const int64_t* __restrict__ ue0,
                                                    const int64_t* __restrict__ ue1, const uint8_t* __restrict__ uex,
                                                    int64_t nunit, int64_t nv, float* __restrict__ acc) {
  __shared__ float sacc[BIN];
  for (int64_t u = blockIdx.x; u < nunit; u += gridDim.x) {
    for (int i = threadIdx.x; i < BIN; i += P2_NT) sacc[i] = 0.f;
    __syncthreads();
    // a segmented wave sum over the 64 consecutive edges of a wave leaves one
    // LDS atomic per run of equal destinations instead of one per edge
    const int64_t e1 = ue1[u];
    const int lane = dev::lane_id();
    for (int64_t eb = ue0[u] + (threadIdx.x & ~(MRH_WAVE - 1)); eb < e1; eb += P2_NT) {
      const int64_t e = eb + lane;
      const bool ok = e < e1;
      const int d = ok ? (int)dst[e] : -1;
      float v = ok ? vals[e] : 0.f;
      const int dprev = __shfl_up(d, 1, MRH_WAVE);
      const int dnext = __shfl_down(d, 1, MRH_WAVE);
      // segmented inclusive scan: stop at the first lane of this destination run
      const uint64_t heads = __ballot(lane == 0 || d != dprev);
      const uint64_t below = heads & ((lane == 63) ? ~0ull : ((2ull << lane) - 1));
      const int head = 63 - __clzll(below);  // highest head lane <= lane
#pragma unroll
      for (int o = 1; o < MRH_WAVE; o <<= 1) {
        const float u2 = __shfl_up(v, o, MRH_WAVE);
        if (lane - o >= head) v += u2;
      }
      const bool tail = ok && (lane == MRH_WAVE - 1 || d != dnext || e + 1 >= e1);
      if (tail) atomicAdd(&sacc[d], v);
    }
    __syncthreads();
    const int64_t base = (int64_t)ub[u] * BIN;
    const bool excl = uex[u] != 0;
    for (int i = threadIdx.x; i < BIN; i += P2_NT) {
      const int64_t v = base + i;
      if (v >= nv) break;
      const float x = sacc[i];
      if (excl) acc[v] = x;
      else if (x != 0.f) atomicAdd(&acc[v], x);
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(P1_NT) void k_pb_scatter_pos(const int32_t* __restrict__ perm2, int64_t m,
                                                         int32_t* __restrict__ out_pos) {
  for (int64_t k = (int64_t)blockIdx.x * P1_NT + threadIdx.x; k < m; k += (int64_t)gridDim.x * P1_NT)
    out_pos[perm2[k]] = (int32_t)k;
}

__global__ __launch_bounds__(P1_NT) void k_pb_gather_dst(const int32_t* __restrict__ perm2,
                                                        const int32_t* __restrict__ dst1, int64_t m,
                                                        uint16_t* __restrict__ dst2) {
  for (int64_t k = (int64_t)blockIdx.x * P1_NT + threadIdx.x; k < m; k += (int64_t)gridDim.x * P1_NT)
    dst2[k] = (uint16_t)(dst1[perm2[k]] & (BIN - 1));
}

unsigned grid_for(int64_t n, int nt) {
  int64_t b = (n + nt - 1) / nt;
  return (unsigned)(b < 1 ? 1 : (b > 65536 ? 65536 : b));
}

}  // namespace

int pb_bin_size() { return BIN; }

void pb_phase1(const int32_t* src, const int32_t* out_pos, int64_t m, const float* c, float* vals, hipStream_t s) {
  if (m <= 0) return;
  hipLaunchKernelGGL(k_pb_phase1, dim3(grid_for(m, P1_NT)), dim3(P1_NT), 0, s, src, out_pos, m, c, vals);
  MRH_CHECK_LAUNCH();
}

void pb_phase2(const float* vals, const uint16_t* dst, const int32_t* ub, const int64_t* ue0, const int64_t* ue1,
               const uint8_t* uex, int64_t nunit, int64_t nv, float* acc, hipStream_t s) {
  if (nunit <= 0) return;
  const unsigned grid = (unsigned)(nunit < 65536 ? nunit : 65536);
  hipLaunchKernelGGL(k_pb_phase2, dim3(grid), dim3(P2_NT), 0, s, vals, dst, ub, ue0, ue1, uex, nunit, nv, acc);
  MRH_CHECK_LAUNCH();
}

void pb_layout(const int32_t* perm2, const int32_t* dst1, int64_t m, int32_t* out_pos, uint16_t* dst2, hipStream_t s) {
  if (m <= 0) return;
  hipLaunchKernelGGL(k_pb_scatter_pos, dim3(grid_for(m, P1_NT)), dim3(P1_NT), 0, s, perm2, m, out_pos);
  MRH_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_pb_gather_dst, dim3(grid_for(m, P1_NT)), dim3(P1_NT), 0, s, perm2, dst1, m, dst2);
  MRH_CHECK_LAUNCH();
}

}  // namespace k
}  // namespace mrh
