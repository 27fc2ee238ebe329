// K-means map with in-mapper combining (the GPMR K-means workload of
// chapter_final.pdf Fig. 6a: 32 M 2-D points per GPU; not in the reference
// code, which only runs IntCount-style jobs on MR-MPI).
//
// One pass over the points: each lane assigns its points to the nearest
// centroid (centroids staged in LDS, D <= 8 dims in registers) and the
// workgroup sums each cluster's points on chip (D <= 3: the transposed
// reduction of k_kmeans_tr, no atomics; else per-cluster LDS accumulators);
// the workgroup then flushes its K x (D+1) partials into a global fp64 array
// with device atomics (global_atomic_add_f64). The map emits (cluster, sums,
// count) KVs from that array — GPMR's "emit (cluster, point) then combine"
// without materialising one KV per point.
#include "common.h"
#include "launch.h"
#include <cstdio>
#include <cstdlib>
#include <cfloat>

namespace mrh {
namespace k {
namespace {

constexpr int NT = 256;
constexpr int PTS_PER_THREAD = 8;

template <int D>
__global__ __launch_bounds__(NT) void k_kmeans(const float* __restrict__ pts, int64_t n,
                                              const float* __restrict__ cen, int K, double* __restrict__ acc) {
  extern __shared__ float sh[];
  float* c = sh;                 // K*D centroids
  float* part = sh + K * D;      // K*(D+1) partial sums (+count)
  for (int i = threadIdx.x; i < K * D; i += NT) c[i] = cen[i];
  for (int i = threadIdx.x; i < K * (D + 1); i += NT) part[i] = 0.f;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * NT * PTS_PER_THREAD;
#pragma unroll 1
  for (int r = 0; r < PTS_PER_THREAD; ++r) {
    const int64_t i = base + (int64_t)r * NT + threadIdx.x;  // coalesced across the block
    if (i >= n) break;
    float x[D];
#pragma unroll
    for (int d = 0; d < D; ++d) x[d] = pts[i * D + d];
    float best = FLT_MAX;
    int bk = 0;
    for (int kk = 0; kk < K; ++kk) {
      float dist = 0.f;
#pragma unroll
      for (int d = 0; d < D; ++d) {
        const float t = x[d] - c[kk * D + d];
        dist = fmaf(t, t, dist);
      }
      if (dist < best) {
        best = dist;
        bk = kk;
      }
    }
#pragma unroll
    for (int d = 0; d < D; ++d) atomicAdd(&part[bk * (D + 1) + d], x[d]);
    atomicAdd(&part[bk * (D + 1) + D], 1.f);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < K * (D + 1); i += NT)
    if (part[i] != 0.f) atomicAdd(&acc[i], (double)part[i]);
}

// Private-accumulator variant (K*(D+1) <= 120): every lane owns a column of
// LDS accumulators laid out [value][lane], so the per-point update is a plain
// conflict-free LDS read-modify-write (no atomics, no contention on popular
// clusters); the workgroup then reduces each accumulator row with one wave
// (64-lane shuffles) and issues one fp64 global atomic per row. Grid-stride
// over the points with a capped grid (~8 workgroups per CU), so each lane
// sees hundreds of points.
constexpr int PNT = 128;
template <int D>
__global__ __launch_bounds__(PNT) void k_kmeans_priv(const float* __restrict__ pts, int64_t n,
                                                    const float* __restrict__ cen, int K, double* __restrict__ acc) {
  extern __shared__ float sh[];
  const int R = K * (D + 1);
  float* c = sh;                    // K*D centroids
  float* priv = sh + ((K * D + 3) & ~3);  // R rows x PNT lanes
  for (int i = threadIdx.x; i < K * D; i += PNT) c[i] = cen[i];
  for (int i = threadIdx.x; i < R * PNT; i += PNT) priv[i] = 0.f;
  __syncthreads();
  const int64_t stride = (int64_t)gridDim.x * PNT;
  for (int64_t i = (int64_t)blockIdx.x * PNT + threadIdx.x; i < n; i += stride) {
    float x[D];
#pragma unroll
    for (int d = 0; d < D; ++d) x[d] = pts[i * D + d];
    float best = FLT_MAX;
    int bk = 0;
    for (int kk = 0; kk < K; ++kk) {
      float dist = 0.f;
#pragma unroll
      for (int d = 0; d < D; ++d) {
        const float t = x[d] - c[kk * D + d];
        dist = fmaf(t, t, dist);
      }
      if (dist < best) {
        best = dist;
        bk = kk;
      }
    }
    float* row = priv + (bk * (D + 1)) * PNT + threadIdx.x;
#pragma unroll
    for (int d = 0; d < D; ++d) row[d * PNT] += x[d];
    row[D * PNT] += 1.f;
  }
  __syncthreads();
  const int w = threadIdx.x / MRH_WAVE, l = dev::lane_id();
  for (int r = w; r < R; r += PNT / MRH_WAVE) {
    float v = 0.f;
#pragma unroll
    for (int j = 0; j < PNT / MRH_WAVE; ++j) v += priv[r * PNT + j * MRH_WAVE + l];
    v = dev::wave_sum(v);
    if (l == 0 && v != 0.f) atomicAdd(&acc[r], (double)v);
  }
}

// Batched variant: every lane loads its PB points up front (independent
// loads in flight instead of one dependent load per loop trip), scores
// centroids as ||c||^2 - 2 x.c from one 16-byte LDS broadcast read per
// centroid ({-2c, ||c||^2}, D <= 3), and adds into per-workgroup LDS
// partials with LDS float atomics.
constexpr int BNT = 256, PB = 8, BCMAX = 16;
template <int D>
__global__ __launch_bounds__(BNT) void k_kmeans_batch(const float* __restrict__ pts, int64_t n,
                                                     const float* __restrict__ cen, int K, int BC,
                                                     double* __restrict__ acc) {
  static_assert(D <= 3, "one float4 per centroid");
  extern __shared__ float sh[];
  float4* c4 = reinterpret_cast<float4*>(sh);      // K x {-2c0, -2c1, -2c2, |c|^2}
  // BC copies of the K*(D+1) partials, one per lane group (lane & (BC-1)),
  // rows at an odd stride RS so equal rows of different copies fall in
  // different banks: lanes of one wave instruction collide on an address
  // only when they share a copy AND a cluster
  const int R = K * (D + 1), RS = R | 1;
  float* part = sh + 4 * K;
  float* mine = part + (threadIdx.x & (BC - 1)) * RS;  // BC: power of two
  for (int kk = threadIdx.x; kk < K; kk += BNT) {
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    float cc = 0.f;
    for (int d = 0; d < D; ++d) {
      const float cd = cen[kk * D + d];
      v[d] = -2.f * cd;
      cc = fmaf(cd, cd, cc);
    }
    v[3] = cc;
    c4[kk] = make_float4(v[0], v[1], v[2], v[3]);
  }
  for (int i = threadIdx.x; i < BC * RS; i += BNT) part[i] = 0.f;
  __syncthreads();
  // grid-stride over tiles of BNT * PB points (any grid size is correct)
  const int64_t ntiles = (n + (int64_t)BNT * PB - 1) / ((int64_t)BNT * PB);
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int64_t base = tile * BNT * PB + threadIdx.x;
    float x[PB][D];
#pragma unroll
    for (int r = 0; r < PB; ++r) {
      const int64_t i = base + (int64_t)r * BNT;
#pragma unroll
      for (int d = 0; d < D; ++d) x[r][d] = (i < n) ? pts[i * D + d] : 0.f;
    }
    float best[PB];
    int bk[PB];
#pragma unroll
    for (int r = 0; r < PB; ++r) {
      best[r] = FLT_MAX;
      bk[r] = 0;
    }
    for (int kk = 0; kk < K; ++kk) {
      const float4 c = c4[kk];
#pragma unroll
      for (int r = 0; r < PB; ++r) {
        float sc = c.w;
        sc = fmaf(x[r][0], c.x, sc);
        if (D > 1) sc = fmaf(x[r][1], c.y, sc);
        if (D > 2) sc = fmaf(x[r][2], c.z, sc);
        const bool lt = sc < best[r];
        best[r] = lt ? sc : best[r];
        bk[r] = lt ? kk : bk[r];
      }
    }
#pragma unroll
    for (int r = 0; r < PB; ++r) {
      if (base + (int64_t)r * BNT >= n) break;
#pragma unroll
      for (int d = 0; d < D; ++d) atomicAdd(&mine[bk[r] * (D + 1) + d], x[r][d]);
      atomicAdd(&mine[bk[r] * (D + 1) + D], 1.f);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < R; i += BNT) {
    double v = 0.0;
    for (int c = 0; c < BC; ++c) v += (double)part[c * RS + i];
    if (v != 0.0) atomicAdd(&acc[i], v);
  }
}

// Transposed-reduction variant (default for D <= 3, K <= 256): no atomics
// in the point loop. PMC on the LDS-atomic kernels (profiles/r2_kmeans_tr.txt)
// showed the LDS array 92-93 % busy at ~200 LDS cycles per ds_add_f32 wave
// instruction — with one shared copy of the partials AND with 16 lane-group
// copies (no address collisions), i.e. LDS float atomics themselves run at
// ~3 cycles per lane. Per tile of 2048 points a workgroup
//   1. scores its points (8 per lane, {-2c, |c|^2} LDS broadcast) and
//      writes the tile's clusters and coordinates (point-major) to LDS;
//   2. transposes the reduction: lane l owns clusters l%32 (+32 g) and the
//      half l/32 of its wave's 512 points, and walks them with broadcast LDS
//      reads (4 points per ds_read_b128), adding the coordinates of the
//      points whose cluster it owns into registers (compare + select + add).
// Persistent grid; at the end the 8 owners of each (cluster, value) fold
// through LDS and the workgroup issues one fp64 global atomic per value.
constexpr int TNT = 256, TPB = 8, TTILE = TNT * TPB, TKG = 8;  // K <= 32 * TKG
template <int D, int KG>  // KG cluster groups of 32 per lane: K <= 32 * KG
__global__ __launch_bounds__(TNT) void k_kmeans_tr(const float* __restrict__ pts, int64_t n,
                                                  const float* __restrict__ cen, int K, double* __restrict__ acc) {
  static_assert(D <= 3, "one float4 per centroid");
  extern __shared__ float sh[];
  float4* c4 = reinterpret_cast<float4*>(sh);       // K x {-2c, |c|^2}
  int* sbk = reinterpret_cast<int*>(sh + 4 * K);    // TTILE cluster ids
  float* sx = sh + 4 * K + TTILE;                   // TTILE x D coordinates
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  for (int kk = tid; kk < K; kk += TNT) {
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    float cc = 0.f;
    for (int d = 0; d < D; ++d) {
      const float cd = cen[kk * D + d];
      v[d] = -2.f * cd;
      cc = fmaf(cd, cd, cc);
    }
    v[3] = cc;
    c4[kk] = make_float4(v[0], v[1], v[2], v[3]);
  }
  float s[KG][D];
  float cnt[KG];
#pragma unroll
  for (int g = 0; g < KG; ++g) {
    cnt[g] = 0.f;
#pragma unroll
    for (int d = 0; d < D; ++d) s[g][d] = 0.f;
  }
  const int own = lane & 31;
  const int j0 = w * (TTILE / 4) + (lane >> 5) * (TTILE / 8);  // this lane's 256 tile points
  const int64_t ntiles = (n + TTILE - 1) / TTILE;
  __syncthreads();
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int64_t base = tile * TTILE;
    float x[TPB][D];
#pragma unroll
    for (int r = 0; r < TPB; ++r) {
      const int64_t i = std::min<int64_t>(base + r * TNT + tid, n - 1);
#pragma unroll
      for (int d = 0; d < D; ++d) x[r][d] = pts[i * D + d];
    }
    float best[TPB];
    int bk[TPB];
#pragma unroll
    for (int r = 0; r < TPB; ++r) {
      best[r] = FLT_MAX;
      bk[r] = 0;
    }
    for (int kk = 0; kk < K; ++kk) {
      const float4 c = c4[kk];
#pragma unroll
      for (int r = 0; r < TPB; ++r) {
        float sc = c.w;
        sc = fmaf(x[r][0], c.x, sc);
        if (D > 1) sc = fmaf(x[r][1], c.y, sc);
        if (D > 2) sc = fmaf(x[r][2], c.z, sc);
        const bool lt = sc < best[r];
        best[r] = lt ? sc : best[r];
        bk[r] = lt ? kk : bk[r];
      }
    }
#pragma unroll
    for (int r = 0; r < TPB; ++r) {
      const int j = r * TNT + tid;
      sbk[j] = (base + j < n) ? bk[r] : -1;  // tail points belong to no cluster
#pragma unroll
      for (int d = 0; d < D; ++d) sx[j * D + d] = x[r][d];  // AoS: a point's coordinates adjacent
    }
    __syncthreads();
    for (int j = j0; j < j0 + TTILE / 8; j += 4) {
      const int4 b4 = *reinterpret_cast<const int4*>(sbk + j);
      float xs[4 * D];  // 4 points x D coordinates, D 16-byte broadcast reads
#pragma unroll
      for (int v = 0; v < D; ++v) {
        const float4 t = *reinterpret_cast<const float4*>(sx + j * D + 4 * v);
        xs[4 * v] = t.x;
        xs[4 * v + 1] = t.y;
        xs[4 * v + 2] = t.z;
        xs[4 * v + 3] = t.w;
      }
      const int bb[4] = {b4.x, b4.y, b4.z, b4.w};
#pragma unroll
      for (int g = 0; g < KG; ++g) {
        const int c = g * 32 + own;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          // one select + D+1 FMAs per point: the count rides along as a float
          // (exact: a lane adds at most ~n / (64 x grid) ones)
          const float m = bb[q] == c ? 1.f : 0.f;
          cnt[g] += m;
#pragma unroll
          for (int d = 0; d < D; ++d) s[g][d] = fmaf(m, xs[q * D + d], s[g][d]);
        }
      }
    }
    __syncthreads();
  }
  // fold the 8 owners (2 halves x 4 waves) of each (cluster, value) through
  // LDS (the tile buffers are free now), then one global atomic per value
  float* red = sx;  // [8 owners][K * (D+1)]
  const int R = K * (D + 1), owner = w * 2 + (lane >> 5);
  for (int g = 0; g < KG; ++g) {
    const int c = g * 32 + own;
    if (c < K) {
#pragma unroll
      for (int d = 0; d < D; ++d) red[owner * R + c * (D + 1) + d] = s[g][d];
      red[owner * R + c * (D + 1) + D] = cnt[g];
    }
  }
  __syncthreads();
  for (int i = tid; i < R; i += TNT) {
    double v = 0.0;
#pragma unroll
    for (int o = 0; o < 8; ++o) v += (double)red[o * R + i];
    if (v != 0.0) atomicAdd(&acc[i], v);
  }
}

// Register-accumulator variant (opt-in, MRH_KMEANS_KERNEL=4; K <= KM = 32,
// D <= 3) — an experiment kept for reference: PMC counters showed the
// batched kernel's waves spending ~60 % of their cycles waiting on LDS
// (SQ_WAIT_INST_LDS / SQ_WAVE_CYCLES) — the per-point LDS float atomics on a
// few hot cluster addresses. Here each lane keeps K x (D+1) running sums in
// VGPRs (a predicated FMA per cluster per point, no memory traffic), walks
// ~128 points grid-stride, and only at the end folds its registers with one
// fp64 wave reduction per accumulator + one global atomic per wave: 8192
// points per wave share each atomic instead of one LDS atomic per point.
constexpr int RNT = 256;
template <int D, int KM>
__global__ __launch_bounds__(RNT) void k_kmeans_reg(const float* __restrict__ pts, int64_t n,
                                                   const float* __restrict__ cen, int K, double* __restrict__ acc) {
  static_assert(D <= 3, "one float4 per centroid");
  __shared__ float4 c4[KM];
  for (int kk = threadIdx.x; kk < KM; kk += RNT) {
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    float cc = 0.f;
    if (kk < K) {
      for (int d = 0; d < D; ++d) {
        const float cd = cen[kk * D + d];
        v[d] = -2.f * cd;
        cc = fmaf(cd, cd, cc);
      }
      v[3] = cc;
    } else {
      v[3] = FLT_MAX;  // padding centroids never win
    }
    c4[kk] = make_float4(v[0], v[1], v[2], v[3]);
  }
  __syncthreads();
  float a[KM][D + 1];
#pragma unroll
  for (int kk = 0; kk < KM; ++kk)
#pragma unroll
    for (int d = 0; d <= D; ++d) a[kk][d] = 0.f;
  const int64_t stride = (int64_t)gridDim.x * RNT;
  for (int64_t i = (int64_t)blockIdx.x * RNT + threadIdx.x; i < n; i += stride) {
    float x[D];
#pragma unroll
    for (int d = 0; d < D; ++d) x[d] = pts[i * D + d];
    float best = FLT_MAX;
    int bk = 0;
#pragma unroll
    for (int kk = 0; kk < KM; ++kk) {
      const float4 c = c4[kk];
      float sc = c.w;
      sc = fmaf(x[0], c.x, sc);
      if (D > 1) sc = fmaf(x[1], c.y, sc);
      if (D > 2) sc = fmaf(x[2], c.z, sc);
      const bool lt = sc < best;
      best = lt ? sc : best;
      bk = lt ? kk : bk;
    }
#pragma unroll
    for (int kk = 0; kk < KM; ++kk) {
      const float m = kk == bk ? 1.f : 0.f;
#pragma unroll
      for (int d = 0; d < D; ++d) a[kk][d] = fmaf(m, x[d], a[kk][d]);
      a[kk][D] += m;
    }
  }
  // fold in fp64 (per-lane fp32 sums cover only ~128 points): one wave
  // reduction per accumulator, one fp64 global atomic per wave
  const int lane = dev::lane_id();
#pragma unroll
  for (int kk = 0; kk < KM; ++kk)
#pragma unroll
    for (int d = 0; d <= D; ++d) {
      const double v = dev::wave_sum((double)a[kk][d]);
      if (lane == 0 && kk < K && v != 0.0) atomicAdd(&acc[kk * (D + 1) + d], v);
    }
}

// ---------------------------------------------------------------- matrix-core kernel (D > 8)
// Higher dimensions score on the matrix cores: x.c is a [points x D] x
// [D x centroids] product, computed per wave on 16-point x 16-centroid tiles
// with v_mfma_f32_16x16x4_f32 (exact f32: one fmaf per product, k-ordered,
// the same numerics as the VALU path) and consumed in registers — the score
// matrix never exists in memory (the hipBLASLt GEMM + argmin it replaces
// wrote and re-read N x K floats). Per wave step:
//   A (points): lane l holds dims 4kk + (l>>4) of point (l&15), kk < DP/4,
//               loaded once per 16 points;
//   B (centroids, LDS): lane l reads c[j][4kk + (l>>4)] of centroid j = l&15
//               of the tile; two centroid tiles in flight (independent
//               accumulators cover the 40-cycle MFMA latency);
//   D: lane l holds x.c for points 4(l>>4)+r (r < 4) against centroid l&15;
//   score = |c|^2 - 2 x.c, running argmin per (point, lane column), then a
//   16-lane butterfly (ties -> lower centroid index: first-minimum, as argmin).
// The winning centroid of each point goes through LDS back to the lanes that
// hold its coordinates, which add them into the workgroup's LDS partials.
constexpr int MNT = 256, MNW = MNT / MRH_WAVE;
template <int DP>
__global__ __launch_bounds__(MNT) void k_kmeans_mfma(const float* __restrict__ pts, int64_t n, int D,
                                                    const float* __restrict__ cen, int K, int KP,
                                                    double* __restrict__ acc) {
  extern __shared__ float sh[];
  float* cs = sh;                   // [KP][DP] centroids, zero padded
  float* cn = cs + (size_t)KP * DP;  // [KP] |c|^2 (padding centroids: +inf)
  float* part = cn + KP;            // [K][D+1] workgroup partial sums / counts
  __shared__ int bestk[MNW][16];
  for (int i = threadIdx.x; i < KP * DP; i += MNT) {
    const int j = i / DP, d = i % DP;
    cs[i] = (j < K && d < D) ? cen[(size_t)j * D + d] : 0.f;
  }
  for (int j = threadIdx.x; j < KP; j += MNT) {
    float v = 0.f;
    if (j < K)
      for (int d = 0; d < D; ++d) v = fmaf(cen[(size_t)j * D + d], cen[(size_t)j * D + d], v);
    cn[j] = j < K ? v : FLT_MAX;
  }
  for (int i = threadIdx.x; i < K * (D + 1); i += MNT) part[i] = 0.f;
  __syncthreads();
  const int l = dev::lane_id(), w = dev::wave_id();
  const int row = l & 15, kq = l >> 4;  // A: point row, k lane-quarter; D: column = row, rows 4kq..4kq+3
  constexpr int KK = DP / 4;
  for (int64_t p0 = ((int64_t)blockIdx.x * MNW + w) * 16; p0 < n; p0 += (int64_t)gridDim.x * MNW * 16) {
    const int64_t pr = p0 + row;
    float a[KK];
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      const int d = 4 * kk + kq;
      a[kk] = (pr < n && d < D) ? pts[pr * D + d] : 0.f;
    }
    float bv[4] = {FLT_MAX, FLT_MAX, FLT_MAX, FLT_MAX};
    int bk[4] = {0, 0, 0, 0};
    for (int jt = 0; jt < KP; jt += 32) {  // two 16-centroid tiles per trip
      typedef float f4 __attribute__((ext_vector_type(4)));
      f4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = {0.f, 0.f, 0.f, 0.f};
      const float* b0 = cs + (size_t)(jt + row) * DP + kq;
      const float* b1 = b0 + 16 * DP;
      const bool two = jt + 16 < KP;
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) {
        c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[kk], b0[4 * kk], c0, 0, 0, 0);
        if (two) c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[kk], b1[4 * kk], c1, 0, 0, 0);
      }
      const float n0 = cn[jt + row], n1 = two ? cn[jt + 16 + row] : FLT_MAX;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float s0 = fmaf(-2.f, c0[r], n0);
        if (s0 < bv[r]) { bv[r] = s0; bk[r] = jt + row; }
        const float s1 = fmaf(-2.f, c1[r], n1);
        if (two && s1 < bv[r]) { bv[r] = s1; bk[r] = jt + 16 + row; }
      }
    }
    // argmin across the 16 lanes (centroid columns) of each lane quarter
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        const float ov = __shfl_xor(bv[r], o, MRH_WAVE);
        const int ok = __shfl_xor(bk[r], o, MRH_WAVE);
        if (ov < bv[r] || (ov == bv[r] && ok < bk[r])) { bv[r] = ov; bk[r] = ok; }
      }
      if (row == 0) bestk[w][4 * kq + r] = bk[r];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (pr < n) {
      const int k = bestk[w][row];
      float* dst = part + (size_t)k * (D + 1);
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) {
        const int d = 4 * kk + kq;
        if (d < D) atomicAdd(dst + d, a[kk]);
      }
      if (kq == 0) atomicAdd(dst + D, 1.f);
    }
    __builtin_amdgcn_wave_barrier();
  }
  __syncthreads();
  for (int i = threadIdx.x; i < K * (D + 1); i += MNT)
    if (part[i] != 0.f) atomicAdd(&acc[i], (double)part[i]);
}

// combine of the library-GEMM path (D > 128): points with their argmin
// cluster -> LDS partial sums (or fp64 global atomics when K*(D+1) floats
// exceed LDS), one fp64 atomic per partial per workgroup
__global__ __launch_bounds__(MNT) void k_kmeans_accum(const float* __restrict__ pts, int64_t n, int D,
                                                     const int64_t* __restrict__ idx, int K, bool lds_part,
                                                     double* __restrict__ acc) {
  extern __shared__ float part[];
  const int R = K * (D + 1);
  if (lds_part) {
    for (int i = threadIdx.x; i < R; i += MNT) part[i] = 0.f;
    __syncthreads();
  }
  const int l = dev::lane_id();
  for (int64_t p = (int64_t)blockIdx.x * MNW + dev::wave_id(); p < n; p += (int64_t)gridDim.x * MNW) {
    const int64_t k = idx[p];
    for (int d = l; d <= D; d += MRH_WAVE) {
      const float v = d < D ? pts[p * D + d] : 1.f;
      if (lds_part) atomicAdd(&part[k * (D + 1) + d], v);
      else atomicAdd(&acc[k * (D + 1) + d], (double)v);
    }
  }
  if (!lds_part) return;
  __syncthreads();
  for (int i = threadIdx.x; i < R; i += MNT)
    if (part[i] != 0.f) atomicAdd(&acc[i], (double)part[i]);
}

int mfma_dp(int D) { return D <= 16 ? 16 : D <= 32 ? 32 : D <= 64 ? 64 : D <= 128 ? 128 : 0; }
size_t mfma_lds(int D, int K) {
  const int DP = mfma_dp(D), KP = (K + 15) & ~15;
  return sizeof(float) * ((size_t)KP * DP + KP + (size_t)K * (D + 1));
}
constexpr size_t kMfmaLds = 120 * 1024;

void launch_mfma(const float* pts, int64_t n, int D, const float* cen, int K, double* acc, hipStream_t s) {
  const int KP = (K + 15) & ~15;
  const size_t lds = mfma_lds(D, K);
  int64_t nb = (n + MNW * 16 - 1) / (MNW * 16);
  if (nb > 2048) nb = 2048;  // each workgroup walks ~16 K points before flushing its partials
  switch (mfma_dp(D)) {
    case 16: hipLaunchKernelGGL((k_kmeans_mfma<16>), dim3((unsigned)nb), dim3(MNT), lds, s, pts, n, D, cen, K, KP, acc); break;
    case 32: hipLaunchKernelGGL((k_kmeans_mfma<32>), dim3((unsigned)nb), dim3(MNT), lds, s, pts, n, D, cen, K, KP, acc); break;
    case 64: hipLaunchKernelGGL((k_kmeans_mfma<64>), dim3((unsigned)nb), dim3(MNT), lds, s, pts, n, D, cen, K, KP, acc); break;
    default: hipLaunchKernelGGL((k_kmeans_mfma<128>), dim3((unsigned)nb), dim3(MNT), lds, s, pts, n, D, cen, K, KP, acc); break;
  }
  MRH_CHECK_LAUNCH();
}

inline size_t batch_lds(int D, int K, int bc) { return sizeof(float) * ((size_t)4 * K + (size_t)bc * ((K * (D + 1)) | 1)); }
// centroids + one tile's (cluster, coordinates) SoA; the final fold reuses
// the coordinate buffer for 8 x K*(D+1) partials
inline size_t tr_lds(int D, int K) {
  return sizeof(float) * ((size_t)4 * K + TTILE + std::max<size_t>((size_t)D * TTILE, (size_t)8 * K * (D + 1)));
}
// copies of the partials: as many (<= 16) as fit in 64 KB with the centroids
inline int batch_copies(int D, int K) {
  int bc = BCMAX;
  while (bc > 1 && batch_lds(D, K, bc) > 64 * 1024) bc >>= 1;
  return bc;
}

template <int D>
void launch(const float* pts, int64_t n, const float* cen, int K, double* acc, hipStream_t s) {
  static const int variant = [] {
    const char* e = std::getenv("MRH_KMEANS_KERNEL");
    return e ? std::atoi(e) : 0;
  }();
  if constexpr (D <= 3) {
    // MRH_KMEANS_KERNEL=4: the register-accumulator kernel. Measured slower
    // (26.0 vs 15.8 ms per 20 iterations, profiles/r1_kmeans_variants.txt):
    // its 128 predicated FMAs per point cost more than the LDS-atomic waits
    // they remove.
    if (variant == 4 && K <= 32) {
      int64_t nb = (n + RNT - 1) / RNT;
      if (nb > 1024) nb = 1024;  // ~128 points per lane at 32 M points
      hipLaunchKernelGGL((k_kmeans_reg<D, 32>), dim3((unsigned)nb), dim3(RNT), 0, s, pts, n, cen, K, acc);
      MRH_CHECK_LAUNCH();
      return;
    }
    // default: the transposed-reduction kernel; MRH_KMEANS_KERNEL=6 keeps
    // the LDS-atomic batched kernel (5: with one shared partial copy)
    if (variant == 0 && K <= 32 * TKG && tr_lds(D, K) <= 64 * 1024) {
      static const int ncu = [] {
        int dev = 0, c = 0;
        MRH_HIP(hipGetDevice(&dev));
        MRH_HIP(hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev));
        return std::max(1, c);
      }();
      int64_t nb = (n + TTILE - 1) / TTILE;
      if (nb > (int64_t)ncu * 8) nb = (int64_t)ncu * 8;  // persistent: ~8 workgroups per CU
      const size_t lds = tr_lds(D, K);
      if (K <= 32) hipLaunchKernelGGL((k_kmeans_tr<D, 1>), dim3((unsigned)nb), dim3(TNT), lds, s, pts, n, cen, K, acc);
      else if (K <= 64) hipLaunchKernelGGL((k_kmeans_tr<D, 2>), dim3((unsigned)nb), dim3(TNT), lds, s, pts, n, cen, K, acc);
      else if (K <= 128) hipLaunchKernelGGL((k_kmeans_tr<D, 4>), dim3((unsigned)nb), dim3(TNT), lds, s, pts, n, cen, K, acc);
      else hipLaunchKernelGGL((k_kmeans_tr<D, TKG>), dim3((unsigned)nb), dim3(TNT), lds, s, pts, n, cen, K, acc);
      MRH_CHECK_LAUNCH();
      return;
    }
    if (variant != 1 && batch_lds(D, K, 1) <= 64 * 1024) {
      const int bc = variant == 5 ? 1 : batch_copies(D, K);  // 5: one shared copy (the r1 kernel)
      // one workgroup per tile: capping the grid (fewer fp64 flush atomics)
      // measured no faster (profiles/r2_kmeans_tr.txt)
      const int64_t nb = (n + (int64_t)BNT * PB - 1) / ((int64_t)BNT * PB);
      const size_t lds = batch_lds(D, K, bc);
      hipLaunchKernelGGL((k_kmeans_batch<D>), dim3((unsigned)nb), dim3(BNT), lds, s, pts, n, cen, K, bc, acc);
      MRH_CHECK_LAUNCH();
      return;
    }
  }
  if (variant == 1 && K * (D + 1) <= 120) {  // <= 61.5 KB of private accumulators
    int64_t nb = (n + PNT - 1) / PNT;
    if (nb > 2048) nb = 2048;
    const size_t lds = sizeof(float) * (size_t)(((K * D + 3) & ~3) + K * (D + 1) * PNT);
    hipLaunchKernelGGL((k_kmeans_priv<D>), dim3((unsigned)nb), dim3(PNT), lds, s, pts, n, cen, K, acc);
    MRH_CHECK_LAUNCH();
    return;
  }
  const int64_t nb = (n + (int64_t)NT * PTS_PER_THREAD - 1) / ((int64_t)NT * PTS_PER_THREAD);
  const size_t lds = sizeof(float) * (size_t)K * (2 * D + 1);
  hipLaunchKernelGGL((k_kmeans<D>), dim3((unsigned)nb), dim3(NT), lds, s, pts, n, cen, K, acc);
  MRH_CHECK_LAUNCH();
}

}  // namespace

// fp32 LDS partials hold at most NT*PTS_PER_THREAD = 2048 points per workgroup,
// so per-cluster counts are exact and sums lose no more than fp32 rounding of
// 2048 terms before the fp64 global accumulation.
void kmeans_accumulate(const float* pts, int64_t n, int D, const int64_t* idx, int K, double* acc, hipStream_t s) {
  if (n <= 0) return;
  const size_t lds = sizeof(float) * (size_t)K * (D + 1);
  const bool lds_part = lds <= 64 * 1024;
  int64_t nb = (n + MNW - 1) / MNW;
  if (nb > 2048) nb = 2048;
  hipLaunchKernelGGL(k_kmeans_accum, dim3((unsigned)nb), dim3(MNT), lds_part ? lds : 0, s, pts, n, D, idx, K, lds_part,
                     acc);
  MRH_CHECK_LAUNCH();
}

bool kmeans_supported(int D, int K) {
  if (K < 1 || D < 1) return false;
  if ((D == 1 || D == 2 || D == 3 || D == 4 || D == 8) && (size_t)K * (2 * D + 1) * 4 <= 64 * 1024) return true;
  return mfma_dp(D) && mfma_lds(D, K) <= kMfmaLds;  // matrix-core kernel
}
// (the private-accumulator kernel uses < 62 KB of LDS: K*(D+1) <= 120 rows x 128 lanes + centroids)

void kmeans_assign_accumulate(const float* pts, int64_t n, int D, const float* cen, int K, double* acc,
                              hipStream_t s) {
  if (n <= 0) return;
  const bool small = (size_t)K * (2 * D + 1) * 4 <= 64 * 1024;
  switch (small ? D : 0) {
    case 1: launch<1>(pts, n, cen, K, acc, s); break;
    case 2: launch<2>(pts, n, cen, K, acc, s); break;
    case 3: launch<3>(pts, n, cen, K, acc, s); break;
    case 4: launch<4>(pts, n, cen, K, acc, s); break;
    case 8: launch<8>(pts, n, cen, K, acc, s); break;
    default:
      check_arg(mfma_dp(D) && mfma_lds(D, K) <= kMfmaLds, "kmeans: unsupported (dimension, clusters)");
      launch_mfma(pts, n, D, cen, K, acc, s);
  }
}

}  // namespace k
}  // namespace mrh
