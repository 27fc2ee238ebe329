// Small engine primitives that used to be ATen tensor expressions on the
// engine's hot paths (min/max probes, fills, offset rebases, the hash ->
// partition map of the out-of-core convert, tri_find_mr's edge callbacks).
// Each ATen expression was one or more at::native / rocPRIM kernels plus
// TensorIterator host overhead per call; these are one launch each, on the
// caller's stream, with no host synchronisation of their own.
#include "common.h"
#include "launch.h"

#include <climits>

namespace mrh {
namespace k {
namespace {

constexpr int NT = 256;
constexpr int MAXB = 1024;  // partial blocks of the two-pass reductions

inline unsigned grid_for(int64_t n, int cap = 4096) {
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + NT - 1) / NT, cap));
}

__device__ __forceinline__ int64_t wave_min(int64_t v) {
  for (int d = 32; d > 0; d >>= 1) v = min(v, (int64_t)__shfl_xor(v, d, 64));
  return v;
}
__device__ __forceinline__ int64_t wave_max(int64_t v) {
  for (int d = 32; d > 0; d >>= 1) v = max(v, (int64_t)__shfl_xor(v, d, 64));
  return v;
}

// per column of a row-major [rows, cols] int64 matrix (cols <= 8): block
// partials part[b][0..cols) = minima, part[b][cols..2cols) = maxima
__global__ __launch_bounds__(NT) void k_col_minmax_part(const int64_t* __restrict__ p, int64_t rows, int cols,
                                                        int64_t* __restrict__ part) {
  __shared__ int64_t smn[NT / 64][8], smx[NT / 64][8];
  int64_t mn[8], mx[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    mn[c] = LLONG_MAX;
    mx[c] = LLONG_MIN;
  }
  for (int64_t r = (int64_t)blockIdx.x * NT + threadIdx.x; r < rows; r += (int64_t)gridDim.x * NT) {
#pragma unroll
    for (int c = 0; c < 8; ++c)
      if (c < cols) {
        const int64_t v = p[r * cols + c];
        mn[c] = min(mn[c], v);
        mx[c] = max(mx[c], v);
      }
  }
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    if (c >= cols) break;
    const int64_t a = wave_min(mn[c]), b = wave_max(mx[c]);
    if (lane == 0) {
      smn[w][c] = a;
      smx[w][c] = b;
    }
  }
  __syncthreads();
  if (threadIdx.x < cols) {
    int64_t a = LLONG_MAX, b = LLONG_MIN;
    for (int i = 0; i < NT / 64; ++i) {
      a = min(a, smn[i][threadIdx.x]);
      b = max(b, smx[i][threadIdx.x]);
    }
    part[(int64_t)blockIdx.x * 2 * cols + threadIdx.x] = a;
    part[(int64_t)blockIdx.x * 2 * cols + cols + threadIdx.x] = b;
  }
}

// fold nb partial rows of `width` words into out[0..width): columns
// [0, nmin) by min, the rest by max (one block)
__global__ __launch_bounds__(NT) void k_minmax_fold(const int64_t* __restrict__ part, int nb, int width, int nmin,
                                                    int64_t* __restrict__ out) {
  __shared__ int64_t s[NT];
  for (int j = 0; j < width; ++j) {
    const bool is_min = j < nmin;
    int64_t v = is_min ? LLONG_MAX : LLONG_MIN;
    for (int b = threadIdx.x; b < nb; b += NT) {
      const int64_t x = part[(int64_t)b * width + j];
      v = is_min ? min(v, x) : max(v, x);
    }
    s[threadIdx.x] = v;
    __syncthreads();
    for (int d = NT / 2; d > 0; d >>= 1) {
      if (threadIdx.x < d)
        s[threadIdx.x] = is_min ? min(s[threadIdx.x], s[threadIdx.x + d]) : max(s[threadIdx.x], s[threadIdx.x + d]);
      __syncthreads();
    }
    if (threadIdx.x == 0) out[j] = s[0];
    __syncthreads();
  }
}

// int32 values widened: part rows of (min, max)
__global__ __launch_bounds__(NT) void k_minmax_i32_part(const int32_t* __restrict__ p, int64_t n,
                                                        int64_t* __restrict__ part) {
  __shared__ int64_t smn[NT / 64], smx[NT / 64];
  int64_t mn = LLONG_MAX, mx = LLONG_MIN;
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) {
    const int64_t v = p[i];
    mn = min(mn, v);
    mx = max(mx, v);
  }
  mn = wave_min(mn);
  mx = wave_max(mx);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    smn[w] = mn;
    smx[w] = mx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < NT / 64; ++i) {
      mn = min(mn, smn[i]);
      mx = max(mx, smx[i]);
    }
    mn = min(mn, smn[0]);
    mx = max(mx, smx[0]);
    part[2 * blockIdx.x] = mn;
    part[2 * blockIdx.x + 1] = mx;
  }
}

__global__ __launch_bounds__(NT) void k_fill_i64(int64_t* __restrict__ p, int64_t n, int64_t v) {
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) p[i] = v;
}

__global__ __launch_bounds__(NT) void k_add_i64(const int64_t* __restrict__ src, int64_t* __restrict__ dst, int64_t n,
                                                int64_t v) {
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) dst[i] = src[i] + v;
}

// partition of a 64-bit grouping hash: ((h >> shift) & mask) % M
__global__ __launch_bounds__(NT) void k_part_of_hash(const uint64_t* __restrict__ h, int64_t n, int shift,
                                                     uint64_t mask, int M, int32_t* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT)
    out[i] = (int32_t)(((h[i] >> shift) & mask) % (uint64_t)M);
}

// edges [n, 2] -> part rows (min of both ends, any a >= b, max of both ends)
__global__ __launch_bounds__(NT) void k_edge_probe_part(const int64_t* __restrict__ e, int64_t n,
                                                        int64_t* __restrict__ part) {
  __shared__ int64_t sb[NT / 64], smn[NT / 64], smx[NT / 64];
  int64_t bad = 0, mn = LLONG_MAX, mx = LLONG_MIN;
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) {
    const int64_t a = e[2 * i], b = e[2 * i + 1];
    bad |= a >= b ? 1 : 0;
    mn = min(mn, min(a, b));
    mx = max(mx, max(a, b));
  }
  bad = wave_max(bad);
  mn = wave_min(mn);
  mx = wave_max(mx);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    sb[w] = bad;
    smn[w] = mn;
    smx[w] = mx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 0; i < NT / 64; ++i) {
      bad = max(bad, sb[i]);
      mn = min(mn, smn[i]);
      mx = max(mx, smx[i]);
    }
    part[3 * blockIdx.x] = mn;  // (min, any a >= b, max)
    part[3 * blockIdx.x + 1] = bad;
    part[3 * blockIdx.x + 2] = mx;
  }
}

// (a, b) -> keys [a..., b...], values [b..., a...]
__global__ __launch_bounds__(NT) void k_edge_both_ways(const int64_t* __restrict__ e, int64_t n,
                                                       int64_t* __restrict__ key, int64_t* __restrict__ val) {
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) {
    const int64_t a = e[2 * i], b = e[2 * i + 1];
    key[i] = a;
    val[i] = b;
    key[n + i] = b;
    val[n + i] = a;
  }
}

// (a, b) -> key a << vb | b (u64), value a (int32)
__global__ __launch_bounds__(NT) void k_edge_pack(const int64_t* __restrict__ e, int64_t n, int vb,
                                                  uint64_t* __restrict__ key, int32_t* __restrict__ val) {
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) {
    const int64_t a = e[2 * i], b = e[2 * i + 1];
    key[i] = ((uint64_t)a << vb) | (uint64_t)b;
    val[i] = (int32_t)a;
  }
}

// (a, b) -> value a (int64), the "marked by vertex" layout
__global__ __launch_bounds__(NT) void k_edge_first(const int64_t* __restrict__ e, int64_t n, int64_t* __restrict__ val) {
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) val[i] = e[2 * i];
}

// edge_upper: flag[i] = (a != b), then (min, max) of the flagged rows at
// their exclusive-scan positions
__global__ __launch_bounds__(NT) void k_edge_ne_flags(const int64_t* __restrict__ e, int64_t n,
                                                      uint32_t* __restrict__ flag) {
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT)
    flag[i] = e[2 * i] != e[2 * i + 1] ? 1u : 0u;
}
__global__ __launch_bounds__(NT) void k_edge_upper_write(const int64_t* __restrict__ e, int64_t n,
                                                         const uint32_t* __restrict__ pos, int64_t* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) {
    const int64_t a = e[2 * i], b = e[2 * i + 1];
    if (a == b) continue;
    const int64_t o = pos[i];
    out[2 * o] = min(a, b);
    out[2 * o + 1] = max(a, b);
  }
}

// zero-copy gather: block (x, p) copies its stride of piece p from pinned
// host memory (device-accessible) into dst; dword granularity when the piece
// allows, bytes otherwise
__global__ __launch_bounds__(NT) void k_gather_pieces(PieceTable t, uint8_t* __restrict__ dst) {
  const int p = blockIdx.y;
  if (p >= t.n) return;
  const uint8_t* __restrict__ s = t.src[p];
  uint8_t* __restrict__ d = dst + t.dst_off[p];
  const int64_t n = t.bytes[p];
  const int64_t tid = (int64_t)blockIdx.x * NT + threadIdx.x, nth = (int64_t)gridDim.x * NT;
  if ((((uintptr_t)s | (uintptr_t)d | (uintptr_t)n) & 3) == 0) {
    const uint32_t* __restrict__ s4 = reinterpret_cast<const uint32_t*>(s);
    uint32_t* __restrict__ d4 = reinterpret_cast<uint32_t*>(d);
    const int64_t w = n >> 2;
    for (int64_t i = tid * 4; i < w; i += nth * 4) {  // four dwords in flight per thread
      if (i + 3 < w) {
        const uint32_t a = __builtin_nontemporal_load(s4 + i), b = __builtin_nontemporal_load(s4 + i + 1);
        const uint32_t c = __builtin_nontemporal_load(s4 + i + 2), e = __builtin_nontemporal_load(s4 + i + 3);
        d4[i] = a;
        d4[i + 1] = b;
        d4[i + 2] = c;
        d4[i + 3] = e;
      } else {
        for (int64_t j = i; j < w; ++j) d4[j] = s4[j];
      }
    }
  } else {
    for (int64_t i = tid; i < n; i += nth) d[i] = s[i];
  }
}

}  // namespace

void gather_pieces(const PieceTable& t, uint8_t* dst, hipStream_t s) {
  if (t.n <= 0) return;
  check_arg(t.n <= PieceTable::kMax, "gather_pieces: too many pieces");
  int64_t mx = 0;
  for (int i = 0; i < t.n; ++i) mx = std::max<int64_t>(mx, t.bytes[i]);
  // ~64 KiB of a piece per block, at most 64 blocks on one piece
  const unsigned gx = (unsigned)std::max<int64_t>(1, std::min<int64_t>(64, (mx + 65535) / 65536));
  hipLaunchKernelGGL(k_gather_pieces, dim3(gx, (unsigned)t.n), dim3(NT), 0, s, t, dst);
  MRH_CHECK_LAUNCH();
}

void edge_ne_flags(const int64_t* e, int64_t n, uint32_t* flag, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_edge_ne_flags, dim3(grid_for(n)), dim3(NT), 0, s, e, n, flag);
  MRH_CHECK_LAUNCH();
}

void edge_upper_write(const int64_t* e, int64_t n, const uint32_t* pos, int64_t* out, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_edge_upper_write, dim3(grid_for(n)), dim3(NT), 0, s, e, n, pos, out);
  MRH_CHECK_LAUNCH();
}

int64_t minmax_scratch_words(int64_t rows, int cols) { return (int64_t)grid_for(rows, MAXB) * 2 * cols + 2 * cols; }

void col_minmax_i64(const int64_t* p, int64_t rows, int cols, int64_t* scratch, int64_t* out, hipStream_t s) {
  check_arg(cols >= 1 && cols <= 8, "col_minmax_i64: 1..8 columns");
  const unsigned nb = grid_for(rows, MAXB);
  hipLaunchKernelGGL(k_col_minmax_part, dim3(nb), dim3(NT), 0, s, p, rows, cols, scratch);
  MRH_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_minmax_fold, dim3(1), dim3(NT), 0, s, scratch, (int)nb, 2 * cols, cols, out);
  MRH_CHECK_LAUNCH();
}

void minmax_i32(const int32_t* p, int64_t n, int64_t* scratch, int64_t* out, hipStream_t s) {
  const unsigned nb = grid_for(n, MAXB);
  hipLaunchKernelGGL(k_minmax_i32_part, dim3(nb), dim3(NT), 0, s, p, n, scratch);
  MRH_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_minmax_fold, dim3(1), dim3(NT), 0, s, scratch, (int)nb, 2, 1, out);
  MRH_CHECK_LAUNCH();
}

void fill_i64(int64_t* p, int64_t n, int64_t v, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_fill_i64, dim3(grid_for(n)), dim3(NT), 0, s, p, n, v);
  MRH_CHECK_LAUNCH();
}

void add_i64(const int64_t* src, int64_t* dst, int64_t n, int64_t v, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_add_i64, dim3(grid_for(n)), dim3(NT), 0, s, src, dst, n, v);
  MRH_CHECK_LAUNCH();
}

void part_of_hash(const uint64_t* h, int64_t n, int shift, uint64_t mask, int M, int32_t* out, hipStream_t s) {
  if (n <= 0) return;
  check_arg(M >= 1, "part_of_hash: M >= 1");
  hipLaunchKernelGGL(k_part_of_hash, dim3(grid_for(n)), dim3(NT), 0, s, h, n, shift, mask, M, out);
  MRH_CHECK_LAUNCH();
}

void edge_probe(const int64_t* e, int64_t n, int64_t* scratch, int64_t* out, hipStream_t s) {
  const unsigned nb = grid_for(n, MAXB);
  hipLaunchKernelGGL(k_edge_probe_part, dim3(nb), dim3(NT), 0, s, e, n, scratch);
  MRH_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_minmax_fold, dim3(1), dim3(NT), 0, s, scratch, (int)nb, 3, 1, out);
  MRH_CHECK_LAUNCH();
}

void edge_both_ways(const int64_t* e, int64_t n, int64_t* key, int64_t* val, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_edge_both_ways, dim3(grid_for(n)), dim3(NT), 0, s, e, n, key, val);
  MRH_CHECK_LAUNCH();
}

void edge_pack(const int64_t* e, int64_t n, int vb, uint64_t* key, int32_t* val, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_edge_pack, dim3(grid_for(n)), dim3(NT), 0, s, e, n, vb, key, val);
  MRH_CHECK_LAUNCH();
}

void edge_first(const int64_t* e, int64_t n, int64_t* val, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_edge_first, dim3(grid_for(n)), dim3(NT), 0, s, e, n, val);
  MRH_CHECK_LAUNCH();
}

}  // namespace k
}  // namespace mrh
