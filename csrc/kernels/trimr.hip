// tri_find_mr: the reference's 4-shuffle triangle pipeline callbacks
// (oink/tri_find.cpp:104-325) as device kernels on the KMV / KV columns.
//
//  k_first_degree   reduce_first_degree (:133-158): every value j of vertex
//                   segment s -> edge (min, max) of (key[s], nbr[j]) with the
//                   degree |s| in the slot of key[s] ({d, 0} or {0, d});
//                   one lane per value, segment by binary search of seg (the
//                   KMV may hold one hub segment of millions of values, so
//                   work is split by value, not by segment)
//  k_second_degree  reduce_second_degree (:164-189): an edge's two records
//                   {di, 0} / {0, dj} merged into {di, dj}
//  k_low_degree     map_low_degree (:195-205): edge keyed by its lower-degree
//                   end (ties: lower id), value = the other end
//  k_emit_count /   reduce_emit_triangles (:282-325): an edge segment that
//  k_emit_write     holds the edge marker (0-byte value) closes every wedge
//                   centre (8-byte value) in it; count per segment, exclusive
//                   scan, write (centre, e0, e1) rows
#include <algorithm>

#include "common.h"
#include "launch.h"

namespace mrh {
namespace k {
namespace {

constexpr int NT = 256;
inline unsigned blocks(int64_t n) { return (unsigned)std::min<int64_t>((n + NT - 1) / NT, 1 << 20); }

// largest s in [0, nseg) with seg[s] <= j (the non-empty segment holding j)
__device__ inline int64_t seg_of(const int64_t* __restrict__ seg, int64_t nseg, int64_t j) {
  int64_t lo = 0, hi = nseg;
  while (hi - lo > 1) {
    const int64_t mid = (lo + hi) >> 1;
    if (seg[mid] <= j) lo = mid;
    else hi = mid;
  }
  return lo;
}

__global__ __launch_bounds__(NT) void k_first_degree(const int64_t* __restrict__ seg, int64_t nkey,
                                                    const int64_t* __restrict__ key, const int64_t* __restrict__ nbr,
                                                    int64_t nval, int64_t* __restrict__ edge,
                                                    int32_t* __restrict__ deg) {
  for (int64_t j = (int64_t)blockIdx.x * NT + threadIdx.x; j < nval; j += (int64_t)gridDim.x * NT) {
    const int64_t s = seg_of(seg, nkey, j);
    const int64_t vi = key[s], vj = nbr[j];
    const int32_t d = (int32_t)(seg[s + 1] - seg[s]);
    const bool lt = vi < vj;
    edge[2 * j] = lt ? vi : vj;
    edge[2 * j + 1] = lt ? vj : vi;
    deg[2 * j] = lt ? d : 0;
    deg[2 * j + 1] = lt ? 0 : d;
  }
}

__global__ __launch_bounds__(NT) void k_second_degree(const int64_t* __restrict__ seg, int64_t nkey,
                                                     const int2* __restrict__ v, int64_t nval,
                                                     int2* __restrict__ out) {
  for (int64_t s = (int64_t)blockIdx.x * NT + threadIdx.x; s < nkey; s += (int64_t)gridDim.x * NT) {
    const int64_t h = seg[s];
    const int2 one = v[h], two = v[h + 1 < nval ? h + 1 : nval - 1];
    const bool use1 = one.x != 0;
    out[s] = make_int2(use1 ? one.x : two.x, use1 ? two.y : one.y);
  }
}

__global__ __launch_bounds__(NT) void k_low_degree(const int64_t* __restrict__ e, const int2* __restrict__ dg,
                                                  int64_t n, int64_t* __restrict__ key, int64_t* __restrict__ val) {
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) {
    const int64_t vi = e[2 * i], vj = e[2 * i + 1];
    const int2 d = dg[i];
    const bool fi = d.x < d.y || (d.x == d.y && vi < vj);
    key[i] = fi ? vi : vj;
    val[i] = fi ? vj : vi;
  }
}

// the wedge centres of the EDGE keys that are also edges: a marker value is
// either empty (voff given: variable-width values) or -1 (voff null: fixed
// 8-byte values, vals)
__global__ __launch_bounds__(NT) void k_emit_count(const int64_t* __restrict__ seg, int64_t nkey,
                                                  const int64_t* __restrict__ voff, const int64_t* __restrict__ vals,
                                                  int64_t* __restrict__ cnt) {
  for (int64_t s = (int64_t)blockIdx.x * NT + threadIdx.x; s < nkey; s += (int64_t)gridDim.x * NT) {
    int64_t c = 0;
    bool marker = false;
    for (int64_t j = seg[s]; j < seg[s + 1]; ++j) {
      if (!voff) {  // fixed 8-byte values: the edge marker is the value -1
        const bool m = vals[j] == -1;
        marker |= m;
        c += !m;
        continue;
      }
      const int64_t l = voff[j + 1] - voff[j];
      marker |= l == 0;
      c += l == 8;
    }
    cnt[s] = marker ? c : 0;
  }
}

__global__ __launch_bounds__(NT) void k_emit_write(const int64_t* __restrict__ seg, int64_t nkey,
                                                  const int64_t* __restrict__ voff, const uint8_t* __restrict__ vdata,
                                                  const int64_t* __restrict__ ekey, const int64_t* __restrict__ pos,
                                                  int64_t* __restrict__ out) {
  for (int64_t s = (int64_t)blockIdx.x * NT + threadIdx.x; s < nkey; s += (int64_t)gridDim.x * NT) {
    int64_t o = pos[s];
    if (pos[s + 1] == o) continue;
    const int64_t e0 = ekey[2 * s], e1 = ekey[2 * s + 1];
    for (int64_t j = seg[s]; j < seg[s + 1]; ++j) {
      int64_t c;
      if (!voff) {
        c = reinterpret_cast<const int64_t*>(vdata)[j];
        if (c == -1) continue;
      } else {
        const int64_t b = voff[j];
        if (voff[j + 1] - b != 8) continue;
        __builtin_memcpy(&c, vdata + b, 8);
      }
      out[3 * o] = c;
      out[3 * o + 1] = e0;
      out[3 * o + 2] = e1;
      ++o;
    }
  }
}

}  // namespace

void trimr_first_degree(const int64_t* seg, int64_t nkey, const int64_t* key, const int64_t* nbr, int64_t nval,
                        int64_t* edge, int32_t* deg, hipStream_t s) {
  if (nval <= 0 || nkey <= 0) return;
  hipLaunchKernelGGL(k_first_degree, dim3(blocks(nval)), dim3(NT), 0, s, seg, nkey, key, nbr, nval, edge, deg);
  MRH_CHECK_LAUNCH();
}

void trimr_second_degree(const int64_t* seg, int64_t nkey, const int32_t* v, int64_t nval, int32_t* out,
                         hipStream_t s) {
  if (nkey <= 0 || nval <= 0) return;
  hipLaunchKernelGGL(k_second_degree, dim3(blocks(nkey)), dim3(NT), 0, s, seg, nkey, (const int2*)v, nval,
                     (int2*)out);
  MRH_CHECK_LAUNCH();
}

void trimr_low_degree(const int64_t* e, const int32_t* dg, int64_t n, int64_t* key, int64_t* val, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_low_degree, dim3(blocks(n)), dim3(NT), 0, s, e, (const int2*)dg, n, key, val);
  MRH_CHECK_LAUNCH();
}

void trimr_emit_count(const int64_t* seg, int64_t nkey, const int64_t* voff, const int64_t* vals, int64_t* cnt,
                      hipStream_t s) {
  if (nkey <= 0) return;
  hipLaunchKernelGGL(k_emit_count, dim3(blocks(nkey)), dim3(NT), 0, s, seg, nkey, voff, vals, cnt);
  MRH_CHECK_LAUNCH();
}

void trimr_emit_write(const int64_t* seg, int64_t nkey, const int64_t* voff, const uint8_t* vdata,
                      const int64_t* ekey, const int64_t* pos, int64_t* out, hipStream_t s) {
  if (nkey <= 0) return;
  hipLaunchKernelGGL(k_emit_write, dim3(blocks(nkey)), dim3(NT), 0, s, seg, nkey, voff, vdata, ekey, pos, out);
  MRH_CHECK_LAUNCH();
}

}  // namespace k
}  // namespace mrh
