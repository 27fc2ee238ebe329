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
                                                  const int64_t* __restrict__ ekey, int64_t* __restrict__ cnt) {
  for (int64_t s = (int64_t)blockIdx.x * NT + threadIdx.x; s < nkey; s += (int64_t)gridDim.x * NT) {
    int64_t c = 0;
    bool marker = false;
    for (int64_t j = seg[s]; j < seg[s + 1]; ++j) {
      if (!voff) {  // fixed 8-byte values: an edge carries its first vertex
        const bool m = vals[j] == ekey[2 * s];
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
        if (c == e0) continue;
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

// Fixed 8-byte values (marker -1): value-parallel instead of a thread per key
// (RMAT-20's last reduce: 1.24 G values over 190 M keys, hub pairs with 10^5
// centres, and uncoalesced per-thread walks). One block per tile of ET_TILE
// values: its first key comes from tk (k_emit_tile_keys, once for the three
// phases), the key of every value from an LDS map (each key's index written
// at its first value, then a max-scan), the marks of its keys are staged in
// LDS, and only values of marked keys (an existing edge: ~8 % of RMAT-20's
// wedge keys) touch the edge key. PHASE 0 marks the keys holding a marker,
// PHASE 1 counts the centres of marked keys per tile, PHASE 2 writes them at
// the tile's offset.
constexpr int ET_IT = 16;
constexpr int ET_TILE = NT * ET_IT;

// an edge key's two vertices: EDGE {vi, vj} words, or (CMP) one packed word
// vi << vb | vj (the compact wedges of large graphs: 8-byte keys, 4-byte values)
template <int CMP>
__device__ __forceinline__ void edge_of(const int64_t* ekey, int64_t k, int vb, int64_t* vi, int64_t* vj) {
  if (CMP) {
    const uint64_t K = (uint64_t)ekey[k];
    *vi = (int64_t)(K >> vb);
    *vj = (int64_t)(K & ((1ull << vb) - 1));
  } else {
    *vi = ekey[2 * k];
    *vj = ekey[2 * k + 1];
  }
}

// the key of every tile's first value (tk[t]), one thread per key: a key
// whose values start tiles writes their entries (every value belongs to one
// key, so each tile is written once); tk[nt] = nkey - 1
__global__ __launch_bounds__(NT) void k_emit_tile_keys(const int64_t* __restrict__ seg, int64_t nkey, int64_t nt,
                                                       int64_t* __restrict__ tk) {
  for (int64_t k = (int64_t)blockIdx.x * NT + threadIdx.x; k < nkey; k += (int64_t)gridDim.x * NT) {
    const int64_t a = seg[k], b = seg[k + 1];
    for (int64_t t = (a + ET_TILE - 1) / ET_TILE; t * ET_TILE < b; ++t) tk[t] = k;
    if (k == nkey - 1) tk[nt] = k;
  }
}

template <int PHASE, int CMP>
__global__ __launch_bounds__(NT) void k_emit_tiles(const int64_t* __restrict__ seg, int64_t nkey, int64_t nval,
                                                   const void* __restrict__ vals_, uint8_t* __restrict__ marked,
                                                   int64_t* __restrict__ tcount, const int64_t* __restrict__ tbase,
                                                   const int64_t* __restrict__ ekey, int64_t* __restrict__ out, int vb,
                                                   const int64_t* __restrict__ tk) {
  // the key of every value of the tile, as an index from k0: each key
  // starting inside the tile writes its index at its first value, a max-scan
  // fills the rest (no per-value search)
  __shared__ uint16_t s_kidx[ET_TILE];
  __shared__ uint8_t s_mark[ET_TILE + 2];
  __shared__ int32_t s_run[NT];
  __shared__ int64_t sh[NT / MRH_WAVE + 1];
  const int64_t t0 = (int64_t)blockIdx.x * ET_TILE;
  const int tn = (int)(nval - t0 < ET_TILE ? nval - t0 : ET_TILE);
  // keys k0 .. k0 + nk - 1: the tile's first value's key to the next tile's
  // (one more than the tile's last key when a key starts the next tile)
  const int64_t k0 = tk[blockIdx.x];
  const int nk = (int)(tk[blockIdx.x + 1] - k0 + 1);
  for (int i = threadIdx.x; i < ET_TILE; i += NT) s_kidx[i] = 0;
  __syncthreads();
  for (int i = threadIdx.x; i < nk; i += NT) {
    const int64_t pos = seg[k0 + i] - t0;
    if (pos > 0 && pos < tn) s_kidx[pos] = (uint16_t)i;
    if (PHASE > 0) s_mark[i] = marked[k0 + i];
  }
  __syncthreads();
  {  // inclusive max-scan: thread t owns entries [ET_IT t, ET_IT t + ET_IT)
    const int b = threadIdx.x * ET_IT;
    int m = 0;
#pragma unroll
    for (int q = 0; q < ET_IT; ++q) m = max(m, (int)s_kidx[b + q]);
    s_run[threadIdx.x] = m;
    __syncthreads();
    // exclusive max over the threads before (a log-step scan in LDS)
    for (int o = 1; o < NT; o <<= 1) {
      const int v = threadIdx.x >= o ? s_run[threadIdx.x - o] : 0;
      __syncthreads();
      s_run[threadIdx.x] = max(s_run[threadIdx.x], v);
      __syncthreads();
    }
    int run = threadIdx.x ? s_run[threadIdx.x - 1] : 0;
#pragma unroll
    for (int q = 0; q < ET_IT; ++q) {
      run = max(run, (int)s_kidx[b + q]);
      s_kidx[b + q] = (uint16_t)run;
    }
  }
  __syncthreads();
  int64_t mine = 0;
  int64_t c_[ET_IT];
  int64_t key_[ET_IT];
#pragma unroll
  for (int it = 0; it < ET_IT; ++it) {
    const int o = it * NT + threadIdx.x;
    key_[it] = -1;
    if (o >= tn) continue;
    const int lk = s_kidx[o];
    if (PHASE > 0 && !s_mark[lk]) continue;  // a key without its edge: no triangle (most keys)
    const int64_t j = t0 + o;
    const int64_t k = k0 + lk;
    const int64_t c = CMP ? (int64_t)static_cast<const uint32_t*>(vals_)[j] : static_cast<const int64_t*>(vals_)[j];
    int64_t vi, vj;
    edge_of<CMP>(ekey, k, vb, &vi, &vj);
    const bool mark = c == vi;  // an edge carries its first vertex
    if (PHASE == 0) {
      if (mark) marked[k] = 1;  // every writer stores the same byte
    } else if (!mark) {
      c_[it] = c;
      key_[it] = k;
      ++mine;
    }
  }
  if (PHASE == 0) return;
  int64_t total;
  const int64_t pre = dev::block_excl_scan<int64_t, NT>(mine, sh, &total);
  if (PHASE == 1) {
    if (threadIdx.x == 0) tcount[blockIdx.x] = total;
    return;
  }
  int64_t o = tbase[blockIdx.x] + pre;
#pragma unroll
  for (int it = 0; it < ET_IT; ++it) {
    if (key_[it] < 0) continue;
    int64_t vi, vj;
    edge_of<CMP>(ekey, key_[it], vb, &vi, &vj);
    out[3 * o] = c_[it];
    out[3 * o + 1] = vi;
    out[3 * o + 2] = vj;
    ++o;
  }
}

}  // namespace

int64_t trimr_emit_tiles(int64_t nval) { return (nval + ET_TILE - 1) / ET_TILE; }

void trimr_emit_tile_keys(const int64_t* seg, int64_t nkey, int64_t nval, int64_t* tk, hipStream_t s) {
  if (nval <= 0 || nkey <= 0) return;
  hipLaunchKernelGGL(k_emit_tile_keys, dim3(blocks(nkey)), dim3(NT), 0, s, seg, nkey, trimr_emit_tiles(nval), tk);
  MRH_CHECK_LAUNCH();
}

void trimr_emit_fixed(int phase, const int64_t* seg, int64_t nkey, int64_t nval, const void* vals, uint8_t* marked,
                      int64_t* tcount, const int64_t* tbase, const int64_t* ekey, int64_t* out, int compact_vb,
                      const int64_t* tk, hipStream_t s) {
  if (nval <= 0 || nkey <= 0) return;
  const unsigned g = (unsigned)trimr_emit_tiles(nval);
  const int vb = compact_vb;
#define MRH_EMIT(P, C)                                                                                             \
  hipLaunchKernelGGL((k_emit_tiles<P, C>), dim3(g), dim3(NT), 0, s, seg, nkey, nval, vals, marked, tcount, tbase, \
                     ekey, out, vb, tk)
  if (vb > 0) {
    if (phase == 0) MRH_EMIT(0, 1);
    else if (phase == 1) MRH_EMIT(1, 1);
    else MRH_EMIT(2, 1);
  } else {
    if (phase == 0) MRH_EMIT(0, 0);
    else if (phase == 1) MRH_EMIT(1, 0);
    else MRH_EMIT(2, 0);
  }
#undef MRH_EMIT
  MRH_CHECK_LAUNCH();
}

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

void trimr_emit_count(const int64_t* seg, int64_t nkey, const int64_t* voff, const int64_t* vals, const int64_t* ekey,
                      int64_t* cnt, hipStream_t s) {
  if (nkey <= 0) return;
  hipLaunchKernelGGL(k_emit_count, dim3(blocks(nkey)), dim3(NT), 0, s, seg, nkey, voff, vals, ekey, cnt);
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
