// Triangle enumeration engine ops (tri.cpp, kernels in csrc/kernels/tri.hip).
#pragma once
#include <ATen/ATen.h>

#include <tuple>
#include <utility>

namespace mrh {
// uniq: sorted unique packed undirected edges (lo<<32|hi, lo<hi), ids < nvert < 2^32-1.
// Vertices are relabelled by (degree, id) rank and every edge points from the
// lower to the higher rank. Returns the oriented CSR in rank ids (rowptr int64
// [nvert+1], col int32 [m], okeys int64 [m] = src<<32|dst sorted) and perm
// (int64 [nvert], perm[rank] = original id).
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> tri_prepare(const at::Tensor& uniq, int64_t nvert);
// the pieces of tri_prepare (also the multi-GPU build, graphplan.cpp):
// degree of every vertex over packed edges (int32 [nvert]); (rank, perm) of
// the (degree, id) order; the edges oriented to the higher rank, packed
// rank_lo << 32 | rank_hi (unsorted); col / rowptr of sorted oriented keys
at::Tensor tri_degrees(const at::Tensor& uniq, int64_t nvert);
// deg[low 32 bits of packed[i]] += 1 over every element (deg: int32 bins, ids
// < deg.numel()): a partitioned LDS count (bucket scatter of u16 ids + 32768-bin
// block histograms), no scattered global atomic per element
void count_low_words(const at::Tensor& packed, at::Tensor& deg);
std::pair<at::Tensor, at::Tensor> tri_rank_perm(const at::Tensor& deg);
at::Tensor tri_orient_keys(const at::Tensor& uniq, const at::Tensor& rank);
at::Tensor tri_col_of(const at::Tensor& okeys);
at::Tensor tri_rowptr_of(const at::Tensor& okeys, int64_t nvert);
// vertices of the hub bitmap path of tri_count (MRH_TRI_HUB, default
// nvert/32 up to 524288 and a quarter of free HBM; 0 = hash kernels only)
int64_t tri_hub_size(int64_t nvert);
// hub vertices the last tri_count on this process used
int64_t tri_last_hub_size();
// number of triangles whose first oriented edge lies in [e0, e1)
int64_t tri_count(const at::Tensor& rowptr, const at::Tensor& col, const at::Tensor& okeys, int64_t e0, int64_t e1);
// number of triangles whose lowest (rank) vertex is a row in [u0, u1): the
// hub bitmap + hash kernels of tri_count over a row range (okeys, the whole
// sorted oriented edge list, only for MRH_TRI_HUB_KERNEL=pull)
int64_t tri_count_range(const at::Tensor& rowptr, const at::Tensor& col, int64_t u0, int64_t u1,
                        const at::Tensor& okeys = {});
// number of triangles u < v < w (in the CSR's id order) over the rows u in
// [u0, u1): rows outside the range are only looked up (the distributed
// graph's halo)
int64_t tri_count_rows(const at::Tensor& rowptr, const at::Tensor& col, int64_t u0, int64_t u1);
// the triangles found on oriented edges [e0, e1) as [T,3] int64 rank ids
at::Tensor tri_list(const at::Tensor& rowptr, const at::Tensor& col, const at::Tensor& okeys, int64_t e0, int64_t e1);

// tri_find_mr callbacks (trimr.cpp; oink/tri_find.cpp:104-325)
struct KV;
struct KMV;
// vertex -> neighbours KMV: per value, the edge (min, max) [nval,2] int64 and
// {deg, 0} / {0, deg} [nval,2] int32 (deg in the key vertex's slot)
std::pair<at::Tensor, at::Tensor> trimr_first_degree(const KMV& m);
// edge -> its two degree records: {di, dj} per edge, [nkey,2] int32
at::Tensor trimr_second_degree(const KMV& m);
// KV(edge, {di, dj}) -> (lower-degree end, other end), int64 each
std::pair<at::Tensor, at::Tensor> trimr_low_degree(const KV& kv);
// edge -> {wedge centres (8 B), edge marker (0 B)}: closed triangles
// (centre, e0, e1) as [T,3] int64
// tri_find_mr's last collate, fixed 8-byte values: an edge (vi, vj) carries
// the value vi (a wedge's centre is never one of its key's endpoints), so
// the pairs stay narrow (vertex-sized values) and group as packed words
// compact_vb > 0: the compact layout of large graphs — keys one packed word
// vi << compact_vb | vj, values u32 (wedges 12 bytes instead of 24)
at::Tensor trimr_emit(const KMV& m, int compact_vb = 0);
at::Tensor trimr_emit_compact(const KMV& m, int vb);
}  // namespace mrh
