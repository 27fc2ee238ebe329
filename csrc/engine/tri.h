// Triangle enumeration engine ops (tri.cpp, kernels in csrc/kernels/tri.hip).
#pragma once
#include <ATen/ATen.h>

#include <tuple>

namespace mrh {
// uniq: sorted unique packed undirected edges (lo<<32|hi, lo<hi), ids < nvert <= 2^32.
// Returns the degree-oriented CSR (rowptr int64 [nvert+1], col int32 [m],
// okeys int64 [m] = src<<32|dst sorted).
std::tuple<at::Tensor, at::Tensor, at::Tensor> tri_prepare(const at::Tensor& uniq, int64_t nvert);
// number of triangles found on oriented edges [e0, e1)
int64_t tri_count(const at::Tensor& rowptr, const at::Tensor& col, const at::Tensor& okeys, int64_t e0, int64_t e1);
// those triangles as [T,3] int64 (u, v, w), u->v->w in orientation order
at::Tensor tri_list(const at::Tensor& rowptr, const at::Tensor& col, const at::Tensor& okeys, int64_t e0, int64_t e1);
}  // namespace mrh
