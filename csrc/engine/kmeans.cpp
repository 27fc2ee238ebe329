// K-means map (GPMR K-means, chapter_final.pdf Fig. 6a): points -> per-cluster
// (coordinate sums, count) KVs, combined in the map (kernels/kmeans.hip).
#include <ATen/hip/HIPContext.h>

#include <cstdlib>
#include <stdexcept>

#include "kernels/launch.h"
#include "kv.h"

namespace mrh {

// points [N, D] float32, centroids [K, D] float32 (same device) ->
// KV(int32 key = cluster*(D+1) + j, double value): j < D the coordinate sum,
// j == D the point count. Low dimensions (1-4, 8) run the fused assign +
// LDS-combine kernel, D <= 128 the matrix-core kernel (v_mfma_f32_16x16x4_f32
// scores + in-register argmin + LDS combine, kernels/kmeans.hip); anything
// larger computes distances as ||c||^2 - 2 X C^T with a library GEMM + argmin
// + index_add.
KV kmeans_map(const at::Tensor& points, const at::Tensor& centroids) {
  if (points.dim() != 2 || centroids.dim() != 2 || points.size(1) != centroids.size(1))
    throw std::runtime_error("kmeans_map: points [N,D] and centroids [K,D] required");
  if (points.scalar_type() != at::kFloat || centroids.scalar_type() != at::kFloat)
    throw std::runtime_error("kmeans_map: float32 points and centroids required");
  const at::Device dev = points.device();
  const int64_t N = points.size(0), D = points.size(1), K = centroids.size(0);
  at::Tensor p = points.contiguous(), c = centroids.to(dev).contiguous();
  at::Tensor acc = at::zeros({K * (D + 1)}, at::TensorOptions().device(dev).dtype(at::kDouble));
  // MRH_KMEANS_GEMM=1 forces the library-GEMM path (the comparison baseline
  // of the matrix-core kernel, profiles/r2_kmeans_mfma.txt)
  static const bool force_gemm = [] {
    const char* e = std::getenv("MRH_KMEANS_GEMM");
    return e && *e == '1';
  }();
  if (dev.is_cuda() && !force_gemm && k::kmeans_supported((int)D, (int)K)) {
    k::kmeans_assign_accumulate(p.data_ptr<float>(), N, (int)D, c.data_ptr<float>(), (int)K,
                                acc.data_ptr<double>(), at::hip::getCurrentHIPStream());
  } else if (N > 0) {
    at::Tensor score = (c * c).sum(1).unsqueeze(0) - 2.0 * at::matmul(p, c.t());  // [N, K]
    at::Tensor idx = score.argmin(1).contiguous();
    if (dev.is_cuda()) {
      k::kmeans_accumulate(p.data_ptr<float>(), N, (int)D, idx.data_ptr<int64_t>(), (int)K, acc.data_ptr<double>(),
                           at::hip::getCurrentHIPStream());
    } else {
      at::Tensor sums = at::zeros({K, D}, acc.options()).index_add_(0, idx, p.to(at::kDouble));
      at::Tensor cnt = bincount_dev(idx, K).to(at::kDouble).unsqueeze(1);
      acc = at::cat({sums, cnt}, 1).reshape({-1});
    }
  }
  KV kv;
  kv.n = K * (D + 1);
  kv.kw = 4;
  kv.vw = 8;
  kv.kdata = at::arange(kv.n, at::TensorOptions().device(dev).dtype(at::kInt)).view(at::kByte);
  kv.vdata = acc.view(at::kByte);
  return kv;
}

}  // namespace mrh
