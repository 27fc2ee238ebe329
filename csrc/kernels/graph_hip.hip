#include "hip/hip_runtime.h"
// Graph generators. R-MAT (Chakrabarti et al.) with the quadrant rule and
// optional per-level noise of oink/map_rmat_generate.cpp:32-66, but with a
// counter-based Philox4x32-10 stream instead of drand48 (rmatfn.h), so edge e
// is a pure function of (seed, e): one edge per thread, reproducible for any
// rank count, bit-identical with the CPU engine path.
#include "common.h"
#include "launch.h"
#include "rmatfn.h"

namespace mrh {
namespace k {
namespace {

constexpr int NT = 256;

__global__ __launch_bounds__(NT) void k_rmat(uint64_t* __restrict__ edges, int64_t nedges, int nlevels,
                                            float a, float b, float c, float d, float fraction,
                                            uint64_t seed, uint64_t first) {
  int64_t e = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (e >= nedges) return;
  uint64_t i, j;
  dev::rmat_edge(first + (uint64_t)e, nlevels, a, b, c, d, fraction, seed, &i, &j);
  // one 16-byte store per edge
  *reinterpret_cast<ulonglong2*>(edges + 2 * e) = make_ulonglong2(i, j);
}

}  // namespace

void rmat_edges(uint64_t* edges, int64_t nedges, int nlevels, float a, float b, float c, float d,
                float fraction, uint64_t seed, uint64_t first_edge, hipStream_t s) {
  if (nedges <= 0) return;
  hipLaunchKernelGGL(k_rmat, dim3((unsigned)((nedges + NT - 1) / NT)), dim3(NT), 0, s, edges, nedges,
                     nlevels, a, b, c, d, fraction, seed, first_edge);
  MRH_CHECK_LAUNCH();
}

}  // namespace k
}  // namespace mrh
