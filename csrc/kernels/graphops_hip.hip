#include "hip/hip_runtime.h"
// Iterative-graph kernels (PageRank over the MapReduce plan of pagerank.py).
//
// The reference's pagerank command is a stub (oink/pagerank.cpp:54-56); the
// algorithm follows oinkdoc/pagerank.txt: weights 1/outdeg (degree_weight),
// r' = (1-alpha)/N + alpha * (sum_in w*r + dangling/N).
//
//  pr_contrib : map+combine of one iteration, fused: for every destination
//               vertex group g (edges pre-sorted by (owner(dst), dst)),
//               send[g] = sum_e r[src_local[e]] * w[e]   (balanced segred)
//  pr_combine : reduce side: acc[vid[g]] = sum of received partials of g
//  pr_update  : r_new = base + alpha*(acc + dangling/N); per-block |r_new-r|
//               and dangling-mass partials for the convergence allreduce
#include "common.h"
#include "launch.h"
#include "segred_hip.h"

namespace mrh {
namespace k {
namespace {

constexpr int NT = 256;

struct ContribGet {
  const int32_t* src;
  const float* w;
  const float* r;
  __device__ __forceinline__ float operator()(int64_t i) const { return r[src[i]] * w[i]; }
};

// unweighted form: r already holds r_i / outdeg_i (written by pr_update), so
// the per-edge weight stream is not read at all
struct ContribGetC {
  const int32_t* src;
  const float* c;
  // the index stream is read once: non-temporal, so it does not evict the
  // gathered rank array from L2 / Infinity Cache
  __device__ __forceinline__ float operator()(int64_t i) const { return c[__builtin_nontemporal_load(src + i)]; }
};

struct PermGet {
  const int32_t* perm;
  const float* v;
  __device__ __forceinline__ float operator()(int64_t i) const { return v[perm[i]]; }
};

__global__ __launch_bounds__(NT) void k_scatter_f32(const float* __restrict__ v, const int32_t* __restrict__ idx,
                                                   int64_t n, float* __restrict__ out) {
  int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (i < n) out[idx[i]] = v[i];
}

__global__ __launch_bounds__(NT) void k_pr_update(const float* __restrict__ acc, const float* __restrict__ r,
                                                 float* __restrict__ rn, const uint8_t* __restrict__ dangling,
                                                 int64_t n, float base, float alpha,
                                                 const double* __restrict__ dmass, double invN,
                                                 const float* __restrict__ invdeg, float* __restrict__ cout,
                                                 double* __restrict__ partial) {
  __shared__ double sh[2][NT / MRH_WAVE];
  const float dterm = (float)(dmass[0] * invN);
  double d = 0.0, dm = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) {
    float x = base + alpha * (acc[i] + dterm);
    rn[i] = x;
    if (cout) cout[i] = x * invdeg[i];
    d += fabs((double)x - (double)r[i]);
    if (dangling[i]) dm += x;
  }
  for (int o = MRH_WAVE / 2; o > 0; o >>= 1) {
    d += __shfl_xor(d, o, MRH_WAVE);
    dm += __shfl_xor(dm, o, MRH_WAVE);
  }
  if (dev::lane_id() == 0) {
    sh[0][dev::wave_id()] = d;
    sh[1][dev::wave_id()] = dm;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double a = 0, b = 0;
    for (int w = 0; w < NT / MRH_WAVE; ++w) {
      a += sh[0][w];
      b += sh[1][w];
    }
    partial[2 * blockIdx.x] = a;
    partial[2 * blockIdx.x + 1] = b;
  }
}

}  // namespace

size_t pr_scratch_bytes(int64_t nval) { return dev::segred_carry_entries(nval) * (sizeof(int64_t) + sizeof(float)) + 64; }

void pr_contrib(const int64_t* seg, int64_t nseg, int64_t nedge, const int32_t* src, const float* w, const float* r,
                float* out, void* scratch, hipStream_t s) {
  size_t nc = dev::segred_carry_entries(nedge);
  int64_t* cs = reinterpret_cast<int64_t*>(scratch);
  float* cv = reinterpret_cast<float*>(reinterpret_cast<char*>(scratch) + nc * sizeof(int64_t));
  if (w)
    dev::segred_launch<float, 0>(ContribGet{src, w, r}, seg, nseg, nedge, out, cs, cv, s);
  else
    dev::segred_launch<float, 0>(ContribGetC{src, r}, seg, nseg, nedge, out, cs, cv, s);
}

void pr_combine(const int64_t* seg, int64_t ngrp, int64_t nrecv, const int32_t* perm, const float* recv,
                const int32_t* vid, float* grp, float* acc, void* scratch, hipStream_t s) {
  size_t nc = dev::segred_carry_entries(nrecv);
  int64_t* cs = reinterpret_cast<int64_t*>(scratch);
  float* cv = reinterpret_cast<float*>(reinterpret_cast<char*>(scratch) + nc * sizeof(int64_t));
  dev::segred_launch<float, 0>(PermGet{perm, recv}, seg, ngrp, nrecv, grp, cs, cv, s);
  if (ngrp > 0)
    hipLaunchKernelGGL(k_scatter_f32, dim3((unsigned)((ngrp + NT - 1) / NT)), dim3(NT), 0, s, grp, vid, ngrp, acc);
  MRH_CHECK_LAUNCH();
}

void scatter_f32(const float* v, const int32_t* idx, int64_t n, float* out, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_scatter_f32, dim3((unsigned)((n + NT - 1) / NT)), dim3(NT), 0, s, v, idx, n, out);
  MRH_CHECK_LAUNCH();
}

int pr_update_blocks(int64_t n) {
  int64_t b = (n + NT - 1) / NT;
  return (int)(b < 1024 ? (b < 1 ? 1 : b) : 1024);
}

void pr_update(const float* acc, const float* r, float* rn, const uint8_t* dangling, int64_t n, float base,
               float alpha, const double* dmass, double invN, const float* invdeg, float* cout, double* partial,
               hipStream_t s) {
  hipLaunchKernelGGL(k_pr_update, dim3(pr_update_blocks(n)), dim3(NT), 0, s, acc, r, rn, dangling, n, base, alpha,
                     dmass, invN, invdeg, cout, partial);
  MRH_CHECK_LAUNCH();
}

}  // namespace k
}  // namespace mrh
