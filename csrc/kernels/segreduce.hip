// Segmented reductions over KMV value lists: the device form of MR-MPI's
// per-key reduce callbacks (oink/reduce_count.cpp, wordfreq's sum, PageRank's
// contribution sum). Load-balanced by value count (segred.h), deterministic.
#include "common.h"
#include "launch.h"
#include "segred.h"
#include <cstdio>
#include <cstdlib>

namespace mrh {
namespace k {
namespace {

constexpr int NT = 256;

template <typename T>
struct LoadVal {
  const T* v;
  __device__ __forceinline__ T operator()(int64_t i) const { return v[i]; }
};

__global__ __launch_bounds__(NT) void k_seg_count(const int64_t* __restrict__ seg, int64_t nseg,
                                                 int32_t* __restrict__ out) {
  int64_t s = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (s < nseg) out[s] = (int32_t)(seg[s + 1] - seg[s]);
}

template <typename T, int OP>
void run(const void* vals, const int64_t* seg, int64_t nseg, int64_t nval, void* out, hipStream_t s) {
  size_t nc = dev::segred_carry_entries(nval);
  char* scratch = nullptr;
  hipMallocAsync((void**)&scratch, nc * (sizeof(int64_t) + sizeof(T)) + 64, s);
  int64_t* cs = reinterpret_cast<int64_t*>(scratch);
  T* cv = reinterpret_cast<T*>(scratch + nc * sizeof(int64_t));
  dev::segred_launch<T, OP>(LoadVal<T>{(const T*)vals}, seg, nseg, nval, (T*)out, cs, cv, s);
  hipFreeAsync(scratch, s);
}

template <typename T>
void run_op(int op, const void* vals, const int64_t* seg, int64_t nseg, int64_t nval, void* out, hipStream_t s) {
  switch (op) {
    case 0: run<T, 0>(vals, seg, nseg, nval, out, s); break;
    case 1: run<T, 1>(vals, seg, nseg, nval, out, s); break;
    case 2: run<T, 2>(vals, seg, nseg, nval, out, s); break;
    default: check_arg(false, "seg_reduce: bad op");
  }
}

}  // namespace

void seg_reduce(const void* vals, int dtype, int op, const int64_t* seg, int64_t nseg, int64_t nval, void* out,
                hipStream_t s) {
  if (nseg <= 0) return;
  switch (dtype) {
    case 0: run_op<int32_t>(op, vals, seg, nseg, nval, out, s); break;
    case 1: run_op<int64_t>(op, vals, seg, nseg, nval, out, s); break;
    case 2: run_op<float>(op, vals, seg, nseg, nval, out, s); break;
    case 3: run_op<double>(op, vals, seg, nseg, nval, out, s); break;
    default: check_arg(false, "seg_reduce: bad dtype");
  }
}

void seg_count(const int64_t* seg, int64_t nseg, int32_t* out, hipStream_t s) {
  if (nseg <= 0) return;
  hipLaunchKernelGGL(k_seg_count, dim3((unsigned)((nseg + NT - 1) / NT)), dim3(NT), 0, s, seg, nseg, out);
  MRH_CHECK_LAUNCH();
}

}  // namespace k
}  // namespace mrh
