#include "hip/hip_runtime.h"
// Segmented reductions over KMV value lists (the device form of MR-MPI's
// per-key reduce callbacks: oink/reduce_count.cpp, the wordfreq sum, PageRank's
// contribution sum). Deterministic: every segment is reduced in value order.
//
// Two-level to survive skew (R-MAT hubs, Zipf words):
//   short segments (<= SHORT_MAX values): one thread per segment;
//   long segments: queued (device atomic counter), then one 256-thread block
//   per long segment with coalesced strided loads + wave/block tree reduce.
#include "common.h"
#include "launch.h"
#include <cstdio>
#include <cstdlib>
#include <cfloat>
#include <climits>

namespace mrh {
namespace k {
namespace {

constexpr int NT = 256;
constexpr int64_t SHORT_MAX = 64;

template <typename T> struct Lim;
template <> struct Lim<int32_t> { __device__ static int32_t lo() { return INT_MIN; } __device__ static int32_t hi() { return INT_MAX; } };
template <> struct Lim<int64_t> { __device__ static int64_t lo() { return LLONG_MIN; } __device__ static int64_t hi() { return LLONG_MAX; } };
template <> struct Lim<float> { __device__ static float lo() { return -FLT_MAX; } __device__ static float hi() { return FLT_MAX; } };
template <> struct Lim<double> { __device__ static double lo() { return -DBL_MAX; } __device__ static double hi() { return DBL_MAX; } };

template <typename T, int OP>
__device__ __forceinline__ T ident() {
  if (OP == 0) return T(0);
  if (OP == 1) return Lim<T>::hi();
  return Lim<T>::lo();
}
template <typename T, int OP>
__device__ __forceinline__ T combine(T a, T b) {
  if (OP == 0) return a + b;
  if (OP == 1) return a < b ? a : b;
  return a > b ? a : b;
}

template <typename T, int OP>
__global__ __launch_bounds__(NT) void k_seg_short(const T* __restrict__ v, const int64_t* __restrict__ seg,
                                                 int64_t nseg, T* __restrict__ out,
                                                 int64_t* __restrict__ long_list,
                                                 unsigned long long* long_count) {
  int64_t s = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (s >= nseg) return;
  int64_t a = seg[s], b = seg[s + 1];
  if (b - a > SHORT_MAX) {
    unsigned long long q = atomicAdd(long_count, 1ull);
    long_list[q] = s;
    return;
  }
  T acc = ident<T, OP>();
  for (int64_t i = a; i < b; ++i) acc = combine<T, OP>(acc, v[i]);
  out[s] = acc;
}

template <typename T, int OP>
__global__ __launch_bounds__(NT) void k_seg_long(const T* __restrict__ v, const int64_t* __restrict__ seg,
                                                T* __restrict__ out, const int64_t* __restrict__ long_list,
                                                const unsigned long long* long_count) {
  __shared__ T sh[NT / MRH_WAVE];
  const unsigned long long nl = *long_count;
  for (unsigned long long li = blockIdx.x; li < nl; li += gridDim.x) {
    int64_t s = long_list[li];
    int64_t a = seg[s], b = seg[s + 1];
    T acc = ident<T, OP>();
    for (int64_t i = a + threadIdx.x; i < b; i += NT) acc = combine<T, OP>(acc, v[i]);
#pragma unroll
    for (int o = MRH_WAVE / 2; o > 0; o >>= 1) acc = combine<T, OP>(acc, __shfl_xor(acc, o, MRH_WAVE));
    if (dev::lane_id() == 0) sh[dev::wave_id()] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
      T r = sh[0];
      for (int w = 1; w < NT / MRH_WAVE; ++w) r = combine<T, OP>(r, sh[w]);
      out[s] = r;
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(NT) void k_seg_count(const int64_t* __restrict__ seg, int64_t nseg,
                                                 int32_t* __restrict__ out) {
  int64_t s = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (s < nseg) out[s] = (int32_t)(seg[s + 1] - seg[s]);
}

template <typename T, int OP>
void run(const void* vals, const int64_t* seg, int64_t nseg, void* out, hipStream_t s) {
  // scratch for the long-segment queue lives right after `out` is not allowed;
  // allocate a small device buffer via hipMallocAsync on the stream (pool-backed).
  int64_t* list = nullptr;
  unsigned long long* cnt = nullptr;
  hipMallocAsync((void**)&list, sizeof(int64_t) * (size_t)(nseg > 0 ? nseg : 1) + 256, s);
  cnt = reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(list) +
                                              sizeof(int64_t) * (size_t)(nseg > 0 ? nseg : 1));
  hipMemsetAsync(cnt, 0, sizeof(unsigned long long), s);
  unsigned g = (unsigned)((nseg + NT - 1) / NT);
  hipLaunchKernelGGL((k_seg_short<T, OP>), dim3(g), dim3(NT), 0, s, (const T*)vals, seg, nseg, (T*)out,
                     list, cnt);
  MRH_CHECK_LAUNCH();
  hipLaunchKernelGGL((k_seg_long<T, OP>), dim3(1024), dim3(NT), 0, s, (const T*)vals, seg, (T*)out,
                     (const int64_t*)list, (const unsigned long long*)cnt);
  MRH_CHECK_LAUNCH();
  hipFreeAsync(list, s);
}

template <typename T>
void run_op(int op, const void* vals, const int64_t* seg, int64_t nseg, void* out, hipStream_t s) {
  switch (op) {
    case 0: run<T, 0>(vals, seg, nseg, out, s); break;
    case 1: run<T, 1>(vals, seg, nseg, out, s); break;
    case 2: run<T, 2>(vals, seg, nseg, out, s); break;
    default: fprintf(stderr, "mrhip seg_reduce: bad op %d\n", op); abort();
  }
}

}  // namespace

void seg_reduce(const void* vals, int dtype, int op, const int64_t* seg, int64_t nseg, void* out,
                hipStream_t s) {
  if (nseg <= 0) return;
  switch (dtype) {
    case 0: run_op<int32_t>(op, vals, seg, nseg, out, s); break;
    case 1: run_op<int64_t>(op, vals, seg, nseg, out, s); break;
    case 2: run_op<float>(op, vals, seg, nseg, out, s); break;
    case 3: run_op<double>(op, vals, seg, nseg, out, s); break;
    default: fprintf(stderr, "mrhip seg_reduce: bad dtype %d\n", dtype); abort();
  }
}

void seg_count(const int64_t* seg, int64_t nseg, int32_t* out, hipStream_t s) {
  if (nseg <= 0) return;
  hipLaunchKernelGGL(k_seg_count, dim3((unsigned)((nseg + NT - 1) / NT)), dim3(NT), 0, s, seg, nseg, out);
  MRH_CHECK_LAUNCH();
}

}  // namespace k
}  // namespace mrh
