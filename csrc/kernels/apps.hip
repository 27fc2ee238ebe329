// Application epilogue kernels.
//
// InvertedIndex reduce: the reference appends "url\tname name ... \n" to a
// per-rank file with one fopen/fclose per key (cuda/InvertedIndex.cu:463-513;
// ~21 s of its 59 s end-to-end). Here the whole output text is formatted in
// HBM in two balanced passes (one thread per value, one per key) from two
// prefix sums, then copied to the host once.
#include "common.h"
#include "launch.h"

namespace mrh {
namespace k {
namespace {

constexpr int NT = 256;

__device__ __forceinline__ int64_t seg_of(const int64_t* seg, int64_t nseg, int64_t i) {
  // largest s with seg[s] <= i
  int64_t lo = 0, hi = nseg - 1;
  while (lo < hi) {
    int64_t mid = (lo + hi + 1) >> 1;
    if (seg[mid] <= i) lo = mid; else hi = mid - 1;
  }
  return lo;
}

__global__ __launch_bounds__(NT) void k_ii_value_len(const int32_t* __restrict__ vals, int64_t nval,
                                                    const int64_t* __restrict__ name_off,
                                                    int32_t* __restrict__ lenv) {
  int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (i >= nval) return;
  int32_t v = vals[i];
  lenv[i] = (int32_t)(name_off[v + 1] - name_off[v]) + 1;
}

__global__ __launch_bounds__(NT) void k_ii_key_len(const int64_t* __restrict__ koff, int64_t nseg,
                                                  int32_t* __restrict__ lens) {
  int64_t s = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (s >= nseg) return;
  lens[s] = (int32_t)(koff[s + 1] - koff[s] - 1) + 2;  // key w/o NUL + '\t' + '\n'
}

__global__ __launch_bounds__(NT) void k_ii_values(const int32_t* __restrict__ vals, int64_t nval,
                                                 const int64_t* __restrict__ seg, int64_t nseg,
                                                 const int64_t* __restrict__ koff,
                                                 const int64_t* __restrict__ cv,
                                                 const int64_t* __restrict__ cs,
                                                 const uint8_t* __restrict__ names,
                                                 const int64_t* __restrict__ name_off,
                                                 uint8_t* __restrict__ out) {
  int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (i >= nval) return;
  int64_t s = seg_of(seg, nseg, i);
  int64_t base = cs[s] + cv[seg[s]];
  int64_t o = base + (koff[s + 1] - koff[s] - 1) + 1 + (cv[i] - cv[seg[s]]);
  int32_t v = vals[i];
  int64_t a = name_off[v], len = name_off[v + 1] - a;
  for (int64_t j = 0; j < len; ++j) out[o + j] = names[a + j];
  out[o + len] = ' ';
}

// 16 lanes per key
__global__ __launch_bounds__(NT) void k_ii_keys(const uint8_t* __restrict__ kd, const int64_t* __restrict__ koff,
                                               const int64_t* __restrict__ seg, int64_t nseg,
                                               const int64_t* __restrict__ cv, const int64_t* __restrict__ cs,
                                               uint8_t* __restrict__ out) {
  const int g = threadIdx.x & 15;
  int64_t s = ((int64_t)blockIdx.x * NT + threadIdx.x) >> 4;
  const int64_t stride = ((int64_t)gridDim.x * NT) >> 4;
  for (; s < nseg; s += stride) {
    int64_t base = cs[s] + cv[seg[s]];
    int64_t a = koff[s], klen = koff[s + 1] - a - 1;
    for (int64_t j = g; j < klen; j += 16) out[base + j] = kd[a + j];
    if (g == 0) {
      out[base + klen] = '\t';
      out[base + klen + 1 + (cv[seg[s + 1]] - cv[seg[s]])] = '\n';
    }
  }
}

inline unsigned nb(int64_t n) { return (unsigned)((n + NT - 1) / NT); }

}  // namespace

void ii_value_len(const int32_t* vals, int64_t nval, const int64_t* name_off, int32_t* lenv, hipStream_t s) {
  if (nval <= 0) return;
  hipLaunchKernelGGL(k_ii_value_len, dim3(nb(nval)), dim3(NT), 0, s, vals, nval, name_off, lenv);
  MRH_CHECK_LAUNCH();
}
void ii_key_len(const int64_t* koff, int64_t nseg, int32_t* lens, hipStream_t s) {
  if (nseg <= 0) return;
  hipLaunchKernelGGL(k_ii_key_len, dim3(nb(nseg)), dim3(NT), 0, s, koff, nseg, lens);
  MRH_CHECK_LAUNCH();
}
void ii_write(const uint8_t* kd, const int64_t* koff, const int32_t* vals, int64_t nval, const int64_t* seg,
              int64_t nseg, const int64_t* cv, const int64_t* cs, const uint8_t* names, const int64_t* name_off,
              uint8_t* out, hipStream_t s) {
  if (nseg <= 0) return;
  if (nval > 0)
    hipLaunchKernelGGL(k_ii_values, dim3(nb(nval)), dim3(NT), 0, s, vals, nval, seg, nseg, koff, cv, cs, names,
                       name_off, out);
  MRH_CHECK_LAUNCH();
  int64_t g = (nseg * 16 + NT - 1) / NT;
  if (g > 65536) g = 65536;
  hipLaunchKernelGGL(k_ii_keys, dim3((unsigned)g), dim3(NT), 0, s, kd, koff, seg, nseg, cv, cs, out);
  MRH_CHECK_LAUNCH();
}

}  // namespace k
}  // namespace mrh
