// Device helpers shared by the CDNA4 kernels: wave64 scans/reductions and
// block-level scans. Everything here assumes a 64-lane wavefront (gfx950).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <string>
#include "hashfn.h"

#define MRH_WAVE 64

namespace mrh {
namespace k {
// Serialize mode (SURVEY.md §5 "race detection"): MRH_SYNC=1 synchronises the
// device after every launch, so an asynchronous fault, or a kernel racing a
// later one on another stream, is reported at the launch site (file:line)
// instead of at some later sync. Diagnostic only: it removes all overlap.
inline bool sync_mode() {
  static const bool on = [] {
    const char* v = std::getenv("MRH_SYNC");
    return v && *v && *v != '0';
  }();
  return on;
}
// A failed launch or (in serialize mode) a failed kernel is a typed error,
// never a local abort(): the exception unwinds through the op, which poisons
// the job's communicator on the way out (comm.h), so peers fail fast too.
struct KernelError : std::runtime_error {
  using std::runtime_error::runtime_error;
};
inline void check_launch(const char* file, int line) {
  hipError_t e = hipGetLastError();
  const bool launched = e == hipSuccess;
  if (launched && sync_mode()) e = hipDeviceSynchronize();
  if (e != hipSuccess) {
    char buf[512];
    std::snprintf(buf, sizeof(buf), "mrhip kernel %s: %s at %s:%d", launched ? "execution failed" : "launch failed",
                  hipGetErrorString(e), file, line);
    throw KernelError(buf);
  }
}
// a runtime call of a launcher (memset, copy, sync): a failure is a KernelError
inline void hip_call(hipError_t e, const char* what, const char* file, int line) {
  if (e == hipSuccess) return;
  char buf[512];
  std::snprintf(buf, sizeof(buf), "mrhip: %s failed: %s at %s:%d", what, hipGetErrorString(e), file, line);
  throw KernelError(buf);
}
// host-side precondition of a launcher (shapes, limits): std::invalid_argument
inline void check_arg(bool ok, const char* what) {
  if (!ok) throw std::invalid_argument(std::string("mrhip: ") + what);
}
}  // namespace k
}  // namespace mrh

#define MRH_CHECK_LAUNCH() ::mrh::k::check_launch(__FILE__, __LINE__)
#define MRH_HIP(call) ::mrh::k::hip_call((call), #call, __FILE__, __LINE__)

namespace mrh {
namespace dev {

__device__ __forceinline__ int lane_id() { return threadIdx.x & (MRH_WAVE - 1); }
__device__ __forceinline__ int wave_id() { return threadIdx.x / MRH_WAVE; }
__device__ __forceinline__ uint64_t lanemask_lt() {
  return (lane_id() == 0) ? 0ull : (~0ull >> (64 - lane_id()));
}

// inclusive wave scan (64 lanes) via DPP-friendly shfl_up
template <typename T>
__device__ __forceinline__ T wave_incl_scan(T v) {
  const int l = lane_id();
#pragma unroll
  for (int o = 1; o < MRH_WAVE; o <<= 1) {
    T u = __shfl_up(v, o, MRH_WAVE);
    if (l >= o) v += u;
  }
  return v;
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int o = MRH_WAVE / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, MRH_WAVE);
  return v;
}

// Block exclusive scan of one value per thread; returns exclusive prefix,
// writes block total to *total. `sh` needs (blockDim/64 + 1) T entries.
template <typename T, int NT>
__device__ __forceinline__ T block_excl_scan(T v, T* sh, T* total) {
  constexpr int NW = NT / MRH_WAVE;
  const int l = lane_id(), w = wave_id();
  T incl = wave_incl_scan(v);
  if (l == MRH_WAVE - 1) sh[w] = incl;
  __syncthreads();
  if (w == 0) {
    T x = (l < NW) ? sh[l] : T(0);
    T xs = wave_incl_scan(x);
    if (l < NW) sh[l] = xs - x;
    if (l == NW - 1) sh[NW] = xs;
  }
  __syncthreads();
  T res = incl - v + sh[w];
  *total = sh[NW];
  __syncthreads();
  return res;
}

// ---------------------------------------------------------------- unaligned byte-string access
// 4 bytes starting at any address p (little-endian) from aligned dword loads
// + v_alignbyte; never touches a dword that does not contain one of p..p+3.
__device__ __forceinline__ uint32_t ld32u(const uint8_t* p) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  const uint32_t* w = reinterpret_cast<const uint32_t*>(a & ~uintptr_t(3));
  const uint32_t r = (uint32_t)(a & 3);
  const uint32_t lo = w[0];
  if (r == 0) return lo;
  return __builtin_amdgcn_alignbyte(w[1], lo, r);
}
// 8 bytes starting at p
__device__ __forceinline__ uint64_t ld64u(const uint8_t* p) {
  return (uint64_t)ld32u(p) | ((uint64_t)ld32u(p + 4) << 32);
}

// lookup3 over a device byte string with dword-wide loads (same result as
// the byte-reader lookup3 in hashfn.h)
__device__ __forceinline__ void lookup3_wide(const uint8_t* k, int64_t length, uint32_t* pc, uint32_t* pb) {
  uint32_t a, b, c;
  a = b = c = 0xdeadbeefu + (uint32_t)length + *pc;
  c += *pb;
  while (length > 12) {
    a += ld32u(k);
    b += ld32u(k + 4);
    c += ld32u(k + 8);
    MRH_L3_MIX(a, b, c);
    length -= 12;
    k += 12;
  }
  if (length == 0) { *pc = c; *pb = b; return; }
  // tail: 1..12 bytes, read whole dwords that lie inside the string, bytes otherwise
  uint32_t t[3] = {0, 0, 0};
  int i = 0;
  for (; i + 4 <= length; i += 4) t[i >> 2] = ld32u(k + i);
  for (; i < length; ++i) t[i >> 2] |= (uint32_t)k[i] << (8 * (i & 3));
  a += t[0]; b += t[1]; c += t[2];
  MRH_L3_FINAL(a, b, c);
  *pc = c;
  *pb = b;
}

// index of the first byte == ch in [p, p+len), or len
__device__ __forceinline__ int64_t find_byte(const uint8_t* p, int64_t len, uint8_t ch) {
  int64_t j = 0;
  const uint64_t pat = 0x0101010101010101ull * ch;
  while (j < len && ((reinterpret_cast<uintptr_t>(p + j)) & 7)) {
    if (p[j] == ch) return j;
    ++j;
  }
  for (; j + 8 <= len; j += 8) {
    uint64_t x = *reinterpret_cast<const uint64_t*>(p + j) ^ pat;
    uint64_t t = (x - 0x0101010101010101ull) & ~x & 0x8080808080808080ull;
    if (t) return j + (__builtin_ctzll(t) >> 3);
  }
  for (; j < len; ++j)
    if (p[j] == ch) return j;
  return len;
}

// byte-string equality with 8-byte loads
__device__ __forceinline__ bool bytes_equal(const uint8_t* a, const uint8_t* b, int64_t len) {
  int64_t j = 0;
  for (; j + 8 <= len; j += 8)
    if (ld64u(a + j) != ld64u(b + j)) return false;
  for (; j < len; ++j)
    if (a[j] != b[j]) return false;
  return true;
}

}  // namespace dev
}  // namespace mrh
