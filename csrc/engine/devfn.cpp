// Device functors (devfn.h): user map / reduce device code compiled at run
// time by hiprtc for gfx950 into two kernels —
//
//   mrd_count  one thread per item (pair / task / key, grid-stride): runs the
//              functor with a counting Emit, stores the item's records, key
//              bytes and value bytes, and min/max record widths (atomics)
//   mrd_write  runs it again with a writing Emit at the item's offsets (the
//              exclusive scans of the counts) into var-width output columns
//
// A uniform output width (every key, every value the same length) turns
// into a fixed-width KV, so later ops keep their fixed-key fast paths.
// Modules are cached per (device, kind, code).
#include "devfn.h"

#include <ATen/hip/HIPContext.h>
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>

#include <cstdlib>
#include <functional>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <unordered_map>
#include <vector>

#include "../kernels/launch.h"

namespace mrh {
namespace devfn {

namespace {
const char* kDevicePrelude = R"MRD(
// ---- mrd: the engine's device-functor prelude (csrc/engine/devfn.cpp) ----
namespace mrd {
typedef unsigned char u8;
typedef long long i64;
typedef unsigned long long u64;
// a key or value: p[0 .. n)
struct Bytes {
  const u8* p;
  i64 n;
  template <class T>
  __device__ T as(i64 off = 0) const {
    T v;
    __builtin_memcpy(&v, p + off, sizeof(T));
    return v;
  }
};
// the values of one key (reduce): n values, fixed width w or offsets off[n+1]
struct Values {
  const u8* d;
  const i64* off;
  i64 w;
  i64 n;
  __device__ Bytes operator[](i64 i) const {
    return off ? Bytes{d + off[i], off[i + 1] - off[i]} : Bytes{d + i * w, w};
  }
  template <class T>
  __device__ T get(i64 i, i64 byte = 0) const { return (*this)[i].template as<T>(byte); }
};
// n bytes to dst: the common widths as single wide copies
__device__ inline void put(u8* dst, const u8* src, i64 n) {
  switch (n) {
    case 0: return;
    case 4: __builtin_memcpy(dst, src, 4); return;
    case 8: __builtin_memcpy(dst, src, 8); return;
    case 12: __builtin_memcpy(dst, src, 12); return;
    case 16: __builtin_memcpy(dst, src, 16); return;
    case 24: __builtin_memcpy(dst, src, 24); return;
    default: for (i64 i = 0; i < n; ++i) dst[i] = src[i];
  }
}
// the emitter: counts in the first pass, writes in the second
struct Emit {
  bool write;
  i64 nrec, kb, vb;
  u64 kmin, kmax, vmin, vmax;
  u8* okd;
  i64* okoff;
  u8* ovd;
  i64* ovoff;
  i64 rlim, klim, vlim;  // write pass: the room the count pass measured (an impure functor cannot overrun it)
  __device__ void emit(const void* k, i64 kn, const void* v, i64 vn) {
    if (write && (nrec >= rlim || kb + kn > klim || vb + vn > vlim)) return;
    if (write) {
      if (okoff) okoff[nrec] = kb;
      if (ovoff) ovoff[nrec] = vb;
      put(okd + kb, (const u8*)k, kn);
      put(ovd + vb, (const u8*)v, vn);
    } else {
      kmin = (u64)kn < kmin ? (u64)kn : kmin;
      kmax = (u64)kn > kmax ? (u64)kn : kmax;
      vmin = (u64)vn < vmin ? (u64)vn : vmin;
      vmax = (u64)vn > vmax ? (u64)vn : vmax;
    }
    ++nrec;
    kb += kn;
    vb += vn;
  }
  template <class K, class V>
  __device__ void emit(const K& k, const V& v) { emit(&k, sizeof(K), &v, sizeof(V)); }
  template <class K>
  __device__ void emit_key(const K& k) { emit(&k, sizeof(K), nullptr, 0); }
};
}  // namespace mrd
// ---- user code ----
)MRD";

// kernels: MRD_REDUCE selects the item kind; seg null = pairs, kd null = tasks
const char* kKernels = R"MRD(
// ---- mrd kernels ----
namespace mrd {
__device__ inline Bytes field(const u8* d, const i64* off, i64 w, i64 i) {
  if (!d) return Bytes{nullptr, 0};
  return off ? Bytes{d + off[i], off[i + 1] - off[i]} : Bytes{d + i * w, w};
}
__device__ inline i64 seg_of(const i64* seg, i64 nseg, i64 j) {
  i64 lo = 0, hi = nseg;
  while (hi - lo > 1) {
    const i64 mid = (lo + hi) >> 1;
    if (seg[mid] <= j) lo = mid;
    else hi = mid;
  }
  return lo;
}
__device__ inline void run_item(const u8* kd, const i64* koff, i64 kw, const u8* vd, const i64* voff, i64 vw,
                                const i64* seg, i64 first, i64 i, Emit& e) {
#if MRD_REDUCE == 2
  // fold: vd = the merged accumulators, voff = each key's first chunk, vw = sizeof(mr_acc)
  mr_acc a;
  __builtin_memcpy(&a, vd + voff[i] * vw, sizeof(mr_acc));
  mr_finish(field(kd, koff, kw, i), a, e);
#elif MRD_REDUCE
  Values vals{vd + 0, voff, vw, seg[i + 1] - seg[i]};
  if (voff) vals.off = voff + seg[i];
  else vals.d = vd + seg[i] * vw;
  mr_reduce(field(kd, koff, kw, i), vals, e);
#else
  mr_map(field(kd, koff, kw, first + i), field(vd, voff, vw, first + i), first + i, e);
#endif
}
}  // namespace mrd
extern "C" __global__ __launch_bounds__(256) void
mrd_count(const mrd::u8* kd, const mrd::i64* koff, mrd::i64 kw, const mrd::u8* vd, const mrd::i64* voff,
          mrd::i64 vw, const mrd::i64* seg, mrd::i64 first, mrd::i64 n, mrd::i64* cnt, mrd::u64* wid, int bytes) {
  mrd::u64 kmin = ~0ull, kmax = 0, vmin = ~0ull, vmax = 0;
  for (mrd::i64 i = (mrd::i64)blockIdx.x * 256 + threadIdx.x; i < n; i += (mrd::i64)gridDim.x * 256) {
    mrd::Emit e{false, 0, 0, 0, ~0ull, 0, ~0ull, 0, nullptr, nullptr, nullptr, nullptr, 0, 0, 0};
    mrd::run_item(kd, koff, kw, vd, voff, vw, seg, first, i, e);
    cnt[i] = e.nrec;
    if (bytes) {  // the byte columns only when the widths turned out not uniform (a second count pass)
      cnt[n + i] = e.kb;
      cnt[2 * n + i] = e.vb;
    }
    kmin = e.kmin < kmin ? e.kmin : kmin;
    kmax = e.kmax > kmax ? e.kmax : kmax;
    vmin = e.vmin < vmin ? e.vmin : vmin;
    vmax = e.vmax > vmax ? e.vmax : vmax;
  }
  // the record widths: wave, then block min / max, one set of atomics per block
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    const mrd::u64 a = __shfl_xor(kmin, d, 64), b = __shfl_xor(kmax, d, 64);
    const mrd::u64 c = __shfl_xor(vmin, d, 64), e = __shfl_xor(vmax, d, 64);
    kmin = a < kmin ? a : kmin;
    kmax = b > kmax ? b : kmax;
    vmin = c < vmin ? c : vmin;
    vmax = e > vmax ? e : vmax;
  }
  __shared__ mrd::u64 red[4][4];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[w][0] = kmin;
    red[w][1] = kmax;
    red[w][2] = vmin;
    red[w][3] = vmax;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < 4; ++i) {
      kmin = red[i][0] < kmin ? red[i][0] : kmin;
      kmax = red[i][1] > kmax ? red[i][1] : kmax;
      vmin = red[i][2] < vmin ? red[i][2] : vmin;
      vmax = red[i][3] > vmax ? red[i][3] : vmax;
    }
    if (kmax || kmin != ~0ull) {
      atomicMin(wid + 0, kmin);
      atomicMax(wid + 1, kmax);
      atomicMin(wid + 2, vmin);
      atomicMax(wid + 3, vmax);
    }
  }
}
#if MRD_REDUCE == 2
// fold tier: a key's values in chunks of C, one thread per chunk (so a key
// with millions of values spreads over the whole GPU), then one thread per
// key merges its chunks' accumulators into the first
extern "C" __global__ void mrd_acc_size(mrd::i64* out) {
  if (blockIdx.x == 0 && threadIdx.x == 0) out[0] = sizeof(mr_acc);
}
extern "C" __global__ __launch_bounds__(256) void
mrd_fold_nchunks(const mrd::i64* seg, mrd::i64 nkey, mrd::i64 C, mrd::i64* cnt, mrd::u64* maxc) {
  mrd::u64 m = 0;
  for (mrd::i64 s = (mrd::i64)blockIdx.x * 256 + threadIdx.x; s < nkey; s += (mrd::i64)gridDim.x * 256) {
    cnt[s] = (seg[s + 1] - seg[s] + C - 1) / C;
    m = (mrd::u64)cnt[s] > m ? (mrd::u64)cnt[s] : m;
  }
  if (m) atomicMax(maxc, m);
}
extern "C" __global__ __launch_bounds__(256) void
mrd_fold_chunks(const mrd::u8* kd, const mrd::i64* koff, mrd::i64 kw, const mrd::u8* vd, const mrd::i64* voff,
                mrd::i64 vw, const mrd::i64* seg, mrd::i64 nkey, const mrd::i64* cstart, mrd::i64 nchunk,
                mrd::i64 C, mrd::u8* accs) {
  for (mrd::i64 c = (mrd::i64)blockIdx.x * 256 + threadIdx.x; c < nchunk; c += (mrd::i64)gridDim.x * 256) {
    const mrd::i64 s = mrd::seg_of(cstart, nkey, c);
    const mrd::i64 a0 = seg[s] + (c - cstart[s]) * C;
    const mrd::i64 a1 = a0 + C < seg[s + 1] ? a0 + C : seg[s + 1];
    mr_acc a;
    mr_init(mrd::field(kd, koff, kw, s), a);
    for (mrd::i64 v = a0; v < a1; ++v) mr_add(a, mrd::field(vd, voff, vw, v));
    __builtin_memcpy(accs + c * sizeof(mr_acc), &a, sizeof(mr_acc));
  }
}
// one level of a fixed pairwise tree: chunk j of a key (j % 2*stride == 0)
// takes in chunk j + stride; log2(most chunks of a key) levels leave each
// key's total in its first chunk, in the same order on every run
extern "C" __global__ __launch_bounds__(256) void
mrd_fold_merge(const mrd::i64* cstart, mrd::i64 nkey, mrd::i64 nchunk, mrd::i64 stride, mrd::u8* accs) {
  for (mrd::i64 c = (mrd::i64)blockIdx.x * 256 + threadIdx.x; c < nchunk; c += (mrd::i64)gridDim.x * 256) {
    const mrd::i64 s = mrd::seg_of(cstart, nkey, c);
    const mrd::i64 j = c - cstart[s];
    if (j % (2 * stride) != 0 || c + stride >= cstart[s + 1]) continue;
    mr_acc a, b;
    __builtin_memcpy(&a, accs + c * sizeof(mr_acc), sizeof(mr_acc));
    __builtin_memcpy(&b, accs + (c + stride) * sizeof(mr_acc), sizeof(mr_acc));
    mr_merge(a, b);
    __builtin_memcpy(accs + c * sizeof(mr_acc), &a, sizeof(mr_acc));
  }
}
#endif
// okw / ovw >= 0: every record's key / value has that width (the count pass
// said so): byte positions follow from the record position, no offsets
extern "C" __global__ __launch_bounds__(256) void
mrd_write(const mrd::u8* kd, const mrd::i64* koff, mrd::i64 kw, const mrd::u8* vd, const mrd::i64* voff,
          mrd::i64 vw, const mrd::i64* seg, mrd::i64 first, mrd::i64 n, const mrd::i64* pr, const mrd::i64* pk,
          const mrd::i64* pv, mrd::i64 okw, mrd::i64 ovw, mrd::u8* okd, mrd::i64* okoff, mrd::u8* ovd,
          mrd::i64* ovoff) {
  // pr / pk / pv: exclusive scans (n + 1) of records, key bytes, value bytes
  // (pk / pv unused when that width is uniform: okw / ovw >= 0)
  for (mrd::i64 i = (mrd::i64)blockIdx.x * 256 + threadIdx.x; i < n; i += (mrd::i64)gridDim.x * 256) {
    const mrd::i64 r = pr[i];
    if (pr[i + 1] == r) continue;
    const mrd::i64 r1 = pr[i + 1];
    const mrd::i64 k0 = okw >= 0 ? r * okw : pk[i], v0 = ovw >= 0 ? r * ovw : pv[i];
    const mrd::i64 k1 = okw >= 0 ? r1 * okw : pk[i + 1], v1 = ovw >= 0 ? r1 * ovw : pv[i + 1];
    mrd::Emit e{true, 0, 0, 0, 0, 0, 0, 0, okd + k0, okw >= 0 ? nullptr : okoff + r, ovd + v0,
                ovw >= 0 ? nullptr : ovoff + r, r1 - r, k1 - k0, v1 - v0};
    mrd::run_item(kd, koff, kw, vd, voff, vw, seg, first, i, e);
    const mrd::i64 nw = e.nrec < r1 - r ? e.nrec : r1 - r;
    for (mrd::i64 j = 0; j < nw; ++j) {  // offsets relative to the item -> absolute
      if (okw < 0) okoff[r + j] += k0;
      if (ovw < 0) ovoff[r + j] += v0;
    }
  }
}
)MRD";

// kind 3: a sort-key functor, __device__ unsigned long long mr_sortkey(mrd::Bytes)
const char* kSortKernel = R"MRD(
// ---- mrd sort-key kernel ----
extern "C" __global__ __launch_bounds__(256) void
mrd_sortkey(const mrd::u8* d, const mrd::i64* off, mrd::i64 w, mrd::i64 n, mrd::u64* key, unsigned int* idx) {
  for (mrd::i64 i = (mrd::i64)blockIdx.x * 256 + threadIdx.x; i < n; i += (mrd::i64)gridDim.x * 256) {
    const mrd::Bytes b = off ? mrd::Bytes{d + off[i], off[i + 1] - off[i]} : mrd::Bytes{d + i * w, w};
    key[i] = mr_sortkey(b);
    idx[i] = (unsigned int)i;
  }
}
)MRD";

struct Module {
  hipModule_t mod = nullptr;
  hipFunction_t count = nullptr, write = nullptr;
  hipFunction_t acc_size = nullptr, nchunks = nullptr, chunks = nullptr, merge = nullptr;  // fold tier
};
const char* kind_name(int kind) {
  return kind == 0 ? "mrd_map.hip" : kind == 1 ? "mrd_reduce.hip" : kind == 2 ? "mrd_fold.hip" : "mrd_sortkey.hip";
}
std::string source_of(const std::string& code, int kind) {
  if (kind == 3) return std::string(kDevicePrelude) + code + "\n" + kSortKernel;
  return "#define MRD_REDUCE " + std::to_string(kind) + "\n" + kDevicePrelude + code + "\n" + kKernels;
}

std::string compile(const std::string& src, const char* name) {
  hiprtcProgram p;
  if (hiprtcCreateProgram(&p, src.c_str(), name, 0, nullptr, nullptr) != HIPRTC_SUCCESS)
    throw std::runtime_error("mrhip: hiprtcCreateProgram failed");
  const char* opts[] = {"--offload-arch=gfx950", "-O3", "-std=c++17"};
  const hiprtcResult r = hiprtcCompileProgram(p, 3, opts);
  size_t ls = 0;
  hiprtcGetProgramLogSize(p, &ls);
  std::string log(ls, '\0');
  if (ls) hiprtcGetProgramLog(p, &log[0]);
  if (r != HIPRTC_SUCCESS) {
    hiprtcDestroyProgram(&p);
    throw std::runtime_error("mrhip: device functor does not compile:\n" + log);
  }
  size_t cs = 0;
  hiprtcGetCodeSize(p, &cs);
  std::string code(cs, '\0');
  hiprtcGetCode(p, &code[0]);
  hiprtcDestroyProgram(&p);
  return code;
}

const Module& module_for(const std::string& code, int kind, int device) {
  static std::mutex mu;
  static std::unordered_map<std::string, std::unique_ptr<Module>> cache;
  const std::string key = std::to_string(device) + ":" + std::to_string(kind) + ":" + code;
  std::lock_guard<std::mutex> lk(mu);
  auto it = cache.find(key);
  if (it != cache.end()) return *it->second;
  const std::string obj = compile(source_of(code, kind), kind_name(kind));
  auto m = std::make_unique<Module>();
  if (kind == 3) {
    if (hipModuleLoadData(&m->mod, obj.data()) != hipSuccess ||
        hipModuleGetFunction(&m->count, m->mod, "mrd_sortkey") != hipSuccess) {
      (void)hipGetLastError();
      throw std::runtime_error("mrhip: loading the sort-key functor's code object failed");
    }
    return *cache.emplace(key, std::move(m)).first->second;
  }
  if (hipModuleLoadData(&m->mod, obj.data()) != hipSuccess ||
      hipModuleGetFunction(&m->count, m->mod, "mrd_count") != hipSuccess ||
      hipModuleGetFunction(&m->write, m->mod, "mrd_write") != hipSuccess ||
      (kind == 2 && (hipModuleGetFunction(&m->acc_size, m->mod, "mrd_acc_size") != hipSuccess ||
                     hipModuleGetFunction(&m->nchunks, m->mod, "mrd_fold_nchunks") != hipSuccess ||
                     hipModuleGetFunction(&m->chunks, m->mod, "mrd_fold_chunks") != hipSuccess ||
                     hipModuleGetFunction(&m->merge, m->mod, "mrd_fold_merge") != hipSuccess))) {
    (void)hipGetLastError();
    throw std::runtime_error("mrhip: loading the device functor's code object failed");
  }
  return *cache.emplace(key, std::move(m)).first->second;
}

template <typename T>
T* P0(const at::Tensor& t) {
  return t.defined() && t.numel() ? reinterpret_cast<T*>(t.data_ptr()) : nullptr;
}
at::TensorOptions opt(at::Device d, at::ScalarType t) { return at::TensorOptions().device(d).dtype(t); }

void launch(hipFunction_t f, int64_t n, void** args, hipStream_t s) {
  const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 65536));
  if (hipModuleLaunchKernel(f, grid, 1, 1, 256, 1, 1, 0, s, args, nullptr) != hipSuccess) {
    (void)hipGetLastError();
    throw std::runtime_error("mrhip: device functor launch failed");
  }
}

struct Items {
  const uint8_t* kd = nullptr;
  const int64_t* koff = nullptr;
  int64_t kw = 0;
  const uint8_t* vd = nullptr;
  const int64_t* voff = nullptr;
  int64_t vw = 0;
  const int64_t* seg = nullptr;
  int64_t first = 0, n = 0;
};

KV run(const Items& it, const std::string& code, int kind, at::Device dev) {
  if (!dev.is_cuda()) throw std::runtime_error("mrhip: device functors run on a GPU MapReduce (device cuda)");
  KV out;
  out.kw = out.vw = -1;
  if (it.n <= 0) {
    out.kw = out.vw = 0;
    out.kdata = at::empty({0}, opt(dev, at::kByte));
    out.vdata = at::empty({0}, opt(dev, at::kByte));
    return out;
  }
  const Module& m = module_for(code, kind, dev.index());
  hipStream_t s = at::hip::getCurrentHIPStream();
  at::Tensor cnt = at::empty({3 * it.n}, opt(dev, at::kLong));
  at::Tensor wid = at::empty({4}, opt(dev, at::kLong));
  const int64_t w0[4] = {-1, 0, -1, 0};  // ~0 = u64 max for the mins
  if (hipMemcpyAsync(wid.data_ptr(), w0, sizeof(w0), hipMemcpyHostToDevice, s) != hipSuccess)
    throw std::runtime_error("mrhip: hipMemcpyAsync failed");
  auto count = [&](int bytes) {
    const uint8_t* kd = it.kd;
    const int64_t* koff = it.koff;
    int64_t kw = it.kw, vw = it.vw, first = it.first, n = it.n;
    const uint8_t* vd = it.vd;
    const int64_t* voff = it.voff;
    const int64_t* seg = it.seg;
    int64_t* c = P0<int64_t>(cnt);
    int64_t* w = P0<int64_t>(wid);
    int b = bytes;
    void* args[] = {&kd, &koff, &kw, &vd, &voff, &vw, &seg, &first, &n, &c, &w, &b};
    launch(m.count, it.n, args, s);
  };
  count(0);
  // the record widths first: uniform widths need only the record scan (the
  // common case); otherwise a second count pass fills the byte columns
  int64_t wh[4] = {0, 0, 0, 0};
  read_small(s, {{P0<int64_t>(wid), wh, 32}});
  const int64_t okw = (wh[0] == wh[1]) ? wh[0] : -1, ovw = (wh[2] == wh[3]) ? wh[2] : -1;
  if (okw < 0 || ovw < 0) count(1);
  at::Tensor pr = exclusive_scan(cnt.narrow(0, 0, it.n));
  at::Tensor pk = okw < 0 ? exclusive_scan(cnt.narrow(0, it.n, it.n)) : at::Tensor();
  at::Tensor pv = ovw < 0 ? exclusive_scan(cnt.narrow(0, 2 * it.n, it.n)) : at::Tensor();
  int64_t tot[3] = {0, 0, 0};
  {
    const SmallRead rec{P0<int64_t>(pr) + it.n, &tot[0], 8};
    if (okw < 0 && ovw < 0)
      read_small(s, {rec, {P0<int64_t>(pk) + it.n, &tot[1], 8}, {P0<int64_t>(pv) + it.n, &tot[2], 8}});
    else if (okw < 0) read_small(s, {rec, {P0<int64_t>(pk) + it.n, &tot[1], 8}});
    else if (ovw < 0) read_small(s, {rec, {P0<int64_t>(pv) + it.n, &tot[2], 8}});
    else read_small(s, {rec});
  }
  const int64_t nout = tot[0];
  if (okw >= 0) tot[1] = nout * okw;
  if (ovw >= 0) tot[2] = nout * ovw;
  out.n = nout;
  out.kdata = at::empty({tot[1]}, opt(dev, at::kByte));
  out.vdata = at::empty({tot[2]}, opt(dev, at::kByte));
  if (nout && okw >= 0) out.kw = (int)okw;
  else out.koff = at::empty({nout + 1}, opt(dev, at::kLong));
  if (nout && ovw >= 0) out.vw = (int)ovw;
  else out.voff = at::empty({nout + 1}, opt(dev, at::kLong));
  if (nout) {
    const uint8_t* kd = it.kd;
    const int64_t* koff = it.koff;
    int64_t kw = it.kw, vw = it.vw, first = it.first, n = it.n, kwo = okw, vwo = ovw;
    const uint8_t* vd = it.vd;
    const int64_t* voff = it.voff;
    const int64_t* seg = it.seg;
    const int64_t* ppr = P0<int64_t>(pr);
    const int64_t* ppk = P0<int64_t>(pk);
    const int64_t* ppv = P0<int64_t>(pv);
    uint8_t* okd = P0<uint8_t>(out.kdata);
    uint8_t* ovd = P0<uint8_t>(out.vdata);
    int64_t* okoff = P0<int64_t>(out.koff);
    int64_t* ovoff = P0<int64_t>(out.voff);
    void* args[] = {&kd, &koff, &kw, &vd, &voff, &vw, &seg, &first, &n, &ppr, &ppk, &ppv, &kwo, &vwo, &okd, &okoff, &ovd, &ovoff};
    launch(m.write, it.n, args, s);
  }
  if (out.koff.defined()) k::fill_i64(P0<int64_t>(out.koff) + nout, 1, tot[1], s);
  if (out.voff.defined()) k::fill_i64(P0<int64_t>(out.voff) + nout, 1, tot[2], s);
  return out;
}
}  // namespace

int kind_of(const std::string& code, bool reduce) {
  return !reduce ? 0 : code.find("mr_finish") != std::string::npos ? 2 : 1;
}

std::string full_source(const std::string& code, bool reduce) { return source_of(code, kind_of(code, reduce)); }

int64_t compile_check_sortkey(const std::string& code) {
  return (int64_t)compile(source_of(code, 3), kind_name(3)).size();
}

std::pair<at::Tensor, at::Tensor> sort_keys_of(const at::Tensor& data, const at::Tensor& off, int w, int64_t n,
                                               const std::string& code, at::Device dev) {
  if (!dev.is_cuda()) throw std::runtime_error("mrhip: device functors run on a GPU MapReduce (device cuda)");
  at::Tensor key = at::empty({std::max<int64_t>(n, 1)}, opt(dev, at::kLong));
  at::Tensor idx = at::empty({std::max<int64_t>(n, 1)}, opt(dev, at::kInt));
  if (n > 0) {
    const Module& m = module_for(code, 3, dev.index());
    const uint8_t* d = P0<uint8_t>(data);
    const int64_t* o = w >= 0 ? nullptr : P0<int64_t>(off);
    int64_t ww = w >= 0 ? w : 0, nn = n;
    int64_t* k = P0<int64_t>(key);
    int32_t* ix = P0<int32_t>(idx);
    void* args[] = {&d, &o, &ww, &nn, &k, &ix};
    launch(m.count, n, args, at::hip::getCurrentHIPStream());
  }
  return {key.narrow(0, 0, n), idx.narrow(0, 0, n)};
}

int64_t compile_check(const std::string& code, bool reduce) {
  return (int64_t)compile(full_source(code, reduce), kind_name(kind_of(code, reduce))).size();
}

KV map_pairs(const KV& kv_in, const std::string& code, at::Device dev, int64_t a, int64_t b) {
  KV kv = kv_in.device() == dev ? kv_in : kv_to(kv_in, dev);
  if (b < 0 || b > kv.n) b = kv.n;
  Items it;
  it.first = a;
  it.kd = P0<uint8_t>(kv.kdata);
  it.koff = kv.kfixed() ? nullptr : P0<int64_t>(kv.koff);
  it.kw = kv.kfixed() ? kv.kw : 0;
  it.vd = P0<uint8_t>(kv.vdata);
  it.voff = kv.vfixed() ? nullptr : P0<int64_t>(kv.voff);
  it.vw = kv.vfixed() ? kv.vw : 0;
  it.n = std::max<int64_t>(0, b - a);
  return run(it, code, 0, dev);
}

KV map_tasks(int64_t first, int64_t n, const std::string& code, at::Device dev) {
  Items it;
  it.first = first;
  it.n = n;
  return run(it, code, 0, dev);
}

KV reduce_groups(const KMV& m, const std::string& code, at::Device dev) {
  if (m.nkey && !m.seg.is_cuda()) throw std::runtime_error("mrhip: reduce_device needs the groups in HBM");
  Items it;
  const KV& k = m.keys;
  it.kd = P0<uint8_t>(k.kdata);
  it.koff = k.kfixed() ? nullptr : P0<int64_t>(k.koff);
  it.kw = k.kfixed() ? k.kw : 0;
  it.vd = P0<uint8_t>(m.vdata);
  it.voff = m.vw >= 0 ? nullptr : P0<int64_t>(m.voff);
  it.vw = m.vw >= 0 ? m.vw : 0;
  it.seg = P0<int64_t>(m.seg);
  it.n = m.nkey;
  if (kind_of(code, true) == 1) return run(it, code, 1, dev);
  // fold tier: accumulators per chunk of values, merged per key, then mr_finish per key
  if (!it.n) return run(it, code, 2, dev);
  const Module& mod = module_for(code, 2, dev.index());
  hipStream_t s = at::hip::getCurrentHIPStream();
  static const int64_t C = [] {
    const char* e = std::getenv("MRH_FOLD_CHUNK");
    return e && std::atoll(e) > 0 ? std::atoll(e) : int64_t(256);
  }();
  at::Tensor asz_t = at::empty({1}, opt(dev, at::kLong));
  {
    int64_t* o = P0<int64_t>(asz_t);
    void* args[] = {&o};
    launch(mod.acc_size, 1, args, s);
  }
  at::Tensor cnt = at::empty({it.n + 1}, opt(dev, at::kLong));  // + the most chunks of one key
  if (hipMemsetAsync(P0<int64_t>(cnt) + it.n, 0, 8, s) != hipSuccess)
    throw std::runtime_error("mrhip: hipMemsetAsync failed");
  {
    const int64_t* seg = it.seg;
    int64_t nkey = it.n, c = C;
    int64_t* o = P0<int64_t>(cnt);
    int64_t* mx = o + it.n;
    void* args[] = {&seg, &nkey, &c, &o, &mx};
    launch(mod.nchunks, it.n, args, s);
  }
  at::Tensor cstart = exclusive_scan(cnt.narrow(0, 0, it.n));
  int64_t asz = 0, nchunk = 0, maxc = 0;
  read_small(s, {{P0<int64_t>(asz_t), &asz, 8}, {P0<int64_t>(cstart) + it.n, &nchunk, 8},
                 {P0<int64_t>(cnt) + it.n, &maxc, 8}});
  at::Tensor accs = at::empty({std::max<int64_t>(1, nchunk * asz)}, opt(dev, at::kByte));
  {
    const uint8_t* kd = it.kd;
    const int64_t* koff = it.koff;
    int64_t kw = it.kw, vw = it.vw, nkey = it.n, nc = nchunk, c = C;
    const uint8_t* vd = it.vd;
    const int64_t* voff = it.voff;
    const int64_t* seg = it.seg;
    const int64_t* cs = P0<int64_t>(cstart);
    uint8_t* a = P0<uint8_t>(accs);
    void* args[] = {&kd, &koff, &kw, &vd, &voff, &vw, &seg, &nkey, &cs, &nc, &c, &a};
    launch(mod.chunks, nchunk, args, s);
    for (int64_t stride = 1; stride < maxc; stride *= 2) {
      int64_t st = stride;
      void* margs[] = {&cs, &nkey, &nc, &st, &a};
      launch(mod.merge, nchunk, margs, s);
    }
  }
  Items f = it;
  f.vd = P0<uint8_t>(accs);
  f.voff = P0<int64_t>(cstart);
  f.vw = asz;
  f.seg = nullptr;
  return run(f, code, 2, dev);
}

}  // namespace devfn
}  // namespace mrh
