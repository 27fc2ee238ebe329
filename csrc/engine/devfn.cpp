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
// the emitter: counts in the first pass, writes in the second
struct Emit {
  bool write;
  i64 nrec, kb, vb;
  u64 kmin, kmax, vmin, vmax;
  u8* okd;
  i64* okoff;
  u8* ovd;
  i64* ovoff;
  __device__ void emit(const void* k, i64 kn, const void* v, i64 vn) {
    if (write) {
      if (okoff) okoff[nrec] = kb;
      if (ovoff) ovoff[nrec] = vb;
      const u8* ks = (const u8*)k;
      const u8* vs = (const u8*)v;
      for (i64 i = 0; i < kn; ++i) okd[kb + i] = ks[i];
      for (i64 i = 0; i < vn; ++i) ovd[vb + i] = vs[i];
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
__device__ inline void run_item(const u8* kd, const i64* koff, i64 kw, const u8* vd, const i64* voff, i64 vw,
                                const i64* seg, i64 first, i64 i, Emit& e) {
#if MRD_REDUCE
  Values vals{vd + 0, voff, vw, seg[i + 1] - seg[i]};
  if (voff) vals.off = voff + seg[i];
  else vals.d = vd + seg[i] * vw;
  mr_reduce(field(kd, koff, kw, i), vals, e);
#else
  mr_map(field(kd, koff, kw, i), field(vd, voff, vw, i), first + i, e);
#endif
}
}  // namespace mrd
extern "C" __global__ void __launch_bounds__(256)
mrd_count(const mrd::u8* kd, const mrd::i64* koff, mrd::i64 kw, const mrd::u8* vd, const mrd::i64* voff,
          mrd::i64 vw, const mrd::i64* seg, mrd::i64 first, mrd::i64 n, mrd::i64* cnt, mrd::u64* wid) {
  mrd::u64 kmin = ~0ull, kmax = 0, vmin = ~0ull, vmax = 0;
  for (mrd::i64 i = (mrd::i64)blockIdx.x * 256 + threadIdx.x; i < n; i += (mrd::i64)gridDim.x * 256) {
    mrd::Emit e{false, 0, 0, 0, ~0ull, 0, ~0ull, 0, nullptr, nullptr, nullptr, nullptr};
    mrd::run_item(kd, koff, kw, vd, voff, vw, seg, first, i, e);
    cnt[i] = e.nrec;
    cnt[n + i] = e.kb;
    cnt[2 * n + i] = e.vb;
    kmin = e.kmin < kmin ? e.kmin : kmin;
    kmax = e.kmax > kmax ? e.kmax : kmax;
    vmin = e.vmin < vmin ? e.vmin : vmin;
    vmax = e.vmax > vmax ? e.vmax : vmax;
  }
  if (kmax || kmin != ~0ull) {
    atomicMin(wid + 0, kmin);
    atomicMax(wid + 1, kmax);
    atomicMin(wid + 2, vmin);
    atomicMax(wid + 3, vmax);
  }
}
// okw / ovw >= 0: every record's key / value has that width (the count pass
// said so): byte positions follow from the record position, no offsets
extern "C" __global__ void __launch_bounds__(256)
mrd_write(const mrd::u8* kd, const mrd::i64* koff, mrd::i64 kw, const mrd::u8* vd, const mrd::i64* voff,
          mrd::i64 vw, const mrd::i64* seg, mrd::i64 first, mrd::i64 n, const mrd::i64* pos, mrd::i64 okw,
          mrd::i64 ovw, mrd::u8* okd, mrd::i64* okoff, mrd::u8* ovd, mrd::i64* ovoff) {
  const mrd::i64 np = n + 1;  // pos: scans of n + 1 (records, then key bytes, value bytes when variable)
  for (mrd::i64 i = (mrd::i64)blockIdx.x * 256 + threadIdx.x; i < n; i += (mrd::i64)gridDim.x * 256) {
    const mrd::i64 r = pos[i];
    if (pos[i + 1] == r) continue;
    const mrd::i64 k0 = okw >= 0 ? r * okw : pos[np + i], v0 = ovw >= 0 ? r * ovw : pos[2 * np + i];
    mrd::Emit e{true, 0, 0, 0, 0, 0, 0, 0, okd + k0, okw >= 0 ? nullptr : okoff + r, ovd + v0,
                ovw >= 0 ? nullptr : ovoff + r};
    mrd::run_item(kd, koff, kw, vd, voff, vw, seg, first, i, e);
    for (mrd::i64 j = 0; j < e.nrec; ++j) {  // offsets relative to the item -> absolute
      if (okw < 0) okoff[r + j] += k0;
      if (ovw < 0) ovoff[r + j] += v0;
    }
  }
}
)MRD";

struct Module {
  hipModule_t mod = nullptr;
  hipFunction_t count = nullptr, write = nullptr;
};

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

const Module& module_for(const std::string& code, bool reduce, int device) {
  static std::mutex mu;
  static std::unordered_map<std::string, std::unique_ptr<Module>> cache;
  const std::string key = std::to_string(device) + (reduce ? "R" : "M") + code;
  std::lock_guard<std::mutex> lk(mu);
  auto it = cache.find(key);
  if (it != cache.end()) return *it->second;
  const std::string obj = compile(full_source(code, reduce), reduce ? "mrd_reduce.hip" : "mrd_map.hip");
  auto m = std::make_unique<Module>();
  if (hipModuleLoadData(&m->mod, obj.data()) != hipSuccess ||
      hipModuleGetFunction(&m->count, m->mod, "mrd_count") != hipSuccess ||
      hipModuleGetFunction(&m->write, m->mod, "mrd_write") != hipSuccess) {
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

KV run(const Items& it, const std::string& code, bool reduce, at::Device dev) {
  if (!dev.is_cuda()) throw std::runtime_error("mrhip: device functors run on a GPU MapReduce (device cuda)");
  KV out;
  out.kw = out.vw = -1;
  if (it.n <= 0) {
    out.kw = out.vw = 0;
    out.kdata = at::empty({0}, opt(dev, at::kByte));
    out.vdata = at::empty({0}, opt(dev, at::kByte));
    return out;
  }
  const Module& m = module_for(code, reduce, dev.index());
  hipStream_t s = at::hip::getCurrentHIPStream();
  at::Tensor cnt = at::empty({3 * it.n}, opt(dev, at::kLong));
  at::Tensor wid = at::empty({4}, opt(dev, at::kLong));
  const int64_t w0[4] = {-1, 0, -1, 0};  // ~0 = u64 max for the mins
  if (hipMemcpyAsync(wid.data_ptr(), w0, sizeof(w0), hipMemcpyHostToDevice, s) != hipSuccess)
    throw std::runtime_error("mrhip: hipMemcpyAsync failed");
  {
    const uint8_t* kd = it.kd;
    const int64_t* koff = it.koff;
    int64_t kw = it.kw, vw = it.vw, first = it.first, n = it.n;
    const uint8_t* vd = it.vd;
    const int64_t* voff = it.voff;
    const int64_t* seg = it.seg;
    int64_t* c = P0<int64_t>(cnt);
    int64_t* w = P0<int64_t>(wid);
    void* args[] = {&kd, &koff, &kw, &vd, &voff, &vw, &seg, &first, &n, &c, &w};
    launch(m.count, it.n, args, s);
  }
  // the record widths first: uniform widths need only the record scan
  int64_t wh[4] = {0, 0, 0, 0};
  read_small(s, {{P0<int64_t>(wid), wh, 32}});
  const int64_t okw = (wh[0] == wh[1]) ? wh[0] : -1, ovw = (wh[2] == wh[3]) ? wh[2] : -1;
  at::Tensor pos = at::empty({3 * (it.n + 1)}, opt(dev, at::kLong));
  for (int c = 0; c < 3; ++c) {
    if ((c == 1 && okw >= 0) || (c == 2 && ovw >= 0)) continue;
    pos.narrow(0, c * (it.n + 1), it.n + 1).copy_(exclusive_scan(cnt.narrow(0, c * it.n, it.n)));
  }
  const int64_t* pp = P0<int64_t>(pos);
  int64_t tot[3] = {0, 0, 0};
  {
    const SmallRead rec{pp + it.n, &tot[0], 8}, kb{pp + 2 * (it.n + 1) - 1, &tot[1], 8},
        vb{pp + 3 * (it.n + 1) - 1, &tot[2], 8};
    if (okw < 0 && ovw < 0) read_small(s, {rec, kb, vb});
    else if (okw < 0) read_small(s, {rec, kb});
    else if (ovw < 0) read_small(s, {rec, vb});
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
    uint8_t* okd = P0<uint8_t>(out.kdata);
    uint8_t* ovd = P0<uint8_t>(out.vdata);
    int64_t* okoff = P0<int64_t>(out.koff);
    int64_t* ovoff = P0<int64_t>(out.voff);
    void* args[] = {&kd, &koff, &kw, &vd, &voff, &vw, &seg, &first, &n, &pp, &kwo, &vwo, &okd, &okoff, &ovd, &ovoff};
    launch(m.write, it.n, args, s);
  }
  if (out.koff.defined()) k::fill_i64(P0<int64_t>(out.koff) + nout, 1, tot[1], s);
  if (out.voff.defined()) k::fill_i64(P0<int64_t>(out.voff) + nout, 1, tot[2], s);
  return out;
}
}  // namespace

std::string full_source(const std::string& code, bool reduce) {
  return std::string("#define MRD_REDUCE ") + (reduce ? "1" : "0") + "\n" + kDevicePrelude + code + "\n" + kKernels;
}

int64_t compile_check(const std::string& code, bool reduce) {
  return (int64_t)compile(full_source(code, reduce), reduce ? "mrd_reduce.hip" : "mrd_map.hip").size();
}

KV map_pairs(const KV& kv_in, const std::string& code, at::Device dev) {
  KV kv = kv_in.device() == dev ? kv_in : kv_to(kv_in, dev);
  Items it;
  it.kd = P0<uint8_t>(kv.kdata);
  it.koff = kv.kfixed() ? nullptr : P0<int64_t>(kv.koff);
  it.kw = kv.kfixed() ? kv.kw : 0;
  it.vd = P0<uint8_t>(kv.vdata);
  it.voff = kv.vfixed() ? nullptr : P0<int64_t>(kv.voff);
  it.vw = kv.vfixed() ? kv.vw : 0;
  it.n = kv.n;
  return run(it, code, false, dev);
}

KV map_tasks(int64_t first, int64_t n, const std::string& code, at::Device dev) {
  Items it;
  it.first = first;
  it.n = n;
  return run(it, code, false, dev);
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
  return run(it, code, true, dev);
}

}  // namespace devfn
}  // namespace mrh
