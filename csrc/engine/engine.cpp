// Engine ops over device-resident KV/KMV tensors. Each op has two branches:
//   cuda (HIP, MI355X): hand-written kernels from csrc/kernels, on the current
//        torch stream;
//   cpu: straightforward host loops with identical semantics and identical
//        output order (they are the oracle the GPU tests compare against).
#include "hostarena.h"
#include "kv.h"
#include "xfer.h"
#include "grouper.h"

#include <ATen/hip/HIPContext.h>
#include <algorithm>
#include <chrono>
#include <cstring>
#include <condition_variable>
#include <cstdlib>
#include <map>
#include <mutex>
#include <thread>
#include <numeric>
#include <stdexcept>

#include "../kernels/hashfn.h"
#include "../kernels/launch.h"
#include "../kernels/rmatfn.h"

namespace mrh {

namespace {

hipStream_t cur_stream() { return at::hip::getCurrentHIPStream(); }


at::TensorOptions opt(at::Device d, at::ScalarType t) { return at::TensorOptions().device(d).dtype(t); }

at::Tensor scratch(size_t bytes, at::Device d) {
  return at::empty({(int64_t)std::max<size_t>(bytes, 1)}, opt(d, at::kByte));
}

template <typename T>
T* P(const at::Tensor& t) {
  return t.defined() && t.numel() ? reinterpret_cast<T*>(t.data_ptr()) : nullptr;
}
template <typename T>
T* P0(const at::Tensor& t) {  // pointer even for empty tensors with storage
  return t.defined() ? reinterpret_cast<T*>(t.data_ptr()) : nullptr;
}

[[noreturn]] void fail(const std::string& m) { throw std::runtime_error("mrhip: " + m); }

int64_t scalar_i64(const at::Tensor& t, int64_t i) { return t[i].item<int64_t>(); }

}  // namespace

// a few device scalars to the host with one stream synchronisation: each
// copied into this thread's pinned staging words (no ATen cat / to / item)
void read_small(hipStream_t s, std::initializer_list<SmallRead> items) {
  static thread_local void* stage = nullptr;
  constexpr size_t kStage = 512;
  if (!stage && hipHostMalloc(&stage, kStage, hipHostMallocDefault) != hipSuccess)
    throw std::runtime_error("mrhip: pinned staging for scalar reads failed");
  size_t off = 0;
  for (const SmallRead& r : items) {
    if (off + r.bytes > kStage) throw std::runtime_error("mrhip: read_small: too many bytes");
    if (hipMemcpyAsync(static_cast<char*>(stage) + off, r.src, r.bytes, hipMemcpyDeviceToHost, s) != hipSuccess)
      throw std::runtime_error("mrhip: read_small copy failed");
    off += (r.bytes + 7) & ~size_t(7);
  }
  if (hipStreamSynchronize(s) != hipSuccess) throw std::runtime_error("mrhip: read_small sync failed");
  off = 0;
  for (const SmallRead& r : items) {
    std::memcpy(r.dst, static_cast<char*>(stage) + off, r.bytes);
    off += (r.bytes + 7) & ~size_t(7);
  }
}

int64_t KV::nbytes() const {
  int64_t b = key_bytes() + value_bytes();
  if (!kfixed()) b += (n + 1) * 8;
  if (!vfixed()) b += (n + 1) * 8;
  return b;
}
int64_t KMV::nbytes() const {
  int64_t b = keys.nbytes() + (nkey + 1) * 8;
  b += vw >= 0 ? nval * vw : (nval ? voff[nval].item<int64_t>() : 0) + (nval + 1) * 8;
  return b;
}

// ====================================================================== construction

KV empty_kv(at::Device dev, int kw, int vw) {
  KV kv;
  kv.kdata = at::empty({0}, opt(dev, at::kByte));
  kv.vdata = at::empty({0}, opt(dev, at::kByte));
  kv.kw = kw;
  kv.vw = vw;
  if (kw < 0) kv.koff = at::zeros({1}, opt(dev, at::kLong));
  if (vw < 0) kv.voff = at::zeros({1}, opt(dev, at::kLong));
  kv.n = 0;
  return kv;
}

at::Tensor fixed_offsets(int64_t n, int w, at::Device dev) {
  return at::arange(n + 1, opt(dev, at::kLong)) * (int64_t)w;
}

KV make_kv(at::Tensor kdata, c10::optional<at::Tensor> koff, at::Tensor vdata, c10::optional<at::Tensor> voff,
           int64_t n, at::Device dev) {
  KV kv;
  kv.n = n;
  kv.kdata = kdata.contiguous().view(at::kByte).reshape({-1}).to(dev);
  kv.vdata = vdata.defined() ? vdata.contiguous().view(at::kByte).reshape({-1}).to(dev)
                             : at::empty({0}, opt(dev, at::kByte));
  if (koff && koff->defined()) {
    kv.koff = koff->to(dev, at::kLong).contiguous();
    kv.kw = -1;
    if (kv.koff.numel() != n + 1) fail("koff must have n+1 entries");
  } else {
    if (n > 0 && kv.kdata.numel() % n) fail("fixed key bytes not divisible by n");
    kv.kw = n > 0 ? (int)(kv.kdata.numel() / n) : 0;
  }
  if (voff && voff->defined()) {
    kv.voff = voff->to(dev, at::kLong).contiguous();
    kv.vw = -1;
    if (kv.voff.numel() != n + 1) fail("voff must have n+1 entries");
  } else {
    if (n > 0 && kv.vdata.numel() % n) fail("fixed value bytes not divisible by n");
    kv.vw = n > 0 ? (int)(kv.vdata.numel() / n) : 0;
  }
  return kv;
}

KV kv_to(const KV& kv, at::Device dev) {
  for (const at::Tensor* t : {&kv.kdata, &kv.vdata, &kv.koff, &kv.voff}) note_xfer(*t, dev);
  KV o = kv;
  o.kdata = to_device(kv.kdata, dev);
  o.vdata = to_device(kv.vdata, dev);
  if (kv.koff.defined()) o.koff = to_device(kv.koff, dev);
  if (kv.voff.defined()) o.voff = to_device(kv.voff, dev);
  return o;
}

KV to_var_keys(const KV& kv) {
  if (!kv.kfixed()) return kv;
  KV o = kv;
  o.koff = fixed_offsets(kv.n, kv.kw, kv.device());
  o.kw = -1;
  return o;
}
KV to_var_values(const KV& kv) {
  if (!kv.vfixed()) return kv;
  KV o = kv;
  o.voff = fixed_offsets(kv.n, kv.vw, kv.device());
  o.vw = -1;
  return o;
}

namespace {
// concat of one column (data + optional offsets)
// cat into a pinned host tensor when `pin` (one copy: no pageable
// intermediate that is pinned afterwards)
at::Tensor cat_maybe_pinned(const std::vector<at::Tensor>& ts, at::Device dev, at::ScalarType ty, bool pin) {
  if (!pin || !dev.is_cpu()) return at::cat(ts, 0);
  int64_t n = 0;
  for (auto& t : ts) n += t.numel();
  at::Tensor out = hostarena::pinned_empty({n}, ty);
  at::cat_out(out, ts, 0);
  return out;
}

void concat_col(const std::vector<const at::Tensor*>& datas, const std::vector<const at::Tensor*>& offs,
                const std::vector<int64_t>& ns, bool fixed, at::Device dev, at::Tensor* data_out,
                at::Tensor* off_out, bool pin) {
  // every part already on the device: the data by one D2D copy per part
  // straight into place, each part's offsets rebased into place by one
  // add kernel (ATen's add + cat were two kernels and a temporary per part)
  bool on_dev = dev.is_cuda() && !datas.empty();
  for (size_t i = 0; i < datas.size() && on_dev; ++i)
    on_dev = datas[i]->device() == dev && datas[i]->is_contiguous() &&
             (fixed || (offs[i]->device() == dev && offs[i]->is_contiguous() && offs[i]->scalar_type() == at::kLong));
  if (on_dev) {
    const hipStream_t s = cur_stream();
    int64_t bytes = 0, rows = 0;
    for (size_t i = 0; i < datas.size(); ++i) {
      bytes += datas[i]->numel() * datas[i]->element_size();
      rows += ns[i];
    }
    *data_out = at::empty({bytes}, opt(dev, at::kByte));
    int64_t b = 0, r = 0;
    for (size_t i = 0; i < datas.size(); ++i) {
      const int64_t nb = datas[i]->numel() * datas[i]->element_size();
      if (nb && hipMemcpyAsync(P0<uint8_t>(*data_out) + b, datas[i]->data_ptr(), (size_t)nb, hipMemcpyDeviceToDevice,
                               s) != hipSuccess)
        fail("concat: device copy failed");
      if (!fixed) {
        if (i == 0) *off_out = at::empty({rows + 1}, opt(dev, at::kLong));
        // the last part brings its end offset too
        k::add_i64(P0<int64_t>(*offs[i]), P0<int64_t>(*off_out) + r, ns[i] + (i + 1 == datas.size() ? 1 : 0), b, s);
      }
      b += nb;
      r += ns[i];
    }
    return;
  }
  std::vector<at::Tensor> d;
  for (auto* t : datas) d.push_back(t->to(dev));
  *data_out = d.empty() ? at::empty({0}, opt(dev, at::kByte)) : cat_maybe_pinned(d, dev, at::kByte, pin);
  if (fixed) return;
  std::vector<at::Tensor> o;
  int64_t base = 0;
  for (size_t i = 0; i < offs.size(); ++i) {
    at::Tensor oi = offs[i]->to(dev);
    o.push_back((i + 1 < offs.size() ? oi.narrow(0, 0, ns[i]) : oi) + base);
    base += datas[i]->numel();
  }
  *off_out = o.empty() ? at::zeros({1}, opt(dev, at::kLong)) : cat_maybe_pinned(o, dev, at::kLong, pin);
}
}  // namespace

KV concat(const std::vector<KV>& parts_in, at::Device dev, bool pin) {
  std::vector<KV> parts;
  for (auto& p : parts_in)
    if (p.n > 0) parts.push_back(p);
  if (parts.empty()) {
    int kw = parts_in.empty() ? 0 : parts_in[0].kw, vw = parts_in.empty() ? 0 : parts_in[0].vw;
    return empty_kv(dev, kw, vw);
  }
  if (parts.size() == 1) return kv_to(parts[0], dev);
  bool kf = true, vf = true;
  for (auto& p : parts) {
    kf = kf && p.kfixed() && p.kw == parts[0].kw;
    vf = vf && p.vfixed() && p.vw == parts[0].vw;
  }
  std::vector<KV> ps;
  for (auto& p : parts) {
    KV q = p;
    if (!kf) q = to_var_keys(q);
    if (!vf) q = to_var_values(q);
    ps.push_back(q);
  }
  KV o;
  o.kw = kf ? parts[0].kw : -1;
  o.vw = vf ? parts[0].vw : -1;
  std::vector<const at::Tensor*> kd, ko, vd, vo;
  std::vector<int64_t> ns;
  for (auto& p : ps) {
    kd.push_back(&p.kdata);
    ko.push_back(&p.koff);
    vd.push_back(&p.vdata);
    vo.push_back(&p.voff);
    ns.push_back(p.n);
    o.n += p.n;
  }
  concat_col(kd, ko, ns, kf, dev, &o.kdata, &o.koff, pin);
  concat_col(vd, vo, ns, vf, dev, &o.vdata, &o.voff, pin);
  return o;
}

KMV kmv_concat(const std::vector<KMV>& parts, at::Device dev, bool pin) {
  std::vector<const KMV*> ps;
  for (const KMV& m : parts)
    if (m.nkey > 0) ps.push_back(&m);
  if (ps.size() == 1) {
    KMV o = *ps[0];
    if (o.seg.device() != dev || (pin && dev.is_cpu() && o.seg.is_cpu() && !o.vdata.is_pinned())) {
      auto mv = [&](const at::Tensor& t) {
        if (!t.defined()) return t;
        note_xfer(t, dev);
        if (pin && dev.is_cpu()) return t.to(at::TensorOptions().device(at::kCPU).pinned_memory(true), false, true);
        return t.to(dev);
      };
      o.keys = concat({o.keys}, dev, pin);
      o.vdata = mv(o.vdata);
      o.voff = mv(o.voff);
      o.seg = mv(o.seg);
    }
    return o;
  }
  KMV out;
  std::vector<KV> keys, vals;
  std::vector<at::Tensor> segs;
  int64_t base = 0;
  for (const KMV* m : ps) {
    keys.push_back(m->keys);
    KV v;
    v.n = m->nval;
    v.kw = 0;
    v.vw = m->vw;
    v.kdata = at::empty({0}, opt(m->vdata.device(), at::kByte));
    v.vdata = m->vdata;
    v.voff = m->voff;
    vals.push_back(v);
    at::Tensor sg = m->seg.narrow(0, 0, m->nkey);
    note_xfer(sg, dev);
    segs.push_back(base ? sg.to(dev) + base : sg.to(dev));
    base += m->nval;
    out.nkey += m->nkey;
  }
  segs.push_back(at::full({1}, base, opt(dev, at::kLong)));
  const KV& like = parts.empty() ? KV() : parts[0].keys;
  out.keys = ps.empty() ? empty_kv(dev, like.kw, 0) : concat(keys, dev, pin);
  out.keys.vw = 0;
  KV vcat = ps.empty() ? empty_kv(dev, 0, parts.empty() ? 0 : parts[0].vw) : concat(vals, dev, pin);
  out.vdata = vcat.vdata;
  out.voff = vcat.voff;
  out.vw = vcat.vw;
  out.nval = base;
  at::Tensor sg = at::cat(segs);
  out.seg = pin && dev.is_cpu() ? sg.pin_memory() : sg;
  return out;
}

double wall_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
UploadTimes& upload_times() {
  static UploadTimes t = [] {
    UploadTimes u;
    const char* e = std::getenv("MRH_OOC_TRACE");
    u.on = e && *e == '2';
    return u;
  }();
  return t;
}

namespace {
// MRH_GATHER_KERNEL=0: pinned pieces go by one hipMemcpyAsync each instead of
// the zero-copy gather kernel (util.hip gather_pieces)
bool gather_kernel() {
  static const bool on = [] {
    const char* e = std::getenv("MRH_GATHER_KERNEL");
    return !(e && *e == '0');
  }();
  return on;
}
// the device reads this host pointer as is (pinned, mapped at the same
// address): only then does a piece go through the gather kernel
bool device_reads_host(const void* p) {
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return a.type == hipMemoryTypeHost && a.devicePointer == p;
}
// MRH_STAGE_PAGEABLE=0: pageable pieces go by ATen's copy_ (the runtime's own path)
bool stage_pageable() {
  static const bool on = [] {
    const char* e = std::getenv("MRH_STAGE_PAGEABLE");
    return !(e && *e == '0');
  }();
  return on;
}
// Pageable host data (a disk-tier piece: a memory-mapped spool file) goes to
// the device through this ring of pinned staging buffers: memcpy into a free
// buffer, hipMemcpyAsync from it, an event per buffer. A hipMemcpyAsync
// straight from pageable memory has the runtime pin the pages (or stage) on
// every call; after a job that held ~180 GB of HBM that path ran ~2x slower
// and made the out-of-core collate's disk-tier partitions host-bound
// (docs/round6.md).
// memcpy of large host ranges split over a few persistent threads (page-cache
// data behind a spool file is copied at ~8 GB/s by one thread; the PCIe link
// takes ~55 GB/s)
class CopyPool {
 public:
  static CopyPool& get() {
    static CopyPool* p = new CopyPool();  // never destroyed: detached workers
    return *p;
  }
  void copy(void* dst, const void* src, size_t n) {
    const int T = (int)workers_;
    if (n < (size_t(1) << 20) || T <= 1) {
      std::memcpy(dst, src, n);
      return;
    }
    const size_t part = (n / (size_t)(T + 1) + 4095) & ~size_t(4095);
    std::unique_lock<std::mutex> l(mu_);
    jobs_.clear();
    size_t o = 0;
    for (int i = 0; i < T && o < n; ++i) {
      const size_t len = std::min(part, n - o);
      jobs_.push_back({static_cast<char*>(dst) + o, static_cast<const char*>(src) + o, len});
      o += len;
    }
    pending_ = (int)jobs_.size();
    next_ = 0;
    ++gen_;
    cv_.notify_all();
    l.unlock();
    if (o < n) std::memcpy(static_cast<char*>(dst) + o, static_cast<const char*>(src) + o, n - o);  // the caller's share
    l.lock();
    done_.wait(l, [&] { return pending_ == 0; });
  }

 private:
  struct Job {
    char* d;
    const char* s;
    size_t n;
  };
  CopyPool() {
    const char* e = std::getenv("MRH_COPY_THREADS");
    workers_ = (size_t)std::max(0, e && *e ? std::atoi(e) : 7);
    for (size_t i = 0; i < workers_; ++i) std::thread([this] { loop(); }).detach();
  }
  void loop() {
    uint64_t seen = 0;
    std::unique_lock<std::mutex> l(mu_);
    for (;;) {
      cv_.wait(l, [&] { return gen_ != seen && next_ < jobs_.size(); });
      const Job j = jobs_[next_++];
      if (next_ >= jobs_.size()) seen = gen_;
      l.unlock();
      std::memcpy(j.d, j.s, j.n);
      l.lock();
      if (--pending_ == 0) done_.notify_all();
    }
  }
  std::mutex mu_;
  std::condition_variable cv_, done_;
  std::vector<Job> jobs_;
  size_t next_ = 0, workers_ = 0;
  int pending_ = 0;
  uint64_t gen_ = 0;
};

class StageRing {
 public:
  static StageRing& get() {
    static StageRing* r = new StageRing();  // never destroyed (pinned memory, events)
    return *r;
  }
  void copy(void* dst, const void* src, size_t bytes, hipStream_t s) {
    std::lock_guard<std::mutex> l(mu_);
    init();
    const char* p = static_cast<const char*>(src);
    char* d = static_cast<char*>(dst);
    while (bytes > 0) {
      Buf& b = bufs_[next_++ % bufs_.size()];
      UploadTimes& ut = upload_times();
      const double t0 = ut.on ? wall_s() : 0;
      if (b.used && hipEventSynchronize(b.ev) != hipSuccess) throw std::runtime_error("mrhip: staging wait failed");
      const double t1 = ut.on ? wall_s() : 0;
      const size_t n = std::min(bytes, kBuf);
      CopyPool::get().copy(b.p, p, n);
      if (ut.on) {
        ut.stage_wait += t1 - t0;
        ut.stage_memcpy += wall_s() - t1;
      }
      if (hipMemcpyAsync(d, b.p, n, hipMemcpyHostToDevice, s) != hipSuccess ||
          hipEventRecord(b.ev, s) != hipSuccess)
        throw std::runtime_error("mrhip: staged host to device copy failed");
      b.used = true;
      p += n;
      d += n;
      bytes -= n;
    }
  }

 private:
  static constexpr size_t kBuf = size_t(16) << 20;
  struct Buf {
    void* p = nullptr;
    hipEvent_t ev = nullptr;
    bool used = false;
  };
  void init() {
    if (!bufs_.empty()) return;
    bufs_.resize(6);
    for (Buf& b : bufs_) {
      if (hipHostMalloc(&b.p, kBuf, hipHostMallocDefault) != hipSuccess ||
          hipEventCreateWithFlags(&b.ev, hipEventDisableTiming) != hipSuccess)
        throw std::runtime_error("mrhip: staging ring allocation failed");
    }
  }
  std::mutex mu_;
  std::vector<Buf> bufs_;
  size_t next_ = 0;
};
}  // namespace

at::Tensor to_device(const at::Tensor& t, at::Device dev, bool non_blocking) {
  if (!t.defined() || !dev.is_cuda() || !t.is_cpu()) return t.defined() ? t.to(dev) : t;
  if (t.is_pinned() || !t.is_contiguous() || !stage_pageable()) return t.to(dev, non_blocking);
  at::Tensor d = at::empty(t.sizes(), t.options().device(dev));
  const size_t nb = (size_t)t.numel() * t.element_size();
  if (nb) StageRing::get().copy(d.data_ptr(), t.data_ptr(), nb, at::hip::getCurrentHIPStream().stream());
  return d;
}

KV concat_upload(const std::vector<KV>& parts_in, at::Device dev, std::vector<at::Tensor>* hold) {
  std::vector<KV> parts;
  for (const KV& p : parts_in)
    if (p.n > 0) parts.push_back(p);
  if (parts.empty() || !dev.is_cuda()) return concat(parts_in, dev);
  bool kf = true, vf = true;
  for (const KV& p : parts) {
    kf = kf && p.kfixed() && p.kw == parts[0].kw;
    vf = vf && p.vfixed() && p.vw == parts[0].vw;
  }
  // one column: data bytes back to back, offsets rebased on the device
  auto column = [&](bool fixed, auto data_of, auto off_of, at::Tensor* data_out, at::Tensor* off_out) {
    int64_t bytes = 0, rows = 0;
    for (const KV& p : parts) {
      bytes += data_of(p).numel();
      rows += p.n;
    }
    UploadTimes& ut = upload_times();
    const double t0 = ut.on ? wall_s() : 0;
    *data_out = at::empty({bytes}, opt(dev, at::kByte));
    if (!fixed) *off_out = at::empty({rows + 1}, opt(dev, at::kLong));
    if (ut.on) ut.alloc += wall_s() - t0;
    int64_t b = 0, r = 0;
    const hipStream_t cs = at::hip::getCurrentHIPStream().stream();
    // a pinned source goes by one hipMemcpyAsync with the caller holding it
    // until the stream passed the copy (`hold`): ATen's copy_ costs ~50 us of
    // host time per call (checks, a host-allocator event), which at a few
    // dozen pieces per partition was the out-of-core pass's critical path
    // pinned data pieces are gathered by kernels in batches (flushed at the end)
    k::PieceTable tab;
    uint8_t* tab_dst = nullptr;
    auto flush = [&] {
      if (tab.n) k::gather_pieces(tab, tab_dst, cs);
      tab.n = 0;
    };
    auto put = [&](const at::Tensor& dst, const at::Tensor& src) {
      const double t1 = ut.on ? wall_s() : 0;
      if (hold && gather_kernel() && src.is_cpu() && src.is_contiguous() && src.is_pinned() && dst.is_contiguous() &&
          dst.scalar_type() == at::kByte && device_reads_host(src.data_ptr())) {
        if (tab.n == k::PieceTable::kMax) flush();
        tab_dst = P0<uint8_t>(*data_out);
        tab.src[tab.n] = static_cast<const uint8_t*>(src.data_ptr());
        tab.dst_off[tab.n] = P0<uint8_t>(dst) - tab_dst;
        tab.bytes[tab.n] = (int64_t)src.numel() * src.element_size();
        ++tab.n;
        hold->push_back(src);
        if (ut.on) {
          ut.pinned += wall_s() - t1;
          ++ut.pinned_calls;
        }
      } else if (hold && src.is_cpu() && src.is_contiguous() && src.is_pinned()) {
        const size_t nb = (size_t)src.numel() * src.element_size();
        if (hipMemcpyAsync(dst.data_ptr(), src.data_ptr(), nb, hipMemcpyHostToDevice, cs) != hipSuccess)
          throw std::runtime_error("mrhip: host to device copy failed");
        hold->push_back(src);
        if (ut.on) {
          ut.pinned += wall_s() - t1;
          ++ut.pinned_calls;
        }
      } else if (hold && src.is_cpu() && src.is_contiguous() && dst.is_contiguous() && stage_pageable()) {
        StageRing::get().copy(dst.data_ptr(), src.data_ptr(), (size_t)src.numel() * src.element_size(), cs);
        if (ut.on) {
          ut.staged += wall_s() - t1;
          ++ut.staged_calls;
        }
      } else {
        dst.copy_(src, /*non_blocking=*/true);
      }
    };
    for (const KV& p : parts) {
      const at::Tensor& d = data_of(p);
      note_xfer(d, dev);
      if (d.numel()) put(data_out->narrow(0, b, d.numel()), d);
      if (!fixed) {
        at::Tensor o = off_of(p).narrow(0, 0, p.n);
        note_xfer(o, dev);
        at::Tensor dst = off_out->narrow(0, r, p.n);
        put(dst, o);
        if (b) k::add_i64(P0<int64_t>(dst), P0<int64_t>(dst), p.n, b, cs);
      }
      b += d.numel();
      r += p.n;
    }
    flush();
    if (!fixed) k::fill_i64(P0<int64_t>(*off_out) + rows, 1, b, cs);
  };
  KV o;
  o.n = 0;
  for (const KV& p : parts) o.n += p.n;
  o.kw = kf ? parts[0].kw : -1;
  o.vw = vf ? parts[0].vw : -1;
  std::vector<KV> ps;
  for (const KV& p : parts) ps.push_back(kf ? (vf ? p : to_var_values(p)) : (vf ? to_var_keys(p) : to_var_values(to_var_keys(p))));
  parts.swap(ps);
  column(kf, [](const KV& p) -> const at::Tensor& { return p.kdata; }, [](const KV& p) -> const at::Tensor& { return p.koff; },
         &o.kdata, &o.koff);
  column(vf, [](const KV& p) -> const at::Tensor& { return p.vdata; }, [](const KV& p) -> const at::Tensor& { return p.voff; },
         &o.vdata, &o.voff);
  return o;
}

// ====================================================================== primitives

// int32 lengths or int64 values -> int64 exclusive offsets (n+1)
at::Tensor exclusive_scan(const at::Tensor& x_in) {
  at::Tensor x = x_in.contiguous();
  const int64_t n = x.numel();
  const at::Device dev = x.device();
  if (x.is_cuda()) {
    auto s = cur_stream();
    at::Tensor tmp = scratch(k::scan_temp_bytes(n), dev);
    if (x.scalar_type() == at::kInt) {
      at::Tensor out = at::empty({n + 1}, opt(dev, at::kLong));
      k::lengths_to_offsets(P0<int32_t>(x), P0<int64_t>(out), n, P0<void>(tmp), s);
      return out;
    } else if (x.scalar_type() == at::kLong) {
      at::Tensor out = at::empty({n + 1}, opt(dev, at::kLong));
      k::exclusive_scan_i64(P0<int64_t>(x), P0<int64_t>(out), n, P0<void>(tmp), s);
      return out;
    }
    fail("exclusive_scan: unsupported dtype");
  }
  at::Tensor out = at::empty({n + 1}, opt(dev, at::kLong));
  int64_t* o = P0<int64_t>(out);
  int64_t acc = 0;
  if (x.scalar_type() == at::kInt) {
    const int32_t* p = P0<int32_t>(x);
    for (int64_t i = 0; i < n; ++i) { o[i] = acc; acc += p[i]; }
  } else {
    const int64_t* p = P0<int64_t>(x);
    for (int64_t i = 0; i < n; ++i) { o[i] = acc; acc += p[i]; }
  }
  o[n] = acc;
  return out;
}

// uint32 (stored in kInt) exclusive scan -> n+1 uint32 (kInt)
at::Tensor scan_u32(const at::Tensor& x) {
  const int64_t n = x.numel();
  const at::Device dev = x.device();
  at::Tensor out = at::empty({n + 1}, opt(dev, at::kInt));
  if (x.is_cuda()) {
    at::Tensor tmp = scratch(k::scan_temp_bytes(n), dev);
    k::exclusive_scan_u32(P0<uint32_t>(x), P0<uint32_t>(out), n, P0<void>(tmp), cur_stream());
    return out;
  }
  const uint32_t* p = P0<uint32_t>(x);
  uint32_t* o = P0<uint32_t>(out);
  uint32_t acc = 0;
  for (int64_t i = 0; i < n; ++i) { o[i] = acc; acc += p[i]; }
  o[n] = acc;
  return out;
}

std::tuple<at::Tensor, at::Tensor, int64_t> radix_sort_pairs(const at::Tensor& keys_in, const at::Tensor& vals_in,
                                                              int begin_bit, int end_bit, bool skip_trivial) {
  at::Tensor keys = keys_in.contiguous();
  at::Tensor vals = vals_in.contiguous();
  const int64_t n = keys.numel();
  const at::Device dev = keys.device();
  if (keys.scalar_type() != at::kLong || vals.scalar_type() != at::kInt) fail("radix_sort_pairs: keys int64, vals int32");
  if (vals.numel() != n || vals.device() != dev) fail("radix_sort_pairs: one int32 value per key, on the keys' device");
  if (begin_bit < 0 || end_bit > 64 || begin_bit > end_bit) fail("radix_sort_pairs: need 0 <= begin_bit <= end_bit <= 64");
  at::Tensor ko = at::empty_like(keys), vo = at::empty_like(vals);
  int passes = 0;
  if (n == 0) return {ko, vo, 0};
  if (keys.is_cuda()) {
    at::Tensor ka = at::empty_like(keys), va = at::empty_like(vals);
    at::Tensor tmp = scratch(k::radix_temp_bytes(n), dev);
    k::radix_sort_u64_u32(P0<uint64_t>(keys), P0<uint32_t>(vals), P0<uint64_t>(ko), P0<uint32_t>(vo),
                          P0<uint64_t>(ka), P0<uint32_t>(va), n, begin_bit, end_bit, P0<void>(tmp), cur_stream(),
                          &passes, skip_trivial);
    return {ko, vo, passes};
  }
  const uint64_t* k = P0<uint64_t>(keys);
  const uint32_t* v = P0<uint32_t>(vals);
  uint64_t mask = 0;
  for (int b = begin_bit; b < end_bit; ++b) mask |= (1ull << b);
  std::vector<int64_t> idx(n);
  std::iota(idx.begin(), idx.end(), 0);
  std::stable_sort(idx.begin(), idx.end(), [&](int64_t a, int64_t b) { return (k[a] & mask) < (k[b] & mask); });
  uint64_t* kop = P0<uint64_t>(ko);
  uint32_t* vop = P0<uint32_t>(vo);
  for (int64_t i = 0; i < n; ++i) {
    kop[i] = k[idx[i]];
    vop[i] = v[idx[i]];
  }
  return {ko, vo, (end_bit - begin_bit + 7) / 8};
}

at::Tensor radix_sort_keys(const at::Tensor& keys_in, int begin_bit, int end_bit, bool skip_trivial) {
  at::Tensor keys = keys_in.contiguous();
  const int64_t n = keys.numel();
  if (keys.scalar_type() != at::kLong) fail("radix_sort_keys: int64 keys");
  if (begin_bit < 0 || end_bit > 64 || begin_bit > end_bit) fail("radix_sort_keys: need 0 <= begin_bit <= end_bit <= 64");
  at::Tensor ko = at::empty_like(keys);
  if (n == 0) return ko;
  if (keys.is_cuda()) {
    at::Tensor ka = at::empty_like(keys);
    at::Tensor tmp = scratch(k::radix_temp_bytes(n), keys.device());
    int passes = 0;
    k::radix_sort_u64_u32(P0<uint64_t>(keys), nullptr, P0<uint64_t>(ko), nullptr, P0<uint64_t>(ka), nullptr, n,
                          begin_bit, end_bit, P0<void>(tmp), cur_stream(), &passes, skip_trivial);
    return ko;
  }
  uint64_t mask = 0;
  for (int b = begin_bit; b < end_bit; ++b) mask |= (1ull << b);
  const uint64_t* k = P0<uint64_t>(keys);
  uint64_t* o = P0<uint64_t>(ko);
  std::copy(k, k + n, o);
  std::stable_sort(o, o + n, [&](uint64_t a, uint64_t b) { return (a & mask) < (b & mask); });
  return ko;
}

at::Tensor hash32_keys(const KV& kv, uint32_t seed) {
  const at::Device dev = kv.device();
  at::Tensor out = at::empty({kv.n}, opt(dev, at::kInt));
  if (kv.n == 0) return out;
  if (dev.is_cuda()) {
    if (kv.kfixed())
      k::hash32_fixed(P0<uint8_t>(kv.kdata), kv.kw, kv.n, seed, P0<uint32_t>(out), cur_stream());
    else
      k::hash32_var(P0<uint8_t>(kv.kdata), P0<int64_t>(kv.koff), kv.n, seed, P0<uint32_t>(out), cur_stream());
    return out;
  }
  const uint8_t* d = P0<uint8_t>(kv.kdata);
  uint32_t* o = P0<uint32_t>(out);
  if (kv.kfixed()) {
    for (int64_t i = 0; i < kv.n; ++i) o[i] = dev::hashlittle(d + i * kv.kw, kv.kw, seed);
  } else {
    const int64_t* off = P0<int64_t>(kv.koff);
    for (int64_t i = 0; i < kv.n; ++i) o[i] = dev::hashlittle(d + off[i], off[i + 1] - off[i], seed);
  }
  return out;
}

at::Tensor hash64_keys(const KV& kv) {
  const at::Device dev = kv.device();
  at::Tensor out = at::empty({kv.n}, opt(dev, at::kLong));
  if (kv.n == 0) return out;
  if (dev.is_cuda()) {
    if (kv.kfixed())
      k::hash64_fixed(P0<uint8_t>(kv.kdata), kv.kw, kv.n, P0<uint64_t>(out), cur_stream());
    else
      k::hash64_var(P0<uint8_t>(kv.kdata), P0<int64_t>(kv.koff), kv.n, P0<uint64_t>(out), cur_stream());
    return out;
  }
  const uint8_t* d = P0<uint8_t>(kv.kdata);
  uint64_t* o = P0<uint64_t>(out);
  if (kv.kfixed()) {
    for (int64_t i = 0; i < kv.n; ++i) o[i] = dev::hash64(d + i * kv.kw, kv.kw);
  } else {
    const int64_t* off = P0<int64_t>(kv.koff);
    for (int64_t i = 0; i < kv.n; ++i) o[i] = dev::hash64(d + off[i], off[i + 1] - off[i]);
  }
  return out;
}

// gather rows of a column. perm: int32 (u32) or int64 row indices.
at::Tensor gather_rows(const at::Tensor& data, const at::Tensor& off, int w, const at::Tensor& perm,
                       at::Tensor* new_off) {
  const at::Device dev = data.device();
  const int64_t n = perm.numel();
  const bool i64 = perm.scalar_type() == at::kLong;
  if (w >= 0) {
    at::Tensor out = at::empty({n * w}, opt(dev, at::kByte));
    if (n == 0 || w == 0) return out;
    if (dev.is_cuda()) {
      if (i64)
        k::gather_fixed_i64idx(P0<uint8_t>(data), w, P0<int64_t>(perm), n, P0<uint8_t>(out), cur_stream());
      else
        k::gather_fixed(P0<uint8_t>(data), w, P0<uint32_t>(perm), n, P0<uint8_t>(out), cur_stream());
      return out;
    }
    const uint8_t* s = P0<uint8_t>(data);
    uint8_t* o = P0<uint8_t>(out);
    for (int64_t i = 0; i < n; ++i) {
      int64_t r = i64 ? P0<int64_t>(perm)[i] : (int64_t)P0<uint32_t>(perm)[i];
      memcpy(o + i * w, s + r * w, w);
    }
    return out;
  }
  at::Tensor p32 = i64 ? perm.to(at::kInt) : perm;  // row ids < 2^32 by construction
  if (dev.is_cuda()) {
    at::Tensor len = at::empty({n}, opt(dev, at::kInt));
    k::gather_var_lengths(P0<int64_t>(off), P0<uint32_t>(p32), n, P0<int32_t>(len), cur_stream());
    *new_off = exclusive_scan(len);
    int64_t tot = n ? scalar_i64(*new_off, n) : 0;
    at::Tensor out = at::empty({tot}, opt(dev, at::kByte));
    k::gather_var_copy(P0<uint8_t>(data), P0<int64_t>(off), P0<uint32_t>(p32), n, P0<uint8_t>(out),
                       P0<int64_t>(*new_off), cur_stream());
    return out;
  }
  const int64_t* so = P0<int64_t>(off);
  const uint32_t* pp = P0<uint32_t>(p32);
  *new_off = at::empty({n + 1}, opt(dev, at::kLong));
  int64_t* no = P0<int64_t>(*new_off);
  int64_t acc = 0;
  for (int64_t i = 0; i < n; ++i) {
    no[i] = acc;
    acc += so[pp[i] + 1] - so[pp[i]];
  }
  no[n] = acc;
  at::Tensor out = at::empty({acc}, opt(dev, at::kByte));
  const uint8_t* s = P0<uint8_t>(data);
  uint8_t* o = P0<uint8_t>(out);
  for (int64_t i = 0; i < n; ++i) memcpy(o + no[i], s + so[pp[i]], no[i + 1] - no[i]);
  return out;
}

KV gather(const KV& kv, const at::Tensor& perm) {
  KV o;
  o.n = perm.numel();
  o.kw = kv.kw;
  o.vw = kv.vw;
  o.kdata = gather_rows(kv.kdata, kv.koff, kv.kw, perm, &o.koff);
  o.vdata = gather_rows(kv.vdata, kv.voff, kv.vw, perm, &o.voff);
  return o;
}

// ====================================================================== group-by

namespace {

at::Tensor iota_u32(int64_t n, at::Device dev) {
  at::Tensor t = at::empty({n}, opt(dev, at::kInt));
  if (n == 0) return t;
  if (dev.is_cuda()) {
    k::iota_u32(P0<uint32_t>(t), n, cur_stream());
  } else {
    uint32_t* p = P0<uint32_t>(t);
    for (int64_t i = 0; i < n; ++i) p[i] = (uint32_t)i;
  }
  return t;
}

// fixed keys <= 8 bytes -> raw little-endian uint64 (exact group key)
at::Tensor raw_keys_u64(const KV& kv, int mode, bool desc, const at::Tensor& data, int w, at::Tensor* idx) {
  const at::Device dev = data.device();
  const int64_t n = kv.n;
  at::Tensor keys = at::empty({n}, opt(dev, at::kLong));
  *idx = at::empty({n}, opt(dev, at::kInt));
  if (n == 0) return keys;
  if (dev.is_cuda()) {
    k::make_sortkeys_fixed(P0<uint8_t>(data), w, n, mode, desc, P0<uint64_t>(keys), P0<uint32_t>(*idx), cur_stream());
    return keys;
  }
  const uint8_t* d = P0<uint8_t>(data);
  uint64_t* kp = P0<uint64_t>(keys);
  uint32_t* ip = P0<uint32_t>(*idx);
  for (int64_t i = 0; i < n; ++i) {
    uint64_t raw = 0;
    for (int b = 0; b < w; ++b) raw |= (uint64_t)d[i * w + b] << (8 * b);
    kp[i] = dev::sortkey(raw, mode, desc);
    ip[i] = (uint32_t)i;
  }
  return keys;
}

// sorted keys -> (flags, pos, seg, nseg)
void segments_from_sorted(const at::Tensor& sk, at::Tensor* flags, at::Tensor* pos, at::Tensor* seg, int64_t* nseg) {
  const int64_t n = sk.numel();
  const at::Device dev = sk.device();
  *flags = at::empty({n}, opt(dev, at::kInt));
  if (dev.is_cuda()) {
    k::head_flags_u64(P0<uint64_t>(sk), n, P0<uint32_t>(*flags), cur_stream());
  } else {
    const uint64_t* k = P0<uint64_t>(sk);
    uint32_t* f = P0<uint32_t>(*flags);
    for (int64_t i = 0; i < n; ++i) f[i] = (i == 0 || k[i] != k[i - 1]) ? 1u : 0u;
  }
  *pos = scan_u32(*flags);
  *nseg = (int64_t)(uint32_t)(*pos)[n].item<int32_t>();
  *seg = at::empty({*nseg + 1}, opt(dev, at::kLong));
  if (dev.is_cuda()) {
    k::compact_heads(P0<uint32_t>(*flags), P0<uint32_t>(*pos), n, P0<int64_t>(*seg), cur_stream());
  } else {
    const uint32_t* f = P0<uint32_t>(*flags);
    const uint32_t* p = P0<uint32_t>(*pos);
    int64_t* s = P0<int64_t>(*seg);
    for (int64_t i = 0; i < n; ++i)
      if (f[i]) s[p[i]] = i;
    s[*nseg] = n;
  }
}

// exact host regroup used only when a 64-bit hash collision was detected
void exact_regroup_host(const KV& kv, const at::Tensor& h64_sorted_dev, at::Tensor* perm_dev, at::Tensor* seg_dev,
                        int64_t* nseg) {
  const at::Device dev = kv.device();
  KV h = kv_to(kv, at::kCPU);
  at::Tensor perm = perm_dev->to(at::kCPU);
  at::Tensor hs = h64_sorted_dev.to(at::kCPU);
  const int64_t n = kv.n;
  const uint8_t* d = P0<uint8_t>(h.kdata);
  const int64_t* off = h.kfixed() ? nullptr : P0<int64_t>(h.koff);
  auto kp = [&](uint32_t r) { return d + (off ? off[r] : (int64_t)r * h.kw); };
  auto kl = [&](uint32_t r) { return off ? off[r + 1] - off[r] : (int64_t)h.kw; };
  uint32_t* pp = P0<uint32_t>(perm);
  const uint64_t* hp = P0<uint64_t>(hs);
  std::vector<int64_t> idx(n);
  std::iota(idx.begin(), idx.end(), 0);
  auto less = [&](int64_t a, int64_t b) {
    if (hp[a] != hp[b]) return hp[a] < hp[b];
    int64_t la = kl(pp[a]), lb = kl(pp[b]);
    int c = memcmp(kp(pp[a]), kp(pp[b]), (size_t)std::min(la, lb));
    if (c) return c < 0;
    return la < lb;
  };
  std::stable_sort(idx.begin(), idx.end(), less);
  at::Tensor np = at::empty({n}, opt(at::kCPU, at::kInt));
  uint32_t* npp = P0<uint32_t>(np);
  std::vector<int64_t> segs;
  for (int64_t i = 0; i < n; ++i) {
    npp[i] = pp[idx[i]];
    if (i == 0 || less(idx[i - 1], idx[i])) segs.push_back(i);
  }
  segs.push_back(n);
  *nseg = (int64_t)segs.size() - 1;
  *perm_dev = np.to(dev);
  *seg_dev = at::from_blob(segs.data(), {(int64_t)segs.size()}, opt(at::kCPU, at::kLong)).clone().to(dev);
}

at::Tensor seg_heads(const at::Tensor& seg, int64_t nseg) { return seg.narrow(0, 0, nseg); }

}  // namespace

at::Tensor segments_from_flags(const at::Tensor& flags_in) {
  const at::Tensor flags = flags_in.contiguous();
  const int64_t n = flags.numel();
  const at::Device dev = flags.device();
  if (n == 0) return at::zeros({1}, opt(dev, at::kLong));
  at::Tensor pos = scan_u32(flags);
  const int64_t nseg = (int64_t)(uint32_t)pos[n].item<int32_t>();
  at::Tensor seg = at::empty({nseg + 1}, opt(dev, at::kLong));
  if (dev.is_cuda()) {
    k::compact_heads(P0<uint32_t>(flags), P0<uint32_t>(pos), n, P0<int64_t>(seg), cur_stream());
  } else {
    const uint32_t* f = P0<uint32_t>(flags);
    const uint32_t* p = P0<uint32_t>(pos);
    int64_t* sp = P0<int64_t>(seg);
    for (int64_t i = 0; i < n; ++i)
      if (f[i]) sp[p[i]] = i;
    sp[nseg] = n;
  }
  return seg;
}

at::Tensor segments_from_bits(const at::Tensor& heads, int64_t n) {
  const at::Device dev = heads.device();
  if (n == 0) return at::zeros({1}, opt(dev, at::kLong));
  const int64_t nw = (n + 63) / 64;
  if (heads.scalar_type() != at::kInt || !heads.is_contiguous() || heads.numel() < 2 * nw)
    fail("segments_from_bits: int32 head words covering n bits");
  if (!dev.is_cuda()) {
    const uint32_t* h = P0<uint32_t>(heads);
    std::vector<int64_t> v;
    for (int64_t i = 0; i < n; ++i)
      if (h[i >> 5] >> (i & 31) & 1u) v.push_back(i);
    v.push_back(n);
    return at::tensor(v, opt(at::kCPU, at::kLong));
  }
  at::Tensor cnt = at::empty({nw}, opt(dev, at::kInt));
  const uint64_t* h64 = reinterpret_cast<const uint64_t*>(heads.data_ptr());
  k::bits_count(h64, nw, P0<uint32_t>(cnt), cur_stream());
  at::Tensor pos = scan_u32(cnt);
  const int64_t nseg = (int64_t)(uint32_t)pos[nw].item<int32_t>();
  at::Tensor seg = at::empty({nseg + 1}, opt(dev, at::kLong));
  k::bits_compact(h64, nw, P0<uint32_t>(pos), n, P0<int64_t>(seg), cur_stream());
  return seg;
}

at::Tensor segments_sorted(const at::Tensor& sorted_keys) {
  at::Tensor flags, pos, seg;
  int64_t nseg = 0;
  segments_from_sorted(sorted_keys.contiguous(), &flags, &pos, &seg, &nseg);
  return seg;
}

// Fixed keys of 2..8 8-byte words (edges, vertex pairs, small tuples) whose
// words, read as unsigned integers, need <= 64 significant bits together
// (an R-MAT-20 edge: 20 + 20) are grouped exactly on one packed u64: no
// 64-bit hash, no verification gather of every key, and the radix sort runs
// only over the packed bits. Returns the packed bit count (0: not narrow).
// per-column minima then maxima of a row-major [rows, cols] int64 matrix
// into out[2 cols] (device: the engine's kernels and one small read; empty:
// LLONG_MAX / LLONG_MIN)
void col_minmax(const at::Tensor& m, int cols, int64_t* out) {
  const int64_t rows = cols ? m.numel() / cols : 0;
  if (m.is_cuda()) {
    const hipStream_t s = cur_stream();
    at::Tensor tmp = at::empty({k::minmax_scratch_words(rows, cols) + 2 * cols}, opt(m.device(), at::kLong));
    int64_t* res = P0<int64_t>(tmp) + k::minmax_scratch_words(rows, cols);
    k::col_minmax_i64(P0<int64_t>(m), rows, cols, P0<int64_t>(tmp), res, s);
    if (hipMemcpyAsync(out, res, (size_t)(2 * cols) * 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
      fail("column range read failed");
    return;
  }
  const int64_t* p = P0<int64_t>(m);
  for (int c = 0; c < cols; ++c) {
    out[c] = INT64_MAX;
    out[cols + c] = INT64_MIN;
  }
  for (int64_t r = 0; r < rows; ++r)
    for (int c = 0; c < cols; ++c) {
      out[c] = std::min(out[c], p[r * cols + c]);
      out[cols + c] = std::max(out[cols + c], p[r * cols + c]);
    }
}

int narrow_keys(const KV& kv, at::Tensor* keys, at::Tensor* idx) {
  if (!kv.kfixed() || kv.kw <= 8 || kv.kw % 8 || kv.kw > 64 || kv.n == 0) return 0;
  if (!kv.kdata.is_contiguous() || reinterpret_cast<uintptr_t>(kv.kdata.data_ptr()) % 8 ||
      kv.kdata.numel() < kv.n * kv.kw)
    return 0;
  const int nw = kv.kw / 8;
  at::Tensor words = kv.kdata.narrow(0, 0, kv.n * kv.kw).view(at::kLong).view({kv.n, nw});
  // unsigned significance: a negative word (top bit set) needs all 64 bits
  std::vector<int64_t> both(2 * nw);
  col_minmax(words, nw, both.data());
  const int64_t* b = both.data();
  k::PackShifts sh{};
  sh.nw = nw;
  int total = 0;
  for (int w = 0; w < nw; ++w) {
    const int64_t lo = b[w], hi = b[nw + w];
    const int bits = lo < 0 ? 64 : (hi == 0 ? 0 : 64 - __builtin_clzll((uint64_t)hi));
    sh.s[w] = bits ? total : -1;
    total += bits;
  }
  if (total > 64) return 0;
  const at::Device dev = kv.device();
  *keys = at::empty({kv.n}, opt(dev, at::kLong));
  *idx = at::empty({kv.n}, opt(dev, at::kInt));
  if (dev.is_cuda()) {
    k::pack_words(reinterpret_cast<const uint64_t*>(kv.kdata.data_ptr()), kv.n, sh, P0<uint64_t>(*keys),
                  P0<uint32_t>(*idx), cur_stream());
  } else {
    const uint64_t* kd = reinterpret_cast<const uint64_t*>(kv.kdata.data_ptr());
    uint64_t* o = P0<uint64_t>(*keys);
    uint32_t* ip = P0<uint32_t>(*idx);
    for (int64_t i = 0; i < kv.n; ++i) {
      uint64_t k = 0;
      for (int w = 0; w < nw; ++w)
        if (sh.s[w] >= 0) k |= kd[i * nw + w] << sh.s[w];
      o[i] = k;
      ip[i] = (uint32_t)i;
    }
  }
  return std::max(total, 1);
}

// MRH_PACKED_PAIRS=0: group every pair through the key sort + index gathers
bool packed_pairs_disabled() {
  static const bool off = [] {
    const char* e = std::getenv("MRH_PACKED_PAIRS");
    return e && *e == '0';
  }();
  return off;
}

// Fixed keys of 8-byte words and fixed 8-byte values whose significant bits
// fit one u64 together — the pairs of graph collates: (vertex, vertex),
// (edge, vertex), ... — are grouped on (packed key << vbits | value): one
// keys-only radix sort over the key bits (stable: every group keeps its
// values in input order), no index column, no gather of keys or values
// afterwards (the values are the low bits, the unique keys unpacked from
// the heads). The pairs may come in parts (a KV with appended parts,
// mapreduce.h): each part is packed in place into its rows of the sort
// input and released, nothing is concatenated. Values may be 4 or 8 bytes.
// Key + value bits past 64 (R-MAT-22 wedges: 44 + 22), or more than 2^31
// pairs, take B bucket bits, a stable partition, then one sort per bucket.
// Up to 2^31 pairs the buckets are the top B key bits (keys come out in key
// order, however skewed the buckets); past that they are (low B key bits) ^
// mix(other key bits) — balanced for skewed keys, and invertible — and keys
// come out bucket by bucket, in key order inside a bucket. Returns false when
// the pairs are not that narrow.
namespace {
inline uint32_t split_mix_host(uint64_t rest, int B) {
  return B ? (uint32_t)((rest * 0x9E3779B97F4A7C15ull) >> (64 - B)) : 0u;
}
// host twins of kvops.hip split_cut / split_join
inline uint32_t split_cut_host(uint64_t K, int B, int hi, uint64_t* rest) {
  if (hi >= 0) {
    *rest = hi >= 64 ? K : (K & ((1ull << hi) - 1));
    return hi >= 64 ? 0u : (uint32_t)(K >> hi);
  }
  *rest = B ? K >> B : K;
  return B ? (uint32_t)(K & ((1ull << B) - 1)) ^ split_mix_host(*rest, B) : 0u;
}
inline uint64_t split_join_host(uint64_t rest, uint32_t bucket, int B, int hi) {
  if (hi >= 0) return hi >= 64 ? rest : (((uint64_t)bucket << hi) | rest);
  return B ? (rest << B) | (uint64_t)((bucket ^ split_mix_host(rest, B)) & ((1u << B) - 1)) : rest;
}
}  // namespace

// sorted packed words -> segment starts (seg[ns] = n), the head words' key
// bits ((w >> vb) & (2^sbits - 1)) and every word's value (the low vb bits,
// vw bytes each, into vout): two reads of the words on the GPU
void segments_packed(const at::Tensor& sk, int vb, int sbits, int vw, uint8_t* vout, at::Tensor* seg,
                     at::Tensor* heads, int64_t* nseg) {
  const int64_t n = sk.numel();
  const at::Device dev = sk.device();
  const uint64_t km = sbits >= 64 ? ~0ull : ((1ull << sbits) - 1);
  const uint64_t* w = P0<uint64_t>(sk);
  if (dev.is_cuda()) {
    const hipStream_t s = cur_stream();
    const int64_t nt = k::seg_packed_tiles(n);
    at::Tensor cnt = at::empty({nt}, opt(dev, at::kLong));
    k::seg_packed_count(w, n, vb, km, P0<int64_t>(cnt), s);  // every tile's head count
    at::Tensor tb = exclusive_scan(cnt);                     // tb[t] = heads before tile t, tb[nt] = all
    read_small(s, {{P0<int64_t>(tb) + nt, nseg, 8}});
    *seg = at::empty({*nseg + 1}, opt(dev, at::kLong));
    *heads = at::empty({*nseg}, opt(dev, at::kLong));
    k::fill_i64(P0<int64_t>(*seg) + *nseg, 1, n, s);
    k::seg_packed_write(w, n, vb, km, P0<int64_t>(tb), P0<int64_t>(*seg), P0<uint64_t>(*heads), vout, vw, s);
    return;
  }
  std::vector<int64_t> sv;
  std::vector<uint64_t> hv;
  const uint64_t vmask = (1ull << vb) - 1;
  for (int64_t i = 0; i < n; ++i) {
    if (i == 0 || (((w[i] ^ w[i - 1]) >> vb) & km) != 0) {
      sv.push_back(i);
      hv.push_back((w[i] >> vb) & km);
    }
    if (vw == 4) reinterpret_cast<uint32_t*>(vout)[i] = (uint32_t)(w[i] & vmask);
    else reinterpret_cast<uint64_t*>(vout)[i] = w[i] & vmask;
  }
  *nseg = (int64_t)sv.size();
  sv.push_back(n);
  *seg = at::from_blob(sv.data(), {(int64_t)sv.size()}, opt(at::kCPU, at::kLong)).clone();
  *heads = at::from_blob(hv.data(), {(int64_t)hv.size()}, opt(at::kCPU, at::kLong)).clone();
}

bool convert_packed_parts(std::vector<KV>& parts_io, KMV* out, ConvertStats* st) {
  if (packed_pairs_disabled()) return false;
  std::vector<KV> parts;
  for (const KV& p : parts_io)
    if (p.n > 0) parts.push_back(p);
  if (parts.empty()) return false;
  // widths and device by value: the parts are released while packing
  const int vw = parts[0].vw, kwidth = parts[0].kw;
  if (kwidth < 8 || kwidth % 8 || kwidth > 64 || (vw != 8 && vw != 4)) return false;
  auto aligned = [&](const at::Tensor& t, int64_t bytes) {
    return t.defined() && t.is_contiguous() && reinterpret_cast<uintptr_t>(t.data_ptr()) % 8 == 0 && t.numel() >= bytes;
  };
  const at::Device dev = parts[0].device();
  const bool cuda = dev.is_cuda();
  const int nw = kwidth / 8;
  int64_t n = 0;
  for (const KV& p : parts) {
    if (p.kw != kwidth || p.vw != vw || p.device() != dev) return false;
    if (!aligned(p.kdata, p.n * p.kw) || !aligned(p.vdata, p.n * vw)) return false;
    n += p.n;
  }
  // every part's key-word and value ranges into one device table, then one
  // host sync for all of them (the engine's min/max kernels, util.hip)
  const int64_t np = (int64_t)parts.size(), row = 2 * nw + 2;
  std::vector<int64_t> allv((size_t)(np * row));
  {
    int64_t scr = 0;
    for (const KV& p : parts) scr = std::max(scr, std::max(k::minmax_scratch_words(p.n, nw), k::minmax_scratch_words(p.n, 1)));
    if (cuda) {
      at::Tensor table = at::empty({np * row}, opt(dev, at::kLong)), tmp = at::empty({scr}, opt(dev, at::kLong));
      const hipStream_t s = cur_stream();
      for (int64_t i = 0; i < np; ++i) {
        const KV& p = parts[(size_t)i];
        int64_t* t = P0<int64_t>(table) + i * row;
        k::col_minmax_i64(reinterpret_cast<const int64_t*>(p.kdata.data_ptr()), p.n, nw, P0<int64_t>(tmp), t, s);
        if (vw == 8) k::col_minmax_i64(reinterpret_cast<const int64_t*>(p.vdata.data_ptr()), p.n, 1, P0<int64_t>(tmp), t + 2 * nw, s);
        else k::minmax_i32(reinterpret_cast<const int32_t*>(p.vdata.data_ptr()), p.n, P0<int64_t>(tmp), t + 2 * nw, s);
      }
      if (hipMemcpyAsync(allv.data(), table.data_ptr(), allv.size() * 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
          hipStreamSynchronize(s) != hipSuccess)
        fail("packed convert: range read failed");
    } else {
      for (int64_t i = 0; i < np; ++i) {
        const KV& p = parts[(size_t)i];
        at::Tensor kw = p.kdata.narrow(0, 0, p.n * p.kw).view(at::kLong).view({p.n, nw});
        at::Tensor vv = p.vdata.narrow(0, 0, p.n * vw).view(vw == 8 ? at::kLong : at::kInt);
        col_minmax(kw, nw, &allv[(size_t)(i * row)]);
        auto [vmn, vmx] = at::aminmax(vv.to(at::kLong));
        allv[(size_t)(i * row + 2 * nw)] = vmn.item<int64_t>();
        allv[(size_t)(i * row + 2 * nw + 1)] = vmx.item<int64_t>();
      }
    }
  }
  const int64_t* ap = allv.data();
  std::vector<int64_t> b(row);
  for (int j = 0; j < row; ++j) {
    const bool is_min = j < nw || j == 2 * nw;
    int64_t v = ap[j];
    for (int64_t i = 1; i < np; ++i) {
      const int64_t x = ap[i * row + j];
      // signed compare is right for the bit-width test below (a negative
      // word needs all its bits either way)
      v = is_min ? std::min(v, x) : std::max(v, x);
    }
    b[j] = v;
  }
  auto bits_of = [](int64_t lo, int64_t hi, int width) {
    return lo < 0 ? width : (hi == 0 ? 0 : 64 - __builtin_clzll((uint64_t)hi));
  };
  const int vbits = std::max(1, bits_of(b[2 * nw], b[2 * nw + 1], 8 * vw));
  if (vbits >= 64) return false;
  k::PackShifts sh{}, wb{};  // key word shifts inside K (from bit 0), and their widths
  sh.nw = wb.nw = nw;
  std::vector<int> kwbits(nw);
  int kbits = 0;
  for (int w = 0; w < nw; ++w) {
    kwbits[w] = bits_of(b[w], b[nw + w], 64);
    sh.s[w] = kwbits[w] ? kbits : -1;
    wb.s[w] = kwbits[w];
    kbits += kwbits[w];
  }
  if (kbits > 64) return false;
  // B bucket bits: what does not fit one sort word, and enough buckets that
  // each stays below 2^30 pairs (sort buffers, 32-bit segment positions)
  int B = std::max(0, kbits + vbits - 64);
  // MRH_PACKED_MIXED=1 takes the mixed cut at any size (tests)
  const char* fm = std::getenv("MRH_PACKED_MIXED");
  const bool force_mixed = fm && *fm == '1';
  const bool mixed = n > (int64_t(1) << 31) || force_mixed;
  if (mixed && n > (int64_t(1) << 31)) {
    int need = 0;
    while ((n >> need) > (int64_t(1) << 30)) ++need;
    B = std::max(B, need);
  }
  if (B > 8 || B > kbits) return false;  // at most 256 buckets (the partition kernels' LDS histogram)
  const int M = 1 << B;
  const int hi = mixed ? -1 : kbits - B;  // ordered cut: bucket = K >> hi
  parts_io.clear();  // from here on this function holds the only references
  const int sbits = kbits - B;  // key bits inside a sort word, above the value
  // every part packed in place into its rows, then released
  at::Tensor words = at::empty({n}, opt(dev, at::kLong));
  at::Tensor bkt = B ? at::empty({n}, opt(dev, at::kInt)) : at::Tensor();
  int64_t row0 = 0;
  for (KV& p : parts) {
    const uint64_t* kd = reinterpret_cast<const uint64_t*>(p.kdata.data_ptr());
    uint64_t* o = P0<uint64_t>(words) + row0;
    int32_t* bo = B ? P0<int32_t>(bkt) + row0 : nullptr;
    if (cuda) {
      k::pack_kv_split(kd, p.vdata.data_ptr(), vw, p.n, sh, vbits, B, hi, o, bo, cur_stream());
    } else {
      for (int64_t i = 0; i < p.n; ++i) {
        uint64_t K = 0;
        for (int w = 0; w < nw; ++w)
          if (sh.s[w] >= 0) K |= kd[i * nw + w] << sh.s[w];
        const uint64_t v = vw == 4 ? (uint64_t)static_cast<const uint32_t*>(p.vdata.data_ptr())[i]
                                   : static_cast<const uint64_t*>(p.vdata.data_ptr())[i];
        uint64_t rest;
        const uint32_t bk = split_cut_host(K, B, hi, &rest);
        o[i] = (rest << vbits) | v;
        if (bo) bo[i] = (int32_t)bk;
      }
    }
    row0 += p.n;
    p = KV();  // the part's memory goes back while the others are packed
  }
  parts.clear();
  // buckets (B > 0): a stable partition of the sort words
  std::vector<int64_t> bcount{n};
  if (B) {
    KV w;
    w.n = n;
    w.kw = 8;
    w.vw = 0;
    w.kdata = words.view(at::kByte);
    w.vdata = at::empty({0}, opt(dev, at::kByte));
    Buckets bk = bucket_local(w, bkt, M);
    bkt = at::Tensor();
    words = bk.kv.kdata.view(at::kLong);
    bcount = bk.count;
  }
  at::Tensor vout = at::empty({n * vw}, opt(dev, at::kByte));
  std::vector<at::Tensor> keys_b, seg_b;
  int64_t v0 = 0, nseg = 0, passes = 0;
  for (int bi = 0; bi < (int)bcount.size(); ++bi) {
    const int64_t nb = bcount[bi];
    if (nb == 0) continue;
    at::Tensor wsl = words.narrow(0, v0, nb);
    at::Tensor sk = sbits > 0 ? radix_sort_keys(wsl, vbits, vbits + sbits, false) : wsl;
    passes += (sbits + 7) / 8;
    // segments, head key bits (a logical shift: the word's top bit may be
    // set) and values straight from the sorted words
    at::Tensor seg, heads;
    int64_t ns = 0;
    segments_packed(sk, vbits, sbits, vw, P0<uint8_t>(vout) + v0 * vw, &seg, &heads, &ns);
    at::Tensor kb = at::empty({ns, nw}, opt(dev, at::kLong));
    if (cuda) {
      k::unpack_split(P0<uint64_t>(heads), ns, bi, B, hi, sh, wb, P0<uint64_t>(kb), cur_stream());
    } else {
      const uint64_t* hp = P0<uint64_t>(heads);
      uint64_t* kp = P0<uint64_t>(kb);
      for (int64_t j = 0; j < ns; ++j) {
        const uint64_t K = split_join_host(hp[j], (uint32_t)bi, B, hi);
        for (int w = 0; w < nw; ++w) {
          uint64_t x = 0;
          if (sh.s[w] >= 0) {
            x = K >> sh.s[w];
            if (wb.s[w] < 64) x &= (1ull << wb.s[w]) - 1;
          }
          kp[j * nw + w] = x;
        }
      }
    }
    keys_b.push_back(kb);
    // one bucket: seg (its last entry is n) is the KMV's as it is
    seg_b.push_back(B == 0 ? seg : (v0 ? seg.narrow(0, 0, ns) + v0 : seg.narrow(0, 0, ns)));
    v0 += nb;
    nseg += ns;
  }
  words = at::Tensor();
  if (B || seg_b.empty()) seg_b.push_back(at::full({1}, n, opt(dev, at::kLong)));
  out->keys.n = nseg;
  out->keys.kw = kwidth;
  out->keys.vw = 0;
  out->keys.kdata = (keys_b.size() == 1 ? keys_b[0] : at::cat(keys_b, 0)).contiguous().view(at::kByte).view({-1});
  out->keys.vdata = at::empty({0}, opt(dev, at::kByte));
  out->vw = vw;
  out->vdata = vout;
  out->seg = seg_b.size() == 1 ? seg_b[0] : at::cat(seg_b, 0);
  out->nkey = nseg;
  out->nval = n;
  st->exact = true;
  st->passes = passes + (B ? 1 : 0);
  return true;
}

bool convert_packed_pairs(const KV& kv, KMV* out, ConvertStats* st) {
  std::vector<KV> parts{kv};
  return convert_packed_parts(parts, out, st);
}

KMV convert(const KV& kv, ConvertStats* st, int force_hash_bits, const at::Tensor& prehash) {
  const at::Device dev = kv.device();
  KMV out;
  ConvertStats local;
  if (!st) st = &local;
  if (kv.n == 0) {
    out.keys = empty_kv(dev, kv.kw, 0);
    out.vw = kv.vw;
    out.vdata = at::empty({0}, opt(dev, at::kByte));
    if (kv.vw < 0) out.voff = at::zeros({1}, opt(dev, at::kLong));
    out.seg = at::zeros({1}, opt(dev, at::kLong));
    return out;
  }
  const int64_t n = kv.n;
  if (force_hash_bits >= 64 && !prehash.defined() && !packed_pairs_disabled() && convert_packed_pairs(kv, &out, st))
    return out;
  if (n > 0xFFFFFFFFll) fail("convert: more than 2^32 pairs on one rank (only narrow pairs group past that)");
  at::Tensor sk_in, idx;
  int end_bit;
  st->exact = kv.kfixed() && kv.kw <= 8 && force_hash_bits >= 64;
  if (st->exact) {
    sk_in = raw_keys_u64(kv, 0, false, kv.kdata, kv.kw, &idx);
    end_bit = 8 * kv.kw;
  } else if (force_hash_bits >= 64 && !prehash.defined() && (end_bit = narrow_keys(kv, &sk_in, &idx)) > 0) {
    st->exact = true;  // wide fixed keys whose words carry <= 64 significant bits together (edges, tuples)
  } else {
    // keys that repeat (words, hot keys): one pass over a hash dictionary of
    // the distinct keys instead of a 64-bit sort of every pair (grouper.h)
    if (force_hash_bits >= 64 && convert_dict(kv, &out, st, prehash)) return out;
    // the 64-bit grouping hash of every key, unless the producer already
    // computed it (the pipelined InvertedIndex map hashes each file's URLs
    // while the next file is still on the PCIe link)
    if (prehash.defined()) {
      if (prehash.numel() != n || prehash.scalar_type() != at::kLong) fail("convert: prehash must be int64 [n]");
      sk_in = prehash.to(dev).contiguous();
    } else {
      sk_in = hash64_keys(kv);
    }
    if (force_hash_bits < 64) sk_in = at::bitwise_and(sk_in, (int64_t)((1ull << force_hash_bits) - 1));
    idx = iota_u32(n, dev);
    end_bit = 64;
  }
  auto [sk, perm, passes] = radix_sort_pairs(sk_in, idx, 0, end_bit);
  st->passes = passes;
  at::Tensor flags, pos, seg;
  int64_t nseg = 0;
  segments_from_sorted(sk, &flags, &pos, &seg, &nseg);
  if (!st->exact) {
    int64_t mism = 0;
    if (dev.is_cuda()) {
      at::Tensor m = at::zeros({1}, opt(dev, at::kLong));
      if (kv.kfixed())
        k::verify_groups_fixed(P0<uint8_t>(kv.kdata), kv.kw, P0<uint32_t>(perm), P0<uint32_t>(flags),
                               P0<uint32_t>(pos), P0<int64_t>(seg), n, P0<unsigned long long>(m), cur_stream());
      else
        k::verify_groups_var(P0<uint8_t>(kv.kdata), P0<int64_t>(kv.koff), P0<uint32_t>(perm), P0<uint32_t>(flags),
                             P0<uint32_t>(pos), P0<int64_t>(seg), n, P0<unsigned long long>(m), cur_stream());
      mism = m.item<int64_t>();
    } else {
      const uint8_t* d = P0<uint8_t>(kv.kdata);
      const int64_t* off = kv.kfixed() ? nullptr : P0<int64_t>(kv.koff);
      const uint32_t* pp = P0<uint32_t>(perm);
      const uint32_t* f = P0<uint32_t>(flags);
      for (int64_t i = 0; i < n; ++i) {
        if (f[i]) continue;
        uint32_t a = pp[i], b = pp[i - 1];  // sorted predecessor, same segment (as the device kernel)
        int64_t a0 = off ? off[a] : (int64_t)a * kv.kw, la = off ? off[a + 1] - a0 : kv.kw;
        int64_t b0 = off ? off[b] : (int64_t)b * kv.kw, lb = off ? off[b + 1] - b0 : kv.kw;
        if (la != lb || memcmp(d + a0, d + b0, la)) ++mism;
      }
    }
    st->collisions = mism;
    if (mism) exact_regroup_host(kv, sk, &perm, &seg, &nseg);
  }
  // unique keys: rows perm[seg[s]]
  at::Tensor head_rows = gather_rows(perm, at::Tensor(), 4, seg_heads(seg, nseg), nullptr).view(at::kInt);
  out.keys.n = nseg;
  out.keys.kw = kv.kw;
  out.keys.vw = 0;
  out.keys.kdata = gather_rows(kv.kdata, kv.koff, kv.kw, head_rows, &out.keys.koff);
  out.keys.vdata = at::empty({0}, opt(dev, at::kByte));
  out.vw = kv.vw;
  out.vdata = gather_rows(kv.vdata, kv.voff, kv.vw, perm, &out.voff);
  out.seg = seg;
  out.nkey = nseg;
  out.nval = n;
  return out;
}

KMV clone(const KV& kv) {
  KMV out;
  const at::Device dev = kv.device();
  out.keys = kv;
  out.keys.vdata = at::empty({0}, opt(dev, at::kByte));
  out.keys.voff = at::Tensor();
  out.keys.vw = 0;
  out.vdata = kv.vdata;
  out.voff = kv.voff;
  out.vw = kv.vw;
  out.seg = at::arange(0, kv.n + 1, opt(dev, at::kLong));
  out.nkey = kv.n;
  out.nval = kv.n;
  return out;
}

KMV collapse(const KV& kv_in, const std::string& key) {
  const at::Device dev = kv_in.device();
  KV kv = to_var_values(to_var_keys(kv_in));
  const int64_t n = kv.n;
  // interleave lengths [k0,v0,k1,v1,...] and bytes
  at::Tensor kl = kv.koff.narrow(0, 1, n) - kv.koff.narrow(0, 0, n);
  at::Tensor vl = kv.voff.narrow(0, 1, n) - kv.voff.narrow(0, 0, n);
  at::Tensor lens = at::stack({kl, vl}, 1).reshape({2 * n});
  at::Tensor off = exclusive_scan(lens);
  // build permutation into a combined [keys|values] byte array
  at::Tensor comb = at::cat({kv.kdata, kv.vdata}, 0);
  at::Tensor src_off_k = kv.koff.narrow(0, 0, n);
  at::Tensor src_off_v = kv.voff.narrow(0, 0, n) + kv.kdata.numel();
  at::Tensor starts = at::stack({src_off_k, src_off_v}, 1).reshape({2 * n});
  // synthetic offsets array for the combined source: row r = [starts[r], starts[r]+lens[r])
  // gather_rows needs off[r+1]-off[r] == len, so copy via a host-free torch gather
  at::Tensor vdata;
  {
    int64_t tot = n ? scalar_i64(off, 2 * n) : 0;
    at::Tensor row_of_byte = segment_ids(off, 2 * n, tot);
    at::Tensor within = at::arange(tot, opt(dev, at::kLong)) - off.narrow(0, 0, 2 * n).index_select(0, row_of_byte);
    vdata = comb.index_select(0, starts.index_select(0, row_of_byte) + within);
  }
  KMV out;
  out.keys = empty_kv(dev, -1, 0);
  std::vector<uint8_t> kb(key.begin(), key.end());
  out.keys.kdata = at::from_blob(kb.data(), {(int64_t)kb.size()}, opt(at::kCPU, at::kByte)).clone().to(dev);
  out.keys.koff = at::tensor({(int64_t)0, (int64_t)kb.size()}, opt(at::kCPU, at::kLong)).to(dev);
  out.keys.n = 1;
  out.vw = -1;
  out.vdata = vdata;
  out.voff = off;
  out.seg = at::tensor({(int64_t)0, 2 * n}, opt(at::kCPU, at::kLong)).to(dev);
  out.nkey = 1;
  out.nval = 2 * n;
  return out;
}

// ====================================================================== reduce builtins

static int dtype_code(const std::string& dt, int* width) {
  if (dt == "int32" || dt == "int") { *width = 4; return 0; }
  if (dt == "int64" || dt == "uint64") { *width = 8; return 1; }
  if (dt == "float32" || dt == "float") { *width = 4; return 2; }
  if (dt == "float64" || dt == "double") { *width = 8; return 3; }
  fail("unknown dtype " + dt);
}

KV reduce_builtin(const KMV& kmv, const std::string& op, const std::string& dtype) {
  const at::Device dev = kmv.keys.device();
  KV out = kmv.keys;
  out.n = kmv.nkey;
  const int64_t ns = kmv.nkey;
  at::Tensor seg = kmv.seg;
  if (op == "count") {
    at::Tensor c = at::empty({ns}, opt(dev, at::kInt));
    if (dev.is_cuda()) k::seg_count(P0<int64_t>(seg), ns, P0<int32_t>(c), cur_stream());
    else if (ns) c.copy_((seg.narrow(0, 1, ns) - seg.narrow(0, 0, ns)).to(at::kInt));
    out.vdata = c.view(at::kByte);
    out.vw = 4;
    out.voff = at::Tensor();
    return out;
  }
  if (op == "first" || op == "last") {
    at::Tensor rows = op == "first" ? seg.narrow(0, 0, ns) : (seg.narrow(0, 1, ns) - 1);
    out.vdata = gather_rows(kmv.vdata, kmv.voff, kmv.vw, rows, &out.voff);
    out.vw = kmv.vw;
    return out;
  }
  int w = 0;
  int dc = dtype_code(dtype, &w);
  if (ns == 0) {  // nothing on this rank (e.g. after a shuffle): an empty result of the requested width
    out.vdata = at::empty({0}, opt(dev, at::kByte));
    out.voff = at::Tensor();
    out.vw = w;
    return out;
  }
  if (kmv.vw != w) fail("reduce " + op + ": values are not fixed-width " + dtype);
  int opc = op == "sum" ? 0 : op == "min" ? 1 : op == "max" ? 2 : -1;
  if (opc < 0) fail("unknown builtin reduce op " + op);
  at::Tensor res = at::empty({ns * w}, opt(dev, at::kByte));
  if (dev.is_cuda()) {
    k::seg_reduce(P0<void>(kmv.vdata), dc, opc, P0<int64_t>(seg), ns, kmv.nval, P0<void>(res), cur_stream());
  } else if (ns) {
    const int64_t* sg = P0<int64_t>(seg);
    auto body = [&](auto* v, auto* o) {
      using T = std::remove_pointer_t<decltype(o)>;
      for (int64_t s = 0; s < ns; ++s) {
        T acc = v[sg[s]];
        for (int64_t i = sg[s] + 1; i < sg[s + 1]; ++i) {
          T x = v[i];
          acc = opc == 0 ? T(acc + x) : opc == 1 ? (x < acc ? x : acc) : (x > acc ? x : acc);
        }
        o[s] = acc;
      }
    };
    switch (dc) {
      case 0: body(P0<int32_t>(kmv.vdata), P0<int32_t>(res)); break;
      case 1: body(P0<int64_t>(kmv.vdata), P0<int64_t>(res)); break;
      case 2: body(P0<float>(kmv.vdata), P0<float>(res)); break;
      default: body(P0<double>(kmv.vdata), P0<double>(res)); break;
    }
  }
  out.vdata = res;
  out.vw = w;
  out.voff = at::Tensor();
  return out;
}

// ====================================================================== sorting

namespace {
bool flag_mode(int flag, int w, int* mode, int* bits) {
  switch (std::abs(flag)) {
    case 1: *mode = 1; *bits = 32; return w >= 4;
    case 2: *mode = 2; *bits = 64; return w >= 8;
    case 3: *mode = 3; *bits = 32; return w >= 4;
    case 4: *mode = 4; *bits = 64; return w >= 8;
    case 7: *mode = 7; *bits = 64; return w >= 8;
    case 8: *mode = 8; *bits = 32; return w >= 4;
    default: return false;
  }
}

// string order on host for tie groups (strcmp semantics: stop at NUL)
int str_cmp(const uint8_t* a, int64_t la, const uint8_t* b, int64_t lb) {
  int64_t i = 0;
  for (;; ++i) {
    int ca = i < la ? a[i] : 0, cb = i < lb ? b[i] : 0;
    if (ca != cb) return ca < cb ? -1 : 1;
    if (ca == 0) return 0;
  }
}

// Device tie-break of a string sort (flags +-5/+-6): `ks`/`perm` are sorted on
// the first 8-byte window. While some group of equal windows is still tied
// and none of its strings ended inside the window (a zero byte: equal windows
// then mean equal strings), its elements are re-keyed on the next 8 bytes and
// re-sorted inside the group — LSD: by the new window, then stably by group
// id — so only tied elements move and the order is stable throughout. Nothing
// but the tied-element count leaves the device (reference compare_str /
// compare_strn driving sort_onepage, src/mapreduce.cpp:2462-2538, 2780-2803).
at::Tensor str_tiebreak_device(at::Tensor ks, at::Tensor perm, const at::Tensor& data, const at::Tensor& off,
                               int64_t n, bool desc) {
  auto s = cur_stream();
  const at::Device dev = ks.device();
  at::Tensor head = at::empty({n}, opt(dev, at::kInt)), active = at::empty({n}, opt(dev, at::kInt));
  k::str_groups(P0<uint64_t>(ks), nullptr, nullptr, n, desc, P0<uint32_t>(head), s);
  at::Tensor alive;
  for (int64_t start = 8;; start += 8) {
    k::str_active(P0<uint64_t>(ks), alive.defined() ? P0<uint8_t>(alive) : nullptr, P0<uint32_t>(head), n, desc,
                  P0<uint32_t>(active), s);
    at::Tensor pos = scan_u32(active);
    const int64_t m = (int64_t)(uint32_t)pos[n].item<int32_t>();
    if (m == 0) break;
    at::Tensor hscan = scan_u32(head);  // hscan[i + 1] = group id of position i (1-based)
    const int64_t ngroups = (int64_t)(uint32_t)hscan[n].item<int32_t>();
    at::Tensor where = at::empty({m}, opt(dev, at::kInt)), nk = at::empty({m}, opt(dev, at::kLong)),
               gk = at::empty({m}, opt(dev, at::kLong));
    k::str_refine(P0<uint32_t>(active), P0<uint32_t>(pos), P0<uint32_t>(hscan) + 1, P0<uint32_t>(perm), P0<uint8_t>(data),
                  P0<int64_t>(off), n, start, desc, P0<int32_t>(where), P0<uint64_t>(nk), P0<uint64_t>(gk), s);
    auto r1 = radix_sort_pairs(nk, iota_u32(m, dev), 0, 64);
    at::Tensor o1 = std::get<1>(r1);
    at::Tensor g1 = gk.index_select(0, o1.to(at::kLong));
    int gbits = 1;
    while (gbits < 63 && (int64_t(1) << gbits) <= ngroups) ++gbits;
    at::Tensor o2 = std::get<1>(radix_sort_pairs(g1, o1, 0, gbits));
    at::Tensor perm2 = perm.clone();
    at::Tensor alive2 = at::zeros({n}, opt(dev, at::kByte));
    k::str_apply(P0<uint32_t>(o2), P0<int32_t>(where), P0<uint64_t>(nk), m, P0<uint32_t>(perm), P0<uint32_t>(perm2),
                 P0<uint64_t>(ks), P0<uint8_t>(alive2), s);
    perm = perm2;
    alive = alive2;
    at::Tensor head2 = at::empty({n}, opt(dev, at::kInt));
    k::str_groups(P0<uint64_t>(ks), P0<uint8_t>(alive), P0<uint32_t>(head), n, desc, P0<uint32_t>(head2), s);
    head = head2;
  }
  return perm;
}

// permutation sorting a (data, off, w) column by flag
at::Tensor sort_perm_column(const at::Tensor& data, const at::Tensor& off, int w, int64_t n, int flag) {
  const at::Device dev = data.device();
  const bool desc = flag < 0;
  int mode = 0, bits = 64;
  if (flag_mode(flag, w, &mode, &bits)) {
    KV dummy;
    dummy.n = n;
    at::Tensor idx;
    at::Tensor sk = raw_keys_u64(dummy, mode, desc, data, std::min(w, bits / 8), &idx);
    auto [ks, perm, passes] = radix_sort_pairs(sk, idx, 0, bits);
    return perm;
  }
  if (std::abs(flag) != 5 && std::abs(flag) != 6) fail("sort flag " + std::to_string(flag) + " unsupported");
  at::Tensor o = w >= 0 ? fixed_offsets(n, w, dev) : off;
  at::Tensor sk = at::empty({n}, opt(dev, at::kLong));
  at::Tensor idx = at::empty({n}, opt(dev, at::kInt));
  if (dev.is_cuda()) {
    k::make_sortkeys_strprefix(P0<uint8_t>(data), P0<int64_t>(o), n, 0, desc, P0<uint64_t>(sk), P0<uint32_t>(idx),
                               cur_stream());
  } else {
    const uint8_t* d = P0<uint8_t>(data);
    const int64_t* op = P0<int64_t>(o);
    uint64_t* kp = P0<uint64_t>(sk);
    uint32_t* ip = P0<uint32_t>(idx);
    for (int64_t i = 0; i < n; ++i) {
      uint64_t kk = 0;
      bool ended = false;  // strcmp semantics: nothing after the first NUL counts
      for (int j = 0; j < 8; ++j) {
        const uint64_t c = (!ended && op[i] + j < op[i + 1]) ? d[op[i] + j] : 0;
        ended |= c == 0;
        kk = (kk << 8) | c;
      }
      kp[i] = desc ? ~kk : kk;
      ip[i] = (uint32_t)i;
    }
  }
  auto [ks, perm, passes] = radix_sort_pairs(sk, idx, 0, 64);
  if (n < 2) return perm;
  if (dev.is_cuda()) return str_tiebreak_device(ks, perm, data, o, n, desc);
  // CPU engine: ties beyond the 8-byte prefix resolved with full strcmp semantics
  if (!at::any(ks.narrow(0, 1, n - 1) == ks.narrow(0, 0, n - 1)).item<bool>()) return perm;
  at::Tensor ksh = ks.to(at::kCPU), ph = perm.to(at::kCPU);
  at::Tensor dh = data.to(at::kCPU), oh = o.to(at::kCPU);
  const uint64_t* kk = P0<uint64_t>(ksh);
  uint32_t* pp = P0<uint32_t>(ph);
  const uint8_t* d = P0<uint8_t>(dh);
  const int64_t* op = P0<int64_t>(oh);
  bool changed = false;
  for (int64_t i = 0; i < n;) {
    int64_t j = i + 1;
    while (j < n && kk[j] == kk[i]) ++j;
    uint64_t pre = desc ? ~kk[i] : kk[i];
    bool has_nul = false;
    for (int b = 0; b < 8; ++b) has_nul |= ((pre >> (8 * b)) & 0xff) == 0;
    if (j - i > 1 && !has_nul) {
      std::stable_sort(pp + i, pp + j, [&](uint32_t a, uint32_t b) {
        int c = str_cmp(d + op[a], op[a + 1] - op[a], d + op[b], op[b + 1] - op[b]);
        return desc ? c > 0 : c < 0;
      });
      changed = true;
    }
    i = j;
  }
  return changed ? ph.to(dev) : perm;
}
}  // namespace

at::Tensor column_sort_keys(const at::Tensor& data, const at::Tensor& off, int w, int64_t n, int flag) {
  const at::Device dev = data.device();
  const bool desc = flag < 0;
  int mode = 0, bits = 64;
  if (flag_mode(flag, w, &mode, &bits)) {
    KV dummy;
    dummy.n = n;
    at::Tensor idx;
    return raw_keys_u64(dummy, mode, desc, data, std::min(w, bits / 8), &idx);
  }
  if (std::abs(flag) != 5 && std::abs(flag) != 6) fail("sort flag " + std::to_string(flag) + " unsupported");
  at::Tensor o = w >= 0 ? fixed_offsets(n, w, dev) : off;
  at::Tensor sk = at::empty({n}, opt(dev, at::kLong));
  if (n == 0) return sk;
  at::Tensor idx = at::empty({n}, opt(dev, at::kInt));
  if (dev.is_cuda()) {
    k::make_sortkeys_strprefix(P0<uint8_t>(data), P0<int64_t>(o), n, 0, desc, P0<uint64_t>(sk), P0<uint32_t>(idx),
                               cur_stream());
  } else {
    const uint8_t* d = P0<uint8_t>(data);
    const int64_t* op = P0<int64_t>(o);
    uint64_t* kp = P0<uint64_t>(sk);
    for (int64_t i = 0; i < n; ++i) {
      uint64_t kk = 0;
      bool ended = false;
      for (int j = 0; j < 8; ++j) {
        const uint64_t c = (!ended && op[i] + j < op[i + 1]) ? d[op[i] + j] : 0;
        ended |= c == 0;
        kk = (kk << 8) | c;
      }
      kp[i] = desc ? ~kk : kk;
    }
  }
  return sk;
}

KV sort_kv(const KV& kv, int flag, bool by_value) {
  if (kv.n <= 1) return kv;
  at::Tensor perm = by_value ? sort_perm_column(kv.vdata, kv.voff, kv.vw, kv.n, flag)
                             : sort_perm_column(kv.kdata, kv.koff, kv.kw, kv.n, flag);
  return gather(kv, perm);
}

// segment id of every value (int64): marks at segment starts + inclusive scan
at::Tensor segment_ids(const at::Tensor& seg_in, int64_t nseg, int64_t nval) {
  const at::Device dev = seg_in.device();
  if (nval <= 0) return at::empty({0}, opt(dev, at::kLong));
  at::Tensor seg = seg_in.contiguous();
  if (dev.is_cuda()) {
    at::Tensor marks = at::empty({nval}, opt(dev, at::kLong));
    k::seg_marks(P0<int64_t>(seg), nseg, nval, P0<int64_t>(marks), cur_stream());
    return exclusive_scan(marks).narrow(0, 1, nval);
  }
  at::Tensor out = at::empty({nval}, opt(dev, at::kLong));
  const int64_t* sp = P0<int64_t>(seg);
  int64_t* o = P0<int64_t>(out);
  int64_t s = 0;
  for (int64_t i = 0; i < nval; ++i) {
    while (s + 1 < nseg && sp[s + 1] <= i) ++s;
    o[i] = s;
  }
  return out;
}

at::Tensor bincount_dev(const at::Tensor& idx_in, int64_t K) {
  const at::Device dev = idx_in.device();
  at::Tensor idx = idx_in.to(at::kLong).contiguous();
  at::Tensor c = at::zeros({std::max<int64_t>(K, 0)}, opt(dev, at::kLong));
  if (idx.numel() == 0 || K <= 0) return c;
  if (dev.is_cuda()) {
    k::histogram(P0<int64_t>(idx), idx.numel(), K, P0<int64_t>(c), cur_stream());
    return c;
  }
  const int64_t* p = P0<int64_t>(idx);
  int64_t* o = P0<int64_t>(c);
  for (int64_t i = 0; i < idx.numel(); ++i)
    if (p[i] >= 0 && p[i] < K) o[p[i]]++;
  return c;
}

at::Tensor mask_indices(const at::Tensor& mask_in) {
  const at::Device dev = mask_in.device();
  at::Tensor m = mask_in.to(at::kBool).contiguous().view(at::kByte);
  const int64_t n = m.numel();
  if (!dev.is_cuda()) return at::nonzero(m).view({-1});
  if (n == 0) return at::empty({0}, opt(dev, at::kLong));
  at::Tensor f = at::empty({n}, opt(dev, at::kLong));
  k::mask_flags(P0<uint8_t>(m), n, P0<int64_t>(f), cur_stream());
  at::Tensor pos = exclusive_scan(f);
  const int64_t cnt = pos[n].item<int64_t>();
  at::Tensor out = at::empty({cnt}, opt(dev, at::kLong));
  if (cnt) k::compact_mask(P0<uint8_t>(m), P0<int64_t>(pos), n, P0<int64_t>(out), cur_stream());
  return out;
}

at::Tensor repeat_index(const at::Tensor& counts) {
  at::Tensor off = exclusive_scan(counts.to(at::kLong));
  const int64_t n = counts.numel();
  const int64_t tot = n ? off[n].item<int64_t>() : 0;
  return segment_ids(off, n, tot);
}

KV expand(const KMV& kmv) {
  at::Tensor sid = segment_ids(kmv.seg, kmv.nkey, kmv.nval);
  KV out;
  out.n = kmv.nval;
  out.kw = kmv.keys.kw;
  out.kdata = gather_rows(kmv.keys.kdata, kmv.keys.koff, kmv.keys.kw, sid, &out.koff);
  out.vw = kmv.vw;
  out.vdata = kmv.vdata;
  out.voff = kmv.voff;
  return out;
}

KMV sort_multivalues(const KMV& kmv, int flag) {
  if (kmv.nval <= 1) return kmv;
  const at::Device dev = kmv.seg.device();
  at::Tensor perm1 = sort_perm_column(kmv.vdata, kmv.voff, kmv.vw, kmv.nval, flag);
  // stable re-sort of perm1 by segment id (LSD: segment major, value minor)
  at::Tensor sid = segment_ids(kmv.seg, kmv.nkey, kmv.nval);
  at::Tensor sid_p = sid.index_select(0, perm1.to(at::kLong));
  auto [ks, perm2, passes] = radix_sort_pairs(sid_p, iota_u32(kmv.nval, dev), 0, 64);
  at::Tensor perm = perm1.to(at::kLong).index_select(0, perm2.to(at::kLong));
  KMV out = kmv;
  out.vdata = gather_rows(kmv.vdata, kmv.voff, kmv.vw, perm, &out.voff);
  return out;
}

// ====================================================================== text & graph maps

KV map_urls(const at::Tensor& text, int64_t n, int32_t doc_id) {
  const at::Device dev = text.device();
  if (text.numel() < n + 32) fail("map_urls: text buffer must be padded by >= 32 bytes");
  KV kv;
  kv.kw = -1;
  kv.vw = 4;
  if (dev.is_cuda()) {
    auto s = cur_stream();
    int64_t nt = k::url_num_tiles(n);
    at::Tensor cnt = at::empty({std::max<int64_t>(nt, 1)}, opt(dev, at::kInt));
    k::url_count(P0<uint8_t>(text), n, P0<uint32_t>(cnt), s);
    at::Tensor toff = scan_u32(cnt.narrow(0, 0, nt));
    int64_t nurl = (int64_t)(uint32_t)toff[nt].item<int32_t>();
    at::Tensor starts = at::empty({std::max<int64_t>(nurl, 1)}, opt(dev, at::kLong));
    k::url_emit_starts(P0<uint8_t>(text), n, P0<uint32_t>(toff), P0<int64_t>(starts), s);
    at::Tensor klen = at::empty({std::max<int64_t>(nurl, 1)}, opt(dev, at::kInt));
    k::url_lengths(P0<uint8_t>(text), n, P0<int64_t>(starts), nurl, P0<int32_t>(klen), s);
    kv.koff = exclusive_scan(klen.narrow(0, 0, nurl));
    int64_t kb = scalar_i64(kv.koff, nurl);
    kv.kdata = at::empty({kb}, opt(dev, at::kByte));
    k::url_copy(P0<uint8_t>(text), P0<int64_t>(starts), P0<int64_t>(kv.koff), nurl, P0<uint8_t>(kv.kdata), s);
    at::Tensor v = at::empty({nurl}, opt(dev, at::kInt));
    k::fill_i32(P0<int32_t>(v), nurl, doc_id, s);
    kv.vdata = v.view(at::kByte);
    kv.n = nurl;
    return kv;
  }
  const uint8_t* t = P0<uint8_t>(text);
  static const char pat[] = "<a href=\"";
  std::vector<int64_t> koff{0};
  std::vector<uint8_t> kd;
  for (int64_t i = 0; i + 8 < n; ++i) {
    if (memcmp(t + i, pat, 9) != 0) continue;
    int64_t a = i + 9, j = a;
    while (j < n && t[j] != '"') ++j;
    kd.insert(kd.end(), t + a, t + j);
    kd.push_back(0);
    koff.push_back((int64_t)kd.size());
  }
  kv.n = (int64_t)koff.size() - 1;
  kv.koff = at::from_blob(koff.data(), {(int64_t)koff.size()}, opt(at::kCPU, at::kLong)).clone();
  kv.kdata = at::from_blob(kd.data(), {(int64_t)kd.size()}, opt(at::kCPU, at::kByte)).clone();
  kv.vdata = at::full({kv.n}, doc_id, opt(at::kCPU, at::kInt)).view(at::kByte);
  return kv;
}

static inline bool is_ws(uint8_t c) { return c == ' ' || c == '\t' || c == '\n' || c == '\f' || c == '\r' || c == 0; }

KV map_words(const at::Tensor& text, int64_t n) {
  const at::Device dev = text.device();
  if (text.numel() < n + 32) fail("map_words: text buffer must be padded by >= 32 bytes");
  KV kv;
  kv.kw = -1;
  kv.vw = 0;
  kv.vdata = at::empty({0}, opt(dev, at::kByte));
  if (dev.is_cuda()) {
    // per-tile words and key bytes, their scans, one host read of both
    // totals, then keys and offsets in one pass (text.hip k_tok_emit2)
    auto s = cur_stream();
    const int64_t nt = k::tok_num_tiles(n);
    if (nt <= 0) {
      kv.n = 0;
      kv.koff = at::zeros({1}, opt(dev, at::kLong));
      kv.kdata = at::empty({0}, opt(dev, at::kByte));
      return kv;
    }
    at::Tensor cw = at::empty({nt}, opt(dev, at::kInt)), cb = at::empty({nt}, opt(dev, at::kInt));
    k::tok_count2(P0<uint8_t>(text), n, P0<uint32_t>(cw), P0<uint32_t>(cb), s);
    at::Tensor tw = scan_u32(cw);        // u32 [nt + 1]
    at::Tensor tb = exclusive_scan(cb);  // i64 [nt + 1]
    uint32_t nw32 = 0;
    int64_t kb = 0;
    read_small(s, {{P0<uint32_t>(tw) + nt, &nw32, 4}, {P0<int64_t>(tb) + nt, &kb, 8}});
    const int64_t nw = (int64_t)nw32;
    kv.koff = at::empty({nw + 1}, opt(dev, at::kLong));
    kv.kdata = at::empty({kb}, opt(dev, at::kByte));
    k::tok_emit2(P0<uint8_t>(text), n, P0<uint32_t>(tw), P0<int64_t>(tb), P0<int64_t>(kv.koff), P0<uint8_t>(kv.kdata),
                 s);
    k::fill_i64(P0<int64_t>(kv.koff) + nw, 1, kb, s);
    kv.n = nw;
    return kv;
  }
  const uint8_t* t = P0<uint8_t>(text);
  std::vector<int64_t> koff{0};
  std::vector<uint8_t> kd;
  for (int64_t i = 0; i < n;) {
    while (i < n && is_ws(t[i])) ++i;
    if (i >= n) break;
    int64_t j = i;
    while (j < n && !is_ws(t[j])) ++j;
    kd.insert(kd.end(), t + i, t + j);
    kd.push_back(0);
    koff.push_back((int64_t)kd.size());
    i = j;
  }
  kv.n = (int64_t)koff.size() - 1;
  kv.koff = at::from_blob(koff.data(), {(int64_t)koff.size()}, opt(at::kCPU, at::kLong)).clone();
  kv.kdata = at::from_blob(kd.data(), {(int64_t)kd.size()}, opt(at::kCPU, at::kByte)).clone();
  return kv;
}

KV map_rmat(int64_t nedges, int nlevels, double a, double b, double c, double d, double fraction, uint64_t seed,
            uint64_t first_edge, at::Device dev) {
  KV kv;
  kv.kw = 16;
  kv.vw = 0;
  kv.n = nedges;
  kv.vdata = at::empty({0}, opt(dev, at::kByte));
  at::Tensor e = at::empty({2 * nedges}, opt(dev, at::kLong));
  if (dev.is_cuda()) {
    k::rmat_edges(P0<uint64_t>(e), nedges, nlevels, (float)a, (float)b, (float)c, (float)d, (float)fraction, seed,
                  first_edge, cur_stream());
  } else {
    uint64_t* ep = P0<uint64_t>(e);
    for (int64_t i = 0; i < nedges; ++i)
      dev::rmat_edge(first_edge + (uint64_t)i, nlevels, (float)a, (float)b, (float)c, (float)d, (float)fraction, seed,
                     &ep[2 * i], &ep[2 * i + 1]);
  }
  kv.kdata = e.view(at::kByte);
  return kv;
}

}  // namespace mrh
