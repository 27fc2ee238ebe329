// Spool (spool.h): HBM -> pinned host -> memory-mapped disk file.
#include "hostarena.h"
#include "xfer.h"
#include "spool.h"

#include <ATen/hip/HIPContext.h>
#include <c10/hip/HIPCachingAllocator.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>

#include <cerrno>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <filesystem>
#include <future>
#include <mutex>
#include <stdexcept>
#include <thread>

namespace mrh {

namespace {

at::TensorOptions opt(at::Device d, at::ScalarType t) { return at::TensorOptions().device(d).dtype(t); }
[[noreturn]] void fail(const std::string& m) { throw std::runtime_error("mrhip spool: " + m); }

std::atomic<int64_t> g_files_live{0};
std::atomic<int64_t> g_counter{0};

SpoolStats& totals() {
  static SpoolStats s;
  return s;
}
// totals are also updated by the background file writers: every access
// (reads included) under this lock
std::mutex g_totals_mu;
void totals_piece() {
  std::lock_guard<std::mutex> g(g_totals_mu);
  totals().pieces++;
}

// one memory-mapped spool file; unmapped and deleted with the last view
struct Mapping {
  void* p = nullptr;
  size_t len = 0;
  std::string path;
  int fd = -1;  // open while the file is being written (pwrite, not through the mapping)
  // the data is in the page cache now: map it again in place (same address,
  // so every view stays valid) with MAP_POPULATE — the page tables are
  // filled in one pass here (a background writer's thread, for async
  // pieces) instead of by a fault per 4 KiB page when the piece is read
  void done_writing() {
    if (fd >= 0) {
      void* q = p && len ? ::mmap(p, len, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_FIXED | MAP_POPULATE, fd, 0) : p;
      const int e = errno;
      ::close(fd);
      fd = -1;
      if (q == MAP_FAILED) fail("cannot map " + path + " again: " + std::strerror(e));
    }
    fd = -1;
  }
  ~Mapping() {
    if (fd >= 0) ::close(fd);
    if (p && len) munmap(p, len);
    if (!path.empty()) {
      ::unlink(path.c_str());
      g_files_live--;
    }
  }
};

constexpr size_t kAlign = 4096;
size_t align_up(size_t x) { return (x + kAlign - 1) & ~(kAlign - 1); }

// host int64 view of an offset column (device columns are copied)
at::Tensor host_i64(const at::Tensor& t) { return t.to(at::kCPU).contiguous(); }

// bytes used by a column of a part: fixed width -> n * w; variable -> off[n]
int64_t col_bytes(const at::Tensor& off, int w, int64_t n, at::Tensor* hoff) {
  if (w >= 0) return n * w;
  *hoff = host_i64(off);
  return hoff->data_ptr<int64_t>()[n] - hoff->data_ptr<int64_t>()[0];
}

struct Layout {
  std::vector<size_t> off;  // byte offset of each column in the file
  size_t total = 0;
  size_t add(size_t bytes) {
    off.push_back(total);
    total = align_up(total + std::max<size_t>(bytes, 1));
    return off.back();
  }
};

std::shared_ptr<Mapping> create_mapping(const std::string& path, size_t len) {
  const int fd = ::open(path.c_str(), O_RDWR | O_CREAT | O_TRUNC, 0600);
  if (fd < 0) fail("cannot create " + path + ": " + std::strerror(errno));
  auto m = std::make_shared<Mapping>();
  m->path = path;
  g_files_live++;
  if (::ftruncate(fd, (off_t)len) != 0) {
    const std::string e = std::strerror(errno);
    ::close(fd);
    fail("cannot size " + path + " to " + std::to_string(len) + " bytes: " + e);
  }
  void* p = ::mmap(nullptr, len, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  if (p == MAP_FAILED) {
    ::close(fd);
    fail("cannot map " + path + ": " + std::strerror(errno));
  }
  m->p = p;
  m->len = len;
  m->fd = fd;
  return m;
}

// The data goes in by pwrite, not through the fresh shared mapping: writing
// the mapping takes a page fault per 4 KiB page (a spooled GB is 250 k
// faults); pwrite fills the page cache the mapping then reads. Device data
// passes through a pinned staging buffer.
void pwrite_all(const std::shared_ptr<Mapping>& m, const void* src, size_t bytes, size_t off) {
  const char* p = static_cast<const char*>(src);
  while (bytes > 0) {
    const ssize_t w = ::pwrite(m->fd, p, bytes, (off_t)off);
    if (w < 0) {
      if (errno == EINTR) continue;
      fail("cannot write " + m->path + ": " + std::strerror(errno));
    }
    p += w;
    off += (size_t)w;
    bytes -= (size_t)w;
  }
}
void write_tensor(const std::shared_ptr<Mapping>& m, const at::Tensor& t_in, size_t off) {
  const at::Tensor t = t_in.contiguous();
  const size_t bytes = (size_t)t.numel() * t.element_size();
  if (bytes == 0) return;
  if (t.is_cpu()) {
    pwrite_all(m, t.data_ptr(), bytes, off);
    return;
  }
  note_xfer(t, at::Device(at::kCPU));
  const size_t chunk = size_t(16) << 20;
  at::Tensor stage = at::empty({(int64_t)std::min(chunk, bytes)}, at::TensorOptions().dtype(at::kByte).pinned_memory(true));
  at::Tensor tb = t.view(at::kByte).view({-1});
  for (size_t a = 0; a < bytes; a += chunk) {
    const size_t c = std::min(chunk, bytes - a);
    at::Tensor st = stage.narrow(0, 0, (int64_t)c);
    st.copy_(tb.narrow(0, (int64_t)a, (int64_t)c));
    pwrite_all(m, st.data_ptr(), c, off + a);
  }
}

// a host tensor viewing [off, off + numel * elem) of the mapping
at::Tensor view(const std::shared_ptr<Mapping>& m, size_t off, int64_t numel, at::ScalarType dt) {
  return at::from_blob(static_cast<char*>(m->p) + off, {numel}, [m](void*) {}, opt(at::kCPU, dt));
}

// concatenated byte column: parts' data [first .. first+bytes) packed
void put_bytes(const std::shared_ptr<Mapping>& m, size_t off, const std::vector<at::Tensor>& data,
               const std::vector<int64_t>& first, const std::vector<int64_t>& bytes) {
  size_t at_ = off;
  for (size_t i = 0; i < data.size(); ++i) {
    if (bytes[i] <= 0) continue;
    write_tensor(m, data[i].view(at::kByte).narrow(0, first[i], bytes[i]), at_);
    at_ += (size_t)bytes[i];
  }
}

// concatenated offset column: part i's offsets rebased to the bytes before it
void put_offsets(const std::shared_ptr<Mapping>& m, size_t off, const std::vector<at::Tensor>& hoff,
                 const std::vector<int64_t>& ns) {
  int64_t total = 0;
  for (int64_t x : ns) total += x;
  std::vector<int64_t> d((size_t)total + 1);
  int64_t row = 0, base = 0;
  d[0] = 0;
  for (size_t i = 0; i < hoff.size(); ++i) {
    const int64_t* s = hoff[i].data_ptr<int64_t>();
    for (int64_t j = 1; j <= ns[i]; ++j) d[row + j] = s[j] - s[0] + base;
    row += ns[i];
    base = d[row];
  }
  pwrite_all(m, d.data(), d.size() * 8, off);
}

struct Col {
  bool fixed = true;
  int w = 0;
  std::vector<at::Tensor> data, hoff;
  std::vector<int64_t> first, bytes, ns;
  int64_t total_bytes = 0, n = 0;
};

// one KV column (keys or values) of `parts`
Col gather_col(const std::vector<KV>& parts, bool keys) {
  Col c;
  for (auto& p : parts) {
    const int w = keys ? p.kw : p.vw;
    if (!c.data.empty() && (w < 0 || w != c.w)) c.fixed = false;
    if (c.data.empty()) {
      c.w = w;
      c.fixed = w >= 0;
    }
    c.data.push_back(keys ? p.kdata : p.vdata);
    c.ns.push_back(p.n);
    c.n += p.n;
  }
  for (size_t i = 0; i < parts.size(); ++i) {
    const KV& p = parts[i];
    const int w = keys ? p.kw : p.vw;
    at::Tensor hoff;
    int64_t b;
    if (w >= 0) {
      b = p.n * w;
      if (!c.fixed) {  // mixed widths: synthesise offsets
        hoff = at::arange(0, (p.n + 1) * (int64_t)w, std::max(w, 1), opt(at::kCPU, at::kLong));
        if (w == 0) hoff = at::zeros({p.n + 1}, opt(at::kCPU, at::kLong));
      }
      c.first.push_back(0);
    } else {
      b = col_bytes(keys ? p.koff : p.voff, w, p.n, &hoff);
      c.first.push_back(hoff.data_ptr<int64_t>()[0]);
    }
    c.hoff.push_back(hoff);
    c.bytes.push_back(b);
    c.total_bytes += b;
  }
  return c;
}

void place_col(Layout& L, const Col& c) {
  L.add((size_t)c.total_bytes);
  if (!c.fixed) L.add((size_t)(c.n + 1) * 8);
}

// write the column at layout slots [slot, slot+1] and return (data, off)
std::pair<at::Tensor, at::Tensor> write_col(const std::shared_ptr<Mapping>& m, const Layout& L, size_t& slot,
                                            const Col& c) {
  const size_t doff = L.off[slot++];
  put_bytes(m, doff, c.data, c.first, c.bytes);
  at::Tensor data = view(m, doff, c.total_bytes, at::kByte), off;
  if (!c.fixed) {
    const size_t ooff = L.off[slot++];
    put_offsets(m, ooff, c.hoff, c.ns);
    off = view(m, ooff, c.n + 1, at::kLong);
  }
  return {data, off};
}

KV kv_of(const std::shared_ptr<Mapping>& m, const Layout& L, size_t& slot, const Col& k, const Col& v) {
  KV o;
  o.n = k.n;
  o.kw = k.fixed ? k.w : -1;
  o.vw = v.fixed ? v.w : -1;
  auto [kd, ko] = write_col(m, L, slot, k);
  auto [vd, vo] = write_col(m, L, slot, v);
  o.kdata = kd;
  o.koff = ko;
  o.vdata = vd;
  o.voff = vo;
  return o;
}

}  // namespace

SpoolStats spool_totals() {
  std::lock_guard<std::mutex> g(g_totals_mu);
  return totals();
}
int64_t spool_files_live() { return g_files_live.load(); }

std::string spool_path(const std::string& dir, const std::string& kind, int instance, int rank) {
  char name[128];
  std::snprintf(name, sizeof(name), "mrmpi.%s.%d.%lld.%d", kind.c_str(), instance, (long long)++g_counter, rank);
  return (std::filesystem::path(dir) / name).string();
}

KV kv_to_file(const std::vector<KV>& parts, const std::string& path) {
  if (parts.empty()) fail("kv_to_file: no parts");
  Col k = gather_col(parts, true), v = gather_col(parts, false);
  Layout L;
  place_col(L, k);
  place_col(L, v);
  auto m = create_mapping(path, L.total);
  size_t slot = 0;
  KV o = kv_of(m, L, slot, k, v);
  m->done_writing();
  {
    std::lock_guard<std::mutex> g(g_totals_mu);
    totals().files++;
    totals().disk_bytes += (int64_t)L.total;
  }
  return o;
}

KMV kmv_to_file(const std::vector<KMV>& parts, const std::string& path) {
  if (parts.empty()) fail("kmv_to_file: no parts");
  std::vector<KV> keys, vals;
  for (auto& p : parts) {
    keys.push_back(p.keys);
    KV v;
    v.n = p.nval;
    v.kw = 0;
    v.vw = p.vw;
    v.kdata = at::empty({0}, opt(at::kCPU, at::kByte));
    v.vdata = p.vdata;
    v.voff = p.voff;
    vals.push_back(v);
  }
  Col kk = gather_col(keys, true), kv0 = gather_col(keys, false), vk = gather_col(vals, true),
      vv = gather_col(vals, false);
  int64_t nkey = 0;
  for (auto& p : parts) nkey += p.nkey;
  Layout L;
  place_col(L, kk);
  place_col(L, kv0);
  place_col(L, vk);
  place_col(L, vv);
  L.add((size_t)(nkey + 1) * 8);  // seg
  auto m = create_mapping(path, L.total);
  size_t slot = 0;
  KMV o;
  o.keys = kv_of(m, L, slot, kk, kv0);
  KV vals_kv = kv_of(m, L, slot, vk, vv);
  o.vdata = vals_kv.vdata;
  o.voff = vals_kv.voff;
  o.vw = vals_kv.vw;
  o.nkey = nkey;
  o.nval = vals_kv.n;
  std::vector<int64_t> sg((size_t)nkey + 1);
  int64_t row = 0, base = 0;
  for (auto& p : parts) {
    at::Tensor s = host_i64(p.seg);
    const int64_t* sp = s.data_ptr<int64_t>();
    for (int64_t j = 0; j < p.nkey; ++j) sg[row + j] = sp[j] - sp[0] + base;
    row += p.nkey;
    base += p.nval;
  }
  sg[nkey] = base;
  pwrite_all(m, sg.data(), sg.size() * 8, L.off[slot]);
  m->done_writing();
  o.seg = view(m, L.off[slot], nkey + 1, at::kLong);
  {
    std::lock_guard<std::mutex> g(g_totals_mu);
    totals().files++;
    totals().disk_bytes += (int64_t)L.total;
  }
  return o;
}

// ---------------------------------------------------------------- disk writer
// The disk tier's background writes go through ONE bounded pool per process:
// MRH_SPOOL_WRITERS threads (default 4) and at most MRH_SPOOL_WRITE_INFLIGHT
// bytes (default 1 GiB) of drained-but-unwritten pinned pieces. submit()
// blocks while the bytes in flight would pass the cap (the caller waits for
// the oldest writes), and a job drops its reference to the pinned piece as
// soon as the file is written, so the pinned chunk it views can go back to the
// host allocator before the spool is read. (Before: one std::async thread per
// piece, each holding its pinned piece until the spool was read — every
// spilled byte pinned at once and chunks x partitions threads.)
class DiskWriter {
 public:
  static DiskWriter& get() {
    static DiskWriter* w = new DiskWriter();  // never destroyed: no join at exit
    return *w;
  }
  std::future<KV> submit(KV piece, std::shared_ptr<DrainEvent> ev, std::string path) {
    const int64_t b = std::max<int64_t>(1, piece.nbytes());
    auto job = std::make_unique<Job>();
    job->piece = std::move(piece);
    job->ev = std::move(ev);
    job->path = std::move(path);
    job->bytes = b;
    std::future<KV> f = job->done.get_future();
    std::unique_lock<std::mutex> l(mu_);
    // one piece bigger than the cap still goes, alone
    room_.wait(l, [&] { return inflight_ == 0 || inflight_ + b <= cap_; });
    inflight_ += b;
    peak_ = std::max(peak_, inflight_);
    q_.push_back(std::move(job));
    if ((int)threads_.size() < nthreads_ && (int)q_.size() > idle_) {
      threads_.emplace_back([this] { loop(); });
      threads_.back().detach();
    }
    work_.notify_one();
    return f;
  }
  WriterStats stats() {
    std::lock_guard<std::mutex> l(mu_);
    WriterStats s;
    s.inflight_bytes = inflight_;
    s.peak_inflight_bytes = peak_;
    s.threads = (int)threads_.size();
    s.cap_bytes = cap_;
    s.jobs = jobs_;
    return s;
  }
  void reset_peak() {
    std::lock_guard<std::mutex> l(mu_);
    peak_ = inflight_;
  }

 private:
  struct Job {
    KV piece;
    std::shared_ptr<DrainEvent> ev;
    std::string path;
    int64_t bytes = 0;
    std::promise<KV> done;
  };
  DiskWriter() {
    const char* t = std::getenv("MRH_SPOOL_WRITERS");
    nthreads_ = std::max(1, t && *t ? std::atoi(t) : 4);
    const char* c = std::getenv("MRH_SPOOL_WRITE_INFLIGHT");
    cap_ = c && *c ? std::max<int64_t>(1, std::atoll(c)) : (int64_t(1) << 30);
  }
  void loop() {
    for (;;) {
      std::unique_ptr<Job> j;
      {
        std::unique_lock<std::mutex> l(mu_);
        ++idle_;
        work_.wait(l, [&] { return !q_.empty(); });
        --idle_;
        j = std::move(q_.front());
        q_.pop_front();
      }
      try {
        const hipError_t r = hipEventSynchronize(j->ev->e);
        if (r != hipSuccess) fail(std::string("asynchronous drain failed: ") + hipGetErrorString(r));
        KV out = kv_to_file({j->piece}, j->path);
        j->piece = KV();  // the pinned source goes back now, not when the spool is read
        j->ev.reset();
        j->done.set_value(std::move(out));
      } catch (...) {
        j->piece = KV();
        j->ev.reset();
        j->done.set_exception(std::current_exception());
      }
      {
        std::lock_guard<std::mutex> l(mu_);
        inflight_ -= j->bytes;
        ++jobs_;
      }
      room_.notify_all();
    }
  }
  std::mutex mu_;
  std::condition_variable work_, room_;
  std::deque<std::unique_ptr<Job>> q_;
  std::vector<std::thread> threads_;
  int nthreads_ = 4, idle_ = 0;
  int64_t cap_ = 0, inflight_ = 0, peak_ = 0, jobs_ = 0;
};

WriterStats spool_writer_stats() { return DiskWriter::get().stats(); }
void spool_writer_reset_peak() { DiskWriter::get().reset_peak(); }

Spool::Spool(at::Device dev, SpoolConfig cfg) : dev_(dev), cfg_(std::move(cfg)) {
  if (!cfg_.budget) cfg_.budget = std::make_shared<SpoolBudget>();
}

Spool::~Spool() {
  try {
    clear();
  } catch (...) {
  }
}

void Spool::sync() {
  // background file writes first (their drains are in pending_ too)
  std::exception_ptr err;
  for (auto& [i, f] : writing_) {
    try {
      pieces_[i] = f.get();
    } catch (...) {
      if (!err) err = std::current_exception();
    }
  }
  writing_.clear();
  if (err) std::rethrow_exception(err);
  for (const auto& ev : pending_) {
    const hipError_t r = hipEventSynchronize(ev->e);
    if (r != hipSuccess) {
      pending_.clear();
      fail(std::string("asynchronous drain failed: ") + hipGetErrorString(r));
    }
  }
  pending_.clear();
}

void fence_after_current(hipStream_t copy) {
  hipStream_t cs = at::hip::getCurrentHIPStream().stream();
  hipEvent_t fence;
  if (hipEventCreateWithFlags(&fence, hipEventDisableTiming) != hipSuccess || hipEventRecord(fence, cs) != hipSuccess ||
      hipStreamWaitEvent(copy, fence, 0) != hipSuccess)
    fail("drain fence failed");
  (void)hipEventDestroy(fence);
}

at::Tensor drain_tensor(const at::Tensor& t, hipStream_t copy) {
  if (!t.defined() || t.is_cpu()) return t;
  at::Tensor src = t.contiguous();
  at::Tensor o = hostarena::pinned_empty(src.sizes(), src.scalar_type());
  note_xfer(src, at::Device(at::kCPU));
  const size_t nb = (size_t)src.numel() * src.element_size();
  if (nb && hipMemcpyAsync(o.data_ptr(), src.data_ptr(), nb, hipMemcpyDeviceToHost, copy) != hipSuccess)
    fail("asynchronous drain copy failed");
  c10::hip::HIPCachingAllocator::recordStream(src.storage().data_ptr(),
                                             c10::hip::getStreamFromExternal(copy, src.device().index()));
  return o;
}

std::shared_ptr<DrainEvent> record_event(hipStream_t s) {
  auto ev = std::make_shared<DrainEvent>();
  if (hipEventCreateWithFlags(&ev->e, hipEventDisableTiming) != hipSuccess || hipEventRecord(ev->e, s) != hipSuccess)
    fail("drain event failed");
  return ev;
}

std::shared_ptr<DrainEvent> drain_to_pinned(const KV& dev_kv, hipStream_t copy, KV* host_out) {
  fence_after_current(copy);
  KV o = dev_kv;
  o.kdata = drain_tensor(dev_kv.kdata, copy);
  o.vdata = drain_tensor(dev_kv.vdata, copy);
  o.koff = drain_tensor(dev_kv.koff, copy);
  o.voff = drain_tensor(dev_kv.voff, copy);
  *host_out = o;
  return record_event(copy);
}

void Spool::add_drained(const KV& piece, const std::shared_ptr<DrainEvent>& ev) {
  if (piece.n == 0) return;
  const int64_t b = piece.nbytes();
  SpoolBudget& B = *cfg_.budget;
  if (B.host >= 0) B.host -= b;
  st_.host_bytes += b;
  pieces_.push_back(piece);
  tier_.push_back(1);
  pending_.push_back(ev);
  n_ += piece.n;
  bytes_ += b;
  st_.pieces++;
  totals_piece();
}

void Spool::add_drained_to_disk(const KV& piece, const std::shared_ptr<DrainEvent>& ev) {
  if (piece.n == 0) return;
  const int64_t b = piece.nbytes();
  writing_.emplace_back(pieces_.size(), DiskWriter::get().submit(piece, ev, next_path()));
  pieces_.push_back(KV());  // filled in by sync()
  tier_.push_back(2);
  st_.disk_bytes += b;
  st_.files++;
  n_ += piece.n;
  bytes_ += b;
  st_.pieces++;
  totals_piece();
}

std::string Spool::next_path() const { return spool_path(cfg_.dir, cfg_.kind, cfg_.instance, cfg_.rank); }

void Spool::release(const KV& piece, int tier) {
  const int64_t b = piece.nbytes();
  SpoolBudget& B = *cfg_.budget;
  if (tier == 0 && B.hbm >= 0) B.hbm += b;
  if (tier == 1 && B.host >= 0) B.host += b;
}

void Spool::add(const KV& piece, hipStream_t copy) {
  if (piece.n == 0) return;
  const int64_t b = piece.nbytes();
  SpoolBudget& B = *cfg_.budget;
  KV p;
  int tier;
  const bool cuda = dev_.is_cuda();
  if (cuda && (B.hbm < 0 || B.hbm >= b)) {
    // a device piece is kept as is, unless it is a view into a larger buffer
    // (a slice of a partitioned chunk): then its own copy, so the tier holds
    // the bytes it counts and the chunk buffer can go
    auto own = [](const at::Tensor& t) {
      if (!t.defined() || !t.is_cuda()) return t;
      const int64_t used = t.numel() * t.element_size();
      return (int64_t)t.storage().nbytes() > used + 4096 ? t.clone() : t;
    };
    if (piece.device() == dev_) {
      p = piece;
      p.kdata = own(piece.kdata);
      p.vdata = own(piece.vdata);
      p.koff = own(piece.koff);
      p.voff = own(piece.voff);
    } else {
      p = kv_to(piece, dev_);
    }
    if (B.hbm >= 0) B.hbm -= b;
    tier = 0;
    st_.hbm_bytes += b;
  } else if (B.host < 0 || B.host >= b) {
    // the host tier (pinned when a GPU will read it back); a device piece
    // with a copy stream drains asynchronously behind the current stream
    if (copy && cuda && piece.device().is_cuda()) {
      pending_.push_back(drain_to_pinned(piece, copy, &p));
    } else {
      auto h = [&](const at::Tensor& t) {
        if (!t.defined()) return t;
        if (t.is_cpu() && (!cuda || t.is_pinned())) return t;
        at::Tensor o = cuda ? hostarena::pinned_empty(t.sizes(), t.scalar_type())
                            : at::empty(t.sizes(), t.options().device(at::kCPU));
        note_xfer(t, at::Device(at::kCPU));
        o.copy_(t);
        return o;
      };
      p = piece;
      p.kdata = h(piece.kdata);
      p.vdata = h(piece.vdata);
      p.koff = h(piece.koff);
      p.voff = h(piece.voff);
    }
    if (B.host >= 0) B.host -= b;
    tier = 1;
    st_.host_bytes += b;
  } else if (copy && cuda && piece.device().is_cuda()) {
    // the disk tier off the caller's path: drain into pinned memory on the
    // copy stream, then a background thread writes and maps the file
    KV hp;
    std::shared_ptr<DrainEvent> done = drain_to_pinned(piece, copy, &hp);
    writing_.emplace_back(pieces_.size(), DiskWriter::get().submit(std::move(hp), std::move(done), next_path()));
    p = KV();  // filled in by sync()
    tier = 2;
    st_.disk_bytes += b;
    st_.files++;
  } else {
    p = kv_to_file({piece}, next_path());
    tier = 2;
    st_.disk_bytes += b;
    st_.files++;
  }
  pieces_.push_back(p);
  tier_.push_back(tier);
  n_ += piece.n;
  bytes_ += b;
  st_.pieces++;
  totals_piece();
}

void Spool::clear() {
  sync();
  for (size_t i = 0; i < pieces_.size(); ++i) release(pieces_[i], tier_[i]);
  pieces_.clear();
  tier_.clear();
  n_ = bytes_ = 0;
}

std::vector<KV> Spool::take() {
  sync();
  std::vector<KV> parts = pieces_;
  clear();
  return parts;
}

KV Spool::gather_host() {
  sync();
  if (pieces_.empty()) {
    clear();
    return empty_kv(at::Device(at::kCPU), 0, 0);
  }
  std::vector<KV> parts = pieces_;
  const int64_t total = bytes_;
  clear();  // budget shares back before deciding where the whole goes
  SpoolBudget& B = *cfg_.budget;
  if (parts.size() == 1 && parts[0].device().is_cpu()) return parts[0];
  if (B.host < 0 || B.host >= total) return concat(parts, at::Device(at::kCPU), /*pin=*/dev_.is_cuda());
  st_.files++;
  st_.disk_bytes += total;
  return kv_to_file(parts, next_path());
}

KV Spool::gather() {
  sync();
  SpoolBudget& B = *cfg_.budget;
  if (dev_.is_cuda()) {
    // what the tiers would hold once this spool's own shares are returned
    int64_t hbm_room = B.hbm;
    if (hbm_room >= 0)
      for (size_t i = 0; i < pieces_.size(); ++i)
        if (tier_[i] == 0) hbm_room += pieces_[i].nbytes();
    if (hbm_room < 0 || hbm_room >= bytes_) {
      std::vector<KV> parts = pieces_;
      clear();
      return concat(parts, dev_);
    }
  } else if (B.host < 0) {
    std::vector<KV> parts = pieces_;
    clear();
    return concat(parts, dev_);
  }
  return gather_host();
}

}  // namespace mrh
