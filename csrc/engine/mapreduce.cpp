// Native MapReduce object (see mapreduce.h). Reference behaviour cited per
// method as src/mapreduce.cpp:<lines>.
#include "devfn.h"
#include "hostarena.h"
#include "xfer.h"
#include "mapreduce.h"
#include "guard.h"
#include "hbmpool.h"
#include "grouper.h"
#include "guardalloc.h"
#include "ooc.h"

#include <c10/hip/HIPCachingAllocator.h>
#include <hip/hip_runtime.h>
#include <rocprofiler-sdk-roctx/roctx.h>

#include <algorithm>
#include <cinttypes>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <filesystem>
#include <fstream>
#include <numeric>
#include <optional>
#include <sstream>
#include <stdexcept>

namespace mrh {

std::atomic<int> MapReduce::instances_now{0}, MapReduce::instances_ever{0};
std::atomic<int64_t> MapReduce::msize{0}, MapReduce::msizemax{0}, MapReduce::rsize{0}, MapReduce::wsize{0},
    MapReduce::cssize{0}, MapReduce::crsize{0};
double MapReduce::commtime = 0.0;

std::function<void(const std::string&)>& screen_sink() {
  static std::function<void(const std::string&)> f = [](const std::string& s) {
    std::fwrite(s.data(), 1, s.size(), stdout);
    std::fflush(stdout);
  };
  return f;
}

namespace {

// roctx range per MapReduce op: `rocprofv3 --marker-trace` shows every op
// (map, aggregate, convert, reduce, ...) around its kernels and RCCL calls
// On scope exit (after the op's return value is computed) an MR with
// outofcore == 1 writes its data to disk — the reference's forced
// out-of-core mode (src/keyvalue.cpp:122,223); the next op reads it back.
//
// With MRH_TRACE set, every op also appends a JSON line (guard.h trace_op):
// wall time with the device synchronised at both ends, local pair counts and
// bytes, and the bytes this rank sent/received in shuffles during the op.
thread_local int g_op_depth = 0;
void device_sync(const MapReduce* mr) {
  if (mr->device().is_cuda()) guard::hip_check(hipDeviceSynchronize(), "trace_sync", mr->comm()->rank());
}
struct OpTrace {
  OpTrace(const char* name, MapReduce* mr) : mr_(mr), name_(name) {
    roctxRangePushA(name);
    if (g_op_depth == 0) guard::set_current_op(name);
    // page pool installed + a page budget B: the op may hold at most 2B of
    // new device memory (output + working set) plus 16 MiB of kernel scratch
    // (sort histograms, scan partials, size-class rounding); past it an
    // allocation fails with "Cannot allocate page" (reference mem_request at
    // maxpage)
    if (g_op_depth == 0 && hbm::installed() && mr->device().is_cuda() && mr->budget() > 0)
      cap_.emplace(mr->device().index() < 0 ? 0 : mr->device().index(), 2 * mr->budget() + (int64_t(16) << 20));
    if (guard::trace_enabled()) {
      device_sync(mr);
      t0_ = Comm::wtime();
      s0_ = MapReduce::cssize.load();
      r0_ = MapReduce::crsize.load();
    }
    ++g_op_depth;
  }
  ~OpTrace() {
    --g_op_depth;
    if (std::uncaught_exceptions() > 0 && g_op_depth == 0 && mr_->comm()->size() > 1) {
      // an op failing on one rank can never complete its collectives on the
      // others: fail the whole job now (reference Error::one -> MPI_Abort,
      // src/error.cpp:47-57) instead of leaving peers blocked in a shuffle
      mr_->comm()->poison(std::string("MapReduce ") + name_ + " raised an error on rank " +
                          std::to_string(mr_->my_proc()));
    }
    if (guard::trace_enabled() && std::uncaught_exceptions() == 0) {
      device_sync(mr_);
      const double t1 = Comm::wtime();
      int64_t b = 0;
      if (mr_->kv) b += mr_->kv->nbytes();
      for (const KMV& m : mr_->kmv_parts()) b += m.nbytes();
      guard::trace_op(mr_->my_proc(), name_, mr_->instance(), g_op_depth, t0_, (t1 - t0_) * 1e3,
                      mr_->kv ? mr_->kv->n : 0, mr_->kmv_keys(), b, MapReduce::cssize.load() - s0_,
                      MapReduce::crsize.load() - r0_);
    }
    // freepage (reference: pages freed after every op, src/mapreduce.cpp:
    // 3483-3517): with an HBM budget in force, blocks the op freed go back to
    // the driver too, so the footprint between ops stays within the budget
    if (mr_->set.freepage && mr_->budget() > 0 && g_op_depth == 0 && mr_->device().is_cuda() &&
        std::uncaught_exceptions() == 0)
      c10::hip::HIPCachingAllocator::emptyCache();
    // MRH_GUARD: every live block's canaries at the end of each top-level op
    if (g_op_depth == 0 && guard::alloc_guard_active()) {
      guard::check_all_blocks(name_);
      guard::set_current_op(nullptr);
    }
    if (mr_->set.outofcore == 1 && std::uncaught_exceptions() == 0) {
      try {
        mr_->spill_disk();
      } catch (const std::exception& e) {
        std::fprintf(stderr, "mrhip: out-of-core write failed: %s\n", e.what());
      }
    }
    roctxRangePop();
  }
  MapReduce* mr_;
  const char* name_;
  double t0_ = 0;
  int64_t s0_ = 0, r0_ = 0;
  std::optional<hbm::OpCap> cap_;
};

[[noreturn]] void fail(const std::string& m) { throw std::runtime_error(m); }

void out(const std::string& s) { screen_sink()(s); }

std::string fmt(const char* f, ...) __attribute__((format(printf, 1, 2)));
std::string fmt(const char* f, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, f);
  vsnprintf(buf, sizeof(buf), f, ap);
  va_end(ap);
  return buf;
}

// one column (keys or values) staged to host memory
struct HostCol {
  at::Tensor data, off;
  int w = 0;
  int64_t base = 0;             // byte shift that makes data + base aligned (aligned layouts)
  std::vector<int64_t> pstart;  // padded row starts (keyalign / valuealign layouts), else empty
  char* d() const { return data.numel() ? (char*)data.data_ptr<uint8_t>() + base : nullptr; }
  int64_t a(int64_t i) const {
    if (!pstart.empty()) return pstart[i];
    return w >= 0 ? i * w : off.data_ptr<int64_t>()[i];
  }
  int64_t len(int64_t i) const { return w >= 0 ? w : off.data_ptr<int64_t>()[i + 1] - off.data_ptr<int64_t>()[i]; }
  char* at(int64_t i) const { return d() ? d() + a(i) : nullptr; }
};
HostCol host_col(const at::Tensor& data, const at::Tensor& off, int w) {
  HostCol c;
  c.data = data.defined() ? data.to(at::kCPU).contiguous() : at::empty({0}, at::TensorOptions().dtype(at::kByte));
  c.off = (w < 0) ? off.to(at::kCPU).contiguous() : at::Tensor();
  c.w = w;
  return c;
}

// keyalign / valuealign (reference src/keyvalue.cpp:345-352, page layout
// `kb | vb | pad | key | pad | value`): the pointer a host callback receives
// for each key (or KV value) is a multiple of `align`; for KMV multivalues
// (seg given) the start of each key's value list is aligned and its values
// stay packed back to back, as in the reference KMV page (src/keymultivalue.
// cpp:830-839). Alignments must be powers of two (src/mapreduce.cpp:3327-3332).
void align_col(HostCol& c, int64_t n, int align, const int64_t* seg = nullptr, int64_t nseg = 0, bool zero = false) {
  if (align < 1 || (align & (align - 1))) throw std::runtime_error("Invalid alignment (keyalign/valuealign must be a power of 2)");
  if (align == 1 || n == 0) return;
  auto up = [&](int64_t x) { return (x + align - 1) & ~(int64_t)(align - 1); };
  std::vector<int64_t> st((size_t)n);
  int64_t pos = 0;
  bool same = ((uintptr_t)c.d() % align) == 0;
  auto place = [&](int64_t i, bool aligned_start) {
    if (aligned_start) pos = up(pos);
    st[i] = pos;
    same = same && pos == c.a(i);
    pos += c.len(i);
  };
  if (seg) {
    for (int64_t s = 0; s < nseg; ++s)
      for (int64_t i = seg[s]; i < seg[s + 1]; ++i) place(i, i == seg[s]);
  } else {
    for (int64_t i = 0; i < n; ++i) place(i, true);
  }
  if (same) return;  // already aligned in place (e.g. fixed widths that are multiples of align)
  // zeropage (reference: pages zeroed when allocated): padding bytes are 0
  at::Tensor buf = zero ? at::zeros({pos + align}, at::TensorOptions().dtype(at::kByte))
                        : at::empty({pos + align}, at::TensorOptions().dtype(at::kByte));
  const int64_t shift = (align - (int64_t)((uintptr_t)buf.data_ptr<uint8_t>() % align)) % align;
  char* dst = (char*)buf.data_ptr<uint8_t>() + shift;
  for (int64_t i = 0; i < n; ++i)
    if (c.len(i)) std::memcpy(dst + st[i], c.at(i), (size_t)c.len(i));
  c.data = buf;
  c.base = shift;
  c.pstart = std::move(st);
}

KV clone_kv(const KV& kv) {
  KV o = kv;
  o.kdata = kv.kdata.clone();
  o.vdata = kv.vdata.clone();
  if (kv.koff.defined()) o.koff = kv.koff.clone();
  if (kv.voff.defined()) o.voff = kv.voff.clone();
  return o;
}
KMV clone_kmv(const KMV& m) {
  KMV o = m;
  o.keys = clone_kv(m.keys);
  o.vdata = m.vdata.clone();
  if (m.voff.defined()) o.voff = m.voff.clone();
  o.seg = m.seg.clone();
  return o;
}
at::Tensor to_host(const at::Tensor& t, bool pin) {
  if (!t.defined()) return t;
  note_xfer(t, at::Device(at::kCPU));
  if (pin && t.is_cuda()) {  // one copy, straight into pinned memory (not pageable, then pinned)
    at::Tensor h = hostarena::pinned_empty(t.sizes(), t.scalar_type());
    h.copy_(t);
    return h;
  }
  return t.to(at::kCPU);
}
KV kv_host(const KV& kv, bool pin) {
  KV o = kv;
  o.kdata = to_host(kv.kdata, pin);
  o.vdata = to_host(kv.vdata, pin);
  o.koff = to_host(kv.koff, pin);
  o.voff = to_host(kv.voff, pin);
  return o;
}
KMV kmv_to(const KMV& m, at::Device d, bool pin) {
  KMV o = m;
  if (d.is_cpu()) {
    o.keys = kv_host(m.keys, pin);
    o.vdata = to_host(m.vdata, pin);
    o.voff = to_host(m.voff, pin);
    o.seg = to_host(m.seg, pin);
  } else {
    o.keys = kv_to(m.keys, d);
    for (const at::Tensor* t : {&m.vdata, &m.voff, &m.seg}) note_xfer(*t, d);
    o.vdata = m.vdata.to(d);
    if (m.voff.defined()) o.voff = m.voff.to(d);
    o.seg = m.seg.to(d);
  }
  return o;
}

std::string fmt_item(const char* p, int64_t n, int flag) {
  switch (flag) {
    case 0: return "NULL";
    case 1: { int32_t x = 0; std::memcpy(&x, p, std::min<int64_t>(n, 4)); return std::to_string(x); }
    case 2: { uint64_t x = 0; std::memcpy(&x, p, std::min<int64_t>(n, 8)); return std::to_string(x); }
    case 3: { float x = 0; std::memcpy(&x, p, std::min<int64_t>(n, 4)); return fmt("%g", x); }
    case 4: { double x = 0; std::memcpy(&x, p, std::min<int64_t>(n, 8)); return fmt("%g", x); }
    case 5: return std::string(p, strnlen(p, (size_t)n));
    case 6: { int32_t x[2] = {0, 0}; std::memcpy(x, p, std::min<int64_t>(n, 8)); return fmt("%d %d", x[0], x[1]); }
    case 7: { uint64_t x[2] = {0, 0}; std::memcpy(x, p, std::min<int64_t>(n, 16));
              return fmt("%" PRIu64 " %" PRIu64, x[0], x[1]); }
  }
  fail("Invalid print args");
}

void expand_path(const std::string& path, int recurse, std::vector<std::string>& outv) {
  namespace fs = std::filesystem;
  std::error_code ec;
  if (fs::is_regular_file(path, ec)) {
    outv.push_back(path);
  } else if (fs::is_directory(path, ec)) {
    std::vector<std::string> names;
    for (auto& e : fs::directory_iterator(path)) names.push_back(e.path().filename().string());
    std::sort(names.begin(), names.end());
    for (auto& n : names) {
      std::string full = (fs::path(path) / n).string();
      if (fs::is_regular_file(full, ec)) outv.push_back(full);
      else if (recurse && fs::is_directory(full, ec)) expand_path(full, recurse, outv);
    }
  } else {
    fail("Invalid filename " + path);
  }
}

std::string join(const std::vector<std::string>& v) {
  std::string s;
  for (auto& x : v) {
    s += x;
    s.push_back('\n');
  }
  return s;
}
std::vector<std::string> split_lines(const std::string& s) {
  std::vector<std::string> v;
  size_t a = 0;
  while (a < s.size()) {
    size_t b = s.find('\n', a);
    if (b == std::string::npos) b = s.size();
    v.push_back(s.substr(a, b - a));
    a = b + 1;
  }
  return v;
}

struct ChunkTask {
  int ifile, itask, ntask;
  int64_t fsize;
};

}  // namespace

// ====================================================================== lifecycle

MapReduce::MapReduce(CommPtr comm) : comm_(std::move(comm)) {
  if (!comm_) comm_ = std::make_shared<Comm>();
  if (const char* p = std::getenv("MRMPI_FPATH")) set.fpath = p;
  instances_now++;
  instance_me_ = ++instances_ever;
  guard::register_mr(this);
}

MapReduce::~MapReduce() {
  drop_disk();
  guard::unregister_mr(this);
  instances_now--;
}

// every op's entry: fault injection point, and data spilled to host (spill()
// or spill-on-OOM) comes back to HBM before the op touches it
void MapReduce::enter(const char* op, bool ooc_ok, bool parts_ok, bool kmv_parts_ok) {
  guard::fault_point(op, comm_->rank());
  if (!parts_ok) flatten();
  if (!kmv_parts_ok) flatten_kmv();
  if (guard::alloc_guard_active()) {  // an overrun found at the end of an earlier op fails the next one
    static size_t raised = 0;
    const auto reps = guard::guard_reports();
    if (reps.size() > raised) {
      const guard::GuardReport& r = reps[raised];
      raised = reps.size();
      throw std::runtime_error("mrhip guard: out-of-bounds device write into a " + std::to_string(r.size) +
                               "-byte block allocated in " + r.alloc_op + ", detected " + r.found_op);
    }
  }
  if (!started_) {
    started_ = true;
    // minpage (reference allocate(), src/mapreduce.cpp:3318-3357): pages
    // claimed up front; here the caching allocator's pool is grown by
    // minpage x memsize once, so the first ops do not pay for hipMalloc
    if (set.minpage > 0 && device().is_cuda()) {
      at::Tensor t = at::empty({(int64_t)set.minpage * block_bytes()}, at::TensorOptions().device(device()).dtype(at::kByte));
    }
  }
  ensure_resident();
  // a group-by index outlives its KV only until the next op sees the KV changed
  if (grouped_ && (!kv || !grouped_->describes(*kv))) grouped_.reset();
  const bool on_host = (kv && !kv->device().is_cuda()) || (kmv && !kmv->keys.device().is_cuda());
  if (!device().is_cuda() || !on_host) return;
  // an op with an out-of-core path leaves host-resident data larger than the
  // HBM budget where it is and streams it; every other op brings it back
  if (ooc_ok && needs_ooc(data_bytes(), budget(), 2.0)) return;
  unspill();
}

// A map/reduce builder of an MR with an HBM or host budget is bounded: its
// chunks go through a Spool (HBM share of the budget, then pinned host up to
// host_budget, then files under fpath), pieces of memsize bytes at most
void MapReduce::bound(KeyValue& b) {
  if (budget() <= 0 && set.host_budget <= 0) return;
  SpoolConfig c;
  c.budget->hbm = budget() > 0 && device().is_cuda() ? budget() : -1;
  c.budget->host = set.host_budget > 0 ? set.host_budget : -1;
  c.dir = set.fpath;
  c.kind = "kv";
  c.instance = instance_me_;
  c.rank = comm_->rank();
  c.piece_bytes = block_bytes();
  if (budget() > 0) c.piece_bytes = std::min<int64_t>(c.piece_bytes, std::max<int64_t>(budget() / 4, 4096));
  b.set_spool(c);
}

OocEnv MapReduce::ooc_env() const {
  OocEnv e;
  e.hbm = budget();
  e.host = set.host_budget > 0 ? set.host_budget : -1;
  e.dir = set.fpath;
  e.instance = instance_me_;
  e.rank = comm_->rank();
  e.streams = set.streams;
  return e;
}

// concatenation of the KV's parts (one pass over all of them): on the
// device, or — for a bounded MR — where the budgets allow (data past the HBM
// budget is written once, to pinned host memory or one spool file)
KV MapReduce::concat_parts(const std::vector<KV>& parts) {
  if (parts.size() == 1) return parts[0];
  int64_t total = 0;
  bool on_dev = true;
  for (const KV& p : parts) {
    total += p.nbytes();
    on_dev = on_dev && p.device() == device();
  }
  if ((budget() <= 0 && set.host_budget <= 0) || !device().is_cuda() || (on_dev && (budget() <= 0 || total <= budget())))
    return concat(parts, device());
  if (set.host_budget <= 0 || total <= set.host_budget) {
    KV o = concat(parts, at::Device(at::kCPU), /*pin=*/true);  // written once, straight to pinned memory
    spool_stats.host_bytes += total;
    return o;
  }
  spool_stats.files++;
  spool_stats.disk_bytes += total;
  return kv_to_file(parts, spool_path(set.fpath, "kv", instance_me_, comm_->rank()));
}

std::vector<KMV> MapReduce::kmv_parts() const {
  std::vector<KMV> p;
  if (kmv) p.push_back(*kmv);
  for (const KMV& t : kmv_tail_) p.push_back(t);
  return p;
}

int64_t MapReduce::kmv_keys() const {
  int64_t n = kmv ? kmv->nkey : 0;
  for (const KMV& t : kmv_tail_) n += t.nkey;
  return n;
}

void MapReduce::flatten_kmv() {
  if (kmv_tail_.empty()) return;
  std::vector<KMV> parts = kmv_parts();
  kmv_tail_.clear();
  const at::Device d = parts[0].seg.device();
  kmv = kmv_concat(parts, d, d.is_cpu() && device().is_cuda());
}

void MapReduce::set_kmv_parts(std::vector<KMV> parts) {
  kmv_tail_.clear();
  kmv.reset();
  for (size_t i = 0; i < parts.size(); ++i) {
    if (i == 0) kmv = parts[0];
    else if (parts[i].nkey) kmv_tail_.push_back(parts[i]);
  }
}

void MapReduce::drop_kmv() {
  kmv.reset();
  kmv_tail_.clear();
}

std::vector<KV> MapReduce::kv_parts() const {
  std::vector<KV> p;
  if (kv) p.push_back(*kv);
  for (const KV& t : kv_tail_) p.push_back(t);
  return p;
}

int64_t MapReduce::kv_rows() const {
  int64_t n = kv ? kv->n : 0;
  for (const KV& t : kv_tail_) n += t.n;
  return n;
}

void MapReduce::flatten() {
  if (kv_tail_.empty()) return;
  std::vector<KV> parts = kv_parts();
  kv_tail_.clear();
  kv = concat_parts(parts);
  grouped_.reset();
}

void MapReduce::set_kv_parts(std::vector<KV> parts) {
  kv_tail_.clear();
  kv.reset();
  grouped_.reset();
  for (size_t i = 0; i < parts.size(); ++i) {
    if (i == 0) kv = parts[0];
    else if (parts[i].n) kv_tail_.push_back(parts[i]);
  }
}

void MapReduce::append_part(const KV& b) {
  grouped_.reset();
  if (!kv) {
    kv = b;
    return;
  }
  if (b.n == 0) return;
  KV p = b;
  if (budget() > 0 && b.device().is_cuda()) {
    int64_t on_dev = b.nbytes();
    for (const KV& x : kv_parts())
      if (x.device().is_cuda()) on_dev += x.nbytes();
    if (on_dev > budget()) {  // the new part leaves HBM through a bounded builder (its pieces only)
      KeyValue tmp(device());
      bound(tmp);
      tmp.add_kv(b);
      p = tmp.finish();
      note_spool(tmp);
    }
  }
  kv_tail_.push_back(p);
}

void MapReduce::note_spool(const KeyValue& b) {
  const SpoolStats s = b.spool_stats();
  spool_stats.add(s);
}

int64_t MapReduce::data_bytes() const {
  int64_t b = 0;
  if (kv) b += kv->nbytes();
  for (const KV& t : kv_tail_) b += t.nbytes();
  if (kmv) b += kmv->nbytes();
  for (const KMV& t : kmv_tail_) b += t.nbytes();
  return b;
}

void MapReduce::note_ooc(const char* op, const OocStats& st) {
  pages_ = std::max<int64_t>(pages_, st.parts);
  spool_stats.files += st.files;
  spool_stats.disk_bytes += st.disk_bytes;
  ooc_hot_keys += st.hot_keys;
  ooc_split_keys += st.split_keys;
  if (set.verbosity > 0 && comm_->rank() == 0)
    out(fmt("%s out of core: %" PRId64 " partitions, %" PRId64 " budget-sized chunks through HBM, %" PRId64
            " spool files\n", op, st.parts, st.chunks, st.files));
}

std::unique_ptr<MapReduce> MapReduce::copy() const {
  const_cast<MapReduce*>(this)->ensure_resident();  // a disk-resident MR copies its data, not nothing
  const_cast<MapReduce*>(this)->flatten();
  const_cast<MapReduce*>(this)->flatten_kmv();
  auto mr = std::make_unique<MapReduce>(comm_);
  mr->set = set;
  if (kv) mr->kv = clone_kv(*kv);
  if (kmv) mr->kmv = clone_kmv(*kmv);
  return mr;
}

void MapReduce::need_kv(const char* what) const {
  if (!kv) fail(std::string("Cannot ") + what + " without KeyValue");
}
void MapReduce::need_kmv(const char* what) const {
  if (!kmv) fail(std::string("Cannot ") + what + " without KeyMultiValue");
}

void MapReduce::start() {
  if (set.timer) {
    if (set.timer == 1) comm_->barrier();
    t0_ = Comm::wtime();
  }
  cs0_ = cssize.load();
  cr0_ = crsize.load();
}

void MapReduce::histo(double v, const char* heading) const {
  std::vector<double> vals = comm_->allgather_f64(v);
  double ave = 0, mx = vals[0], mn = vals[0];
  for (double x : vals) {
    ave += x;
    mx = std::max(mx, x);
    mn = std::min(mn, x);
  }
  ave /= vals.size();
  int h[10] = {0};
  const double d = mx - mn;
  for (double x : vals) {
    int m = d == 0.0 ? 0 : (int)((x - mn) / d * 10.0);
    h[std::min(m, 9)]++;
  }
  if (comm_->rank() == 0) {
    std::string s = fmt("%-13s %g ave %g max %g min\n", heading, ave, mx, mn);
    s += fmt("%-13s", "  Histogram:");
    for (int i = 0; i < 10; ++i) s += fmt(" %d", h[i]);
    out(s + "\n");
  }
}

// per-op stats (reference :3112-3179)
void MapReduce::stats(const char* heading, int which) {
  if (guard::check_enabled()) {
    if (kv) guard::check_kv(*kv, heading);
    for (const KMV& m : kmv_parts()) guard::check_kmv(m, heading);
  }
  const int64_t b = data_bytes();
  msize = b;
  if (b > msizemax) msizemax = b;
  if (set.timer) {
    if (set.timer == 1) {
      comm_->barrier();
      if (comm_->rank() == 0) out(fmt("%s time (secs) = %g\n", heading, Comm::wtime() - t0_));
    } else if (set.timer == 2) {
      histo(Comm::wtime() - t0_, (std::string(heading) + " time (secs) =").c_str());
    }
  }
  if (set.verbosity == 0) return;
  if (which == 0) {
    if (comm_->rank() == 0) out(std::string(heading) + " KV = ");
    kv_stats(set.verbosity);
  } else {
    if (comm_->rank() == 0) out(std::string(heading) + " KMV = ");
    kmv_stats(set.verbosity);
  }
  std::vector<int64_t> sr = comm_->allreduce({cssize - cs0_, crsize - cr0_}, Comm::SUM);
  if (sr[0] || sr[1]) {
    const double mb = 1024.0 * 1024.0;
    if (comm_->rank() == 0) out(fmt("%s Comm = %.3g Mb send, %.3g Mb recv\n", heading, sr[0] / mb, sr[1] / mb));
    if (set.verbosity == 2) {
      histo((cssize - cs0_) / mb, "  Send (Mb):");
      histo((crsize - cr0_) / mb, "  Recv (Mb):");
    }
  }
}

void MapReduce::note_shuffle(const ShuffleStats& st) {
  cssize += st.send_bytes;
  crsize += st.recv_bytes;
  commtime += st.seconds;
}

// ====================================================================== add / open / close

uint64_t MapReduce::add(MapReduce& other) {  // :348-374
  // O(appended): other's pairs become parts of this KV where they are (the
  // reference reopens only the last page, src/keyvalue.cpp:185-209); nothing
  // this object holds is copied
  start();
  OpTrace tr_(__func__, this);
  enter(__func__, true, true);
  need_kv("add");
  other.ensure_resident();
  if (!other.kv) fail("MapReduce passed to add() does not have KeyValue pairs");
  for (const KV& p : other.kv_parts()) append_part(p);
  stats("Add", 0);
  return count(kv_rows());
}

void MapReduce::open(int addflag) {  // :1648-1664
  open_ = std::make_unique<KeyValue>(device());
  bound(*open_);
  open_add_ = addflag;
  drop_kmv();
}

KeyValue& MapReduce::kv_open() {
  if (!open_) fail("MapReduce is not open");
  return *open_;
}

uint64_t MapReduce::close() {  // :658-672
  if (!open_) fail("Cannot close MapReduce that is not open");
  KV n = open_->finish();
  std::shared_ptr<GroupIndex> g = open_->take_group();
  open_.reset();
  if (open_add_) ensure_resident();  // appending to data that was spilled to disk
  else drop_disk();                  // replacing it: the spilled copy must never be read back over n
  if (open_add_ && kv) {
    append_part(n);
  } else {
    kv_tail_.clear();
    kv = n;
    grouped_ = g;
  }
  stats("Close", 0);
  return count(kv_rows());
}

// ====================================================================== map

std::vector<int> MapReduce::my_tasks(int nmap) {  // :1102-1225
  const int P = comm_->size(), me = comm_->rank();
  std::vector<int> t;
  if (set.mapstyle == 0 || P == 1) {
    for (int i = (int)((int64_t)me * nmap / P); i < (int)((int64_t)(me + 1) * nmap / P); ++i) t.push_back(i);
  } else if (set.mapstyle == 1) {
    for (int i = me; i < nmap; i += P) t.push_back(i);
  } else {
    // mapstyle 2: the reference dedicates rank 0 as a master handing out task
    // ids over MPI (:1164-1211); here every rank, rank 0 included, pulls the
    // next id from an atomic counter in the rendezvous store.
    static std::atomic<int64_t> ncall{0};
    comm_->barrier();
    const std::string key = "mrh_mapstyle2_" + std::to_string(instance_me_) + "_" + std::to_string(ncall++);
    for (int64_t i = comm_->next_task(key); i < nmap; i = comm_->next_task(key)) t.push_back((int)i);
    comm_->barrier();
  }
  return t;
}

uint64_t MapReduce::finish_map(KeyValue& kvb, int addflag, const char* heading) {
  // the builder's chunks / spool pieces become the KV's parts (no concatenation)
  std::vector<KV> n = kvb.finish_parts();
  note_spool(kvb);
  std::shared_ptr<GroupIndex> g = kvb.take_group();
  if (addflag && kv) {
    for (const KV& p : n) append_part(p);
  } else {
    set_kv_parts(std::move(n));
    grouped_ = g;
  }
  drop_kmv();
  stats(heading, 0);
  return count(kv_rows());
}

uint64_t MapReduce::map(int nmap, const MapTaskFn& fn, int addflag) {  // :1044-1051
  start();
  OpTrace tr_(__func__, this);
  drop_for_map(addflag);
  enter(__func__);
  KeyValue kvb(device());
  bound(kvb);
  for (int t : my_tasks(nmap)) fn(t, kvb);
  return finish_map(kvb, addflag);
}

std::vector<std::string> MapReduce::find_files(const Comm& comm, const std::vector<std::string>& files,
                                               int selfflag, int recurse, int readflag) {  // :2812-2931
  auto local = [&]() {
    std::vector<std::string> v;
    for (auto& f : files) {
      if (readflag) {
        std::ifstream in(f);
        if (!in) fail("Could not open file " + f);
        std::string line;
        while (std::getline(in, line)) {
          std::istringstream ss(line);
          std::string w;
          if (ss >> w) expand_path(w, recurse, v);
        }
      } else {
        expand_path(f, recurse, v);
      }
    }
    return v;
  };
  if (selfflag) return local();
  std::string s = comm.rank() == 0 ? join(local()) : std::string();
  return split_lines(comm.bcast(s, 0));
}

uint64_t MapReduce::map_file(const std::vector<std::string>& files, int selfflag, int recurse, int readflag,
                             const MapFileFn& fn, int addflag) {  // :1060-1092
  start();
  OpTrace tr_(__func__, this);
  drop_for_map(addflag);
  enter(__func__);
  auto fl = find_files(*comm_, files, selfflag, recurse, readflag);
  mapfilecount = (int)fl.size();
  KeyValue kvb(device());
  bound(kvb);
  if (selfflag) {
    for (int i = 0; i < (int)fl.size(); ++i) fn(i, fl[i].c_str(), kvb);
  } else {
    for (int t : my_tasks((int)fl.size())) fn(t, fl[t].c_str(), kvb);
  }
  return finish_map(kvb, addflag);
}

uint64_t MapReduce::map_file_char(int nmap, const std::vector<std::string>& files, int selfflag, int recurse,
                                  int readflag, char sepchar, int delta, const MapChunkFn& fn, int addflag) {
  return map_chunks(nmap, files, selfflag, recurse, readflag, std::string(1, sepchar), true, delta, fn, addflag);
}

uint64_t MapReduce::map_file_str(int nmap, const std::vector<std::string>& files, int selfflag, int recurse,
                                 int readflag, const std::string& sepstr, int delta, const MapChunkFn& fn,
                                 int addflag) {
  return map_chunks(nmap, files, selfflag, recurse, readflag, sepstr, false, delta, fn, addflag);
}

// split files into ~nmap byte ranges, fix record boundaries with the
// separator and a `delta` look-ahead (reference map_chunks/map_file_wrapper
// :1312-1552)
uint64_t MapReduce::map_chunks(int nmap, const std::vector<std::string>& files, int selfflag, int recurse,
                               int readflag, const std::string& sep, bool is_char, int delta, const MapChunkFn& fn,
                               int addflag) {
  start();
  OpTrace tr_(__func__, this);
  drop_for_map(addflag);
  enter(__func__);
  auto fl = find_files(*comm_, files, selfflag, recurse, readflag);
  mapfilecount = (int)fl.size();
  const int nfile = (int)fl.size();
  std::vector<int64_t> sizes(nfile, 0);
  if (comm_->rank() == 0 || selfflag)
    for (int i = 0; i < nfile; ++i) sizes[i] = (int64_t)std::filesystem::file_size(fl[i]);
  if (!selfflag) sizes = comm_->allreduce(sizes, Comm::SUM);
  std::vector<ChunkTask> plan;
  if (nfile) {
    nmap = std::max(nmap, nfile);
    int64_t total = std::accumulate(sizes.begin(), sizes.end(), (int64_t)0);
    int64_t ideal = std::max<int64_t>(1, total / nmap);
    std::vector<int> tpf(nfile);
    int ntasks = 0;
    for (int i = 0; i < nfile; ++i) ntasks += (tpf[i] = (int)std::max<int64_t>(1, sizes[i] / ideal));
    while (ntasks < nmap) {
      bool prog = false;
      for (int i = 0; i < nfile && ntasks < nmap; ++i)
        if (sizes[i] > ideal) {
          tpf[i]++;
          ntasks++;
          prog = true;
        }
      if (!prog) break;
    }
    while (ntasks > nmap)
      for (int i = 0; i < nfile && ntasks > nmap; ++i)
        if (tpf[i] > 1) {
          tpf[i]--;
          ntasks--;
        }
    for (int i = 0; i < nfile; ++i)
      while (tpf[i] > 1 && sizes[i] / tpf[i] <= delta) tpf[i]--;
    for (int i = 0; i < nfile; ++i)
      for (int j = 0; j < tpf[i]; ++j) plan.push_back({i, j, tpf[i], sizes[i]});
  }
  KeyValue kvb(device());
  bound(kvb);
  std::vector<int> tasks;
  if (selfflag) {
    tasks.resize(plan.size());
    std::iota(tasks.begin(), tasks.end(), 0);
  } else {
    tasks = my_tasks((int)plan.size());
  }
  std::string buf;
  for (int t : tasks) {
    const ChunkTask& c = plan[t];
    const int64_t st = (int64_t)c.itask * c.fsize / c.ntask, nx = (int64_t)(c.itask + 1) * c.fsize / c.ntask;
    const int64_t rs = std::min<int64_t>(nx - st + delta, c.fsize - st);
    buf.assign((size_t)rs + 1, '\0');
    std::FILE* f = std::fopen(fl[c.ifile].c_str(), "rb");
    if (!f) fail("Could not open file " + fl[c.ifile]);
    std::fseek(f, (long)st, SEEK_SET);
    size_t got = std::fread(&buf[0], 1, (size_t)rs, f);
    std::fclose(f);
    rsize += (int64_t)got;
    int64_t s0 = 0, s1 = (int64_t)got;
    if (c.itask > 0) {
      size_t p = buf.find(sep, 0);
      if (p == std::string::npos || (int64_t)p > delta) fail("Could not find file separator within delta");
      s0 = (int64_t)p + (is_char ? (int64_t)sep.size() : 0);
    }
    if (c.itask < c.ntask - 1) {
      size_t p = buf.find(sep, (size_t)(nx - st));
      if (p == std::string::npos || (int64_t)p >= (int64_t)got) fail("Could not find file separator within delta");
      s1 = (int64_t)p + (is_char ? 1 : 0);
    }
    buf[s1] = '\0';  // the reference NUL-terminates the chunk for strtok-style callbacks
    fn(t, &buf[s0], (int)(s1 - s0), kvb);
  }
  return finish_map(kvb, addflag);
}

uint64_t MapReduce::map_mr(MapReduce& src, const MapKVFn& fn, int addflag) {  // :1560-1642
  start();
  OpTrace tr_(__func__, this);
  drop_for_map(addflag, &src);
  enter(__func__);
  src.ensure_resident();
  src.flatten();
  src.flatten_kmv();
  if (!src.kv) fail("MapReduce passed to map() does not have KeyValue pairs");
  KV s = *src.kv;
  HostCol k = host_col(s.kdata, s.koff, s.kw), v = host_col(s.vdata, s.voff, s.vw);
  align_col(k, s.n, src.set.keyalign, nullptr, 0, src.set.zeropage);
  align_col(v, s.n, src.set.valuealign, nullptr, 0, src.set.zeropage);
  KeyValue kvb(device());
  bound(kvb);
  for (int64_t i = 0; i < s.n; ++i) fn((uint64_t)i, k.at(i), (int)k.len(i), v.at(i), (int)v.len(i), kvb);
  if (&src == this && addflag) {
    KV n = kvb.finish();
    note_spool(kvb);
    kv = s;
    append_part(n);
    drop_kmv();
    stats("Map", 0);
    return count(kv_rows());
  }
  return finish_map(kvb, addflag);
}

uint64_t MapReduce::map_mr_batch(MapReduce& src, const MapBatchFn& fn, int addflag) {
  start();
  OpTrace tr_(__func__, this);
  drop_for_map(addflag, &src);
  enter(__func__);
  src.ensure_resident();
  src.flatten();
  src.flatten_kmv();
  if (!src.kv) fail("MapReduce passed to map() does not have KeyValue pairs");
  KV s = *src.kv;
  KeyValue kvb(device());
  bound(kvb);
  fn(s, kvb);
  if (&src == this && addflag) {
    KV n = kvb.finish();
    note_spool(kvb);
    kv = s;
    append_part(n);
    drop_kmv();
    stats("Map", 0);
    return count(kv_rows());
  }
  return finish_map(kvb, addflag);
}

// ====================================================================== shuffle

uint64_t MapReduce::aggregate(const HashFn& hash) {  // :385-563
  start();
  OpTrace tr_(__func__, this);
  enter(__func__, true, !comm_->distributed());  // one rank: nothing moves, appended parts stay
  need_kv("aggregate");
  if (comm_->distributed() && ooc_shuffle()) {
    // larger than the budget: budget-sized chunks in lock-step, received into
    // host memory (ooc.h ooc_exchange); a custom hash runs on the host first
    at::Tensor d;
    if (hash) d = host_dest(hash);
    ShuffleStats st;
    OocStats os;
    kv = ooc_exchange(*kv, d, *comm_, ooc_env(), device(), set.all2all, &os, &st);
    note_shuffle(st);
    note_ooc("Aggregate", os);
  } else if (comm_->distributed()) {
    ShuffleStats st;
    if (!hash) {
      kv = oom_retry(this, device(), my_proc(), "aggregate", [&] { return mrh::aggregate(*kv, *comm_, xopts(), &st); });
    } else {
      kv = exchange(std::move(*kv), host_dest(hash).to(device()), *comm_, xopts(), &st);
    }
    note_shuffle(st);
  }
  stats("Aggregate", 0);
  return count(kv_rows());
}

// owner rank of every pair by a user hash (MR-MPI's hash callback, run on the
// host over the KV's bytes; src/mapreduce.cpp:469-472)
at::Tensor MapReduce::host_dest(const HashFn& hash) const {
  HostCol k = host_col(kv->kdata, kv->koff, kv->kw);
  at::Tensor d = at::empty({kv->n}, at::TensorOptions().dtype(at::kInt));
  int32_t* dp = d.data_ptr<int32_t>();
  const int P = comm_->size();
  for (int64_t i = 0; i < kv->n; ++i) {
    int h = hash(k.at(i), (int)k.len(i));
    dp[i] = (int32_t)(((int64_t)h % P + P) % P);
  }
  return d;
}

// a shuffle of more than half the HBM budget on any rank streams through
// ooc_exchange on every rank (the paths' collectives differ, so the choice is
// collective: one host allreduce, and only for an MR with a budget)
bool MapReduce::ooc_shuffle() const {
  if (budget() <= 0) return false;
  const int64_t mine = kv && needs_ooc(kv->nbytes(), budget(), 2.0) ? 1 : 0;
  return comm_->allreduce(mine, Comm::MAX) != 0;
}

uint64_t MapReduce::aggregate_dest(const at::Tensor& dest) {
  start();
  OpTrace tr_(__func__, this);
  enter(__func__, true, !comm_->distributed());
  need_kv("aggregate");
  if (comm_->distributed()) {
    ShuffleStats st;
    at::Tensor d = dest.to(device()).to(at::kInt).contiguous();
    if (d.numel() != kv->n) fail("aggregate: one destination per pair");
    if (d.numel()) {
      auto mm = at::aminmax(d);
      if (std::get<0>(mm).item<int>() < 0 || std::get<1>(mm).item<int>() >= comm_->size())
        fail("aggregate: destination rank out of range");
    }
    if (ooc_shuffle()) {
      OocStats os;
      kv = ooc_exchange(*kv, d.to(at::kCPU), *comm_, ooc_env(), device(), set.all2all, &os, &st);
      note_ooc("Aggregate", os);
    } else {
      kv = exchange(std::move(*kv), d, *comm_, xopts(), &st);
    }
    note_shuffle(st);
  }
  stats("Aggregate", 0);
  return count(kv_rows());
}

uint64_t MapReduce::broadcast(int root) {  // :569-623
  start();
  OpTrace tr_(__func__, this);
  enter(__func__);
  need_kv("broadcast");
  if (comm_->distributed()) kv = mrh::broadcast(*kv, root, *comm_);
  stats("Broadcast", 0);
  return count(kv->n);
}

uint64_t MapReduce::gather(int nprocs) {  // :893-1036
  start();
  OpTrace tr_(__func__, this);
  enter(__func__, true);
  need_kv("gather");
  if (nprocs < 1 || nprocs > comm_->size()) fail("Invalid proc count for gather");
  if (comm_->distributed() && (nprocs < comm_->size() || comm_->uses_rccl())) {
    ShuffleStats st;
    if (ooc_shuffle()) {  // rank r's pairs to r % nprocs, budget-sized chunks into host memory
      OocStats os;
      at::Tensor d = at::full({kv->n}, comm_->rank() % nprocs, at::TensorOptions().dtype(at::kInt));
      kv = ooc_exchange(*kv, d, *comm_, ooc_env(), device(), set.all2all, &os, &st);
      note_ooc("Gather", os);
    } else {
      kv = gather_to(std::move(*kv), nprocs, *comm_, xopts(), &st);
    }
    note_shuffle(st);
  }
  stats("Gather", 0);
  return count(kv->n);
}

// ====================================================================== group-by

uint64_t MapReduce::convert() { return convert_prehashed(at::Tensor()); }

uint64_t MapReduce::convert_prehashed(const at::Tensor& prehash) {  // :861-886
  start();
  OpTrace tr_("convert", this);
  enter("convert", true, !prehash.defined());
  need_kv("convert");
  last_convert = ConvertStats();
  if (needs_ooc(data_bytes(), budget(), 4.0)) {
    OocStats os;
    // hash-partitioned spools (src/keymultivalue.cpp:645-789), fed from every
    // part where it lies
    set_kmv_parts(ooc_convert_parts(kv_parts(), ooc_env(), device(), &os));
    note_ooc("Convert", os);
  } else if (grouped_ && grouped_->describes(*kv) && !prehash.defined()) {
    // grouped while the map produced it: only the two short sorts are left
    KMV m;
    if (grouped_->finish(&m, &last_convert)) {
      kmv = std::move(m);
      last_convert.grouped = 1;
    } else {
      last_convert = ConvertStats();
      kmv = mrh::convert(*kv, &last_convert, 64);  // a 64-bit hash collision: exact regroup
      last_convert.grouped = 2;
    }
  } else if (!prehash.defined() && (!kv_tail_.empty() || kv->kfixed())) {
    // narrow pairs, possibly in parts: grouped with every part read in place
    // and released once packed (packed pairs), else concatenated once for
    // the other paths
    std::vector<KV> parts = kv_parts();
    bool all_dev = true;
    for (const KV& p : parts) all_dev = all_dev && p.device() == device();
    KMV m;
    bool done = false;
    if (all_dev) {
      // the converter holds the only references: every part is freed once packed
      kv.reset();
      kv_tail_.clear();
      grouped_.reset();
      done = convert_packed_parts(parts, &m, &last_convert);
      if (!done) set_kv_parts(std::move(parts));
    }
    if (done) {
      kmv = std::move(m);
    } else {
      flatten();
      flatten_kmv();
      kmv = oom_retry(this, device(), my_proc(), "convert", [&] { return mrh::convert(*kv, &last_convert, 64); });
    }
  } else {
    kmv = oom_retry(this, device(), my_proc(), "convert",
                    [&] { return mrh::convert(*kv, &last_convert, 64, prehash); });
  }
  grouped_.reset();
  kv.reset();
  kv_tail_.clear();
  stats("Convert", 1);
  return count(kmv_keys());
}

uint64_t MapReduce::collate(const HashFn& hash) {  // :710-738
  start();
  OpTrace tr_(__func__, this);
  // with a budget: aggregate and convert stream out-of-core data themselves;
  // on one rank they also read appended parts in place
  enter(__func__, true, !comm_->distributed());
  need_kv("collate");
  // pipelined collate: the hash-partition exchange hands every received round
  // to a GroupIndex, which groups it on the compute stream while the next
  // round is on the wire (alltoallv k || group k-1); the
  // group-by is done when the last round lands. MRH_PIPELINE_COLLATE=0 turns
  // it off; out-of-core data (an HBM budget in force) keeps aggregate+convert.
  static const bool pipeline_env = [] {
    const char* e = std::getenv("MRH_PIPELINE_COLLATE");
    return !(e && *e == '0');
  }();
  const bool pipeline = set.pipeline < 0 ? pipeline_env : set.pipeline != 0;
  if (pipeline && !hash && comm_->distributed() && budget() == 0) {
    ShuffleStats st;
    GroupIndex g(device());
    ExchangeOpts o = xopts();
    o.round_sink = [&](const KV& r) { g.add(r); };
    KV rest = exchange(std::move(*kv), at::Tensor(), *comm_, o, &st);
    note_shuffle(st);
    last_convert = ConvertStats();
    if (g.size() == 0) {
      kv = rest;
      kmv = mrh::convert(*kv, &last_convert);
    } else {
      kv = g.kv();
      KMV m;
      if (g.finish(&m, &last_convert)) {
        kmv = std::move(m);
        last_convert.grouped = 1;
      } else {
        last_convert = ConvertStats();
        kmv = mrh::convert(*kv, &last_convert, 64);
        last_convert.grouped = 2;
      }
    }
    kv.reset();
    grouped_.reset();
    stats("Collate", 1);
    return count(kmv_keys());
  }
  const int v = set.verbosity, t = set.timer;
  set.verbosity = set.timer = 0;
  aggregate(hash);
  convert();
  set.verbosity = v;
  set.timer = t;
  stats("Collate", 1);
  return count(kmv_keys());
}

// compress's local group-by: out of core (hash-partitioned spools) past the budget
KMV MapReduce::local_groups(const char* heading) {
  last_convert = ConvertStats();
  if (needs_ooc(kv->nbytes(), budget(), 4.0)) {
    OocStats os;
    KMV m = ooc_convert({*kv}, ooc_env(), device(), &os);
    note_ooc(heading, os);
    return m;
  }
  return mrh::convert(*kv, &last_convert);
}

uint64_t MapReduce::clone() {  // :631-652
  start();
  OpTrace tr_(__func__, this);
  enter(__func__, true);  // one value per key: a host-resident KV is cloned where it lives
  need_kv("clone");
  kmv = oom_retry(this, device(), my_proc(), "clone", [&] { return mrh::clone(*kv); });
  kv.reset();
  stats("Clone", 1);
  return count(kmv_keys());
}

uint64_t MapReduce::collapse(const char* key, int kb) {  // :681-702
  start();
  OpTrace tr_(__func__, this);
  enter(__func__);
  need_kv("collapse");
  kmv = mrh::collapse(*kv, std::string(key, (size_t)kb));
  kv.reset();
  stats("Collapse", 1);
  return count(kmv_keys());
}

uint64_t MapReduce::scrunch(int nprocs, const char* key, int kb) {  // :2075-2095
  start();
  OpTrace tr_(__func__, this);
  enter(__func__);
  const int v = set.verbosity, t = set.timer;
  set.verbosity = set.timer = 0;
  gather(nprocs);
  collapse(key, kb);
  set.verbosity = v;
  set.timer = t;
  stats("Scrunch", 1);
  return count(kmv_keys());
}

// ====================================================================== reduce family

ExchangeOpts MapReduce::xopts() const {
  ExchangeOpts o;
  o.chunk_bytes = set.chunk_bytes > 0 ? set.chunk_bytes : 2 * block_bytes();
  o.hbm_budget = budget();
  o.all2all = set.all2all;
  return o;
}

int64_t MapReduce::budget() const {
  if (set.hbm_budget > 0) return set.hbm_budget;
  if (set.maxpage > 0) return (int64_t)set.maxpage * block_bytes();
  return 0;
}

int64_t MapReduce::block_bytes() const {
  // one "page" of values per host block: memsize MB (negative = bytes)
  return set.memsize > 0 ? (int64_t)set.memsize << 20 : std::max<int64_t>(512, -(int64_t)set.memsize);
}

// Drive a host callback over every KMV pair. Keys whose values exceed one page
// use the reference's multi-block protocol (:1828-1848): mv == nullptr,
// nvalues == 0, valuebytes == (int*)this, then multivalue_blocks/_block.
void MapReduce::run_host_kmv(const KMV& m, const std::function<void(char*, int, char*, int, int*)>& fn) {
  HostCol k = host_col(m.keys.kdata, m.keys.koff, m.keys.kw), v = host_col(m.vdata, m.voff, m.vw);
  at::Tensor seg = m.seg.to(at::kCPU).contiguous();
  const int64_t* s = seg.data_ptr<int64_t>();
  align_col(k, m.nkey, set.keyalign, nullptr, 0, set.zeropage);
  align_col(v, m.nval, set.valuealign, s, m.nkey, set.zeropage);
  std::vector<int> vsz((size_t)m.nval);
  for (int64_t j = 0; j < m.nval; ++j) vsz[j] = (int)v.len(j);
  const int64_t page = block_bytes();
  for (int64_t i = 0; i < m.nkey; ++i) {
    const int64_t a = s[i], b = s[i + 1];
    char* mv = v.at(a);
    const int64_t mvbytes = b > a ? v.a(b - 1) + v.len(b - 1) - v.a(a) : 0;
    if (mvbytes <= page || b - a <= 1) {
      fn(k.at(i), (int)k.len(i), mv ? mv : k.at(i), (int)(b - a), vsz.data() + a);
      continue;
    }
    blk_.mv = mv;
    blk_.sizes = vsz.data() + a;
    blk_.nval = b - a;
    blk_.start.clear();
    blk_.boff.clear();
    int64_t acc = 0, off = 0;
    for (int64_t j = 0; j < b - a; ++j) {
      if (j == 0 || acc + vsz[a + j] > page) {
        blk_.start.push_back(j);
        blk_.boff.push_back(off);
        acc = 0;
      }
      acc += vsz[a + j];
      off += vsz[a + j];
    }
    blk_.start.push_back(b - a);
    fn(k.at(i), (int)k.len(i), nullptr, 0, reinterpret_cast<int*>(this));
    blk_ = Blocks();
  }
}

uint64_t MapReduce::multivalue_blocks(int& nblock) const {
  nblock = blk_.start.empty() ? 0 : (int)blk_.start.size() - 1;
  return (uint64_t)blk_.nval;
}

int MapReduce::multivalue_block(int iblock, char** mv, int** valuebytes) {
  if (iblock < 0 || iblock + 1 >= (int)blk_.start.size()) fail("Invalid page request for multivalue_block");
  const int64_t j0 = blk_.start[iblock], j1 = blk_.start[iblock + 1];
  *mv = blk_.mv + blk_.boff[iblock];
  *valuebytes = const_cast<int*>(blk_.sizes + j0);
  return (int)(j1 - j0);
}

uint64_t MapReduce::reduce(const ReduceFn& fn) {  // :1769-1867
  start();
  OpTrace tr_(__func__, this);
  enter(__func__, true, false, true);  // host callbacks read host-resident data (every KMV part) in place
  need_kmv("reduce");
  KeyValue kvb(device());
  bound(kvb);
  for (const KMV& m : kmv_parts())
    run_host_kmv(m, [&](char* k, int kb, char* mv, int nv, int* vb) { fn(k, kb, mv, nv, vb, kvb); });
  set_kv_parts(kvb.finish_parts());
  note_spool(kvb);
  drop_kmv();
  stats("Reduce", 0);
  return count(kv_rows());
}

uint64_t MapReduce::reduce_builtin(const std::string& op, const std::string& dtype) {
  start();
  OpTrace tr_(__func__, this);
  enter(__func__, true, false, kmv_part_count() > 1);
  need_kmv("reduce");
  if (kmv_part_count() > 1 && budget() <= 0) {
    // parts left by an out-of-core convert, but no budget now (it was lowered
    // to 0 = unlimited): each part reduced whole on the engine device (the
    // block path would cut pieces of env.hbm / 4 = 1 byte)
    std::vector<KV> outs;
    for (const KMV& m : kmv_parts()) {
      const KMV dm = m.seg.device() == device() ? m : kmv_to(m, device(), false);
      outs.push_back(oom_retry(this, device(), my_proc(), "reduce_builtin",
                               [&] { return mrh::reduce_builtin(dm, op, dtype.empty() ? "int32" : dtype); }));
    }
    set_kv_parts(std::move(outs));
  } else if (kmv_part_count() > 1 || needs_ooc(kmv->nbytes(), budget(), 2.0)) {
    // values stream through HBM in budget-sized key ranges, part by part
    OocStats os;
    std::vector<KV> outs;
    for (const KMV& m : kmv_parts()) outs.push_back(ooc_reduce_builtin(m, op, dtype.empty() ? "int32" : dtype, ooc_env(), device(), &os));
    set_kv_parts(std::move(outs));
    note_ooc("Reduce", os);
  } else {
    kv = oom_retry(this, device(), my_proc(), "reduce_builtin",
                   [&] { return mrh::reduce_builtin(*kmv, op, dtype.empty() ? "int32" : dtype); });
  }
  drop_kmv();
  stats("Reduce", 0);
  return count(kv_rows());
}

uint64_t MapReduce::reduce_batch(const ReduceBatchFn& fn) {
  start();
  OpTrace tr_(__func__, this);
  enter(__func__, true, false, kmv_part_count() > 1);
  need_kmv("reduce");
  KeyValue kvb(device());
  bound(kvb);
  if (kmv_part_count() > 1 || needs_ooc(kmv->nbytes(), budget(), 2.0)) {
    // key ranges whose values fit the budget go to HBM one at a time, part
    // by part; the batch callback sees each as a KMV of its own (in key order)
    OocStats os;
    for (const KMV& m : kmv_parts())
      ooc_for_each_kmv_piece(m, ooc_env(), device(), [&](const KMV& piece) { fn(piece, kvb); }, &os);
    note_ooc("Reduce", os);
  } else {
    fn(*kmv, kvb);
  }
  set_kv_parts(kvb.finish_parts());
  note_spool(kvb);
  drop_kmv();
  stats("Reduce", 0);
  return count(kv_rows());
}

uint64_t MapReduce::compress(const ReduceFn& fn) {  // :749-851
  start();
  OpTrace tr_(__func__, this);
  enter(__func__, true);  // host callbacks read the (host-resident) groups in place
  need_kv("compress");
  KMV m = local_groups("Compress");
  KeyValue kvb(device());
  bound(kvb);
  run_host_kmv(m, [&](char* k, int kb, char* mv, int nv, int* vb) { fn(k, kb, mv, nv, vb, kvb); });
  set_kv_parts(kvb.finish_parts());
  note_spool(kvb);
  stats("Compress", 0);
  return count(kv_rows());
}

// compress with a batch callback: the local groups of this rank's pairs as one
// KMV (pieces of it when they exceed the budget), fn emits tensors — the
// combiner form of reduce_batch (reference compress, src/mapreduce.cpp:749-851)
uint64_t MapReduce::compress_batch(const ReduceBatchFn& fn) {
  start();
  OpTrace tr_(__func__, this);
  enter(__func__, true);
  need_kv("compress");
  KMV m = local_groups("Compress");
  KeyValue kvb(device());
  bound(kvb);
  if (needs_ooc(m.nbytes(), budget(), 2.0) || (device().is_cuda() && !m.seg.is_cuda())) {
    OocStats os;
    ooc_for_each_kmv_piece(m, ooc_env(), device(), [&](const KMV& piece) { fn(piece, kvb); }, &os);
    note_ooc("Compress", os);
  } else {
    fn(m, kvb);
  }
  set_kv_parts(kvb.finish_parts());
  note_spool(kvb);
  stats("Compress", 0);
  return count(kv_rows());
}

// ====================================================================== device functors

namespace {
// items per functor launch: all of them, unless the builder is bounded (out
// of core): then about a spool piece's worth (the count / scan scratch and the
// output take ~128 bytes per item), so the launch fits the HBM budget
int64_t functor_chunk(const KeyValue& out, int64_t n) {
  const int64_t pb = out.piece_bytes();
  return pb > 0 ? std::max<int64_t>(4096, pb / 128) : std::max<int64_t>(n, 1);
}
}  // namespace

uint64_t MapReduce::map_device(MapReduce& src, const std::string& code, int addflag) {
  const at::Device dev = device();
  return map_mr_batch(
      src,
      [&](const KV& kv, KeyValue& out) {
        if (!kv.n) return;
        const KV d = kv.device() == dev ? kv : kv_to(kv, dev);
        const int64_t step = functor_chunk(out, d.n);
        for (int64_t a = 0; a < d.n; a += step) {
          KV o = devfn::map_pairs(d, code, dev, a, std::min(d.n, a + step));
          if (o.n) out.add_kv(o);
        }
      },
      addflag);
}

uint64_t MapReduce::map_device_tasks(int64_t ntask, const std::string& code, int addflag) {
  // one map task per rank-sized range of the ntask items: task t runs
  // [t * ntask / P, (t + 1) * ntask / P) in one launch (any mapstyle)
  const int64_t P = comm_->size();
  const at::Device dev = device();
  return map(
      (int)P,
      [&](int t, KeyValue& out) {
        const int64_t a = (int64_t)t * ntask / P, b = (int64_t)(t + 1) * ntask / P;
        const int64_t step = functor_chunk(out, b - a);
        for (int64_t x = a; x < b; x += step) {
          KV o = devfn::map_tasks(x, std::min(b, x + step) - x, code, dev);
          if (o.n) out.add_kv(o);
        }
      },
      addflag);
}

uint64_t MapReduce::reduce_device(const std::string& code) {
  const at::Device dev = device();
  return reduce_batch([&](const KMV& m, KeyValue& out) {
    if (!m.nkey) return;
    KV o = devfn::reduce_groups(m, code, dev);
    if (o.n) out.add_kv(o);
  });
}

namespace {
// stable radix sort of the pairs by the functor's 64-bit keys of one column
KV sort_by_functor(const KV& kv_in, const std::string& code, int bits, bool by_value, at::Device dev) {
  if (kv_in.n <= 1) return kv_in;
  const KV kv = kv_in.device() == dev ? kv_in : kv_to(kv_in, dev);
  auto [key, idx] = by_value ? devfn::sort_keys_of(kv.vdata, kv.voff, kv.vw, kv.n, code, dev)
                             : devfn::sort_keys_of(kv.kdata, kv.koff, kv.kw, kv.n, code, dev);
  auto [ks, perm, passes] = radix_sort_pairs(key, idx, 0, std::max(1, std::min(bits, 64)));
  (void)ks;
  (void)passes;
  return gather(kv, perm);
}
}  // namespace

uint64_t MapReduce::sort_keys_device(const std::string& code, int bits) {
  start();
  OpTrace tr_(__func__, this);
  enter(__func__);
  need_kv("sort_keys");
  kv = sort_by_functor(*kv, code, bits, false, device());
  stats("Sort_keys", 0);
  return count(kv->n);
}

uint64_t MapReduce::sort_values_device(const std::string& code, int bits) {
  start();
  OpTrace tr_(__func__, this);
  enter(__func__);
  need_kv("sort_values");
  kv = sort_by_functor(*kv, code, bits, true, device());
  stats("Sort_values", 0);
  return count(kv->n);
}

uint64_t MapReduce::compress_device(const std::string& code) {
  const at::Device dev = device();
  return compress_batch([&](const KMV& m, KeyValue& out) {
    if (!m.nkey) return;
    KV o = devfn::reduce_groups(m, code, dev);
    if (o.n) out.add_kv(o);
  });
}

uint64_t MapReduce::compress_builtin(const std::string& op, const std::string& dtype) {
  start();
  OpTrace tr_(__func__, this);
  enter(__func__, true);
  need_kv("compress");
  KMV m = local_groups("Compress");
  if (needs_ooc(m.nbytes(), budget(), 2.0)) {
    OocStats os;
    kv = ooc_reduce_builtin(m, op, dtype.empty() ? "int32" : dtype, ooc_env(), device(), &os);
    note_ooc("Compress", os);
  } else {
    kv = mrh::reduce_builtin(m, op, dtype.empty() ? "int32" : dtype);
  }
  stats("Compress", 0);
  return count(kv->n);
}

uint64_t MapReduce::scan_kv(const ScanKVFn& fn) {  // :1933-1976
  start();
  OpTrace tr_(__func__, this);
  enter(__func__, true);  // host callbacks read host-resident data in place
  need_kv("scan");
  HostCol k = host_col(kv->kdata, kv->koff, kv->kw), v = host_col(kv->vdata, kv->voff, kv->vw);
  align_col(k, kv->n, set.keyalign, nullptr, 0, set.zeropage);
  align_col(v, kv->n, set.valuealign, nullptr, 0, set.zeropage);
  for (int64_t i = 0; i < kv->n; ++i) fn(k.at(i), (int)k.len(i), v.at(i), (int)v.len(i));
  stats("Scan", 0);
  return count(kv->n);
}

uint64_t MapReduce::scan_kmv(const ScanKMVFn& fn) {  // :1984-2065
  start();
  OpTrace tr_(__func__, this);
  enter(__func__, true, false, true);  // host callbacks read host-resident data (every KMV part) in place
  need_kmv("scan");
  for (const KMV& m : kmv_parts()) run_host_kmv(m, fn);
  stats("Scan", 1);
  return count(kmv_keys());
}

// ====================================================================== sorting

namespace {
// host stable sort of one column with a user comparator -> device int32 perm
at::Tensor host_perm(const at::Tensor& data, const at::Tensor& off, int w, int64_t n, const CompareFn& fn,
                     at::Device dev) {
  HostCol c = host_col(data, off, w);
  std::vector<int32_t> p((size_t)n);
  std::iota(p.begin(), p.end(), 0);
  std::stable_sort(p.begin(), p.end(),
                   [&](int32_t a, int32_t b) { return fn(c.at(a), (int)c.len(a), c.at(b), (int)c.len(b)) < 0; });
  return at::from_blob(p.data(), {n}, at::TensorOptions().dtype(at::kInt)).clone().to(dev);
}
}  // namespace

uint64_t MapReduce::sort_keys(int flag) {  // :2102-2126
  start();
  OpTrace tr_(__func__, this);
  enter(__func__, true);
  need_kv("sort_keys");
  if (needs_ooc(kv->nbytes(), budget(), 4.0)) {
    OocStats os;
    kv = ooc_sort(*kv, flag, false, ooc_env(), device(), &os);  // sample sort over host spools
    note_ooc("Sort_keys", os);
  } else {
    kv = oom_retry(this, device(), my_proc(), "sort_keys", [&] { return sort_kv(*kv, flag, false); });
  }
  stats("Sort_keys", 0);
  return count(kv->n);
}
uint64_t MapReduce::sort_keys(const CompareFn& fn) {  // :2134-2149
  start();
  OpTrace tr_(__func__, this);
  enter(__func__);
  need_kv("sort_keys");
  if (kv->n > 1) kv = mrh::gather(*kv, host_perm(kv->kdata, kv->koff, kv->kw, kv->n, fn, device()));
  stats("Sort_keys", 0);
  return count(kv->n);
}
uint64_t MapReduce::sort_values(int flag) {  // :2156-2180
  start();
  OpTrace tr_(__func__, this);
  enter(__func__, true);
  need_kv("sort_values");
  if (needs_ooc(kv->nbytes(), budget(), 4.0)) {
    OocStats os;
    kv = ooc_sort(*kv, flag, true, ooc_env(), device(), &os);
    note_ooc("Sort_values", os);
  } else {
    kv = oom_retry(this, device(), my_proc(), "sort_values", [&] { return sort_kv(*kv, flag, true); });
  }
  stats("Sort_values", 0);
  return count(kv->n);
}
uint64_t MapReduce::sort_values(const CompareFn& fn) {  // :2188-2203
  start();
  OpTrace tr_(__func__, this);
  enter(__func__);
  need_kv("sort_values");
  if (kv->n > 1) kv = mrh::gather(*kv, host_perm(kv->vdata, kv->voff, kv->vw, kv->n, fn, device()));
  stats("Sort_values", 0);
  return count(kv->n);
}
uint64_t MapReduce::sort_multivalues(int flag) {  // :2210-2352
  start();
  OpTrace tr_(__func__, this);
  enter(__func__);
  need_kmv("sort_multivalues");
  kmv = mrh::sort_multivalues(*kmv, flag);
  stats("Sort_multivalues", 1);
  return count(kmv_keys());
}
uint64_t MapReduce::sort_multivalues(const CompareFn& fn) {
  start();
  OpTrace tr_(__func__, this);
  enter(__func__);
  need_kmv("sort_multivalues");
  KMV& m = *kmv;
  HostCol v = host_col(m.vdata, m.voff, m.vw);
  at::Tensor seg = m.seg.to(at::kCPU).contiguous();
  const int64_t* s = seg.data_ptr<int64_t>();
  std::vector<int32_t> p((size_t)m.nval);
  std::iota(p.begin(), p.end(), 0);
  for (int64_t i = 0; i < m.nkey; ++i)
    std::stable_sort(p.begin() + s[i], p.begin() + s[i + 1], [&](int32_t a, int32_t b) {
      return fn(v.at(a), (int)v.len(a), v.at(b), (int)v.len(b)) < 0;
    });
  at::Tensor perm = at::from_blob(p.data(), {m.nval}, at::TensorOptions().dtype(at::kInt)).clone().to(device());
  at::Tensor noff;
  m.vdata = gather_rows(m.vdata, m.voff, m.vw, perm, m.vw < 0 ? &noff : nullptr);
  if (m.vw < 0) m.voff = noff;
  stats("Sort_multivalues", 1);
  return count(m.nkey);
}

// ====================================================================== print

void MapReduce::print(int proc, int nstride, int kflag, int vflag) { print(nullptr, 0, proc, nstride, kflag, vflag); }

void MapReduce::print(const char* file, int fflag, int proc, int nstride, int kflag, int vflag) {
  ensure_resident();
  flatten();
  flatten_kmv();
  if (!kv && !kmv) fail("Cannot print without KeyValue or KeyMultiValue");
  if (kflag < 0 || kflag > 7 || vflag < 0 || vflag > 7 || nstride < 1) fail("Invalid print args");
  const int me = comm_->rank();
  std::string text;
  int cnt = 0;
  if (kv) {
    HostCol k = host_col(kv->kdata, kv->koff, kv->kw), v = host_col(kv->vdata, kv->voff, kv->vw);
    for (int64_t i = 0; i < kv->n; ++i) {
      if (++cnt != nstride) continue;
      cnt = 0;
      text += fmt("KV pair: proc %d, sizes %d %d, key ", me, (int)k.len(i), (int)v.len(i)) +
              fmt_item(k.at(i), k.len(i), kflag) + ", value " + fmt_item(v.at(i), v.len(i), vflag) + "\n";
    }
  } else {
    HostCol k = host_col(kmv->keys.kdata, kmv->keys.koff, kmv->keys.kw), v = host_col(kmv->vdata, kmv->voff, kmv->vw);
    at::Tensor seg = kmv->seg.to(at::kCPU).contiguous();
    const int64_t* s = seg.data_ptr<int64_t>();
    for (int64_t i = 0; i < kmv->nkey; ++i) {
      if (++cnt != nstride) continue;
      cnt = 0;
      int64_t mvb = 0;
      std::string vs;
      for (int64_t j = s[i]; j < s[i + 1]; ++j) {
        mvb += v.len(j);
        if (vflag) vs += fmt_item(v.at(j), v.len(j), vflag) + " ";
      }
      if (!vflag) vs = "NULL";
      text += fmt("KMV pair: proc %d, nvalues %d, sizes %d %d, key ", me, (int)(s[i + 1] - s[i]), (int)k.len(i),
                  (int)mvb) +
              fmt_item(k.at(i), k.len(i), kflag) + ", values " + vs + "\n";
    }
  }
  auto emit = [&](const char* path, const char* mode) {
    if (!path) {
      out(text);
      return;
    }
    std::FILE* f = std::fopen(path, mode);
    if (!f) fail(std::string("Could not open print file ") + path);
    std::fwrite(text.data(), 1, text.size(), f);
    std::fclose(f);
    wsize += (int64_t)text.size();
  };
  if (proc >= 0) {
    if (proc == me) emit(file, "w");
    return;
  }
  if (file && fflag == 1) {
    std::string p = std::string(file) + "." + std::to_string(me);
    emit(p.c_str(), "w");
    return;
  }
  // token ring: ranks print in order (reference :1696-1709)
  if (file && me == 0) emit(file, "w");
  for (int r = 0; r < comm_->size(); ++r) {
    comm_->barrier();
    if (r == me && !(file && me == 0)) emit(file, "a");
  }
  comm_->barrier();
}

// ====================================================================== stats

uint64_t MapReduce::kv_stats(int level) {  // :2937-2966
  ensure_resident();
  flatten();
  flatten_kmv();
  need_kv("print stats");
  std::vector<int64_t> t =
      comm_->allreduce({kv->n, kv->key_bytes(), kv->value_bytes(), kv->nbytes(), pages(kv->nbytes())}, Comm::SUM);
  const double mb = 1024.0 * 1024.0;
  if (level == 1 && comm_->rank() == 0)
    out(fmt("%" PRId64 " pairs, %.3g Mb keys, %.3g Mb values, %.3g Mb, %" PRId64 " pages\n", t[0], t[1] / mb,
            t[2] / mb, t[3] / mb, t[4]));
  if (level == 2) {
    histo((double)kv->n, "  KV pairs:");
    histo(kv->key_bytes() / mb, "  Kdata (Mb):");
    histo(kv->value_bytes() / mb, "  Vdata (Mb):");
  }
  return (uint64_t)t[0];
}

uint64_t MapReduce::kmv_stats(int level) {  // :2972-3001
  ensure_resident();
  need_kmv("print stats");
  const KMV& m = *kmv;
  const int64_t vb = m.vw >= 0 ? m.nval * m.vw : (m.nval ? m.voff[m.nval].item<int64_t>() : 0);
  std::vector<int64_t> t = comm_->allreduce({m.nkey, m.keys.key_bytes(), vb, m.nbytes(), pages(m.nbytes())}, Comm::SUM);
  const double mb = 1024.0 * 1024.0;
  if (level == 1 && comm_->rank() == 0)
    out(fmt("%" PRId64 " pairs, %.3g Mb keys, %.3g Mb values, %.3g Mb, %" PRId64 " pages\n", t[0], t[1] / mb,
            t[2] / mb, t[3] / mb, t[4]));
  if (level == 2) {
    histo((double)m.nkey, "  KMV pairs:");
    histo(m.keys.key_bytes() / mb, "  Kdata (Mb):");
    histo(vb / mb, "  Vdata (Mb):");
  }
  return (uint64_t)t[0];
}

void MapReduce::cummulative_stats(int level, int reset) {  // :3007-3066
  const double mb = 1024.0 * 1024.0, gb = mb * 1024.0;
  const int me = comm_->rank();
  if (me == 0) out("MapReduce-MPI (gpu_mapreduce_amd native engine)\n");
  int64_t mx = comm_->allreduce(msizemax.load(), Comm::MAX), sm = comm_->allreduce(msizemax.load(), Comm::SUM);
  if (me == 0) out(fmt("Cummulative hi-water mem = %.3g Mb any proc, %.3g Gb all procs\n", mx / mb, sm / gb));
  std::vector<int64_t> c = comm_->allreduce({cssize.load(), crsize.load()}, Comm::SUM);
  double ct = comm_->allreduce_f64(commtime, Comm::SUM);
  if (c[0] || c[1]) {
    if (me == 0)
      out(fmt("Cummulative comm = %.3g Mb send, %.3g Mb recv, %.3g secs\n", c[0] / mb, c[1] / mb,
              ct / comm_->size()));
    if (level == 2) {
      histo(cssize / mb, "  Send (Mb):");
      histo(crsize / mb, "  Recv (Mb):");
    }
  }
  std::vector<int64_t> io = comm_->allreduce({rsize.load(), wsize.load()}, Comm::SUM);
  if ((io[0] || io[1]) && me == 0) out(fmt("Cummulative I/O = %.3g Mb read, %.3g Mb write\n", io[0] / mb, io[1] / mb));
  if (hbm::installed() && device().is_cuda()) {  // the page pool's hi-water mark (reference hiwater())
    const hbm::PoolStats ps = hbm::stats(device().index() < 0 ? 0 : device().index());
    const int64_t hp = comm_->allreduce(ps.peak, Comm::MAX);
    if (me == 0)
      out(fmt("HBM page pool: hi-water %.3g Mb any proc, %.3g Mb in use, %.3g Mb reserved, %lld failed requests\n",
              hp / mb, ps.in_use / mb, ps.reserved / mb, (long long)ps.failures));
  }
  if (reset) rsize = wsize = cssize = crsize = 0;
}

// ====================================================================== spill tier

void MapReduce::spill() {
  flatten();
  flatten_kmv();
  const bool pin = device().is_cuda();
  if (kv) kv = kv_host(*kv, pin);
  if (kmv) kmv = kmv_to(*kmv, at::Device(at::kCPU), pin);
}

void MapReduce::unspill() {
  flatten_kmv();
  if (kv) kv = kv_to(*kv, device());
  if (kmv) kmv = kmv_to(*kmv, device(), false);
}

}  // namespace mrh

// ====================================================================== checkpoint

namespace mrh {

namespace {
constexpr char kMagic[8] = {'M', 'R', 'H', 'K', 'V', '0', '0', '1'};

std::string rank_path(const std::string& p, const Comm& c) {
  return c.size() > 1 ? p + "." + std::to_string(c.rank()) : p;
}
void put_i64(std::FILE* f, int64_t v) {
  if (std::fwrite(&v, 8, 1, f) != 1) throw std::runtime_error("save: write failed");
}
int64_t get_i64(std::FILE* f) {
  int64_t v = 0;
  if (std::fread(&v, 8, 1, f) != 1) throw std::runtime_error("load: truncated file");
  return v;
}
// tensor as (present, dtype, numel, bytes)
void put_t(std::FILE* f, const at::Tensor& t) {
  put_i64(f, t.defined() ? 1 : 0);
  if (!t.defined()) return;
  at::Tensor h = t.to(at::kCPU).contiguous();
  put_i64(f, (int64_t)h.scalar_type());
  put_i64(f, h.numel());
  const size_t nb = (size_t)h.numel() * h.element_size();
  if (nb && std::fwrite(h.data_ptr(), 1, nb, f) != nb) throw std::runtime_error("save: write failed");
}
at::Tensor get_t(std::FILE* f, at::Device dev) {
  const int64_t present = get_i64(f);
  if (present == 0) return at::Tensor();
  if (present != 1) throw std::runtime_error("load: corrupt tensor header");
  const int64_t code = get_i64(f);
  // only the dtypes a KV/KMV column can have (byte arenas, int32/int64 offsets)
  if (code != (int64_t)at::kByte && code != (int64_t)at::kInt && code != (int64_t)at::kLong)
    throw std::runtime_error("load: unexpected tensor dtype code " + std::to_string(code));
  const int64_t n = get_i64(f);
  if (n < 0 || n > (int64_t(1) << 46)) throw std::runtime_error("load: corrupt tensor length");
  at::Tensor h = at::empty({n}, at::TensorOptions().dtype((at::ScalarType)code));
  const size_t nb = (size_t)n * h.element_size();
  if (nb && std::fread(h.data_ptr(), 1, nb, f) != nb) throw std::runtime_error("load: truncated file");
  return h.to(dev);
}
void put_kv(std::FILE* f, const KV& kv) {
  put_i64(f, kv.n);
  put_i64(f, kv.kw);
  put_i64(f, kv.vw);
  put_t(f, kv.kdata);
  put_t(f, kv.koff);
  put_t(f, kv.vdata);
  put_t(f, kv.voff);
}
KV get_kv(std::FILE* f, at::Device dev) {
  KV kv;
  kv.n = get_i64(f);
  const int64_t kw = get_i64(f), vw = get_i64(f);
  if (kv.n < 0 || kw < -1 || vw < -1 || kw > (1 << 30) || vw > (1 << 30))
    throw std::runtime_error("load: corrupt KV header");
  kv.kw = (int)kw;
  kv.vw = (int)vw;
  kv.kdata = get_t(f, dev);
  kv.koff = get_t(f, dev);
  kv.vdata = get_t(f, dev);
  kv.voff = get_t(f, dev);
  return kv;
}
}  // namespace

void MapReduce::save(const std::string& path) const {
  if (disk_path_.empty() && !kv && !kmv) fail("Cannot save without KeyValue or KeyMultiValue");
  const_cast<MapReduce*>(this)->ensure_resident();
  const_cast<MapReduce*>(this)->flatten();
  const_cast<MapReduce*>(this)->flatten_kmv();
  write_file(rank_path(path, *comm_));
}

namespace {
struct FileCloser {
  void operator()(std::FILE* f) const {
    if (f) std::fclose(f);
  }
};
using FilePtr = std::unique_ptr<std::FILE, FileCloser>;
}  // namespace

void MapReduce::write_file(const std::string& p) const {
  FilePtr f(std::fopen(p.c_str(), "wb"));
  if (!f) fail("Could not open checkpoint file " + p);
  try {
    if (std::fwrite(kMagic, 1, 8, f.get()) != 8) throw std::runtime_error("save: write failed");
    if (kv) {
      put_i64(f.get(), 0);
      put_kv(f.get(), *kv);
    } else {
      put_i64(f.get(), 1);
      put_kv(f.get(), kmv->keys);
      put_i64(f.get(), kmv->nkey);
      put_i64(f.get(), kmv->nval);
      put_i64(f.get(), kmv->vw);
      put_t(f.get(), kmv->vdata);
      put_t(f.get(), kmv->voff);
      put_t(f.get(), kmv->seg);
    }
    const long bytes = std::ftell(f.get());
    // a full disk shows up at the final flush: never leave a truncated file that looks valid
    if (std::fclose(f.release()) != 0) throw std::runtime_error("save: close failed (disk full?)");
    wsize += bytes;
  } catch (...) {
    f.reset();
    std::remove(p.c_str());
    throw;
  }
}

uint64_t MapReduce::load(const std::string& path) {
  drop_disk();
  return count(read_file(rank_path(path, *comm_)));
}

int64_t MapReduce::read_file(const std::string& p) {
  FilePtr f(std::fopen(p.c_str(), "rb"));
  if (!f) fail("Could not open checkpoint file " + p);
  char magic[8];
  if (std::fread(magic, 1, 8, f.get()) != 8 || std::memcmp(magic, kMagic, 8) != 0)
    fail("Not a gpu_mapreduce_amd checkpoint: " + p);
  int64_t n = 0;
  const int64_t kind = get_i64(f.get());
  if (kind == 0) {
    KV k = get_kv(f.get(), device());
    guard::check_kv(k, "load");  // offsets/arena sizes consistent before any kernel reads them
    kv = k;
    kv_tail_.clear();
    drop_kmv();
    n = kv->n;
  } else if (kind == 1) {
    KMV m;
    m.keys = get_kv(f.get(), device());
    m.nkey = get_i64(f.get());
    m.nval = get_i64(f.get());
    const int64_t vw = get_i64(f.get());
    if (m.nkey < 0 || m.nval < 0 || vw < -1 || vw > (1 << 30)) throw std::runtime_error("load: corrupt KMV header");
    m.vw = (int)vw;
    m.vdata = get_t(f.get(), device());
    m.voff = get_t(f.get(), device());
    m.seg = get_t(f.get(), device());
    guard::check_kmv(m, "load");
    kmv = m;
    kv.reset();
    kv_tail_.clear();
    n = m.nkey;
  } else {
    fail("load: corrupt checkpoint kind in " + p);
  }
  rsize += std::ftell(f.get());
  return n;
}

// ---------------------------------------------------------------- disk tier
// The third memory tier (HBM -> pinned host -> disk): the data goes to a
// per-rank file named like the reference's out-of-core files
// (fpath/mrmpi.<kv|kmv>.<instance>.<counter>.<rank>, src/mapreduce.cpp:3187-3205)
// and comes back on the MR's next op (ensure_resident, called from enter()).
void MapReduce::spill_disk() {
  flatten();
  flatten_kmv();
  if (!kv && !kmv) return;
  char name[96];
  std::snprintf(name, sizeof(name), "mrmpi.%s.%d.%d.%d", kv ? "kv" : "kmv", instance_me_, ++disk_counter_,
                comm_->rank());
  const std::string p = (std::filesystem::path(set.fpath) / name).string();
  write_file(p);
  kv.reset();
  drop_kmv();
  disk_path_ = p;
}

void MapReduce::ensure_resident() {
  if (disk_path_.empty()) return;
  const std::string p = disk_path_;
  disk_path_.clear();
  read_file(p);
  std::remove(p.c_str());
}

void MapReduce::drop_for_map(int addflag, const MapReduce* src) {
  // the reference deletes kv/kmv at the start of a map too (src/mapreduce.cpp:1044-1051)
  if (addflag || src == this) return;
  drop_disk();
  kv.reset();
  kv_tail_.clear();
  drop_kmv();
  grouped_.reset();
}

void MapReduce::drop_disk() {
  if (disk_path_.empty()) return;
  std::remove(disk_path_.c_str());
  disk_path_.clear();
}

}  // namespace mrh
