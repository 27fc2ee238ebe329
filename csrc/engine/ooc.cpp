// Out-of-core engine ops: convert, sort and builtin reduce over a KV / KMV
// larger than the MapReduce object's HBM budget (mapreduce.h Settings::
// hbm_budget, or maxpage x memsize).
//
// The reference pages everything through fixed-size pages and disk spools:
// convert partitions the unique-key table by hash bits into Spools when it
// overflows (src/keymultivalue.cpp:645-789, partition2sets :1056-1132), sort
// sorts page-sized runs and 2-way merges them on disk (src/mapreduce.cpp:
// 2395-2445, 2547-2633). Here the data sits in pinned host memory (the spill
// tier) and HBM holds one budget-sized piece at a time:
//
//  convert  pass 1: each chunk goes to HBM, a 64-bit key hash picks one of M
//           partitions, the shuffle's partition kernels (bucket_local) cut the
//           chunk into M contiguous buckets, which drain to M host spools;
//           pass 2: each partition (all values of a key live in one) is
//           converted in HBM and its KMV drains to the host. M is chosen so a
//           partition and its working set fit the budget.
//  sort     sample sort instead of a run merge: pass 1 samples the radix sort
//           key (column_sort_keys) of every chunk and picks M-1 splitters;
//           pass 2 range-partitions every chunk into M host spools (equal keys
//           always share a bucket; the partition is stable); pass 3 sorts each
//           bucket in HBM and appends it. Bucket order is key order, so no
//           merge is needed, and stability holds end to end.
//  reduce   builtin segmented reduces stream the KMV in key ranges whose values
//           fit the budget.
// Tiers (spool.h): the partition spools hold their pieces in pinned host
// memory up to the host budget (Settings::host_budget) and in memory-mapped
// files under fpath beyond it; results are pinned while they fit the host
// budget, else one memory-mapped file. The MapReduce object brings a result
// back to HBM on a later op when it fits.
// Streaming: chunk k+1 is copied host -> HBM on a side stream while chunk k
// is partitioned, and chunk k's buckets drain HBM -> host on a copy stream
// (Spool::add with a stream) while chunk k+1 is partitioned.
#include <ATen/ATen.h>
#include <ATen/hip/HIPContext.h>
#include <c10/hip/HIPCachingAllocator.h>
#include <c10/hip/HIPGuard.h>

#include <algorithm>
#include <cstdio>
#include <string>
#include <utility>
#include <cstring>
#include <limits>
#include <stdexcept>
#include <tuple>
#include <unordered_map>

#include "hostarena.h"
#include "../kernels/launch.h"
#include "kv.h"
#include "comm.h"
#include "ooc.h"
#include "spool.h"
#include "xfer.h"

namespace mrh {

namespace {

at::TensorOptions opt(at::Device d, at::ScalarType t) { return at::TensorOptions().device(d).dtype(t); }

// MRH_OOC_TRACE=1: host time per phase of an out-of-core op (device
// synchronised at each mark), summed by name and printed at the end
// MRH_OOC_TRACE=1: device-synchronised phase times (each phase's GPU work
// included); =2: host wall time per phase without synchronising (where the
// host thread spends its time, blocking waits included, GPU left alone)
struct PhaseClock {
  bool on = false, sync = false;
  double t = 0;
  std::vector<std::pair<std::string, double>> acc;
  const char* op;
  explicit PhaseClock(const char* o) : op(o) {
    const char* e = std::getenv("MRH_OOC_TRACE");
    on = e && (*e == '1' || *e == '2');
    sync = on && *e == '1';
    if (on) {
      if (sync) (void)hipDeviceSynchronize();
      t = Comm::wtime();
    }
  }
  void operator()(const char* what) {
    if (!on) return;
    if (sync) (void)hipDeviceSynchronize();
    const double now = Comm::wtime();
    for (auto& [k, v] : acc)
      if (k == what) {
        v += now - t;
        t = now;
        return;
      }
    acc.emplace_back(what, now - t);
    t = now;
  }
  ~PhaseClock() {
    if (!on) return;
    for (auto& [k, v] : acc) std::fprintf(stderr, "mrhip ooc %s %-18s %9.2f ms\n", op, k.c_str(), 1e3 * v);
    UploadTimes& u = upload_times();
    if (u.on) {
      std::fprintf(stderr, "mrhip ooc %s upload totals: alloc %.2f ms, pinned copies %.2f ms (%lld), staged %.2f ms (%lld: "
                   "buffer waits %.2f ms, memcpy %.2f ms)\n",
                   op, 1e3 * u.alloc, 1e3 * u.pinned, (long long)u.pinned_calls, 1e3 * u.staged,
                   (long long)u.staged_calls, 1e3 * u.stage_wait, 1e3 * u.stage_memcpy);
      u = UploadTimes{true};
    }
  }
};

at::Tensor host(const at::Tensor& t) {
  if (!t.defined()) return t;
  if (t.is_cpu()) return t.contiguous();
  note_xfer(t, at::Device(at::kCPU));
  at::Tensor h = hostarena::pinned_empty(t.sizes(), t.scalar_type());
  h.copy_(t);
  return h;
}
KV kv_host(const KV& kv) {
  KV o = kv;
  o.kdata = host(kv.kdata);
  o.vdata = host(kv.vdata);
  o.koff = host(kv.koff);
  o.voff = host(kv.voff);
  return o;
}
KMV kmv_host(const KMV& m) {
  KMV o = m;
  o.keys = kv_host(m.keys);
  o.vdata = host(m.vdata);
  o.voff = host(m.voff);
  o.seg = host(m.seg);
  return o;
}

// pairs [a, b) of a KV as a KV of their own (views of fixed columns; offsets rebased)
KV kv_slice(const KV& kv, int64_t a, int64_t b, const int64_t* hkoff, const int64_t* hvoff) {
  KV o;
  o.n = b - a;
  o.kw = kv.kw;
  o.vw = kv.vw;
  const at::Device dev = kv.device();
  if (kv.kfixed()) {
    o.kdata = kv.kdata.narrow(0, a * kv.kw, (b - a) * kv.kw);
  } else {
    o.kdata = kv.kdata.narrow(0, hkoff[a], hkoff[b] - hkoff[a]);
    o.koff = kv.koff.narrow(0, a, b - a + 1) - hkoff[a];
  }
  if (kv.vfixed()) {
    o.vdata = kv.vdata.narrow(0, a * kv.vw, (b - a) * kv.vw);
  } else {
    o.vdata = kv.vdata.narrow(0, hvoff[a], hvoff[b] - hvoff[a]);
    o.voff = kv.voff.narrow(0, a, b - a + 1) - hvoff[a];
  }
  (void)dev;
  return o;
}

// host copies of the offset columns (for byte-sized chunking and slicing)
struct HostOff {
  at::Tensor k, v;
  const int64_t* kp() const { return k.defined() ? k.data_ptr<int64_t>() : nullptr; }
  const int64_t* vp() const { return v.defined() ? v.data_ptr<int64_t>() : nullptr; }
};
HostOff host_off(const KV& kv) {
  HostOff h;
  if (!kv.kfixed()) h.k = kv.koff.to(at::kCPU).contiguous();
  if (!kv.vfixed()) h.v = kv.voff.to(at::kCPU).contiguous();
  return h;
}

int64_t row_bytes(const KV& kv, const HostOff& h, int64_t a, int64_t b) {
  int64_t x = 0;
  x += kv.kfixed() ? (b - a) * kv.kw : h.kp()[b] - h.kp()[a] + 8 * (b - a);
  x += kv.vfixed() ? (b - a) * kv.vw : h.vp()[b] - h.vp()[a] + 8 * (b - a);
  return x;
}

// largest b in (a, n] with fits(b) (fits is monotone, b = a + 1 always taken)
template <typename F>
int64_t grow(int64_t a, int64_t n, F&& fits) {
  int64_t b = a + 1, step = 1;
  while (b < n) {
    const int64_t nb = std::min(n, b + step);
    if (!fits(nb)) break;
    b = nb;
    step *= 2;
  }
  int64_t lo = b, hi = std::min(n, b + step);
  while (lo < hi) {
    const int64_t mid = (lo + hi + 1) / 2;
    if (fits(mid)) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// pair ranges whose bytes are <= cap (at least one pair each)
std::vector<std::pair<int64_t, int64_t>> chunks(const KV& kv, const HostOff& h, int64_t cap) {
  std::vector<std::pair<int64_t, int64_t>> out;
  for (int64_t a = 0; a < kv.n;) {
    const int64_t b = grow(a, kv.n, [&](int64_t e) { return row_bytes(kv, h, a, e) <= cap; });
    out.push_back({a, b});
    a = b;
  }
  return out;
}

// a KV column set copied to `dev` on stream `side` (non-blocking from pinned
// memory); the tensors are marked for use on `use` so the caching allocator
// does not recycle them while `use` still reads them
KV kv_to_async(const KV& kv, at::Device dev, const c10::hip::HIPStream& side, const c10::hip::HIPStream& use) {
  c10::hip::HIPStreamGuard g(side);
  auto one = [&](const at::Tensor& t) {
    if (!t.defined()) return t;
    note_xfer(t, dev);
    at::Tensor d = to_device(t, dev, /*non_blocking=*/true);  // pageable (spool file) pieces: staging ring
    if (d.is_cuda()) c10::hip::HIPCachingAllocator::recordStream(d.storage().data_ptr(), use);
    return d;
  };
  KV o = kv;
  o.kdata = one(kv.kdata);
  o.vdata = one(kv.vdata);
  o.koff = one(kv.koff);
  o.voff = one(kv.voff);
  return o;
}

SpoolConfig spool_cfg(const OocEnv& env, const std::shared_ptr<SpoolBudget>& b, const char* kind) {
  SpoolConfig c;
  c.budget = b;
  c.dir = env.dir;
  c.kind = kind;
  c.instance = env.instance;
  c.rank = env.rank;
  return c;
}

// spool the chunks of the parts (in order) into M bucket spools by a per-pair
// bucket id produced on the device by `dest_of(chunk)`; the spools share the
// host budget and go to disk beyond it (HBM holds only the chunks in flight)
template <typename F>
std::vector<Spool> spool(const std::vector<KV>& kvs, int64_t cap, at::Device dev, int M, F&& dest_of,
                         const OocEnv& env, OocStats* st) {
  auto budget = std::make_shared<SpoolBudget>();
  // an HBM tier of a quarter of the budget (the chunk in flight and the
  // per-partition converts use the rest): the first pieces stay on the
  // device, then pinned host memory, then disk
  budget->hbm = dev.is_cuda() && env.hbm > 0 ? env.hbm / 4 : 0;
  budget->host = env.host;
  std::vector<Spool> parts;
  parts.reserve((size_t)M);
  for (int d = 0; d < M; ++d) parts.emplace_back(dev, spool_cfg(env, budget, "part"));
  // every chunk of every part, in order: (part, first pair, end pair)
  std::vector<HostOff> h;
  struct Ch {
    size_t part;
    int64_t a, b;
  };
  std::vector<Ch> ch;
  bool host_side = false;
  for (size_t p = 0; p < kvs.size(); ++p) {
    h.push_back(host_off(kvs[p]));
    for (auto [a, b] : chunks(kvs[p], h.back(), cap)) ch.push_back({p, a, b});
    host_side = host_side || kvs[p].device().is_cpu();
  }
  const bool cuda = dev.is_cuda() && host_side && env.streams != 1;
  c10::optional<c10::hip::HIPStream> side, drain, main;
  if (cuda) {
    main = c10::hip::getCurrentHIPStream(dev.index());
    side = c10::hip::getStreamFromPool(false, dev.index());
    drain = c10::hip::getStreamFromPool(false, dev.index());
  }
  auto load = [&](size_t i) {
    const KV& kv = kvs[ch[i].part];
    const KV slice = kv_slice(kv, ch[i].a, ch[i].b, h[ch[i].part].kp(), h[ch[i].part].vp());
    if (!cuda || !kv.device().is_cpu()) return kv_to(slice, dev);
    return kv_to_async(slice, dev, *side, *main);
  };
  std::vector<hipEvent_t> ready(2, nullptr);
  if (cuda)
    for (auto& e : ready)
      if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) throw std::runtime_error("ooc: event");
  struct Ev {
    std::vector<hipEvent_t>* v;
    ~Ev() {
      for (auto e : *v)
        if (e) (void)hipEventDestroy(e);
    }
  } ev_guard{&ready};
  PhaseClock clk("spool");
  KV next;
  if (!ch.empty()) {
    next = load(0);
    if (cuda && hipEventRecord(ready[0], side->stream()) != hipSuccess) throw std::runtime_error("ooc: event");
  }
  for (size_t i = 0; i < ch.size(); ++i) {
    KV c = next;
    if (cuda && hipStreamWaitEvent(main->stream(), ready[i % 2], 0) != hipSuccess)
      throw std::runtime_error("ooc: stream wait");
    if (i + 1 < ch.size()) {  // chunk i+1 on the PCIe link while chunk i partitions
      next = load(i + 1);
      if (cuda && hipEventRecord(ready[(i + 1) % 2], side->stream()) != hipSuccess)
        throw std::runtime_error("ooc: event");
    }
    clk("load");
    at::Tensor dest = dest_of(c);
    clk("dest");
    Buckets B = bucket_local(c, dest, M);
    clk("bucket");
    const HostOff bh = host_off(B.kv);
    clk("partition");
    int64_t s = 0;
    if (cuda && B.kv.kfixed() && B.kv.vfixed() && B.kv.device().is_cuda()) {
      // the whole partitioned chunk drains in one copy per column; each
      // partition's piece is a view of the pinned buffer (fixed widths: no
      // offsets to rebase before the copy lands), kept as the host tier or
      // written to its file by a background thread; the buffer is freed with
      // the last piece viewing it
      // the HBM tier first: partitions [0, dk) of this chunk while it has
      // room (each piece its own device copy), then the rest drains
      const int64_t row = (int64_t)B.kv.kw + B.kv.vw;
      int dk = 0;
      for (int64_t left = budget->hbm; dk < M && B.count[dk] * row <= left; ++dk) left -= B.count[dk] * row;
      for (int d = 0; d < dk; ++d) {
        const int64_t e = s + B.count[d];
        if (e > s) parts[d].add(kv_slice(B.kv, s, e, nullptr, nullptr));
        s = e;
      }
      clk("hbm tier");
      const int64_t s0 = s;
      if (s0 < B.kv.n) {
        KV hk;
        const std::shared_ptr<DrainEvent> ev =
            drain_to_pinned(s0 ? kv_slice(B.kv, s0, B.kv.n, nullptr, nullptr) : B.kv, drain->stream(), &hk);
        clk("drain issue");
        for (int d = dk; d < M; ++d) {
          const int64_t e = s + B.count[d];
          if (e > s) {
            const KV piece = kv_slice(hk, s - s0, e - s0, nullptr, nullptr);
            const int64_t room = parts[d].host_room();
            if (room < 0 || room >= piece.nbytes()) parts[d].add_drained(piece, ev);
            else parts[d].add_drained_to_disk(piece, ev);
          }
          s = e;
        }
      }
    } else {
      for (int d = 0; d < M; ++d) {
        const int64_t e = s + B.count[d];
        if (e > s) parts[d].add(kv_slice(B.kv, s, e, bh.kp(), bh.vp()), cuda ? drain->stream() : nullptr);
        s = e;
      }
    }
    clk("spool add");
    if (st) {
      st->chunks++;
      st->bytes_staged += row_bytes(kvs[ch[i].part], h[ch[i].part], ch[i].a, ch[i].b);
    }
  }
  // no sync here: each spool waits for its own drains and background file
  // writes when it is read (take / gather), so the last chunks' disk writes
  // overlap the first partitions' work
  if (st)
    for (auto& p : parts) {
      st->files += p.stats().files;
      st->disk_bytes += p.stats().disk_bytes;
    }
  return parts;
}

// results of the per-partition pass: pinned while the host budget lasts,
// files beyond it; finish() = one pinned KV, or one memory-mapped file
struct KVSink {
  const OocEnv& env;
  OocStats* st;
  int64_t used = 0;
  std::vector<KV> parts;
  void add(const KV& x) {
    const int64_t b = x.nbytes();
    if (env.host < 0 || used + b <= env.host) {
      parts.push_back(kv_host(x));
      used += b;
    } else {
      parts.push_back(kv_to_file({x.device().is_cpu() ? x : kv_host(x)}, spool_path(env.dir, "sort", env.instance,
                                                                                     env.rank)));
      if (st) {
        st->files++;
        st->disk_bytes += b;
      }
    }
  }
  int64_t total() const {
    int64_t t = 0;
    for (auto& p : parts) t += p.nbytes();
    return t;
  }
  KV finish(const KV& like) {
    if (parts.empty()) return kv_host(empty_kv(at::Device(at::kCPU), like.kw, like.vw));
    if (env.host < 0 || total() <= env.host) return kv_host(concat(parts, at::Device(at::kCPU)));
    if (st) st->files++;
    return kv_to_file(parts, spool_path(env.dir, "kv", env.instance, env.rank));
  }
};

int parts_for(int64_t bytes, int64_t budget, double factor) {
  const int64_t per = std::max<int64_t>(1, (int64_t)(budget / factor));
  return (int)std::min<int64_t>(std::max<int64_t>(2, (bytes + per - 1) / per), 4096);
}

KMV kmv_concat_host(const std::vector<KMV>& parts, const KV& like) {
  KMV out;
  std::vector<KV> keys, vals;
  std::vector<at::Tensor> segs;
  int64_t base = 0;
  for (const KMV& m : parts) {
    keys.push_back(m.keys);
    KV v;
    v.n = m.nval;
    v.kw = 0;
    v.vw = m.vw;
    v.kdata = at::empty({0}, opt(at::kCPU, at::kByte));
    v.vdata = m.vdata;
    v.voff = m.voff;
    vals.push_back(v);
    segs.push_back(m.seg.narrow(0, 0, m.nkey) + base);
    base += m.nval;
    out.nkey += m.nkey;
  }
  segs.push_back(at::full({1}, base, opt(at::kCPU, at::kLong)));
  out.keys = parts.empty() ? empty_kv(at::Device(at::kCPU), like.kw, 0) : concat(keys, at::Device(at::kCPU));
  out.keys.vw = 0;
  KV vcat = parts.empty() ? empty_kv(at::Device(at::kCPU), 0, like.vw) : concat(vals, at::Device(at::kCPU));
  out.vdata = vcat.vdata;
  out.voff = vcat.voff;
  out.vw = vcat.vw;
  out.nval = base;
  out.seg = at::cat(segs);
  return kmv_host(out);
}

}  // namespace

bool needs_ooc(int64_t bytes, int64_t budget, double factor) { return budget > 0 && bytes * factor > budget; }

namespace {

// one KMV whose single key holds every value of `pieces` (host / file KVs of
// one key, in order): the key once, the values concatenated where the host
// budget allows, else in one file. Every key is checked equal to the first on
// the device (the pieces were routed by a 64-bit hash).
KMV one_key_kmv(std::vector<KV>& pieces, const OocEnv& env, at::Device dev, OocStats* st, bool* in_file) {
  const int64_t cap = std::max<int64_t>(env.hbm / 4, 1);
  KV first;
  std::vector<KV> vals;
  int64_t n = 0, vbytes = 0;
  for (KV& p : pieces) {
    if (p.n == 0) continue;
    const HostOff h = host_off(p);
    if (!first.kdata.defined()) first = kv_host(kv_slice(p, 0, 1, h.kp(), h.vp()));
    at::Tensor k0 = first.kdata.to(dev);
    for (auto [a, b] : chunks(p, h, cap)) {
      const KV c = kv_slice(p, a, b, h.kp(), h.vp());
      at::Tensor kd = c.kdata.to(dev);
      bool same;
      if (c.kfixed()) {
        same = c.kw == 0 || kd.view({c.n, c.kw}).eq(k0.view({1, c.kw})).all().item<bool>();
      } else {
        at::Tensor ko = c.koff.to(dev);
        at::Tensor len = ko.narrow(0, 1, c.n) - ko.narrow(0, 0, c.n);
        const int64_t L = k0.numel();
        same = len.eq(L).all().item<bool>() && (L == 0 || kd.view({c.n, L}).eq(k0.view({1, L})).all().item<bool>());
      }
      if (!same) throw std::runtime_error("out-of-core convert: 64-bit key hash collision between hot keys");
    }
    KV v;
    v.n = p.n;
    v.kw = 0;
    v.vw = p.vw;
    v.kdata = at::empty({0}, opt(at::kCPU, at::kByte));
    v.vdata = p.vdata;
    v.voff = p.voff;
    vals.push_back(v);
    n += p.n;
    vbytes += p.nbytes();
  }
  pieces.clear();
  KMV m;
  m.keys = first;
  m.keys.vw = 0;
  m.keys.vdata = at::empty({0}, opt(at::kCPU, at::kByte));
  m.keys.voff = at::Tensor();
  m.nkey = 1;
  m.nval = n;
  m.seg = at::tensor({int64_t(0), n}, opt(at::kCPU, at::kLong));
  KV vcat;
  *in_file = false;
  if (env.host < 0 || vbytes <= env.host) {
    vcat = concat(vals, at::Device(at::kCPU), /*pin=*/dev.is_cuda());
  } else {
    vcat = kv_to_file(vals, spool_path(env.dir, "kmv", env.instance, env.rank));
    *in_file = true;
    if (st) {
      st->files++;
      st->disk_bytes += vbytes;
    }
  }
  m.vw = vcat.vw;
  m.vdata = vcat.vdata;
  m.voff = vcat.voff;
  return m;
}

// sub-partition hash of level L (independent of the first pass's bits)
at::Tensor level_hash(const at::Tensor& h, int level) {
  static const int64_t mult[4] = {(int64_t)0x9E3779B97F4A7C15ull, (int64_t)0xC2B2AE3D27D4EB4Full,
                                  (int64_t)0x165667B19E3779F9ull, (int64_t)0xD6E8FEB86659FD93ull};
  at::Tensor x = at::bitwise_xor(h, at::bitwise_right_shift(h, 29)).mul_(mult[level & 3]);
  return at::bitwise_right_shift(x, 33).bitwise_and_((int64_t(1) << 31) - 1);
}

// A partition more than a quarter of the budget (one key, or a few, hold most
// of it: the extended-KMV case of the reference, src/keymultivalue.cpp:845-846,
// 974-999): count pass — every chunk's keys counted on the device, candidates
// (over 1/nchunks of the hot threshold in some chunk) summed on the host;
// split pass — hot keys' pairs to a spool each, the rest re-partitioned by a
// new hash; then each hot key becomes one KMV pair of values on the host (no
// HBM copy of it ever), each sub-partition is converted in HBM or split again.
void ooc_convert_big(std::vector<KV> pieces, const OocEnv& env, at::Device dev, OocStats* st, int level,
                     const std::function<void(KMV&&, bool)>& keep) {
  const int64_t budget = env.hbm, cap = std::max<int64_t>(budget / 4, 1);
  int64_t n = 0, bytes = 0;
  for (const KV& p : pieces) {
    n += p.n;
    bytes += p.nbytes();
  }
  if (n == 0) return;
  // hot threshold: a quarter of a chunk's pairs
  const int64_t chunk_pairs = std::max<int64_t>(1, (int64_t)((double)n * (double)cap / (double)std::max<int64_t>(bytes, 1)));
  const int64_t T = std::max<int64_t>(2, chunk_pairs / 4);
  std::vector<std::tuple<size_t, int64_t, int64_t>> ch;  // piece, a, b
  std::vector<HostOff> hs;
  hs.reserve(pieces.size());
  for (size_t q = 0; q < pieces.size(); ++q) {
    hs.push_back(host_off(pieces[q]));
    for (auto [a, b] : chunks(pieces[q], hs.back(), cap)) ch.emplace_back(q, a, b);
  }
  const int64_t per_chunk = std::max<int64_t>(1, T / (int64_t)std::max<size_t>(ch.size(), 1));
  std::unordered_map<uint64_t, int64_t> cand;
  {
    for (size_t i = 0; i < ch.size(); ++i) {
      const size_t pi = std::get<0>(ch[i]);
      KV c = kv_to(kv_slice(pieces[pi], std::get<1>(ch[i]), std::get<2>(ch[i]), hs[pi].kp(), hs[pi].vp()), dev);
      at::Tensor h = std::get<0>(at::sort(hash64_keys(c)));
      auto [u, inv, cnt] = at::unique_consecutive(h, false, true);
      at::Tensor sel = cnt.gt(per_chunk);
      at::Tensor hu = u.masked_select(sel).to(at::kCPU), hc = cnt.masked_select(sel).to(at::kCPU);
      const int64_t* up = hu.data_ptr<int64_t>();
      const int64_t* cp = hc.data_ptr<int64_t>();
      for (int64_t j = 0; j < hu.numel(); ++j) cand[(uint64_t)up[j]] += cp[j];
    }
  }
  std::vector<std::pair<int64_t, uint64_t>> hot;
  for (auto& [k, c] : cand)
    if (c >= T / 2) hot.emplace_back(c, k);
  std::sort(hot.begin(), hot.end(), std::greater<>());
  if (hot.size() > 64) hot.resize(64);
  const int H = (int)hot.size();
  const int M2 = std::min(parts_for(bytes, budget, 4.0), 256 - H);
  if (level >= 6 || (H == 0 && M2 < 2)) {  // nothing left to cut: convert as it is
    KV p = kv_to(concat(pieces, at::Device(at::kCPU)), dev);
    keep(convert(p), false);
    return;
  }
  std::vector<uint64_t> hk;
  for (auto& x : hot) hk.push_back(x.second);
  std::sort(hk.begin(), hk.end(), [](uint64_t a, uint64_t b) { return (int64_t)a < (int64_t)b; });
  at::Tensor hot_dev = at::from_blob(hk.data(), {(int64_t)hk.size()}, opt(at::kCPU, at::kLong)).clone().to(dev);
  auto parts = spool(pieces, cap, dev, M2 + H, [&](const KV& c) {
    at::Tensor h = hash64_keys(c);
    at::Tensor sub = at::remainder(level_hash(h, level), M2);
    if (H == 0) return sub.to(at::kInt);
    at::Tensor idx = at::searchsorted(hot_dev, h).clamp_max_(H - 1);
    at::Tensor is_hot = hot_dev.index_select(0, idx).eq(h);
    return at::where(is_hot, idx + M2, sub).to(at::kInt);
  }, env, st);
  pieces.clear();
  for (int d = 0; d < M2; ++d) {
    if (parts[d].empty()) continue;
    if (parts[d].bytes() * 4 <= budget) {
      KV p = concat_upload(parts[d].take(), dev);
      keep(convert(p), false);
    } else {
      ooc_convert_big(parts[d].take(), env, dev, st, level + 1, keep);
    }
  }
  for (int j = 0; j < H; ++j) {
    if (parts[M2 + j].empty()) continue;
    std::vector<KV> pc = parts[M2 + j].take();
    bool in_file = false;
    KMV m = one_key_kmv(pc, env, dev, st, &in_file);
    keep(std::move(m), in_file);
    if (st) st->hot_keys++;
  }
}

}  // namespace

std::vector<KMV> ooc_convert_parts(const std::vector<KV>& kvs, const OocEnv& env, at::Device dev, OocStats* st) {
  const int64_t budget = env.hbm;
  int64_t bytes = 0;
  for (const KV& k : kvs) bytes += k.nbytes();
  const KV& kv = kvs.at(0);
  const int M = parts_for(bytes, budget, 4.0);
  if (st) st->parts = M;
  PhaseClock clk("convert");
  auto parts = spool(kvs, std::max<int64_t>(budget / 4, 1), dev, M, [&](const KV& c) {
    // a hash independent of the shuffle's owner hash (every key on this rank
    // has the same owner hash mod P): bits 20.. of the 64-bit grouping hash
    at::Tensor h = hash64_keys(c);
    if (h.is_cuda()) {  // one kernel (util.hip) instead of shift, and, remainder and a cast
      at::Tensor d = at::empty({h.numel()}, opt(h.device(), at::kInt));
      k::part_of_hash(reinterpret_cast<const uint64_t*>(h.data_ptr<int64_t>()), h.numel(), 20,
                      (uint64_t(1) << 40) - 1, M, d.data_ptr<int32_t>(), at::hip::getCurrentHIPStream());
      return d;
    }
    return at::remainder(at::bitwise_right_shift(h, 20).bitwise_and_((int64_t(1) << 40) - 1), M).to(at::kInt);
  }, env, st);
  clk("partition pass");
  std::vector<KMV> out;
  int64_t used = 0;
  // on a GPU the pass is a pipeline: partition d+1 uploads on one side stream
  // while d converts, and d's result drains to pinned memory on another
  const bool pipe = dev.is_cuda();
  c10::optional<c10::hip::HIPStream> ups, dns;
  if (pipe) {
    ups = c10::hip::getStreamFromPool(false, dev.index());
    dns = c10::hip::getStreamFromPool(false, dev.index());
  }
  std::vector<std::shared_ptr<DrainEvent>> drains;
  // in_file: a hot key whose values one_key_kmv already put in a file
  auto keep = [&](KMV&& m, bool in_file) {
    const int64_t b = m.nbytes();
    const bool on_host = m.seg.is_cpu();
    if (env.host < 0 || used + b <= env.host || in_file) {
      // pinned results while the host budget lasts (a file-backed hot key
      // stays where it is)
      if (on_host) {
        out.push_back(m);
      } else if (pipe) {
        const hipStream_t c = dns->stream();
        fence_after_current(c);
        KMV h = m;
        h.keys.kdata = drain_tensor(m.keys.kdata, c);
        h.keys.vdata = drain_tensor(m.keys.vdata, c);
        h.keys.koff = drain_tensor(m.keys.koff, c);
        h.keys.voff = drain_tensor(m.keys.voff, c);
        h.vdata = drain_tensor(m.vdata, c);
        h.voff = drain_tensor(m.voff, c);
        h.seg = drain_tensor(m.seg, c);
        drains.push_back(record_event(c));
        out.push_back(h);
      } else {
        out.push_back(kmv_host(m));
      }
      if (!in_file) used += b;
    } else {  // the disk tier: one file per partition result
      out.push_back(kmv_to_file({m}, spool_path(env.dir, "kmv", env.instance, env.rank)));
      if (st) {
        st->files++;
        st->disk_bytes += b;
      }
    }
  };
  auto fits = [&](int d) { return !parts[d].empty() && parts[d].bytes() * 4 <= budget; };
  // partition d's pieces straight into one device KV (no host concat); on
  // the upload stream when pipelined (the pool orders the new blocks there)
  // pinned pieces of an upload, held until its event passed
  std::vector<std::pair<std::shared_ptr<DrainEvent>, std::vector<at::Tensor>>> held;
  auto upload = [&](int d, std::shared_ptr<DrainEvent>* ev) {
    if (!pipe) return concat_upload(parts[d].take(), dev);
    for (size_t i = 0; i < held.size();)  // release the sources of finished uploads
      if (hipEventQuery(held[i].first->e) == hipSuccess) held.erase(held.begin() + (long)i);
      else ++i;
    KV p;
    std::vector<at::Tensor> hold;
    {
      c10::hip::HIPStreamGuard g(*ups);
      std::vector<KV> pieces = parts[d].take();
      clk("take (drains, file writes)");
      p = concat_upload(pieces, dev, &hold);
      clk("upload issue");
    }
    *ev = record_event(ups->stream());
    held.emplace_back(*ev, std::move(hold));
    return p;
  };
  int pre_d = -1;
  KV pre;
  std::shared_ptr<DrainEvent> pre_ev;
  for (int d = 0; d < M; ++d) {
    // (a prefetched partition's spool is already empty: its pieces are in pre)
    if (pre_d != d && parts[d].empty()) continue;
    if (pre_d != d && !fits(d)) {  // over budget: a hot key (or a few)
      ooc_convert_big(parts[d].take(), env, dev, st, 1, keep);
      continue;
    }
    KV p;
    std::shared_ptr<DrainEvent> ev;
    if (pre_d == d) {
      p = std::move(pre);
      ev = std::move(pre_ev);
      pre = KV();
      pre_d = -1;
    } else {
      p = upload(d, &ev);
    }
    if (ev) {  // the current stream reads what the upload stream wrote
      const hipStream_t cs = at::hip::getCurrentHIPStream().stream();
      if (hipStreamWaitEvent(cs, ev->e, 0) != hipSuccess) throw std::runtime_error("ooc: upload wait");
      for (const at::Tensor* t : {&p.kdata, &p.vdata, &p.koff, &p.voff})
        if (t->defined() && t->is_cuda())
          c10::hip::HIPCachingAllocator::recordStream(t->storage().data_ptr(), at::hip::getCurrentHIPStream());
    }
    clk("to device");
    int n = d + 1;
    while (n < M && parts[n].empty()) ++n;
    if (n < M && fits(n)) {  // (on the CPU too: the same bookkeeping, no streams)
      pre = upload(n, &pre_ev);
      pre_d = n;
    }
    clk("prefetch");
    KMV m = convert(p);
    p = KV();
    clk("convert");
    keep(std::move(m), false);
    clk("result to host");
  }
  for (const auto& e : drains)
    if (hipEventSynchronize(e->e) != hipSuccess) throw std::runtime_error("ooc: result drain failed");
  for (const auto& h : held)
    if (hipEventSynchronize(h.first->e) != hipSuccess) throw std::runtime_error("ooc: upload failed");
  clk("drain sync");
  if (out.empty()) out.push_back(kmv_concat_host(out, kv));  // an empty KMV of the KV's widths
  return out;
}

KMV ooc_convert(const std::vector<KV>& kvs, const OocEnv& env, at::Device dev, OocStats* st) {
  std::vector<KMV> out = ooc_convert_parts(kvs, env, dev, st);
  if (out.size() == 1) return out[0];
  int64_t total = 0;
  for (auto& m : out) total += m.nbytes();
  if (env.host < 0 || total <= env.host) return kmv_concat_host(out, kvs.at(0));
  if (st) st->files++;
  return kmv_to_file(out, spool_path(env.dir, "kmv", env.instance, env.rank));
}

KV ooc_sort(const KV& kv, int flag, bool by_value, const OocEnv& env, at::Device dev, OocStats* st) {
  const int64_t budget = env.hbm;
  const int M = std::min(parts_for(kv.nbytes(), budget, 4.0), 4096);
  if (st) st->parts = M;
  const int64_t cap = std::max<int64_t>(budget / 4, 1);
  auto skeys = [&](const KV& c) {
    return by_value ? column_sort_keys(c.vdata, c.voff, c.vw, c.n, flag)
                    : column_sort_keys(c.kdata, c.koff, c.kw, c.n, flag);
  };
  // pass 1: sample the unsigned radix keys of every chunk
  const HostOff h = host_off(kv);
  const auto ch = chunks(kv, h, cap);
  std::vector<uint64_t> sample;
  const int64_t want = std::max<int64_t>(64, 32 * M);
  for (auto [a, b] : ch) {
    KV c = kv_to(kv_slice(kv, a, b, h.kp(), h.vp()), dev);
    at::Tensor sk = skeys(c);
    const int64_t stride = std::max<int64_t>(1, (b - a) * (int64_t)ch.size() / want);
    at::Tensor smp = sk.slice(0, 0, sk.numel(), stride).to(at::kCPU).contiguous();
    const uint64_t* p = reinterpret_cast<const uint64_t*>(smp.data_ptr<int64_t>());
    sample.insert(sample.end(), p, p + smp.numel());
  }
  std::sort(sample.begin(), sample.end());
  // M-1 distinct splitters (unsigned radix-key order)
  std::vector<uint64_t> split;
  for (int j = 1; j < M && !sample.empty(); ++j) {
    const uint64_t v = sample[std::min(sample.size() - 1, sample.size() * j / M)];
    if (split.empty() || v != split.back()) split.push_back(v);
  }
  const int MB = (int)split.size() + 1;
  at::Tensor sp = at::from_blob(split.data(), {(int64_t)split.size()}, opt(at::kCPU, at::kLong)).clone().to(dev);
  // pass 2: range partition, bucket = number of splitters below the key
  // (a binary search over the splitters in LDS, k_bucket_by_splitters)
  auto parts = spool({kv}, cap, dev, MB, [&](const KV& c) {
    at::Tensor k = skeys(c).contiguous();
    at::Tensor out = at::empty({c.n}, opt(dev, at::kInt));
    if (c.n == 0) return out;
    if (dev.is_cuda()) {
      k::bucket_by_splitters(reinterpret_cast<const uint64_t*>(k.data_ptr()), c.n,
                             reinterpret_cast<const uint64_t*>(sp.data_ptr()), (int)split.size(),
                             out.data_ptr<int32_t>(), at::hip::getCurrentHIPStream());
    } else {
      const uint64_t* kp = reinterpret_cast<const uint64_t*>(k.data_ptr());
      int32_t* o = out.data_ptr<int32_t>();
      for (int64_t i = 0; i < c.n; ++i) o[i] = (int32_t)(std::lower_bound(split.begin(), split.end(), kp[i]) - split.begin());
    }
    return out;
  }, env, st);
  if (st) st->parts = MB;
  // pass 3: sort each bucket in HBM, append in bucket (= key) order
  KVSink sink{env, st};
  for (int d = 0; d < MB; ++d) {
    if (parts[d].empty()) continue;
    KV p = kv_to(parts[d].gather_host(), dev);
    parts[d].clear();
    sink.add(sort_kv(p, flag, by_value));
  }
  if (sink.parts.empty()) return kv_host(kv);
  return sink.finish(kv);
}

KV ooc_exchange(const KV& kv, const at::Tensor& dest_host, const Comm& comm, const OocEnv& env, at::Device dev,
                int all2all, OocStats* st, ShuffleStats* sst) {
  const int64_t cap = std::max<int64_t>(env.hbm / 4, 1);
  const HostOff h = host_off(kv);
  const auto ch = chunks(kv, h, cap);
  // lock-step chunks: a rank with fewer (or none) joins with empty ones
  const int64_t R = comm.allreduce((int64_t)ch.size(), Comm::MAX);
  at::Tensor dh = dest_host.defined() ? dest_host.to(at::kCPU).to(at::kInt).contiguous() : at::Tensor();
  if (dh.defined() && dh.numel() != kv.n) throw std::runtime_error("ooc_exchange: one destination per pair");
  ExchangeOpts o;
  o.chunk_bytes = cap;           // receive rounds of at most one chunk
  o.host_sink = dev.is_cuda();   // received pairs land in pinned host memory, not HBM
  o.all2all = all2all;
  KVSink sink{env, st};
  for (int64_t r = 0; r < R; ++r) {
    const bool mine = r < (int64_t)ch.size();
    KV c = mine ? kv_to(kv_slice(kv, ch[r].first, ch[r].second, h.kp(), h.vp()), dev) : empty_kv(dev, kv.kw, kv.vw);
    at::Tensor d;
    if (dh.defined())
      d = (mine ? dh.narrow(0, ch[r].first, ch[r].second - ch[r].first) : at::empty({0}, opt(at::kCPU, at::kInt))).to(dev);
    ShuffleStats s1;
    KV out = exchange(std::move(c), d, comm, o, &s1);
    if (sst) {
      sst->send_bytes += s1.send_bytes;
      sst->recv_bytes += s1.recv_bytes;
      sst->send_pairs += s1.send_pairs;
      sst->recv_pairs += s1.recv_pairs;
      sst->rounds += s1.rounds;
      sst->seconds += s1.seconds;
    }
    if (out.n) sink.add(out);
    if (st) {
      st->chunks++;
      if (mine) st->bytes_staged += row_bytes(kv, h, ch[r].first, ch[r].second);
    }
  }
  if (st) st->parts = R;
  return sink.finish(kv);
}

void ooc_for_each_kmv_block(const KMV& kmv, const OocEnv& env, at::Device dev,
                            const std::function<void(const KMV&, int)>& fn, bool split, OocStats* st) {
  const int64_t budget = env.hbm;
  at::Tensor seg = kmv.seg.to(at::kCPU).contiguous();
  const int64_t* s = seg.data_ptr<int64_t>();
  at::Tensor vo = kmv.vw < 0 ? kmv.voff.to(at::kCPU).contiguous() : at::Tensor();
  at::Tensor ko = kmv.keys.kw < 0 ? kmv.keys.koff.to(at::kCPU).contiguous() : at::Tensor();
  const int64_t* vop = vo.defined() ? vo.data_ptr<int64_t>() : nullptr;
  const int64_t* kop = ko.defined() ? ko.data_ptr<int64_t>() : nullptr;
  auto vbytes_rows = [&](int64_t j0, int64_t j1) {  // values [j0, j1)
    return kmv.vw >= 0 ? (j1 - j0) * kmv.vw : vop[j1] - vop[j0] + 8 * (j1 - j0);
  };
  auto vbytes = [&](int64_t a, int64_t b) { return vbytes_rows(s[a], s[b]); };  // values of keys [a, b)
  // keys [a, b), values [j0, j1) (a block of key a when b == a + 1 and the
  // range is part of its values) as a device KMV
  auto piece = [&](int64_t a, int64_t b, int64_t j0, int64_t j1) {
    KMV m;
    m.nkey = b - a;
    m.nval = j1 - j0;
    m.keys = kv_slice(kmv.keys, a, b, kop, nullptr);
    m.vw = kmv.vw;
    if (kmv.vw >= 0) {
      m.vdata = kmv.vdata.narrow(0, j0 * kmv.vw, m.nval * kmv.vw);
    } else {
      m.vdata = kmv.vdata.narrow(0, vop[j0], vop[j1] - vop[j0]);
      m.voff = kmv.voff.narrow(0, j0, m.nval + 1) - vop[j0];
    }
    if (j0 == s[a] && j1 == s[b]) m.seg = kmv.seg.narrow(0, a, m.nkey + 1) - s[a];
    else m.seg = at::tensor({int64_t(0), m.nval}, opt(at::kCPU, at::kLong));
    KMV md = m;
    md.keys = kv_to(m.keys, dev);
    note_xfer(m.vdata, dev);
    note_xfer(m.voff, dev);
    note_xfer(m.seg, dev);
    md.vdata = to_device(m.vdata, dev);
    if (m.voff.defined()) md.voff = to_device(m.voff, dev);
    md.seg = to_device(m.seg, dev);
    return md;
  };
  const int64_t cap = std::max<int64_t>(budget / 4, 1);
  PhaseClock clk("kmv pieces");
  clk("host offsets");
  int64_t a = 0;
  while (a < kmv.nkey) {
    if (split && vbytes(a, a + 1) > cap && s[a + 1] - s[a] > 1) {
      // one key past the piece size (an extended KMV pair): its values in
      // blocks of at most cap bytes, first / last flagged
      int64_t j0 = s[a];
      const int64_t je = s[a + 1];
      while (j0 < je) {
        int64_t j1;
        if (kmv.vw > 0) {
          j1 = std::min(je, j0 + std::max<int64_t>(1, cap / kmv.vw));
        } else if (kmv.vw == 0) {
          j1 = je;
        } else {
          j1 = grow(j0, je, [&](int64_t e) { return vbytes_rows(j0, e) <= cap; });
        }
        int flags = kBlock;
        if (j0 == s[a]) flags |= kFirst;
        if (j1 == je) flags |= kLast;
        fn(piece(a, a + 1, j0, j1), flags);
        if (st) st->chunks++;
        j0 = j1;
      }
      if (st) st->split_keys++;
      ++a;
      continue;
    }
    const int64_t b = grow(a, kmv.nkey, [&](int64_t e) { return vbytes(a, e) <= cap; });
    KMV pc = piece(a, b, s[a], s[b]);
    clk("piece to device");
    fn(pc, 0);
    clk("callback");
    if (st) st->chunks++;
    a = b;
  }
}

void ooc_for_each_kmv_piece(const KMV& kmv, const OocEnv& env, at::Device dev, const std::function<void(const KMV&)>& fn,
                            OocStats* st) {
  ooc_for_each_kmv_block(kmv, env, dev, [&](const KMV& m, int) { fn(m); }, false, st);
}

namespace {
// fold a block's partial result (one pair, host) into the key's running one
void fold_partial(KV& acc, const KV& part, const std::string& op, const std::string& dtype) {
  if (op == "first") return;
  if (op == "last") {
    acc = part;
    return;
  }
  if (op == "count") {
    int32_t* a = reinterpret_cast<int32_t*>(acc.vdata.data_ptr());
    *a += *reinterpret_cast<const int32_t*>(part.vdata.data_ptr());
    return;
  }
  const int opc = op == "sum" ? 0 : op == "min" ? 1 : 2;
  auto f = [&](auto* a, const auto* b) {
    using T = std::remove_pointer_t<decltype(a)>;
    const T x = *b;
    *a = opc == 0 ? T(*a + x) : opc == 1 ? (x < *a ? x : *a) : (x > *a ? x : *a);
  };
  void* ap = acc.vdata.data_ptr();
  const void* bp = part.vdata.data_ptr();
  if (dtype == "int32" || dtype == "int" || dtype == "uint32") f((int32_t*)ap, (const int32_t*)bp);
  else if (dtype == "int64" || dtype == "uint64") f((int64_t*)ap, (const int64_t*)bp);
  else if (dtype == "float32" || dtype == "float") f((float*)ap, (const float*)bp);
  else f((double*)ap, (const double*)bp);
}
}  // namespace

KV ooc_reduce_builtin(const KMV& kmv, const std::string& op, const std::string& dtype, const OocEnv& env,
                      at::Device dev, OocStats* st) {
  KVSink sink{env, st};
  KV acc;  // the split key's running result (host, one pair)
  ooc_for_each_kmv_block(kmv, env, dev, [&](const KMV& md, int flags) {
    KV r = reduce_builtin(md, op, dtype);
    if (!(flags & kBlock)) {
      sink.add(r);
      return;
    }
    // a key cut across pieces: partials carried to its last block
    KV rh = kv_host(r);
    rh.vdata = rh.vdata.clone();
    if (flags & kFirst) acc = rh;
    else fold_partial(acc, rh, op, dtype);
    if (flags & kLast) {
      sink.add(acc);
      acc = KV();
    }
  }, true, st);
  if (sink.parts.empty()) return kv_host(reduce_builtin(kmv, op, dtype));
  return sink.finish(sink.parts[0]);
}

}  // namespace mrh
