// WordCounter (wordcount.h): host driver of the in-mapper combining kernels.
#include "wordcount.h"

#include <ATen/hip/HIPContext.h>
#include <c10/hip/HIPFunctions.h>

#include <cstring>
#include <stdexcept>

#include "kernels/launch.h"

namespace mrh {

namespace {

at::TensorOptions opt(at::Device d, at::ScalarType t) { return at::TensorOptions().device(d).dtype(t); }
template <typename T>
T* P(const at::Tensor& t) {
  return t.numel() ? reinterpret_cast<T*>(t.data_ptr()) : nullptr;
}
hipStream_t cur() { return at::hip::getCurrentHIPStream(); }
bool is_ws(uint8_t c) { return c == ' ' || c == '\t' || c == '\n' || c == '\f' || c == '\r' || c == 0; }
int64_t pow2_at_least(int64_t x) {
  int64_t p = 1;
  while (p < x) p <<= 1;
  return p;
}
constexpr int64_t kMaxArena = int64_t(1) << 31;  // arena offsets are 31-bit

}  // namespace

WordCounter::WordCounter(at::Device dev, int64_t init_slots)
    : dev_(dev.is_cuda() && !dev.has_index() ? at::Device(at::kCUDA, c10::hip::current_device()) : dev),
      init_(pow2_at_least(std::max<int64_t>(init_slots, 1024))) {}

// make room for `new_words` possibly-distinct words of `new_bytes` text:
// the table stays <= 75 % full (so every probe sequence ends at a match or a
// free slot) and the arena can hold every new word plus its NUL
void WordCounter::reserve(int64_t used, int64_t new_words, int64_t new_bytes) {
  const int64_t need = used + new_words;
  if (!slots_.defined() || need * 4 > cap_ * 3) {
    int64_t cap = std::max(init_, cap_);
    while (need * 2 > cap) cap <<= 1;  // grow to <= 50 % load
    at::Tensor ns = at::zeros({cap}, opt(dev_, at::kLong));
    at::Tensor nc = at::zeros({cap}, opt(dev_, at::kInt));
    if (slots_.defined() && used > 0)
      k::wc_rehash(P<uint64_t>(slots_), P<uint32_t>(counts_), cap_, P<uint8_t>(arena_), P<uint64_t>(ns),
                   P<uint32_t>(nc), cap, cur());
    slots_ = ns;
    counts_ = nc;
    cap_ = cap;
  }
  const int64_t need_a = arena_used_ + new_bytes + new_words + 1;
  if (need_a > kMaxArena)
    throw std::runtime_error("WordCounter: the distinct words of one map task exceed the 2 GiB key arena; "
                             "use more map tasks");
  if (!arena_.defined() || need_a > arena_.numel()) {
    int64_t a = std::max<int64_t>(int64_t(64) << 20, arena_.defined() ? arena_.numel() : 0);
    while (a < need_a) a <<= 1;
    a = std::min(a, kMaxArena);
    at::Tensor na = at::empty({a}, opt(dev_, at::kByte));
    if (arena_used_) na.narrow(0, 0, arena_used_).copy_(arena_.narrow(0, 0, arena_used_));
    arena_ = na;
  }
}

void WordCounter::add(const at::Tensor& text, int64_t n) {
  if (n <= 0) return;
  if (text.device() != dev_) throw std::runtime_error("WordCounter::add: text is on another device");
  if (text.numel() < n + 32) throw std::runtime_error("WordCounter::add: text buffer must be padded by >= 32 bytes");
  if (n >= (int64_t(1) << 31)) throw std::runtime_error("WordCounter::add: chunks must be < 2 GiB");
  const uint8_t* t = P<uint8_t>(text);
  if (!dev_.is_cuda()) {
    for (int64_t i = 0; i < n;) {
      while (i < n && is_ws(t[i])) ++i;
      if (i >= n) break;
      int64_t j = i;
      while (j < n && !is_ws(t[j])) ++j;
      ++host_[std::string((const char*)t + i, (size_t)(j - i))];
      ++words_;
      i = j;
    }
    return;
  }
  hipStream_t s = cur();
  // words in this chunk (upper bound of new distinct words) with the tokenizer's tile counts
  const int64_t nt = k::tok_num_tiles(n);
  at::Tensor cnt = at::empty({nt}, opt(dev_, at::kInt));
  k::tok_count(t, n, P<uint32_t>(cnt), s);
  if (!ctr_.defined()) ctr_ = at::zeros({2}, opt(dev_, at::kLong));
  at::Tensor info = at::cat({cnt.to(at::kLong).sum().view({1}), ctr_}).to(at::kCPU);  // one sync per chunk
  const int64_t W = info.data_ptr<int64_t>()[0];
  used_ = info.data_ptr<int64_t>()[1];
  arena_used_ = info.data_ptr<int64_t>()[2];
  if (W == 0) return;
  words_ += W;
  reserve(used_, W, n);
  at::Tensor newlist = at::empty({W}, opt(dev_, at::kInt));
  k::wc_count(t, n, P<uint64_t>(slots_), P<uint32_t>(counts_), cap_, P<int32_t>(newlist), P<uint64_t>(ctr_),
              (uint64_t)used_, P<uint8_t>(arena_), s);
  k::wc_migrate(t, n, P<uint64_t>(slots_), cap_, P<int32_t>(newlist), P<uint64_t>(ctr_), (uint64_t)used_,
                P<uint8_t>(arena_), W, s);
}

KV WordCounter::finish() {
  if (words_ > INT32_MAX)
    throw std::runtime_error("WordCounter: more than 2^31 words in one map task; use more map tasks");
  KV kv;
  kv.kw = -1;
  kv.vw = 4;
  if (!dev_.is_cuda()) {
    std::string kd;
    std::vector<int64_t> koff{0};
    std::vector<int32_t> vals;
    for (auto& [w, c] : host_) {
      kd += w;
      kd.push_back('\0');
      koff.push_back((int64_t)kd.size());
      vals.push_back((int32_t)c);
    }
    host_.clear();
    kv.n = (int64_t)vals.size();
    kv.kdata = at::empty({(int64_t)kd.size()}, opt(dev_, at::kByte));
    if (!kd.empty()) std::memcpy(kv.kdata.data_ptr(), kd.data(), kd.size());
    kv.koff = at::tensor(koff, opt(dev_, at::kLong));
    kv.vdata = vals.empty() ? at::empty({0}, opt(dev_, at::kByte))
                            : at::tensor(vals, opt(dev_, at::kInt)).view(at::kByte);
    return kv;
  }
  if (!slots_.defined()) {
    kv.n = 0;
    kv.kdata = at::empty({0}, opt(dev_, at::kByte));
    kv.koff = at::zeros({1}, opt(dev_, at::kLong));
    kv.vdata = at::empty({0}, opt(dev_, at::kByte));
    return kv;
  }
  hipStream_t s = cur();
  // occupied slots, in slot order: flags + scan + scatter (no rocPRIM compaction)
  const int64_t cap = slots_.numel();
  at::Tensor flags = at::empty({cap}, opt(dev_, at::kInt));
  k::nz_flags(P<uint64_t>(slots_), cap, P<int32_t>(flags), s);
  at::Tensor pos = exclusive_scan(flags);
  const int64_t nk = pos[cap].item<int64_t>();
  at::Tensor idx = at::empty({std::max<int64_t>(nk, 1)}, opt(dev_, at::kLong));
  k::compact_nz(P<uint64_t>(slots_), P<int64_t>(pos), cap, P<int64_t>(idx), s);
  at::Tensor starts = at::empty({std::max<int64_t>(nk, 1)}, opt(dev_, at::kLong));
  at::Tensor lens = at::empty({std::max<int64_t>(nk, 1)}, opt(dev_, at::kInt));
  k::wc_keys(P<uint64_t>(slots_), P<int64_t>(idx), nk, P<uint8_t>(arena_), P<int64_t>(starts), P<int32_t>(lens), s);
  kv.koff = exclusive_scan(lens.narrow(0, 0, nk));
  const int64_t kb = nk ? kv.koff[nk].item<int64_t>() : 0;
  kv.kdata = at::empty({kb}, opt(dev_, at::kByte));
  k::copy_strings_nul(P<uint8_t>(arena_), P<int64_t>(starts), P<int64_t>(kv.koff), nk, P<uint8_t>(kv.kdata), s);
  kv.vdata = counts_.index_select(0, idx).view(at::kByte);
  kv.n = nk;
  slots_ = counts_ = arena_ = ctr_ = at::Tensor();
  cap_ = used_ = arena_used_ = 0;
  return kv;
}

}  // namespace mrh
