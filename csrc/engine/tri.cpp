// Triangle enumeration engine ops (kernels: csrc/kernels/tri.hip) with CPU
// twins of identical semantics.
#include <ATen/hip/HIPContext.h>
#include <c10/hip/HIPCachingAllocator.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <vector>
#include <string>

#include "../kernels/launch.h"
#include "kv.h"
#include "tri.h"

namespace mrh {

namespace {
at::TensorOptions opt(at::Device d, at::ScalarType t) { return at::TensorOptions().device(d).dtype(t); }
template <typename T>
T* P0(const at::Tensor& t) {
  return t.defined() ? reinterpret_cast<T*>(t.data_ptr()) : nullptr;
}
hipStream_t cur() { return at::hip::getCurrentHIPStream(); }

template <bool EMIT>
int64_t intersect_host(const int64_t* rp, const int32_t* col, uint32_t u, uint32_t v, std::vector<int64_t>* out) {
  int64_t i = rp[u], i1 = rp[u + 1], j = rp[v], j1 = rp[v + 1], n = 0;
  while (i < i1 && j < j1) {
    const uint32_t x = (uint32_t)col[i], y = (uint32_t)col[j];
    if (x < y) ++i;
    else if (y < x) ++j;
    else {
      if (EMIT) {
        out->push_back(u);
        out->push_back(v);
        out->push_back(x);
      }
      ++n;
      ++i;
      ++j;
    }
  }
  return n;
}
}  // namespace

at::Tensor tri_degrees(const at::Tensor& uniq_in, int64_t nvert) {
  at::Tensor uniq = uniq_in.contiguous();
  if (uniq.scalar_type() != at::kLong) throw std::runtime_error("tri_degrees: packed int64 edges expected");
  if (nvert > (int64_t(1) << 32)) throw std::runtime_error("tri_degrees: vertex ids must fit in 32 bits");
  const at::Device dev = uniq.device();
  const int64_t m = uniq.numel();
  nvert = std::max<int64_t>(nvert, 1);
  at::Tensor deg = at::zeros({nvert}, opt(dev, at::kInt));
  static const bool dbg = std::getenv("MRH_TRI_DEBUG") != nullptr;
  auto stage = [&](const char* what) {
    if (!dbg) return;
    if (uniq.is_cuda()) (void)hipDeviceSynchronize();
    std::fprintf(stderr, "mrhip tri_degrees: %s done\n", what);
  };
  if (uniq.is_cuda()) {
    const int nb = k::tri_deg_buckets(nvert);
    if (nb > 0 && m > 0) {
      // partitioned count (tri.hip k_deg_*): no scattered atomic per edge
      k::tri_deg_lo(P0<uint64_t>(uniq), m, P0<uint32_t>(deg), cur());
      stage("deg_lo");
      count_low_words(uniq, deg);
    } else {
      k::tri_degree(P0<uint64_t>(uniq), m, P0<uint32_t>(deg), cur());
    }
  } else {
    const uint64_t* e = P0<uint64_t>(uniq);
    int32_t* d = P0<int32_t>(deg);
    for (int64_t i = 0; i < m; ++i) {
      d[e[i] >> 32]++;
      d[(uint32_t)e[i]]++;
    }
  }
  return deg;
}

void count_low_words(const at::Tensor& packed_in, at::Tensor& deg) {
  at::Tensor packed = packed_in.contiguous();
  const at::Device dev = packed.device();
  const int64_t m = packed.numel(), nvert = deg.numel();
  if (m == 0) return;
  static const bool dbg = std::getenv("MRH_TRI_DEBUG") != nullptr;
  auto stage = [&](const char* what) {
    if (!dbg) return;
    if (packed.is_cuda()) (void)hipDeviceSynchronize();
    std::fprintf(stderr, "mrhip count_low_words: %s done\n", what);
  };
  if (!packed.is_cuda()) {
    const uint64_t* e = P0<uint64_t>(packed);
    int32_t* d = P0<int32_t>(deg);
    for (int64_t i = 0; i < m; ++i) d[(uint32_t)e[i]]++;
    return;
  }
  const hipStream_t s = cur();
  const int nb = k::tri_deg_buckets(nvert);
  if (nb <= 0) {
    k::count_low_atomic(P0<uint64_t>(packed), m, P0<uint32_t>(deg), s);
    return;
  }
  {
    const at::Tensor& uniq = packed;
    {
      at::Tensor bcount = at::zeros({nb}, opt(dev, at::kInt));
      k::tri_deg_count(P0<uint64_t>(uniq), m, nb, P0<unsigned int>(bcount), s);
      stage("deg_count");
      at::Tensor bstart = exclusive_scan(bcount.to(at::kLong).contiguous()).contiguous();  // nb + 1
      at::Tensor cursor = bstart.narrow(0, 0, nb).clone();
      at::Tensor ids = at::empty({m}, opt(dev, at::kShort));
      k::tri_deg_scatter(P0<uint64_t>(uniq), m, nb, P0<unsigned long long>(cursor), P0<uint16_t>(ids), s);
      stage("deg_scatter");
      // (bucket, piece) items: a bucket up to 2 M endpoints is one block's
      // (plain stores), a larger one (R-MAT hub ids) is split (atomic adds)
      at::Tensor bc = bcount.to(at::kCPU);
      const int32_t* bcp = bc.data_ptr<int32_t>();
      constexpr int64_t PIECE = int64_t(1) << 21;
      std::vector<int64_t> items;
      std::vector<int32_t> ilen;
      std::vector<uint8_t> whole;
      for (int b = 0; b < nb; ++b) {
        const int64_t c = (uint32_t)bcp[b];
        if (c == 0) continue;
        for (int64_t o = 0; o < c; o += PIECE) {
          items.push_back((int64_t)(((uint64_t)b << 40) | (uint64_t)o));
          ilen.push_back((int32_t)std::min<int64_t>(PIECE, c - o));
          whole.push_back(c <= PIECE ? 1 : 0);
        }
      }
      const int64_t ni = (int64_t)items.size();
      if (ni > 0) {
        at::Tensor ti = at::from_blob(items.data(), {ni}, opt(at::kCPU, at::kLong)).to(dev);
        at::Tensor tl = at::from_blob(ilen.data(), {ni}, opt(at::kCPU, at::kInt)).to(dev);
        at::Tensor tw = at::from_blob(whole.data(), {ni}, opt(at::kCPU, at::kByte)).to(dev);
        k::tri_deg_hist(P0<uint16_t>(ids), P0<unsigned long long>(bstart), P0<uint64_t>(ti), P0<uint32_t>(tl),
                        P0<uint8_t>(tw), ni, nvert, P0<uint32_t>(deg), s);
      }
    }
  }
}

std::pair<at::Tensor, at::Tensor> tri_rank_perm(const at::Tensor& deg) {
  const at::Device dev = deg.device();
  const int64_t nvert = deg.numel();
  // rank = position in (degree, id) order; perm[rank] = original id
  // the LSD radix sort is stable: sorting the degrees alone keeps equal
  // degrees in id order, i.e. (degree, id) order
  at::Tensor perm32 = std::get<1>(radix_sort_pairs(deg.to(at::kLong), at::arange(nvert, opt(dev, at::kInt)), 0, 32));
  at::Tensor perm = perm32.to(at::kLong);
  at::Tensor rank = at::empty({nvert}, opt(dev, at::kInt));
  if (deg.is_cuda()) k::tri_rank(P0<int32_t>(perm32), nvert, P0<int32_t>(rank), cur());
  else rank.index_put_({perm}, at::arange(nvert, opt(dev, at::kInt)));
  return {rank, perm};
}

at::Tensor tri_orient_keys(const at::Tensor& uniq_in, const at::Tensor& rank) {
  at::Tensor uniq = uniq_in.contiguous();
  const int64_t m = uniq.numel();
  at::Tensor oriented = at::empty({m}, uniq.options());
  if (m == 0) return oriented;
  if (uniq.is_cuda()) {
    k::tri_orient(P0<uint64_t>(uniq), m, P0<uint32_t>(rank), P0<uint64_t>(oriented), cur());
  } else {
    const uint64_t* e = P0<uint64_t>(uniq);
    const int32_t* r = P0<int32_t>(rank);
    uint64_t* o = P0<uint64_t>(oriented);
    for (int64_t i = 0; i < m; ++i) {
      const uint64_t ra = (uint32_t)r[e[i] >> 32], rb = (uint32_t)r[(uint32_t)e[i]];
      o[i] = ra < rb ? (ra << 32 | rb) : (rb << 32 | ra);
    }
  }
  return oriented;
}

at::Tensor tri_col_of(const at::Tensor& okeys) {
  const int64_t m = okeys.numel();
  if (okeys.is_cuda()) {
    at::Tensor col = at::empty({m}, opt(okeys.device(), at::kInt));
    if (m) k::tri_col(P0<uint64_t>(okeys), m, P0<uint32_t>(col), cur());
    return col;
  }
  return at::bitwise_and(okeys, (int64_t)0xffffffff).to(at::kInt);
}

at::Tensor tri_rowptr_of(const at::Tensor& okeys, int64_t nvert) {
  if (okeys.is_cuda()) {
    at::Tensor rowptr = at::empty({nvert + 1}, opt(okeys.device(), at::kLong));
    k::tri_rowptr(P0<uint64_t>(okeys), okeys.numel(), nvert, P0<int64_t>(rowptr), cur());
    return rowptr;
  }
  at::Tensor src = at::bitwise_right_shift(okeys, 32);
  at::Tensor cnt = bincount_dev(src, nvert);
  return exclusive_scan(cnt.to(at::kLong).contiguous());
}

std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> tri_prepare(const at::Tensor& uniq_in, int64_t nvert) {
  at::Tensor uniq = uniq_in.contiguous();
  nvert = std::max<int64_t>(nvert, 1);
  at::Tensor deg = tri_degrees(uniq, nvert);
  auto [rank, perm] = tri_rank_perm(deg);
  deg = at::Tensor();
  at::Tensor oriented = tri_orient_keys(uniq, rank);
  // keys-only: the oriented edges carry no payload
  at::Tensor okeys = oriented.numel() ? radix_sort_keys(oriented, 0, 64) : oriented;
  return {tri_rowptr_of(okeys, nvert), tri_col_of(okeys), okeys, perm};
}

// hub bitmap size: MRH_TRI_HUB vertices (0 = off); default nvert / 64 capped
// at 524288 (a 32 GB bitmap) and at a quarter of the free HBM — the best of
// a sweep on RMAT-24 (16.8 M vertices) with the sorted-word sparse hub kernel:
// 128 K / 192 K / 224 K / 256 K / 288 K / 320 K / 384 K / 512 K hubs = 214.8 /
// 164.9 / 159.6 / 159.6-162.9 / 172.0 / 173.0 / 176.5 / 181.6 ms
// (profiles/r3_trifind_hub_sweep.txt; nvert / 32 was best for the earlier
// kernel, profiles/r2_trifind_hub_sweep.txt); a multiple of 64, at most nvert
static int64_t g_last_hub = 0;
int64_t tri_last_hub_size() { return g_last_hub; }

int64_t tri_hub_size(int64_t nvert) {
  static const int64_t env = [] {
    const char* e = std::getenv("MRH_TRI_HUB");
    return e ? std::atoll(e) : int64_t(-1);
  }();
  int64_t want = env >= 0 ? env : std::min<int64_t>(nvert / 64, 524288);
  size_t free_b = 0, total_b = 0;
  if (env < 0 && hipMemGetInfo(&free_b, &total_b) == hipSuccess && free_b > 0) {
    if ((size_t)want * (size_t)want / 8 > free_b / 4) {  // blocks cached by the allocator count as free
      c10::hip::HIPCachingAllocator::emptyCache();
      if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) free_b = 0;  // then the hub budget stays as set above
    }
    while (want > 64 && (size_t)want * (size_t)want / 8 > free_b / 4) want /= 2;
  }
  int64_t K = std::min<int64_t>(std::max<int64_t>(want, 0), 524288);
  K = std::min<int64_t>(K, nvert) / 64 * 64;
  return K;
}

// dense core size: MRH_TRI_CORE ranks (default 0 = off), a multiple of 64, <= the hub set.
// Off by default: on RMAT-24 a core of 4 K-32 K ranks measured 351 / 350 /
// 348 / 359 ms against 351 ms without (profiles/r2_trifind_core_mfma.txt) —
// the hub kernel's time is in the sparse lower hub rows, not the dense core
int64_t tri_core_size(int64_t K) {
  static const int64_t env = [] {
    const char* e = std::getenv("MRH_TRI_CORE");
    return e ? std::atoll(e) : int64_t(0);
  }();
  return std::min<int64_t>(std::max<int64_t>(env, 0), K) / 64 * 64;
}

// triangles whose lowest vertex u is a core rank in [u0, u1): the core's
// oriented adjacency A (int8 0/1, top T ranks) gives |N+(u) ∩ N+(v)| =
// (A A^T)[u][v] for all core pairs at once on the matrix cores (hipBLASLt
// int8 GEMM, int32 accumulation: exact); the count is sum(A .* (A A^T)) over
// the rows, in row blocks that bound the int32 product
static int64_t tri_core_count(const at::Tensor& rowptr, const at::Tensor& col, int64_t cb, int64_t T, int64_t u0,
                              int64_t u1) {
  const at::Device dev = rowptr.device();
  at::Tensor A = at::empty({T, T}, opt(dev, at::kChar));
  k::tri_core_build(P0<int64_t>(rowptr), P0<uint32_t>(col), cb, T, P0<int8_t>(A), cur());
  const int64_t ra = std::max<int64_t>(u0 - cb, 0), rb = std::min<int64_t>(u1 - cb, T);
  at::Tensor At = A.t();
  at::Tensor tot = at::zeros({}, opt(dev, at::kLong));
  const int64_t RB = std::max<int64_t>(64, ((int64_t)1 << 28) / T) / 64 * 64;  // <= 1 GiB of int32 per block
  // rows in multiples of 64 (the GEMM's shape rules); rows outside [ra, rb) masked
  for (int64_t r = ra / 64 * 64; r < rb; r += RB) {
    const int64_t n = std::min<int64_t>(RB, T - r);
    at::Tensor Ar = A.narrow(0, r, n);
    at::Tensor C = at::_int_mm(Ar, At);
    at::Tensor M = Ar;
    if (r < ra || r + n > rb) {
      M = Ar.clone();
      if (r < ra) M.narrow(0, 0, ra - r).zero_();
      if (r + n > rb) M.narrow(0, rb - r, r + n - rb).zero_();
    }
    tot += at::mul(C, M).sum(at::kLong);
  }
  return tot.item<int64_t>();
}

// hub-row kernel (MRH_TRI_HUB_KERNEL): "bitmap" (default; AND/popcount of
// bitmap rows), "pull" (rows grouped by the middle vertex, streamed row tails
// against an LDS table of N+(v): 40 G element tests on RMAT-24, 364 ms vs
// 231 ms, profiles/r3_trifind_pull.txt) or "lds" (LDS bitmap of N+(u),
// streamed N+(v))
static int tri_hub_mode() {
  static const int m = [] {
    const char* e = std::getenv("MRH_TRI_HUB_KERNEL");
    if (e && std::string(e) == "pull") return 0;
    if (!e || !*e || std::string(e) == "bitmap" || std::string(e) == "lds") return 1;  // tri_hub_count picks
    throw std::runtime_error("MRH_TRI_HUB_KERNEL must be pull, bitmap or lds");
  }();
  return m;
}

// the hub rows [ua, ub) counted v-major (tri.hip k_tri_hub_pull): their edges
// sorted by destination give every hub v its in-edges (u, v); each in-edge's
// row tail past v is streamed against N+(v)
static void tri_hub_pull_count(const at::Tensor& rowptr, const at::Tensor& col, const at::Tensor& okeys, int64_t hb,
                               int64_t K, int64_t ua, int64_t ub, const at::Tensor& H, at::Tensor& tot) {
  if (ub <= ua || K <= 0) return;
  const at::Device dev = rowptr.device();
  const hipStream_t s = cur();
  const int64_t ea = rowptr[ua].item<int64_t>(), n = rowptr[ub].item<int64_t>() - ea;
  if (n <= 0) return;
  at::Tensor tk = at::empty({n}, opt(dev, at::kLong));
  at::Tensor endx = at::empty({n}, opt(dev, at::kInt));
  k::tri_hub_pull_prep(P0<uint32_t>(col), P0<uint64_t>(okeys), P0<int64_t>(rowptr), hb, ea, n, P0<uint64_t>(tk),
                       P0<uint32_t>(endx), s);
  int kb = 1;
  while ((int64_t(1) << kb) < K) ++kb;
  at::Tensor tks = radix_sort_keys(tk, 32, 32 + kb);  // keys-only: the edge index rides in the low word
  tk = at::Tensor();
  at::Tensor tptr = at::empty({K + 1}, opt(dev, at::kLong));
  k::tri_rowptr(P0<uint64_t>(tks), n, K, P0<int64_t>(tptr), s);
  at::Tensor np = at::empty({K}, opt(dev, at::kLong));
  k::tri_hub_pull_npieces(P0<int64_t>(tptr), P0<int64_t>(rowptr), hb, K, P0<int64_t>(np), s);
  at::Tensor off = exclusive_scan(np).to(at::kLong).contiguous();  // K + 1 entries, off[K] = item count
  const int64_t cap = k::tri_hub_pull_max_items(n, K);
  at::Tensor items = at::empty({cap}, opt(dev, at::kLong)), big = at::empty({cap}, opt(dev, at::kLong));
  at::Tensor nbig = at::empty({1}, opt(dev, at::kInt));
  k::tri_hub_pull(P0<int64_t>(rowptr), P0<uint32_t>(col), hb, K, ea, P0<uint64_t>(tks), P0<int64_t>(tptr),
                  P0<uint32_t>(endx), P0<int64_t>(off), P0<uint64_t>(items), P0<uint64_t>(big), P0<unsigned int>(nbig),
                  P0<uint64_t>(H), P0<unsigned long long>(tot), s);
}

int64_t tri_count(const at::Tensor& rowptr, const at::Tensor& col, const at::Tensor& okeys, int64_t e0, int64_t e1) {
  e1 = std::min<int64_t>(e1, okeys.numel());
  if (e1 <= e0) return 0;
  if (okeys.is_cuda()) {
    // vertex-centric: this call owns the vertices whose first out-edge lies in [e0, e1)
    const int64_t m = okeys.numel(), nvert = rowptr.numel() - 1;
    auto src = [&](int64_t e) { return (int64_t)((uint64_t)okeys[e].item<int64_t>() >> 32); };
    const int64_t u0 = e0 == 0 ? 0 : src(e0 - 1) + 1;
    const int64_t u1 = e1 == m ? nvert : src(e1 - 1) + 1;
    return tri_count_range(rowptr, col, u0, u1, okeys);
  }
  const int64_t* rp = P0<int64_t>(rowptr);
  const int32_t* c = P0<int32_t>(col);
  const uint64_t* k = P0<uint64_t>(okeys);
  int64_t n = 0;
  for (int64_t e = e0; e < e1; ++e) n += intersect_host<false>(rp, c, (uint32_t)(k[e] >> 32), (uint32_t)k[e], nullptr);
  return n;
}

int64_t tri_count_range(const at::Tensor& rowptr, const at::Tensor& col, int64_t u0, int64_t u1,
                        const at::Tensor& okeys) {
  if (u1 <= u0) return 0;
  if (!rowptr.is_cuda()) return tri_count_rows(rowptr, col, u0, u1);
  {
    const int64_t nvert = rowptr.numel() - 1;
    at::Tensor tot = at::zeros({1}, opt(rowptr.device(), at::kLong));
    // the top-K ranks (hubs) go to the bitmap kernel, the rest to the hash kernels
    const int64_t K = tri_hub_size(nvert);
    g_last_hub = K;
    const int64_t hb = nvert - K;
    const int64_t uh = K ? std::max(u0, std::min(u1, hb)) : u1;
    // the top T of the hubs (the dense core) go to the matrix cores instead
    const int64_t T = K ? tri_core_size(K) : 0, cb = nvert - T;
    at::Tensor H;
    if (K) {
      // the bitmaps serve both the hub kernel and the hub probes of the hash kernels
      H = at::empty({K * (K / 64)}, opt(rowptr.device(), at::kLong));
      const int64_t ua = std::max(u0, hb), ub = std::max(std::min(u1, cb), hb);
      const bool pull = tri_hub_mode() == 0;
      // pull: tri_hub_count only builds the bitmaps (an empty row range)
      k::tri_hub_count(P0<int64_t>(rowptr), P0<uint32_t>(col), hb, K, ua, pull ? ua : ub, P0<uint64_t>(H),
                       P0<unsigned long long>(tot), cur());
      if (pull && !okeys.defined())
        throw std::runtime_error("MRH_TRI_HUB_KERNEL=pull needs the whole oriented edge list (one rank)");
      if (pull) tri_hub_pull_count(rowptr, col, okeys, hb, K, ua, ub, H, tot);
    }
    int64_t ncore = 0;
    if (T && u1 > cb) ncore = tri_core_count(rowptr, col, cb, T, std::max(u0, cb), u1);
    if (uh > u0) {
      at::Tensor big = at::empty({2 * std::max<int64_t>(uh - u0, 1)}, opt(rowptr.device(), at::kInt));
      at::Tensor nbig = at::zeros({2}, opt(rowptr.device(), at::kInt));
      k::tri_count_hash(P0<int64_t>(rowptr), P0<uint32_t>(col), u0, uh, P0<uint32_t>(big), P0<uint32_t>(nbig),
                        P0<unsigned long long>(tot), cur(), K ? P0<uint64_t>(H) : nullptr, hb, K);
    }
    return tot.item<int64_t>() + ncore;
  }
}

int64_t tri_count_rows(const at::Tensor& rowptr, const at::Tensor& col, int64_t u0, int64_t u1) {
  if (u1 <= u0) return 0;
  if (rowptr.is_cuda()) {
    const at::Device dev = rowptr.device();
    at::Tensor tot = at::zeros({1}, opt(dev, at::kLong));
    at::Tensor big = at::empty({2 * std::max<int64_t>(u1 - u0, 1)}, opt(dev, at::kInt));
    at::Tensor nbig = at::zeros({2}, opt(dev, at::kInt));
    k::tri_count_hash(P0<int64_t>(rowptr), P0<uint32_t>(col), u0, u1, P0<uint32_t>(big), P0<uint32_t>(nbig),
                      P0<unsigned long long>(tot), cur());
    return tot.item<int64_t>();
  }
  at::Tensor rp_h = rowptr.to(at::kCPU).contiguous(), col_h = col.to(at::kCPU).contiguous();
  const int64_t* rp = P0<int64_t>(rp_h);
  const int32_t* c = P0<int32_t>(col_h);
  int64_t n = 0;
  for (int64_t u = u0; u < u1; ++u)
    for (int64_t e = rp[u]; e < rp[u + 1]; ++e) n += intersect_host<false>(rp, c, (uint32_t)u, (uint32_t)c[e], nullptr);
  return n;
}

at::Tensor tri_list(const at::Tensor& rowptr, const at::Tensor& col, const at::Tensor& okeys, int64_t e0, int64_t e1) {
  e1 = std::min<int64_t>(e1, okeys.numel());
  const at::Device dev = okeys.device();
  if (e1 <= e0) return at::empty({0, 3}, opt(dev, at::kLong));
  if (okeys.is_cuda()) {
    at::Tensor cnt = at::empty({e1 - e0}, opt(dev, at::kInt));
    at::Tensor tot = at::zeros({1}, opt(dev, at::kLong));
    k::tri_count(P0<int64_t>(rowptr), P0<uint32_t>(col), P0<uint64_t>(okeys), e0, e1, P0<uint32_t>(cnt),
                 P0<unsigned long long>(tot), cur());
    at::Tensor off = exclusive_scan(cnt);
    const int64_t T = off[e1 - e0].item<int64_t>();
    at::Tensor out = at::empty({T, 3}, opt(dev, at::kLong));
    if (T) k::tri_emit(P0<int64_t>(rowptr), P0<uint32_t>(col), P0<uint64_t>(okeys), e0, e1, P0<int64_t>(off),
                       P0<uint64_t>(out), cur());
    return out;
  }
  const int64_t* rp = P0<int64_t>(rowptr);
  const int32_t* c = P0<int32_t>(col);
  const uint64_t* k = P0<uint64_t>(okeys);
  std::vector<int64_t> v;
  for (int64_t e = e0; e < e1; ++e) intersect_host<true>(rp, c, (uint32_t)(k[e] >> 32), (uint32_t)k[e], &v);
  return at::from_blob(v.data(), {(int64_t)v.size() / 3, 3}, opt(at::kCPU, at::kLong)).clone();
}

}  // namespace mrh
