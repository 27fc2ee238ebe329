// Exact hash-dictionary group-by for gfx950: the device side of HashDict /
// GroupIndex (csrc/engine/grouper.h), i.e. MR-MPI's convert (reference
// src/keymultivalue.cpp:645-789 kv2unique: a hash table of the unique keys)
// done in one streaming pass over the pairs — part by part while the KV is
// still being produced (GroupIndex), or over a whole KV (convert of a KV with
// few distinct keys: words, hot keys).
//
// Table (power-of-two capacity, <= 50 % load by construction):
//   slots[cap] : 32-byte records {u64 key hash (0 = empty; a zero hash is
//                stored as 1), i32 group id + 1 (0 until published), i32 key
//                length, the key's first 16 bytes}
//   rep[g]     : i64 row of group g's first key (-1 until published)
//   ghash[g]   : u64 hash of group g
//   gcount[g]  : u64 pairs in group g (optional)
//   ctr        : [groups, collisions, rows left unassigned, full flag]
// k_dict_insert, per pair: lookup3 hashlittle2 of the key bytes (or a given
// hash), probe; an empty slot is claimed with one 64-bit CAS, the claimer
// takes the next group id and fills the record, then publishes the id
// (release). The other pairs of that hash compare their key with the
// record's bytes (and, past 16 bytes, with the group's first key): grouping
// is exact, a true 64-bit collision is counted and the host falls back to
// the sort path with exact regrouping. Claims and waits are separate phases
// of the loop body, so every lane of a wave publishes before any lane waits.
// Pair counts per group are pre-aggregated in a direct-mapped LDS cache (the
// first group of a block to use an entry keeps it: the 13.7 % word of a Zipf
// text is one LDS counter per block, not one global atomic per occurrence).
// Past `limit` groups no new slot is claimed: the rows left are marked
// unassigned and counted, the host grows the table and runs the insert again
// over them (retry mode).
#include <algorithm>

#include "common.h"
#include "launch.h"

namespace mrh {
namespace k {
namespace {

using dev::rot32;  // lookup3's mix / final macros

constexpr int NT = 256;
constexpr int32_t NONE = -1;

unsigned blocks_for(int64_t n) {
  int64_t b = (n + NT - 1) / NT;
  return (unsigned)(b < 1 ? 1 : (b > (1 << 20) ? (1 << 20) : b));
}

__device__ __forceinline__ uint64_t nz(uint64_t h) { return h ? h : 1ull; }
// slot of a hash: the low half of lookup3's hashlittle2 is its "b" word, the
// high half "c"; xor-folding keeps both in play for small tables
__device__ __forceinline__ uint64_t home(uint64_t h, uint64_t mask) { return (h ^ (h >> 32)) & mask; }

// key bytes of row r
struct Keys {
  const uint8_t* d;
  const int64_t* off;  // null: fixed width w
  int w;
  __device__ __forceinline__ const uint8_t* at(int64_t r) const { return off ? d + off[r] : d + r * (int64_t)w; }
  __device__ __forceinline__ int64_t len(int64_t r) const { return off ? off[r + 1] - off[r] : (int64_t)w; }
};

// the first min(len, 16) bytes at p as 4 little-endian words, zero past the
// end, from aligned dword loads that each hold at least one byte of the key
// (never past the key's last dword: no read beyond an allocation)
__device__ __forceinline__ void load_key16(const uint8_t* p, int64_t len, uint32_t w[4]) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  const uint32_t* q = reinterpret_cast<const uint32_t*>(a & ~uintptr_t(3));
  const uint32_t r = (uint32_t)(a & 3);
  const int nb = len < 16 ? (int)len : 16;
  const int nd = (int)((r + nb + 3) >> 2);
  uint32_t d[5];
#pragma unroll
  for (int j = 0; j < 5; ++j) d[j] = j < nd ? q[j] : 0u;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    uint32_t v = r ? __builtin_amdgcn_alignbyte(d[j + 1], d[j], r) : d[j];
    const int valid = nb - 4 * j;
    if (valid <= 0) v = 0;
    else if (valid < 4) v &= (1u << (8 * valid)) - 1u;
    w[j] = v;
  }
}

// hash64 (hashfn.h: lookup3 hashlittle2, seeds 0x9e3779b9 / 0x7f4a7c15) of
// a key of <= 16 bytes from its zero-padded words — lookup3's byte-wise tail
// is the same as adding zero-padded little-endian words
__device__ __forceinline__ uint64_t hash64_words(const uint32_t w[4], int64_t len) {
  uint32_t a, b, c;
  a = b = c = 0xdeadbeefu + (uint32_t)len + 0x9e3779b9u;
  c += 0x7f4a7c15u;
  if (len == 0) return ((uint64_t)c << 32) | b;
  a += w[0];
  b += w[1];
  c += w[2];
  if (len > 12) {
    MRH_L3_MIX(a, b, c);
    a += w[3];
  }
  MRH_L3_FINAL(a, b, c);
  return ((uint64_t)c << 32) | b;
}

__device__ __forceinline__ uint64_t ld_l2_u64(const void* p) {
  return __hip_atomic_load(reinterpret_cast<const unsigned long long*>(p), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}

// k_dict_insert: see the file comment. Slot records are 32 bytes: the probe
// reads {hash, gid+1, len} in one 16-byte load and the key's first 16 bytes
// from the same cache line; gid+1 is 0 until the claimer publishes it
// (release, after len / key / rep / ghash), and a published value is final —
// a record whose header shows it published was read from a line filled after
// the publication, key bytes included. Only an unpublished header, or a
// mismatch (possibly a stale line), goes to L2 again.
__global__ __launch_bounds__(NT) void k_dict_insert(Keys K, const uint64_t* __restrict__ h, int64_t n, int64_t row0,
                                                   DictTable T, int32_t* __restrict__ gid, int retry) {
  unsigned long long bad = 0, left = 0;
  const int64_t stride = (int64_t)gridDim.x * NT;
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i - threadIdx.x < n; i += stride) {
    const int64_t row = row0 + i;
    bool live = i < n;
    if (live && retry) live = gid[row] == NONE;
    unsigned long long hv = 0;
    const uint8_t* p = nullptr;
    int64_t len = 0;
    uint32_t w[4] = {0, 0, 0, 0};
    uint64_t s = 0;
    uint4 hdr = make_uint4(0, 0, 0, 0);
    int state = 0;  // 0 idle, 1 matched, 2 claimed, 3 unassigned
    if (live) {
      p = K.at(row);
      len = K.len(row);
      load_key16(p, len, w);
      if (h) {
        hv = nz(h[i]);
      } else if (len <= 16) {
        hv = nz(hash64_words(w, len));
      } else {
        uint32_t c = 0x9e3779b9u, b = 0x7f4a7c15u;
        dev::lookup3_wide(p, len, &c, &b);
        hv = nz(((uint64_t)c << 32) | b);
      }
      s = home(hv, T.mask);
      for (uint64_t probe = 0;; ++probe) {
        // a slot's hash only ever goes 0 -> hash once: a stale 0 costs the CAS
        // below (which returns the live value), a non-zero value is final
        hdr = *reinterpret_cast<const uint4*>(&T.slots[s]);
        unsigned long long v = ((unsigned long long)hdr.y << 32) | hdr.x;
        if (v == 0) {
          if (__hip_atomic_load(&T.ctr[3], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
            state = 3;  // full: no new groups
            break;
          }
          v = atomicCAS(&T.slots[s].hash, 0ull, hv);
          if (v == 0) {
            state = 2;
            break;
          }
          hdr.z = 0;  // claimed by another pair just now: not published yet
        }
        if (v == hv) {
          state = 1;
          break;
        }
        s = (s + 1) & T.mask;
        if (probe >= T.mask) {
          state = 3;
          break;
        }
      }
    }
    int32_t g = NONE;
    // phase 2: claimers publish (before any lane of the wave waits below)
    if (state == 2) {
      g = (int32_t)atomicAdd(&T.ctr[0], 1ull);
      DictSlot& sl = T.slots[s];
      sl.len = (int32_t)len;
      *reinterpret_cast<uint4*>(sl.key) = make_uint4(w[0], w[1], w[2], w[3]);
      T.rep[g] = row;
      T.ghash[g] = hv;
      __hip_atomic_store(&sl.gid1, g + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      if ((int64_t)g + 1 >= T.limit) __hip_atomic_store(&T.ctr[3], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // phase 3: the others read the published group and check the key bytes
    if (state == 1) {
      const DictSlot& sl = T.slots[s];
      bool fresh = false;  // header read from L2 (the key line may still be stale in L1)
      while (hdr.z == 0) {
        __builtin_amdgcn_s_sleep(1);
        const uint64_t gl = ld_l2_u64(&sl.gid1);
        hdr.z = (uint32_t)gl;
        hdr.w = (uint32_t)(gl >> 32);
        fresh = true;
      }
      g = (int32_t)hdr.z - 1;
      uint4 kk = fresh ? make_uint4(0, 0, 0, 0) : *reinterpret_cast<const uint4*>(sl.key);
      bool same = !fresh && (int64_t)(int32_t)hdr.w == len && kk.x == w[0] && kk.y == w[1] && kk.z == w[2] &&
                  kk.w == w[3];
      if (!same) {  // from L2: a stale line, or a true collision
        const uint64_t k01 = ld_l2_u64(&sl.key[0]), k23 = ld_l2_u64(&sl.key[2]);
        const uint64_t gl = ld_l2_u64(&sl.gid1);
        same = (int64_t)(int32_t)(gl >> 32) == len && (uint32_t)k01 == w[0] && (uint32_t)(k01 >> 32) == w[1] &&
               (uint32_t)k23 == w[2] && (uint32_t)(k23 >> 32) == w[3];
      }
      if (same && len > 16) {  // the bytes past the first 16 against the group's first key
        int64_t b = T.rep[g];
        if (b < 0) b = (int64_t)ld_l2_u64(&T.rep[g]);
        same = dev::bytes_equal(p + 16, K.at(b) + 16, len - 16);
      }
      if (!same) ++bad;
    }
    if (state == 3) ++left;
    if (live) gid[row] = g;
  }
  bad = dev::wave_sum(bad);
  left = dev::wave_sum(left);
  if (dev::lane_id() == 0) {
    if (bad) atomicAdd(&T.ctr[1], bad);
    if (left) atomicAdd(&T.ctr[2], left);
  }
}

// Pairs per group without a global atomic per pair (scattered global atomics
// run at the memory side, ~17x below streaming: a Zipf text's tail words
// would cost more than the whole insert): groups [w0, w0 + HW) are counted in
// one LDS histogram per block (u32, 128 KiB: one 1024-thread block per CU),
// written as a per-block partial row; k_dict_hist_reduce sums the rows. One
// pass per window of 32k groups over the (streamed, 4-byte) group ids.
constexpr int HW = 32768;
constexpr int HNT = 1024;
constexpr int kDictHistRows = 256;  // partial rows (blocks) at most

__global__ __launch_bounds__(HNT) void k_dict_hist(const int32_t* __restrict__ gid, int64_t n, int64_t w0,
                                                  int64_t wlen, uint32_t* __restrict__ partial) {
  __shared__ uint32_t hist[HW];
  for (int j = threadIdx.x; j < HW; j += HNT) hist[j] = 0;
  __syncthreads();
  const int64_t n4 = n >> 2;
  const int4* g4 = reinterpret_cast<const int4*>(gid);
  auto add = [&](int32_t g) {
    const uint64_t d = (uint64_t)((int64_t)g - w0);
    if (d < (uint64_t)wlen) atomicAdd(&hist[d], 1u);
  };
  for (int64_t i = (int64_t)blockIdx.x * HNT + threadIdx.x; i < n4; i += (int64_t)gridDim.x * HNT) {
    const int4 v = g4[i];
    add(v.x);
    add(v.y);
    add(v.z);
    add(v.w);
  }
  if (blockIdx.x == 0)
    for (int64_t i = (n4 << 2) + threadIdx.x; i < n; i += HNT) add(gid[i]);
  __syncthreads();
  uint32_t* row = partial + (int64_t)blockIdx.x * HW;
  for (int j = threadIdx.x; j < wlen; j += HNT) row[j] = hist[j];
}

__global__ __launch_bounds__(NT) void k_dict_hist_reduce(const uint32_t* __restrict__ partial, int rows,
                                                        int64_t w0, int64_t wlen, unsigned long long* __restrict__ cnt) {
  const int64_t j = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (j >= wlen) return;
  unsigned long long s = 0;
  for (int r = 0; r < rows; ++r) s += partial[(int64_t)r * HW + j];
  cnt[w0 + j] = s;
}

// move every slot record into a larger table (group ids are kept)
__global__ __launch_bounds__(NT) void k_dict_rehash(const DictSlot* __restrict__ os, int64_t ocap,
                                                   DictSlot* __restrict__ ns, uint64_t nmask) {
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < ocap; i += (int64_t)gridDim.x * NT) {
    const DictSlot v = os[i];
    if (!v.hash) continue;
    uint64_t s = home(v.hash, nmask);
    while (atomicCAS(&ns[s].hash, 0ull, v.hash) != 0ull) s = (s + 1) & nmask;
    ns[s].gid1 = v.gid1;
    ns[s].len = v.len;
    *reinterpret_cast<uint4*>(ns[s].key) = *reinterpret_cast<const uint4*>(v.key);
  }
}

// strided sample of key hashes (the host counts distinct ones to size a table)
__global__ __launch_bounds__(NT) void k_dict_sample(Keys K, int64_t n, int64_t m, uint64_t* __restrict__ out) {
  const int64_t j = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (j >= m) return;
  const int64_t r = (int64_t)((__uint128_t)j * (uint64_t)n / (uint64_t)m);
  uint32_t c = 0x9e3779b9u, b = 0x7f4a7c15u;
  dev::lookup3_wide(K.at(r), K.len(r), &c, &b);
  out[j] = nz(((uint64_t)c << 32) | b);
}

// per-group counts in rank order: cnt[j] = gcount[order[j]]
__global__ __launch_bounds__(NT) void k_dict_ranked_counts(const uint32_t* __restrict__ order, int64_t m,
                                                          const unsigned long long* __restrict__ gcount,
                                                          int64_t* __restrict__ cnt) {
  for (int64_t j = (int64_t)blockIdx.x * NT + threadIdx.x; j < m; j += (int64_t)gridDim.x * NT)
    cnt[j] = (int64_t)gcount[order[j]];
}

// variable column append: the part's offsets shifted by the arena's byte
// end (the host's running sum of part sizes: parts carry no slack bytes,
// koff[n] == kdata.numel(), the same convention as concat())
__global__ __launch_bounds__(NT) void k_grp_append_off(const int64_t* __restrict__ poff, int64_t n, int64_t base,
                                                      int64_t* __restrict__ aoff) {
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i <= n; i += (int64_t)gridDim.x * NT)
    aoff[i] = poff[i] + base;
}

__global__ __launch_bounds__(NT) void k_grp_rank(const uint32_t* __restrict__ order, int64_t m,
                                                const int64_t* __restrict__ rep, uint32_t* __restrict__ rank,
                                                uint32_t* __restrict__ heads) {
  for (int64_t j = (int64_t)blockIdx.x * NT + threadIdx.x; j < m; j += (int64_t)gridDim.x * NT) {
    const uint32_t g = order[j];
    rank[g] = (uint32_t)j;
    heads[j] = (uint32_t)rep[g];
  }
}

__global__ __launch_bounds__(NT) void k_grp_pairkey(const int32_t* __restrict__ gid, int64_t n,
                                                   const uint32_t* __restrict__ rank, uint64_t* __restrict__ key) {
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT)
    key[i] = rank[gid[i]];
}

// seg[r] = first sorted position of rank r (sorted ranks are dense 0..m-1)
__global__ __launch_bounds__(NT) void k_grp_seg(const uint64_t* __restrict__ sk, int64_t n, int64_t m,
                                               int64_t* __restrict__ seg) {
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) {
    const uint64_t r = sk[i];
    if (i == 0 || sk[i - 1] != r) seg[r] = i;
    if (i == n - 1) seg[m] = n;
  }
}

}  // namespace

void dict_insert(const uint8_t* kd, const int64_t* koff, int kw, const uint64_t* h, int64_t n, int64_t row0,
                 const DictTable& t, int32_t* gid, bool retry, hipStream_t s) {
  if (n <= 0) return;
  check_arg(t.mask > 0 && ((t.mask + 1) & t.mask) == 0, "dict_insert: table capacity must be a power of two");
  check_arg(!retry || gid, "dict_insert: retry needs the row group ids");
  Keys K{kd, koff, kw};
  // a resident grid (8 blocks of 256 per CU) striding over the pairs: the
  // LDS counters of a block then cover ~n/(8 CUs) pairs before one flush
  static int cus[64] = {0};
  int dev = 0;
  MRH_HIP(hipGetDevice(&dev));
  if (dev >= 0 && dev < 64 && cus[dev] == 0) MRH_HIP(hipDeviceGetAttribute(&cus[dev], hipDeviceAttributeMultiprocessorCount, dev));
  const int ncu = dev >= 0 && dev < 64 && cus[dev] > 0 ? cus[dev] : 256;
  const int64_t grid = std::min<int64_t>((n + NT - 1) / NT, (int64_t)ncu * 8);
  hipLaunchKernelGGL(k_dict_insert, dim3((unsigned)std::max<int64_t>(grid, 1)), dim3(NT), 0, s, K, h, n, row0, t, gid,
                     retry ? 1 : 0);
  MRH_CHECK_LAUNCH();
}

void dict_rehash(const DictSlot* old_slots, int64_t old_cap, DictSlot* new_slots, int64_t new_cap, hipStream_t s) {
  if (old_cap <= 0) return;
  check_arg(new_cap > 0 && (new_cap & (new_cap - 1)) == 0, "dict_rehash: capacity must be a power of two");
  hipLaunchKernelGGL(k_dict_rehash, dim3(blocks_for(old_cap)), dim3(NT), 0, s, old_slots, old_cap, new_slots,
                     (uint64_t)new_cap - 1);
  MRH_CHECK_LAUNCH();
}

void dict_sample(const uint8_t* kd, const int64_t* koff, int kw, int64_t n, int64_t m, uint64_t* out, hipStream_t s) {
  if (m <= 0 || n <= 0) return;
  Keys K{kd, koff, kw};
  hipLaunchKernelGGL(k_dict_sample, dim3((unsigned)((m + NT - 1) / NT)), dim3(NT), 0, s, K, n, m, out);
  MRH_CHECK_LAUNCH();
}

int64_t dict_counts_ws_elems() { return (int64_t)kDictHistRows * HW; }

void dict_counts(const int32_t* gid, int64_t n, int64_t m, uint64_t* cnt, uint32_t* partial, hipStream_t s) {
  if (m <= 0) return;
  static int cus[64] = {0};
  int dev = 0;
  MRH_HIP(hipGetDevice(&dev));
  if (dev >= 0 && dev < 64 && cus[dev] == 0) MRH_HIP(hipDeviceGetAttribute(&cus[dev], hipDeviceAttributeMultiprocessorCount, dev));
  const int ncu = dev >= 0 && dev < 64 && cus[dev] > 0 ? cus[dev] : 256;
  const int rows = (int)std::max<int64_t>(
      1, std::min<int64_t>(std::min(ncu, kDictHistRows), (n + 4LL * HNT - 1) / (4LL * HNT)));
  for (int64_t w0 = 0; w0 < m; w0 += HW) {
    const int64_t wlen = std::min<int64_t>(HW, m - w0);
    if (n > 0) {
      hipLaunchKernelGGL(k_dict_hist, dim3(rows), dim3(HNT), 0, s, gid, n, w0, wlen, partial);
      MRH_CHECK_LAUNCH();
    } else {
      MRH_HIP(hipMemsetAsync(partial, 0, (size_t)rows * HW * sizeof(uint32_t), s));
    }
    hipLaunchKernelGGL(k_dict_hist_reduce, dim3((unsigned)((wlen + NT - 1) / NT)), dim3(NT), 0, s, partial, rows, w0,
                       wlen, (unsigned long long*)cnt);
    MRH_CHECK_LAUNCH();
  }
}

void dict_ranked_counts(const uint32_t* order, int64_t m, const uint64_t* gcount, int64_t* cnt, hipStream_t s) {
  if (m <= 0) return;
  hipLaunchKernelGGL(k_dict_ranked_counts, dim3(blocks_for(m)), dim3(NT), 0, s, order, m,
                     (const unsigned long long*)gcount, cnt);
  MRH_CHECK_LAUNCH();
}

void grp_append_off(const int64_t* poff, int64_t n, int64_t base, int64_t* aoff, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_grp_append_off, dim3(blocks_for(n + 1)), dim3(NT), 0, s, poff, n, base, aoff);
  MRH_CHECK_LAUNCH();
}

void grp_rank(const uint32_t* order, int64_t m, const int64_t* rep, uint32_t* rank, uint32_t* heads, hipStream_t s) {
  if (m <= 0) return;
  hipLaunchKernelGGL(k_grp_rank, dim3(blocks_for(m)), dim3(NT), 0, s, order, m, rep, rank, heads);
  MRH_CHECK_LAUNCH();
}

void grp_pairkey(const int32_t* gid, int64_t n, const uint32_t* rank, uint64_t* key, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_grp_pairkey, dim3(blocks_for(n)), dim3(NT), 0, s, gid, n, rank, key);
  MRH_CHECK_LAUNCH();
}

void grp_seg(const uint64_t* sorted_rank, int64_t n, int64_t m, int64_t* seg, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_grp_seg, dim3(blocks_for(n)), dim3(NT), 0, s, sorted_rank, n, m, seg);
  MRH_CHECK_LAUNCH();
}

}  // namespace k
}  // namespace mrh
