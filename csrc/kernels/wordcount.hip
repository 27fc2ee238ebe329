// In-mapper combining word count for gfx950: tokenize + count in one pass.
//
// The reference's word count (examples/wordfreq.cpp:104-130,
// oink/map_read_words.cpp:14-30) strtok()s every word on the host and
// kv->add()s it; the combiner (MR-MPI compress, src/mapreduce.cpp:749-851)
// would then convert + reduce the full KV. Materialising one KV per word costs
// a key-arena copy, a 64-bit hash radix sort and an exact-key verification
// over every occurrence (143 M words per GiB of Zipf text). Here the map
// itself combines: each word is hashed once and counted in a device hash
// table, so only (distinct word, count) pairs ever become KVs.
//
//   LDS level   each workgroup tokenizes 16 KiB of text (4 sub-tiles of 16 B
//               per lane, the tokenizer's word-start bitmask) into a 2048-entry
//               LDS table (64-bit ds_cmpst claims, LDS atomic counts). Zipf
//               hot words collapse here, so the global table sees each
//               distinct word once per workgroup instead of once per use.
//   global      open-addressing table in HBM: slot = [tag32 | loc32],
//               count[slot] += c with device atomics. loc is the word's
//               offset in the current text chunk (words claimed in this
//               chunk) or, with bit 31 set, in the key arena (words from
//               earlier chunks, moved there by k_wc_migrate after each chunk).
//               Every match is EXACT: tag equality is followed by a byte
//               compare against the stored word — no hash-equality grouping.
//   bounds      the host guarantees before each chunk that the table keeps
//               >= 25 % free slots even if every word of the chunk is new
//               (growing + rehashing otherwise), so probing always ends, and
//               that the arena can take every new word; nothing is dropped.
#include "common.h"
#include "launch.h"
#include <cstdio>
#include <cstdlib>

namespace mrh {
namespace k {
namespace {

constexpr int NT = 256;
constexpr int SUB = NT * 16;          // 4 KiB per sub-tile (16 B per lane)
constexpr uint32_t ARENA_BIT = 0x80000000u;

__device__ __forceinline__ bool is_ws(uint32_t c) {
  return c == ' ' || c == '\t' || c == '\n' || c == '\f' || c == '\r' || c == 0;
}

__device__ __forceinline__ uint32_t word_start_mask(const uint8_t* text, int64_t p, int64_t n) {
  uint4 a = *reinterpret_cast<const uint4*>(text + p);
  uint32_t prev = (p == 0) ? 0u : (uint32_t)text[p - 1];
  uint32_t w[4] = {a.x, a.y, a.z, a.w};
  uint32_t m = 0;
  bool prev_ws = is_ws(prev);
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    uint32_t c = (w[k >> 2] >> (8 * (k & 3))) & 0xffu;
    bool ws = is_ws(c) | (p + k >= n);
    m |= (uint32_t)(!ws && prev_ws) << k;
    prev_ws = ws;
  }
  return m;
}

__device__ __forceinline__ int64_t word_len(const uint8_t* t, int64_t a, int64_t n) {
  int64_t j = a;
  while (j < n && !is_ws(t[j])) ++j;
  return j - a;
}

__device__ __forceinline__ uint64_t word_hash(const uint8_t* w, int64_t len) {
  uint32_t c = 0x9e3779b9u, b = 0x7f4a7c15u;
  dev::lookup3_wide(w, len, &c, &b);
  return ((uint64_t)c << 32) | b;
}

// is the stored word at `loc` (text chunk of n bytes, or NUL-terminated in the
// arena) equal to w[0..len)? Reads stop at the first mismatch, so an arena
// read never passes the stored word's NUL and a text read never passes n.
__device__ __forceinline__ bool word_eq(const uint8_t* w, int64_t len, const uint8_t* text, int64_t n,
                                        const uint8_t* arena, uint32_t loc) {
  if (loc & ARENA_BIT) {
    const uint8_t* s = arena + (loc & ~ARENA_BIT);
    for (int64_t i = 0; i < len; ++i)
      if (s[i] != w[i]) return false;
    return s[len] == 0;
  }
  if ((int64_t)loc + len > n) return false;
  const uint8_t* s = text + loc;
  for (int64_t i = 0; i < len; ++i)
    if (s[i] != w[i]) return false;
  return (int64_t)loc + len == n || is_ws(s[len]);
}

struct Table {
  unsigned long long* slots;
  uint32_t* counts;
  uint64_t mask;
  int32_t* newlist;            // slots claimed during this chunk
  unsigned long long* ctr;     // [0] used slots, [1] arena bytes
  unsigned long long used0;    // used slots at the start of this chunk
  const uint8_t* arena;
};

__device__ void g_insert(const Table& T, const uint8_t* text, int64_t n, uint32_t pos, int64_t len, uint64_t h,
                         uint32_t cnt) {
  const uint32_t tag = (uint32_t)(h >> 32) | 1u;
  const unsigned long long mine = ((unsigned long long)tag << 32) | pos;
  uint64_t slot = h & T.mask;
  for (;;) {
    unsigned long long v = __hip_atomic_load(&T.slots[slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (v == 0) {
      v = atomicCAS(&T.slots[slot], 0ull, mine);
      if (v == 0) {
        atomicAdd(&T.counts[slot], cnt);
        const unsigned long long i = atomicAdd(&T.ctr[0], 1ull) - T.used0;
        T.newlist[i] = (int32_t)slot;
        return;
      }
    }
    if ((uint32_t)(v >> 32) == tag && word_eq(text + pos, len, text, n, T.arena, (uint32_t)v)) {
      atomicAdd(&T.counts[slot], cnt);
      return;
    }
    slot = (slot + 1) & T.mask;
  }
}

// SUBS sub-tiles (4 KiB each) of text per workgroup, LDS_N-entry LDS table,
// LDS_PROBES probes before a word is counted straight in the global table
template <int SUBS, int LDS_N, int LDS_PROBES>
__global__ __launch_bounds__(NT) void k_wc_count(const uint8_t* __restrict__ text, int64_t n, Table T) {
  __shared__ unsigned long long lkey[LDS_N];
  __shared__ uint32_t lcnt[LDS_N];
  for (int i = threadIdx.x; i < LDS_N; i += NT) {
    lkey[i] = 0;
    lcnt[i] = 0;
  }
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * (SUB * SUBS);
  for (int s = 0; s < SUBS; ++s) {
    const int64_t p = base + (int64_t)s * SUB + (int64_t)threadIdx.x * 16;
    uint32_t m = (p < n) ? word_start_mask(text, p, n) : 0u;
    while (m) {
      const int k = __ffs(m) - 1;
      m &= m - 1;
      const int64_t a = p + k;
      const int64_t len = word_len(text, a, n);
      const uint64_t h = word_hash(text + a, len);
      const uint32_t tag = (uint32_t)(h >> 32) | 1u;
      const unsigned long long mine = ((unsigned long long)tag << 32) | (uint32_t)a;
      uint32_t e = (uint32_t)((h ^ (h >> 29)) & (LDS_N - 1));
      bool done = false;
      for (int probe = 0; probe < LDS_PROBES && !done; ++probe) {
        unsigned long long v = lkey[e];
        if (v == 0) {
          v = atomicCAS(&lkey[e], 0ull, mine);
          if (v == 0) {
            atomicAdd(&lcnt[e], 1u);
            done = true;
            break;
          }
        }
        if ((uint32_t)(v >> 32) == tag && word_eq(text + a, len, text, n, T.arena, (uint32_t)v)) {
          atomicAdd(&lcnt[e], 1u);
          done = true;
          break;
        }
        e = (e + 1) & (LDS_N - 1);
      }
      if (!done) g_insert(T, text, n, (uint32_t)a, len, h, 1u);  // LDS table crowded: count globally
    }
  }
  __syncthreads();
  // flush the workgroup's partial counts into the global table
  for (int i = threadIdx.x; i < LDS_N; i += NT) {
    const uint32_t c = lcnt[i];
    if (!c) continue;
    const uint32_t pos = (uint32_t)lkey[i];
    const int64_t len = word_len(text, pos, n);
    g_insert(T, text, n, pos, len, word_hash(text + pos, len), c);
  }
}

// words claimed during the chunk move to the arena before the text buffer is reused
__global__ __launch_bounds__(NT) void k_wc_migrate(const uint8_t* __restrict__ text, int64_t n, Table T,
                                                  uint8_t* __restrict__ arena, int64_t max_new) {
  const int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x;
  const int64_t nnew = (int64_t)(__hip_atomic_load(&T.ctr[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - T.used0);
  if (i >= nnew || i >= max_new) return;
  const int32_t slot = T.newlist[i];
  const unsigned long long v = T.slots[slot];
  const uint32_t pos = (uint32_t)v;
  const int64_t len = word_len(text, pos, n);
  const unsigned long long dst = atomicAdd(&T.ctr[1], (unsigned long long)(len + 1));
  for (int64_t j = 0; j < len; ++j) arena[dst + j] = text[pos + j];
  arena[dst + len] = 0;
  T.slots[slot] = (v & 0xffffffff00000000ull) | ARENA_BIT | (uint32_t)dst;
}

// move every entry into a bigger table (all entries are arena-resident here)
__global__ __launch_bounds__(NT) void k_wc_rehash(const unsigned long long* __restrict__ old_slots,
                                                 const uint32_t* __restrict__ old_counts, int64_t old_cap,
                                                 const uint8_t* __restrict__ arena, unsigned long long* new_slots,
                                                 uint32_t* new_counts, uint64_t new_mask) {
  const int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (i >= old_cap) return;
  const unsigned long long v = old_slots[i];
  if (v == 0) return;
  const uint8_t* w = arena + ((uint32_t)v & ~ARENA_BIT);
  int64_t len = 0;
  while (w[len]) ++len;
  uint64_t slot = word_hash(w, len) & new_mask;
  while (atomicCAS(&new_slots[slot], 0ull, v) != 0ull) slot = (slot + 1) & new_mask;
  new_counts[slot] = old_counts[i];
}

// arena locations + lengths (incl. NUL) of the listed slots
__global__ __launch_bounds__(NT) void k_wc_keys(const unsigned long long* __restrict__ slots,
                                               const int64_t* __restrict__ idx, int64_t nk,
                                               const uint8_t* __restrict__ arena, int64_t* __restrict__ starts,
                                               int32_t* __restrict__ lens) {
  const int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (i >= nk) return;
  const uint32_t loc = (uint32_t)slots[idx[i]] & ~ARENA_BIT;
  int64_t len = 0;
  while (arena[loc + len]) ++len;
  starts[i] = loc;
  lens[i] = (int32_t)(len + 1);
}

Table make_table(void* slots, void* counts, int64_t cap, int32_t* newlist, void* ctr, uint64_t used0,
                 const uint8_t* arena) {
  Table T;
  T.slots = (unsigned long long*)slots;
  T.counts = (uint32_t*)counts;
  T.mask = (uint64_t)cap - 1;
  T.newlist = newlist;
  T.ctr = (unsigned long long*)ctr;
  T.used0 = used0;
  T.arena = arena;
  return T;
}

}  // namespace

template <int SUBS, int LDS_N, int PROBES>
void launch_count(const uint8_t* text, int64_t n, const Table& T, hipStream_t s) {
  const int64_t nb = (n + SUB * SUBS - 1) / (SUB * SUBS);
  hipLaunchKernelGGL((k_wc_count<SUBS, LDS_N, PROBES>), dim3((unsigned)nb), dim3(NT), 0, s, text, n, T);
  MRH_CHECK_LAUNCH();
}

void wc_count(const uint8_t* text, int64_t n, uint64_t* slots, uint32_t* counts, int64_t cap, int32_t* newlist,
              uint64_t* ctr, uint64_t used0, const uint8_t* arena, hipStream_t s) {
  if (n <= 0) return;
  const Table T = make_table(slots, counts, cap, newlist, ctr, used0, arena);
  // 16 KiB of text per workgroup, 2048-entry LDS table, 16 probes: the best
  // of a sweep over 4-256 KiB tiles and 1K-8K LDS entries on MI355X (wordfreq
  // bench, 1 GiB Zipf text: 25-28 ms/step vs 30-51 ms for the others; bigger
  // tiles lose more to lower occupancy / fewer workgroups than they save in
  // global flushes)
  launch_count<4, 2048, 16>(text, n, T, s);
}

void wc_migrate(const uint8_t* text, int64_t n, uint64_t* slots, int64_t cap, int32_t* newlist, uint64_t* ctr,
                uint64_t used0, uint8_t* arena, int64_t max_new, hipStream_t s) {
  if (max_new <= 0) return;
  hipLaunchKernelGGL(k_wc_migrate, dim3((unsigned)((max_new + NT - 1) / NT)), dim3(NT), 0, s, text, n,
                     make_table(slots, nullptr, cap, newlist, ctr, used0, arena), arena, max_new);
  MRH_CHECK_LAUNCH();
}

void wc_rehash(const uint64_t* old_slots, const uint32_t* old_counts, int64_t old_cap, const uint8_t* arena,
               uint64_t* new_slots, uint32_t* new_counts, int64_t new_cap, hipStream_t s) {
  if (old_cap <= 0) return;
  hipLaunchKernelGGL(k_wc_rehash, dim3((unsigned)((old_cap + NT - 1) / NT)), dim3(NT), 0, s,
                     (const unsigned long long*)old_slots, old_counts, old_cap, arena,
                     (unsigned long long*)new_slots, new_counts, (uint64_t)new_cap - 1);
  MRH_CHECK_LAUNCH();
}

void wc_keys(const uint64_t* slots, const int64_t* idx, int64_t nk, const uint8_t* arena, int64_t* starts,
             int32_t* lens, hipStream_t s) {
  if (nk <= 0) return;
  hipLaunchKernelGGL(k_wc_keys, dim3((unsigned)((nk + NT - 1) / NT)), dim3(NT), 0, s,
                     (const unsigned long long*)slots, idx, nk, arena, starts, lens);
  MRH_CHECK_LAUNCH();
}

}  // namespace k
}  // namespace mrh
