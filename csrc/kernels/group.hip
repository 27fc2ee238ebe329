// Incremental exact group-by for gfx950: the device side of GroupIndex
// (csrc/engine/grouper.h), i.e. MR-MPI's convert (reference
// src/keymultivalue.cpp:645-789 kv2unique hash buckets) done part by part
// while the KV is still being produced.
//
// Every appended part is grouped into one open-addressing table in HBM:
//   slots[cap] : u64 64-bit key hash (0 = empty; a zero hash is stored as 1)
//   sgid[cap]  : i32 dense group id of the slot
//   rep[g]     : i64 row (in the appended KV) of group g's first key
//   ghash[g]   : u64 hash of group g
// k_grp_insert claims or finds the slot of every pair's hash (one 64-bit CAS
// per new group, a relaxed load per probe, no spinning on other lanes: a
// pair that finds its hash claimed by another pair only records the slot).
// After the kernel boundary k_grp_resolve turns slots into group ids and
// checks the key BYTES of every non-claiming pair against its group's first
// key: grouping is exact, a true 64-bit collision is counted and the host
// falls back to the sort path with exact regrouping.
#include "common.h"
#include "launch.h"

namespace mrh {
namespace k {
namespace {

constexpr int NT = 256;
constexpr uint32_t CLAIM = 0x80000000u;

unsigned blocks_for(int64_t n) {
  int64_t b = (n + NT - 1) / NT;
  return (unsigned)(b < 1 ? 1 : (b > (1 << 20) ? (1 << 20) : b));
}

__device__ __forceinline__ uint64_t nz(uint64_t h) { return h ? h : 1ull; }
// slot of a hash: the low half of lookup3's hashlittle2 is its "b" word, the
// high half "c"; xor-folding keeps both in play for small tables
__device__ __forceinline__ uint64_t home(uint64_t h, uint64_t mask) { return (h ^ (h >> 32)) & mask; }

__global__ __launch_bounds__(NT) void k_grp_insert(const uint64_t* __restrict__ h, int64_t n, int64_t row0,
                                                  unsigned long long* __restrict__ slots, int32_t* __restrict__ sgid,
                                                  uint64_t mask, unsigned long long* __restrict__ ctr,
                                                  int64_t* __restrict__ rep, uint64_t* __restrict__ ghash,
                                                  uint32_t* __restrict__ code) {
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) {
    const unsigned long long hv = nz(h[i]);
    uint64_t s = home(hv, mask);
    for (;;) {
      // plain load: a slot only ever goes 0 -> hash once, so a stale 0 just
      // costs the CAS below (which returns the live value) and a non-zero
      // value is final; hot keys then hit in the CU's L1 instead of L2
      unsigned long long v = slots[s];
      if (v == 0) {
        v = atomicCAS(&slots[s], 0ull, hv);
        if (v == 0) {
          const int32_t g = (int32_t)atomicAdd(&ctr[0], 1ull);
          sgid[s] = g;
          rep[g] = row0 + i;
          ghash[g] = hv;
          code[i] = CLAIM | (uint32_t)g;
          break;
        }
      }
      if (v == hv) {
        code[i] = (uint32_t)s;
        break;
      }
      s = (s + 1) & mask;
    }
  }
}

// key bytes of arena row r
struct Keys {
  const uint8_t* d;
  const int64_t* off;  // null: fixed width w
  int w;
  __device__ __forceinline__ const uint8_t* at(int64_t r) const { return off ? d + off[r] : d + r * (int64_t)w; }
  __device__ __forceinline__ int64_t len(int64_t r) const { return off ? off[r + 1] - off[r] : (int64_t)w; }
};

__global__ __launch_bounds__(NT) void k_grp_resolve(const uint32_t* __restrict__ code, int64_t n, int64_t row0,
                                                   const int32_t* __restrict__ sgid, const int64_t* __restrict__ rep,
                                                   Keys K, int32_t* __restrict__ gid,
                                                   unsigned long long* __restrict__ ctr) {
  unsigned long long bad = 0;
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) {
    const uint32_t c = code[i];
    if (c & CLAIM) {
      gid[row0 + i] = (int32_t)(c & ~CLAIM);
      continue;
    }
    const int32_t g = sgid[c];
    gid[row0 + i] = g;
    const int64_t a = row0 + i, b = rep[g];
    const int64_t la = K.len(a);
    if (la != K.len(b) || !dev::bytes_equal(K.at(a), K.at(b), la)) ++bad;
  }
  bad = dev::wave_sum(bad);
  if (dev::lane_id() == 0 && bad) atomicAdd(&ctr[1], bad);
}

__global__ __launch_bounds__(NT) void k_grp_rehash(const unsigned long long* __restrict__ os,
                                                  const int32_t* __restrict__ og, int64_t ocap,
                                                  unsigned long long* __restrict__ ns, int32_t* __restrict__ ng,
                                                  uint64_t nmask) {
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < ocap; i += (int64_t)gridDim.x * NT) {
    const unsigned long long v = os[i];
    if (!v) continue;
    uint64_t s = home(v, nmask);
    while (atomicCAS(&ns[s], 0ull, v) != 0ull) s = (s + 1) & nmask;
    ng[s] = og[i];
  }
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

void grp_insert(const uint64_t* h, int64_t n, int64_t row0, uint64_t* slots, int32_t* sgid, int64_t cap,
                uint64_t* ctr, int64_t* rep, uint64_t* ghash, uint32_t* code, hipStream_t s) {
  if (n <= 0) return;
  check_arg(cap > 0 && (cap & (cap - 1)) == 0, "grp_insert: table capacity must be a power of two");
  hipLaunchKernelGGL(k_grp_insert, dim3(blocks_for(n)), dim3(NT), 0, s, h, n, row0, (unsigned long long*)slots, sgid,
                     (uint64_t)cap - 1, (unsigned long long*)ctr, rep, ghash, code);
  MRH_CHECK_LAUNCH();
}

void grp_resolve(const uint32_t* code, int64_t n, int64_t row0, const int32_t* sgid, const int64_t* rep,
                 const uint8_t* kd, const int64_t* koff, int kw, int32_t* gid, uint64_t* ctr, hipStream_t s) {
  if (n <= 0) return;
  Keys K{kd, koff, kw};
  hipLaunchKernelGGL(k_grp_resolve, dim3(blocks_for(n)), dim3(NT), 0, s, code, n, row0, sgid, rep, K, gid,
                     (unsigned long long*)ctr);
  MRH_CHECK_LAUNCH();
}

void grp_rehash(const uint64_t* old_slots, const int32_t* old_gid, int64_t old_cap, uint64_t* new_slots,
                int32_t* new_gid, int64_t new_cap, hipStream_t s) {
  if (old_cap <= 0) return;
  check_arg(new_cap > 0 && (new_cap & (new_cap - 1)) == 0, "grp_rehash: capacity must be a power of two");
  hipLaunchKernelGGL(k_grp_rehash, dim3(blocks_for(old_cap)), dim3(NT), 0, s, (const unsigned long long*)old_slots,
                     old_gid, old_cap, (unsigned long long*)new_slots, new_gid, (uint64_t)new_cap - 1);
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
