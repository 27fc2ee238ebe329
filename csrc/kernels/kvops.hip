// KV/KMV data-movement kernels: sort-key construction, row gathers (fixed and
// variable width), segment (group) boundary detection and group verification.
// These replace KeyValue::add / KeyMultiValue::kv2kmv scatter loops of MR-MPI
// (reference src/keyvalue.cpp:343-392, src/keymultivalue.cpp:1139-1209).
#include "common.h"
#include "launch.h"
#include <cstdio>
#include <cstdlib>

namespace mrh {
namespace k {
namespace {

constexpr int NT = 256;
inline unsigned nblk(int64_t n, int per = NT) { return (unsigned)((n + per - 1) / per); }

__device__ __forceinline__ uint64_t load_le(const uint8_t* p, int w) {
  uint64_t v = 0;
  for (int b = 0; b < w; ++b) v |= (uint64_t)p[b] << (8 * b);
  return v;
}

__global__ __launch_bounds__(NT) void k_sortkeys_fixed(const uint8_t* __restrict__ d, int w, int64_t n,
                                                      int mode, bool desc, uint64_t* __restrict__ keys,
                                                      uint32_t* __restrict__ idx) {
  int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (i >= n) return;
  uint64_t raw;
  if (w == 8) raw = *reinterpret_cast<const uint64_t*>(d + i * 8);
  else if (w == 4) raw = *reinterpret_cast<const uint32_t*>(d + i * 4);
  else raw = load_le(d + i * w, w);
  keys[i] = dev::sortkey(raw, mode, desc);
  idx[i] = (uint32_t)i;
}

__global__ __launch_bounds__(NT) void k_sortkeys_str(const uint8_t* __restrict__ d,
                                                    const int64_t* __restrict__ off, int64_t n,
                                                    int64_t start, bool desc, uint64_t* __restrict__ keys,
                                                    uint32_t* __restrict__ idx) {
  int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (i >= n) return;
  int64_t a = off[i] + start, b = off[i + 1];
  uint64_t k = 0;
  bool ended = false;  // strcmp semantics: nothing after the first NUL counts
  for (int j = 0; j < 8; ++j) {
    uint64_t c = (!ended && a + j < b) ? d[a + j] : 0;
    ended |= c == 0;
    k = (k << 8) | c;
  }
  keys[i] = desc ? ~k : k;
  idx[i] = (uint32_t)i;
}

// ---- device tie-break of the string sort (flags +-5/+-6), one round per
// 8-byte window: elements whose groups are still tied after the window at
// `start` are re-keyed on the next window and re-sorted inside their group

__device__ __forceinline__ bool window_ended(uint64_t k, bool desc) {
  const uint64_t x = desc ? ~k : k;
  // any zero byte: the string ended inside this window (equal windows = equal strings)
  return ((x - 0x0101010101010101ull) & ~x & 0x8080808080808080ull) != 0;
}

// head / active flags after the round whose keys are ks (valid for alive elements)
__global__ __launch_bounds__(NT) void k_str_groups(const uint64_t* __restrict__ ks, const uint8_t* __restrict__ alive,
                                                   const uint32_t* __restrict__ head_in, int64_t n, bool desc,
                                                   uint32_t* __restrict__ head_out) {
  int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (i >= n) return;
  const bool al = alive ? alive[i] != 0 : true;
  bool h = i == 0 || (head_in && head_in[i]);
  if (!h && al) {
    const bool prev_al = alive ? alive[i - 1] != 0 : true;
    h = !prev_al || ks[i] != ks[i - 1];
  }
  if (!h && !al) h = true;  // a settled element is its own group
  head_out[i] = h ? 1u : 0u;
}
__global__ __launch_bounds__(NT) void k_str_active(const uint64_t* __restrict__ ks, const uint8_t* __restrict__ alive,
                                                   const uint32_t* __restrict__ head, int64_t n, bool desc,
                                                   uint32_t* __restrict__ active) {
  int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (i >= n) return;
  const bool al = alive ? alive[i] != 0 : true;
  const bool multi = !head[i] || (i + 1 < n && !head[i + 1]);
  active[i] = (al && multi && !window_ended(ks[i], desc)) ? 1u : 0u;
}

// compact the active elements: position, next-window key, group id
__global__ __launch_bounds__(NT) void k_str_refine(const uint32_t* __restrict__ active, const uint32_t* __restrict__ pos,
                                                   const uint32_t* __restrict__ gid_incl, const uint32_t* __restrict__ perm,
                                                   const uint8_t* __restrict__ d, const int64_t* __restrict__ off,
                                                   int64_t n, int64_t start, bool desc, int32_t* __restrict__ where,
                                                   uint64_t* __restrict__ nk, uint64_t* __restrict__ gk) {
  int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (i >= n || !active[i]) return;
  const uint32_t j = pos[i];
  const uint32_t r = perm[i];
  int64_t a = off[r] + start, b = off[r + 1];
  uint64_t k = 0;
  bool ended = false;
  for (int q = 0; q < 8; ++q) {
    uint64_t c = (!ended && a + q < b) ? d[a + q] : 0;
    ended |= c == 0;
    k = (k << 8) | c;
  }
  where[j] = (int32_t)i;
  nk[j] = desc ? ~k : k;
  gk[j] = gid_incl[i];
}

// apply the in-group order: element j of the sorted compact list takes the
// j-th active position (groups are contiguous in both)
__global__ __launch_bounds__(NT) void k_str_apply(const uint32_t* __restrict__ order, const int32_t* __restrict__ where,
                                                  const uint64_t* __restrict__ nk, int64_t m,
                                                  const uint32_t* __restrict__ perm_in, uint32_t* __restrict__ perm_out,
                                                  uint64_t* __restrict__ ks, uint8_t* __restrict__ alive) {
  int64_t j = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (j >= m) return;
  const int32_t dst = where[j], src = where[order[j]];
  perm_out[dst] = perm_in[src];
  ks[dst] = nk[order[j]];
  alive[dst] = 1;
}

__global__ __launch_bounds__(NT) void k_iota(uint32_t* __restrict__ idx, int64_t n) {
  int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (i < n) idx[i] = (uint32_t)i;
}

template <typename T, typename I>
__global__ __launch_bounds__(NT) void k_gather_words(const T* __restrict__ src, int words,
                                                    const I* __restrict__ idx, int64_t n,
                                                    T* __restrict__ dst) {
  // one thread per (row, word); consecutive threads -> consecutive words of a row
  int64_t t = (int64_t)blockIdx.x * NT + threadIdx.x;
  int64_t total = n * words;
  if (t >= total) return;
  int64_t r = t / words;
  int c = (int)(t - r * words);
  dst[t] = src[(int64_t)idx[r] * words + c];
}

__global__ __launch_bounds__(NT) void k_var_lengths(const int64_t* __restrict__ off,
                                                   const uint32_t* __restrict__ idx, int64_t n,
                                                   int32_t* __restrict__ len) {
  int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (i >= n) return;
  uint32_t r = idx ? idx[i] : (uint32_t)i;
  len[i] = (int32_t)(off[r + 1] - off[r]);
}

// 16 lanes per row, 4 rows per wave in flight.
__global__ __launch_bounds__(NT) void k_var_copy(const uint8_t* __restrict__ src,
                                                const int64_t* __restrict__ soff,
                                                const uint32_t* __restrict__ idx, int64_t n,
                                                uint8_t* __restrict__ dst,
                                                const int64_t* __restrict__ doff) {
  const int g = threadIdx.x & 15;
  int64_t row = ((int64_t)blockIdx.x * NT + threadIdx.x) >> 4;
  const int64_t stride = ((int64_t)gridDim.x * NT) >> 4;
  for (; row < n; row += stride) {
    uint32_t r = idx ? idx[row] : (uint32_t)row;
    int64_t a = soff[r], len = soff[r + 1] - a;
    int64_t o = doff[row];
    for (int64_t j = g; j < len; j += 16) dst[o + j] = src[a + j];
  }
}

__global__ __launch_bounds__(NT) void k_head_flags(const uint64_t* __restrict__ keys, int64_t n,
                                                  uint32_t* __restrict__ flags) {
  int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (i >= n) return;
  flags[i] = (i == 0 || keys[i] != keys[i - 1]) ? 1u : 0u;
}

__global__ __launch_bounds__(NT) void k_compact_heads(const uint32_t* __restrict__ flags,
                                                     const uint32_t* __restrict__ pos, int64_t n,
                                                     int64_t* __restrict__ seg) {
  int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (i < n && flags[i]) seg[pos[i]] = i;
  if (i == 0) seg[pos[n]] = n;
}

// fixed keys of nw 8-byte words whose significant bits fit one u64 together:
// key i -> OR of (word w << shift[w]) (an exact group key; words with no
// significant bit have shift -1)
__global__ __launch_bounds__(NT) void k_pack_words(const uint64_t* __restrict__ kd, int64_t n, PackShifts sh,
                                                  uint64_t* __restrict__ out, uint32_t* __restrict__ idx) {
  const int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (i >= n) return;
  uint64_t k = 0;
  for (int w = 0; w < sh.nw; ++w)
    if (sh.s[w] >= 0) k |= kd[i * sh.nw + w] << sh.s[w];
  out[i] = k;
  idx[i] = (uint32_t)i;
}

// narrow keys with narrow 8-byte values: pair i -> (packed key words) | value
// (key word w at shift s[w] >= vbits, the value below vbits)
__global__ __launch_bounds__(NT) void k_pack_kv(const uint64_t* __restrict__ kd, const uint64_t* __restrict__ vd,
                                               int64_t n, PackShifts sh, uint64_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (i >= n) return;
  uint64_t k = vd[i];
  for (int w = 0; w < sh.nw; ++w)
    if (sh.s[w] >= 0) k |= kd[i * sh.nw + w] << sh.s[w];
  out[i] = k;
}

// narrow pairs whose key and value bits together exceed one u64 by B <= 16
// bits (or whose count asks for buckets): the key K (words at shifts s[w],
// relative to bit 0) is cut into a bucket and a rest, and the sort word is
// rest << vbits | value. Two cuts:
//  * hi >= 0 (ordered): bucket = K >> hi, rest = the low hi bits — buckets in
//    key order, so the KMV's keys stay sorted (used while every bucket fits
//    a sort, however skewed);
//  * hi < 0 (mixed): rest = K >> B, bucket = (K & (2^B - 1)) ^ mix(rest) —
//    balanced for skewed keys (more than 2^31 pairs), and invertible.
// vw: value width 4 (u32) or 8 (u64).
__device__ __forceinline__ uint32_t split_mix(uint64_t rest, int B) {
  return B ? (uint32_t)((rest * 0x9E3779B97F4A7C15ull) >> (64 - B)) : 0u;
}
__device__ __forceinline__ uint32_t split_cut(uint64_t K, int B, int hi, uint64_t* rest) {
  if (hi >= 0) {
    *rest = hi >= 64 ? K : (K & ((1ull << hi) - 1));
    return hi >= 64 ? 0u : (uint32_t)(K >> hi);
  }
  *rest = B ? K >> B : K;
  return B ? (uint32_t)(K & ((1ull << B) - 1)) ^ split_mix(*rest, B) : 0u;
}
__device__ __forceinline__ uint64_t split_join(uint64_t rest, uint32_t bucket, int B, int hi) {
  if (hi >= 0) return hi >= 64 ? rest : (((uint64_t)bucket << hi) | rest);
  return B ? (rest << B) | (uint64_t)((bucket ^ split_mix(rest, B)) & ((1u << B) - 1)) : rest;
}
__global__ __launch_bounds__(NT) void k_pack_kv_split(const uint64_t* __restrict__ kd, const void* __restrict__ vd,
                                                     int vw, int64_t n, PackShifts sh, int vbits, int B, int hi,
                                                     uint64_t* __restrict__ out, int32_t* __restrict__ bkt) {
  const int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (i >= n) return;
  uint64_t K = 0;
  for (int w = 0; w < sh.nw; ++w)
    if (sh.s[w] >= 0) K |= kd[i * sh.nw + w] << sh.s[w];
  const uint64_t v = vw == 4 ? (uint64_t)static_cast<const uint32_t*>(vd)[i] : static_cast<const uint64_t*>(vd)[i];
  uint64_t rest;
  const uint32_t b = split_cut(K, B, hi, &rest);
  out[i] = (rest << vbits) | v;
  if (bkt) bkt[i] = (int32_t)b;
}

// the unique keys of one bucket back to key words: heads hold rest (the
// sorted words shifted down by vbits); K = split_join(rest, bucket);
// word w = (K >> s[w]) & mask[w]
__global__ __launch_bounds__(NT) void k_unpack_split(const uint64_t* __restrict__ heads, int64_t m, int bucket, int B,
                                                    int hi, PackShifts sh, PackShifts bits,
                                                    uint64_t* __restrict__ keys) {
  const int64_t j = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (j >= m) return;
  const uint64_t K = split_join(heads[j], (uint32_t)bucket, B, hi);
  for (int w = 0; w < sh.nw; ++w) {
    uint64_t x = 0;
    if (sh.s[w] >= 0) {
      x = K >> sh.s[w];
      if (bits.s[w] < 64) x &= (1ull << bits.s[w]) - 1;
    }
    keys[j * sh.nw + w] = x;
  }
}

// values of sorted words: the low vbits, as u32 (vw 4) or u64 (vw 8)
__global__ __launch_bounds__(NT) void k_split_values(const uint64_t* __restrict__ words, int64_t n, int vbits, int vw,
                                                    void* __restrict__ vout) {
  const int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (i >= n) return;
  const uint64_t v = vbits >= 64 ? words[i] : words[i] & ((1ull << vbits) - 1);
  if (vw == 4) static_cast<uint32_t*>(vout)[i] = (uint32_t)v;
  else static_cast<uint64_t*>(vout)[i] = v;
}

// Segments of sorted packed words (key bits [vb, vb + sbits), value bits
// below vb) without materialising the keys: a tile of SG_TILE words counts
// its heads (word i starts a segment when its key bits differ from word
// i - 1's); after the scan of the tile counts the second kernel writes every
// head's position and key bits and every word's value (coalesced, word i of
// step j is base + j * SG_NT + thread). Two reads of the words replace the
// shift, mask, flag, scan, compact, head-gather and value-split passes.
constexpr int SG_NT = 256, SG_IT = 16, SG_TILE = SG_NT * SG_IT;
__device__ __forceinline__ bool sg_head(const uint64_t* __restrict__ w, int64_t i, uint64_t cur, int vb,
                                        uint64_t km) {
  return i == 0 || (((cur ^ w[i - 1]) >> vb) & km) != 0;
}
__global__ __launch_bounds__(SG_NT) void k_seg_packed_count(const uint64_t* __restrict__ w, int64_t n, int vb,
                                                           uint64_t km, int64_t* __restrict__ tcnt) {
  __shared__ int64_t red[SG_NT / MRH_WAVE];
  const int64_t base = (int64_t)blockIdx.x * SG_TILE;
  int c = 0;
#pragma unroll
  for (int j = 0; j < SG_IT; ++j) {
    const int64_t i = base + (int64_t)j * SG_NT + threadIdx.x;
    if (i < n) c += sg_head(w, i, w[i], vb, km) ? 1 : 0;
  }
  c = dev::wave_sum(c);
  if (dev::lane_id() == 0) red[dev::wave_id()] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t t = 0;
    for (int q = 0; q < SG_NT / MRH_WAVE; ++q) t += red[q];
    tcnt[blockIdx.x] = t;
  }
}
__global__ __launch_bounds__(SG_NT) void k_seg_packed_write(const uint64_t* __restrict__ w, int64_t n, int vb,
                                                           uint64_t km, const int64_t* __restrict__ tbase,
                                                           int64_t* __restrict__ seg, uint64_t* __restrict__ heads,
                                                           void* __restrict__ vout, int vw) {
  constexpr int NW = SG_NT / MRH_WAVE;
  __shared__ uint32_t wc[SG_IT * NW];
  const int lane = dev::lane_id(), wid = dev::wave_id();
  const int64_t base = (int64_t)blockIdx.x * SG_TILE;
  const uint64_t vmask = vb >= 64 ? ~0ull : ((1ull << vb) - 1);
  uint64_t kk[SG_IT], hm[SG_IT];
#pragma unroll
  for (int j = 0; j < SG_IT; ++j) {
    const int64_t i = base + (int64_t)j * SG_NT + threadIdx.x;
    const bool valid = i < n;
    kk[j] = valid ? w[i] : 0ull;
    const bool h = valid && sg_head(w, i, kk[j], vb, km);
    hm[j] = __ballot(h);
    if (lane == 0) wc[j * NW + wid] = (uint32_t)__popcll(hm[j]);
    if (valid) {
      if (vw == 4) static_cast<uint32_t*>(vout)[i] = (uint32_t)(kk[j] & vmask);
      else static_cast<uint64_t*>(vout)[i] = kk[j] & vmask;
    }
  }
  __syncthreads();
  if (threadIdx.x < MRH_WAVE) {  // SG_IT * NW = 64 counts, index order (step, wave)
    const uint32_t x = wc[threadIdx.x];
    const uint32_t inc = dev::wave_incl_scan(x);
    wc[threadIdx.x] = inc - x;
  }
  __syncthreads();
  const int64_t tb = tbase[blockIdx.x];
  const uint64_t lt = dev::lanemask_lt();
#pragma unroll
  for (int j = 0; j < SG_IT; ++j) {
    if ((hm[j] >> lane) & 1ull) {
      const int64_t pos = tb + wc[j * NW + wid] + __popcll(hm[j] & lt);
      seg[pos] = base + (int64_t)j * SG_NT + threadIdx.x;
      heads[pos] = (kk[j] >> vb) & km;
    }
  }
}
static_assert(SG_IT * (SG_NT / MRH_WAVE) == MRH_WAVE, "k_seg_packed_write scans its step counts in one wave");

// head bitmap (bit i of 64-bit word i / 64 set where a segment starts) ->
// per-word counts, then the positions of the set bits (one word per thread)
__global__ __launch_bounds__(NT) void k_bits_count(const uint64_t* __restrict__ H, int64_t nw,
                                                  uint32_t* __restrict__ cnt) {
  const int64_t w = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (w < nw) cnt[w] = (uint32_t)__popcll(H[w]);
}
__global__ __launch_bounds__(NT) void k_bits_compact(const uint64_t* __restrict__ H, int64_t nw,
                                                    const uint32_t* __restrict__ pos, int64_t n,
                                                    int64_t* __restrict__ seg) {
  const int64_t w = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (w < nw) {
    uint64_t b = H[w];
    int64_t o = pos[w];
    while (b) {
      seg[o++] = w * 64 + (__ffsll((long long)b) - 1);
      b &= b - 1;
    }
  }
  if (w == 0) seg[pos[nw]] = n;
}

// 16 lanes per pair: each group compares one non-head key with its sorted
// predecessor (same segment, so equality along the chain = equality with the
// head; the count is > 0 iff some segment mixes keys). The predecessor's perm
// entry sits next to the row's own, so the dependent-load chain is
// perm -> off -> bytes (3 levels, not pos -> seg -> perm -> off -> bytes).
// Bytes: 4 per lane per step via aligned dword loads + v_alignbyte (ld32u), so
// a ~64-byte URL is one 64-byte sweep per key; the < 4-byte tail uses bytes.
__global__ __launch_bounds__(NT) void k_verify_var(const uint8_t* __restrict__ kd,
                                                  const int64_t* __restrict__ off,
                                                  const uint32_t* __restrict__ perm,
                                                  const uint32_t* __restrict__ flags, int64_t n,
                                                  unsigned long long* mism) {
  const int g = threadIdx.x & 15;
  const int gbase = (threadIdx.x & 63) & ~15;
  int64_t row = ((int64_t)blockIdx.x * NT + threadIdx.x) >> 4;
  const int64_t stride = ((int64_t)gridDim.x * NT) >> 4;
  int64_t bad = 0;
  for (; row < n; row += stride) {  // row is uniform within a 16-lane group
    if (flags[row]) continue;       // row 0 is always a head, so row - 1 >= 0
    const uint32_t a = perm[row], b = perm[row - 1];
    const int64_t a0 = off[a], la = off[a + 1] - a0, b0 = off[b], lb = off[b + 1] - b0;
    bool diff = la != lb;
    if (!diff) {
      for (int64_t j = 4 * g; j < la; j += 64) {
        if (la - j >= 4) {
          diff |= dev::ld32u(kd + a0 + j) != dev::ld32u(kd + b0 + j);
        } else {
          for (int64_t t = j; t < la; ++t) diff |= kd[a0 + t] != kd[b0 + t];
        }
      }
    }
    const unsigned long long m = __ballot(diff);
    if (g == 0 && ((m >> gbase) & 0xffffull)) ++bad;
  }
  if (bad) atomicAdd(mism, (unsigned long long)bad);
}

__global__ __launch_bounds__(NT) void k_verify_fixed(const uint8_t* __restrict__ kd, int kw,
                                                    const uint32_t* __restrict__ perm,
                                                    const uint32_t* __restrict__ flags,
                                                    const uint32_t* __restrict__ pos,
                                                    const int64_t* __restrict__ seg, int64_t n,
                                                    unsigned long long* mism) {
  int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (i >= n || flags[i]) return;
  const uint8_t* pa = kd + (int64_t)perm[i] * kw;
  const uint8_t* pb = kd + (int64_t)perm[i - 1] * kw;  // sorted predecessor, as k_verify_var
  bool diff = false;
  for (int j = 0; !diff && j < kw; ++j) diff = pa[j] != pb[j];
  if (diff) atomicAdd(mism, 1ull);
}

__global__ __launch_bounds__(NT) void k_dest_bytes(const int32_t* __restrict__ dest,
                                                  const int64_t* __restrict__ off, int64_t n, int P,
                                                  int64_t* __restrict__ bytes) {
  __shared__ unsigned long long hist[1024];
  for (int i = threadIdx.x; i < P; i += NT) hist[i] = 0;
  __syncthreads();
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT)
    atomicAdd(&hist[dest[i]], (unsigned long long)(off[i + 1] - off[i]));
  __syncthreads();
  for (int i = threadIdx.x; i < P; i += NT)
    if (hist[i]) atomicAdd((unsigned long long*)&bytes[i], hist[i]);
}

__global__ __launch_bounds__(NT) void k_off_to_len(const int64_t* __restrict__ off, int64_t n,
                                                  int32_t* __restrict__ len) {
  int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (i < n) len[i] = (int32_t)(off[i + 1] - off[i]);
}

template <typename I>
void gather_fixed_t(const uint8_t* src, int w, const I* idx, int64_t n, uint8_t* dst, hipStream_t s) {
  if (n <= 0 || w <= 0) return;
  if (w % 8 == 0 && ((uintptr_t)src % 8 == 0) && ((uintptr_t)dst % 8 == 0)) {
    int words = w / 8;
    hipLaunchKernelGGL((k_gather_words<uint64_t, I>), dim3(nblk(n * words)), dim3(NT), 0, s,
                       (const uint64_t*)src, words, idx, n, (uint64_t*)dst);
  } else if (w % 4 == 0 && ((uintptr_t)src % 4 == 0) && ((uintptr_t)dst % 4 == 0)) {
    int words = w / 4;
    hipLaunchKernelGGL((k_gather_words<uint32_t, I>), dim3(nblk(n * words)), dim3(NT), 0, s,
                       (const uint32_t*)src, words, idx, n, (uint32_t*)dst);
  } else {
    hipLaunchKernelGGL((k_gather_words<uint8_t, I>), dim3(nblk(n * w)), dim3(NT), 0, s, src, w, idx, n,
                       dst);
  }
  MRH_CHECK_LAUNCH();
}


// range bucket of every key: the number of splitters strictly below it
// (lower_bound over the sorted unsigned splitters, staged in LDS; up to
// 4096 splitters = 32 KiB) — the out-of-core sample sort's partition pass
constexpr int SPLIT_MAX = 4096;
template <bool RIGHT>
__global__ __launch_bounds__(256) void k_bucket_by_splitters(const uint64_t* __restrict__ keys, int64_t n,
                                                            const uint64_t* __restrict__ split, int ns,
                                                            int32_t* __restrict__ out) {
  __shared__ uint64_t sp[SPLIT_MAX];
  for (int i = threadIdx.x; i < ns; i += 256) sp[i] = split[i];
  __syncthreads();
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
    const uint64_t k = keys[i];
    int lo = 0, hi = ns;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (RIGHT ? sp[mid] <= k : sp[mid] < k) lo = mid + 1;
      else hi = mid;
    }
    out[i] = lo;
  }
}

}  // namespace

void make_sortkeys_fixed(const uint8_t* data, int w, int64_t n, int mode, bool descending, uint64_t* keys,
                         uint32_t* idx, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_sortkeys_fixed, dim3(nblk(n)), dim3(NT), 0, s, data, w, n, mode, descending, keys,
                     idx);
  MRH_CHECK_LAUNCH();
}
void make_sortkeys_strprefix(const uint8_t* data, const int64_t* off, int64_t n, int64_t start,
                             bool descending, uint64_t* keys, uint32_t* idx, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_sortkeys_str, dim3(nblk(n)), dim3(NT), 0, s, data, off, n, start, descending, keys,
                     idx);
  MRH_CHECK_LAUNCH();
}
void str_groups(const uint64_t* ks, const uint8_t* alive, const uint32_t* head_in, int64_t n, bool desc,
                uint32_t* head_out, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_str_groups, dim3(nblk(n)), dim3(NT), 0, s, ks, alive, head_in, n, desc, head_out);
  MRH_CHECK_LAUNCH();
}
void str_active(const uint64_t* ks, const uint8_t* alive, const uint32_t* head, int64_t n, bool desc, uint32_t* active,
                hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_str_active, dim3(nblk(n)), dim3(NT), 0, s, ks, alive, head, n, desc, active);
  MRH_CHECK_LAUNCH();
}
void str_refine(const uint32_t* active, const uint32_t* pos, const uint32_t* gid_incl, const uint32_t* perm,
                const uint8_t* data, const int64_t* off, int64_t n, int64_t start, bool desc, int32_t* where,
                uint64_t* nk, uint64_t* gk, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_str_refine, dim3(nblk(n)), dim3(NT), 0, s, active, pos, gid_incl, perm, data, off, n, start,
                     desc, where, nk, gk);
  MRH_CHECK_LAUNCH();
}
void str_apply(const uint32_t* order, const int32_t* where, const uint64_t* nk, int64_t m, const uint32_t* perm_in,
               uint32_t* perm_out, uint64_t* ks, uint8_t* alive, hipStream_t s) {
  if (m <= 0) return;
  hipLaunchKernelGGL(k_str_apply, dim3(nblk(m)), dim3(NT), 0, s, order, where, nk, m, perm_in, perm_out, ks, alive);
  MRH_CHECK_LAUNCH();
}
void iota_u32(uint32_t* idx, int64_t n, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_iota, dim3(nblk(n)), dim3(NT), 0, s, idx, n);
  MRH_CHECK_LAUNCH();
}
void gather_fixed(const uint8_t* src, int w, const uint32_t* idx, int64_t n, uint8_t* dst, hipStream_t s) {
  gather_fixed_t<uint32_t>(src, w, idx, n, dst, s);
}
void gather_fixed_i64idx(const uint8_t* src, int w, const int64_t* idx, int64_t n, uint8_t* dst,
                         hipStream_t s) {
  gather_fixed_t<int64_t>(src, w, idx, n, dst, s);
}
void gather_var_lengths(const int64_t* src_off, const uint32_t* idx, int64_t n, int32_t* len,
                        hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_var_lengths, dim3(nblk(n)), dim3(NT), 0, s, src_off, idx, n, len);
  MRH_CHECK_LAUNCH();
}
void gather_var_copy(const uint8_t* src, const int64_t* src_off, const uint32_t* idx, int64_t n,
                     uint8_t* dst, const int64_t* dst_off, hipStream_t s) {
  if (n <= 0) return;
  unsigned g = nblk(n * 16);
  if (g > 65536) g = 65536;
  hipLaunchKernelGGL(k_var_copy, dim3(g), dim3(NT), 0, s, src, src_off, idx, n, dst, dst_off);
  MRH_CHECK_LAUNCH();
}
void head_flags_u64(const uint64_t* keys, int64_t n, uint32_t* flags, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_head_flags, dim3(nblk(n)), dim3(NT), 0, s, keys, n, flags);
  MRH_CHECK_LAUNCH();
}
void compact_heads(const uint32_t* flags, const uint32_t* pos, int64_t n, int64_t* seg, hipStream_t s) {
  hipLaunchKernelGGL(k_compact_heads, dim3(n > 0 ? nblk(n) : 1), dim3(NT), 0, s, flags, pos, n, seg);
  MRH_CHECK_LAUNCH();
}
void pack_words(const uint64_t* kd, int64_t n, const PackShifts& sh, uint64_t* out, uint32_t* idx, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_pack_words, dim3(nblk(n)), dim3(NT), 0, s, kd, n, sh, out, idx);
  MRH_CHECK_LAUNCH();
}
void pack_kv(const uint64_t* kd, const uint64_t* vd, int64_t n, const PackShifts& sh, uint64_t* out, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_pack_kv, dim3(nblk(n)), dim3(NT), 0, s, kd, vd, n, sh, out);
  MRH_CHECK_LAUNCH();
}
void pack_kv_split(const uint64_t* kd, const void* vd, int vw, int64_t n, const PackShifts& sh, int vbits, int B, int hi,
                   uint64_t* out, int32_t* bkt, hipStream_t s) {
  if (n <= 0) return;
  check_arg(vw == 4 || vw == 8, "pack_kv_split: 4- or 8-byte values");
  check_arg(B >= 0 && B <= 16, "pack_kv_split: at most 16 bucket bits");
  hipLaunchKernelGGL(k_pack_kv_split, dim3(nblk(n)), dim3(NT), 0, s, kd, vd, vw, n, sh, vbits, B, hi, out, bkt);
  MRH_CHECK_LAUNCH();
}
void unpack_split(const uint64_t* heads, int64_t m, int bucket, int B, int hi, const PackShifts& sh, const PackShifts& bits,
                  uint64_t* keys, hipStream_t s) {
  if (m <= 0) return;
  hipLaunchKernelGGL(k_unpack_split, dim3(nblk(m)), dim3(NT), 0, s, heads, m, bucket, B, hi, sh, bits, keys);
  MRH_CHECK_LAUNCH();
}
int64_t seg_packed_tiles(int64_t n) { return (n + SG_TILE - 1) / SG_TILE; }
void seg_packed_count(const uint64_t* w, int64_t n, int vb, uint64_t km, int64_t* tcnt, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_seg_packed_count, dim3((unsigned)seg_packed_tiles(n)), dim3(SG_NT), 0, s, w, n, vb, km, tcnt);
  MRH_CHECK_LAUNCH();
}
void seg_packed_write(const uint64_t* w, int64_t n, int vb, uint64_t km, const int64_t* tbase, int64_t* seg,
                      uint64_t* heads, void* vout, int vw, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_seg_packed_write, dim3((unsigned)seg_packed_tiles(n)), dim3(SG_NT), 0, s, w, n, vb, km, tbase,
                     seg, heads, vout, vw);
  MRH_CHECK_LAUNCH();
}
void split_values(const uint64_t* words, int64_t n, int vbits, int vw, void* vout, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_split_values, dim3(nblk(n)), dim3(NT), 0, s, words, n, vbits, vw, vout);
  MRH_CHECK_LAUNCH();
}
void bits_count(const uint64_t* H, int64_t nw, uint32_t* cnt, hipStream_t s) {
  if (nw <= 0) return;
  hipLaunchKernelGGL(k_bits_count, dim3(nblk(nw)), dim3(NT), 0, s, H, nw, cnt);
  MRH_CHECK_LAUNCH();
}
void bits_compact(const uint64_t* H, int64_t nw, const uint32_t* pos, int64_t n, int64_t* seg, hipStream_t s) {
  hipLaunchKernelGGL(k_bits_compact, dim3(nw > 0 ? nblk(nw) : 1), dim3(NT), 0, s, H, nw, pos, n, seg);
  MRH_CHECK_LAUNCH();
}
void verify_groups_var(const uint8_t* kdata, const int64_t* koff, const uint32_t* perm, const uint32_t* flags,
                       const uint32_t* pos, const int64_t* seg, int64_t n, unsigned long long* mism,
                       hipStream_t s) {
  if (n <= 0) return;
  int64_t g = (n * 16 + NT - 1) / NT;
  if (g > 65536) g = 65536;
  hipLaunchKernelGGL(k_verify_var, dim3((unsigned)g), dim3(NT), 0, s, kdata, koff, perm, flags, n, mism);
  MRH_CHECK_LAUNCH();
}
void verify_groups_fixed(const uint8_t* kdata, int kw, const uint32_t* perm, const uint32_t* flags,
                         const uint32_t* pos, const int64_t* seg, int64_t n, unsigned long long* mism,
                         hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_verify_fixed, dim3(nblk(n)), dim3(NT), 0, s, kdata, kw, perm, flags, pos, seg, n,
                     mism);
  MRH_CHECK_LAUNCH();
}
void dest_byte_counts(const int32_t* dest, const int64_t* off, int64_t n, int P, int64_t* bytes,
                      hipStream_t s) {
  MRH_HIP(hipMemsetAsync(bytes, 0, sizeof(int64_t) * P, s));
  if (n <= 0) return;
  unsigned g = nblk(n);
  if (g > 2048) g = 2048;
  hipLaunchKernelGGL(k_dest_bytes, dim3(g), dim3(NT), 0, s, dest, off, n, P, bytes);
  MRH_CHECK_LAUNCH();
}
void bucket_by_splitters(const uint64_t* keys, int64_t n, const uint64_t* split, int nsplit, int32_t* out,
                         hipStream_t s, bool right) {
  check_arg(nsplit >= 0 && nsplit <= SPLIT_MAX, "bucket_by_splitters: at most 4096 splitters");
  if (n <= 0) return;
  int64_t g = (n + 255) / 256;
  if (g > 8192) g = 8192;
  if (right) hipLaunchKernelGGL(k_bucket_by_splitters<true>, dim3((unsigned)g), dim3(256), 0, s, keys, n, split, nsplit, out);
  else hipLaunchKernelGGL(k_bucket_by_splitters<false>, dim3((unsigned)g), dim3(256), 0, s, keys, n, split, nsplit, out);
  MRH_CHECK_LAUNCH();
}

void offsets_to_lengths(const int64_t* off, int64_t n, int32_t* len, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_off_to_len, dim3(nblk(n)), dim3(NT), 0, s, off, n, len);
  MRH_CHECK_LAUNCH();
}

}  // namespace k
}  // namespace mrh
