// Text map kernels.
//
// InvertedIndex: the reference marks `<a href="` with one thread per byte and
// an int32 mask per byte, then thrust::sequence + count + copy_if + a
// divergent per-URL length scan (reference cuda/InvertedIndex.cu:79-135,324-370).
// Here each thread owns 16 text bytes held in registers as 32-bit words and
// tests all 16 alignments with v_alignbyte funnel shifts (3 word compares per
// position, no per-byte loads and no per-byte mask array); matches are
// compacted with a block scan into the URL start array (no iota, no mask).
//
// wordfreq: whitespace tokenizer (the reference's strtok " \t\n\f\r\0",
// examples/wordfreq.cpp:122-127) with the same count -> scan -> emit scheme.
//
// Text buffers must be padded with >= 32 readable bytes past n (the engine
// allocates them that way); bytes past n are treated as separators.
#include "common.h"
#include "launch.h"
#include <cstdio>
#include <cstdlib>

namespace mrh {
namespace k {
namespace {

constexpr int NT = 256;
constexpr int BYTES_PER_THREAD = 16;
constexpr int TILE = NT * BYTES_PER_THREAD;  // 4 KiB of text per block

// "<a h" "ref=" '"'  (little-endian words)
constexpr uint32_t P0 = 0x6820613Cu;
constexpr uint32_t P1 = 0x3D666572u;
constexpr uint32_t P2 = 0x22u;

__device__ __forceinline__ uint32_t align_bytes(uint32_t hi, uint32_t lo, int r) {
  return __builtin_amdgcn_alignbyte(hi, lo, (uint32_t)r);
}

// loads 16 + 12 bytes starting at p (p 16-aligned), returns 7 words (last = 0)
__device__ __forceinline__ void load_window(const uint8_t* text, int64_t p, uint32_t w[8]) {
  uint4 a = *reinterpret_cast<const uint4*>(text + p);
  uint2 b = *reinterpret_cast<const uint2*>(text + p + 16);
  uint32_t c = *reinterpret_cast<const uint32_t*>(text + p + 24);
  w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w; w[4] = b.x; w[5] = b.y; w[6] = c; w[7] = 0;
}

// bit k set if the pattern starts at p+k and lies fully inside [0, n)
__device__ __forceinline__ uint32_t url_match_mask(const uint8_t* text, int64_t p, int64_t n) {
  uint32_t w[8];
  load_window(text, p, w);
  uint32_t m = 0;
#pragma unroll
  for (int k = 0; k < BYTES_PER_THREAD; ++k) {
    const int q = k >> 2, r = k & 3;
    uint32_t x0 = r ? align_bytes(w[q + 1], w[q], r) : w[q];
    uint32_t x1 = r ? align_bytes(w[q + 2], w[q + 1], r) : w[q + 1];
    uint32_t x2 = (r ? align_bytes(w[q + 3], w[q + 2], r) : w[q + 2]) & 0xffu;
    bool hit = (x0 == P0) & (x1 == P1) & (x2 == P2) & (p + k + 8 < n);
    m |= (uint32_t)hit << k;
  }
  return m;
}

__global__ __launch_bounds__(NT) void k_url_count(const uint8_t* __restrict__ text, int64_t n,
                                                 uint32_t* __restrict__ tile_counts) {
  __shared__ uint32_t sh[NT / MRH_WAVE];
  const int64_t p = (int64_t)blockIdx.x * TILE + (int64_t)threadIdx.x * BYTES_PER_THREAD;
  uint32_t c = (p < n) ? (uint32_t)__popc(url_match_mask(text, p, n)) : 0u;
  c = dev::wave_sum(c);
  if (dev::lane_id() == 0) sh[dev::wave_id()] = c;
  __syncthreads();
  if (threadIdx.x == 0) tile_counts[blockIdx.x] = sh[0] + sh[1] + sh[2] + sh[3];
}

__global__ __launch_bounds__(NT) void k_url_emit(const uint8_t* __restrict__ text, int64_t n,
                                                const uint32_t* __restrict__ tile_off,
                                                int64_t* __restrict__ starts) {
  __shared__ uint32_t sh[NT / MRH_WAVE + 1];
  const int64_t p = (int64_t)blockIdx.x * TILE + (int64_t)threadIdx.x * BYTES_PER_THREAD;
  uint32_t m = (p < n) ? url_match_mask(text, p, n) : 0u;
  uint32_t total;
  uint32_t pos = dev::block_excl_scan<uint32_t, NT>((uint32_t)__popc(m), sh, &total);
  int64_t o = (int64_t)tile_off[blockIdx.x] + pos;
  while (m) {
    int k = __ffs(m) - 1;
    m &= m - 1;
    starts[o++] = p + k + 9;
  }
}

__global__ __launch_bounds__(NT) void k_url_len(const uint8_t* __restrict__ text, int64_t n,
                                               const int64_t* __restrict__ starts, int64_t nurl,
                                               int32_t* __restrict__ keylen) {
  int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (i >= nurl) return;
  int64_t a = starts[i];
  int64_t len = dev::find_byte(text + a, n - a, (uint8_t)'"');
  keylen[i] = (int32_t)(len + 1);  // + NUL terminator, as the reference's kv->add(url, len+1)
}

__device__ __forceinline__ bool is_ws(uint32_t c) {
  return c == ' ' || c == '\t' || c == '\n' || c == '\f' || c == '\r' || c == 0;
}

// bit k set if a word starts at p+k
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

__global__ __launch_bounds__(NT) void k_tok_count(const uint8_t* __restrict__ text, int64_t n,
                                                 uint32_t* __restrict__ tile_counts) {
  __shared__ uint32_t sh[NT / MRH_WAVE];
  const int64_t p = (int64_t)blockIdx.x * TILE + (int64_t)threadIdx.x * 16;
  uint32_t c = (p < n) ? (uint32_t)__popc(word_start_mask(text, p, n)) : 0u;
  c = dev::wave_sum(c);
  if (dev::lane_id() == 0) sh[dev::wave_id()] = c;
  __syncthreads();
  if (threadIdx.x == 0) tile_counts[blockIdx.x] = sh[0] + sh[1] + sh[2] + sh[3];
}

__global__ __launch_bounds__(NT) void k_tok_emit(const uint8_t* __restrict__ text, int64_t n,
                                                const uint32_t* __restrict__ tile_off,
                                                int64_t* __restrict__ starts, int32_t* __restrict__ keylen) {
  __shared__ uint32_t sh[NT / MRH_WAVE + 1];
  const int64_t p = (int64_t)blockIdx.x * TILE + (int64_t)threadIdx.x * 16;
  uint32_t m = (p < n) ? word_start_mask(text, p, n) : 0u;
  uint32_t total;
  uint32_t pos = dev::block_excl_scan<uint32_t, NT>((uint32_t)__popc(m), sh, &total);
  int64_t o = (int64_t)tile_off[blockIdx.x] + pos;
  while (m) {
    int k = __ffs(m) - 1;
    m &= m - 1;
    int64_t a = p + k, j = a;
    while (j < n && !is_ws(text[j])) ++j;
    starts[o] = a;
    keylen[o] = (int32_t)(j - a + 1);
    ++o;
  }
}

// wordfreq's pairs in one pass (map_words): a thread's 16 bytes give a start
// mask S, an end mask E (last byte of a word) and a non-separator mask; the
// keys are the words compacted with a NUL after each, so byte i of a word
// lands at (non-separator bytes before i) + (words ended before i), and word
// w's offset is where its first byte lands. k_tok_count2 counts per tile
// (words; non-separator bytes + ends), k_tok_emit2 writes the key bytes and
// offsets from the two scans — no start array, no per-word length walk, no
// separate copy kernel.
__device__ __forceinline__ void word_masks(const uint8_t* text, int64_t p, int64_t n, uint32_t* S, uint32_t* E,
                                           uint32_t* B) {
  const uint4 a = *reinterpret_cast<const uint4*>(text + p);
  const uint32_t nxt = (uint32_t)text[p + 16];
  const uint32_t prev = (p == 0) ? 0u : (uint32_t)text[p - 1];
  const uint32_t w[4] = {a.x, a.y, a.z, a.w};
  bool ws[18];
  ws[0] = is_ws(prev);
#pragma unroll
  for (int k = 0; k < 16; ++k) ws[k + 1] = is_ws((w[k >> 2] >> (8 * (k & 3))) & 0xffu) | (p + k >= n);
  ws[17] = is_ws(nxt) | (p + 16 >= n);
  uint32_t s = 0, e = 0, b = 0;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    s |= (uint32_t)(!ws[k + 1] && ws[k]) << k;
    e |= (uint32_t)(!ws[k + 1] && ws[k + 2]) << k;
    b |= (uint32_t)(!ws[k + 1]) << k;
  }
  *S = s;
  *E = e;
  *B = b;
}

__global__ __launch_bounds__(NT) void k_tok_count2(const uint8_t* __restrict__ text, int64_t n,
                                                  uint32_t* __restrict__ tile_words,
                                                  uint32_t* __restrict__ tile_bytes) {
  __shared__ uint32_t sh[2][NT / MRH_WAVE];
  const int64_t p = (int64_t)blockIdx.x * TILE + (int64_t)threadIdx.x * 16;
  uint32_t cw = 0, cb = 0;
  if (p < n) {
    uint32_t S, E, B;
    word_masks(text, p, n, &S, &E, &B);
    cw = (uint32_t)__popc(S);
    cb = (uint32_t)(__popc(B) + __popc(E));
  }
  cw = dev::wave_sum(cw);
  cb = dev::wave_sum(cb);
  if (dev::lane_id() == 0) {
    sh[0][dev::wave_id()] = cw;
    sh[1][dev::wave_id()] = cb;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    tile_words[blockIdx.x] = sh[0][0] + sh[0][1] + sh[0][2] + sh[0][3];
    tile_bytes[blockIdx.x] = sh[1][0] + sh[1][1] + sh[1][2] + sh[1][3];
  }
}

// The block stages its output in LDS — key bytes at their offset from the
// 16-byte-aligned base below the block's first byte, word offsets in word
// order — then writes both with coalesced stores: 16-byte stores for the
// aligned interior of the key bytes (byte stores only at the block's two
// ragged ends, never past its own range), one int64 store per offset. (Each
// thread writing its own bytes and offsets straight to memory left every
// store instruction touching ~16 scattered cache lines.)
__global__ __launch_bounds__(NT) void k_tok_emit2(const uint8_t* __restrict__ text, int64_t n,
                                                 const uint32_t* __restrict__ toff_w,
                                                 const int64_t* __restrict__ toff_b,
                                                 int64_t* __restrict__ koff, uint8_t* __restrict__ kd) {
  __shared__ uint32_t shw[NT / MRH_WAVE + 1];
  __shared__ uint32_t shb[NT / MRH_WAVE + 1];
  __shared__ __attribute__((aligned(16))) uint8_t sbytes[2 * TILE + 16];  // <= 2 bytes per text byte (a NUL per word)
  __shared__ int64_t soffs[TILE / 2 + 1];                                // <= 1 word per 2 text bytes
  const int64_t p = (int64_t)blockIdx.x * TILE + (int64_t)threadIdx.x * 16;
  uint32_t S = 0, E = 0, B = 0;
  if (p < n) word_masks(text, p, n, &S, &E, &B);
  uint32_t tw, tb;
  const uint32_t pw = dev::block_excl_scan<uint32_t, NT>((uint32_t)__popc(S), shw, &tw);
  const uint32_t pb = dev::block_excl_scan<uint32_t, NT>((uint32_t)(__popc(B) + __popc(E)), shb, &tb);
  const int64_t wb = (int64_t)toff_w[blockIdx.x];
  const int64_t ob = toff_b[blockIdx.x];
  const int lead = (int)((reinterpret_cast<uintptr_t>(kd) + (uintptr_t)ob) & 15);  // LDS index of byte ob: 16-aligned addresses stay 16-aligned
  if (S | B) {
    uint32_t w = pw, o = pb;
    const uint4 a = *reinterpret_cast<const uint4*>(text + p);
    const uint32_t wd[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      if ((S >> k) & 1u) soffs[w++] = ob + o;
      if ((B >> k) & 1u) sbytes[lead + o++] = (uint8_t)((wd[k >> 2] >> (8 * (k & 3))) & 0xffu);
      if ((E >> k) & 1u) sbytes[lead + o++] = 0;
    }
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < tw; i += NT) koff[wb + i] = soffs[i];
  // key bytes [ob, ob + tb) in 16-byte chunks of the aligned base ob - lead
  const int64_t base = ob - lead, end = ob + tb;
  const int64_t nchunk = (end - base + 15) >> 4;
  for (int64_t c = threadIdx.x; c < nchunk; c += NT) {
    const int64_t g0 = base + 16 * c;
    if (g0 >= ob && g0 + 16 <= end) {
      *reinterpret_cast<uint4*>(kd + g0) = *reinterpret_cast<const uint4*>(sbytes + 16 * c);
    } else {
      for (int k = 0; k < 16; ++k) {
        const int64_t g = g0 + k;
        if (g >= ob && g < end) kd[g] = sbytes[16 * c + k];
      }
    }
  }
}

// 16 lanes per string
__global__ __launch_bounds__(NT) void k_copy_nul(const uint8_t* __restrict__ text,
                                                const int64_t* __restrict__ starts,
                                                const int64_t* __restrict__ koff, int64_t n,
                                                uint8_t* __restrict__ kd) {
  const int g = threadIdx.x & 15;
  int64_t row = ((int64_t)blockIdx.x * NT + threadIdx.x) >> 4;
  const int64_t stride = ((int64_t)gridDim.x * NT) >> 4;
  for (; row < n; row += stride) {
    int64_t a = starts[row], o = koff[row], len = koff[row + 1] - o - 1;
    for (int64_t j = g; j < len; j += 16) kd[o + j] = text[a + j];
    if (g == 0) kd[o + len] = 0;
  }
}

__global__ __launch_bounds__(NT) void k_fill_i32(int32_t* p, int64_t n, int32_t v) {
  int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (i < n) p[i] = v;
}

}  // namespace

int64_t url_num_tiles(int64_t n) { return (n + TILE - 1) / TILE; }
int64_t tok_num_tiles(int64_t n) { return (n + TILE - 1) / TILE; }

void url_count(const uint8_t* text, int64_t n, uint32_t* tile_counts, hipStream_t s) {
  int64_t nt = url_num_tiles(n);
  if (nt <= 0) return;
  hipLaunchKernelGGL(k_url_count, dim3((unsigned)nt), dim3(NT), 0, s, text, n, tile_counts);
  MRH_CHECK_LAUNCH();
}
void url_emit_starts(const uint8_t* text, int64_t n, const uint32_t* tile_off, int64_t* starts,
                     hipStream_t s) {
  int64_t nt = url_num_tiles(n);
  if (nt <= 0) return;
  hipLaunchKernelGGL(k_url_emit, dim3((unsigned)nt), dim3(NT), 0, s, text, n, tile_off, starts);
  MRH_CHECK_LAUNCH();
}
void url_lengths(const uint8_t* text, int64_t n, const int64_t* starts, int64_t nurl, int32_t* keylen,
                 hipStream_t s) {
  if (nurl <= 0) return;
  hipLaunchKernelGGL(k_url_len, dim3((unsigned)((nurl + NT - 1) / NT)), dim3(NT), 0, s, text, n, starts,
                     nurl, keylen);
  MRH_CHECK_LAUNCH();
}
void copy_strings_nul(const uint8_t* text, const int64_t* starts, const int64_t* koff, int64_t n,
                      uint8_t* kdata, hipStream_t s) {
  if (n <= 0) return;
  int64_t g = (n * 16 + NT - 1) / NT;
  if (g > 65536) g = 65536;
  hipLaunchKernelGGL(k_copy_nul, dim3((unsigned)g), dim3(NT), 0, s, text, starts, koff, n, kdata);
  MRH_CHECK_LAUNCH();
}
void url_copy(const uint8_t* text, const int64_t* starts, const int64_t* koff, int64_t nurl,
              uint8_t* kdata, hipStream_t s) {
  copy_strings_nul(text, starts, koff, nurl, kdata, s);
}
void tok_count2(const uint8_t* text, int64_t n, uint32_t* tile_words, uint32_t* tile_bytes, hipStream_t s) {
  const int64_t nt = tok_num_tiles(n);
  if (nt <= 0) return;
  hipLaunchKernelGGL(k_tok_count2, dim3((unsigned)nt), dim3(NT), 0, s, text, n, tile_words, tile_bytes);
  MRH_CHECK_LAUNCH();
}
void tok_emit2(const uint8_t* text, int64_t n, const uint32_t* toff_w, const int64_t* toff_b, int64_t* koff,
               uint8_t* kd, hipStream_t s) {
  const int64_t nt = tok_num_tiles(n);
  if (nt <= 0) return;
  hipLaunchKernelGGL(k_tok_emit2, dim3((unsigned)nt), dim3(NT), 0, s, text, n, toff_w, toff_b, koff, kd);
  MRH_CHECK_LAUNCH();
}
void tok_count(const uint8_t* text, int64_t n, uint32_t* tile_counts, hipStream_t s) {
  int64_t nt = tok_num_tiles(n);
  if (nt <= 0) return;
  hipLaunchKernelGGL(k_tok_count, dim3((unsigned)nt), dim3(NT), 0, s, text, n, tile_counts);
  MRH_CHECK_LAUNCH();
}
void tok_emit(const uint8_t* text, int64_t n, const uint32_t* tile_off, int64_t* starts, int32_t* keylen,
              hipStream_t s) {
  int64_t nt = tok_num_tiles(n);
  if (nt <= 0) return;
  hipLaunchKernelGGL(k_tok_emit, dim3((unsigned)nt), dim3(NT), 0, s, text, n, tile_off, starts, keylen);
  MRH_CHECK_LAUNCH();
}
void fill_i32(int32_t* p, int64_t n, int32_t v, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_fill_i32, dim3((unsigned)((n + NT - 1) / NT)), dim3(NT), 0, s, p, n, v);
  MRH_CHECK_LAUNCH();
}

}  // namespace k
}  // namespace mrh
