// Shuffle partition kernels: the device side of MapReduce::aggregate's
// per-KV owner computation and send-buffer packing (reference hot loops C1/C2:
// hash loop src/mapreduce.cpp:453-473, pack loop src/irregular.cpp:283-288).
//
// Two passes over fixed tiles of TILE = 256 x 16 pairs (block b owns pairs
// [b*TILE, (b+1)*TILE), pair i of round r at i = b*TILE + r*256 + threadIdx.x,
// so every global read is coalesced):
//
//  k_part_count   owner d = hashlittle(key, kb, P) % P (or a given dest),
//                 per-(d, block) pair counts and, for variable-width columns,
//                 key / value byte sums -> cnt[d*nb + b] (d-major, so one
//                 exclusive scan gives every (d, b) its base in a bucketed
//                 send buffer where bucket d is contiguous);
//  k_part_scatter stable in-tile rank of each pair among the pairs with the
//                 same owner: wave64 "match any" (one ballot per distinct
//                 owner present in the wave, <= min(64, P)), per-wave counts
//                 in LDS, prefix over the 4 waves, running per-owner base.
//                 Fixed-width columns are moved straight into the send
//                 buffer (the pack IS the scatter: no permutation gather, no
//                 second pass); variable-width columns get the permutation +
//                 lengths, and the bytes follow in one cooperative copy after
//                 a scan of the lengths.
//
// Stable means the send buffer (and so the receiver's pairs from each sender)
// keeps input order: the shuffle is deterministic.
#include <string>

#include "common.h"
#include "launch.h"

namespace mrh {
namespace k {
namespace {

constexpr int NT = 256, NW = NT / MRH_WAVE, IPT = 16, TILE = NT * IPT, PMAX = 1024;

// lanes of this wave with the same owner (match-any emulation) ; -1 = no pair
__device__ __forceinline__ uint64_t match_owner(int d) {
  uint64_t active = __ballot(d >= 0), mine = 0;
  while (active) {
    const int leader = __ffsll((unsigned long long)active) - 1;
    const int ld = __shfl(d, leader, MRH_WAVE);
    const uint64_t m = __ballot(d == ld);
    if (d == ld) mine = m;
    active &= ~m;
  }
  return mine;
}

template <int MODE>  // 0: dest given, 1: hash fixed-width keys, 2: hash variable keys
__device__ __forceinline__ int owner(int64_t i, const int32_t* dest_in, const uint8_t* kd, int kw,
                                     const int64_t* koff, int P) {
  if (MODE == 0) return dest_in[i];
  uint32_t h;
  if (MODE == 1) {
    h = dev::hashlittle(kd + i * kw, kw, (uint32_t)P);
  } else {
    uint32_t c = (uint32_t)P, b = 0;
    const int64_t a = koff[i];
    dev::lookup3_wide(kd + a, koff[i + 1] - a, &c, &b);
    h = c;
  }
  return (int)(h % (uint32_t)P);
}

template <int MODE>
__global__ __launch_bounds__(NT) void k_part_count(const int32_t* __restrict__ dest_in, const uint8_t* __restrict__ kd,
                                                  int kw, const int64_t* __restrict__ koff,
                                                  const int64_t* __restrict__ voff, int64_t n, int P, int nb,
                                                  int32_t* __restrict__ dest_out, int64_t* __restrict__ cnt,
                                                  int64_t* __restrict__ kbytes, int64_t* __restrict__ vbytes) {
  __shared__ uint32_t hc[PMAX];
  __shared__ unsigned long long hk[PMAX], hv[PMAX];
  for (int d = threadIdx.x; d < P; d += NT) {
    hc[d] = 0;
    hk[d] = 0;
    hv[d] = 0;
  }
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * TILE;
  const int lane = dev::lane_id();
  for (int r = 0; r < IPT; ++r) {
    const int64_t i = base + r * NT + threadIdx.x;
    const bool valid = i < n;
    int d = -1;
    unsigned long long kl = 0, vl = 0;
    if (valid) {
      d = owner<MODE>(i, dest_in, kd, kw, koff, P);
      if (MODE != 0) dest_out[i] = d;
      if (kbytes) kl = (unsigned long long)(koff[i + 1] - koff[i]);
      if (vbytes) vl = (unsigned long long)(voff[i + 1] - voff[i]);
    }
    // per distinct owner in the wave: its pair count and byte sums by wave
    // reductions, one LDS atomic each by the group's leader (a per-lane
    // atomic on the same owner serialised 64-fold at small P)
    uint64_t active = __ballot(d >= 0);
    while (active) {
      const int leader = __ffsll((unsigned long long)active) - 1;
      const int ld = __shfl(d, leader, MRH_WAVE);
      const bool in = d == ld;
      const uint64_t m = __ballot(in);
      const unsigned long long ks = kbytes ? dev::wave_sum(in ? kl : 0ull) : 0ull;
      const unsigned long long vs = vbytes ? dev::wave_sum(in ? vl : 0ull) : 0ull;
      if (lane == leader) {
        atomicAdd(&hc[ld], (uint32_t)__popcll(m));
        if (kbytes) atomicAdd(&hk[ld], ks);
        if (vbytes) atomicAdd(&hv[ld], vs);
      }
      active &= ~m;
    }
  }
  __syncthreads();
  for (int d = threadIdx.x; d < P; d += NT) {
    const int64_t o = (int64_t)d * nb + blockIdx.x;
    cnt[o] = hc[d];
    if (kbytes) kbytes[o] = (int64_t)hk[d];
    if (vbytes) vbytes[o] = (int64_t)hv[d];
  }
}

// copy one fixed-width row (w bytes) with the widest aligned word size
__device__ __forceinline__ void copy_row(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, int w) {
  if ((w & 7) == 0) {
    const uint64_t* s = reinterpret_cast<const uint64_t*>(src);
    uint64_t* t = reinterpret_cast<uint64_t*>(dst);
    for (int j = 0; j < (w >> 3); ++j) t[j] = s[j];
  } else if ((w & 3) == 0) {
    const uint32_t* s = reinterpret_cast<const uint32_t*>(src);
    uint32_t* t = reinterpret_cast<uint32_t*>(dst);
    for (int j = 0; j < (w >> 2); ++j) t[j] = s[j];
  } else {
    for (int j = 0; j < w; ++j) dst[j] = src[j];
  }
}

__global__ __launch_bounds__(NT) void k_part_scatter(const int32_t* __restrict__ dest, int64_t n, int P, int nb,
                                                    const int64_t* __restrict__ cbase,
                                                    const uint8_t* __restrict__ kd, int kw,
                                                    const uint8_t* __restrict__ vd, int vw,
                                                    const int64_t* __restrict__ koff,
                                                    const int64_t* __restrict__ voff,
                                                    uint8_t* __restrict__ ksend, uint8_t* __restrict__ vsend,
                                                    int64_t* __restrict__ perm, int32_t* __restrict__ klen,
                                                    int32_t* __restrict__ vlen) {
  __shared__ int64_t run[PMAX];
  __shared__ uint32_t wc[NW][PMAX];
  for (int d = threadIdx.x; d < P; d += NT) {
    run[d] = cbase[(int64_t)d * nb + blockIdx.x];
#pragma unroll
    for (int w = 0; w < NW; ++w) wc[w][d] = 0;
  }
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * TILE;
  const int lane = dev::lane_id(), wv = dev::wave_id();
  for (int r = 0; r < IPT; ++r) {
    if (base + r * NT >= n) break;  // block-uniform
    const int64_t i = base + r * NT + threadIdx.x;
    const bool valid = i < n;
    const int d = valid ? dest[i] : -1;
    const uint64_t peers = match_owner(d);
    const bool leader = valid && (__ffsll((unsigned long long)peers) - 1) == lane;
    if (leader) wc[wv][d] = (uint32_t)__popcll(peers);
    __syncthreads();
    if (valid) {
      int64_t pos = run[d] + (int64_t)__popcll(peers & dev::lanemask_lt());
      for (int w = 0; w < wv; ++w) pos += wc[w][d];
      if (kw >= 0) copy_row(kd + i * kw, ksend + pos * kw, kw);
      if (vw >= 0) copy_row(vd + i * vw, vsend + pos * vw, vw);
      if (perm) perm[pos] = i;
      if (klen) klen[pos] = (int32_t)(koff[i + 1] - koff[i]);
      if (vlen) vlen[pos] = (int32_t)(voff[i + 1] - voff[i]);
    }
    __syncthreads();
    for (int dd = threadIdx.x; dd < P; dd += NT) {
      uint32_t s = 0;
#pragma unroll
      for (int w = 0; w < NW; ++w) s += wc[w][dd];
      run[dd] += s;
    }
    __syncthreads();
    if (leader) wc[wv][d] = 0;
  }
}

// variable rows gathered by an int64 permutation. One wave per tile of 64
// rows copies the tile's destination bytes [doff[r0], doff[r0 + 64)) with all
// 64 lanes busy: lane l owns byte base + l of each 64-byte step and finds its
// row by a binary search over the tile's destination offsets (held one per
// lane, read with shuffles). The stores of a step are one contiguous 64-byte
// run (the 16-lanes-per-row version left 9 of 16 lanes idle on ~7-byte words
// and scattered its stores: 61 ms for wordfreq's 1.15 G keys).
__global__ __launch_bounds__(NT) void k_copy_var_i64(const uint8_t* __restrict__ src, const int64_t* __restrict__ soff,
                                                    const int64_t* __restrict__ perm, int64_t n,
                                                    uint8_t* __restrict__ dst, const int64_t* __restrict__ doff) {
  const int lane = threadIdx.x & 63;
  const int64_t ntile = (n + 63) >> 6;
  const int64_t nwave = ((int64_t)gridDim.x * NT) >> 6;
  for (int64_t t = ((int64_t)blockIdx.x * NT + threadIdx.x) >> 6; t < ntile; t += nwave) {
    const int64_t r0 = t << 6;
    const int rows = (int)min<int64_t>(64, n - r0);
    // this lane's row: its destination start and source start
    int64_t dv = 0, sv = 0;
    if (lane < rows) {
      dv = doff[r0 + lane];
      sv = soff[perm[r0 + lane]];
    }
    const int64_t d_lo = __shfl(dv, 0, 64);
    const int64_t d_hi = doff[r0 + rows];  // same address on every lane: one broadcast load
    for (int64_t base = d_lo; base < d_hi; base += 64) {  // uniform over the wave
      const int64_t b = base + lane;
      // largest row i < rows with doff[r0 + i] <= b (rows are non-empty or
      // empty; an empty row shares its start with the next and loses the tie)
      int lo = 0;
#pragma unroll
      for (int step = 32; step >= 1; step >>= 1) {
        const int cand = lo + step;
        const int64_t dc = __shfl(dv, cand & 63, 64);
        if (cand < rows && dc <= b) lo = cand;
      }
      const int64_t drow = __shfl(dv, lo, 64), srow = __shfl(sv, lo, 64);
      if (b < d_hi) dst[b] = src[srow + (b - drow)];
    }
  }
}

// The same gather by block tiles of 256 rows: the tile's destination
// offsets and source starts are staged in LDS once; every lane owns 16
// consecutive destination bytes per step (4 KiB per block step), finds the
// row of its first byte by a binary search in LDS and walks on across row
// boundaries (empty rows included), gathers its bytes and writes them with one
// 16-byte store (byte stores only at a tile's ragged ends). No cross-lane
// shuffles per byte: the wave version spends 8 per byte. dst 16-aligned.
constexpr int CV_ROWS = NT;
__global__ __launch_bounds__(NT) void k_copy_var_blk(const uint8_t* __restrict__ src, const int64_t* __restrict__ soff,
                                                    const int64_t* __restrict__ perm, int64_t n,
                                                    uint8_t* __restrict__ dst, const int64_t* __restrict__ doff) {
  __shared__ int64_t ldo[CV_ROWS + 1];
  __shared__ int64_t lso[CV_ROWS];
  const int t = threadIdx.x;
  const int64_t ntile = (n + CV_ROWS - 1) / CV_ROWS;
  for (int64_t tile = blockIdx.x; tile < ntile; tile += gridDim.x) {  // uniform over the block
    const int64_t r0 = tile * CV_ROWS;
    const int rows = (int)min<int64_t>(CV_ROWS, n - r0);
    if (t < rows) {
      ldo[t] = doff[r0 + t];
      lso[t] = soff[perm[r0 + t]];
    }
    if (t == 0) ldo[rows] = doff[r0 + rows];
    __syncthreads();
    const int64_t d_lo = ldo[0], d_hi = ldo[rows];
    for (int64_t base = (d_lo & ~int64_t(15)) + 16 * (int64_t)t; base < d_hi; base += 16 * NT) {
      const int64_t q = base < d_lo ? d_lo : base;
      int lo = 0, hi = rows - 1;  // the last row starting at or before q (an empty row loses the tie)
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (ldo[mid] <= q) lo = mid;
        else hi = mid - 1;
      }
      int r = lo;
      int64_t rbeg = ldo[r], rend = ldo[r + 1], sbeg = lso[r];
      uint32_t wv[4] = {0, 0, 0, 0};
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int64_t pos = base + k;
        if (pos >= d_lo && pos < d_hi) {
          while (pos >= rend) {
            ++r;
            rbeg = rend;
            rend = ldo[r + 1];
            sbeg = lso[r];
          }
          wv[k >> 2] |= (uint32_t)src[sbeg + (pos - rbeg)] << (8 * (k & 3));
        }
      }
      if (base >= d_lo && base + 16 <= d_hi) {
        *reinterpret_cast<uint4*>(dst + base) = make_uint4(wv[0], wv[1], wv[2], wv[3]);
      } else {
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          const int64_t pos = base + k;
          if (pos >= d_lo && pos < d_hi) dst[pos] = (uint8_t)(wv[k >> 2] >> (8 * (k & 3)));
        }
      }
    }
    __syncthreads();  // the next tile overwrites the staged offsets
  }
}

// header row of this rank for the exchange: per owner d {pairs, key bytes,
// value bytes} from the scanned per-(d, block) tables (fixed columns: count x
// width), then the two width codes
__global__ void k_part_header(const int64_t* __restrict__ cs, const int64_t* __restrict__ ks,
                              const int64_t* __restrict__ vs, int P, int nb, int kw, int vw, int64_t kcode,
                              int64_t vcode, int64_t* __restrict__ hdr) {
  for (int d = threadIdx.x; d < P; d += blockDim.x) {
    const int64_t a = (int64_t)d * nb, b = a + nb;
    const int64_t c = cs[b] - cs[a];
    hdr[3 * d + 0] = c;
    hdr[3 * d + 1] = kw >= 0 ? c * kw : ks[b] - ks[a];
    hdr[3 * d + 2] = vw >= 0 ? c * vw : vs[b] - vs[a];
  }
  if (threadIdx.x == 0) {
    hdr[3 * P] = kcode;
    hdr[3 * P + 1] = vcode;
  }
}

// bytes of piece k of bucket d (pairs [start_d + c_d*k/R, start_d + c_d*(k+1)/R))
// of a variable column whose send offsets are soff (n+1)
__global__ void k_piece_bytes(const int64_t* __restrict__ soff, const int64_t* __restrict__ start, int P, int R,
                              int64_t* __restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)P * R) return;
  const int d = (int)(t / R), k = (int)(t % R);
  const int64_t s = start[d], c = start[d + 1] - s;
  const int64_t a = s + c * k / R, b = s + c * (k + 1) / R;
  out[t] = soff[b] - soff[a];
}

// counts[v % P] over an int64 id column: LDS histogram per block, one global
// atomic per (block, bin)
__global__ __launch_bounds__(NT) void k_count_mod(const int64_t* __restrict__ v, int64_t n, int P,
                                                 int64_t* __restrict__ counts) {
  __shared__ uint32_t h[PMAX];
  for (int d = threadIdx.x; d < P; d += NT) h[d] = 0;
  __syncthreads();
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT)
    atomicAdd(&h[(int)(v[i] % P)], 1u);
  __syncthreads();
  for (int d = threadIdx.x; d < P; d += NT)
    if (h[d]) atomicAdd((unsigned long long*)&counts[d], (unsigned long long)h[d]);
}

}  // namespace

int part_tile() { return TILE; }

void count_mod(const int64_t* v, int64_t n, int P, int64_t* counts, hipStream_t s) {
  if (n <= 0) return;
  check_arg(P >= 1 && P <= PMAX, "count_mod: 1 <= P <= 1024");
  int64_t g = (n + NT - 1) / NT;
  if (g > 2048) g = 2048;
  hipLaunchKernelGGL(k_count_mod, dim3((unsigned)g), dim3(NT), 0, s, v, n, P, counts);
  MRH_CHECK_LAUNCH();
}

void part_count(const int32_t* dest_in, const uint8_t* kd, int kw, const int64_t* koff, const int64_t* voff,
                int64_t n, int P, int nb, int32_t* dest_out, int64_t* cnt, int64_t* kbytes, int64_t* vbytes,
                hipStream_t s) {
  if (nb <= 0) return;
  check_arg(P >= 1 && P <= PMAX, "part_count: 1 <= P <= 1024");
  if (dest_in)
    hipLaunchKernelGGL(k_part_count<0>, dim3(nb), dim3(NT), 0, s, dest_in, kd, kw, koff, voff, n, P, nb, dest_out,
                       cnt, kbytes, vbytes);
  else if (koff)
    hipLaunchKernelGGL(k_part_count<2>, dim3(nb), dim3(NT), 0, s, dest_in, kd, kw, koff, voff, n, P, nb, dest_out,
                       cnt, kbytes, vbytes);
  else
    hipLaunchKernelGGL(k_part_count<1>, dim3(nb), dim3(NT), 0, s, dest_in, kd, kw, koff, voff, n, P, nb, dest_out,
                       cnt, kbytes, vbytes);
  MRH_CHECK_LAUNCH();
}

void part_scatter(const int32_t* dest, int64_t n, int P, int nb, const int64_t* cbase, const uint8_t* kd, int kw,
                  const uint8_t* vd, int vw, const int64_t* koff, const int64_t* voff, uint8_t* ksend,
                  uint8_t* vsend, int64_t* perm, int32_t* klen, int32_t* vlen, hipStream_t s) {
  if (nb <= 0 || n <= 0) return;
  check_arg(P >= 1 && P <= PMAX, "part_scatter: 1 <= P <= 1024");
  hipLaunchKernelGGL(k_part_scatter, dim3(nb), dim3(NT), 0, s, dest, n, P, nb, cbase, kd, kw, vd, vw, koff, voff,
                     ksend, vsend, perm, klen, vlen);
  MRH_CHECK_LAUNCH();
}

void copy_var_i64(const uint8_t* src, const int64_t* soff, const int64_t* perm, int64_t n, uint8_t* dst,
                  const int64_t* doff, hipStream_t s) {
  if (n <= 0) return;
  static const bool wave = [] {  // MRH_COPY_VAR=wave: the wave-per-64-rows version (A/B)
    const char* e = std::getenv("MRH_COPY_VAR");
    return e && std::string(e) == "wave";
  }();
  if (!wave && (reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
    const int64_t g = std::min<int64_t>((n + CV_ROWS - 1) / CV_ROWS, 65536);
    hipLaunchKernelGGL(k_copy_var_blk, dim3((unsigned)g), dim3(NT), 0, s, src, soff, perm, n, dst, doff);
    MRH_CHECK_LAUNCH();
    return;
  }
  int64_t g = ((n + 63) / 64 * 64 + NT - 1) / NT;  // a wave per 64-row tile
  if (g > 65536) g = 65536;
  hipLaunchKernelGGL(k_copy_var_i64, dim3((unsigned)g), dim3(NT), 0, s, src, soff, perm, n, dst, doff);
  MRH_CHECK_LAUNCH();
}

void part_header(const int64_t* cs, const int64_t* ks, const int64_t* vs, int P, int nb, int kw, int vw,
                 int64_t kcode, int64_t vcode, int64_t* hdr, hipStream_t s) {
  hipLaunchKernelGGL(k_part_header, dim3(1), dim3(256), 0, s, cs, ks, vs, P, nb, kw, vw, kcode, vcode, hdr);
  MRH_CHECK_LAUNCH();
}

void piece_bytes(const int64_t* soff, const int64_t* start, int P, int R, int64_t* out, hipStream_t s) {
  const int64_t t = (int64_t)P * R;
  if (t <= 0) return;
  hipLaunchKernelGGL(k_piece_bytes, dim3((unsigned)((t + 255) / 256)), dim3(256), 0, s, soff, start, P, R, out);
  MRH_CHECK_LAUNCH();
}

}  // namespace k
}  // namespace mrh
