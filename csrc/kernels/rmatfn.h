// Host+device R-MAT edge generator (shared by graph.hip and the CPU engine
// path so both produce bit-identical graphs). Quadrant rule and per-level
// noise follow oink/map_rmat_generate.cpp:32-66; the random stream is
// Philox4x32-7 keyed by the seed and countered by (edge id, block), so an
// edge is a pure function of (seed, edge id). One Philox call gives eight
// 16-bit uniforms (a quadrant choice against a, b, c of ~0.2-0.6 needs no
// more resolution): an RMAT-26 edge costs 4 calls x 7 rounds instead of 7 x 10
// — the generator was bound by the rounds' 32-bit multiplies (24 ms of an
// RMAT-26 setup, profiles/r4_pagerank_setup_stages.txt). Philox4x32-7 is the
// fewest rounds the Random123 authors found Crush-resistant.
#pragma once
#include <cstdint>
#include "hashfn.h"

namespace mrh {
namespace dev {

struct u32x4 { uint32_t x, y, z, w; };

MRH_HD inline uint32_t mulhi32(uint32_t a, uint32_t b) { return (uint32_t)(((uint64_t)a * b) >> 32); }

template <int ROUNDS>
MRH_HD inline u32x4 philox4x32(u32x4 c, uint32_t k0, uint32_t k1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < ROUNDS; ++r) {
    uint32_t hi0 = mulhi32(M0, c.x), lo0 = M0 * c.x;
    uint32_t hi1 = mulhi32(M1, c.z), lo1 = M1 * c.z;
    c = u32x4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    k0 += W0;
    k1 += W1;
  }
  return c;
}

MRH_HD inline float u01_16(uint32_t x) { return (float)(x & 0xFFFFu) * (1.0f / 65536.0f); }

struct RmatRng {
  uint64_t ge;
  uint32_t k0, k1, blk;
  u32x4 r;
  int used;
  MRH_HD inline float next() {  // the 8 halves of a call, low half first
    if (used == 8) {
      r = philox4x32<7>(u32x4{(uint32_t)ge, (uint32_t)(ge >> 32), blk++, 0x52u}, k0, k1);
      used = 0;
    }
    const int w = used >> 1;
    uint32_t v = w == 0 ? r.x : w == 1 ? r.y : w == 2 ? r.z : r.w;
    if (used & 1) v >>= 16;
    ++used;
    return u01_16(v);
  }
};

MRH_HD inline void rmat_edge(uint64_t ge, int nlevels, float a, float b, float c, float d, float fraction,
                             uint64_t seed, uint64_t* vi, uint64_t* vj) {
  RmatRng rng{ge, (uint32_t)seed, (uint32_t)(seed >> 32), 0u, u32x4{0, 0, 0, 0}, 8};
  uint64_t i = 0, j = 0;
  uint64_t delta = (nlevels >= 1) ? (1ull << (nlevels - 1)) : 0ull;
  float a1 = a, b1 = b, c1 = c, d1 = d;
  for (int l = 0; l < nlevels; ++l) {
    float rn = rng.next();
    if (rn < a1) {
    } else if (rn < a1 + b1) {
      j += delta;
    } else if (rn < a1 + b1 + c1) {
      i += delta;
    } else {
      i += delta;
      j += delta;
    }
    delta >>= 1;
    if (fraction > 0.0f) {
      a1 += a1 * fraction * (rng.next() - 0.5f);
      b1 += b1 * fraction * (rng.next() - 0.5f);
      c1 += c1 * fraction * (rng.next() - 0.5f);
      d1 += d1 * fraction * (rng.next() - 0.5f);
      float t = a1 + b1 + c1 + d1;
      a1 /= t; b1 /= t; c1 /= t; d1 /= t;
    }
  }
  *vi = i;
  *vj = j;
}

}  // namespace dev
}  // namespace mrh
