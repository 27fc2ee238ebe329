// Host+device bijection of the vertex ids [0, N) used to pick the owner rank
// of a vertex in the multi-GPU PageRank plan: owner = sigma(v) % P, local id =
// sigma(v) / P.
//
// Why not v % P (the edge plan's rule, and MR-MPI's owner of an integer key
// when hashed by value): R-MAT ids are not scrambled (the generator is the
// reference's quadrant rule, oink/map_rmat_generate.cpp:32-66), so every id
// bit is 1 with probability c + d = 0.24 for sources and b + d = 0.24 for
// destinations. v % 8 then gives rank 0 0.76^3 = 44 % of the edges and rank 7
// 1.4 % — an 8-GPU job would run at the speed of its first rank. sigma mixes
// every bit of v into the low bits: two rounds of (odd multiply, xorshift) on
// b = ceil(log2 N) bits, each a bijection of [0, 2^b), and cycle walking
// (repeat until < N) makes it a bijection of [0, N) for any N.
#pragma once
#include <cstdint>

#include "hashfn.h"

namespace mrh {
namespace dev {

constexpr uint64_t VMIX_K1 = 0x9E3779B97F4A7C15ull, VMIX_K2 = 0xD6E8FEB86659FD93ull;

// inverse of an odd number mod 2^64 (Newton: each step doubles the good bits)
MRH_HD constexpr uint64_t vmix_inv(uint64_t k) {
  uint64_t x = k;
  for (int i = 0; i < 6; ++i) x *= 2 - k * x;
  return x;
}

MRH_HD inline uint64_t vmix_round(uint64_t x, int b, uint64_t mask) {
  const int s = (b + 1) / 2;
  x = (x * VMIX_K1) & mask;
  x ^= x >> s;
  x = (x * VMIX_K2) & mask;
  x ^= x >> s;
  return x;
}

MRH_HD inline uint64_t vmix_unround(uint64_t y, int b, uint64_t mask) {
  const int s = (b + 1) / 2;
  // y = x ^ (x >> s)  =>  x = y ^ (x >> s), exact after ceil(b / s) steps
  uint64_t x = y;
  for (int t = 0; t < b; t += s) x = y ^ (x >> s);
  x = (x * vmix_inv(VMIX_K2)) & mask;
  y = x;
  for (int t = 0; t < b; t += s) x = y ^ (x >> s);
  return (x * vmix_inv(VMIX_K1)) & mask;
}

// bits of the mixing domain: smallest b with 2^b >= n
MRH_HD inline int vmix_bits(int64_t n) {
  int b = 0;
  while (b < 62 && (int64_t(1) << b) < n) ++b;
  return b;
}

// sigma(v) for v in [0, n), b = vmix_bits(n)
MRH_HD inline uint64_t vmix(uint64_t v, int64_t n, int b) {
  const uint64_t mask = b >= 64 ? ~0ull : ((1ull << b) - 1);
  uint64_t x = vmix_round(v, b, mask);
  while (x >= (uint64_t)n) x = vmix_round(x, b, mask);  // cycle walking: < 2 rounds expected
  return x;
}

MRH_HD inline uint64_t vunmix(uint64_t y, int64_t n, int b) {
  const uint64_t mask = b >= 64 ? ~0ull : ((1ull << b) - 1);
  uint64_t x = vmix_unround(y, b, mask);
  while (x >= (uint64_t)n) x = vmix_unround(x, b, mask);
  return x;
}

}  // namespace dev
}  // namespace mrh
