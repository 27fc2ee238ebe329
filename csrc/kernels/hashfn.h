// Host+device hash and sort-key helpers (usable from g++ host code and hipcc
// device code). lookup3 is Bob Jenkins' public-domain hash, re-expressed from
// its published description; MR-MPI partitions with hashlittle()
// (reference src/hash.cpp:129-298, src/mapreduce.cpp:472).
#pragma once
#include <cstdint>
#if defined(__HIPCC__)
#define MRH_HD __host__ __device__
#else
#define MRH_HD
#endif

namespace mrh {
namespace dev {

// lookup3 (Bob Jenkins, public domain algorithm) — written from the published
// specification; bit-exact with hashlittle()/hashlittle2() on little-endian.
MRH_HD inline uint32_t rot32(uint32_t x, int k) {
  return (x << k) | (x >> (32 - k));
}
#define MRH_L3_MIX(a, b, c)   \
  {                           \
    a -= c; a ^= rot32(c, 4);  c += b; \
    b -= a; b ^= rot32(a, 6);  a += c; \
    c -= b; c ^= rot32(b, 8);  b += a; \
    a -= c; a ^= rot32(c, 16); c += b; \
    b -= a; b ^= rot32(a, 19); a += c; \
    c -= b; c ^= rot32(b, 4);  b += a; \
  }
#define MRH_L3_FINAL(a, b, c) \
  {                           \
    c ^= b; c -= rot32(b, 14); \
    a ^= c; a -= rot32(c, 11); \
    b ^= a; b -= rot32(a, 25); \
    c ^= b; c -= rot32(b, 16); \
    a ^= c; a -= rot32(c, 4);  \
    b ^= a; b -= rot32(a, 14); \
    c ^= b; c -= rot32(b, 24); \
  }

// Generic byte-reader form: works for any alignment; `ld` returns byte i.
MRH_HD inline uint32_t le32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

// lookup3 core. Returns c in *pc and b in *pb (hashlittle2 semantics when
// *pb is the secondary seed; hashlittle == hashlittle2 with pb=0, result pc).
MRH_HD inline void lookup3(const uint8_t* k, int64_t length, uint32_t* pc,
                                                 uint32_t* pb) {
  uint32_t a, b, c;
  a = b = c = 0xdeadbeefu + (uint32_t)length + *pc;
  c += *pb;
  while (length > 12) {
    a += le32(k);
    b += le32(k + 4);
    c += le32(k + 8);
    MRH_L3_MIX(a, b, c);
    length -= 12;
    k += 12;
  }
  switch (length) {
    case 12: c += ((uint32_t)k[11]) << 24; [[fallthrough]];
    case 11: c += ((uint32_t)k[10]) << 16; [[fallthrough]];
    case 10: c += ((uint32_t)k[9]) << 8; [[fallthrough]];
    case 9: c += k[8]; [[fallthrough]];
    case 8: b += ((uint32_t)k[7]) << 24; [[fallthrough]];
    case 7: b += ((uint32_t)k[6]) << 16; [[fallthrough]];
    case 6: b += ((uint32_t)k[5]) << 8; [[fallthrough]];
    case 5: b += k[4]; [[fallthrough]];
    case 4: a += ((uint32_t)k[3]) << 24; [[fallthrough]];
    case 3: a += ((uint32_t)k[2]) << 16; [[fallthrough]];
    case 2: a += ((uint32_t)k[1]) << 8; [[fallthrough]];
    case 1: a += k[0]; break;
    case 0: *pc = c; *pb = b; return;
  }
  MRH_L3_FINAL(a, b, c);
  *pc = c;
  *pb = b;
}

MRH_HD inline uint32_t hashlittle(const uint8_t* k, int64_t len, uint32_t seed) {
  uint32_t c = seed, b = 0;
  lookup3(k, len, &c, &b);
  return c;
}
MRH_HD inline uint64_t hash64(const uint8_t* k, int64_t len) {
  uint32_t c = 0x9e3779b9u, b = 0x7f4a7c15u;
  lookup3(k, len, &c, &b);
  return ((uint64_t)c << 32) | b;
}

// Key transforms so that unsigned integer order == requested order.
MRH_HD inline uint64_t sortkey_transform(uint64_t raw, int mode) {
  switch (mode) {
    case 1: return (uint64_t)((uint32_t)raw ^ 0x80000000u);           // int32
    case 3: {                                                         // float
      uint32_t u = (uint32_t)raw;
      // the reference's comparator (src/mapreduce.cpp:2736-2752) has -0.0 ==
      // +0.0: one key, so a stable sort keeps their input order; every NaN
      // is one key above +inf (numpy's order: NaNs last)
      if ((u & 0x7fffffffu) == 0) u = 0;
      else if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x007fffffu)) u = 0x7fc00000u;
      u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
      return u;
    }
    case 4: {                                                         // double
      uint64_t u = raw;
      if ((u & 0x7fffffffffffffffull) == 0) u = 0;
      else if ((u & 0x7ff0000000000000ull) == 0x7ff0000000000000ull && (u & 0x000fffffffffffffull))
        u = 0x7ff8000000000000ull;
      u = (u & 0x8000000000000000ull) ? ~u : (u | 0x8000000000000000ull);
      return u;
    }
    case 7: return raw ^ 0x8000000000000000ull;                      // int64
    case 8: return (uint32_t)raw;                                     // uint32
    default: return raw;                                              // raw / uint64
  }
}

// the radix key of one fixed-width value for flag `mode`, descending when
// `desc`: the complement of the ascending key, except that NaN (flags 3 and
// 4) stays the largest key — NaNs sort last in both directions, like
// numpy / pandas (the reference's comparators leave NaN order undefined)
MRH_HD inline bool sortkey_is_nan_key(uint64_t k, int mode) {
  return (mode == 3 && k == (uint64_t)(0x7fc00000u | 0x80000000u)) ||
         (mode == 4 && k == (0x7ff8000000000000ull | 0x8000000000000000ull));
}
MRH_HD inline uint64_t sortkey(uint64_t raw, int mode, bool desc) {
  const uint64_t k = sortkey_transform(raw, mode);
  if (!desc) return k;
  // all ones: above every complemented key in the low 32 bits (a 4-byte
  // column's sort) and in all 64
  return sortkey_is_nan_key(k, mode) ? ~uint64_t(0) : ~k;
}

}  // namespace dev
}  // namespace mrh
