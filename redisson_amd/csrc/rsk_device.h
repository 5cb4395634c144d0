// rsk_device.h -- device-side hashing primitives for the gfx950 sketch engine.
//
// Each routine restates the upstream algorithm the reference path reaches
// (SURVEY.md 8a):
//   murmur64a*  : Redis 3.2.0 hyperloglog.c MurmurHash64A, seed 0xadc83b19
//                 (reached from RedissonHyperLogLog.java:65-76 via PFADD)
//   hll_rank    : Redis 3.2.0 hllPatLen (rank in [1,50])
//   xxh64*      : OpenHFT LongHashFunction.xx_r39() (RedissonBloomFilter.java:117)
//   farm_uo64*  : OpenHFT LongHashFunction.farmUo()  (RedissonBloomFilter.java:118)
//   FastMod63   : the `% size` of RedissonBloomFilter.java:123 as a multiply-high
//                 by a host-precomputed reciprocal (exact for dividends < 2^63).
//
// Byte access convention: keys are read with unaligned 8/4-byte global loads
// (gfx950 runs in unaligned-access mode) that never extend past the key's
// last byte, so user blobs need no padding.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define RSK_DEV __device__ __forceinline__

namespace rsk {

constexpr uint64_t MM_M = 0xc6a4a7935bd1e995ULL;
constexpr uint32_t HLL_SEED = 0xadc83b19U;
constexpr int HLL_P = 14;
constexpr int HLL_REGS = 1 << HLL_P;

RSK_DEV uint64_t ld_u64(const uint8_t* p) {
  uint64_t v;
  __builtin_memcpy(&v, p, 8);
  return v;
}
RSK_DEV uint32_t ld_u32(const uint8_t* p) {
  uint32_t v;
  __builtin_memcpy(&v, p, 4);
  return v;
}
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
// 16-byte streaming load with the nontemporal hint (keys are read once).
RSK_DEV uint4 ld_nt16(const void* p) {
  u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
}
// XCD-aware work order: blocks b and b + 8 share an XCD (its L2), so a
// persistent grid (a multiple of 8 blocks) that walks items in rounds of
// gridDim.x gives XCD b % 8 the consecutive slots [(b % 8) n, (b % 8 + 1) n),
// n = gridDim.x / 8: neighbouring items, which share boundary cache lines or
// whole inputs, are then fetched into one L2.  Placement is a speed hint only.
RSK_DEV uint32_t xcd_slot(uint32_t b, uint32_t grid) {
  return (grid & 7u) ? b : (b & 7u) * (grid >> 3) + (b >> 3);
}
RSK_DEV uint64_t rotr(uint64_t v, int s) { return (v >> s) | (v << (64 - s)); }
RSK_DEV uint64_t rotl(uint64_t v, int s) { return (v << s) | (v >> (64 - s)); }

// Last `t` (1..7) bytes of key [p, p+len) as a little-endian integer, read
// without touching memory past p+len-1.
RSK_DEV uint64_t ld_tail(const uint8_t* p, uint64_t len, uint32_t t) {
  if (len >= 8) return ld_u64(p + len - 8) >> (8 * (8 - t));
  // Short key: aligned words overlapping the key never cross a page.
  const uint8_t* q = p + len - t;
  uintptr_t a = reinterpret_cast<uintptr_t>(q) & ~uintptr_t(7);
  uint32_t sh = (uint32_t)(reinterpret_cast<uintptr_t>(q) & 7);
  uint64_t lo = *reinterpret_cast<const uint64_t*>(a);
  uint64_t v = lo >> (8 * sh);
  if (sh + t > 8) v |= (*reinterpret_cast<const uint64_t*>(a + 8)) << (8 * (8 - sh));
  return t == 8 ? v : (v & ((1ULL << (8 * t)) - 1));
}

// ------------------------------------------------------------ MurmurHash64A
RSK_DEV uint64_t mm_mix(uint64_t k) {
  k *= MM_M;
  k ^= k >> 47;
  k *= MM_M;
  return k;
}
RSK_DEV uint64_t mm_final(uint64_t h) {
  h ^= h >> 47;
  h *= MM_M;
  h ^= h >> 47;
  return h;
}
// 16-byte key held in two little-endian words (the C2/C3/C5 fast path).
RSK_DEV uint64_t murmur64a_16(uint64_t w0, uint64_t w1) {
  uint64_t h = (uint64_t)HLL_SEED ^ (16ULL * MM_M);
  h ^= mm_mix(w0);
  h *= MM_M;
  h ^= mm_mix(w1);
  h *= MM_M;
  return mm_final(h);
}
// 8-byte key (fixed-stride longs).
RSK_DEV uint64_t murmur64a_8(uint64_t w0) {
  uint64_t h = (uint64_t)HLL_SEED ^ (8ULL * MM_M);
  h ^= mm_mix(w0);
  h *= MM_M;
  return mm_final(h);
}
// Any length, bytes in global memory.
RSK_DEV uint64_t murmur64a(const uint8_t* p, uint64_t len) {
  uint64_t h = (uint64_t)HLL_SEED ^ (len * MM_M);
  uint64_t nb = len >> 3;
  for (uint64_t j = 0; j < nb; ++j) {
    h ^= mm_mix(ld_u64(p + 8 * j));
    h *= MM_M;
  }
  uint32_t t = (uint32_t)(len & 7);
  if (t) {
    h ^= ld_tail(p, len, t);
    h *= MM_M;
  }
  return mm_final(h);
}

// The same for keys of at most 64 bytes with every load issued up front (one
// memory round trip per key instead of one per 8-byte block).  Words past
// the key are not loaded (predicated) and the tail is read ending at the
// key's last byte, so nothing beyond the key is touched.
RSK_DEV uint64_t murmur64a_le64(const uint8_t* p, uint32_t len) {
  uint64_t w[8];
  const uint32_t nb = len >> 3, t = len & 7;
#pragma unroll
  for (int j = 0; j < 8; ++j) w[j] = (uint32_t)j < nb ? ld_u64(p + 8 * j) : 0;
  const uint64_t tail = t ? ld_tail(p, len, t) : 0;
  uint64_t h = (uint64_t)HLL_SEED ^ ((uint64_t)len * MM_M);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    if ((uint32_t)j < nb) {
      h ^= mm_mix(w[j]);
      h *= MM_M;
    }
  }
  if (t) {
    h ^= tail;
    h *= MM_M;
  }
  return mm_final(h);
}

// hllPatLen (Redis 3.2.0): rank = 1 + zeros from bit 14 up, bit 63 forced.
RSK_DEV uint32_t hll_rank(uint64_t h) {
  uint64_t v = (h >> HLL_P) | (1ULL << (63 - HLL_P));
  return 1u + (uint32_t)__builtin_ctzll(v);
}
RSK_DEV uint32_t hll_index(uint64_t h) { return (uint32_t)(h & (HLL_REGS - 1)); }

// ------------------------------------------------------------------- XXH64
constexpr uint64_t XP1 = 0x9E3779B185EBCA87ULL;
constexpr uint64_t XP2 = 0xC2B2AE3D27D4EB4FULL;
constexpr uint64_t XP3 = 0x165667B19E3779F9ULL;
constexpr uint64_t XP4 = 0x85EBCA77C2B2AE63ULL;
constexpr uint64_t XP5 = 0x27D4EB2F165667C5ULL;

RSK_DEV uint64_t xx_round(uint64_t acc, uint64_t in) {
  acc += in * XP2;
  acc = rotl(acc, 31);
  return acc * XP1;
}
RSK_DEV uint64_t xx_merge(uint64_t acc, uint64_t v) {
  acc ^= xx_round(0, v);
  return acc * XP1 + XP4;
}
RSK_DEV uint64_t xx_avalanche(uint64_t h) {
  h ^= h >> 33;
  h *= XP2;
  h ^= h >> 29;
  h *= XP3;
  h ^= h >> 32;
  return h;
}
RSK_DEV uint64_t xxh64_16(uint64_t w0, uint64_t w1) {
  uint64_t h = XP5 + 16;
  h ^= xx_round(0, w0);
  h = rotl(h, 27) * XP1 + XP4;
  h ^= xx_round(0, w1);
  h = rotl(h, 27) * XP1 + XP4;
  return xx_avalanche(h);
}
RSK_DEV uint64_t xxh64(const uint8_t* p, uint64_t len) {
  const uint8_t* end = p + len;
  uint64_t h;
  if (len >= 32) {
    const uint8_t* limit = end - 32;
    uint64_t v1 = XP1 + XP2, v2 = XP2, v3 = 0, v4 = 0 - XP1;
    do {
      v1 = xx_round(v1, ld_u64(p));
      v2 = xx_round(v2, ld_u64(p + 8));
      v3 = xx_round(v3, ld_u64(p + 16));
      v4 = xx_round(v4, ld_u64(p + 24));
      p += 32;
    } while (p <= limit);
    h = rotl(v1, 1) + rotl(v2, 7) + rotl(v3, 12) + rotl(v4, 18);
    h = xx_merge(h, v1);
    h = xx_merge(h, v2);
    h = xx_merge(h, v3);
    h = xx_merge(h, v4);
  } else {
    h = XP5;
  }
  h += len;
  while (p + 8 <= end) {
    h ^= xx_round(0, ld_u64(p));
    h = rotl(h, 27) * XP1 + XP4;
    p += 8;
  }
  if (p + 4 <= end) {
    h ^= (uint64_t)ld_u32(p) * XP1;
    h = rotl(h, 23) * XP2 + XP3;
    p += 4;
  }
  while (p < end) {
    h ^= (uint64_t)(*p) * XP5;
    h = rotl(h, 11) * XP1;
    ++p;
  }
  return xx_avalanche(h);
}

// --------------------------------------------------------- farmhash na / uo
constexpr uint64_t FK0 = 0xc3a5c85c97cb3127ULL;
constexpr uint64_t FK1 = 0xb492b66fbe98f273ULL;
constexpr uint64_t FK2 = 0x9ae16a3b2f90404fULL;

RSK_DEV uint64_t shift_mix(uint64_t v) { return v ^ (v >> 47); }
RSK_DEV uint64_t hash_len16(uint64_t u, uint64_t v, uint64_t mul) {
  uint64_t a = (u ^ v) * mul;
  a ^= (a >> 47);
  uint64_t b = (v ^ a) * mul;
  b ^= (b >> 47);
  b *= mul;
  return b;
}
// farmhashna::HashLen0to16, 16-byte specialisation (len = 16 >= 8 branch).
RSK_DEV uint64_t farm_16(uint64_t w0, uint64_t w1) {
  const uint64_t mul = FK2 + 32;
  uint64_t a = w0 + FK2;
  uint64_t b = w1;
  uint64_t c = rotr(b, 37) * mul + a;
  uint64_t d = (rotr(a, 25) + b) * mul;
  return hash_len16(c, d, mul);
}
RSK_DEV uint64_t farm_na_0to16(const uint8_t* s, uint64_t len) {
  if (len >= 8) {
    uint64_t mul = FK2 + len * 2;
    uint64_t a = ld_u64(s) + FK2;
    uint64_t b = ld_u64(s + len - 8);
    uint64_t c = rotr(b, 37) * mul + a;
    uint64_t d = (rotr(a, 25) + b) * mul;
    return hash_len16(c, d, mul);
  }
  if (len >= 4) {
    uint64_t mul = FK2 + len * 2;
    uint64_t a = ld_u32(s);
    return hash_len16(len + (a << 3), ld_u32(s + len - 4), mul);
  }
  if (len > 0) {
    uint8_t a = s[0], b = s[len >> 1], c = s[len - 1];
    uint32_t y = (uint32_t)a + ((uint32_t)b << 8);
    uint32_t z = (uint32_t)len + ((uint32_t)c << 2);
    return shift_mix((uint64_t)y * FK2 ^ (uint64_t)z * FK0) * FK2;
  }
  return FK2;
}
RSK_DEV uint64_t farm_na_17to32(const uint8_t* s, uint64_t len) {
  uint64_t mul = FK2 + len * 2;
  uint64_t a = ld_u64(s) * FK1;
  uint64_t b = ld_u64(s + 8);
  uint64_t c = ld_u64(s + len - 8) * mul;
  uint64_t d = ld_u64(s + len - 16) * FK2;
  return hash_len16(rotr(a + b, 43) + rotr(c, 30) + d, a + rotr(b + FK2, 18) + c, mul);
}
RSK_DEV uint64_t farm_na_33to64(const uint8_t* s, uint64_t len) {
  uint64_t mul = FK2 + len * 2;
  uint64_t a = ld_u64(s) * FK2;
  uint64_t b = ld_u64(s + 8);
  uint64_t c = ld_u64(s + len - 8) * mul;
  uint64_t d = ld_u64(s + len - 16) * FK2;
  uint64_t y = rotr(a + b, 43) + rotr(c, 30) + d;
  uint64_t z = hash_len16(y, a + rotr(b + FK2, 18) + c, mul);
  uint64_t e = ld_u64(s + 16) * mul;
  uint64_t f = ld_u64(s + 24);
  uint64_t g = (y + ld_u64(s + len - 32)) * mul;
  uint64_t h = (z + ld_u64(s + len - 24)) * mul;
  return hash_len16(rotr(e + f, 43) + rotr(g, 30) + h, e + rotr(f + a, 18) + g, mul);
}
struct U64Pair {
  uint64_t first, second;
};
RSK_DEV U64Pair weak32(const uint8_t* s, uint64_t a, uint64_t b) {
  uint64_t w = ld_u64(s), x = ld_u64(s + 8), y = ld_u64(s + 16), z = ld_u64(s + 24);
  a += w;
  b = rotr(b + a + z, 21);
  uint64_t c = a;
  a += x;
  a += y;
  b += rotr(a, 44);
  return U64Pair{a + z, b + c};
}
RSK_DEV uint64_t uo_h(uint64_t x, uint64_t y, uint64_t mul, int r) {
  uint64_t a = (x ^ y) * mul;
  a ^= (a >> 47);
  uint64_t b = (y ^ a) * mul;
  return rotr(b, r) * mul;
}
// farmhashuo::Hash64WithSeeds(s, len, 81, 0), len > 64 (parity unpinned).
RSK_DEV uint64_t farm_uo_long(const uint8_t* s, uint64_t len) {
  const uint64_t seed0 = 81, seed1 = 0;
  uint64_t x = seed0;
  uint64_t y = seed1 * FK2 + 113;
  uint64_t z = shift_mix(y * FK2) * FK2;
  U64Pair v{seed0, seed1}, w{0, 0};
  uint64_t u = x - z;
  x *= FK2;
  uint64_t mul = FK2 + (u & 0x82);
  const uint8_t* end = s + ((len - 1) / 64) * 64;
  const uint8_t* last64 = end + ((len - 1) & 63) - 63;
  do {
    uint64_t a0 = ld_u64(s), a1 = ld_u64(s + 8), a2 = ld_u64(s + 16), a3 = ld_u64(s + 24);
    uint64_t a4 = ld_u64(s + 32), a5 = ld_u64(s + 40), a6 = ld_u64(s + 48), a7 = ld_u64(s + 56);
    x += a0 + a1;
    y += a2;
    z += a3;
    v.first += a4;
    v.second += a5 + a1;
    w.first += a6;
    w.second += a7;
    x = rotr(x, 26);
    x *= 9;
    y = rotr(y, 29);
    z *= mul;
    v.first = rotr(v.first, 33);
    v.second = rotr(v.second, 30);
    w.first ^= x;
    w.first *= 9;
    z = rotr(z, 32);
    z += w.second;
    w.second += z;
    z *= 9;
    { uint64_t t = u; u = y; y = t; }
    z += a0 + a6;
    v.first += a2;
    v.second += a3;
    w.first += a4;
    w.second += a5 + a6;
    x += a1;
    y += a7;
    y += v.first;
    v.first += x - y;
    v.second += w.first;
    w.first += v.second;
    w.second += x - y;
    x += w.second;
    w.second = rotr(w.second, 34);
    { uint64_t t = u; u = z; z = t; }
    s += 64;
  } while (s != end);
  s = last64;
  u *= 9;
  v.second = rotr(v.second, 28);
  v.first = rotr(v.first, 20);
  w.first += ((len - 1) & 63);
  u += y;
  y += u;
  x = rotr(y - x + v.first + ld_u64(s + 8), 37) * mul;
  y = rotr(y ^ v.second ^ ld_u64(s + 48), 42) * mul;
  x ^= w.second * 9;
  y += v.first + ld_u64(s + 40);
  z = rotr(z + w.first, 33) * mul;
  v = weak32(s, v.second * mul, x + w.first);
  w = weak32(s + 32, z + w.second, y + ld_u64(s + 16));
  return uo_h(hash_len16(v.first + x, w.first ^ y, mul) + z - u,
              uo_h(v.second + w.second, w.first + v.first, mul, 30) + x, mul, 31);
}
RSK_DEV uint64_t farm_uo64(const uint8_t* s, uint64_t len) {
  if (len <= 16) return farm_na_0to16(s, len);
  if (len <= 32) return farm_na_17to32(s, len);
  if (len <= 64) return farm_na_33to64(s, len);
  return farm_uo_long(s, len);
}

// ------------------------------------------------------------ exact u63 mod
// floor(x/d) = mulhi(x, M) >> (l-1) for x < 2^63, l = ceil(log2 d) >= 1,
// M = ceil(2^(63+l)/d)  (round-up method; M < 2^64).  d == 1 -> l == 0.
struct FastMod63 {
  uint64_t d;
  uint64_t M;
  uint64_t r63;  // 2^63 mod d (ProbeSeq)
  uint32_t l;
  uint32_t pad;
};
RSK_DEV uint64_t fastmod63(uint64_t x, const FastMod63& f) {
  if (f.l == 0) return 0;
  uint64_t q = __umul64hi(x, f.M) >> (f.l - 1);
  return x - q * f.d;
}
// Bloom probe indices idx_t = (h_t & Long.MAX_VALUE) % size, h_0 = h1,
// h_{t+1} = h_t + (t even ? h2 : h1) mod 2^64 (RedissonBloomFilter.java:116-131),
// with two divisions per key instead of k.  With v_t = h_t mod 2^63 and
// b = (step addend) mod 2^63:  v_{t+1} = v_t + b - c*2^63, c = bit 63 of
// v_t + b, so  idx_{t+1} = idx_t + (b mod size) - c*(2^63 mod size)  (mod size).
// Both addends, b mod size and (b - 2^63) mod size, are reduced once per key
// (r1 / r1c for h1, r2 / r2c for h2), so a step is one add of the addend c
// selects and one conditional subtract.
struct ProbeSeq {
  uint64_t v = 0, idx = 0, v1 = 0, v2 = 0, r1 = 0, r2 = 0, r1c = 0, r2c = 0;
  ProbeSeq() = default;
  RSK_DEV ProbeSeq(uint64_t h1, uint64_t h2, const FastMod63& f) {
    v1 = h1 & 0x7FFFFFFFFFFFFFFFULL;
    v2 = h2 & 0x7FFFFFFFFFFFFFFFULL;
    init(fastmod63(v1, f), fastmod63(v2, f), f);
  }
  // residues r1 = v1 mod d, r2 = v2 mod d given (timing variants)
  RSK_DEV void init(uint64_t m1, uint64_t m2, const FastMod63& f) {
    r1 = m1;
    r2 = m2;
    r1c = r1 >= f.r63 ? r1 - f.r63 : r1 + (f.d - f.r63);
    r2c = r2 >= f.r63 ? r2 - f.r63 : r2 + (f.d - f.r63);
    v = v1;
    idx = r1;
  }
  // idx_t -> idx_{t+1}
  // (values selected, never member lvalues: a conditional over members with a
  // run-time t puts the whole struct in scratch memory)
  RSK_DEV void next(int t, const FastMod63& f) {
    const bool odd = t & 1;
    const uint64_t b = odd ? v1 : v2, ra = odd ? r1 : r2, rc = odd ? r1c : r2c;
    const uint64_t s = v + b;  // < 2^64
    const uint64_t x = idx + ((s >> 63) ? rc : ra);  // < 2 * size
    idx = x >= f.d ? x - f.d : x;
    v = s & 0x7FFFFFFFFFFFFFFFULL;
  }
};

// ------------------------------------------------------ Bloom probe indices
// RedissonBloomFilter.hash (:116-131): h1 = xx_r39(bytes), h2 = farmUo(bytes),
// idx_t = (h_t & Long.MAX_VALUE) % size with h_0 = h1, h_{t+1} = h_t + (t even ? h2 : h1).
constexpr uint64_t JAVA_LONG_MAX = 0x7FFFFFFFFFFFFFFFULL;

template <bool FIXED16>
RSK_DEV void bloom_key_hashes(const uint8_t* __restrict__ data, const uint64_t* __restrict__ offsets,
                              uint32_t fixed_len, uint64_t i, uint64_t& h1, uint64_t& h2) {
  if (FIXED16) {
    uint4 v = ld_nt16(reinterpret_cast<const uint4*>(data) + i);
    uint64_t w0 = ((uint64_t)v.y << 32) | v.x, w1 = ((uint64_t)v.w << 32) | v.z;
    h1 = xxh64_16(w0, w1);
    h2 = farm_16(w0, w1);
  } else {
    uint64_t s = offsets ? offsets[i] : i * fixed_len;
    uint64_t len = offsets ? offsets[i + 1] - s : fixed_len;
    h1 = xxh64(data + s, len);
    h2 = farm_uo64(data + s, len);
  }
}

// Bit i of the Redis string (byte i>>3, mask 0x80>>(i&7); bitops.c) inside
// its little-endian u32 word i>>5.  Any base that is a multiple of 32 bits
// keeps the mask, so slice-local indices use it too.
// Workgroup barrier that orders LDS only: each wave waits for its own LDS
// traffic (lgkmcnt) and meets the others, but its global loads, stores and
// atomics stay in flight (__syncthreads' release fence would drain them:
// s_waitcnt vmcnt(0) before every barrier).  For kernels whose global
// writes are not read back by other waves of the same launch.
RSK_DEV void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

RSK_DEV uint32_t bloom_bit_mask(uint64_t idx) {
  return 1u << ((uint32_t)((idx >> 3) & 3) * 8 + 7 - (uint32_t)(idx & 7));
}

// ------------------------------------------------------- synthetic streams
RSK_DEV uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ULL;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

}  // namespace rsk
