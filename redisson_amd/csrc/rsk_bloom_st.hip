// rsk_bloom_st.hip -- Bloom insert for large batches by super-tile partition (gfx950).
//
// RedissonBloomFilter.add (src/main/java/org/redisson/RedissonBloomFilter.java:80-114)
// sets k bits per element (k SETBITs, :94-98) at idx_t = (h_t & Long.MAX_VALUE)
// % size (:116-131).  Setting bits is an OR, so the probes may be applied in
// any order; this path routes them to 64 KiB slices of the filter (2^19 bits)
// and ORs each slice in LDS, without knowing any count in advance:
//
//   st1   : one pass over the keys.  A super-tile = 2 keys per lane (k <= 8) or
//           1 (k <= 16) of a 512-lane workgroup: each lane hashes its keys once
//           (XXH64 + farmhash), keeps its <= 16 probes in registers, ranks them
//           by coarse bin (idx >> (19 + f2), <= 256 bins) with one LDS atomic
//           each, places them in an LDS image (double-buffered: the write-out
//           of one super-tile overlaps the hashing of the next) and writes the
//           bin-sorted super-tile CONTIGUOUSLY at its own slot (probes 26 bits:
//           the position inside the coarse bin) plus a u16 header of bin
//           offsets.  No histogram pass, no global offsets.
//   hdrT  : header transposed to [bin][super-tile] (coalesced reads below).
//   size  : per (coarse bin c, part p): probes and a tile budget for st2.
//   st2   : one workgroup per (c, p) reads segment c of the super-tiles of
//           part p (16 waves, each its own groups of 64 consecutive
//           super-tiles, R2 = 14 slots of 64 probes per lane, the chunk ->
//           segment map a ballot over the lanes' chunk prefix sums), ranks by
//           fine bin (the 2^f2 slices of c), and writes bin-sorted tiles
//           contiguously into the (c, p) region, with u16 headers (19-bit
//           slice offsets).
//   apply : one workgroup per slice: 64 KiB of filter in LDS, every segment
//           of that slice in the tiles of its coarse bin ORed in with ds_or
//           (UA segments' loads in flight per wave), the slice written back once.
// Filters of <= 256 slices skip st2 (apply reads the st1 tiles directly).
//
// HBM per key at k probes: 16 B of key + 4k (st1 write) + 4k + 4k (st2) + 4k
// (apply) + ~1 % headers, plus 2 x the filter per chunk; LDS per probe: rank
// atomic + lstart read + place + read-out (st1, st2) + ds_or (apply).  The
// earlier pipeline (rsk_bloom_part.hip: histogram pass over the keys, exact
// global offsets, sbin/dlt scatter) remains for k > 16 and as the fallback.
// Measured variants: a paged layout (runs appended to 4 KiB
// pages, whole-page reads) made apply faster but the scattered run writes cost
// more than the segment reads they replaced.
#include <cstdlib>
#include <cstring>

#include "rsk_bloom_sa.h"

namespace rsk {

namespace {

constexpr int T1_DEFAULT = 512;                        // st1 workgroup (RSK_BLOOM_ST_T1 = 512 | 1024)
constexpr int T2_DEFAULT = 1024;                       // st2 workgroup (RSK_BLOOM_ST_T2 = 512 | 1024)
constexpr int R2 = 14;                                 // st2 probe slots per lane
constexpr int TA = 1024;                               // apply workgroup
constexpr int UA_DEFAULT = 8;                          // apply: segments loaded at once per wave (RSK_BLOOM_ST_UA = 4 | 8)
constexpr uint64_t DEFAULT_PROBE_CHUNK = 1ull << 33;   // probes per chunk (2 x 32 GiB of scratch)


// Super-tile st = keys [st*KST, st*KST + KST): bin-sorted probes at
// out[st * KST * k ...], header hdr[st][0..nb1] (bin offsets, [nb1] = total).
// The sorted image is double-buffered in LDS, so a tile's write-out overlaps
// the next tile's hashing: three barriers per super-tile.
template <bool FIXED16, int KMAX, int T1>
__global__ __launch_bounds__(T1) void bloom_st1_kernel(const uint8_t* __restrict__ data,
                                                       const uint64_t* __restrict__ offsets, uint32_t fixed_len,
                                                       uint64_t n, FastMod63 fm, int k, uint32_t shift1, uint32_t nb1,
                                                       uint64_t nst, uint32_t* __restrict__ out,
                                                       uint16_t* __restrict__ hdr) {
  constexpr int KPL = 16 / KMAX;        // keys per lane
  constexpr uint32_t KST = T1 * KPL;    // keys per super-tile
  constexpr int NP = KPL * KMAX;        // probe slots per lane (16)
  __shared__ __attribute__((aligned(16))) uint32_t srt[2][T1 * NP];
  __shared__ uint32_t hist[256], lstart[256], s_total;
  const uint64_t low = (1ull << shift1) - 1;
  const uint64_t stride = (uint64_t)KST * (uint64_t)k;
  if (threadIdx.x < 256) hist[threadIdx.x] = 0;
  const uint4* keys16 = reinterpret_cast<const uint4*>(data);
  uint4 nxt[KPL];
  auto fetch = [&](uint64_t st) {
#pragma unroll
    for (int u = 0; u < KPL; ++u) {
      const uint64_t i = st * KST + threadIdx.x + (uint64_t)u * T1;
      nxt[u] = (FIXED16 && st < nst && i < n) ? ld_nt16(keys16 + i) : make_uint4(0, 0, 0, 0);
    }
  };
  if (FIXED16) fetch(blockIdx.x);
  __syncthreads();  // hist zeroed
  uint32_t buf = 0;
  for (uint64_t st = blockIdx.x; st < nst; st += gridDim.x, buf ^= 1) {
    const uint64_t k0 = st * KST;
    const uint32_t nk = (uint32_t)(n - k0 < KST ? n - k0 : KST);
    uint4 cur[KPL];
#pragma unroll
    for (int u = 0; u < KPL; ++u) cur[u] = nxt[u];
    if (FIXED16) fetch(st + gridDim.x);  // the next super-tile's keys stream in meanwhile
    uint32_t pay[NP], tag[NP];
#pragma unroll
    for (int u = 0; u < KPL; ++u) {
      const uint32_t q = threadIdx.x + u * T1;
      const bool ok = q < nk;
      uint64_t h1 = 0, h2 = 0;
      if (ok) {
        if (FIXED16) {
          uint64_t w0, w1;
          key_words(cur[u], &w0, &w1);
          h1 = xxh64_16(w0, w1);
          h2 = farm_16(w0, w1);
        } else {
          bloom_key_hashes<false>(data, offsets, fixed_len, k0 + q, h1, h2);
        }
      }
      ProbeSeq ps(h1, h2, fm);
#pragma unroll
      for (int t = 0; t < KMAX; ++t) {
        const int s = u * KMAX + t;
        tag[s] = INVALID;
        pay[s] = 0;
        if (ok && t < k) {
          const uint64_t idx = ps.idx;
          const uint32_t bin = (uint32_t)(idx >> shift1);
          pay[s] = (uint32_t)(idx & low);
          tag[s] = (bin << 16) | atomicAdd(&hist[bin], 1u);
          if (t + 1 < k) ps.next(t, fm);
        }
      }
    }
    __syncthreads();  // (A) every rank taken
    if (threadIdx.x < 64) wave0_bin_starts<256>(hist, lstart, nb1, hdr + st * (nb1 + 1), &s_total);
    __syncthreads();  // (B) lstart / total ready, hist zeroed
    uint32_t* img = srt[buf];  // last read by the write-out of st - 2 gridDim.x, before every wave reached (B)
#pragma unroll
    for (int s = 0; s < NP; ++s)
      if (tag[s] != INVALID) img[lstart[tag[s] >> 16] + (tag[s] & 0xFFFFu)] = pay[s];
    const uint32_t total = s_total;
    __syncthreads();  // (C) image complete
    uint4* o4 = reinterpret_cast<uint4*>(out + st * stride);  // 16-byte aligned (stride * 4 B = 16 KiB * k)
    const uint4* s4 = reinterpret_cast<const uint4*>(img);
    for (uint32_t j = threadIdx.x; j < total / 4; j += T1) {
      const uint4 v = s4[j];
      u32x4 x = {v.x, v.y, v.z, v.w};
      __builtin_nontemporal_store(x, reinterpret_cast<u32x4*>(o4 + j));
    }
    for (uint32_t j = (total & ~3u) + threadIdx.x; j < total; j += T1) out[st * stride + j] = img[j];
  }
}

// ---------------------------------------------------------------- sizing
// (c, p) = blockIdx.x: probes of coarse bin c in st1 tiles [t0, t1) of part p,
// and st2's tile budget (see bloom_add_supertile).
RSK_DEV void part_range(uint64_t nst, uint32_t P, uint32_t p, uint64_t* t0, uint64_t* t1) {
  *t0 = nst * p / P;
  *t1 = nst * (p + 1) / P;
}

// A st2 tile holds `slots` = waves x R2 slots of 64 probes; a slot is short
// only when it ends a segment, so a (c, p) needs at most
// (probes / 64 + segments) / slots tiles when its waves stay balanced; twice
// that is budgeted (an overflow is caught and redone, see bloom_add_supertile).
RSK_DEV uint32_t tile_budget(uint64_t probes, uint64_t segs, uint32_t slots) {
  return (uint32_t)(2 * ((probes / 64 + segs) / slots) + 4);
}

__global__ __launch_bounds__(256) void st_size_kernel(const uint16_t* __restrict__ h1t, uint64_t nst, uint32_t P,
                                                      uint32_t slots, int tiny_budget, uint64_t* __restrict__ tot,
                                                      uint32_t* __restrict__ bud) {
  __shared__ uint64_t part[4];
  const uint32_t cp = blockIdx.x, c = cp / P, p = cp - c * P;
  uint64_t t0, t1;
  part_range(nst, P, p, &t0, &t1);
  const uint16_t* a = h1t + (uint64_t)c * nst;
  const uint16_t* b = a + nst;
  uint64_t s = 0;
  for (uint64_t t = t0 + threadIdx.x; t < t1; t += 256) s += (uint32_t)(b[t] - a[t]);
  for (int o = 32; o > 0; o >>= 1) s += __shfl_down(s, o, 64);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint64_t total = part[0] + part[1] + part[2] + part[3];
    tot[cp] = total;
    bud[cp] = tiny_budget ? 1u : tile_budget(total, t1 - t0, slots);  // tiny: tests of the overflow fallback
  }
}


// ------------------------------------------------------------------- st2
// Workgroup (c, p): segment c of the st1 tiles of part p -- wave w takes the
// groups of 64 consecutive tiles t0 + 64 (w + NW i) + [0, 64), one coalesced
// header load per group (the next group prefetched) -- bin-sorted by fine bin
// (pay >> 19) into tiles written contiguously at out + reg_off[cp]; tile j of
// (c, p) gets header h2[tile_off[cp] + j][0..nb2] and its start tb2.
// A wave's R2 slots per tile are chunks of 64 probes of its cached segments:
// the chunk -> segment map is a ballot over the lanes' chunk prefix sums.
template <int T2>
__global__ __launch_bounds__(T2) void bloom_st2_kernel(const uint32_t* __restrict__ in,
                                                       const uint16_t* __restrict__ h1t, uint64_t nst,
                                                       uint64_t stride1, uint32_t P, uint32_t nb2,
                                                       const uint64_t* __restrict__ reg_off,
                                                       const uint32_t* __restrict__ tile_off,
                                                       const uint32_t* __restrict__ bud, uint32_t* __restrict__ used,
                                                       uint32_t* __restrict__ out, uint16_t* __restrict__ h2,
                                                       uint64_t* __restrict__ tb2, uint32_t* __restrict__ overflow) {
  constexpr uint32_t NW = T2 / 64;
  __shared__ __attribute__((aligned(16))) uint32_t srt[2][T2 * R2];
  __shared__ uint32_t hist[128], lstart[128], s_total;
  __shared__ uint16_t s_hdr[129];
  const uint32_t cp = blockIdx.x, c = cp / P, p = cp - c * P;
  // the wave index as a scalar: every per-wave cursor below stays in SGPRs
  const uint32_t lane = threadIdx.x & 63, w = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  uint64_t t0, t1;
  part_range(nst, P, p, &t0, &t1);
  const uint16_t* ha = h1t + (uint64_t)c * nst;
  const uint16_t* hb = ha + nst;
  if (threadIdx.x < 128) hist[threadIdx.x] = 0;
  // segment cache (lane l: segment of tile g + l) and the prefetched next group
  uint64_t g_next = t0 + 64ull * w;
  uint32_t plen = 0, clen = 0;
  uint64_t ppos = 0, cpos = 0;
  bool pvalid = false;
  auto load_group = [&]() {
    pvalid = g_next < t1;
    const uint64_t t = g_next + lane;
    plen = 0;
    ppos = 0;
    if (t < t1) {
      const uint32_t a = ha[t];
      plen = (uint32_t)hb[t] - a;
      ppos = t * stride1 + a;
    }
    g_next += 64ull * NW;
  };
  uint32_t pref = 0, ct = 0, q = 0;  // inclusive chunk prefix (per lane), chunks in cache, next chunk
  auto refill = [&]() {  // make q < ct; false when this wave's segments are exhausted
    while (q >= ct) {
      if (!pvalid) return false;
      clen = plen;
      cpos = ppos;
      pref = wave_scan_incl((clen + 63) >> 6, lane);
      ct = rdl(pref, 63);
      q = 0;
      load_group();
    }
    return true;
  };
  load_group();
  bool have = refill();
  const uint64_t base = reg_off[cp];
  const uint32_t tbeg = tile_off[cp], tcap = bud[cp];
  uint64_t written = 0;
  uint32_t ntile = 0, buf = 0;
  __syncthreads();  // hist zeroed
  for (;;) {
    uint32_t pay[R2], tag[R2];
#pragma unroll
    for (int r = 0; r < R2; ++r) {
      pay[r] = INVALID;
      if (have) {
        const uint32_t sg = (uint32_t)__builtin_popcountll(__ballot(pref <= q));  // segment of chunk q
        const uint32_t first = sg ? rdl(pref, sg - 1) : 0;
        const uint32_t o = (q - first) * 64 + lane;
        if (o < rdl(clen, sg)) pay[r] = __builtin_nontemporal_load(&in[rdl64(cpos, sg) + o]);
        ++q;
        if (q >= ct) have = refill();
      }
    }
#pragma unroll
    for (int r = 0; r < R2; ++r) {
      tag[r] = INVALID;
      if (pay[r] != INVALID) {
        const uint32_t bin = pay[r] >> SL_LOG;
        tag[r] = (bin << 16) | atomicAdd(&hist[bin], 1u);
      }
    }
    const int more = __syncthreads_or(have ? 1 : 0);  // (A) every rank taken
    if (threadIdx.x < 64) wave0_bin_starts<128>(hist, lstart, nb2, s_hdr, &s_total);
    __syncthreads();  // (B)
    const uint32_t total = s_total;
    if (total) {
      if (ntile < tcap) {
        if (threadIdx.x <= nb2) h2[(uint64_t)(tbeg + ntile) * (nb2 + 1) + threadIdx.x] = s_hdr[threadIdx.x];
        if (threadIdx.x == 0) tb2[tbeg + ntile] = base + written;
      } else if (threadIdx.x == 0) {
        atomicOr(overflow, 1u);  // budget exceeded (adversarial input): the host redoes the chunk
      }
      uint32_t* img = srt[buf];
#pragma unroll
      for (int r = 0; r < R2; ++r)
        if (tag[r] != INVALID) img[lstart[tag[r] >> 16] + (tag[r] & 0xFFFFu)] = pay[r] & ((1u << SL_LOG) - 1);
      __syncthreads();  // (C) image complete
      uint32_t* o = out + base + written;
      for (uint32_t j = threadIdx.x; j < total; j += T2) o[j] = img[j];
      written += total;
      ++ntile;
      buf ^= 1;
    }
    if (!more) break;
  }
  if (threadIdx.x == 0) used[cp] = ntile < tcap ? ntile : tcap;
}

// ----------------------------------------------------------------- apply
// Slice s: OR every probe of s into the 64 KiB slice held in LDS.  Two-level:
// the tiles of coarse bin c = s >> f2 (per part p: [tile_off[cp], + used[cp])),
// segment f = s & (2^f2 - 1), rows f / f+1 of the transposed st2 headers, tile
// starts tb[tile].  One level (f2 = 0, tile_off == nullptr): the st1 tiles
// [0, nst), rows s / s+1 of the transposed st1 headers, tile t at t * stride.
template <int UA>
__global__ __launch_bounds__(TA) void bloom_st_apply_kernel(const uint32_t* __restrict__ probes,
                                                            const uint16_t* __restrict__ ht, uint64_t row_stride,
                                                            uint32_t f2, const uint64_t* __restrict__ tb,
                                                            uint64_t stride, uint64_t nst,
                                                            const uint32_t* __restrict__ tile_off,
                                                            const uint32_t* __restrict__ used, uint32_t P,
                                                            uint32_t nslices, uint32_t* __restrict__ bits,
                                                            uint64_t nwords) {
  __shared__ __attribute__((aligned(16))) uint32_t sl[SL_WORDS];
  // the wave index as a scalar: every per-wave cursor below stays in SGPRs
  const uint32_t lane = threadIdx.x & 63, w = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  constexpr uint32_t NW = TA / 64;
  for (uint32_t s = blockIdx.x; s < nslices; s += gridDim.x) {
    const uint64_t w0 = (uint64_t)s * SL_WORDS;
    const uint32_t nw4 = (uint32_t)((nwords - w0 < SL_WORDS ? nwords - w0 : SL_WORDS) / 4);
    uint4* g4 = reinterpret_cast<uint4*>(bits + w0);
    uint4* l4 = reinterpret_cast<uint4*>(sl);
    for (uint32_t q = threadIdx.x; q < nw4; q += TA) l4[q] = g4[q];
    __syncthreads();
    const uint32_t c = s >> f2, f = tile_off ? (s & ((1u << f2) - 1)) : s;
    const uint16_t* ra = ht + (uint64_t)f * row_stride;
    const uint16_t* rb = ra + row_stride;
    const uint32_t nranges = tile_off ? P : 1;
    for (uint32_t pr = 0; pr < nranges; ++pr) {
      uint64_t ta, te;
      if (tile_off) {
        ta = tile_off[(uint64_t)c * P + pr];
        te = ta + used[(uint64_t)c * P + pr];
      } else {
        ta = 0;
        te = nst;
      }
      // wave w: groups of 64 consecutive tiles ta + 64 (w + NW i), one coalesced
      // header load each, the next group's issued before this one is processed
      uint32_t nlen = 0;
      uint64_t npos = 0;
      auto hload = [&](uint64_t gg) {
        const uint64_t t = gg + lane;
        nlen = 0;
        npos = 0;
        if (t < te) {
          const uint32_t beg = ra[t];
          nlen = (uint32_t)rb[t] - beg;
          npos = (tb ? tb[t] : t * stride) + beg;
        }
      };
      hload(ta + 64ull * w);
      for (uint64_t g = ta + 64ull * w; g < te; g += 64ull * NW) {
        const uint32_t len = nlen;
        const uint64_t pos = npos;
        hload(g + 64ull * NW);
        const uint32_t ng = (uint32_t)(te - g < 64 ? te - g : 64);
        for (uint32_t j = 0; j < ng; j += UA) {  // UA segments' loads in flight per lane
          uint32_t v[2 * UA];
#pragma unroll
          for (int q = 0; q < UA; ++q) {
            const uint32_t jj = j + q < ng ? j + q : ng - 1;
            const uint32_t sl_len = (j + q < ng) ? rdl(len, jj) : 0;
            const uint64_t sp = rdl64(pos, jj);
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              const uint32_t o = lane + 64 * h;
              v[2 * q + h] = o < sl_len ? __builtin_nontemporal_load(&probes[sp + o]) : INVALID;
            }
            for (uint32_t o = lane + 128; o < sl_len; o += 64) {  // long segments (rare)
              const uint32_t x = probes[sp + o];
              atomicOr(&sl[x >> 5], bloom_bit_mask(x));
            }
          }
#pragma unroll
          for (int q = 0; q < 2 * UA; ++q)
            if (v[q] != INVALID) atomicOr(&sl[v[q] >> 5], bloom_bit_mask(v[q]));
        }
      }
    }
    __syncthreads();
    for (uint32_t q = threadIdx.x; q < nw4; q += TA) g4[q] = l4[q];
    __syncthreads();
  }
}


// Apply for the append pipeline's sa2 tiles: every fine-bin segment starts
// 16-byte aligned and is padded to a multiple of 4 probes (INVALID), so a
// half-wave loads one segment as up to 32 uint4 (128 probes) in one
// instruction: UA segments per wave take UA/2 16-byte loads per lane.
template <int UA>
__global__ __launch_bounds__(TA, 8) void bloom_sa_apply_kernel(const uint32_t* __restrict__ probes,
                                                            const uint16_t* __restrict__ ht, uint64_t row_stride,
                                                            uint32_t f2, const uint64_t* __restrict__ tb,
                                                            const uint32_t* __restrict__ tile_off,
                                                            const uint32_t* __restrict__ used, uint32_t P,
                                                            uint32_t nslices, uint32_t* __restrict__ bits,
                                                            uint64_t nwords) {
  static_assert(UA % 2 == 0, "two segments per load instruction");
  __shared__ __attribute__((aligned(16))) uint32_t sl[SL_WORDS];
  const uint32_t lane = threadIdx.x & 63, w = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const uint32_t half = lane >> 5, l32 = lane & 31;
  constexpr uint32_t NW = TA / 64;
  const uint4* p4 = reinterpret_cast<const uint4*>(probes);
  for (uint32_t s = blockIdx.x; s < nslices; s += gridDim.x) {
    const uint64_t w0 = (uint64_t)s * SL_WORDS;
    const uint32_t nw4 = (uint32_t)((nwords - w0 < SL_WORDS ? nwords - w0 : SL_WORDS) / 4);
    uint4* g4 = reinterpret_cast<uint4*>(bits + w0);
    uint4* l4 = reinterpret_cast<uint4*>(sl);
    for (uint32_t q = threadIdx.x; q < nw4; q += TA) l4[q] = g4[q];
    lds_barrier();  // LDS only: the previous slice's write-back stays in flight
    const uint32_t c = s >> f2, f = s & ((1u << f2) - 1);
    const uint16_t* ra = ht + (uint64_t)f * row_stride;
    const uint16_t* rb = ra + row_stride;
    for (uint32_t pr = 0; pr < P; ++pr) {
      const uint64_t ta = tile_off[(uint64_t)c * P + pr], te = ta + used[(uint64_t)c * P + pr];
      uint32_t nlen = 0;
      uint64_t npos = 0;
      auto hload = [&](uint64_t gg) {
        const uint64_t t = gg + lane;
        nlen = 0;
        npos = 0;
        if (t < te) {
          const uint32_t beg = ra[t];
          nlen = (uint32_t)rb[t] - beg;  // a multiple of 4
          npos = tb[t] + beg;            // a multiple of 4
        }
      };
      hload(ta + 64ull * w);
      for (uint64_t g = ta + 64ull * w; g < te; g += 64ull * NW) {
        const uint32_t len = nlen;
        const uint64_t pos = npos;
        hload(g + 64ull * NW);
        const uint32_t ng = (uint32_t)(te - g < 64 ? te - g : 64);
        for (uint32_t j = 0; j < ng; j += UA) {
          uint4 v[UA / 2];
#pragma unroll
          for (int q = 0; q < UA / 2; ++q) {
            const uint32_t ja = j + 2 * q, jb = ja + 1;
            const uint32_t la = ja < ng ? rdl(len, ja < 63 ? ja : 63) : 0;
            const uint32_t lb = jb < ng ? rdl(len, jb < 63 ? jb : 63) : 0;
            const uint64_t pa = rdl64(pos, ja < 63 ? ja : 63), pb = rdl64(pos, jb < 63 ? jb : 63);
            const uint32_t my4 = (half ? lb : la) / 4;
            const uint64_t mp4 = (half ? pb : pa) / 4;
            v[q] = l32 < my4 ? ld_nt16(p4 + mp4 + l32) : make_uint4(INVALID, INVALID, INVALID, INVALID);
            for (uint32_t o = l32 + 32; o < my4; o += 32) {  // segments longer than 128 probes (rare)
              const uint4 x = p4[mp4 + o];
              if (x.x != INVALID) atomicOr(&sl[x.x >> 5], bloom_bit_mask(x.x));
              if (x.y != INVALID) atomicOr(&sl[x.y >> 5], bloom_bit_mask(x.y));
              if (x.z != INVALID) atomicOr(&sl[x.z >> 5], bloom_bit_mask(x.z));
              if (x.w != INVALID) atomicOr(&sl[x.w >> 5], bloom_bit_mask(x.w));
            }
          }
#pragma unroll
          for (int q = 0; q < UA / 2; ++q) {
            if (v[q].x != INVALID) atomicOr(&sl[v[q].x >> 5], bloom_bit_mask(v[q].x));
            if (v[q].y != INVALID) atomicOr(&sl[v[q].y >> 5], bloom_bit_mask(v[q].y));
            if (v[q].z != INVALID) atomicOr(&sl[v[q].z >> 5], bloom_bit_mask(v[q].z));
            if (v[q].w != INVALID) atomicOr(&sl[v[q].w >> 5], bloom_bit_mask(v[q].w));
          }
        }
      }
    }
    lds_barrier();
    for (uint32_t q = threadIdx.x; q < nw4; q += TA) g4[q] = l4[q];
    lds_barrier();
  }
}

int st_mode() {
  const char* e = std::getenv("RSK_BLOOM_ST");  // unset: auto; "0": never; "1": always (any batch size)
  if (!e || !*e) return -1;
  return e[0] == '0' ? 0 : 1;
}

uint64_t probe_chunk() {
  const char* e = std::getenv("RSK_BLOOM_ST_CHUNK");  // probes per chunk (tests force small chunks)
  const uint64_t v = (e && *e) ? std::strtoull(e, nullptr, 10) : 0;
  return v ? v : DEFAULT_PROBE_CHUNK;
}

uint32_t env_u32(const char* name, uint32_t dflt) {  // tuning knobs
  const char* e = std::getenv(name);
  return (e && *e) ? (uint32_t)std::strtoul(e, nullptr, 10) : dflt;
}

// Persistent grid: as many workgroups as are resident at once (occupancy API),
// never more than `units` -- a queued workgroup of a persistent loop would
// only start once a resident one had finished all of its units.
template <class F>
void launch_persistent(const void* kernel, int threads, uint64_t units, rsk_ctx* c, F&& launch) {
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, threads, 0) != hipSuccess || per_cu < 1) {
    (void)hipGetLastError();
    per_cu = 1;
  }
  launch((uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(units, (uint64_t)per_cu * (uint64_t)c->num_cus)));
}

uint32_t nbits(uint64_t v) {  // bits needed to hold v (0 -> 0)
  uint32_t b = 0;
  while (v) {
    ++b;
    v >>= 1;
  }
  return b;
}

// The append pipeline (sa1 -> sa2 -> apply) for filters of more than 256 slices.
bool bloom_add_append(rsk_ctx* c, rsk_bloom* b, const DevKeys& keys, bool f16, uint32_t kmax, uint32_t t1,
                      uint64_t kst, uint32_t f2, uint32_t shift1, uint32_t nb1, uint32_t P, uint64_t chunk,
                      bool kpl4) {
  const uint64_t k = (uint64_t)b->k;
  const uint32_t ns = (uint32_t)(((uint64_t)b->size + (1ull << SL_LOG) - 1) >> SL_LOG);
  const uint32_t nb2 = 1u << f2;
  const uint32_t ncp = nb1 * P;
  const uint32_t cus = (uint32_t)c->num_cus;
  const uint32_t ua_env = env_u32("RSK_BLOOM_ST_UA", UA_DEFAULT);
  const uint32_t ua = ua_env == 16 ? 16 : ua_env == 8 ? 8 : 4;
  const uint32_t dbg = env_u32("RSK_BLOOM_SA_DBG", 0);
  const uint64_t max_nst = (chunk + kst - 1) / kst;
  const uint64_t max_np = max_nst * kst * k;
  auto al = [](uint64_t x) { return (x + 255) & ~uint64_t(255); };
  // Workgroups per CU from the kernels' own budgets, not from
  // hipOccupancyMaxActiveBlocksPerMultiprocessor: in a process that has
  // imported torch the runtime reads these code objects' metadata through
  // torch's comgr and answers 1 (scripts/occ_probe.py), a third of the grid.
  // sa1<512>: __launch_bounds__(512, 6) caps it at 80 VGPRs (6 waves per
  // SIMD), 43 KiB of LDS -> 3; sa1<1024>: 78 KiB of LDS, 4 waves per SIMD -> 1.
  const int per_cu = kpl4 ? 2 : (t1 == 512 ? 3 : 1);  // KPL 4: 73 KiB of LDS
  // W persistent sa1 workgroups; each gets 1.25x its expected share of a full
  // coarse bin per bin, plus one whole super-tile (a tile's run can be that
  // long) and the <= 3 padding slots per run of each of its tiles.
  const uint32_t W = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>({max_nst, (uint64_t)per_cu * cus, SA2_WMAX}));
  const double share = (double)(1ull << shift1) / (double)(uint64_t)b->size;
  const bool tiny = env_u32("RSK_BLOOM_SA_TINY", 0) != 0;  // tests force the overflow fallback
  // quota > one tile's probes: a valid run offset b quota + pos - lstart never equals INVALID
  const uint64_t q64 = (uint64_t)(1.25 * share * (double)max_np / W) + kst * k + 3 * (max_nst / W + 1) + 64;
  const uint32_t quota = (uint32_t)((q64 + 3) & ~uint64_t(3));
  const uint32_t limit = tiny ? 32 : quota;
  const uint64_t region_probes = (uint64_t)W * nb1 * quota;
  if (q64 >= (1ull << 31) || (uint64_t)nb1 * quota >= (1ull << 32)) return false;  // u32 offsets -> exact-offset pipeline
  const uint64_t tt_max = (max_np + 3ull * nb1 * max_nst) / SA2_SLOTS + (uint64_t)W * nb1 + 64;  // bound on sa2 tiles
  const uint64_t l2_probes = max_np + 3ull * nb1 * max_nst + tt_max * SA2_PAD + 4ull * ncp;  // sa2 output, padded
  const uint64_t h2_bytes = al(tt_max * (nb2 + 1) * 2);
  const uint64_t meta = al(8 * (ncp + 1)) * 2 + al(4 * (ncp + 1)) * 3 + al(4ull * W * nb1) + 256;
  const uint64_t bytes = al(4 * region_probes) + al(4 * l2_probes) + 2 * h2_bytes + al(8 * tt_max) + meta;
  uint8_t* w = c->work(bytes);
  uint8_t* q = w;
  auto take = [&](uint64_t n) {
    uint8_t* r = q;
    q += n;
    return r;
  };
  uint32_t* region = reinterpret_cast<uint32_t*>(take(al(4 * region_probes)));
  uint32_t* l2 = reinterpret_cast<uint32_t*>(take(al(4 * l2_probes)));
  uint16_t* h2 = reinterpret_cast<uint16_t*>(take(h2_bytes));
  uint16_t* h2t = reinterpret_cast<uint16_t*>(take(h2_bytes));
  uint64_t* tb2 = reinterpret_cast<uint64_t*>(take(al(8 * tt_max)));
  uint64_t* tot = reinterpret_cast<uint64_t*>(take(al(8 * (ncp + 1))));
  uint64_t* reg_off = reinterpret_cast<uint64_t*>(take(al(8 * (ncp + 1))));
  uint32_t* bud = reinterpret_cast<uint32_t*>(take(al(4 * (ncp + 1))));
  uint32_t* tile_off = reinterpret_cast<uint32_t*>(take(al(4 * (ncp + 1))));
  uint32_t* tiles = reinterpret_cast<uint32_t*>(take(al(4 * (ncp + 1))));
  uint32_t* used = reinterpret_cast<uint32_t*>(take(al(4ull * W * nb1)));
  uint32_t* overflow = reinterpret_cast<uint32_t*>(take(256));

  std::vector<DevKeys> redo;
  for (uint64_t first = 0; first < keys.n; first += chunk) {
    const uint64_t m = std::min<uint64_t>(chunk, keys.n - first);
    const uint64_t nst = (m + kst - 1) / kst;
    const uint32_t Wc = (uint32_t)std::min<uint64_t>(W, nst);
    DevKeys dk = keys;
    dk.n = m;
    if (keys.offsets) dk.offsets = keys.offsets + first;
    else dk.data = keys.data + first * keys.fixed_len;
    RSK_HIP(hipMemsetAsync(overflow, 0, 4, c->stream));
    {
      ProfScope ps(c, "bloom_st1");
#define RSK_SA1(F16, KM, TT, ...)                                                                               \
  hipLaunchKernelGGL((bloom_sa1_kernel<F16, KM, TT, uint32_t, ##__VA_ARGS__>), dim3(Wc), dim3(TT), 0, c->stream, dk.data, dk.offsets,    \
                     dk.fixed_len, m, b->fm, b->k, shift1, nb1, nst, region, quota, limit, used, overflow,    \
                     (int)(dbg & 1))
      const uint32_t diag = env_u32("RSK_BLOOM_SA1_DIAG", 0);  // timing diagnostics (not a filter)
      if (kpl4) {
        if (diag == 1) RSK_SA1(true, 8, 512, 1, 4);
        else if (diag == 2) RSK_SA1(true, 8, 512, 2, 4);
        else if (diag == 3) RSK_SA1(true, 8, 512, 3, 4);
        else RSK_SA1(true, 8, 512, 0, 4);
      } else if (diag && f16 && kmax == 8 && t1 == 512) {
        if (diag == 1) RSK_SA1(true, 8, 512, 1);
        else RSK_SA1(true, 8, 512, 2);
      } else if (t1 == 1024) {
        if (f16 && kmax == 8) RSK_SA1(true, 8, 1024);
        else if (f16) RSK_SA1(true, 16, 1024);
        else if (kmax == 8) RSK_SA1(false, 8, 1024);
        else RSK_SA1(false, 16, 1024);
      } else {
        if (f16 && kmax == 8) RSK_SA1(true, 8, 512);
        else if (f16) RSK_SA1(true, 16, 512);
        else if (kmax == 8) RSK_SA1(false, 8, 512);
        else RSK_SA1(false, 16, 512);
      }
#undef RSK_SA1
      RSK_CHECK_LAUNCH("bloom_sa1");
    }
    {
      ProfScope ps(c, "bloom_st_mid");
      hipLaunchKernelGGL(sa_size_kernel<uint32_t>, dim3((ncp + 255) / 256), dim3(256), 0, c->stream, used, Wc, nb1, P, ncp, tot,
                         bud);
      RSK_CHECK_LAUNCH("bloom_sa_size");
      hipLaunchKernelGGL(st_offsets_kernel, dim3(1), dim3(1024), 0, c->stream, tot, bud, ncp, reg_off, tile_off);
      RSK_CHECK_LAUNCH("bloom_st_offsets");
    }
    {
      ProfScope ps(c, "bloom_st2");
      auto k2 = env_u32("RSK_BLOOM_SA2_PF", 0) ? bloom_sa2_kernel<uint32_t, true> : bloom_sa2_kernel<uint32_t, false>;
      hipLaunchKernelGGL(k2, dim3(ncp), dim3(SA2_T), 0, c->stream, region, quota, used, Wc, nb1, P, nb2,
                         reg_off, tile_off, tiles, l2, h2, tb2, (int)(dbg & 2));
      RSK_CHECK_LAUNCH("bloom_sa2");
    }
    {
      ProfScope ps(c, "bloom_st_mid");
      hipLaunchKernelGGL(st_transpose_kernel, dim3((uint32_t)((tt_max + 63) / 64), (nb2 + 1 + 63) / 64), dim3(256), 0,
                         c->stream, h2, tt_max, nb2 + 1, h2t);
      RSK_CHECK_LAUNCH("bloom_st_transpose2");
    }
    {
      ProfScope ps(c, "bloom_st_apply");
      // __launch_bounds__(TA, 8): <= 64 VGPRs, 64 KiB of LDS -> 2 workgroups per CU
      const uint32_t ga = std::min<uint32_t>(ns, 2 * cus);
#define RSK_APPLY(U)                                                                                          \
  hipLaunchKernelGGL((bloom_sa_apply_kernel<U>), dim3(ga), dim3(TA), 0, c->stream, l2, h2t, tt_max, f2, tb2,   \
                     tile_off, tiles, P, ns, b->d_bits, b->nwords)
      if (ua == 16) RSK_APPLY(16);
      else if (ua == 8) RSK_APPLY(8);
      else RSK_APPLY(4);
#undef RSK_APPLY
      RSK_CHECK_LAUNCH("bloom_st_apply");
    }
    uint32_t ov = 0;
    RSK_HIP(hipMemcpyAsync(c->h_small + 8448, overflow, 4, hipMemcpyDeviceToHost, c->stream));
    RSK_HIP(hipStreamSynchronize(c->stream));
    std::memcpy(&ov, c->h_small + 8448, 4);
    if (ov) redo.push_back(dk);
  }
  // A sub-region that filled up (only adversarial inputs can) lost some
  // probes of its chunk; ORing is idempotent, so the chunk is redone by the
  // exact-offset pipeline.
  for (const DevKeys& dk : redo)
    if (!bloom_add_partitioned(c, b, dk)) bloom_add_direct_launch(c, b, dk);
  return true;
}

}  // namespace

// Occupancy of the two persistent Bloom kernels as this process sees it
// (diagnostic: the grids are sized from it).
int bloom_occupancy_probe(int which, int* per_cu) {
  const void* k = which == 0 ? (const void*)bloom_sa1_kernel<true, 8, 512, uint32_t> : (const void*)bloom_sa_apply_kernel<8>;
  const int threads = which == 0 ? 512 : TA;
  *per_cu = -1;
  const hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(per_cu, k, threads, 0);
  if (e != hipSuccess) (void)hipGetLastError();
  return (int)e;
}

bool bloom_add_supertile(rsk_ctx* c, rsk_bloom* b, const DevKeys& keys) {
  const int mode = st_mode();
  const uint64_t k = (uint64_t)b->k;
  const uint64_t nslices = ((uint64_t)b->size + (1ull << SL_LOG) - 1) >> SL_LOG;
  if (mode == 0 || k > 16 || nslices > SL_MAX || keys.n == 0) return false;
  if (mode < 0 && keys.n * k < (1ull << 22)) return false;  // small batches: direct atomics
  const bool f16 =
      keys.offsets == nullptr && keys.fixed_len == 16 && (reinterpret_cast<uintptr_t>(keys.data) & 15) == 0;
  const uint32_t kmax = k <= 8 ? 8 : 16;
  const uint32_t t1 = env_u32("RSK_BLOOM_ST_T1", T1_DEFAULT) == 1024 ? 1024 : 512;
  const uint64_t kst = (uint64_t)t1 * (16 / kmax);
  const uint32_t t2 = env_u32("RSK_BLOOM_ST_T2", T2_DEFAULT) == 512 ? 512 : 1024;
  const uint32_t slots2 = (t2 / 64) * R2;  // probe slots of 64 per st2 tile
  const uint32_t ua = env_u32("RSK_BLOOM_ST_UA", UA_DEFAULT) == 8 ? 8 : 4;
  const uint32_t sb = nbits(nslices - 1);
  const uint32_t f2 = sb > 8 ? sb - 8 : 0;
  const uint32_t shift1 = SL_LOG + f2;
  const uint32_t nb1 = (uint32_t)(((nslices - 1) >> f2) + 1);
  const uint32_t nb2 = 1u << f2;
  const uint32_t ns = (uint32_t)nslices;
  const uint32_t cus = (uint32_t)c->num_cus;
  // parts per coarse bin (sa2 workgroups per bin); RSK_BLOOM_SA_P overrides (tuning)
  const uint32_t P = f2 ? std::max<uint32_t>(1, env_u32("RSK_BLOOM_SA_P", (4 * cus + nb1 - 1) / nb1)) : 1;
  const uint32_t ncp = nb1 * P;
  uint64_t chunk = std::max<uint64_t>(1, probe_chunk() / k / kst) * kst;  // keys per chunk, whole super-tiles
  chunk = std::min<uint64_t>(chunk, keys.n);
  if (f2 && env_u32("RSK_BLOOM_SA", 1)) {
    // 16-byte keys, k <= 8: 4 keys per lane (2048-key super-tiles, bin runs
    // twice as long; 2 workgroups per CU): insert 36.0 -> 35.3 ms at C3, sa2
    // and apply gaining from the longer runs (RSK_BLOOM_SA1_KPL=2: 2 per lane)
    const bool kpl4 = f16 && kmax == 8 && t1 == 512 && env_u32("RSK_BLOOM_SA1_KPL", 4) == 4;
    // sa2 parts per coarse bin: at most two rounds of the two resident
    // 1024-lane workgroups per CU (C3: 143 bins x 7 = 1001 <= 1024 workgroups;
    // 8 parts left a third round 12 % full: sa2 10.9 -> 10.1 ms)
    const uint32_t Psa = std::max<uint32_t>(1, env_u32("RSK_BLOOM_SA_P", 4 * cus / nb1));
    const uint64_t kst_a = kpl4 ? 2048 : kst;
    const uint64_t chunk_a = std::min<uint64_t>(std::max<uint64_t>(1, probe_chunk() / k / kst_a) * kst_a, keys.n);
    return bloom_add_append(c, b, keys, f16, kmax, t1, kst_a, f2, shift1, nb1, Psa, chunk_a, kpl4);
  }
  const uint64_t max_nst = (chunk + kst - 1) / kst;
  const uint64_t max_np = max_nst * kst * k;
  auto al = [](uint64_t x) { return (x + 255) & ~uint64_t(255); };
  // tile-budget bound of the whole chunk (sum over (c, p) of tile_budget)
  const uint64_t tt_max = 2 * ((max_np / 64 + (uint64_t)nb1 * max_nst) / slots2) + 4ull * ncp + 64;
  const uint64_t h1_bytes = al(max_nst * (nb1 + 1) * 2);
  const uint64_t h2_bytes = f2 ? al(tt_max * (nb2 + 1) * 2) : 0;
  const uint64_t meta = al(8 * (ncp + 1)) * 2 + al(4 * (ncp + 1)) * 3 + 256;
  const uint64_t bytes = al(4 * max_np) * (f2 ? 2 : 1) + 2 * h1_bytes + 2 * h2_bytes + (f2 ? al(8 * tt_max) : 0) + meta;
  uint8_t* w = c->work(bytes);
  uint8_t* q = w;
  auto take = [&](uint64_t n) {
    uint8_t* r = q;
    q += n;
    return r;
  };
  uint32_t* l1 = reinterpret_cast<uint32_t*>(take(al(4 * max_np)));
  uint32_t* l2 = f2 ? reinterpret_cast<uint32_t*>(take(al(4 * max_np))) : nullptr;
  uint16_t* h1 = reinterpret_cast<uint16_t*>(take(h1_bytes));
  uint16_t* h1t = reinterpret_cast<uint16_t*>(take(h1_bytes));
  uint16_t* h2 = reinterpret_cast<uint16_t*>(take(h2_bytes));
  uint16_t* h2t = reinterpret_cast<uint16_t*>(take(h2_bytes));
  uint64_t* tb2 = f2 ? reinterpret_cast<uint64_t*>(take(al(8 * tt_max))) : nullptr;
  uint64_t* tot = reinterpret_cast<uint64_t*>(take(al(8 * (ncp + 1))));
  uint64_t* reg_off = reinterpret_cast<uint64_t*>(take(al(8 * (ncp + 1))));
  uint32_t* bud = reinterpret_cast<uint32_t*>(take(al(4 * (ncp + 1))));
  uint32_t* tile_off = reinterpret_cast<uint32_t*>(take(al(4 * (ncp + 1))));
  uint32_t* used = reinterpret_cast<uint32_t*>(take(al(4 * (ncp + 1))));
  uint32_t* overflow = reinterpret_cast<uint32_t*>(take(256));

  std::vector<DevKeys> redo;
  for (uint64_t first = 0; first < keys.n; first += chunk) {
    const uint64_t m = std::min<uint64_t>(chunk, keys.n - first);
    const uint64_t nst = (m + kst - 1) / kst;
    DevKeys dk = keys;
    dk.n = m;
    if (keys.offsets) dk.offsets = keys.offsets + first;
    else dk.data = keys.data + first * keys.fixed_len;
    {
      ProfScope ps(c, "bloom_st1");
#define RSK_ST1(F16, KM, TT)                                                                                   \
  launch_persistent((const void*)bloom_st1_kernel<F16, KM, TT>, TT, nst, c, [&](uint32_t grid) {            \
    hipLaunchKernelGGL((bloom_st1_kernel<F16, KM, TT>), dim3(grid), dim3(TT), 0, c->stream, dk.data,         \
                       dk.offsets, dk.fixed_len, m, b->fm, b->k, shift1, nb1, nst, l1, h1);                   \
  })
      if (t1 == 1024) {
        if (f16 && kmax == 8) RSK_ST1(true, 8, 1024);
        else if (f16) RSK_ST1(true, 16, 1024);
        else if (kmax == 8) RSK_ST1(false, 8, 1024);
        else RSK_ST1(false, 16, 1024);
      } else {
        if (f16 && kmax == 8) RSK_ST1(true, 8, 512);
        else if (f16) RSK_ST1(true, 16, 512);
        else if (kmax == 8) RSK_ST1(false, 8, 512);
        else RSK_ST1(false, 16, 512);
      }
#undef RSK_ST1
      RSK_CHECK_LAUNCH("bloom_st1");
    }
    {
      ProfScope ps(c, "bloom_st_mid");
      hipLaunchKernelGGL(st_transpose_kernel, dim3((uint32_t)((nst + 63) / 64), (nb1 + 1 + 63) / 64), dim3(256), 0,
                         c->stream, h1, nst, nb1 + 1, h1t);
      RSK_CHECK_LAUNCH("bloom_st_transpose1");
      if (f2) {
        hipLaunchKernelGGL(st_size_kernel, dim3(ncp), dim3(256), 0, c->stream, h1t, nst, P, slots2,
                           env_u32("RSK_BLOOM_ST_TINY_BUDGET", 0) ? 1 : 0, tot, bud);
        RSK_CHECK_LAUNCH("bloom_st_size");
        hipLaunchKernelGGL(st_offsets_kernel, dim3(1), dim3(1024), 0, c->stream, tot, bud, ncp, reg_off, tile_off);
        RSK_CHECK_LAUNCH("bloom_st_offsets");
        RSK_HIP(hipMemsetAsync(overflow, 0, 4, c->stream));
      }
    }
    if (f2) {
      {
        ProfScope ps(c, "bloom_st2");
        if (t2 == 512)
          hipLaunchKernelGGL(bloom_st2_kernel<512>, dim3(ncp), dim3(512), 0, c->stream, l1, h1t, nst, kst * k, P,
                             nb2, reg_off, tile_off, bud, used, l2, h2, tb2, overflow);
        else
          hipLaunchKernelGGL(bloom_st2_kernel<1024>, dim3(ncp), dim3(1024), 0, c->stream, l1, h1t, nst, kst * k, P,
                             nb2, reg_off, tile_off, bud, used, l2, h2, tb2, overflow);
        RSK_CHECK_LAUNCH("bloom_st2");
      }
      {
        ProfScope ps(c, "bloom_st_mid");
        hipLaunchKernelGGL(st_transpose_kernel, dim3((uint32_t)((tt_max + 63) / 64), (nb2 + 1 + 63) / 64), dim3(256),
                           0, c->stream, h2, tt_max, nb2 + 1, h2t);
        RSK_CHECK_LAUNCH("bloom_st_transpose2");
      }
    }
    {
      ProfScope ps(c, "bloom_st_apply");
#define RSK_APPLY(U)                                                                                            \
  launch_persistent((const void*)bloom_st_apply_kernel<U>, TA, ns, c, [&](uint32_t grid) {                    \
    if (f2)                                                                                                     \
      hipLaunchKernelGGL((bloom_st_apply_kernel<U>), dim3(grid), dim3(TA), 0, c->stream, l2, h2t, tt_max, f2,    \
                         tb2, (uint64_t)0, (uint64_t)0, tile_off, used, P, ns, b->d_bits, b->nwords);           \
    else                                                                                                        \
      hipLaunchKernelGGL((bloom_st_apply_kernel<U>), dim3(grid), dim3(TA), 0, c->stream, l1, h1t, nst, 0u,       \
                         (const uint64_t*)nullptr, kst * k, nst, (const uint32_t*)nullptr,                      \
                         (const uint32_t*)nullptr, 1u, ns, b->d_bits, b->nwords);                               \
  })
      if (ua == 8) RSK_APPLY(8);
      else RSK_APPLY(4);
#undef RSK_APPLY
      RSK_CHECK_LAUNCH("bloom_st_apply");
    }
    if (f2) {
      uint32_t ov = 0;
      RSK_HIP(hipMemcpyAsync(c->h_small + 8448, overflow, 4, hipMemcpyDeviceToHost, c->stream));
      RSK_HIP(hipStreamSynchronize(c->stream));
      std::memcpy(&ov, c->h_small + 8448, 4);
      if (ov) redo.push_back(dk);
    }
  }
  // A (c, p) that ran out of tile budget (only adversarial inputs can) left
  // some probes of its chunk unapplied.  ORing is idempotent, so such a chunk
  // is simply redone by the exact-offset pipeline (after the loop: it may
  // regrow the scratch the pointers above live in).
  for (const DevKeys& dk : redo)
    if (!bloom_add_partitioned(c, b, dk)) bloom_add_direct_launch(c, b, dk);
  return true;
}

}  // namespace rsk
