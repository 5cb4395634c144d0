// rsk_bloom_st.hip -- Bloom insert for large batches: probes routed to 64 KiB
// filter slices (2^19 bits) held in LDS (gfx950).
//
// RedissonBloomFilter.add (src/main/java/org/redisson/RedissonBloomFilter.java:80-114)
// sets k bits per element (k SETBITs, :94-98) at idx_t = (h_t & Long.MAX_VALUE)
// % size (:116-131).  Setting bits is an OR, so the probes may be applied in
// any order; this path routes them to 64 KiB slices of the filter and ORs each
// slice in LDS, without knowing any count in advance.  Two routes, by filter
// size:
//
//   filters of <= 256 slices (one level):
//   st1   : one pass over the keys.  A super-tile = 2 keys per lane (k <= 8) or
//           1 (k <= 16) of a 512-lane workgroup: each lane hashes its keys once
//           (XXH64 + farmhash), keeps its <= 16 probes in registers, ranks them
//           by slice with one LDS atomic each, places them in an LDS image
//           (double-buffered: the write-out of one super-tile overlaps the
//           hashing of the next) and writes the slice-sorted super-tile
//           CONTIGUOUSLY at its own slot plus a u16 header of slice offsets.
//   hdrT  : header transposed to [slice][super-tile] (coalesced reads below).
//   apply : one workgroup per slice: 64 KiB of filter in LDS, the slice's
//           segment of every super-tile ORed in with ds_or, written back once.
//
//   larger filters (two levels): the append pipeline sa1 -> sa2 -> apply
//   (rsk_bloom_sa.h): sa1 appends each coarse bin's run (2^(19+f2) bits) to
//   its workgroup's private sub-region, sa2 re-sorts every coarse bin by
//   slice into 16-byte aligned tiles, apply ORs each slice's runs in LDS.
//
// HBM per key at k probes: 16 B of key + 4k per record pass (one level: st1
// write, apply read; two levels: sa1 write, sa2 read + write, apply read) +
// ~1 % headers, plus 2 x the filter per chunk.  The exact-offset pipeline
// (rsk_bloom_part.hip) takes k > 16 and chunks whose sub-regions overflow
// (adversarial keys).  Measured variants and their numbers: DESIGN.md 4.
#include <cstdlib>
#include <cstring>

#include "rsk_bloom_sa.h"

namespace rsk {

namespace {

constexpr int T1 = 512;                                // st1 / sa1 workgroup
constexpr int TA = 1024;                               // apply workgroup
constexpr int UA = 8;                                  // apply: segments loaded at once per wave
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

// ----------------------------------------------------------------- apply
// One level: slice s takes its segment of every st1 super-tile t in [0, nst)
// (rows s / s+1 of the transposed headers; super-tile t at t * stride) and
// ORs it into the 64 KiB slice held in LDS.
__global__ __launch_bounds__(TA) void bloom_st_apply_kernel(const uint32_t* __restrict__ probes,
                                                            const uint16_t* __restrict__ ht, uint64_t stride,
                                                            uint64_t nst, uint32_t nslices, uint32_t* __restrict__ bits,
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
    const uint16_t* ra = ht + (uint64_t)s * nst;
    const uint16_t* rb = ra + nst;
    // wave w: groups of 64 consecutive super-tiles 64 (w + NW i), one coalesced
    // header load each, the next group's issued before this one is processed
    uint32_t nlen = 0;
    uint64_t npos = 0;
    auto hload = [&](uint64_t gg) {
      const uint64_t t = gg + lane;
      nlen = 0;
      npos = 0;
      if (t < nst) {
        const uint32_t beg = ra[t];
        nlen = (uint32_t)rb[t] - beg;
        npos = t * stride + beg;
      }
    };
    hload(64ull * w);
    for (uint64_t g = 64ull * w; g < nst; g += 64ull * NW) {
      const uint32_t len = nlen;
      const uint64_t pos = npos;
      hload(g + 64ull * NW);
      const uint32_t ng = (uint32_t)(nst - g < 64 ? nst - g : 64);
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
    __syncthreads();
    for (uint32_t q = threadIdx.x; q < nw4; q += TA) g4[q] = l4[q];
    __syncthreads();
  }
}

// Apply for the append pipeline's sa2h tiles (16-bit records, rsk_bloom_sa.h).
// Slice s = bucket row f = s mod 2^f2 of coarse bin c = s >> f2; the bin's
// tiles are contiguous over its parts.  Lane l of a wave fetches tile g + l's
// row-f uint4 (its 8 bucket starts), the segment end (row f + 1) and the
// tile's base; then a quarter-wave takes one tile's segment [beg, end): each
// of its 16 lanes loads one aligned uint4 (8 records; 128 per quarter), two
// segments per quarter in flight, and derives the 8 records' sub-buckets
// (offset bits 16..18) from the 7 inner starts at once: nibble e of S counts
// the starts at or below position p0 + e.  (One segment per lane instead was
// 2.3x slower: 64 scattered 16-byte loads per instruction.)
RSK_DEV uint32_t shfl32(uint32_t v, uint32_t src) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src << 2), (int)v);
}
RSK_DEV void sah_prep(uint32_t p0, uint32_t beg, uint32_t end, const uint32_t* hk, uint32_t& S, uint32_t& vm) {
  uint32_t sub0 = 0, cnt = 0;
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    sub0 += p0 >= hk[k] ? 1u : 0u;
    const uint32_t d = hk[k] - p0;  // wraps when hk[k] < p0: then >= 8
    cnt += (d - 1u < 7u) ? 1u << (4 * d) : 0u;
  }
  S = (sub0 + cnt) * 0x11111111u;  // nibble e: sub0 + the starts in (p0, p0 + e]
  const uint32_t lo = beg > p0 ? beg - p0 : 0, hi = end - p0 < 8 ? end - p0 : 8;
  vm = ((1u << hi) - 1u) & ~((1u << lo) - 1u);
}
constexpr int SAH_NR = 2;  // segments per quarter in flight (64 VGPRs at 8 waves per SIMD)

// Redis bit i of a 32-bit word (byte i>>3, MSB first) <-> natural bit i
// (1 << i): the bits of every byte reversed, an involution.
RSK_DEV uint32_t byte_bitrev(uint32_t x) { return __builtin_bswap32(__builtin_bitreverse32(x)); }
RSK_DEV uint4 byte_bitrev4(const uint4& v) {
  return make_uint4(byte_bitrev(v.x), byte_bitrev(v.y), byte_bitrev(v.z), byte_bitrev(v.w));
}

// The slice is held in LDS in natural bit order (converted on load and
// write-back), so a record's mask is one shift: 6.07 -> 5.46 ms at C3 (the
// kernel is VALU-bound, profiles/r05_c3_sq.json).  No branch per record (a
// slot outside the segment ORs 0 into its word) measured 8.9 ms: more LDS ops.
__global__ __launch_bounds__(TA, 8) void bloom_sah_apply_kernel(const uint16_t* __restrict__ recs,
                                                             const uint4* __restrict__ hp, uint64_t hp_stride,
                                                             uint32_t f2, const uint32_t* __restrict__ tb,
                                                             const uint64_t* __restrict__ reg_off,
                                                             const uint32_t* __restrict__ tile_off,
                                                             const uint32_t* __restrict__ used, uint32_t P,
                                                             uint32_t nslices, uint32_t* __restrict__ bits,
                                                             uint64_t nwords) {
  __shared__ __attribute__((aligned(16))) uint32_t sl[SL_WORDS];
  const uint32_t lane = threadIdx.x & 63, w = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const uint32_t qt = lane >> 4, ql = lane & 15;  // quarter of the wave, lane inside it
  constexpr uint32_t NW = TA / 64;
  auto apply8 = [&](const uint4& x, uint32_t S, uint32_t vm) {
    const uint32_t wv[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
    for (int e = 0; e < 8; ++e)
      if (vm & (1u << e)) {
        const uint32_t off = (((S >> (4 * e)) & 15u) << 16) | ((wv[e >> 1] >> (16 * (e & 1))) & 0xFFFFu);
        atomicOr(&sl[off >> 5], 1u << (off & 31u));
      }
  };
  for (uint32_t s = xcd_slot(blockIdx.x, gridDim.x); s < nslices; s += gridDim.x) {  // neighbours share segment edges
    const uint64_t w0 = (uint64_t)s * SL_WORDS;
    const uint32_t nw4 = (uint32_t)((nwords - w0 < SL_WORDS ? nwords - w0 : SL_WORDS) / 4);
    uint4* g4 = reinterpret_cast<uint4*>(bits + w0);
    uint4* l4 = reinterpret_cast<uint4*>(sl);
    for (uint32_t q = threadIdx.x; q < nw4; q += TA) l4[q] = byte_bitrev4(g4[q]);
    lds_barrier();  // LDS only: the previous slice's write-back stays in flight
    const uint32_t c = s >> f2, f = s & ((1u << f2) - 1);
    const uint4* hrow = hp + (uint64_t)f * hp_stride;
    const uint32_t* erow = reinterpret_cast<const uint32_t*>(hp + (uint64_t)(f + 1) * hp_stride);
    const uint32_t te = tile_off[(uint64_t)c * P + P - 1] + used[(uint64_t)c * P + P - 1];
    // the bin's records (all parts: contiguous, < 4 GiB) off one uniform base: 32-bit lane offsets
    const uint32_t base8 = (uint32_t)(reg_off[(uint64_t)c * P] / 8);
    const char* rb = reinterpret_cast<const char*>(recs) + 16ull * base8;
    auto rec4 = [&](uint32_t i) { return reinterpret_cast<const uint4*>(rb + 16u * (i - base8)); };
    // lane l: tile g + l -- its 8 bucket starts (pairs), the segment end, its first uint4
    uint32_t nh[5], ntb = 0;
    auto hload = [&](uint32_t gg) {
      const uint32_t t = gg + lane;
      const uint4 v = t < te ? *reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(hrow) + 16u * t)
                             : make_uint4(0, 0, 0, 0);
      nh[0] = v.x;
      nh[1] = v.y;
      nh[2] = v.z;
      nh[3] = v.w;
      nh[4] = t < te ? *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(erow) + 16u * t) & 0xFFFFu : 0;
      ntb = t < te ? *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(tb) + 4u * t) : 0;
    };
    const uint32_t ta = tile_off[(uint64_t)c * P];
    hload(ta + 64 * w);
    for (uint32_t g = ta + 64 * w; g < te; g += 64 * NW) {
      uint32_t h[5];
#pragma unroll
      for (int j = 0; j < 5; ++j) h[j] = nh[j];
      const uint32_t tbl = ntb;
      hload(g + 64 * NW);
      const uint32_t ng = te - g < 64 ? te - g : 64;
      for (uint32_t j = 0; j < ng; j += 4 * SAH_NR) {
        uint4 v[SAH_NR];
        uint32_t S[SAH_NR], vm[SAH_NR], pe[SAH_NR], tbq[SAH_NR];
#pragma unroll
        for (int rd = 0; rd < SAH_NR; ++rd) {
          const uint32_t ti = j + 4 * rd + qt, src = ti < 63 ? ti : 63;
          uint32_t H[5];
#pragma unroll
          for (int k = 0; k < 5; ++k) H[k] = shfl32(h[k], src);
          tbq[rd] = shfl32(tbl, src);
          const uint32_t beg = H[0] & 0xFFFFu, end = ti < ng ? H[4] : beg;
          const uint32_t hk[7] = {H[0] >> 16, H[1] & 0xFFFFu, H[1] >> 16, H[2] & 0xFFFFu,
                                  H[2] >> 16, H[3] & 0xFFFFu, H[3] >> 16};
          const uint32_t p0 = (beg & ~7u) + 8 * ql;
          v[rd] = p0 < end ? ld_nt16(rec4(tbq[rd] + p0 / 8)) : make_uint4(0, 0, 0, 0);
          pe[rd] = end > p0 + 128 ? end : 0;  // nonzero: a long segment (the rest after this pass)
          vm[rd] = 0;
          S[rd] = 0;
          if (p0 < end) sah_prep(p0, beg, end, hk, S[rd], vm[rd]);
        }
#pragma unroll
        for (int rd = 0; rd < SAH_NR; ++rd) {
          apply8(v[rd], S[rd], vm[rd]);
          if (pe[rd]) {  // segments longer than 128 records (rare): starts again
            const uint32_t t = g + j + 4 * rd + qt;
            const uint4 hv = *reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(hrow) + 16u * t);
            const uint32_t hk[7] = {hv.x >> 16, hv.y & 0xFFFFu, hv.y >> 16, hv.z & 0xFFFFu,
                                    hv.z >> 16, hv.w & 0xFFFFu, hv.w >> 16};
            const uint32_t beg = hv.x & 0xFFFFu;
            for (uint32_t p0 = (beg & ~7u) + 8 * ql + 128; p0 < pe[rd]; p0 += 128) {
              uint32_t S2, vm2;
              sah_prep(p0, beg, pe[rd], hk, S2, vm2);
              apply8(*rec4(tbq[rd] + p0 / 8), S2, vm2);
            }
          }
        }
      }
    }
    lds_barrier();
    for (uint32_t q = threadIdx.x; q < nw4; q += TA) g4[q] = byte_bitrev4(l4[q]);
    lds_barrier();
  }
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

// A chunk whose sub-regions (sa1) overflowed lost some probes; ORing is
// idempotent, so it is redone by the exact-offset pipeline (after the chunk
// loop: that may regrow the scratch the pipeline's pointers live in).
void redo_chunks(rsk_ctx* c, rsk_bloom* b, const std::vector<DevKeys>& redo) {
  for (const DevKeys& dk : redo)
    if (!bloom_add_partitioned(c, b, dk)) bloom_add_direct_launch(c, b, dk);
}

// The append pipeline (sa1 -> sa2 -> apply) for filters of more than 256 slices.
// kpl4: 16-byte keys with k <= 8 take 4 keys per lane (2048-key super-tiles,
// bin runs twice as long; 2 workgroups per CU): insert 36.0 -> 35.3 ms at C3.
bool bloom_add_append(rsk_ctx* c, rsk_bloom* b, const DevKeys& keys, bool f16, uint32_t kmax, uint64_t kst,
                      uint32_t f2, uint32_t shift1, uint32_t nb1, uint32_t P, uint64_t chunk, bool kpl4) {
  const uint64_t k = (uint64_t)b->k;
  const uint32_t ns = (uint32_t)(((uint64_t)b->size + (1ull << SL_LOG) - 1) >> SL_LOG);
  const uint32_t nb2 = 1u << f2;
  const uint32_t ncp = nb1 * P;
  const uint32_t cus = (uint32_t)c->num_cus;
  const uint64_t max_nst = (chunk + kst - 1) / kst;
  const uint64_t max_np = max_nst * kst * k;
  auto al = [](uint64_t x) { return (x + 255) & ~uint64_t(255); };
  // Workgroups per CU from the kernels' own budgets, not from
  // hipOccupancyMaxActiveBlocksPerMultiprocessor: in a process that has
  // imported torch the runtime reads these code objects' metadata through
  // torch's comgr and answers 1, a third of the grid.
  // sa1<512>: __launch_bounds__(512, 6) caps it at 80 VGPRs (6 waves per
  // SIMD), 43 KiB of LDS -> 3; with 4 keys per lane 73 KiB of LDS -> 2.
  const int per_cu = kpl4 ? 2 : 3;
  // W persistent sa1 workgroups; each gets 1.25x its expected share of a full
  // coarse bin per bin, plus one whole super-tile (a tile's run can be that
  // long) and the <= 3 padding slots per run of each of its tiles.
  const uint32_t W = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>({max_nst, (uint64_t)per_cu * cus, SA2_WMAX}));
  const double share = (double)(1ull << shift1) / (double)(uint64_t)b->size;
  // quota > one tile's probes: a valid run offset b quota + pos - lstart never equals INVALID
  const uint64_t q64 = (uint64_t)(1.25 * share * (double)max_np / W) + kst * k + 3 * (max_nst / W + 1) + 64;
  const uint32_t quota = (uint32_t)((q64 + 3) & ~uint64_t(3));
  const uint32_t limit = c->tune.sa_tiny ? 32 : quota;  // tests force the overflow fallback
  const uint64_t region_probes = (uint64_t)W * nb1 * quota;
  if (q64 >= (1ull << 31) || (uint64_t)nb1 * quota >= (1ull << 32)) return false;  // u32 offsets -> exact-offset pipeline
  const uint32_t nbk = nb2 << SAH_SUB;  // sa2h buckets per coarse bin
  const int V2 = c->tune.sa_v == 6 || c->tune.sa_v == 8 ? c->tune.sa_v : SA2_V;  // sa2h: uint4 per lane per tile
  const uint32_t slots2 = SA2_T * 4 * V2;
  const uint64_t tt_max = (max_np + 3ull * nb1 * max_nst) / slots2 + (uint64_t)W * nb1 + 64;  // bound on sa2 tiles
  const uint64_t l2_slots = max_np + 3ull * nb1 * max_nst + 8 * tt_max + 8ull * ncp;  // sa2h output (u16), aligned tiles
  const uint64_t hp_bytes = al(16 * tt_max * (nb2 + 1));  // bucket-start rows: nb2 + 1 rows of tt_max uint4
  // apply's 32-bit uint4 indices of the records
  if (l2_slots / 8 >= (1ull << 32)) return false;
  const uint64_t meta = al(8 * (ncp + 1)) * 2 + al(4 * (ncp + 1)) * 3 + al(4ull * W * nb1) + 256;
  const uint64_t bytes = al(4 * region_probes) + al(2 * l2_slots) + hp_bytes + al(4 * tt_max) + meta;
  uint8_t* w = c->work(bytes);
  uint8_t* q = w;
  auto take = [&](uint64_t n) {
    uint8_t* r = q;
    q += n;
    return r;
  };
  uint32_t* region = reinterpret_cast<uint32_t*>(take(al(4 * region_probes)));
  uint16_t* l2 = reinterpret_cast<uint16_t*>(take(al(2 * l2_slots)));
  uint4* hp = reinterpret_cast<uint4*>(take(hp_bytes));
  uint32_t* tb2 = reinterpret_cast<uint32_t*>(take(al(4 * tt_max)));
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
    // the timing-only contiguous form needs nst whole images in the region
    const int sa_dbg = c->tune.sa_dbg && nst * (kst * kmax + 1024) <= region_probes ? 1 : 0;
    {
      ProfScope ps(c, "bloom_st1");
#define RSK_SA1(F16, KM, ...)                                                                                   \
  hipLaunchKernelGGL((bloom_sa1_kernel<F16, KM, T1, uint32_t, ##__VA_ARGS__>), dim3(Wc), dim3(T1), 0, c->stream, \
                     dk.data, dk.offsets, dk.fixed_len, m, b->fm, b->k, shift1, nb1, nst, region, quota, limit,  \
                     used, overflow, 0u, 1u, sa_dbg | (c->tune.sa_full < 0 ? 2 : 0))
      if (kpl4 && b->k == 7 && c->tune.sa_hash == 1) RSK_SA1(true, 8, 4, false, 7, 1);  // timing only
      else if (kpl4 && b->k == 7 && c->tune.sa_hash == 2) RSK_SA1(true, 8, 4, false, 7, 2);  // timing only
      else if (kpl4 && b->k == 7 && c->tune.sa_kc >= 0) RSK_SA1(true, 8, 4, false, 7);  // C3's k (1 % FPP)
      else if (kpl4) RSK_SA1(true, 8, 4);
      else if (f16 && kmax == 8) RSK_SA1(true, 8);
      else if (f16) RSK_SA1(true, 16);
      else if (kmax == 8) RSK_SA1(false, 8);
      else RSK_SA1(false, 16);
#undef RSK_SA1
      RSK_CHECK_LAUNCH("bloom_sa1");
    }
    if (sa_dbg) continue;  // timing-only sa1 form: its output is not the sub-regions
    {
      ProfScope ps(c, "bloom_st_mid");
      hipLaunchKernelGGL(sah_size_kernel, dim3((ncp + 255) / 256), dim3(256), 0, c->stream, used, Wc, nb1, P, ncp,
                         tot, bud, slots2);
      RSK_CHECK_LAUNCH("bloom_sa_size");
      hipLaunchKernelGGL(st_offsets_kernel, dim3(1), dim3(1024), 0, c->stream, tot, bud, ncp, reg_off, tile_off);
      RSK_CHECK_LAUNCH("bloom_st_offsets");
    }
    {
      ProfScope ps(c, "bloom_st2");
#define RSK_SA2H(V)                                                                                              \
  hipLaunchKernelGGL((bloom_sa2h_kernel<uint16_t, V>), dim3(ncp), dim3(SA2_T), 0, c->stream, region, quota, used, Wc, \
                     nb1, P, nbk, reg_off, tile_off, tiles, l2, hp, tt_max, tb2)
      if (V2 == 8) RSK_SA2H(8);
      else if (V2 == 6) RSK_SA2H(6);
      else RSK_SA2H(SA2_V);
#undef RSK_SA2H
      RSK_CHECK_LAUNCH("bloom_sa2");
    }
    {
      ProfScope ps(c, "bloom_st_apply");
      // __launch_bounds__(TA, 8): <= 64 VGPRs, 64 KiB of LDS -> 2 workgroups per CU
      const uint32_t ga = std::min<uint32_t>(ns, 2 * cus);
      hipLaunchKernelGGL(bloom_sah_apply_kernel, dim3(ga), dim3(TA), 0, c->stream, l2, hp, tt_max, f2, tb2, reg_off,
                         tile_off, tiles, P, ns, b->d_bits, b->nwords);
      RSK_CHECK_LAUNCH("bloom_st_apply");
    }
    uint32_t ov = 0;
    RSK_HIP(hipMemcpyAsync(c->h_small + 8448, overflow, 4, hipMemcpyDeviceToHost, c->stream));
    RSK_HIP(hipStreamSynchronize(c->stream));
    std::memcpy(&ov, c->h_small + 8448, 4);
    if (ov) redo.push_back(dk);
  }
  redo_chunks(c, b, redo);
  return true;
}

// One level (<= 256 slices): st1 -> header transpose -> apply.
void bloom_add_one_level(rsk_ctx* c, rsk_bloom* b, const DevKeys& keys, bool f16, uint32_t kmax, uint64_t kst,
                         uint64_t chunk) {
  const uint64_t k = (uint64_t)b->k;
  const uint32_t ns = (uint32_t)(((uint64_t)b->size + (1ull << SL_LOG) - 1) >> SL_LOG);
  const uint64_t max_nst = (chunk + kst - 1) / kst;
  const uint64_t max_np = max_nst * kst * k;
  auto al = [](uint64_t x) { return (x + 255) & ~uint64_t(255); };
  const uint64_t h1_bytes = al(max_nst * (ns + 1) * 2);
  uint8_t* q = c->work(al(4 * max_np) + 2 * h1_bytes);
  uint32_t* l1 = reinterpret_cast<uint32_t*>(q);
  uint16_t* h1 = reinterpret_cast<uint16_t*>(q + al(4 * max_np));
  uint16_t* h1t = h1 + h1_bytes / 2;
  for (uint64_t first = 0; first < keys.n; first += chunk) {
    const uint64_t m = std::min<uint64_t>(chunk, keys.n - first);
    const uint64_t nst = (m + kst - 1) / kst;
    DevKeys dk = keys;
    dk.n = m;
    if (keys.offsets) dk.offsets = keys.offsets + first;
    else dk.data = keys.data + first * keys.fixed_len;
    {
      ProfScope ps(c, "bloom_st1");
#define RSK_ST1(F16, KM)                                                                                       \
  launch_persistent((const void*)bloom_st1_kernel<F16, KM, T1>, T1, nst, c, [&](uint32_t grid) {            \
    hipLaunchKernelGGL((bloom_st1_kernel<F16, KM, T1>), dim3(grid), dim3(T1), 0, c->stream, dk.data,         \
                       dk.offsets, dk.fixed_len, m, b->fm, b->k, (uint32_t)SL_LOG, ns, nst, l1, h1);         \
  })
      if (f16 && kmax == 8) RSK_ST1(true, 8);
      else if (f16) RSK_ST1(true, 16);
      else if (kmax == 8) RSK_ST1(false, 8);
      else RSK_ST1(false, 16);
#undef RSK_ST1
      RSK_CHECK_LAUNCH("bloom_st1");
    }
    {
      ProfScope ps(c, "bloom_st_mid");
      hipLaunchKernelGGL(st_transpose_kernel, dim3((uint32_t)((nst + 63) / 64), (ns + 1 + 63) / 64), dim3(256), 0,
                         c->stream, h1, nst, ns + 1, h1t);
      RSK_CHECK_LAUNCH("bloom_st_transpose1");
    }
    {
      ProfScope ps(c, "bloom_st_apply");
      launch_persistent((const void*)bloom_st_apply_kernel, TA, ns, c, [&](uint32_t grid) {
        hipLaunchKernelGGL(bloom_st_apply_kernel, dim3(grid), dim3(TA), 0, c->stream, l1, h1t, kst * k, nst, ns,
                           b->d_bits, b->nwords);
      });
      RSK_CHECK_LAUNCH("bloom_st_apply");
    }
  }
}

}  // namespace

bool bloom_add_supertile(rsk_ctx* c, rsk_bloom* b, const DevKeys& keys) {
  const int route = c->tune.bloom_stream;  // 0 auto, 1 at any batch size, -1 never
  const uint64_t k = (uint64_t)b->k;
  const uint64_t nslices = ((uint64_t)b->size + (1ull << SL_LOG) - 1) >> SL_LOG;
  if (route < 0 || k > 16 || nslices > SL_MAX || keys.n == 0) return false;
  if (route == 0 && keys.n * k < (1ull << 22)) return false;  // small batches: direct atomics
  const bool f16 =
      keys.offsets == nullptr && keys.fixed_len == 16 && (reinterpret_cast<uintptr_t>(keys.data) & 15) == 0;
  const uint32_t kmax = k <= 8 ? 8 : 16;
  const uint32_t sb = nbits(nslices - 1);
  const uint32_t f2 = sb > 8 ? sb - 8 : 0;
  const uint64_t probe_chunk = c->tune.bloom_chunk ? c->tune.bloom_chunk : DEFAULT_PROBE_CHUNK;
  if (f2 == 0) {
    const uint64_t kst = (uint64_t)T1 * (16 / kmax);
    const uint64_t chunk = std::min<uint64_t>(std::max<uint64_t>(1, probe_chunk / k / kst) * kst, keys.n);
    bloom_add_one_level(c, b, keys, f16, kmax, kst, chunk);
    return true;
  }
  const uint32_t shift1 = SL_LOG + f2;
  const uint32_t nb1 = (uint32_t)(((nslices - 1) >> f2) + 1);
  const uint32_t cus = (uint32_t)c->num_cus;
  const bool kpl4 = f16 && kmax == 8;
  // sa2 parts per coarse bin: at most two rounds of the two resident
  // 1024-lane workgroups per CU (C3: 143 bins x 7 = 1001 <= 1024 workgroups;
  // 8 parts left a third round 12 % full: sa2 10.9 -> 10.1 ms)
  const uint32_t P = std::max<uint32_t>(1, c->tune.sa_parts ? c->tune.sa_parts : 4 * cus / nb1);
  const uint64_t kst = kpl4 ? 2048 : (uint64_t)T1 * (16 / kmax);
  const uint64_t chunk = std::min<uint64_t>(std::max<uint64_t>(1, probe_chunk / k / kst) * kst, keys.n);
  return bloom_add_append(c, b, keys, f16, kmax, kst, f2, shift1, nb1, P, chunk, kpl4);
}

}  // namespace rsk
