// rsk_bloom_reply.hip -- RBloomFilter.add() replies for large batches (gfx950).
//
// RedissonBloomFilter.add (src/main/java/org/redisson/RedissonBloomFilter.java:80-114)
// sends the k SETBITs of an element in one pipeline and answers true iff one
// of the FIRST k-1 replies was 0 (:100-107).  Over a batch the SETBITs run in
// sequence order p = i k + t, so probe p finds its bit clear iff the bit was
// clear before the batch and no probe q < p hit the same bit.  For the reply
// of key i only the smallest KEY over the probes of a bit matters: if
// minkey[b_t] == i for some t < k-1, the first of key i's own probes on that
// bit (t* <= t < k-1) found it clear; otherwise every one of them followed an
// earlier key's probe (or the bit was set before the batch).  Instead of
// sorting all k n (bit, p) pairs, this path partitions 8-byte records
// (key << 32 | offset) down to 2 KiB blocks (2^14 bits) of the filter and takes the
// minimum key per bit in LDS:
//
//   rp1, rp2 : the append partition's sa1 / sa2 (rsk_bloom_sa.h) with 8-byte
//              records: coarse bins, then 64 KiB slices of the filter.
//   rp3      : one workgroup per slice re-sorts its records into the slice's
//              32 blocks of 2^14 bits through LDS (tiles of RP3_TILE records,
//              a 33-entry u16 header per tile), written contiguously.
//   rp_apply : one workgroup per block: minkey[16384] in LDS (64 KiB),
//              atomicMin of every record's key; then the block's first-key
//              table fk[bit] = minkey (NONE where the bit was already set: no
//              probe finds it clear) and the block ORed into the filter.
//   rp_reply : per key, its first k-1 probe indices again; true at the first
//              t with fk[idx_t] == i (early exit, ~1.4 gathers per key at the
//              C3 fill).
// Chunks (< 2^32 - 1 keys, and a bound on the probes for scratch) run one
// after the other, each seeing the filter the previous ones left, exactly
// like the sequential SETBITs; C3 (1B keys, k = 7) is one chunk.
// HBM per probe: 8 B (rp1 write) + 16 (rp2) + 16 (rp3) + 8 (rp_apply), plus
// 4 B per filter bit (fk) and 2 x the filter per chunk, plus the reply pass.
#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "rsk_bloom_sa.h"

namespace rsk {

namespace {

constexpr int RB_LOG = 14;                            // bits per block
constexpr uint32_t RB_BITS = 1u << RB_LOG;            // 16384: minkey in LDS = 64 KiB (2 workgroups per CU)
constexpr uint32_t RB_WORDS = RB_BITS / 32;           // 512 filter words per block
constexpr uint32_t RB_PER_SL = 1u << (SL_LOG - RB_LOG);  // 32 blocks per slice
constexpr uint32_t RP3_CHUNKS = 128;                  // rp3: 64-record chunks per round
constexpr uint32_t NONE = 0xFFFFFFFFu;                // fk: no probe finds this bit clear (never a key index)
constexpr uint32_t RP3_T = 1024;                      // rp3 workgroup
constexpr uint32_t RP3_PER = 8;                       // records per lane per rp3 round
constexpr uint32_t RP3_TILE = RP3_T * RP3_PER;        // 8192 records per rp3 tile
constexpr uint32_t RP3_GROUP = RP3_T;                 // sa2 tiles per rp3 group (one header per lane)
constexpr uint32_t RA_T = 1024;                       // rp_apply workgroup
constexpr uint64_t MAX_CHUNK_KEYS = 0xFFFFFFFEull;    // key indices < NONE
constexpr uint64_t DEFAULT_CHUNK_PROBES = 1ull << 33;  // scratch bound: ~2.3 x 8 B per probe
#ifndef RSK_RP_U
#define RSK_RP_U 2  // rp_reply: keys (gather chains) per lane (1, 2 and 4 measured alike)
#endif

// ------------------------------------------------------------------ sizing
// Slice s = blockIdx.x: its records in the sa2 tiles of coarse bin s >> f2
// (all parts), and the bound on its rp3 tiles (a group of <= RP3_GROUP sa2
// tiles of one part ends in at most one partial rp3 tile).
__global__ __launch_bounds__(256) void rp_size_kernel(const uint16_t* __restrict__ h2t, uint64_t row_stride,
                                                      uint32_t f2, const uint32_t* __restrict__ tile_off,
                                                      const uint32_t* __restrict__ ntile, uint32_t P,
                                                      uint64_t* __restrict__ tot, uint32_t* __restrict__ bud) {
  __shared__ uint64_t part[4];
  const uint32_t s = blockIdx.x, c = s >> f2, f = s & ((1u << f2) - 1);
  const uint16_t* ra = h2t + (uint64_t)f * row_stride;
  const uint16_t* rb = ra + row_stride;
  uint64_t n = 0;
  uint32_t groups = 0;
  for (uint32_t pr = 0; pr < P; ++pr) {
    const uint64_t t0 = tile_off[(uint64_t)c * P + pr], nt = ntile[(uint64_t)c * P + pr];
    for (uint64_t t = t0 + threadIdx.x; t < t0 + nt; t += 256) n += (uint32_t)(rb[t] - ra[t]);
    groups += (uint32_t)((nt + RP3_GROUP - 1) / RP3_GROUP);
  }
  for (int o = 32; o > 0; o >>= 1) n += __shfl_down(n, o, 64);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = n;
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint64_t total = part[0] + part[1] + part[2] + part[3];
    const uint32_t rounds = (uint32_t)((total + RP3_TILE - 1) / RP3_TILE) + groups;
    tot[s] = total + (uint64_t)RB_PER_SL * rounds;  // records + a pad per odd block segment; even (16-byte aligned)
    bud[s] = rounds;
  }
}

// --------------------------------------------------------------------- rp3
// Workgroup = slice s.  Its input is one segment (the slice's fine bin) of
// every sa2 tile of coarse bin c: taken a group of <= 1024 tiles at a time
// (lane j: tile j's segment; a block scan gives the concatenation), in rounds
// of RP3_TILE records: record i of the round is found from a table of the
// segment holding each 64-record chunk start (then a short forward walk over
// the group's starts), ranked by block with an LDS atomic, placed in an LDS
// image and written contiguously at the slice's region with a header
// h3[tile][0..32] (block starts) and its position tb3[tile].  Padding records
// (low word INVALID) are dropped.  The round's barriers order LDS only
// (lds_barrier): a wave's record loads and tile stores stay in flight across
// them (no global data is shared inside the workgroup).
__global__ __launch_bounds__(RP3_T) void rp3_kernel(const uint64_t* __restrict__ in, const uint16_t* __restrict__ h2t,
                                                    uint64_t row_stride, uint32_t f2, const uint64_t* __restrict__ tb2,
                                                    const uint32_t* __restrict__ tile_off,
                                                    const uint32_t* __restrict__ ntile, uint32_t P,
                                                    const uint64_t* __restrict__ slice_off,
                                                    const uint32_t* __restrict__ tile3_off,
                                                    uint64_t* __restrict__ out, uint16_t* __restrict__ h3,
                                                    uint64_t* __restrict__ tb3, uint32_t* __restrict__ ntile3) {
  __shared__ __attribute__((aligned(16))) uint64_t img[RP3_TILE + RB_PER_SL];  // + one pad per odd block segment
  __shared__ uint64_t s_pos[RP3_GROUP];
  __shared__ uint32_t s_pre[RP3_GROUP + 1];
  __shared__ uint16_t tbl[RP3_CHUNKS];
  __shared__ uint32_t wsum[RP3_T / 64];
  __shared__ uint32_t hist[RB_PER_SL + 1], lstart[RB_PER_SL + 1];
  const uint32_t s = blockIdx.x, c = s >> f2, f = s & ((1u << f2) - 1);
  const uint16_t* ra = h2t + (uint64_t)f * row_stride;
  const uint16_t* rb = ra + row_stride;
  const uint64_t base = slice_off[s];
  const uint32_t tbeg = tile3_off[s];
  if (threadIdx.x <= RB_PER_SL) hist[threadIdx.x] = 0;
  uint64_t written = 0;
  uint32_t nt3 = 0;
  // a round's image is written out during the next round, after its record
  // loads and ranks (one vmcnt counts loads and stores: the stores then have
  // the scan and the scatter to drain before the next loads are waited for)
  uint32_t pend = 0;
  uint64_t pend_at = 0;
  auto write_out = [&]() {
    u32x4* o4 = reinterpret_cast<u32x4*>(out + base + pend_at);
    const uint4* i4 = reinterpret_cast<const uint4*>(img);
    for (uint32_t j = threadIdx.x; j < pend / 2; j += RP3_T) {
      const uint4 v = i4[j];
      u32x4 x = {v.x, v.y, v.z, v.w};
      __builtin_nontemporal_store(x, o4 + j);
    }
  };
  for (uint32_t pr = 0; pr < P; ++pr) {
    const uint64_t t0 = tile_off[(uint64_t)c * P + pr], nt = ntile[(uint64_t)c * P + pr];
    for (uint64_t g0 = 0; g0 < nt; g0 += RP3_GROUP) {
      const uint32_t ng = (uint32_t)(nt - g0 < RP3_GROUP ? nt - g0 : RP3_GROUP);
      uint32_t len = 0;
      if (threadIdx.x < ng) {
        const uint64_t t = t0 + g0 + threadIdx.x;
        const uint32_t beg = ra[t];
        len = (uint32_t)rb[t] - beg;
        s_pos[threadIdx.x] = tb2[t] + beg;
      }
      uint32_t total;
      const uint32_t pre = block_scan<RP3_T>(len, &total, wsum);  // (barriers inside)
      if (threadIdx.x < ng) s_pre[threadIdx.x] = pre;
      s_pre[ng] = total;  // (sentinel; written by every lane, same value)
      __syncthreads();
      for (uint32_t r0 = 0; r0 < total; r0 += RP3_TILE) {
        // chunk table: tbl[c] = the segment holding record r0 + 64 c (each
        // non-empty segment claims the chunk starts that fall inside it)
        if (threadIdx.x < ng && len) {
          const uint32_t a = pre, e = pre + len;
          const uint32_t c0 = a > r0 ? (a - r0 + 63) >> 6 : 0;
          const uint32_t c1 = e > r0 ? min(RP3_CHUNKS, (e - r0 + 63) >> 6) : 0;
          for (uint32_t cc = c0; cc < c1; ++cc) tbl[cc] = (uint16_t)threadIdx.x;
        }
        lds_barrier();
        uint64_t rec[RP3_PER];
        uint32_t tag[RP3_PER];
        // two records per lane and load: segments start at even records of
        // 16-byte aligned tiles and have even lengths (sa2 pads runs), so a
        // pair never straddles two segments
#pragma unroll
        for (uint32_t m = 0; m < RP3_PER / 2; ++m) {
          const uint32_t i = r0 + 2 * (m * RP3_T + threadIdx.x);
          rec[2 * m] = rec[2 * m + 1] = rec_pad<uint64_t>();
          if (i < total) {
            uint32_t j = tbl[(i - r0) >> 6];  // then forward over the (few) segments of the chunk
            while (s_pre[j + 1] <= i) ++j;
            unpack16<uint64_t>(ld_nt16(in + s_pos[j] + (i - s_pre[j])), rec + 2 * m);
          }
        }
#pragma unroll
        for (uint32_t m = 0; m < RP3_PER; ++m) {
          tag[m] = INVALID;
          const uint32_t off = rec_off(rec[m]);
          if (off != INVALID) {
            const uint32_t blk = off >> RB_LOG;
            tag[m] = (blk << 16) | atomicAdd(&hist[blk], 1u);
          }
        }
        write_out();  // the previous round
        lds_barrier();
        if (threadIdx.x < 64) {  // block segments padded to even lengths: 16-byte aligned record pairs
          const uint32_t lane = threadIdx.x;
          const uint32_t v = lane < RB_PER_SL ? hist[lane] : 0, v2 = (v + 1) & ~1u;
          const uint32_t incl = wave_scan_incl(v2, lane);
          if (lane < RB_PER_SL) {
            lstart[lane] = incl - v2;
            hist[lane] = 0;
            if (v & 1) img[incl - 1] = rec_pad<uint64_t>();
            h3[(uint64_t)(tbeg + nt3) * (RB_PER_SL + 1) + lane] = (uint16_t)(incl - v2);
          }
          const uint32_t tot = rdl(incl, RB_PER_SL - 1);
          if (lane == 0) {
            h3[(uint64_t)(tbeg + nt3) * (RB_PER_SL + 1) + RB_PER_SL] = (uint16_t)tot;
            tb3[tbeg + nt3] = base + written;
            lstart[RB_PER_SL] = tot;
          }
        }
        lds_barrier();
#pragma unroll
        for (uint32_t m = 0; m < RP3_PER; ++m)
          if (tag[m] != INVALID) img[lstart[tag[m] >> 16] + (tag[m] & 0xFFFFu)] = rec[m];
        pend = lstart[RB_PER_SL];  // even: every segment is
        pend_at = written;
        written += pend;
        ++nt3;
        // the next round's first barrier orders this image before its write-out
      }
    }
  }
  lds_barrier();
  write_out();
  if (threadIdx.x == 0) ntile3[s] = nt3;
}

// ---------------------------------------------------------------- rp_apply
// Workgroup = block b (bits [b 2^14, (b + 1) 2^14), RB_LOG = 14): every segment of it in
// its slice's rp3 tiles (wave w takes tiles w, w + 16, ...; 4 records per lane
// in flight), atomicMin of the key into minkey; then fk[bit] and the filter words,
// 64 bits per wave step (a ballot of "touched" is the MSB-first word pair).
__global__ __launch_bounds__(RA_T) void rp_apply_kernel(const uint64_t* __restrict__ in,
                                                        const uint16_t* __restrict__ h3,
                                                        const uint64_t* __restrict__ tb3,
                                                        const uint32_t* __restrict__ tile3_off,
                                                        const uint32_t* __restrict__ ntile3, uint64_t nblocks,
                                                        uint32_t* __restrict__ bits, uint64_t nwords,
                                                        uint32_t* __restrict__ fk) {
  __shared__ __attribute__((aligned(16))) uint32_t ms[RB_BITS];
  __shared__ uint32_t f0[RB_WORDS];
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  constexpr uint32_t NW = RA_T / 64;
  for (uint64_t b = blockIdx.x; b < nblocks; b += gridDim.x) {
    const uint64_t wbase = b * RB_WORDS;
    uint4* m4 = reinterpret_cast<uint4*>(ms);
    for (uint32_t q = threadIdx.x; q < RB_BITS / 4; q += RA_T) m4[q] = make_uint4(NONE, NONE, NONE, NONE);
    for (uint32_t q = threadIdx.x; q < RB_WORDS; q += RA_T) f0[q] = wbase + q < nwords ? bits[wbase + q] : 0u;
    lds_barrier();
    const uint32_t s = (uint32_t)(b / RB_PER_SL), sub = (uint32_t)(b % RB_PER_SL);
    const uint32_t t0 = tile3_off[s], nt = ntile3[s];
    for (uint32_t j = w; j < nt; j += NW) {
      const uint16_t* hr = h3 + (uint64_t)(t0 + j) * (RB_PER_SL + 1);
      const uint32_t beg = hr[sub], end = hr[sub + 1];
      // segments are even and 16-byte aligned: record pairs, 2 loads in flight per lane
      const uint4* seg = reinterpret_cast<const uint4*>(in + tb3[t0 + j]);
      for (uint32_t o = beg / 2 + lane; o < end / 2; o += 2 * 64) {
        uint64_t r[4];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const uint32_t x = o + 64 * u;
          if (x < end / 2) unpack16<uint64_t>(ld_nt16(seg + x), r + 2 * u);
          else r[2 * u] = r[2 * u + 1] = rec_pad<uint64_t>();
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (rec_off(r[u]) != INVALID) atomicMin(&ms[rec_off(r[u]) & (RB_BITS - 1)], (uint32_t)(r[u] >> 32));
      }
    }
    lds_barrier();
    uint32_t* fkb = fk + b * RB_BITS;
    for (uint32_t o = threadIdx.x; o < RB_BITS; o += RA_T) {  // a wave covers 64 bits = words o/32, o/32 + 1
      const uint32_t v = ms[o];
      const uint32_t was = f0[o >> 5] & bloom_bit_mask(o);
      __builtin_nontemporal_store(was ? NONE : v, &fkb[o]);  // read back by rp_reply's gathers only
      const uint64_t hit = __ballot(v != NONE);
      if (lane == 0 || lane == 32) {
        const uint32_t lo = (uint32_t)(lane == 0 ? hit : hit >> 32);
        const uint32_t word = o >> 5;  // MSB-first bytes of a LE u32 word: bit j -> byte j/8, 0x80 >> j%8
        const uint32_t msk = __builtin_bswap32(__builtin_bitreverse32(lo));
        if (wbase + word < nwords) bits[wbase + word] = f0[word] | msk;
      }
    }
    lds_barrier();  // ms / f0 are reset for the next block
  }
}

// ---------------------------------------------------------------- rp_reply
// Key i of the chunk: true iff fk[idx_t] == i for some t < k - 1.  U
// keys per lane keep U gather chains in flight; a wave stops when every key
// is decided.
template <bool FIXED16, int U>
__global__ __launch_bounds__(256) void rp_reply_kernel(const uint8_t* __restrict__ data,
                                                       const uint64_t* __restrict__ offsets, uint32_t fixed_len,
                                                       uint64_t n, FastMod63 fm, int k,
                                                       const uint32_t* __restrict__ fk, uint8_t* __restrict__ out) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x * U;
  for (uint64_t base = (uint64_t)blockIdx.x * blockDim.x * U + threadIdx.x; base < n; base += stride) {
    ProbeSeq ps[U];
    bool live[U], yes[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t i = base + (uint64_t)u * blockDim.x;
      live[u] = i < n;
      yes[u] = false;
      if (live[u]) {
        uint64_t h1, h2;
        bloom_key_hashes<FIXED16>(data, offsets, fixed_len, i, h1, h2);
        ps[u] = ProbeSeq(h1, h2, fm);
      }
    }
    bool open[U];
#pragma unroll
    for (int u = 0; u < U; ++u) open[u] = live[u];
    for (int t = 0; t < k - 1; ++t) {
      uint32_t v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = open[u] ? fk[ps[u].idx] : NONE;
      bool any = false;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (open[u] && v[u] == (uint32_t)(base + (uint64_t)u * blockDim.x)) {
          yes[u] = true;
          open[u] = false;
        }
        if (t + 2 < k) ps[u].next(t, fm);
        any |= open[u];
      }
      if (!__any(any)) break;
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (live[u]) out[base + (uint64_t)u * blockDim.x] = (uint8_t)yes[u];
  }
}

}  // namespace

// add() with replies through the partition (see the file comment).  Returns
// false when it does not apply: then the caller's sort path runs.
bool bloom_add_replies_append(rsk_ctx* c, rsk_bloom* b, const DevKeys& keys, uint8_t* d_out) {
  const uint64_t k = (uint64_t)b->k;
  const uint64_t nslices = ((uint64_t)b->size + (1ull << SL_LOG) - 1) >> SL_LOG;
  const int route = c->tune.reply;  // 0 auto, 1 this path at any batch size, -1 always the sort path
  const bool force = route > 0;
  if (route < 0 || keys.n == 0 || k > 16 || nslices > SL_MAX) return false;
  if (!force && keys.n * k < (1ull << 22)) return false;
  if (k == 1) {  // no reply looks at any probe (the first k-1 = none)
    RSK_HIP(hipMemsetAsync(d_out, 0, keys.n, c->stream));
    bloom_add_launch(c, b, keys);
    return true;
  }
  const bool f16 =
      keys.offsets == nullptr && keys.fixed_len == 16 && (reinterpret_cast<uintptr_t>(keys.data) & 15) == 0;
  const uint32_t kmax = k <= 8 ? 8 : 16;
  constexpr uint32_t T1 = 512;
  const uint64_t kst = (uint64_t)T1 * (16 / kmax);
  uint32_t sb = 0;
  for (uint64_t v = nslices - 1; v; v >>= 1) ++sb;
  const uint32_t f2 = sb > 8 ? sb - 8 : 0;
  const uint32_t shift1 = SL_LOG + f2;
  const uint32_t nb1 = (uint32_t)(((nslices - 1) >> f2) + 1);
  const uint32_t nb2 = 1u << f2;
  const uint32_t ns = (uint32_t)nslices;
  const uint64_t nblocks = ((uint64_t)b->size + RB_BITS - 1) / RB_BITS;
  const uint32_t cus = (uint32_t)c->num_cus;
  const uint32_t P = std::max<uint32_t>(1, c->tune.sa_parts ? c->tune.sa_parts : 4 * cus / nb1);  // as the insert's sa2
  const uint32_t ncp = nb1 * P;
  const uint64_t probe_cap = c->tune.reply_chunk ? c->tune.reply_chunk : DEFAULT_CHUNK_PROBES;
  uint64_t chunk = std::max<uint64_t>(1, probe_cap / k / kst) * kst;  // keys per chunk, whole super-tiles
  if (chunk > MAX_CHUNK_KEYS) chunk = MAX_CHUNK_KEYS / kst * kst;
  chunk = std::min<uint64_t>(chunk, keys.n);
  const uint64_t max_nst = (chunk + kst - 1) / kst;
  const uint64_t max_np = max_nst * kst * k;
  auto al = [](uint64_t x) { return (x + 255) & ~uint64_t(255); };
  // sa1<u64>: 73 KiB of LDS and <= 128 VGPRs -> 2 workgroups per CU
  const uint32_t W = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>({max_nst, 2ull * cus, SA2_WMAX}));
  const double share = std::min(1.0, (double)(1ull << shift1) / (double)(uint64_t)b->size);  // of a coarse bin
  const uint64_t q64 = (uint64_t)(1.25 * share * (double)max_np / W) + kst * k + (max_nst / W + 1) + 64;
  const uint32_t quota = (uint32_t)((q64 + 3) & ~uint64_t(3));
  const uint32_t limit = c->tune.sa_tiny ? 32 : quota;  // tests force the overflow fallback
  if (q64 >= (1ull << 31) || (uint64_t)nb1 * quota >= (1ull << 32)) return false;
  const uint64_t region_probes = (uint64_t)W * nb1 * quota;
  const uint64_t slots = sa2_slots<uint64_t>();
  const uint64_t tt_max = (max_np + (uint64_t)nb1 * max_nst) / slots + (uint64_t)W * nb1 + 64;  // sa2 tiles
  const uint64_t l2_probes = max_np + (uint64_t)nb1 * max_nst + tt_max * sa2_pad<uint64_t>() + 2ull * ncp;
  const uint64_t tt3_max = l2_probes / RP3_TILE + (uint64_t)ns * (1 + P) + (uint64_t)nb2 * (tt_max / RP3_GROUP + 1) + 64;
  const uint64_t reg_probes = std::max(region_probes, l2_probes + RB_PER_SL * tt3_max);  // rp3 writes into the sa1 region
  const uint64_t h2_bytes = al(tt_max * (nb2 + 1) * 2);
  const uint64_t meta = al(8 * (ncp + 1)) * 2 + al(4 * (ncp + 1)) * 3 + al(4ull * W * nb1) + 256 +
                        al(8 * (ns + 1)) * 2 + al(4 * (ns + 1)) * 3;
  const uint64_t bytes = al(8 * reg_probes) + al(8 * l2_probes) + 2 * h2_bytes + al(8 * tt_max) +
                         al(tt3_max * (RB_PER_SL + 1) * 2) + al(8 * tt3_max) + al(4 * nblocks * RB_BITS) + meta;
  // The scratch (4 B of first-key table per filter bit, 8-byte records of
  // three passes: ~165 GB at C3) must fit the device next to everything
  // else: when it does not, the sort path answers the batch instead (it
  // needs far less).  Reserved before any chunk is applied.
  {
    size_t free_b = 0, total_b = 0;
    if (bytes > c->work_bytes) {  // growing frees the old buffer first
      if (hipMemGetInfo(&free_b, &total_b) == hipSuccess && (double)bytes > 0.9 * (double)(free_b + c->work_bytes))
        return false;
      (void)hipGetLastError();
    }
    try {
      c->work(bytes);
    } catch (const RskError& e) {
      if (e.code != RSK_ERR_OUT_OF_MEMORY) throw;
      (void)hipGetLastError();
      return false;
    }
  }
  for (uint64_t first = 0; first < keys.n; first += chunk) {
    // Scratch is per chunk; taken again each chunk (the sort fallback below may
    // have regrown the work buffer).
    uint8_t* q = c->work(bytes);
    auto take = [&](uint64_t n) {
      uint8_t* r = q;
      q += n;
      return r;
    };
    uint64_t* region = reinterpret_cast<uint64_t*>(take(al(8 * reg_probes)));
    uint64_t* l2 = reinterpret_cast<uint64_t*>(take(al(8 * l2_probes)));
    uint16_t* h2 = reinterpret_cast<uint16_t*>(take(h2_bytes));
    uint16_t* h2t = reinterpret_cast<uint16_t*>(take(h2_bytes));
    uint64_t* tb2 = reinterpret_cast<uint64_t*>(take(al(8 * tt_max)));
    uint16_t* h3 = reinterpret_cast<uint16_t*>(take(al(tt3_max * (RB_PER_SL + 1) * 2)));
    uint64_t* tb3 = reinterpret_cast<uint64_t*>(take(al(8 * tt3_max)));
    uint32_t* fk = reinterpret_cast<uint32_t*>(take(al(4 * nblocks * RB_BITS)));
    uint64_t* tot = reinterpret_cast<uint64_t*>(take(al(8 * (ncp + 1))));
    uint64_t* reg_off = reinterpret_cast<uint64_t*>(take(al(8 * (ncp + 1))));
    uint32_t* bud = reinterpret_cast<uint32_t*>(take(al(4 * (ncp + 1))));
    uint32_t* tile_off = reinterpret_cast<uint32_t*>(take(al(4 * (ncp + 1))));
    uint32_t* tiles = reinterpret_cast<uint32_t*>(take(al(4 * (ncp + 1))));
    uint32_t* used = reinterpret_cast<uint32_t*>(take(al(4ull * W * nb1)));
    uint32_t* overflow = reinterpret_cast<uint32_t*>(take(256));
    uint64_t* tot3 = reinterpret_cast<uint64_t*>(take(al(8 * (ns + 1))));
    uint64_t* slice_off = reinterpret_cast<uint64_t*>(take(al(8 * (ns + 1))));
    uint32_t* bud3 = reinterpret_cast<uint32_t*>(take(al(4 * (ns + 1))));
    uint32_t* tile3_off = reinterpret_cast<uint32_t*>(take(al(4 * (ns + 1))));
    uint32_t* ntile3 = reinterpret_cast<uint32_t*>(take(al(4 * (ns + 1))));
    const uint64_t m = std::min<uint64_t>(chunk, keys.n - first);
    const uint64_t nst = (m + kst - 1) / kst;
    const uint32_t Wc = (uint32_t)std::min<uint64_t>(W, nst);
    DevKeys dk = keys;
    dk.n = m;
    if (keys.offsets) dk.offsets = keys.offsets + first;
    else dk.data = keys.data + first * keys.fixed_len;
    RSK_HIP(hipMemsetAsync(overflow, 0, 4, c->stream));
    {
      ProfScope ps(c, "bloom_rp1");
#define RSK_RP1(F16, KM)                                                                                          \
  hipLaunchKernelGGL((bloom_sa1_kernel<F16, KM, T1, uint64_t>), dim3(Wc), dim3(T1), 0, c->stream, dk.data,        \
                     dk.offsets, dk.fixed_len, m, b->fm, b->k, shift1, nb1, nst, region, quota, limit, used, overflow)
      if (f16 && kmax == 8) RSK_RP1(true, 8);
      else if (f16) RSK_RP1(true, 16);
      else if (kmax == 8) RSK_RP1(false, 8);
      else RSK_RP1(false, 16);
#undef RSK_RP1
      RSK_CHECK_LAUNCH("bloom_rp1");
    }
    uint32_t ov = 0;
    RSK_HIP(hipMemcpyAsync(c->h_small + 8448, overflow, 4, hipMemcpyDeviceToHost, c->stream));
    RSK_HIP(hipStreamSynchronize(c->stream));
    std::memcpy(&ov, c->h_small + 8448, 4);
    if (ov) {
      // A sub-region filled up (only adversarial keys can): nothing of this
      // chunk has been applied, so the sort path answers it exactly.
      bloom_add_replies_sorted(c, b, dk, d_out + first);
      continue;
    }
    {
      ProfScope ps(c, "bloom_rp_mid");
      hipLaunchKernelGGL(sa_size_kernel<uint64_t>, dim3((ncp + 255) / 256), dim3(256), 0, c->stream, used, Wc, nb1, P,
                         ncp, tot, bud);
      RSK_CHECK_LAUNCH("bloom_rp_size2");
      hipLaunchKernelGGL(st_offsets_kernel, dim3(1), dim3(1024), 0, c->stream, tot, bud, ncp, reg_off, tile_off);
      RSK_CHECK_LAUNCH("bloom_rp_offsets2");
    }
    {
      ProfScope ps(c, "bloom_rp2");
      hipLaunchKernelGGL(bloom_sa2_kernel<uint64_t>, dim3(ncp), dim3(SA2_T), 0, c->stream, region, quota, used, Wc,
                         nb1, P, nb2, reg_off, tile_off, tiles, l2, h2, tb2);
      RSK_CHECK_LAUNCH("bloom_rp2");
    }
    {
      ProfScope ps(c, "bloom_rp_mid");
      hipLaunchKernelGGL(st_transpose_kernel, dim3((uint32_t)((tt_max + 63) / 64), (nb2 + 1 + 63) / 64), dim3(256), 0,
                         c->stream, h2, tt_max, nb2 + 1, h2t);
      RSK_CHECK_LAUNCH("bloom_rp_transpose");
      hipLaunchKernelGGL(rp_size_kernel, dim3(ns), dim3(256), 0, c->stream, h2t, tt_max, f2, tile_off, tiles, P, tot3,
                         bud3);
      RSK_CHECK_LAUNCH("bloom_rp_size3");
      hipLaunchKernelGGL(st_offsets_kernel, dim3(1), dim3(1024), 0, c->stream, tot3, bud3, ns, slice_off, tile3_off);
      RSK_CHECK_LAUNCH("bloom_rp_offsets3");
    }
    {
      ProfScope ps(c, "bloom_rp3");
      hipLaunchKernelGGL(rp3_kernel, dim3(ns), dim3(RP3_T), 0, c->stream, l2, h2t, tt_max, f2, tb2, tile_off, tiles,
                         P, slice_off, tile3_off, region, h3, tb3, ntile3);
      RSK_CHECK_LAUNCH("bloom_rp3");
    }
    {
      ProfScope ps(c, "bloom_rp_apply");
      // 66 KiB of LDS: two workgroups per CU, each looping over its blocks
      const uint32_t ga = (uint32_t)std::min<uint64_t>(nblocks, 2ull * cus);
      hipLaunchKernelGGL(rp_apply_kernel, dim3(ga), dim3(RA_T), 0, c->stream, region, h3, tb3, tile3_off, ntile3,
                         nblocks, b->d_bits, b->nwords, fk);
      RSK_CHECK_LAUNCH("bloom_rp_apply");
    }
    {
      ProfScope ps(c, "bloom_rp_reply");
      constexpr int U = RSK_RP_U;  // keys (gather chains) per lane
      const uint64_t g = (m + 256 * U - 1) / (256 * U);
      const uint32_t grid = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(g, 32ull * cus));
      if (f16)
        hipLaunchKernelGGL((rp_reply_kernel<true, U>), dim3(grid), dim3(256), 0, c->stream, dk.data, dk.offsets,
                           dk.fixed_len, m, b->fm, b->k, fk, d_out + first);
      else
        hipLaunchKernelGGL((rp_reply_kernel<false, U>), dim3(grid), dim3(256), 0, c->stream, dk.data, dk.offsets,
                           dk.fixed_len, m, b->fm, b->k, fk, d_out + first);
      RSK_CHECK_LAUNCH("bloom_rp_reply");
    }
  }
  return true;
}

}  // namespace rsk
