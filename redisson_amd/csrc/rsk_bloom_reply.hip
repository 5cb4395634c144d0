// rsk_bloom_reply.hip -- RBloomFilter.add() replies for large batches (gfx950).
//
// RedissonBloomFilter.add (src/main/java/org/redisson/RedissonBloomFilter.java:80-114)
// sends the k SETBITs of an element in one pipeline and answers true iff one
// of the FIRST k-1 replies was 0 (:100-107; BitSetReplayConvertor: true = the
// old bit was 0).  Over a batch the SETBITs run in sequence order p = i k + t,
// so key i answers true iff for some t < k-1 its probe (i, t) is the FIRST
// probe of bit b_t in the batch and b_t was clear before it.
//
// Key groups.  The keys of a chunk are cut into <= 32766 groups of
// consecutive keys (a group = gs super-tiles of one sa1 workgroup's
// contiguous range), numbered in key order: tag(i).  The first prober of a
// bit then lies in the group with the smallest tag among the bit's probes,
// and when that group probed the bit only once, that one probe is the first.
// So the partition only has to carry each probe's 15-bit group tag, not its
// key index, and the per-bit answer is 2 bytes:
//
//   rp1 (sa1, TAGGED) : keys hashed once, 4-byte records (bin offset | group
//                       in the top 6 bits) appended to per-workgroup
//                       sub-regions of 2^26-bit coarse bins.
//   rp2 (sa2h<u32>)   : each coarse bin re-sorted into buckets of 2^16 bits;
//                       records (tag << 16 | offset).
//   rp_tapply         : one workgroup per bucket: e[bit] = (min tag << 1) |
//                       (min tag seen once) in 128 KiB of LDS (u16 per bit,
//                       CAS on the word pair); T[bit] = e, or NONE where the
//                       bit was set before the batch; the bucket ORed into
//                       the filter.
//   rp_treply         : one workgroup per group: key i's first k-1 probes
//                       gathered from T (early exit): T == tag(i) << 1 | 1 ->
//                       true.  T == tag(i) << 1 (the group probed the bit more
//                       than once: rare, ~2.5 x group size per chunk) leaves
//                       the key pending; the workgroup then scans its group's
//                       keys again for the pending bits (LDS hash, minimum
//                       (key, t) per bit) and answers them exactly.
//
// A chunk whose sub-regions overflow (adversarial keys; before anything is
// applied), or whose pending probes do not fit a group's LDS tables (e.g. a
// batch of adjacent duplicates), is answered by the sort path: in the second
// case the filter is first restored from T (bits with T != NONE were clear).
// HBM per probe: 4 B (rp1 write) + 8 (rp2) + 4 (rp_tapply) = 16 B, plus 2 B
// of T per filter bit and 2 x the filter per chunk, the keys read twice and
// the reply pass's ~1.4 random 2-byte gathers per key.
#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "rsk_bloom_sa.h"

namespace rsk {

namespace {

constexpr uint32_t BK_LOG = 16;                        // bits per bucket (rp2's unit)
constexpr uint32_t BK_BITS = 1u << BK_LOG;             // u16 entry per bit in LDS: 128 KiB
constexpr uint32_t T_NONE = 0xFFFFu;                   // T: no probe finds this bit clear
constexpr uint32_t MAX_TAGS = 32766;                   // group tags: (tag << 1) | 1 < T_NONE
constexpr uint32_t TA_T = 1024;                        // rp_tapply workgroup
constexpr uint32_t RR_T = 256;                         // rp_treply workgroup
constexpr uint32_t PEND_CAP = 256;                     // rp_treply: pending keys per group
constexpr uint32_t HS = 1024;                          // rp_treply: hash slots for pending bits
constexpr uint32_t HS_MAX = 768;                       // ... at most this many distinct bits
constexpr uint64_t HS_EMPTY = ~0ull;
constexpr uint64_t MAX_CHUNK_KEYS = 1ull << 32;
constexpr uint64_t DEFAULT_CHUNK_PROBES = 1ull << 33;  // scratch bound: ~10 B per probe

RSK_DEV uint32_t shfl_u32(uint32_t v, uint32_t src) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src << 2), (int)v);
}

// e = (tag << 1) | once: fold one probe of group `tag` into the u16 entry of
// bit `off` (two entries per LDS word; CAS on the word).  (A first CAS that
// assumes the word untouched instead of reading it measured 27.8 against
// 22.0 ms for the whole pass: the failed CASes cost more than the reads.)
RSK_DEV void tap_fold(uint32_t* tt, uint32_t rec) {
  const uint32_t tag = rec >> 16, off = rec & 0xFFFFu;
  uint32_t* wp = tt + (off >> 1);
  const uint32_t sh = (off & 1u) * 16u;
  uint32_t old = *wp;
  while (true) {
    const uint32_t cur = (old >> sh) & 0xFFFFu, ctag = cur >> 1;
    if (tag > ctag || (tag == ctag && !(cur & 1u))) break;  // an earlier group, or already seen twice
    const uint32_t ne = tag < ctag ? (tag << 1) | 1u : tag << 1;
    const uint32_t nw = (old & ~(0xFFFFu << sh)) | (ne << sh);
    const uint32_t prev = atomicCAS(wp, old, nw);
    if (prev == old) break;
    old = prev;
  }
}

// ---------------------------------------------------------------- rp_tapply
// Workgroup = bucket u (bits [u 2^16, (u + 1) 2^16)) = sub-bucket e = u mod 8
// of slice s = u / 8, in coarse bin c = s >> f2 (row f = s mod 2^f2 of the
// rp2 headers: per tile one uint4 of the 8 u16 starts of the slice's
// buckets; row f + 1's first u16 ends sub-bucket 7).  Lane l of a wave loads
// tile g + l's bounds; then four lanes take one tile's segment (two aligned
// uint4 each = 32 record slots, the rest of a long segment in a loop), 16
// segments per wave step, the loads of S steps issued before the first of
// them is folded.  A record is folded by an LDS read and a CAS (retried when
// another record took the word).  One workgroup per CU, so the latencies at
// a bucket's start are exposed: the next bucket's filter words and each
// wave's first 64 tile bounds are loaded during this bucket's write-out.
// Consecutive buckets run on one XCD (xcd_slot): the 8 buckets of a slice
// share their segments' cache lines in its L2.  (Measured at C3, rp2 tiles of
// 24576 records: S = 1 20.9 ms, 2 20.5, 4 21.3; a step's 8 records folded as
// a batch -- every read, then every CAS -- 21.9; a software pipeline, next
// step's loads during this step's folds, 21.8; half buckets, two workgroups
// per CU, 26.5.)
template <int S, int SU = 2>
__global__ __launch_bounds__(TA_T) void rp_tapply_kernel(const uint32_t* __restrict__ recs,
                                                         const uint4* __restrict__ hp, uint64_t hp_stride,
                                                         uint32_t f2, const uint32_t* __restrict__ tb,
                                                         const uint32_t* __restrict__ tile_off,
                                                         const uint32_t* __restrict__ ntiles, uint32_t P,
                                                         uint64_t nbuckets, uint32_t* __restrict__ bits,
                                                         uint64_t nwords, uint16_t* __restrict__ T, int dbg,
                                                         int strided) {
  __shared__ __attribute__((aligned(16))) uint32_t tt[BK_BITS / 2];
  __shared__ __attribute__((aligned(16))) uint32_t f0[BK_BITS / 32];
  constexpr uint32_t FW = BK_BITS / 32 / TA_T;  // filter words per lane (2)
  const uint32_t lane = threadIdx.x & 63, w = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  constexpr uint32_t NW = TA_T / 64;
  const uint4* r4 = reinterpret_cast<const uint4*>(recs);
  auto fold1 = [&](uint32_t x) {
    if (dbg & 1) tt[x & 0x7FFFu] |= x >> 31;  // timing only: one plain LDS op per record
    else tap_fold(tt, x);
  };
  // a bucket's place in the rp2 output
  struct Bk {
    uint32_t e, ta, te;
    const uint4* hrow;
    const uint32_t* erow;
  };
  auto bucket = [&](uint64_t u) {
    const uint32_t s = (uint32_t)(u >> 3), c = s >> f2, f = s & ((1u << f2) - 1);
    Bk k;
    k.e = (uint32_t)(u & 7);
    k.hrow = hp + (uint64_t)f * hp_stride;
    k.erow = reinterpret_cast<const uint32_t*>(hp + (uint64_t)(f + 1) * hp_stride);
    k.ta = tile_off[(uint64_t)c * P];
    k.te = tile_off[(uint64_t)c * P + P - 1] + ntiles[(uint64_t)c * P + P - 1];
    return k;
  };
  // the wave's share of the bucket's tiles: an equal slice each (a wave of 64
  // lanes loads 64 tiles' bounds at a time), so no wave runs a round more than
  // another -- at C3 a bucket has ~1500 tiles: waves striding by 1024 tiles
  // left half of them with two full rounds of 64 tiles, the rest with one
  // (strided, A/B: route reply_bal = -1 -- wave w takes tiles w*64.. then every 1024th)
  const uint32_t gstep = strided ? 64 * NW : 64;
  auto wrange = [&](const Bk& k, uint32_t& a, uint32_t& b) {
    const uint64_t T = k.te - k.ta;
    a = strided ? k.ta + 64 * w : k.ta + (uint32_t)(T * w / NW);
    b = strided ? k.te : k.ta + (uint32_t)(T * (w + 1) / NW);
  };
  // lane's tile g + lane (below lim): segment bounds of the bucket and the tile's first uint4
  auto hload = [&](const Bk& k, uint32_t g, uint32_t lim, uint32_t& beg, uint32_t& end, uint32_t& tbl) {
    const uint32_t t = g + lane;
    beg = end = tbl = 0;
    if (t < lim) {
      const uint4 v = k.hrow[t];
      const uint32_t hw[4] = {v.x, v.y, v.z, v.w};
      beg = (hw[k.e >> 1] >> (16 * (k.e & 1))) & 0xFFFFu;
      end = k.e < 7 ? (hw[(k.e + 1) >> 1] >> (16 * ((k.e + 1) & 1))) & 0xFFFFu : k.erow[4ull * t] & 0xFFFFu;
      tbl = tb[t];
    }
  };
  uint64_t u = xcd_slot(blockIdx.x, gridDim.x);
  // prefetched for bucket u: its filter words and this wave's first tile bounds
  uint32_t pfw[FW], pbeg = 0, pend = 0, ptb = 0;
  Bk k{};
  uint32_t wa = 0, wb = 0;  // this wave's tiles of the current bucket
  if (u < nbuckets) {
    k = bucket(u);
    wrange(k, wa, wb);
#pragma unroll
    for (uint32_t i = 0; i < FW; ++i) {
      const uint64_t q = u * (BK_BITS / 32) + threadIdx.x + i * TA_T;
      pfw[i] = q < nwords ? bits[q] : 0u;
    }
    hload(k, wa, wb, pbeg, pend, ptb);
  }
  for (; u < nbuckets; u += gridDim.x) {
    uint4* t4 = reinterpret_cast<uint4*>(tt);
    for (uint32_t q = threadIdx.x; q < BK_BITS / 8; q += TA_T) t4[q] = make_uint4(~0u, ~0u, ~0u, ~0u);
#pragma unroll
    for (uint32_t i = 0; i < FW; ++i) f0[threadIdx.x + i * TA_T] = pfw[i];
    lds_barrier();
    for (uint32_t g = wa; g < wb; g += gstep) {
      uint32_t beg, end, tbl;
      if (g == wa) {
        beg = pbeg;
        end = pend;
        tbl = ptb;
      } else {
        hload(k, g, wb, beg, end, tbl);
      }
      const uint32_t ng = wb - g < 64 ? wb - g : 64;
      for (uint32_t j0 = 0; j0 < ng; j0 += 16 * S) {
        uint4 v[S][SU];
        uint32_t sb[S], se[S], st[S], p0[S];
#pragma unroll
        for (int q = 0; q < S; ++q) {
          const uint32_t si = j0 + 16 * q + (lane >> 2), src = si < 63 ? si : 63;
          sb[q] = shfl_u32(beg, src);
          const uint32_t se0 = shfl_u32(end, src);
          st[q] = shfl_u32(tbl, src);
          se[q] = si < ng ? se0 : sb[q];
          p0[q] = (sb[q] & ~3u) + 4 * (lane & 3);
          // plain loads: the slice's 8 buckets (on one XCD at about the same time) share these lines in L2
#pragma unroll
          for (int i = 0; i < SU; ++i)
            v[q][i] = p0[q] + 16 * i < se[q] ? r4[st[q] + p0[q] / 4 + 4 * i] : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int q = 0; q < S; ++q) {
#pragma unroll
          for (int i = 0; i < SU; ++i) {
            const uint32_t x[4] = {v[q][i].x, v[q][i].y, v[q][i].z, v[q][i].w};
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const uint32_t pos = p0[q] + 16 * i + r;
              if (pos >= sb[q] && pos < se[q]) fold1(x[r]);
            }
          }
          for (uint32_t p = p0[q] + 16 * SU; p < se[q]; p += 16) {  // long segments (rare)
            const uint4 v = r4[st[q] + p / 4];
            const uint32_t y[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int r = 0; r < 4; ++r)
              if (p + r >= sb[q] && p + r < se[q]) fold1(y[r]);
          }
        }
      }
    }
    // the next bucket's filter words and first tile bounds, in flight during the write-out
    const uint64_t un = u + gridDim.x;
    const uint64_t w0 = u * (BK_BITS / 32);
    if (un < nbuckets) {
      const Bk kn = bucket(un);
#pragma unroll
      for (uint32_t i = 0; i < FW; ++i) {
        const uint64_t q = un * (BK_BITS / 32) + threadIdx.x + i * TA_T;
        pfw[i] = q < nwords ? bits[q] : 0u;
      }
      uint32_t na, nb;
      wrange(kn, na, nb);
      hload(kn, na, nb, pbeg, pend, ptb);
      k = kn;
      wa = na;
      wb = nb;
    }
    lds_barrier();
    // T and the filter, one byte of the Redis string (8 bits, MSB first) per lane step
    uint4* T4 = reinterpret_cast<uint4*>(T + u * BK_BITS);
    uint8_t* fb = reinterpret_cast<uint8_t*>(f0);
    for (uint32_t q = threadIdx.x; q < BK_BITS / 8; q += TA_T) {
      const uint4 v = t4[q];
      const uint32_t hw[4] = {v.x, v.y, v.z, v.w};
      const uint32_t was = fb[q];  // byte q of the bucket: bits 8q .. 8q+7, bit 8q at 0x80
      // two entries per dword: entry 2h (low half) is bit 7 - 2h of the byte, 2h + 1 bit 6 - 2h;
      // a bit set before the batch turns its entry into NONE (all ones: an OR)
      uint32_t probed = 0, o[4];
#pragma unroll
      for (int h = 0; h < 4; ++h) {
        const uint32_t wb = was >> (6 - 2 * h);  // bit 1: entry 2h, bit 0: entry 2h + 1
        o[h] = hw[h] | ((wb & 2u) ? 0x0000FFFFu : 0u) | ((wb & 1u) ? 0xFFFF0000u : 0u);
        const uint32_t nx = ~hw[h];  // a half is nonzero iff its entry is not NONE
        probed |= ((nx & 0xFFFFu) ? 2u : 0u) << (6 - 2 * h);
        probed |= ((nx >> 16) ? 1u : 0u) << (6 - 2 * h);
      }
      u32x4 ov = {o[0], o[1], o[2], o[3]};
      if (!(dbg & 2)) __builtin_nontemporal_store(ov, reinterpret_cast<u32x4*>(T4 + q));  // read back by rp_treply's gathers only
      fb[q] = (uint8_t)(was | probed);
    }
    lds_barrier();
    for (uint32_t q = threadIdx.x; q < BK_BITS / 32; q += TA_T)
      if (w0 + q < nwords) bits[w0 + q] = f0[q];
    lds_barrier();  // f0 read out before the next bucket loads it
  }
}

// ---------------------------------------------------------------- rp_treply
// Workgroup = group tag = blockIdx.x = w Gw + g: super-tiles
// [w S + g gs, min(w S + (g + 1) gs, (w + 1) S, nst)) of the chunk.
RSK_DEV uint32_t hs_slot(uint64_t b) { return (uint32_t)((b * 0x9E3779B97F4A7C15ull) >> (64 - 10)); }

template <bool FIXED16, int U>
__global__ __launch_bounds__(RR_T) void rp_treply_kernel(const uint8_t* __restrict__ data,
                                                         const uint64_t* __restrict__ offsets, uint32_t fixed_len,
                                                         uint64_t m, FastMod63 fm, int k,
                                                         const uint16_t* __restrict__ T, uint8_t* __restrict__ out,
                                                         uint64_t kst, uint32_t S, uint32_t gs, uint32_t Gw,
                                                         uint64_t nst, uint32_t* __restrict__ fallback) {
  __shared__ uint32_t p_key[PEND_CAP], p_mask[PEND_CAP];
  __shared__ uint64_t hkey[HS];
  __shared__ uint32_t hmin[HS];
  __shared__ uint32_t s_np, s_nh;
  const uint32_t tag = blockIdx.x, w = tag / Gw, g = tag - w * Gw;
  const uint64_t sw = (uint64_t)w * S, st_a = sw + (uint64_t)g * gs;
  const uint64_t st_b = std::min<uint64_t>(st_a + gs, std::min<uint64_t>(sw + S, nst));
  if (st_a >= st_b || st_a * kst >= m) return;  // an empty group (uniform)
  const uint64_t ka = st_a * kst, kb = std::min<uint64_t>(st_b * kst, m);
  if (threadIdx.x == 0) {
    s_np = 0;
    s_nh = 0;
  }
  __syncthreads();
  // U keys per lane (gather chains in flight); a wave stops when each of its
  // keys is decided.  (Chains that take their next key as soon as theirs is
  // decided -- a gather per chain every round -- measured 48-54 ms against
  // 33: every round then repeats the hashing for the lanes that refill.)
  for (uint64_t base = ka + threadIdx.x; base < kb; base += (uint64_t)RR_T * U) {
    ProbeSeq ps[U];
    bool live[U], open[U], yes[U];
    uint32_t pend[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t i = base + (uint64_t)u * RR_T;
      live[u] = i < kb;
      yes[u] = false;
      pend[u] = 0;
      if (live[u]) {
        uint64_t h1, h2;
        bloom_key_hashes<FIXED16>(data, offsets, fixed_len, i, h1, h2);
        ps[u] = ProbeSeq(h1, h2, fm);
      }
      open[u] = live[u];
    }
    for (int t = 0; t < k - 1; ++t) {
      uint32_t v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = open[u] ? (uint32_t)T[ps[u].idx] : T_NONE;
      bool any = false;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (open[u] && (v[u] >> 1) == tag) {
          if (v[u] & 1u) {
            yes[u] = true;
            open[u] = false;
          } else {
            pend[u] |= 1u << t;  // the group probed this bit more than once
          }
        }
        if (t + 2 < k) ps[u].next(t, fm);
        any |= open[u];
      }
      if (!__any(any)) break;
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (live[u]) {
        const uint64_t i = base + (uint64_t)u * RR_T;
        out[i] = (uint8_t)yes[u];
        if (!yes[u] && pend[u]) {
          const uint32_t q = atomicAdd(&s_np, 1u);
          if (q < PEND_CAP) {
            p_key[q] = (uint32_t)(i - ka);
            p_mask[q] = pend[u];
          }
        }
      }
  }
  __syncthreads();
  const uint32_t np = s_np;
  if (np == 0) return;
  if (np > PEND_CAP) {
    if (threadIdx.x == 0) atomicOr(fallback, 1u);
    return;
  }
  // Pending keys: is (i, t) the group's first probe of b_t?  The minimum
  // (key - ka) << 4 | t over every probe of the group on each pending bit.
  for (uint32_t q = threadIdx.x; q < HS; q += RR_T) {
    hkey[q] = HS_EMPTY;
    hmin[q] = ~0u;
  }
  __syncthreads();
  auto probes_of = [&](uint64_t i) {
    uint64_t h1, h2;
    bloom_key_hashes<FIXED16>(data, offsets, fixed_len, i, h1, h2);
    return ProbeSeq(h1, h2, fm);
  };
  for (uint32_t e = threadIdx.x; e < np; e += RR_T) {
    ProbeSeq ps = probes_of(ka + p_key[e]);
    const uint32_t mask = p_mask[e];
    for (int t = 0; t < k - 1; ++t) {
      if ((mask >> t) & 1u) {
        uint32_t sl = hs_slot(ps.idx);
        for (uint32_t n = 0; n < HS; ++n) {
          const uint64_t old = atomicCAS(reinterpret_cast<unsigned long long*>(&hkey[sl]), HS_EMPTY, ps.idx);
          if (old == HS_EMPTY) {
            atomicAdd(&s_nh, 1u);
            break;
          }
          if (old == ps.idx) break;
          sl = (sl + 1) & (HS - 1);
        }
      }
      if (t + 2 < k) ps.next(t, fm);
    }
  }
  __syncthreads();
  if (s_nh > HS_MAX) {
    if (threadIdx.x == 0) atomicOr(fallback, 1u);
    return;
  }
  auto lookup = [&](uint64_t b) {
    uint32_t sl = hs_slot(b);
    while (true) {
      const uint64_t x = hkey[sl];
      if (x == b) return sl;
      if (x == HS_EMPTY) return HS;
      sl = (sl + 1) & (HS - 1);
    }
  };
  for (uint64_t j = ka + threadIdx.x; j < kb; j += RR_T) {
    ProbeSeq ps = probes_of(j);
    for (int t = 0; t < k; ++t) {
      const uint32_t sl = lookup(ps.idx);
      if (sl < HS) atomicMin(&hmin[sl], ((uint32_t)(j - ka) << 4) | (uint32_t)t);
      if (t + 1 < k) ps.next(t, fm);
    }
  }
  __syncthreads();
  for (uint32_t e = threadIdx.x; e < np; e += RR_T) {
    ProbeSeq ps = probes_of(ka + p_key[e]);
    const uint32_t mask = p_mask[e];
    bool y = false;
    for (int t = 0; t < k - 1; ++t) {
      if ((mask >> t) & 1u) y |= hmin[lookup(ps.idx)] == ((p_key[e] << 4) | (uint32_t)t);
      if (t + 2 < k) ps.next(t, fm);
    }
    if (y) out[ka + p_key[e]] = 1;
  }
  if (threadIdx.x == 0) atomicAdd(fallback + 1, 1u);  // a group resolved in LDS (counted for tests)
}

// The filter as it was before the chunk: bits with T != NONE were clear.
__global__ __launch_bounds__(256) void rp_restore_kernel(uint32_t* __restrict__ bits, uint64_t nwords,
                                                         const uint16_t* __restrict__ T) {
  for (uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; q < nwords; q += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t wv = bits[q];
    if (!wv) continue;
    const uint4* t4 = reinterpret_cast<const uint4*>(T + 32 * q);
    uint32_t clear = 0;
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      const uint4 v = t4[h];
      const uint32_t hw[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (((hw[j >> 1] >> (16 * (j & 1))) & 0xFFFFu) != T_NONE) clear |= bloom_bit_mask(8 * h + j);
    }
    bits[q] = wv & ~clear;
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
  const bool kpl4 = f16 && kmax == 8;  // 4 keys per lane, as the insert's sa1
  constexpr uint32_t T1 = 512;
  const uint64_t kst = kpl4 ? 2048 : (uint64_t)T1 * (16 / kmax);
  uint32_t sb = 0;
  for (uint64_t v = nslices - 1; v; v >>= 1) ++sb;
  const uint32_t f2 = sb > 8 ? sb - 8 : 0;
  const uint32_t shift1 = SL_LOG + f2;
  const uint32_t nb1 = (uint32_t)(((nslices - 1) >> f2) + 1);
  const uint32_t nb2 = 1u << f2;
  const uint32_t nbk = nb2 << SAH_SUB;  // rp2 buckets per coarse bin
  const uint64_t nbuckets = ((uint64_t)b->size + BK_BITS - 1) / BK_BITS;
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
  // sa1 workgroups per CU from their budgets (not the occupancy query: DESIGN.md 2):
  // 4 keys per lane 73 KiB of LDS -> 2; otherwise 80 VGPRs, 43 KiB -> 3
  const uint32_t W = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>({max_nst, (kpl4 ? 2ull : 3ull) * cus, SA2_WMAX}));
  const double share = std::min(1.0, (double)(1ull << shift1) / (double)(uint64_t)b->size);  // of a coarse bin
  const uint64_t q64 = (uint64_t)(1.25 * share * (double)max_np / W) + kst * k + 3 * (max_nst / W + 1) + 64;
  const uint32_t quota = (uint32_t)((q64 + 3) & ~uint64_t(3));
  const uint32_t limit = c->tune.sa_tiny ? 32 : quota;  // tests force the overflow fallback
  if (q64 >= (1ull << 31) || (uint64_t)nb1 * quota >= (1ull << 32)) return false;
  const uint64_t region_probes = (uint64_t)W * nb1 * quota;
  // rp2: uint4 per lane per tile; 6 (24576-record tiles, one workgroup per CU): bucket segments
  // twice as long as at 3, apply 27.5 -> 20.9 ms at C3 with rp2 unchanged (11.1 -> 10.8); 8
  // (32768): rp2 10.9 -> 10.5, apply 20.6 -> 20.3
  const int V2 = c->tune.reply_v == 3 ? 3 : c->tune.reply_v == 6 ? 6 : 8;
  const uint32_t slots2 = SA2_T * 4 * V2;          // records per rp2 tile
  const uint64_t tt_max = (max_np + 3ull * nb1 * max_nst) / slots2 + (uint64_t)W * nb1 + 64;  // bound on rp2 tiles
  const uint64_t l2_slots = max_np + 3ull * nb1 * max_nst + 8 * tt_max + 8ull * ncp;  // rp2 output (u32), aligned tiles
  if (l2_slots / 4 >= (1ull << 32)) return false;  // rp_tapply's 32-bit uint4 indices
  const uint64_t hp_bytes = al(16 * tt_max * (nb2 + 1));
  // T (2 B per bit of whole buckets) reuses rp1's region, dead once rp2 has read it
  const uint64_t reg_bytes = std::max(al(4 * region_probes), al(2 * nbuckets * BK_BITS));
  const uint64_t meta = al(8 * (ncp + 1)) * 2 + al(4 * (ncp + 1)) * 3 + al(4ull * W * nb1) + 256;
  const uint64_t bytes = reg_bytes + al(4 * l2_slots) + hp_bytes + al(4 * tt_max) + meta;
  // Reserved before any chunk is applied; when it does not fit next to
  // everything else the sort path answers the batch instead.
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
    uint8_t* reg = take(reg_bytes);
    uint32_t* region = reinterpret_cast<uint32_t*>(reg);
    uint16_t* T = reinterpret_cast<uint16_t*>(reg);
    uint32_t* l2 = reinterpret_cast<uint32_t*>(take(al(4 * l2_slots)));
    uint4* hp = reinterpret_cast<uint4*>(take(hp_bytes));
    uint32_t* tb2 = reinterpret_cast<uint32_t*>(take(al(4 * tt_max)));
    uint64_t* tot = reinterpret_cast<uint64_t*>(take(al(8 * (ncp + 1))));
    uint64_t* reg_off = reinterpret_cast<uint64_t*>(take(al(8 * (ncp + 1))));
    uint32_t* bud = reinterpret_cast<uint32_t*>(take(al(4 * (ncp + 1))));
    uint32_t* tile_off = reinterpret_cast<uint32_t*>(take(al(4 * (ncp + 1))));
    uint32_t* tiles = reinterpret_cast<uint32_t*>(take(al(4 * (ncp + 1))));
    uint32_t* used = reinterpret_cast<uint32_t*>(take(al(4ull * W * nb1)));
    uint32_t* flags = reinterpret_cast<uint32_t*>(take(256));  // [0] sub-region overflow, [1] reply fallback, [2] groups resolved
    const uint64_t m = std::min<uint64_t>(chunk, keys.n - first);
    const uint64_t nst = (m + kst - 1) / kst;
    // contiguous super-tile ranges of S per sa1 workgroup, groups of gs super-tiles
    const uint32_t Wc = (uint32_t)std::min<uint64_t>(W, nst);
    const uint32_t S = (uint32_t)((nst + Wc - 1) / Wc);
    const uint32_t Wl = (uint32_t)((nst + S - 1) / S);
    const uint32_t Gw = std::min<uint32_t>(63, MAX_TAGS / Wl);
    const uint32_t gs = (S + Gw - 1) / Gw;
    DevKeys dk = keys;
    dk.n = m;
    if (keys.offsets) dk.offsets = keys.offsets + first;
    else dk.data = keys.data + first * keys.fixed_len;
    if ((uint64_t)gs * kst >= (1ull << 28)) {  // rp_treply packs (key - group start) << 4 | t in 32 bits
      bloom_add_replies_sorted(c, b, dk, d_out + first);
      continue;
    }
    RSK_HIP(hipMemsetAsync(flags, 0, 12, c->stream));
    {
      ProfScope ps(c, "bloom_rp1");
#define RSK_RP1(F16, KM, KPL, ...)                                                                                  \
  hipLaunchKernelGGL((bloom_sa1_kernel<F16, KM, T1, uint32_t, KPL, true, ##__VA_ARGS__>), dim3(Wl), dim3(T1), 0,    \
                     c->stream,                                                                                       \
                     dk.data, dk.offsets, dk.fixed_len, m, b->fm, b->k, shift1, nb1, nst, region, quota, limit, used, \
                     flags, S, gs, c->tune.sa_full < 0 ? 2 : 0)
      if (kpl4 && b->k == 7 && c->tune.sa_kc >= 0) RSK_RP1(true, 8, 4, 7);  // C3's k as a constant
      else if (kpl4) RSK_RP1(true, 8, 4);
      else if (f16) RSK_RP1(true, 16, 1);
      else if (kmax == 8) RSK_RP1(false, 8, 2);
      else RSK_RP1(false, 16, 1);
#undef RSK_RP1
      RSK_CHECK_LAUNCH("bloom_rp1");
    }
    uint32_t ov = 0;
    RSK_HIP(hipMemcpyAsync(c->h_small + 8448, flags, 4, hipMemcpyDeviceToHost, c->stream));
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
      hipLaunchKernelGGL(sah_size_kernel, dim3((ncp + 255) / 256), dim3(256), 0, c->stream, used, Wl, nb1, P, ncp,
                         tot, bud, slots2);
      RSK_CHECK_LAUNCH("bloom_rp_size2");
      hipLaunchKernelGGL(st_offsets_kernel, dim3(1), dim3(1024), 0, c->stream, tot, bud, ncp, reg_off, tile_off);
      RSK_CHECK_LAUNCH("bloom_rp_offsets2");
    }
    {
      ProfScope ps(c, "bloom_rp2");
      if (V2 == 8)
        hipLaunchKernelGGL((bloom_sa2h_kernel<uint32_t, 8>), dim3(ncp), dim3(SA2_T), 0, c->stream, region, quota, used,
                           Wl, nb1, P, nbk, reg_off, tile_off, tiles, l2, hp, tt_max, tb2, Gw);
      else if (V2 == 6)
        hipLaunchKernelGGL((bloom_sa2h_kernel<uint32_t, 6>), dim3(ncp), dim3(SA2_T), 0, c->stream, region, quota, used,
                           Wl, nb1, P, nbk, reg_off, tile_off, tiles, l2, hp, tt_max, tb2, Gw);
      else
        hipLaunchKernelGGL((bloom_sa2h_kernel<uint32_t, 3>), dim3(ncp), dim3(SA2_T), 0, c->stream, region, quota, used,
                           Wl, nb1, P, nbk, reg_off, tile_off, tiles, l2, hp, tt_max, tb2, Gw);
      RSK_CHECK_LAUNCH("bloom_rp2");
    }
    {
      ProfScope ps(c, "bloom_rp_apply");
      // 136 KiB of LDS: one workgroup per CU, each looping over its buckets
      const uint32_t ga = (uint32_t)std::min<uint64_t>(nbuckets, cus);
#define RSK_TAP(S)                                                                                                \
  hipLaunchKernelGGL(rp_tapply_kernel<S>, dim3(ga), dim3(TA_T), 0, c->stream, l2, hp, tt_max, f2, tb2, tile_off, \
                     tiles, P, nbuckets, b->d_bits, b->nwords, T, c->tune.reply_dbg, c->tune.reply_bal < 0)
#define RSK_TAP2(S, SU)                                                                                              \
  hipLaunchKernelGGL((rp_tapply_kernel<S, SU>), dim3(ga), dim3(TA_T), 0, c->stream, l2, hp, tt_max, f2, tb2,     \
                     tile_off, tiles, P, nbuckets, b->d_bits, b->nwords, T, c->tune.reply_dbg, c->tune.reply_bal < 0)
      if (V2 == 8) RSK_TAP2(2, 3);  // segments of ~32 records: 48 slots per four lanes
      else if (c->tune.reply_s == 1) RSK_TAP(1);
      else if (c->tune.reply_s == 4) RSK_TAP(4);
      else RSK_TAP(2);
#undef RSK_TAP2
#undef RSK_TAP
      RSK_CHECK_LAUNCH("bloom_rp_apply");
    }
    {
      ProfScope ps(c, "bloom_rp_reply");
      const uint32_t ng = Wl * Gw;  // one workgroup per key group
#define RSK_RPR(F16, U)                                                                                            \
  hipLaunchKernelGGL((rp_treply_kernel<F16, U>), dim3(ng), dim3(RR_T), 0, c->stream, dk.data, dk.offsets,         \
                     dk.fixed_len, m, b->fm, b->k, T, d_out + first, kst, S, gs, Gw, nst, flags + 1)
      const int u = c->tune.reply_u;  // gather chains per lane (default 2)
      if (!f16) RSK_RPR(false, 2);
      else if (u == 1) RSK_RPR(true, 1);
      else if (u == 4) RSK_RPR(true, 4);
      else RSK_RPR(true, 2);
#undef RSK_RPR
      RSK_CHECK_LAUNCH("bloom_rp_reply");
    }
    uint32_t fb[2] = {0, 0};
    RSK_HIP(hipMemcpyAsync(c->h_small + 8448, flags + 1, 8, hipMemcpyDeviceToHost, c->stream));
    RSK_HIP(hipStreamSynchronize(c->stream));
    std::memcpy(fb, c->h_small + 8448, 8);
    c->rp_pending_groups += fb[1];
    if (fb[0]) {
      ++c->rp_fallbacks;
      // A group's pending probes overflowed its LDS tables (many repeated
      // keys inside one group): undo the chunk's bits and let the sort path
      // answer it.
      ProfScope ps(c, "bloom_rp_fallback");
      const uint32_t gr = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((b->nwords + 255) / 256, 8ull * cus));
      hipLaunchKernelGGL(rp_restore_kernel, dim3(gr), dim3(256), 0, c->stream, b->d_bits, b->nwords, T);
      RSK_CHECK_LAUNCH("bloom_rp_restore");
      bloom_add_replies_sorted(c, b, dk, d_out + first);
    }
  }
  return true;
}

}  // namespace rsk
