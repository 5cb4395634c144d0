// rsk_bloom_sa.h -- the append partition's first two stages (gfx950), shared
// by the Bloom insert (rsk_bloom_st.hip: bin offsets, then 16-bit bucket
// offsets) and the add()-with-replies pipeline (rsk_bloom_reply.hip: the same
// records with the key's group tag).  Everything lives in an anonymous
// namespace: each translation unit instantiates its own kernels.  See
// rsk_bloom_st.hip for the pipeline.
#pragma once
#include <type_traits>

#include "rsk_internal.h"

namespace rsk {
namespace {
constexpr int SL_LOG = 19;                             // bits per slice
constexpr uint32_t SL_WORDS = 1u << (SL_LOG - 5);      // 16384 u32 = 64 KiB of LDS
constexpr uint32_t SL_MAX = 32768;                     // slices (2^34 bits) handled here
constexpr uint32_t INVALID = 0xFFFFFFFFu;              // no probe (payloads are < 2^26)

RSK_DEV uint32_t rdl(uint32_t v, uint32_t l) { return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l); }
RSK_DEV uint64_t rdl64(uint64_t v, uint32_t l) {
  return ((uint64_t)rdl((uint32_t)(v >> 32), l) << 32) | rdl((uint32_t)v, l);
}

RSK_DEV void key_words(const uint4& v, uint64_t* w0, uint64_t* w1) {
  *w0 = ((uint64_t)v.y << 32) | v.x;
  *w1 = ((uint64_t)v.w << 32) | v.z;
}

// ------------------------------------------------------------------- st1
// Wave 0 turns the bin counts (<= 256, 4 per lane) into bin starts: lstart
// (LDS), the super-tile header row (global, [nb] = total) and the total.
RSK_DEV uint32_t wave_scan_incl(uint32_t x, uint32_t lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, 64);
    if (lane >= (uint32_t)o) x += y;
  }
  return x;
}

template <int NBMAX>
RSK_DEV void wave0_bin_starts(uint32_t* hist, uint32_t* lstart, uint32_t nb, uint16_t* hdr_row, uint32_t* s_total) {
  constexpr int PER = NBMAX / 64;
  const uint32_t lane = threadIdx.x & 63;
  uint32_t v[PER], sum = 0;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const uint32_t b = lane * PER + i;
    v[i] = b < nb ? hist[b] : 0;
    if (b < nb) hist[b] = 0;  // reset for the next tile (visible after the next barrier)
    sum += v[i];
  }
  const uint32_t incl = wave_scan_incl(sum, lane);
  uint32_t run = incl - sum;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const uint32_t b = lane * PER + i;
    if (b < nb) {
      lstart[b] = run;
      hdr_row[b] = (uint16_t)run;
    }
    run += v[i];
  }
  const uint32_t total = rdl(incl, 63);
  if (lane == 0) {
    hdr_row[nb] = (uint16_t)total;
    *s_total = total;
  }
}

// Probe records of the append partition: the probe's bit offset inside its
// coarse bin (< 2^26; the replies pipeline keeps its key group in bits
// 26..31, group <= 62), so 0xFFFFFFFF (INVALID) is free for padding.
template <class R>
constexpr R rec_pad() { return (R)~(R)0; }

// ------------------------------------------------------ header transpose
// in [rows][cols] -> out [cols][rows] (u16), 64 x 64 tiles through LDS.
__global__ __launch_bounds__(256) __attribute__((unused)) void st_transpose_kernel(const uint16_t* __restrict__ in, uint64_t rows,
                                                           uint32_t cols, uint16_t* __restrict__ out) {
  __shared__ uint16_t t[64][66];
  const uint64_t r0 = (uint64_t)blockIdx.x * 64;
  const uint32_t c0 = blockIdx.y * 64;
  for (uint32_t i = threadIdx.x; i < 64 * 64; i += 256) {
    const uint32_t rr = i >> 6, cc = i & 63;
    const uint64_t r = r0 + rr;
    const uint32_t c = c0 + cc;
    t[rr][cc] = (r < rows && c < cols) ? in[r * cols + c] : 0;
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < 64 * 64; i += 256) {
    const uint32_t cc = i >> 6, rr = i & 63;
    const uint64_t r = r0 + rr;
    const uint32_t c = c0 + cc;
    if (r < rows && c < cols) out[(uint64_t)c * rows + r] = t[rr][cc];
  }
}

// One workgroup: exclusive prefix sums reg_off (u64) / tile_off (u32) over
// ncp entries, with the totals at [ncp].
__global__ __launch_bounds__(1024) void st_offsets_kernel(const uint64_t* __restrict__ tot,
                                                          const uint32_t* __restrict__ bud, uint32_t ncp,
                                                          uint64_t* __restrict__ reg_off,
                                                          uint32_t* __restrict__ tile_off) {
  __shared__ uint64_t s_tot[1024];
  __shared__ uint32_t s_bud[1024];
  const uint32_t per = (ncp + 1023) / 1024, b0 = threadIdx.x * per;
  uint64_t a = 0;
  uint32_t c = 0;
  for (uint32_t i = b0; i < b0 + per && i < ncp; ++i) {
    a += tot[i];
    c += bud[i];
  }
  s_tot[threadIdx.x] = a;
  s_bud[threadIdx.x] = c;
  __syncthreads();
  if (threadIdx.x == 0) {  // 1024 partials, serial (tiny)
    uint64_t ra = 0;
    uint32_t rc = 0;
    for (int i = 0; i < 1024; ++i) {
      const uint64_t x = s_tot[i];
      const uint32_t y = s_bud[i];
      s_tot[i] = ra;
      s_bud[i] = rc;
      ra += x;
      rc += y;
    }
    reg_off[ncp] = ra;
    tile_off[ncp] = rc;
  }
  __syncthreads();
  a = s_tot[threadIdx.x];
  c = s_bud[threadIdx.x];
  for (uint32_t i = b0; i < b0 + per && i < ncp; ++i) {
    reg_off[i] = a;
    tile_off[i] = c;
    a += tot[i];
    c += bud[i];
  }
}

// ============================================ append variant (two-level filters)
// sa1: the st1 super-tile (one hash pass, ranks by coarse bin, bin-sorted LDS
// image), but each coarse bin's run is APPENDED to this workgroup's private
// sub-region for that bin: sub-region (w, c) = probes [(w nb1 + c) quota,
// + quota), so a run's destination is known as soon as the tile's bin counts
// are (no global atomics, no headers); the workgroup records how many probes
// it appended per bin (used[w][c]).
// sa2: one workgroup per (c, p) streams the sub-regions (w, c) of the
// workgroups w of part p with coalesced 16-byte loads (a tile never spans two
// sub-regions), ranks by fine bin and writes bin-sorted tiles exactly like
// st2, whose output the apply kernel reads unchanged.  A sub-region that
// overflows (only adversarial inputs: 1.25x the expected share per
// workgroup) sets `overflow`; the chunk is redone.
#ifndef RSK_SA2_V
#define RSK_SA2_V 3
#endif
constexpr int SA2_V = RSK_SA2_V;    // sa2: uint4 loads per lane per tile (u32: 96 probes per fine bin: apply's 2 x 64 fast path)
constexpr uint32_t SA2_T = 1024;    // sa2 workgroup
constexpr uint32_t SA2_WMAX = 1024;  // sa1 workgroups per sa2 part, at most (the host keeps W <= this)
constexpr uint32_t SA2_SLOTS = SA2_T * SA2_V * 4;  // records per sa2h tile

// 512-lane workgroups: at most 80 VGPRs, so 3 workgroups (6 waves per SIMD)
// share a CU; with 4 keys per lane (73 KiB of LDS) 2.
// KPL: keys per lane (default 16 / KMAX); more keys per super-tile make every
// bin's run longer.  KC: the filter's k as a constant (0: the runtime k).
//
// TAGGED (the add()-with-replies pipeline, rsk_bloom_reply.hip): workgroup w
// takes the CONTIGUOUS super-tiles [w S, (w + 1) S) instead of every
// gridDim.x-th one, and each record carries in its top 6 bits the key group
// g = (super-tile - w S) / gs of its key (offsets are < 2^26): along any
// sub-region (w, c) g never decreases, so key order is known per group.
// HX (timing only, diag route sa_hash): 1 = the key words as h1 / h2 (no
// hashes), 2 = also no mods (idx_0 = h1 mod 2^32) -- wrong filters.
template <bool FIXED16, int KMAX, int T1, class R, int KPL = 16 / KMAX, bool TAGGED = false, int KC = 0, int HX = 0>
__global__ __launch_bounds__(T1, KPL * KMAX > 16 ? 4 : (T1 == 512 ? 6 : 4)) void bloom_sa1_kernel(
    const uint8_t* __restrict__ data, const uint64_t* __restrict__ offsets, uint32_t fixed_len, uint64_t n,
    FastMod63 fm, int k, uint32_t shift1, uint32_t nb1, uint64_t nst, R* __restrict__ region, uint32_t quota,
    uint32_t limit, uint32_t* __restrict__ used, uint32_t* __restrict__ overflow, uint32_t S = 0, uint32_t gs = 1,
    int dbg = 0) {
  constexpr uint32_t KST = T1 * KPL;
  constexpr int NP = KPL * KMAX;
  const int kk = KC ? KC : k;  // KC: k known at compile time (the probe loop without the t < k tests)
  constexpr int PER = 4;  // bins per wave-0 lane (<= 256 bins)
  static_assert(sizeof(R) == 4, "4-byte probe records");
  constexpr uint32_t RG = 16 / sizeof(R);  // records per 16-byte group
  // runs are padded to whole 16-byte groups (rec_pad), so the write-out
  // moves 16-byte groups of one bin to 16-byte aligned destinations
  constexpr uint32_t IMG = T1 * NP + RG * 256;
  __shared__ __attribute__((aligned(16))) R img[IMG];
  __shared__ uint8_t ibin[IMG / RG];
  __shared__ uint32_t hist[256], lstart[256], pos[256], dst[256], s_total;
  const uint64_t low = (1ull << shift1) - 1;
  if (threadIdx.x < 256) {
    hist[threadIdx.x] = 0;
    pos[threadIdx.x] = 0;
  }
  R* const mine = region + (uint64_t)blockIdx.x * nb1 * quota;  // sub-regions (blockIdx.x, 0..nb1)
  const uint4* keys16 = reinterpret_cast<const uint4*>(data);
  // super-tiles of this workgroup: [s_beg, s_end) in steps of s_step
  const uint64_t s_beg = TAGGED ? (uint64_t)blockIdx.x * S : blockIdx.x;
  const uint64_t s_end = TAGGED ? (s_beg + S < nst ? s_beg + S : nst) : nst;
  const uint64_t s_step = TAGGED ? 1 : gridDim.x;
  uint4 nxt[KPL];
  auto fetch = [&](uint64_t st) {
#pragma unroll
    for (int u = 0; u < KPL; ++u) {
      const uint64_t i = st * KST + threadIdx.x + (uint64_t)u * T1;
      nxt[u] = (FIXED16 && st < s_end && i < n) ? ld_nt16(keys16 + i) : make_uint4(0, 0, 0, 0);
    }
  };
  // The image of tile t is written out during tile t + 1, after its hashes
  // and ranks (`pend4` 16-byte groups still in img; dst / ibin stay valid
  // until barrier (A)).  gfx9 counts loads and stores in one vmcnt, so a wait
  // for the keys is a wait for every store issued before it: the order
  // [wait keys t] [hash t] [loads t+1] [stores t-1] [scan, scatter t] leaves
  // the scan and scatter between the stores and the next wait, and the loads
  // of t + 1 are never in the wait that precedes their own issue.
  uint64_t wst = 0;  // dbg: the super-tile being written out
  auto write_out = [&](uint32_t total4) {
    const uint4* img4 = reinterpret_cast<const uint4*>(img);
    if (dbg & 1) {  // TIMING ONLY (the host stops after this pass): each tile's image stored contiguously
      u32x4* o4 = reinterpret_cast<u32x4*>(region + wst * IMG);
      for (uint32_t g = threadIdx.x; g < total4; g += T1) {
        const uint4 v = img4[g];
        o4[g] = u32x4{v.x, v.y, v.z, v.w};
      }
      return;
    }
    for (uint32_t g = threadIdx.x; g < total4; g += T1) {
      const uint32_t d = dst[ibin[g]];
      if (d != INVALID) {
        const uint4 v = img4[g];
        u32x4 x = {v.x, v.y, v.z, v.w};
        // 8-byte records (the replies pipeline's rp1): streaming stores measured 19.4 -> 18.4 ms;
        // 4-byte records (the insert's sa1): no gain
        *reinterpret_cast<u32x4*>(mine + (RG * g + d)) = x;  // (streaming stores: no gain measured)
      }
    }
  };
  uint32_t pend4 = 0;
  if (FIXED16) fetch(s_beg);
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63;
  for (uint64_t st = s_beg; st < s_end; st += s_step) {
    const uint64_t k0 = st * KST;
    const uint32_t gtag = TAGGED ? (uint32_t)((st - s_beg) / gs) << 26 : 0u;
    const uint32_t nk = (uint32_t)(n - k0 < KST ? n - k0 : KST);
    uint4 cur[KPL];
#pragma unroll
    for (int u = 0; u < KPL; ++u) cur[u] = nxt[u];
    if (FIXED16) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // keys t here, before the loads of t + 1 issue
    R pay[NP];
    uint32_t tag[NP];
    // A full super-tile (every one but a chunk's last) with k a constant takes
    // its hashes and ranks without a per-key or per-probe test: no exec-mask
    // branches around the 4 x 7 probes (FULL = std::true_type).
    const bool full = nk == KST && !(dbg & 2);  // dbg bit 1: the general path only (A/B)
    auto hash_rank = [&](auto full_c) {
      constexpr bool FULL = decltype(full_c)::value;
#pragma unroll
      for (int u = 0; u < KPL; ++u) {
        const uint32_t q = threadIdx.x + u * T1;
        const bool ok = FULL || q < nk;
        uint64_t h1 = 0, h2 = 0;
        if (ok) {
          if (FIXED16) {
            uint64_t w0, w1;
            key_words(cur[u], &w0, &w1);
            h1 = HX ? w0 : xxh64_16(w0, w1);
            h2 = HX ? w1 : farm_16(w0, w1);
          } else {
            bloom_key_hashes<false>(data, offsets, fixed_len, k0 + q, h1, h2);
          }
        }
        ProbeSeq ps;
        if (HX == 2) {
          ps.v1 = h1 & JAVA_LONG_MAX;
          ps.v2 = h2 & JAVA_LONG_MAX;
          ps.init((uint32_t)h1, (uint32_t)h2, fm);
        } else {
          ps = ProbeSeq(h1, h2, fm);
        }
#pragma unroll
        for (int t = 0; t < KMAX; ++t) {
          const int s = u * KMAX + t;
          tag[s] = INVALID;
          pay[s] = 0;
          if (ok && t < kk) {
            const uint64_t idx = ps.idx;
            const uint32_t bin = (uint32_t)(idx >> shift1);
            pay[s] = (R)((uint32_t)(idx & low) | gtag);
            tag[s] = (bin << 16) | atomicAdd(&hist[bin], 1u);
            if (t + 1 < kk) ps.next(t, fm);
          }
        }
      }
    };
    if (KC && full) hash_rank(std::true_type{});
    else hash_rank(std::false_type{});
    if (FIXED16) fetch(st + s_step);
    write_out(pend4);  // tile t - 1
    wst = st;
    lds_barrier();  // (A) every rank taken, the previous image written out
    // wave 0: bin starts and run destinations (runs of L probes take
    // L4 = round_up(L, RG) slots, the tail rec_pad): image position j of bin b
    // goes to mine[j + dst[b]] (mod 2^32), dst[b] = b quota + pos[b] - lstart[b]
    if (threadIdx.x < 64) {
      uint32_t v[PER], sum = 0;
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        const uint32_t b = lane * PER + i;
        v[i] = b < nb1 ? hist[b] : 0;
        if (b < nb1) hist[b] = 0;
        sum += (v[i] + RG - 1) & ~(RG - 1);
      }
      const uint32_t incl = wave_scan_incl(sum, lane);
      uint32_t at = incl - sum;
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        const uint32_t b = lane * PER + i;
        const uint32_t l4 = (v[i] + RG - 1) & ~(RG - 1);
        if (b < nb1) {
          lstart[b] = at;
          for (uint32_t j = at + v[i]; j < at + l4; ++j) img[j] = rec_pad<R>();
          const uint32_t p = pos[b];
          if (p + l4 <= limit) {  // limit = quota (< quota only in tests)
            dst[b] = b * quota + p - at;
            pos[b] = p + l4;
          } else {  // sub-region full: drop the run (the host redoes the chunk)
            if (v[i]) atomicOr(overflow, 1u);
            dst[b] = INVALID;
          }
        }
        at += l4;
      }
      if (lane == 63) s_total = incl;
    }
    lds_barrier();  // (B) lstart / dst / total ready
    auto scatter = [&](auto full_c) {
      constexpr bool FULL = decltype(full_c)::value;  // every tag valid
#pragma unroll
      for (int s = 0; s < NP; ++s)
        if (FULL || tag[s] != INVALID) {
          const uint32_t b = tag[s] >> 16, r = tag[s] & 0xFFFFu, j = lstart[b] + r;
          img[j] = pay[s];
          if ((r & (RG - 1)) == 0) ibin[j / RG] = (uint8_t)b;  // the group's first slot always holds a probe
        }
    };
    if (KC && KC == KMAX && full) scatter(std::true_type{});
    else scatter(std::false_type{});
    pend4 = s_total / RG;
    lds_barrier();  // (C) image complete
  }
  write_out(pend4);  // the last tile
  __syncthreads();
  if (threadIdx.x < nb1) used[(uint64_t)blockIdx.x * nb1 + threadIdx.x] = pos[threadIdx.x];
}

// ==================================== sa2 with 16-bit records (the insert)
// The insert's second pass re-sorts each coarse bin by BUCKET = the slice and
// the top 3 bits of the 19-bit offset inside it (2^(f2+3) <= 1024 buckets), so
// every output record keeps only the low 16 bits: half the bytes sa2 writes
// and apply reads.  A tile's buckets are contiguous and unpadded (the tile
// itself starts 16-byte aligned).  Its bucket starts go straight to the
// layout apply reads: row f (slice f of the bin) holds, per tile, one uint4 =
// the 8 u16 starts of buckets 8f .. 8f+7; row 2^f2 holds the tile's record
// count in .x, so slice f's segment ends where row f + 1 starts.  The 16-byte
// pieces of consecutive tiles of one workgroup fill a row's cache lines in L2.
constexpr uint32_t SAH_BK_MAX = 1024;  // buckets per coarse bin, at most (f2 <= 7)
constexpr uint32_t SAH_SUB = 3;         // offset bits [16, 19) sorted by bucket

// tot[cp] = u16 slots of (c, p)'s sa2h tiles (records + up to 7 of alignment
// per tile), bud[cp] = its tiles.
__global__ __launch_bounds__(256) __attribute__((unused)) void sah_size_kernel(const uint32_t* __restrict__ used, uint32_t W, uint32_t nb1,
                                                       uint32_t P, uint32_t ncp, uint64_t* __restrict__ tot,
                                                       uint32_t* __restrict__ bud, uint32_t slots = SA2_SLOTS) {
  const uint32_t cp = blockIdx.x * blockDim.x + threadIdx.x;
  if (cp >= ncp) return;
  const uint32_t c = cp / P, p = cp - c * P;
  uint64_t recs = 0;
  uint32_t tiles = 0;
  for (uint32_t w = W * p / P; w < W * (p + 1) / P; ++w) {
    const uint32_t u = used[(uint64_t)w * nb1 + c];
    recs += u;
    tiles += (u + slots - 1) / slots;
  }
  tot[cp] = ((recs + 7) & ~7ull) + 8ull * tiles;
  bud[cp] = tiles;
}

// O = uint16_t: the insert (16-bit offsets inside the bucket).  O = uint32_t:
// the add()-with-replies pipeline, whose input records carry the key group g
// in bits 26..31 (bloom_sa1_kernel<..., TAGGED>): the output record is
// (tag << 16) | offset with tag = w Gw + g, w the sub-region's sa1
// workgroup -- groups numbered in key order across the whole chunk.
// V: uint4 loads per lane per tile (tile = 4096 V records; V = 6 takes 96 KiB
// of LDS: one workgroup per CU).
template <class O, int V = SA2_V>
__global__ __launch_bounds__(SA2_T, V > 3 ? 4 : 8) __attribute__((unused)) void bloom_sa2h_kernel(const uint32_t* __restrict__ region, uint32_t quota,
                                                           const uint32_t* __restrict__ used, uint32_t W,
                                                           uint32_t nb1, uint32_t P, uint32_t nbk,
                                                           const uint64_t* __restrict__ reg_off,
                                                           const uint32_t* __restrict__ tile_off,
                                                           uint32_t* __restrict__ tiles_out,
                                                           O* __restrict__ out, uint4* __restrict__ hp,
                                                           uint64_t hp_stride, uint32_t* __restrict__ tb2,
                                                           uint32_t Gw = 0) {
  constexpr bool TAGGED = sizeof(O) == 4;
  constexpr uint32_t RPU = 16 / sizeof(O);  // records per uint4
  constexpr uint32_t OFFM = TAGGED ? (1u << 26) - 1 : 0xFFFFFFFFu;
  constexpr int NV = V * 4;  // records per lane per tile
  constexpr uint32_t SLOTS = SA2_T * V * 4;
  constexpr uint32_t PER = SAH_BK_MAX / 64;  // buckets per wave-0 lane
  __shared__ __attribute__((aligned(16))) O img[SLOTS + 8];
  __shared__ uint32_t hist[SAH_BK_MAX], lstart[SAH_BK_MAX + 1];
  __shared__ uint32_t s_used[SA2_WMAX];
  const uint32_t cp = blockIdx.x, c = cp / P, p = cp - c * P;
  for (uint32_t b = threadIdx.x; b < SAH_BK_MAX; b += SA2_T) hist[b] = 0;
  const uint64_t base = reg_off[cp];
  const uint32_t tbeg = tile_off[cp];
  uint64_t written = 0;
  uint32_t ntile = 0;
  const uint32_t wbeg = W * p / P, wend = W * (p + 1) / P;
  for (uint32_t i = threadIdx.x; i < wend - wbeg; i += SA2_T) s_used[i] = used[(uint64_t)(wbeg + i) * nb1 + c];
  __syncthreads();
  uint32_t w = wbeg, t0 = 0, nu = 0;
  while (w < wend && (nu = s_used[w - wbeg]) == 0) ++w;
  // tile t's image is written out during tile t + 1, after its ranks (one
  // vmcnt for loads and stores: see bloom_sa1_kernel)
  auto write_out = [&](uint32_t total, uint64_t at) {
    u32x4* o4 = reinterpret_cast<u32x4*>(out + base + at);  // base, at: multiples of 8 slots
    const uint4* i4 = reinterpret_cast<const uint4*>(img);
    for (uint32_t j = threadIdx.x; j < (total + RPU - 1) / RPU; j += SA2_T) {
      const uint4 v = i4[j];
      u32x4 x = {v.x, v.y, v.z, v.w};
      __builtin_nontemporal_store(x, o4 + j);
    }
  };
  bool have = w < wend;
  uint32_t pend = 0;
  uint64_t pend_at = 0;
  const uint32_t lane = threadIdx.x & 63;
  while (have) {
    const uint4* in = reinterpret_cast<const uint4*>(region + ((uint64_t)w * nb1 + c) * quota);
    uint4 cur[V];
#pragma unroll
    for (int v = 0; v < V; ++v) {
      const uint32_t q4 = t0 / 4 + v * SA2_T + threadIdx.x;
      cur[v] = 4 * q4 < nu ? ld_nt16(in + q4) : make_uint4(INVALID, INVALID, INVALID, INVALID);
    }
    const uint32_t ct0 = t0, cnu = nu, tagbase = w * Gw;  // a tile never spans two sub-regions
    t0 += SLOTS;
    if (t0 >= nu) {
      t0 = 0;
      do ++w;
      while (w < wend && (nu = s_used[w - wbeg]) == 0);
    }
    have = w < wend;
    uint32_t pay[NV], tag[NV];
#pragma unroll
    for (int v = 0; v < V; ++v) {
      const uint32_t q4 = ct0 / 4 + v * SA2_T + threadIdx.x;
      const uint32_t x[4] = {cur[v].x, cur[v].y, cur[v].z, cur[v].w};
#pragma unroll
      for (int e = 0; e < 4; ++e) pay[4 * v + e] = 4 * q4 + e < cnu ? x[e] : INVALID;
    }
#pragma unroll
    for (int r = 0; r < NV; ++r) {
      tag[r] = INVALID;
      if (pay[r] != INVALID) {
        const uint32_t bk = (pay[r] & OFFM) >> 16;
        tag[r] = (bk << 16) | atomicAdd(&hist[bk], 1u);
      }
    }
    write_out(pend, pend_at);  // tile t - 1
    lds_barrier();             // (A) ranks taken, the previous image written out
    if (threadIdx.x < 64) {    // bucket starts (and counts reset)
      uint32_t v[PER], sum = 0;
#pragma unroll
      for (uint32_t i = 0; i < PER; ++i) {
        const uint32_t b = lane * PER + i;
        v[i] = b < nbk ? hist[b] : 0;
        if (b < nbk) hist[b] = 0;
        sum += v[i];
      }
      const uint32_t incl = wave_scan_incl(sum, lane);
      uint32_t run = incl - sum;
#pragma unroll
      for (uint32_t i = 0; i < PER; ++i) {
        const uint32_t b = lane * PER + i;
        if (b < nbk) lstart[b] = run;
        run += v[i];
      }
      if (lane == 63) lstart[nbk] = incl;
    }
    lds_barrier();  // (B)
    const uint32_t total = lstart[nbk];
    if (threadIdx.x <= nbk / 8) {  // row f: starts of buckets 8f .. 8f+7; row nbk / 8: the count
      const uint32_t* ls = lstart + 8 * threadIdx.x;
      const uint4 v = threadIdx.x < nbk / 8
                          ? make_uint4(ls[0] | ls[1] << 16, ls[2] | ls[3] << 16, ls[4] | ls[5] << 16, ls[6] | ls[7] << 16)
                          : make_uint4(total, 0, 0, 0);
      hp[(uint64_t)threadIdx.x * hp_stride + tbeg + ntile] = v;
    }
    if (threadIdx.x == 0) tb2[tbeg + ntile] = (uint32_t)((base + written) / RPU);  // the tile's first uint4
#pragma unroll
    for (int r = 0; r < NV; ++r)
      if (tag[r] != INVALID) {
        const uint32_t x = pay[r];
        img[lstart[tag[r] >> 16] + (tag[r] & 0xFFFFu)] =
            TAGGED ? (O)(((tagbase + (x >> 26)) << 16) | (x & 0xFFFFu)) : (O)x;
      }
    pend = total;
    pend_at = written;
    written += (total + 7) & ~7u;
    ++ntile;
    lds_barrier();  // (C)
  }
  write_out(pend, pend_at);
  if (threadIdx.x == 0) tiles_out[cp] = ntile;
}

}  // namespace
}  // namespace rsk
