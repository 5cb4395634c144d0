// rsk_hll_group.hip -- grouped PFADD (rsk_hll_add_grouped, BASELINE C5) for
// large batches: pairs partitioned by sketch, each group of sketches updated in
// LDS and written once; PFCOUNT estimated on the way out.
#include <hipcub/hipcub.hpp>

#include "rsk_hllcount.h"
#include "rsk_internal.h"
#include "rsk_part.h"

namespace rsk {

// ===================================================== grouped PFADD (C5)
// RHyperLogLog.add on many sketches (rsk_hll_add_grouped, C5): pair i adds
// key i to sketch groups[i].  Issued directly every pair is a random 4 B
// read plus a memory-side CAS into a 16 GiB pool (the CAS dominates when the
// sketches are fresh).  For large batches the pairs are instead partitioned
// by sketch and each 8-sketch group (128 KiB) is updated in LDS:
//   gcount : cnt1[c][b] = pairs of block b in coarse bin c = g >> 12 (<= 256 bins)
//   gpart1 : block b hashes its pairs into records rec = (g & 0xFFF) << 20 |
//            idx << 6 | rank and counting-sorts them by coarse bin (exact offsets)
//   gcount2: cnt2[c*256 + f][b] = records of unit (c, b) in fine bin f = rec >> 24
//            (16 sketches)
//   part2  : the Bloom part2 kernel re-sorts each unit by fine bin (records kept)
//   gapply : one workgroup per (fine bin, half): 8 sketches' registers in LDS
//            (byte max by LDS CAS), read and written back once
// HBM per pair: 4 (gcount) + 20 + 4 (gpart1) + 4 (gcount2) + 8 (part2) + 8 (gapply,
// two halves), plus 32 KiB per touched sketch -- against a random read + CAS.
constexpr uint32_t GP_BIN_SHIFT = 12;  // sketches per coarse bin = 4096 (rec keeps 12 bits of g)
#ifndef RSK_GP_SK
#define RSK_GP_SK 8
#endif
constexpr uint32_t GP_SK = RSK_GP_SK;  // sketches per gapply workgroup (GP_SK x 16 KiB of LDS)
constexpr uint32_t GP_NP = 16 / GP_SK; // gapply parts per fine bin (each reads the bin's records)
constexpr int GP_U = 4;                // record loads in flight per gapply lane
constexpr uint32_t GP_T = 1024;        // gcount / gapply workgroup
#ifndef RSK_GP_TILE
#define RSK_GP_TILE 8192
#endif
constexpr uint32_t GP_TILE = RSK_GP_TILE;  // records per gpart1 tile
constexpr int GP_E = GP_TILE / PT;
constexpr uint32_t GP_GU = 8;          // gpart1 blocks per part2 unit (G1 is a multiple)

__global__ __launch_bounds__(GP_T) void hll_gcount_kernel(const uint32_t* __restrict__ groups, uint64_t n,
                                                          uint64_t per, uint64_t G, uint32_t nbins,
                                                          uint32_t* __restrict__ cnt) {
  __shared__ uint32_t h[PT];
  for (uint32_t s = threadIdx.x; s < PT; s += GP_T) h[s] = 0;
  __syncthreads();
  uint64_t begin, end;
  key_range(n, per, &begin, &end);
  for (uint64_t i = begin + threadIdx.x; i < end; i += GP_T) {
    const uint32_t g = __builtin_nontemporal_load(&groups[i]);
    if (g < G) atomicAdd(&h[g >> GP_BIN_SHIFT], 1u);
  }
  __syncthreads();
  for (uint32_t s = threadIdx.x; s < nbins; s += GP_T) cnt[(uint64_t)s * gridDim.x + blockIdx.x] = h[s];
}

__global__ __launch_bounds__(PT) void hll_gpart1_kernel(const uint4* __restrict__ keys,
                                                        const uint32_t* __restrict__ groups, uint64_t n, uint64_t per,
                                                        uint64_t G, uint32_t nbins, const uint32_t* __restrict__ start,
                                                        uint32_t* __restrict__ out) {
  __shared__ SortLds<GP_TILE> L;
  uint64_t begin, end;
  key_range(n, per, &begin, &end);
  L.hist[threadIdx.x] = 0;
  if (threadIdx.x < nbins) L.cur[threadIdx.x] = start[(uint64_t)threadIdx.x * gridDim.x + blockIdx.x];
  for (uint64_t k0 = begin; k0 < end; k0 += GP_TILE) {
    uint4 v[GP_E];
    uint32_t g[GP_E];
#pragma unroll
    for (int e = 0; e < GP_E; ++e) {
      const uint64_t i = k0 + threadIdx.x + (uint64_t)e * PT;
      const bool ok = i < end;
      v[e] = ok ? ld_nt16(keys + i) : make_uint4(0, 0, 0, 0);
      g[e] = ok ? __builtin_nontemporal_load(&groups[i]) : 0xFFFFFFFFu;
    }
    __syncthreads();  // the previous tile's hist reset is visible
    uint32_t rec[GP_E], tag[GP_E];
#pragma unroll
    for (int e = 0; e < GP_E; ++e) {
      tag[e] = 0xFFFFFFFFu;
      if (g[e] < G) {
        const uint64_t hsh = murmur64a_16(((uint64_t)v[e].y << 32) | v[e].x, ((uint64_t)v[e].w << 32) | v[e].z);
        rec[e] = ((g[e] & ((1u << GP_BIN_SHIFT) - 1)) << 20) | (hll_index(hsh) << 6) | hll_rank(hsh);
        const uint32_t b = g[e] >> GP_BIN_SHIFT;
        tag[e] = (b << 16) | atomicAdd(&L.hist[b], 1u);
      }
    }
    const uint32_t cnt = tile_bins(L);
    const uint32_t np = L.lstart[PT - 1] + L.hist[PT - 1];  // records placed in this tile
#pragma unroll
    for (int e = 0; e < GP_E; ++e)
      if (tag[e] != 0xFFFFFFFFu) tile_place(L, tag[e], rec[e]);
    tile_write(L, np, cnt, out);
  }
}

// unit u = c * G1 + b is [off1[u], off1[u+1]); cnt2[(c * 256 + f) * G1 + b].
__global__ __launch_bounds__(PT) void hll_gcount2_kernel(const uint32_t* __restrict__ recs,
                                                         const uint32_t* __restrict__ off1, uint32_t G1,
                                                         uint32_t* __restrict__ cnt2) {
  __shared__ uint32_t h[PT];
  const uint32_t u = blockIdx.x;
  h[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t a = off1[u], e = off1[u + 1];
  for (uint32_t i = a + threadIdx.x; i < e; i += PT) atomicAdd(&h[__builtin_nontemporal_load(&recs[i]) >> 24], 1u);
  __syncthreads();
  const uint32_t c = u / G1, b = u - c * G1;
  cnt2[((uint64_t)c * PT + threadIdx.x) * G1 + b] = h[threadIdx.x];
}

// part2 units: GU part1 blocks each, or one block each in a coarse bin whose
// GU-block units would be above a quarter of a part2 workgroup's share of the
// records (skewed groups: Zipf(1.1) puts ~60 % of all pairs into bin 0, whose
// GU-block units were ten shares each).  One workgroup; lane c = bin c.
__global__ __launch_bounds__(PT) void hll_gunits_kernel(const uint32_t* __restrict__ off1, uint32_t G1, uint32_t GU,
                                                        uint32_t nbins1, uint32_t p2_grid,
                                                        uint32_t* __restrict__ ustart, uint32_t* __restrict__ d_nunits) {
  __shared__ uint32_t cnt[PT];
  const uint32_t c = threadIdx.x;
  const uint64_t total = off1[(uint64_t)nbins1 * G1];
  uint32_t gu = GU, n = 0;
  if (c < nbins1) {
    const uint64_t r = off1[(uint64_t)(c + 1) * G1] - off1[(uint64_t)c * G1];
    if (r * GU > (uint64_t)G1 * (total / (4ull * p2_grid) + 1)) gu = 1;
    n = G1 / gu;
  }
  cnt[c] = n;
  __syncthreads();
  if (c == 0) {  // exclusive prefix over <= 256 bins
    uint32_t run = 0;
    for (uint32_t i = 0; i < PT; ++i) {
      const uint32_t v = cnt[i];
      cnt[i] = run;
      run += v;
    }
    ustart[run] = nbins1 * G1;
    *d_nunits = run;
  }
  __syncthreads();
  for (uint32_t q = 0; q < n; ++q) ustart[cnt[c] + q] = c * G1 + q * gu;
}

// A fine bin's records beyond its first GP_CH go to hll_gapply_extra (skewed
// groups, e.g. the Zipf(1.1) C5 variant, put a third of all pairs into one
// bin: one workgroup would otherwise walk them alone).
constexpr uint32_t GP_CH = 1u << 20;

// work item w: fine bin s = w / GP_NP (16 sketches from c*4096 + f*16), part w % GP_NP.
// With pc.pcount: the PFCOUNT of every row written is estimated from LDS on
// the way out (the write-back's uint4 i of each thread belongs to sketch i)
// and left in pc (hll_count_kernel takes it instead of re-reading the row);
// rows of split heavy bins and inexact sums are left for the count kernel.
__global__ __launch_bounds__(GP_T) void hll_gapply_kernel(const uint32_t* __restrict__ recs,
                                                          const uint32_t* __restrict__ off2, uint32_t G1,
                                                          uint32_t nfine, uint64_t G, int pool_zero,
                                                          int write_all, uint8_t* __restrict__ regs, PCount pc,
                                                          const double* __restrict__ lc) {
  __shared__ __attribute__((aligned(16))) uint32_t r32[GP_SK * HLL_REGS / 4];
  __shared__ SumD part[GP_T / 64];
  // the GP_NP parts of a fine bin read the same records: one XCD (one L2) for both
  for (uint32_t w = xcd_slot(blockIdx.x, gridDim.x); w < GP_NP * nfine; w += gridDim.x) {
    const uint32_t s = w / GP_NP, half = w % GP_NP;
    const uint32_t a = off2[(uint64_t)s * G1], e0 = off2[(uint64_t)(s + 1) * G1];
    const uint32_t e = e0 - a > GP_CH ? a + GP_CH : e0;  // the rest: hll_gapply_extra
    const uint64_t g0 = (uint64_t)(s >> 8) * (1u << GP_BIN_SHIFT) + (uint64_t)(s & 255) * 16 + half * GP_SK;
    if ((a == e && !write_all) || g0 >= G) continue;  // uniform across the workgroup
    const uint32_t nsk = (uint32_t)(G - g0 < GP_SK ? G - g0 : GP_SK);
    const uint32_t n4 = nsk * (HLL_REGS / 16);
    uint4* gp = reinterpret_cast<uint4*>(regs + g0 * HLL_REGS);
    uint4* lp = reinterpret_cast<uint4*>(r32);
    if (pool_zero)  // the pool is known to be all zero: nothing to read
      for (uint32_t q = threadIdx.x; q < n4; q += GP_T) lp[q] = make_uint4(0, 0, 0, 0);
    else
      for (uint32_t q = threadIdx.x; q < n4; q += GP_T) lp[q] = gp[q];
    // LDS-only barriers (lds_barrier) throughout: the previous item's
    // write-back stores stay in flight while this item's LDS file is cleared
    // and its records are applied (one workgroup per CU: a full fence here
    // serialised every item's 128 KiB write behind its record phase)
    lds_barrier();
    for (uint32_t i0 = a + threadIdx.x; i0 < e; i0 += GP_T * GP_U) {
      uint32_t rv[GP_U];  // GP_U record loads in flight per lane
#pragma unroll
      for (int u = 0; u < GP_U; ++u) {
        const uint32_t i = i0 + u * GP_T;
        rv[u] = i < e ? __builtin_nontemporal_load(&recs[i]) : 0xFFFFFFFFu;
      }
#pragma unroll
      for (int u = 0; u < GP_U; ++u) {
        const uint32_t r = rv[u];
        const uint32_t sk = (r >> 20) & 15u;  // sketch within the fine bin
        if (r == 0xFFFFFFFFu || sk / GP_SK != half) continue;  // (rank 63 never occurs: no real record is all ones)
        const uint32_t byte = (sk % GP_SK) * HLL_REGS + ((r >> 6) & (HLL_REGS - 1));
        const uint32_t rank = r & 63u, sh = (byte & 3u) * 8;
        uint32_t* word = &r32[byte >> 2];
        uint32_t old = *word;
        while (((old >> sh) & 0xFFu) < rank) {
          const uint32_t prev = atomicCAS(word, old, (old & ~(0xFFu << sh)) | (rank << sh));
          if (prev == old) break;
          old = prev;
        }
      }
    }
    lds_barrier();
    const bool est = pc.pcount && e0 - a <= GP_CH;  // (a split bin's extra chunks change the rows later)
    if (!est) {
      for (uint32_t q = threadIdx.x; q < n4; q += GP_T) gp[q] = lp[q];
      if (pc.pcount && threadIdx.x < nsk) pc.pepoch[g0 + threadIdx.x] = 0;  // no estimate for these rows
    } else {
      static_assert(GP_T / 64 == 2 * GP_SK, "two waves per sketch");
      // wave w writes back (and sums) half w & 1 of sketch w >> 1: 8 uint4 per lane, one reduction per wave
      const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6, i = wv >> 1;
      SumD sd{0.0, 0, 0};
      if (i < nsk) {
        const uint32_t q0 = i * (HLL_REGS / 16) + (wv & 1) * (HLL_REGS / 32);
#pragma unroll
        for (int u = 0; u < HLL_REGS / 32 / 64; ++u) {
          const uint32_t q = q0 + u * 64 + lane;
          const uint4 v = lp[q];
          gp[q] = v;
          acc_word(sd, v.x);
          acc_word(sd, v.y);
          acc_word(sd, v.z);
          acc_word(sd, v.w);
        }
      }
      sd = wave_reduce(sd);
      if (lane == 0) part[wv] = sd;
      lds_barrier();
      if (threadIdx.x < nsk) {  // one lane per sketch: its two wave partials
        const SumD p0 = part[2 * threadIdx.x], p1 = part[2 * threadIdx.x + 1];  // exact sums: any order
        SumD t{p0.t + p1.t, p0.ez + p1.ez, p0.rmax > p1.rmax ? p0.rmax : p1.rmax};
        const uint64_t g = g0 + threadIdx.x;
        if (exact_total(t)) {
          pc.pcount[g] = hll_estimate(t.t, (int)t.ez, lc);
          pc.pepoch[g] = pc.epoch;
        } else {
          pc.pepoch[g] = 0;  // Redis's dense order: left to hll_count_kernel
        }
      }
    }
    lds_barrier();  // every lane has read the LDS file (its stores may still be in flight)
  }
}

// List the extra work items: entry (s << 13) | (part << 12) | j for chunk
// j >= 1 of fine bin s, part `part` (records [a + j GP_CH, min(e, a + (j+1) GP_CH))).
__global__ __launch_bounds__(256) void hll_gextra_list_kernel(const uint32_t* __restrict__ off2, uint32_t G1,
                                                              uint32_t nfine, uint32_t cap,
                                                              uint32_t* __restrict__ list, uint32_t* __restrict__ nlist) {
  for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < nfine; s += gridDim.x * blockDim.x) {
    const uint32_t n = off2[(uint64_t)(s + 1) * G1] - off2[(uint64_t)s * G1];
    if (n <= GP_CH) continue;
    const uint32_t extra = (n - 1) / GP_CH;
    const uint32_t at = atomicAdd(nlist, extra * GP_NP);
    for (uint32_t j = 1; j <= extra; ++j)
      for (uint32_t h = 0; h < GP_NP; ++h) {
        const uint32_t q = at + (j - 1) * GP_NP + h;
        if (q < cap) list[q] = (s << 13) | (h << 12) | j;
      }
  }
}

// Extra chunks of heavy fine bins, after hll_gapply wrote every row: the
// chunk's records are maxed into zeroed LDS registers, then each non-zero
// word is folded into the pool row by a bytewise-max CAS (only the few
// workgroups of one heavy bin contend for its words).
__global__ __launch_bounds__(GP_T) void hll_gapply_extra_kernel(const uint32_t* __restrict__ recs,
                                                                const uint32_t* __restrict__ off2, uint32_t G1,
                                                                uint64_t G, const uint32_t* __restrict__ list,
                                                                const uint32_t* __restrict__ nlist, uint32_t cap,
                                                                uint8_t* __restrict__ regs) {
  __shared__ __attribute__((aligned(16))) uint32_t r32[GP_SK * HLL_REGS / 4];
  const uint32_t nl = min(*nlist, cap);
  for (uint32_t w = blockIdx.x; w < nl; w += gridDim.x) {
    const uint32_t ent = list[w], s = ent >> 13, half = (ent >> 12) & 1u, j = ent & 4095u;
    const uint32_t a0 = off2[(uint64_t)s * G1], e0 = off2[(uint64_t)(s + 1) * G1];
    const uint32_t a = a0 + j * GP_CH, e = e0 - a > GP_CH ? a + GP_CH : e0;
    const uint64_t g0 = (uint64_t)(s >> 8) * (1u << GP_BIN_SHIFT) + (uint64_t)(s & 255) * 16 + half * GP_SK;
    if (g0 >= G) continue;
    const uint32_t nsk = (uint32_t)(G - g0 < GP_SK ? G - g0 : GP_SK);
    for (uint32_t q = threadIdx.x; q < GP_SK * HLL_REGS / 4; q += GP_T) r32[q] = 0;
    __syncthreads();
    for (uint32_t i0 = a + threadIdx.x; i0 < e; i0 += GP_T * GP_U) {
      uint32_t rv[GP_U];
#pragma unroll
      for (int u = 0; u < GP_U; ++u) {
        const uint32_t i = i0 + u * GP_T;
        rv[u] = i < e ? __builtin_nontemporal_load(&recs[i]) : 0xFFFFFFFFu;
      }
#pragma unroll
      for (int u = 0; u < GP_U; ++u) {
        const uint32_t r = rv[u];
        const uint32_t sk = (r >> 20) & 15u;
        if (r == 0xFFFFFFFFu || sk / GP_SK != half) continue;
        const uint32_t byte = (sk % GP_SK) * HLL_REGS + ((r >> 6) & (HLL_REGS - 1));
        const uint32_t rank = r & 63u, sh = (byte & 3u) * 8;
        uint32_t* word = &r32[byte >> 2];
        uint32_t old = *word;
        while (((old >> sh) & 0xFFu) < rank) {
          const uint32_t prev = atomicCAS(word, old, (old & ~(0xFFu << sh)) | (rank << sh));
          if (prev == old) break;
          old = prev;
        }
      }
    }
    __syncthreads();
    uint32_t* gw = reinterpret_cast<uint32_t*>(regs + g0 * HLL_REGS);
    for (uint32_t q = threadIdx.x; q < nsk * (HLL_REGS / 4); q += GP_T) {
      const uint32_t v = r32[q];
      if (!v) continue;
      uint32_t old = gw[q];
      for (;;) {
        uint32_t m = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) m |= max((old >> (8 * b)) & 0xFFu, (v >> (8 * b)) & 0xFFu) << (8 * b);
        if (m == old) break;
        const uint32_t prev = atomicCAS(&gw[q], old, m);
        if (prev == old) break;
        old = prev;
      }
    }
    __syncthreads();
  }
}

bool hll_grouped_partition_applies(const rsk_ctx* c, const DevKeys& keys, uint64_t G) {
  const int mode = c->tune.gpart;  // 0 auto, 1 always, -1 never
  const bool f16 =
      keys.offsets == nullptr && keys.fixed_len == 16 && (reinterpret_cast<uintptr_t>(keys.data) & 15) == 0;
  if (mode < 0 || !f16 || keys.n == 0 || G == 0 || G > (1ull << (GP_BIN_SHIFT + 8))) return false;
  // auto: large batches dense enough that reading + writing each touched sketch once pays
  if (mode == 0 && (keys.n < (1ull << 22) || keys.n < 16 * G)) return false;
  return true;
}

// write_all (a pending lazy clear, pool_zero too): hll_gapply writes every
// row of the pool, zero rows for sketches without records.
bool hll_add_grouped_partitioned(rsk_ctx* c, const DevKeys& keys, const uint32_t* d_groups, uint8_t* d_regs,
                                 uint64_t G, bool pool_zero, bool write_all, PCount pc) {
  if (!hll_grouped_partition_applies(c, keys, G)) return false;
  const uint32_t nbins1 = (uint32_t)(((G - 1) >> GP_BIN_SHIFT) + 1);
  const uint32_t nfine = nbins1 * PT;
  const uint32_t cus = (uint32_t)c->num_cus;
  constexpr uint32_t GU = GP_GU;   // part1 blocks per part2 unit
  constexpr uint32_t gpc = 2;      // gcount / gpart1 blocks per CU
  const uint32_t G1 = GU * ((gpc * cus + GU - 1) / GU);  // a multiple of GU
  const uint32_t p2_grid = 4 * cus;
  const uint64_t chunk = PROBE_CAP;
  const uint64_t max_np = std::min<uint64_t>(keys.n, chunk);
  const uint64_t ncnt1 = (uint64_t)nbins1 * G1 + 1, ncnt2 = (uint64_t)nfine * G1 + 1;
  size_t sb1 = 0, sb2 = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, sb1, (uint32_t*)nullptr, (uint32_t*)nullptr, (int)ncnt1, c->stream);
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, sb2, (uint32_t*)nullptr, (uint32_t*)nullptr, (int)ncnt2, c->stream);
  auto al = [](uint64_t x) { return (x + 255) & ~uint64_t(255); };
  const uint32_t xcap = (uint32_t)(GP_NP * (chunk / GP_CH + 1) + 16);  // extra work items per chunk, at most
  const uint64_t meta = 2 * al(4 * ncnt1) + 2 * al(4 * ncnt2) + al(std::max(sb1, sb2)) + al(4 * (xcap + 1)) +
                        al(4 * (ncnt1 + 1));
  uint8_t* w = c->work(meta + 2 * al(4 * max_np));
  uint32_t* cnt1 = reinterpret_cast<uint32_t*>(w);
  uint32_t* off1 = reinterpret_cast<uint32_t*>(w + al(4 * ncnt1));
  uint32_t* cnt2 = reinterpret_cast<uint32_t*>(w + 2 * al(4 * ncnt1));
  uint32_t* off2 = reinterpret_cast<uint32_t*>(w + 2 * al(4 * ncnt1) + al(4 * ncnt2));
  void* scan_tmp = w + 2 * al(4 * ncnt1) + 2 * al(4 * ncnt2);
  uint32_t* xlist = reinterpret_cast<uint32_t*>(w + 2 * al(4 * ncnt1) + 2 * al(4 * ncnt2) + al(std::max(sb1, sb2)));
  uint32_t* xcount = xlist + xcap;
  uint32_t* ustart = reinterpret_cast<uint32_t*>(w + meta - al(4 * (ncnt1 + 1)));  // part2 units + [ncnt1]: count
  uint32_t* d_nunits = ustart + ncnt1;
  uint32_t* buf_a = reinterpret_cast<uint32_t*>(w + meta);
  uint32_t* buf_b = reinterpret_cast<uint32_t*>(w + meta + al(4 * max_np));
  for (uint64_t first = 0; first < keys.n; first += chunk) {
    const uint64_t m = std::min<uint64_t>(chunk, keys.n - first);
    const uint64_t per = (m + G1 - 1) / G1;
    const uint4* kd = reinterpret_cast<const uint4*>(keys.data) + first;
    const uint32_t* gd = d_groups + first;
    {
      ProfScope ps(c, "hll_gpart_count");
      RSK_HIP(hipMemsetAsync(cnt1 + ncnt1 - 1, 0, 4, c->stream));
      hipLaunchKernelGGL(hll_gcount_kernel, dim3(G1), dim3(GP_T), 0, c->stream, gd, m, per, G, nbins1, cnt1);
      RSK_CHECK_LAUNCH("hll_gcount");
      RSK_HIP(hipcub::DeviceScan::ExclusiveSum(scan_tmp, sb1, cnt1, off1, (int)ncnt1, c->stream));
    }
    {
      ProfScope ps(c, "hll_gpart1");
      hipLaunchKernelGGL(hll_gpart1_kernel, dim3(G1), dim3(PT), 0, c->stream, kd, gd, m, per, G, nbins1, off1, buf_a);
      RSK_CHECK_LAUNCH("hll_gpart1");
    }
    {
      ProfScope ps(c, "hll_gpart2");
      RSK_HIP(hipMemsetAsync(cnt2 + ncnt2 - 1, 0, 4, c->stream));
      hipLaunchKernelGGL(hll_gcount2_kernel, dim3(nbins1 * G1), dim3(PT), 0, c->stream, buf_a, off1, G1, cnt2);
      RSK_CHECK_LAUNCH("hll_gcount2");
      RSK_HIP(hipcub::DeviceScan::ExclusiveSum(scan_tmp, sb2, cnt2, off2, (int)ncnt2, c->stream));
      hipLaunchKernelGGL(hll_gunits_kernel, dim3(1), dim3(PT), 0, c->stream, off1, G1, GU, nbins1, p2_grid, ustart,
                         d_nunits);
      RSK_CHECK_LAUNCH("hll_gunits");
      part2_launch(c, p2_grid, buf_a, off1, off2, G1, GU, nbins1 * (G1 / GU), 8u, nfine, 24u, 0xFFFFFFFFu, ustart,
                   d_nunits, buf_b);
      RSK_CHECK_LAUNCH("hll_gpart2");
    }
    {
      ProfScope ps(c, "hll_gapply");
      const uint32_t per_cu = (160u * 1024) / (GP_SK * HLL_REGS + 1024);  // workgroups resident per CU
      hipLaunchKernelGGL(hll_gapply_kernel, dim3(std::min<uint32_t>(GP_NP * nfine, 2 * per_cu * cus)), dim3(GP_T), 0,
                         c->stream,
                         buf_b, off2, G1, nfine, G, (pool_zero && first == 0) ? 1 : 0,
                         (write_all && first == 0) ? 1 : 0, d_regs, pc, c->d_lc);
      RSK_CHECK_LAUNCH("hll_gapply");
      RSK_HIP(hipMemsetAsync(xcount, 0, 4, c->stream));
      hipLaunchKernelGGL(hll_gextra_list_kernel, dim3((nfine + 255) / 256), dim3(256), 0, c->stream, off2, G1, nfine,
                         xcap, xlist, xcount);
      RSK_CHECK_LAUNCH("hll_gextra_list");
      hipLaunchKernelGGL(hll_gapply_extra_kernel, dim3(2 * cus), dim3(GP_T), 0, c->stream, buf_b, off2, G1, G, xlist,
                         xcount, xcap, d_regs);
      RSK_CHECK_LAUNCH("hll_gapply_extra");
    }
  }
  return true;
}

}  // namespace rsk
