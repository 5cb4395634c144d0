// rsk_bloom_part.hip -- partitioned Bloom add for large batches (gfx950).
//
// RedissonBloomFilter.add (src/main/java/org/redisson/RedissonBloomFilter.java:80-114)
// sets k bits per element (k SETBITs, :94-98).  Issued directly, every bit is
// a random 4-byte atomicOr; on gfx950 integer atomics execute at the memory
// side (one 64-B request per lane when the 64 lanes hit 64 lines), so a
// filter larger than the caches runs at ~20 G bit-RMW/s (MI355X_MICROARCH.md,
// "Global float atomics": 64 lanes in 64 rows ~17x slower than contiguous).
//
// Bit setting is an OR, so the order of the probes does not matter.  For
// batches of millions of keys the probes are instead partitioned by the
// 64 KiB slice (2^19 bits) of the filter they land in, and each slice is
// then updated in LDS with ds_or_b32 and written back once.  Every output
// position is computed up front (no global atomics, deterministic layout):
//
//   hist   : G blocks, block b hashes its contiguous key range and writes
//            cnt[s][b] = its probes in slice s (LDS histogram, <= 32768 slices)
//   scan   : off2 = exclusive sum of cnt in slice-major order, so slice s's
//            probes occupy [off2[s][0], off2[s+1][0]) and block b's share of
//            them starts at off2[s][b]
//   coarse : (filters > 256 slices) coarse bucket c = 2^f2 consecutive slices;
//            off1[c][b] = where block b's coarse-c probes go in the part1 buffer
//   part1  : block b hashes its keys again, counting-sorts each 4096-probe
//            tile in LDS by coarse bucket and appends each bucket's run at its
//            LDS cursor (initialised from off1 / off2)
//   part2  : (two levels) unit (c, b) = block b's coarse-c run, re-sorted by
//            slice and appended at off2[s][b]
//   apply  : one workgroup per slice: load the 64 KiB slice into LDS, ds_or
//            every probe, store the slice back
//
// HBM traffic per key (16-byte keys, k probes): 16 (hist) + 16 + 4k (part1)
// + 8k (part2) + 4k (apply) bytes, plus 2 x the filter per chunk -- all
// streaming or run-coalesced, against k random memory-side atomics for the
// direct kernel.
#include <hipcub/hipcub.hpp>

#include <cstdlib>

#include "rsk_internal.h"
#include "rsk_part.h"

namespace rsk {

#ifndef RSK_BLOOM_TILE2
#define RSK_BLOOM_TILE2 8192
#endif
constexpr int SLICE_LOG = 19;                            // bits per slice = 2^19
constexpr uint32_t SLICE_WORDS = 1u << (SLICE_LOG - 5);  // 16384 u32 = 64 KiB of LDS
constexpr uint32_t MAX_SLICES = 32768;                   // filters up to 2^34 bits (2 GiB)
#ifndef RSK_BLOOM_TILE1
#define RSK_BLOOM_TILE1 4096
#endif
#ifndef RSK_BLOOM_KT
#define RSK_BLOOM_KT 4
#endif
constexpr uint32_t TILE = RSK_BLOOM_TILE1;               // probes per part1 tile
constexpr int KT = RSK_BLOOM_KT;                         // keys per lane per part1 tile
constexpr uint32_t TILE2 = RSK_BLOOM_TILE2;              // probes per part2 tile (longer output runs)
constexpr int ET = TILE2 / PT;                           // elements per lane per part2 tile
constexpr int HIST_T = 1024;
constexpr int HIST_U = 4;  // 16-byte keys in flight per lane in hist
constexpr int APPLY_T = 1024;
constexpr int APPLY_U = 4;

template <typename F>
RSK_DEV void for_probes(uint64_t h1, uint64_t h2, int k, const FastMod63& fm, F&& f) {
  ProbeSeq ps(h1, h2, fm);
  for (int t = 0; t < k; ++t) {
    f(t, ps.idx);
    if (t + 1 < k) ps.next(t, fm);
  }
}

// hist: cnt[s * G + b] = probes of block b's keys that land in slice s.
template <bool FIXED16>
__global__ __launch_bounds__(HIST_T) void bloom_slice_hist_kernel(const uint8_t* __restrict__ data,
                                                                  const uint64_t* __restrict__ offsets,
                                                                  uint32_t fixed_len, uint64_t n, uint64_t per,
                                                                  FastMod63 fm, int k, uint32_t nslices,
                                                                  uint32_t* __restrict__ cnt) {
  __shared__ uint32_t h[MAX_SLICES];
  for (uint32_t s = threadIdx.x; s < nslices; s += HIST_T) h[s] = 0;
  __syncthreads();
  uint64_t begin, end;
  key_range(n, per, &begin, &end);
  auto count = [&](int, uint64_t idx) { atomicAdd(&h[(uint32_t)(idx >> SLICE_LOG)], 1u); };
  if (FIXED16) {
    const uint4* keys = reinterpret_cast<const uint4*>(data);
    for (uint64_t i = begin + threadIdx.x; i < end; i += (uint64_t)HIST_T * HIST_U) {
      uint4 v[HIST_U];
#pragma unroll
      for (int u = 0; u < HIST_U; ++u) {
        const uint64_t j = i + (uint64_t)u * HIST_T;
        v[u] = j < end ? ld_nt16(keys + j) : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < HIST_U; ++u) {
        if (i + (uint64_t)u * HIST_T >= end) break;
        const uint64_t w0 = ((uint64_t)v[u].y << 32) | v[u].x, w1 = ((uint64_t)v[u].w << 32) | v[u].z;
        for_probes(xxh64_16(w0, w1), farm_16(w0, w1), k, fm, count);
      }
    }
  } else {
    for (uint64_t i = begin + threadIdx.x; i < end; i += HIST_T) {
      uint64_t h1, h2;
      bloom_key_hashes<false>(data, offsets, fixed_len, i, h1, h2);
      for_probes(h1, h2, k, fm, count);
    }
  }
  __syncthreads();
  for (uint32_t s = threadIdx.x; s < nslices; s += HIST_T) cnt[(uint64_t)s * gridDim.x + blockIdx.x] = h[s];
}

// coarse: off1[c * G + b] for coarse bucket c = slices [c << f2, (c+1) << f2).
// Bucket c's region of the part1 buffer starts where slice c << f2 starts
// (off2[(c << f2) * G]) and holds block 0's run, block 1's run, ...
__global__ __launch_bounds__(PT) void bloom_coarse_offsets_kernel(const uint32_t* __restrict__ cnt,
                                                                  const uint32_t* __restrict__ off2, uint32_t G,
                                                                  uint32_t f2, uint32_t nslices,
                                                                  uint32_t* __restrict__ off1) {
  const uint32_t c = blockIdx.x;
  const uint32_t s0 = c << f2, s1 = min((c + 1) << f2, nslices);
  const uint32_t per = (G + PT - 1) / PT;  // consecutive blocks per lane
  const uint32_t b0 = threadIdx.x * per;
  uint32_t sum = 0;
  for (uint32_t b = b0; b < b0 + per && b < G; ++b)
    for (uint32_t s = s0; s < s1; ++s) sum += cnt[(uint64_t)s * G + b];
  uint32_t total;
  uint32_t run = off2[(uint64_t)s0 * G] + block_excl_scan256(sum, &total);
  for (uint32_t b = b0; b < b0 + per && b < G; ++b) {
    off1[(uint64_t)c * G + b] = run;
    for (uint32_t s = s0; s < s1; ++s) run += cnt[(uint64_t)s * G + b];
  }
  if (c == gridDim.x - 1 && threadIdx.x == 0) off1[(uint64_t)gridDim.x * G] = off2[(uint64_t)nslices * G];
}

struct TileLds : SortLds<TILE> {  // + probes staged in LDS (part1: k probes per key, k is runtime)
  uint32_t pay[TILE], tag[TILE];
};

__device__ __forceinline__ void tile_scatter(TileLds& L, uint32_t np, uint32_t* __restrict__ out) {
  const uint32_t cnt = tile_bins(L);
  for (uint32_t p = threadIdx.x; p < np; p += PT) tile_place(L, L.tag[p], L.pay[p]);
  tile_write(L, np, cnt, out);
}

// part1: block b's keys -> probes, partitioned by bin = idx >> shift1 (< 256);
// bin's run of block b starts at start[bin * G + b].
template <bool FIXED16>
__global__ __launch_bounds__(PT) void bloom_part1_kernel(const uint8_t* __restrict__ data,
                                                         const uint64_t* __restrict__ offsets, uint32_t fixed_len,
                                                         uint64_t n, uint64_t per, FastMod63 fm, int k,
                                                         uint32_t shift1, uint32_t nbins,
                                                         const uint32_t* __restrict__ start,
                                                         uint32_t* __restrict__ out) {
  __shared__ TileLds L;
  uint64_t begin, end;
  key_range(n, per, &begin, &end);
  const uint32_t kpt = min((uint32_t)(PT * KT), TILE / (uint32_t)k);  // keys per tile
  const uint64_t low = (1ull << shift1) - 1;
  L.hist[threadIdx.x] = 0;
  if (threadIdx.x < nbins) L.cur[threadIdx.x] = start[(uint64_t)threadIdx.x * gridDim.x + blockIdx.x];
  auto hash_tile_key = [&](uint32_t q, uint64_t h1, uint64_t h2) {
    for_probes(h1, h2, k, fm, [&](int t, uint64_t idx) {
      const uint32_t b = (uint32_t)(idx >> shift1);
      const uint32_t r = atomicAdd(&L.hist[b], 1u);
      const uint32_t p = q * (uint32_t)k + (uint32_t)t;
      L.pay[p] = (uint32_t)(idx & low);
      L.tag[p] = (b << 16) | r;
    });
  };
  if (FIXED16) {
    const uint4* keys = reinterpret_cast<const uint4*>(data);
    uint4 nxt[KT];
    auto fetch = [&](uint64_t k0) {
#pragma unroll
      for (int u = 0; u < KT; ++u) {
        const uint32_t q = threadIdx.x + u * PT;
        nxt[u] = (q < kpt && k0 + q < end) ? ld_nt16(keys + k0 + q) : make_uint4(0, 0, 0, 0);
      }
    };
    fetch(begin);
    for (uint64_t k0 = begin; k0 < end; k0 += kpt) {
      const uint32_t nk = (uint32_t)(end - k0 < kpt ? end - k0 : kpt);
      uint4 cur[KT];
#pragma unroll
      for (int u = 0; u < KT; ++u) cur[u] = nxt[u];
      fetch(k0 + kpt);  // next tile's keys stream in while this one is sorted
      __syncthreads();
#pragma unroll
      for (int u = 0; u < KT; ++u) {
        const uint32_t q = threadIdx.x + u * PT;
        if (q < nk) {
          const uint64_t w0 = ((uint64_t)cur[u].y << 32) | cur[u].x, w1 = ((uint64_t)cur[u].w << 32) | cur[u].z;
          hash_tile_key(q, xxh64_16(w0, w1), farm_16(w0, w1));
        }
      }
      tile_scatter(L, nk * (uint32_t)k, out);
    }
  } else {
    for (uint64_t k0 = begin; k0 < end; k0 += kpt) {
      const uint32_t nk = (uint32_t)(end - k0 < kpt ? end - k0 : kpt);
      __syncthreads();
      for (uint32_t q = threadIdx.x; q < nk; q += PT) {
        uint64_t h1, h2;
        bloom_key_hashes<false>(data, offsets, fixed_len, k0 + q, h1, h2);
        hash_tile_key(q, h1, h2);
      }
      tile_scatter(L, nk * (uint32_t)k, out);
    }
  }
}

// part2: unit u = (c, blocks [bb*GU, (bb+1)*GU)), u = c * (G/GU) + bb, in order
// (= the part1 buffer in order): bucket c's runs of GU consecutive part1 blocks
// are contiguous in the input and so are their slice-s outputs (off2 is
// slice-major), so one unit covers them with one cursor per slice.  bin =
// value >> bin_shift < 2^f2; value & pay_mask is written (Bloom slice offsets,
// or HLL records as they are).  Workgroup w takes the units whose start falls
// in its equal share of the buffer, re-sorts each unit by slice (2^f2 bins)
// and appends slice s's run at off2[s * G + b] (b = the unit's first block).
// With a unit table (ustart != nullptr, the grouped PFADD): unit v starts at
// part1 block ustart[v] (linear c * G + b, ascending, [nunits] = the end) and
// nunits is read from d_nunits -- units of one part1 block in buckets whose
// runs would otherwise make units far above a workgroup's share (skewed groups).
__global__ __launch_bounds__(PT) void bloom_part2_kernel(const uint32_t* __restrict__ in,
                                                         const uint32_t* __restrict__ off1,
                                                         const uint32_t* __restrict__ off2, uint32_t G,
                                                         uint32_t GU, uint32_t nunits_arg, uint32_t f2,
                                                         uint32_t nslices, uint32_t bin_shift, uint32_t pay_mask,
                                                         const uint32_t* __restrict__ ustart,
                                                         const uint32_t* __restrict__ d_nunits,
                                                         uint32_t* __restrict__ out) {
  __shared__ SortLds<TILE2> L;
  __shared__ uint32_t range[2];
  const uint32_t NB = G / GU;  // units per coarse bucket (no unit table)
  const uint32_t nunits = ustart ? *d_nunits : nunits_arg;
  auto ublock = [&](uint32_t v) -> uint64_t {  // linear first part1 block of unit v (v == nunits: the end)
    return ustart ? (uint64_t)ustart[v] : (uint64_t)(v / NB) * G + (v % NB) * GU;
  };
  auto ust = [&](uint32_t v) { return off1[ublock(v)]; };
  const uint32_t total = ust(nunits);
  if (threadIdx.x < 2) {  // first unit starting at or after a share boundary
    const uint64_t edge = (uint64_t)total * (blockIdx.x + threadIdx.x) / gridDim.x;
    uint32_t lo = 0, hi = nunits;
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (ust(mid) < edge) lo = mid + 1;
      else hi = mid;
    }
    range[threadIdx.x] = (blockIdx.x + threadIdx.x == gridDim.x) ? nunits : lo;
  }
  L.hist[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t u_end = range[1];
  const uint32_t nb = 1u << f2;
  // tile cursor: unit u, element j (absolute); the next tile is prefetched
  uint32_t u = range[0];
  uint32_t j = u < u_end ? ust(u) : 0;
  auto skip_empty = [&]() {
    while (u < u_end && j >= ust(u + 1)) {
      ++u;
      if (u < u_end) j = ust(u);
    }
  };
  skip_empty();
  uint32_t nxt[ET];
  auto fetch = [&](uint32_t fu, uint32_t fj) {
    const uint32_t lim = fu < u_end ? ust(fu + 1) : 0;
#pragma unroll
    for (int e = 0; e < ET; ++e) {
      const uint32_t p = fj + threadIdx.x + e * PT;
      nxt[e] = (fu < u_end && p < lim && p < fj + TILE2) ? __builtin_nontemporal_load(&in[p]) : 0;
    }
  };
  fetch(u, j);
  uint32_t loaded_unit = 0xFFFFFFFFu;
  while (u < u_end) {
    const uint32_t ue = ust(u + 1);
    const uint32_t np = ue - j < TILE2 ? ue - j : TILE2;
    uint32_t vals[ET];
#pragma unroll
    for (int e = 0; e < ET; ++e) vals[e] = nxt[e];
    const uint32_t cu = u;
    // advance to the next tile and prefetch it
    j += np;
    skip_empty();
    fetch(u, j);
    __syncthreads();
    if (cu != loaded_unit) {  // new unit: its slice cursors
      const uint64_t lb = ublock(cu);
      const uint32_t c = (uint32_t)(lb / G), b = (uint32_t)(lb - (uint64_t)c * G);
      const uint32_t s = (c << f2) + threadIdx.x;
      if (threadIdx.x < nb && s < nslices) L.cur[threadIdx.x] = off2[(uint64_t)s * G + b];
      loaded_unit = cu;
    }
    uint32_t tag[ET];  // payload and rank stay in registers
#pragma unroll
    for (int e = 0; e < ET; ++e) {
      const uint32_t p = threadIdx.x + e * PT;
      if (p < np) {
        const uint32_t bin = vals[e] >> bin_shift;
        tag[e] = (bin << 16) | atomicAdd(&L.hist[bin], 1u);
      }
    }
    const uint32_t cnt = tile_bins(L);
#pragma unroll
    for (int e = 0; e < ET; ++e)
      if (threadIdx.x + e * PT < np) tile_place(L, tag[e], vals[e] & pay_mask);
    tile_write(L, np, cnt, out);
  }
}

// apply: slice s = bits words [s*16384, (s+1)*16384), probes [off2[s*G], off2[(s+1)*G]).
__global__ __launch_bounds__(APPLY_T) void bloom_slice_apply_kernel(const uint32_t* __restrict__ probes,
                                                                    const uint32_t* __restrict__ off2, uint32_t G,
                                                                    uint32_t nslices, uint32_t* __restrict__ bits,
                                                                    uint64_t nwords) {
  __shared__ __attribute__((aligned(16))) uint32_t sl[SLICE_WORDS];
  for (uint32_t s = blockIdx.x; s < nslices; s += gridDim.x) {
    const uint32_t a = off2[(uint64_t)s * G], e = off2[(uint64_t)(s + 1) * G];
    if (a == e) continue;  // uniform across the workgroup
    const uint64_t w0 = (uint64_t)s * SLICE_WORDS;
    const uint32_t nw4 = (uint32_t)((nwords - w0 < SLICE_WORDS ? nwords - w0 : SLICE_WORDS) / 4);
    uint4* g4 = reinterpret_cast<uint4*>(bits + w0);
    uint4* l4 = reinterpret_cast<uint4*>(sl);
    for (uint32_t q = threadIdx.x; q < nw4; q += APPLY_T) l4[q] = g4[q];
    __syncthreads();
    for (uint32_t q = a + threadIdx.x; q < e; q += APPLY_T * APPLY_U) {
      uint32_t v[APPLY_U];
#pragma unroll
      for (int t = 0; t < APPLY_U; ++t) {
        const uint32_t i = q + t * APPLY_T;
        v[t] = i < e ? __builtin_nontemporal_load(&probes[i]) : 0xFFFFFFFFu;
      }
#pragma unroll
      for (int t = 0; t < APPLY_U; ++t)
        if (v[t] != 0xFFFFFFFFu) atomicOr(&sl[v[t] >> 5], bloom_bit_mask(v[t]));
    }
    __syncthreads();
    for (uint32_t q = threadIdx.x; q < nw4; q += APPLY_T) g4[q] = l4[q];
    __syncthreads();
  }
}

static uint32_t bits_for(uint64_t v) {  // bits needed to hold v (0 -> 0)
  uint32_t b = 0;
  while (v) {
    ++b;
    v >>= 1;
  }
  return b;
}

bool bloom_add_partitioned(rsk_ctx* c, rsk_bloom* b, const DevKeys& keys) {
  const int mode = c->tune.bloom_part;  // 0 auto, 1 at any batch size, -1 never
  const uint64_t k = (uint64_t)b->k;
  const uint64_t nslices = ((uint64_t)b->size + (1ull << SLICE_LOG) - 1) >> SLICE_LOG;
  if (mode < 0 || k < 1 || k > TILE || nslices > MAX_SLICES || keys.n == 0) return false;
  if (mode == 0 && keys.n * k < (1ull << 22)) return false;  // small batches: direct atomics
  const bool f16 =
      keys.offsets == nullptr && keys.fixed_len == 16 && (reinterpret_cast<uintptr_t>(keys.data) & 15) == 0;
  const uint32_t sb = bits_for(nslices - 1);
  const uint32_t f2 = sb > 8 ? sb - 8 : 0;
  const uint32_t shift1 = SLICE_LOG + f2;
  const uint32_t nbins1 = (uint32_t)(((nslices - 1) >> f2) + 1);
  const uint32_t ns = (uint32_t)nslices;
  const uint32_t cus = (uint32_t)c->num_cus;
  const uint32_t G = 2 * cus;        // hist / part1 blocks (3 and 4 per CU measured slower)
  const uint32_t p2_grid = 4 * cus;

  const uint64_t chunk = std::max<uint64_t>(1, PROBE_CAP / k);
  const uint64_t max_np = std::min<uint64_t>(keys.n, chunk) * k;
  const uint64_t ncnt = (uint64_t)ns * G + 1;
  const uint64_t noff1 = (uint64_t)nbins1 * G + 1;
  size_t scan_bytes = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, (uint32_t*)nullptr, (uint32_t*)nullptr, (int)ncnt,
                                         c->stream);
  auto al = [](uint64_t x) { return (x + 255) & ~uint64_t(255); };
  const uint64_t meta = 2 * al(4 * ncnt) + al(4 * noff1) + al(scan_bytes);
  uint8_t* w = c->work(meta + (f2 ? 2 : 1) * al(4 * max_np));
  uint32_t* cnt = reinterpret_cast<uint32_t*>(w);
  uint32_t* off2 = reinterpret_cast<uint32_t*>(w + al(4 * ncnt));
  uint32_t* off1 = reinterpret_cast<uint32_t*>(w + 2 * al(4 * ncnt));
  void* scan_tmp = w + 2 * al(4 * ncnt) + al(4 * noff1);
  uint32_t* buf_a = reinterpret_cast<uint32_t*>(w + meta);
  uint32_t* buf_b = f2 ? reinterpret_cast<uint32_t*>(w + meta + al(4 * max_np)) : buf_a;

  for (uint64_t first = 0; first < keys.n; first += chunk) {
    const uint64_t m = std::min<uint64_t>(chunk, keys.n - first);
    const uint64_t per = (m + G - 1) / G;
    DevKeys dk = keys;
    dk.n = m;
    if (keys.offsets) dk.offsets = keys.offsets + first;
    else dk.data = keys.data + first * keys.fixed_len;
    {
      ProfScope ps(c, "bloom_part_hist");
      RSK_HIP(hipMemsetAsync(cnt + ncnt - 1, 0, 4, c->stream));
      if (f16)
        hipLaunchKernelGGL(bloom_slice_hist_kernel<true>, dim3(G), dim3(HIST_T), 0, c->stream, dk.data, nullptr, 16u,
                           m, per, b->fm, b->k, ns, cnt);
      else
        hipLaunchKernelGGL(bloom_slice_hist_kernel<false>, dim3(G), dim3(HIST_T), 0, c->stream, dk.data, dk.offsets,
                           dk.fixed_len, m, per, b->fm, b->k, ns, cnt);
      RSK_CHECK_LAUNCH("bloom_slice_hist");
      RSK_HIP(hipcub::DeviceScan::ExclusiveSum(scan_tmp, scan_bytes, cnt, off2, (int)ncnt, c->stream));
      if (f2) {
        hipLaunchKernelGGL(bloom_coarse_offsets_kernel, dim3(nbins1), dim3(PT), 0, c->stream, cnt, off2, G, f2, ns,
                           off1);
        RSK_CHECK_LAUNCH("bloom_coarse_offsets");
      }
    }
    {
      ProfScope ps(c, "bloom_part1");
      const uint32_t* start = f2 ? off1 : off2;
      if (f16)
        hipLaunchKernelGGL(bloom_part1_kernel<true>, dim3(G), dim3(PT), 0, c->stream, dk.data, nullptr, 16u, m, per,
                           b->fm, b->k, shift1, nbins1, start, buf_a);
      else
        hipLaunchKernelGGL(bloom_part1_kernel<false>, dim3(G), dim3(PT), 0, c->stream, dk.data, dk.offsets,
                           dk.fixed_len, m, per, b->fm, b->k, shift1, nbins1, start, buf_a);
      RSK_CHECK_LAUNCH("bloom_part1");
    }
    if (f2) {
      ProfScope ps(c, "bloom_part2");
      hipLaunchKernelGGL(bloom_part2_kernel, dim3(p2_grid), dim3(PT), 0, c->stream, buf_a, off1, off2, G,
                         1u, nbins1 * G, f2, ns, (uint32_t)SLICE_LOG, (1u << SLICE_LOG) - 1,
                         (const uint32_t*)nullptr, (const uint32_t*)nullptr, buf_b);
      RSK_CHECK_LAUNCH("bloom_part2");
    }
    {
      ProfScope ps(c, "bloom_slice_apply");
      hipLaunchKernelGGL(bloom_slice_apply_kernel, dim3(std::min<uint32_t>(ns, 2 * cus)), dim3(APPLY_T), 0, c->stream,
                         buf_b, off2, G, ns, b->d_bits, b->nwords);
      RSK_CHECK_LAUNCH("bloom_slice_apply");
    }
  }
  return true;
}


}  // namespace rsk
