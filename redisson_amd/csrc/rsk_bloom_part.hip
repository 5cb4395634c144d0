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

#include "rsk_hllcount.h"
#include "rsk_internal.h"

namespace rsk {

#ifndef RSK_BLOOM_TILE2
#define RSK_BLOOM_TILE2 8192
#endif
constexpr int SLICE_LOG = 19;                            // bits per slice = 2^19
constexpr uint32_t SLICE_WORDS = 1u << (SLICE_LOG - 5);  // 16384 u32 = 64 KiB of LDS
constexpr uint32_t MAX_SLICES = 32768;                   // filters up to 2^34 bits (2 GiB)
constexpr int PT = 256;                                  // partition workgroup
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
// Probes per chunk: positions and offsets are u32, and every loop bound in
// part2/apply stays below 2^32 - 2^24 + TILE without wrapping.  1B keys at
// k = 7 take 2 chunks, i.e. 2 read+write passes of the filter in apply.
constexpr uint64_t PROBE_CAP = (1ull << 32) - (1ull << 24);

// Exclusive scan of one value per lane over a 256-lane workgroup.
__device__ __forceinline__ uint32_t block_excl_scan256(uint32_t v, uint32_t* total) {
  __shared__ uint32_t wsum[PT / 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    uint32_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  uint32_t pre = 0, tot = 0;
#pragma unroll
  for (int q = 0; q < PT / 64; ++q) {
    pre += q < w ? wsum[q] : 0;
    tot += wsum[q];
  }
  *total = tot;
  __syncthreads();
  return pre + x - v;
}

RSK_DEV void key_range(uint64_t n, uint64_t per, uint64_t* begin, uint64_t* end) {
  *begin = (uint64_t)blockIdx.x * per;
  if (*begin > n) *begin = n;
  *end = *begin + per < n ? *begin + per : n;
}

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

// LDS image of one partition tile: probe p has payload pay[p] and tag[p] =
// bin << 16 | rank inside its bin; the tile is counting-sorted by bin into
// srt/sbin and each bin's run is appended at cur[bin] (dlt[bin] = cur[bin] -
// lstart[bin] maps a sorted position to its output position).
template <uint32_t TS>
struct SortLds {
  uint32_t hist[PT], lstart[PT], cur[PT], dlt[PT];
  uint32_t srt[TS];
  uint8_t sbin[TS];
};
struct TileLds : SortLds<TILE> {  // + probes staged in LDS (part1: k probes per key, k is runtime)
  uint32_t pay[TILE], tag[TILE];
};

// After the ranking atomics: bin starts inside the tile.  Returns this lane's bin count.
template <class S>
__device__ __forceinline__ uint32_t tile_bins(S& L) {
  __syncthreads();
  const uint32_t cnt = L.hist[threadIdx.x];
  uint32_t total;
  const uint32_t ls = block_excl_scan256(cnt, &total);
  L.lstart[threadIdx.x] = ls;
  L.dlt[threadIdx.x] = L.cur[threadIdx.x] - ls;
  __syncthreads();
  return cnt;
}

template <class S>
__device__ __forceinline__ void tile_place(S& L, uint32_t tg, uint32_t pay) {
  const uint32_t b = tg >> 16;
  const uint32_t pos = L.lstart[b] + (tg & 0xFFFFu);
  L.srt[pos] = pay;
  L.sbin[pos] = (uint8_t)b;
}

// Sorted tile -> runs in global memory; advances the cursors.
template <class S>
__device__ __forceinline__ void tile_write(S& L, uint32_t np, uint32_t cnt, uint32_t* __restrict__ out) {
  __syncthreads();
  for (uint32_t j = threadIdx.x; j < np; j += PT) out[L.dlt[L.sbin[j]] + j] = L.srt[j];
  __syncthreads();
  L.cur[threadIdx.x] += cnt;
  L.hist[threadIdx.x] = 0;
}

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
__global__ __launch_bounds__(PT) void bloom_part2_kernel(const uint32_t* __restrict__ in,
                                                         const uint32_t* __restrict__ off1,
                                                         const uint32_t* __restrict__ off2, uint32_t G,
                                                         uint32_t GU, uint32_t nunits, uint32_t f2, uint32_t nslices,
                                                         uint32_t bin_shift, uint32_t pay_mask,
                                                         uint32_t* __restrict__ out) {
  __shared__ SortLds<TILE2> L;
  __shared__ uint32_t range[2];
  const uint32_t NB = G / GU;  // units per coarse bucket
  auto ust = [&](uint32_t v) { return off1[(uint64_t)(v / NB) * G + (v % NB) * GU]; };  // v == nunits: sentinel
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
      const uint32_t c = cu / NB, b = (cu - c * NB) * GU;
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

static int part_mode() {
  const char* e = std::getenv("RSK_BLOOM_PARTITION");  // unset: auto; "0": never; "1": always
  if (!e || !*e) return -1;
  return e[0] == '0' ? 0 : 1;
}

static uint32_t env_u32(const char* name, uint32_t dflt) {  // tuning knobs (scripts/bloom_part_tune.py)
  const char* e = std::getenv(name);
  return (e && *e) ? (uint32_t)std::strtoul(e, nullptr, 10) : dflt;
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
  const int mode = part_mode();
  const uint64_t k = (uint64_t)b->k;
  const uint64_t nslices = ((uint64_t)b->size + (1ull << SLICE_LOG) - 1) >> SLICE_LOG;
  if (mode == 0 || k < 1 || k > TILE || nslices > MAX_SLICES || keys.n == 0) return false;
  if (mode < 0 && keys.n * k < (1ull << 22)) return false;  // small batches: direct atomics
  const bool f16 =
      keys.offsets == nullptr && keys.fixed_len == 16 && (reinterpret_cast<uintptr_t>(keys.data) & 15) == 0;
  const uint32_t sb = bits_for(nslices - 1);
  const uint32_t f2 = sb > 8 ? sb - 8 : 0;
  const uint32_t shift1 = SLICE_LOG + f2;
  const uint32_t nbins1 = (uint32_t)(((nslices - 1) >> f2) + 1);
  const uint32_t ns = (uint32_t)nslices;
  const uint32_t cus = (uint32_t)c->num_cus;
  const uint32_t G = std::max<uint32_t>(1, env_u32("RSK_BLOOM_G_PER_CU", 2)) * cus;  // hist / part1 blocks
  const uint32_t p2_grid = std::max<uint32_t>(1, env_u32("RSK_BLOOM_P2_PER_CU", 4)) * cus;

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
                         1u, nbins1 * G, f2, ns, (uint32_t)SLICE_LOG, (1u << SLICE_LOG) - 1, buf_b);
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
  for (uint32_t w = blockIdx.x; w < GP_NP * nfine; w += gridDim.x) {
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
    __syncthreads();
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
    __syncthreads();
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
      __syncthreads();
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
    __syncthreads();
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

static int gpart_mode() {
  const char* e = std::getenv("RSK_HLL_GPART");  // unset: auto; "0": never; "1": always
  if (!e || !*e) return -1;
  return e[0] == '0' ? 0 : 1;
}

bool hll_grouped_partition_applies(const DevKeys& keys, uint64_t G) {
  const int mode = gpart_mode();
  const bool f16 =
      keys.offsets == nullptr && keys.fixed_len == 16 && (reinterpret_cast<uintptr_t>(keys.data) & 15) == 0;
  if (mode == 0 || !f16 || keys.n == 0 || G == 0 || G > (1ull << (GP_BIN_SHIFT + 8))) return false;
  // auto: large batches dense enough that reading + writing each touched sketch once pays
  if (mode < 0 && (keys.n < (1ull << 22) || keys.n < 16 * G)) return false;
  return true;
}

// write_all (a pending lazy clear, pool_zero too): hll_gapply writes every
// row of the pool, zero rows for sketches without records.
bool hll_add_grouped_partitioned(rsk_ctx* c, const DevKeys& keys, const uint32_t* d_groups, uint8_t* d_regs,
                                 uint64_t G, bool pool_zero, bool write_all, PCount pc) {
  if (!hll_grouped_partition_applies(keys, G)) return false;
  const uint32_t nbins1 = (uint32_t)(((G - 1) >> GP_BIN_SHIFT) + 1);
  const uint32_t nfine = nbins1 * PT;
  const uint32_t cus = (uint32_t)c->num_cus;
  const uint32_t GU = std::max<uint32_t>(1, env_u32("RSK_HLL_GPART_GU", GP_GU));  // part1 blocks per part2 unit
  const uint32_t gpc = std::max<uint32_t>(1, env_u32("RSK_HLL_GPART_G", 2));     // gcount / gpart1 blocks per CU
  const uint32_t G1 = GU * ((gpc * cus + GU - 1) / GU);                          // a multiple of GU
  const uint32_t p2_grid = std::max<uint32_t>(1, env_u32("RSK_HLL_GPART_P2", 4)) * cus;
  const uint64_t chunk = PROBE_CAP;
  const uint64_t max_np = std::min<uint64_t>(keys.n, chunk);
  const uint64_t ncnt1 = (uint64_t)nbins1 * G1 + 1, ncnt2 = (uint64_t)nfine * G1 + 1;
  size_t sb1 = 0, sb2 = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, sb1, (uint32_t*)nullptr, (uint32_t*)nullptr, (int)ncnt1, c->stream);
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, sb2, (uint32_t*)nullptr, (uint32_t*)nullptr, (int)ncnt2, c->stream);
  auto al = [](uint64_t x) { return (x + 255) & ~uint64_t(255); };
  const uint32_t xcap = (uint32_t)(GP_NP * (chunk / GP_CH + 1) + 16);  // extra work items per chunk, at most
  const uint64_t meta = 2 * al(4 * ncnt1) + 2 * al(4 * ncnt2) + al(std::max(sb1, sb2)) + al(4 * (xcap + 1));
  uint8_t* w = c->work(meta + 2 * al(4 * max_np));
  uint32_t* cnt1 = reinterpret_cast<uint32_t*>(w);
  uint32_t* off1 = reinterpret_cast<uint32_t*>(w + al(4 * ncnt1));
  uint32_t* cnt2 = reinterpret_cast<uint32_t*>(w + 2 * al(4 * ncnt1));
  uint32_t* off2 = reinterpret_cast<uint32_t*>(w + 2 * al(4 * ncnt1) + al(4 * ncnt2));
  void* scan_tmp = w + 2 * al(4 * ncnt1) + 2 * al(4 * ncnt2);
  uint32_t* xlist = reinterpret_cast<uint32_t*>(w + 2 * al(4 * ncnt1) + 2 * al(4 * ncnt2) + al(std::max(sb1, sb2)));
  uint32_t* xcount = xlist + xcap;
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
      hipLaunchKernelGGL(bloom_part2_kernel, dim3(p2_grid), dim3(PT), 0, c->stream, buf_a, off1, off2, G1, GU,
                         nbins1 * (G1 / GU), 8u, nfine, 24u, 0xFFFFFFFFu, buf_b);
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
