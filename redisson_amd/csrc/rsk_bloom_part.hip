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
// then updated in LDS with ds_or_b32 and written back once:
//
//   hist   : hash the keys, count probes per slice (LDS histogram, <= 32768 slices)
//   scan   : exclusive sum -> slice_start[]; cursors; part2 tile map
//   part1  : hash again, counting-sort each 4096-probe tile in LDS by coarse
//            bucket (<= 256), write the tile as contiguous runs (u32 payload:
//            index inside the coarse bucket)
//   part2  : (filters > 256 slices) the same by slice inside each coarse bucket
//   apply  : one workgroup per slice: load the 64 KiB slice into LDS, ds_or
//            every probe, store the slice back
//
// HBM traffic per key (16-byte keys, k probes): 16 (hist) + 16 + 4k (part1)
// + 8k (part2) + 4k (apply) bytes, plus 2 x the filter per chunk -- all
// streaming, against k random memory-side atomics for the direct kernel.
#include <hipcub/hipcub.hpp>

#include <cstdlib>

#include "rsk_internal.h"

namespace rsk {

constexpr int SLICE_LOG = 19;                            // bits per slice = 2^19
constexpr uint32_t SLICE_WORDS = 1u << (SLICE_LOG - 5);  // 16384 u32 = 64 KiB of LDS
constexpr uint32_t MAX_SLICES = 32768;                   // filters up to 2^34 bits (2 GiB)
constexpr int PT = 256;                                  // partition workgroup
constexpr uint32_t TILE = 4096;                          // probes per partition tile
constexpr int HIST_T = 1024;
constexpr int APPLY_T = 1024;
constexpr uint64_t PROBE_CAP = 1ull << 31;  // probes per chunk (u32 positions)

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

// Per-slice probe counts for the whole batch.
template <bool FIXED16>
__global__ __launch_bounds__(HIST_T) void bloom_slice_hist_kernel(const uint8_t* __restrict__ data,
                                                                  const uint64_t* __restrict__ offsets,
                                                                  uint32_t fixed_len, uint64_t n, FastMod63 fm, int k,
                                                                  uint32_t nslices, uint32_t* __restrict__ hist) {
  __shared__ uint32_t h[MAX_SLICES];
  for (uint32_t s = threadIdx.x; s < nslices; s += HIST_T) h[s] = 0;
  __syncthreads();
  for (uint64_t i = (uint64_t)blockIdx.x * HIST_T + threadIdx.x; i < n; i += (uint64_t)gridDim.x * HIST_T) {
    uint64_t h1, h2;
    bloom_key_hashes<FIXED16>(data, offsets, fixed_len, i, h1, h2);
    uint64_t x = h1;
    for (int t = 0; t < k; ++t) {
      const uint64_t idx = fastmod63(x & JAVA_LONG_MAX, fm);
      atomicAdd(&h[(uint32_t)(idx >> SLICE_LOG)], 1u);
      x += (t & 1) ? h1 : h2;
    }
  }
  __syncthreads();
  for (uint32_t s = threadIdx.x; s < nslices; s += HIST_T)
    if (h[s]) atomicAdd(&hist[s], h[s]);
}

// Cursors and the part2 tile map from slice_start[0..nslices] (one block).
// Coarse bucket c covers slices [c << f2, (c+1) << f2).
__global__ __launch_bounds__(PT) void bloom_part_init_kernel(const uint32_t* __restrict__ slice_start,
                                                             uint32_t nslices, uint32_t f2, uint32_t nbins1,
                                                             uint32_t* __restrict__ cursor1,
                                                             uint32_t* __restrict__ cursor2,
                                                             uint32_t* __restrict__ tiles_before) {
  for (uint32_t s = threadIdx.x; s < nslices; s += PT) cursor2[s] = slice_start[s];
  const uint32_t c = threadIdx.x;
  uint32_t tiles = 0;
  if (c < nbins1) {
    const uint32_t lo = slice_start[c << f2];
    const uint32_t hi = slice_start[min((c + 1) << f2, nslices)];
    cursor1[c] = lo;
    tiles = (hi - lo + TILE - 1) / TILE;
  }
  uint32_t total;
  const uint32_t before = block_excl_scan256(tiles, &total);
  if (c <= nbins1) tiles_before[c] = c < nbins1 ? before : total;
  if (c == PT - 1 && nbins1 == PT) tiles_before[PT] = total;
}

// Scatter one LDS tile: probe p has payload pay[p] and tag[p] = bin << 16 |
// rank inside its bin; the tile is counting-sorted by bin in LDS and each
// bin's run is written contiguously at a slot claimed from cursor[bin].
struct TileLds {
  uint32_t hist[PT], lstart[PT], gbase[PT];
  uint32_t pay[TILE], tag[TILE], srt[TILE];
  uint8_t sbin[TILE];
};

__device__ __forceinline__ void tile_scatter(TileLds& L, uint32_t np, uint32_t* __restrict__ cursor,
                                             uint32_t* __restrict__ out) {
  __syncthreads();
  const uint32_t cnt = L.hist[threadIdx.x];
  uint32_t total;
  L.lstart[threadIdx.x] = block_excl_scan256(cnt, &total);
  if (cnt) L.gbase[threadIdx.x] = atomicAdd(&cursor[threadIdx.x], cnt);
  __syncthreads();
  for (uint32_t p = threadIdx.x; p < np; p += PT) {
    const uint32_t tg = L.tag[p], b = tg >> 16;
    const uint32_t pos = L.lstart[b] + (tg & 0xFFFFu);
    L.srt[pos] = L.pay[p];
    L.sbin[pos] = (uint8_t)b;
  }
  __syncthreads();
  for (uint32_t j = threadIdx.x; j < np; j += PT) {
    const uint32_t b = L.sbin[j];
    out[L.gbase[b] + (j - L.lstart[b])] = L.srt[j];
  }
  __syncthreads();
  L.hist[threadIdx.x] = 0;
}

// part1: keys -> probes, partitioned by coarse bucket idx >> shift1 (< 256).
template <bool FIXED16>
__global__ __launch_bounds__(PT) void bloom_part1_kernel(const uint8_t* __restrict__ data,
                                                         const uint64_t* __restrict__ offsets, uint32_t fixed_len,
                                                         uint64_t n, FastMod63 fm, int k, uint32_t shift1,
                                                         uint32_t* __restrict__ cursor1, uint32_t* __restrict__ out) {
  __shared__ TileLds L;
  const uint32_t kpt = TILE / (uint32_t)k;
  const uint64_t ntiles = (n + kpt - 1) / kpt;
  const uint64_t low = (1ull << shift1) - 1;
  L.hist[threadIdx.x] = 0;
  for (uint64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const uint64_t k0 = tile * kpt;
    const uint32_t nk = (uint32_t)(n - k0 < kpt ? n - k0 : kpt);
    __syncthreads();
    for (uint32_t q = threadIdx.x; q < nk; q += PT) {
      uint64_t h1, h2;
      bloom_key_hashes<FIXED16>(data, offsets, fixed_len, k0 + q, h1, h2);
      uint64_t x = h1;
      for (int t = 0; t < k; ++t) {
        const uint64_t idx = fastmod63(x & JAVA_LONG_MAX, fm);
        const uint32_t b = (uint32_t)(idx >> shift1);
        const uint32_t r = atomicAdd(&L.hist[b], 1u);
        const uint32_t p = q * (uint32_t)k + (uint32_t)t;
        L.pay[p] = (uint32_t)(idx & low);
        L.tag[p] = (b << 16) | r;
        x += (t & 1) ? h1 : h2;
      }
    }
    tile_scatter(L, nk * (uint32_t)k, cursor1, out);
  }
}

// part2: each coarse bucket's probes, partitioned by slice (< 2^f2 per bucket).
// Tiles never straddle a coarse bucket: tile t belongs to the bucket c with
// tiles_before[c] <= t < tiles_before[c+1].
__global__ __launch_bounds__(PT) void bloom_part2_kernel(const uint32_t* __restrict__ in,
                                                         const uint32_t* __restrict__ slice_start,
                                                         const uint32_t* __restrict__ tiles_before, uint32_t nbins1,
                                                         uint32_t f2, uint32_t nslices,
                                                         uint32_t* __restrict__ cursor2, uint32_t* __restrict__ out) {
  __shared__ TileLds L;
  __shared__ uint32_t tb[PT + 1];
  for (uint32_t c = threadIdx.x; c <= nbins1; c += PT) tb[c] = tiles_before[c];
  L.hist[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t total_tiles = tb[nbins1];
  const uint32_t low = (1u << SLICE_LOG) - 1;
  for (uint32_t tile = blockIdx.x; tile < total_tiles; tile += gridDim.x) {
    uint32_t lo_c = 0, hi_c = nbins1;  // largest c with tb[c] <= tile
    while (hi_c - lo_c > 1) {
      const uint32_t mid = (lo_c + hi_c) >> 1;
      if (tb[mid] <= tile) lo_c = mid;
      else hi_c = mid;
    }
    const uint32_t c = lo_c;
    const uint32_t end = slice_start[min((c + 1) << f2, nslices)];
    const uint32_t j0 = slice_start[c << f2] + (tile - tb[c]) * TILE;
    const uint32_t np = end - j0 < TILE ? end - j0 : TILE;
    __syncthreads();
    for (uint32_t p = threadIdx.x; p < np; p += PT) {
      const uint32_t v = __builtin_nontemporal_load(&in[j0 + p]);
      const uint32_t b = v >> SLICE_LOG;
      const uint32_t r = atomicAdd(&L.hist[b], 1u);
      L.pay[p] = v & low;
      L.tag[p] = (b << 16) | r;
    }
    tile_scatter(L, np, cursor2 + ((uint64_t)c << f2), out);
  }
}

// apply: slice s = bits words [s*16384, (s+1)*16384) updated in LDS.
__global__ __launch_bounds__(APPLY_T) void bloom_slice_apply_kernel(const uint32_t* __restrict__ probes,
                                                                    const uint32_t* __restrict__ slice_start,
                                                                    uint32_t nslices, uint32_t* __restrict__ bits,
                                                                    uint64_t nwords) {
  __shared__ __attribute__((aligned(16))) uint32_t sl[SLICE_WORDS];
  for (uint32_t s = blockIdx.x; s < nslices; s += gridDim.x) {
    const uint32_t a = slice_start[s], e = slice_start[s + 1];
    if (a == e) continue;  // uniform across the workgroup
    const uint64_t w0 = (uint64_t)s * SLICE_WORDS;
    const uint32_t nw4 = (uint32_t)((nwords - w0 < SLICE_WORDS ? nwords - w0 : SLICE_WORDS) / 4);
    uint4* g4 = reinterpret_cast<uint4*>(bits + w0);
    uint4* l4 = reinterpret_cast<uint4*>(sl);
    for (uint32_t j = threadIdx.x; j < nw4; j += APPLY_T) l4[j] = g4[j];
    __syncthreads();
    for (uint32_t j = a + threadIdx.x; j < e; j += APPLY_T) {
      const uint32_t v = __builtin_nontemporal_load(&probes[j]);
      atomicOr(&sl[v >> 5], bloom_bit_mask(v));
    }
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < nw4; j += APPLY_T) g4[j] = l4[j];
    __syncthreads();
  }
}

static int part_mode() {
  const char* e = std::getenv("RSK_BLOOM_PARTITION");  // unset: auto; "0": never; "1": always
  if (!e || !*e) return -1;
  return e[0] == '0' ? 0 : 1;
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

  const uint64_t chunk = std::max<uint64_t>(1, PROBE_CAP / k);
  const uint64_t max_np = std::min<uint64_t>(keys.n, chunk) * k;
  size_t scan_bytes = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, (uint32_t*)nullptr, (uint32_t*)nullptr, (int)(ns + 1),
                                         c->stream);
  auto al = [](uint64_t x) { return (x + 255) & ~uint64_t(255); };
  const uint64_t meta = 2 * al(4ull * (ns + 1)) + al(4 * PT) + al(4ull * ns) + al(4 * (PT + 1)) + al(scan_bytes);
  uint8_t* w = c->work(meta + (f2 ? 2 : 1) * al(4 * max_np));
  uint32_t* hist = reinterpret_cast<uint32_t*>(w);
  uint32_t* slice_start = reinterpret_cast<uint32_t*>(w + al(4ull * (ns + 1)));
  uint32_t* cursor1 = reinterpret_cast<uint32_t*>(w + 2 * al(4ull * (ns + 1)));
  uint32_t* cursor2 = reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(cursor1) + al(4 * PT));
  uint32_t* tiles_before = reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(cursor2) + al(4ull * ns));
  void* scan_tmp = reinterpret_cast<uint8_t*>(tiles_before) + al(4 * (PT + 1));
  uint32_t* buf_a = reinterpret_cast<uint32_t*>(w + meta);
  uint32_t* buf_b = f2 ? reinterpret_cast<uint32_t*>(w + meta + al(4 * max_np)) : buf_a;

  const uint32_t cus = (uint32_t)c->num_cus;
  for (uint64_t first = 0; first < keys.n; first += chunk) {
    const uint64_t m = std::min<uint64_t>(chunk, keys.n - first);
    DevKeys dk = keys;
    dk.n = m;
    if (keys.offsets) dk.offsets = keys.offsets + first;
    else dk.data = keys.data + first * keys.fixed_len;
    {
      ProfScope ps(c, "bloom_part_hist");
      RSK_HIP(hipMemsetAsync(hist, 0, 4ull * (ns + 1), c->stream));
      const uint32_t g = (uint32_t)std::min<uint64_t>(cus, (m + HIST_T - 1) / HIST_T);
      if (f16)
        hipLaunchKernelGGL(bloom_slice_hist_kernel<true>, dim3(g), dim3(HIST_T), 0, c->stream, dk.data, nullptr, 16u,
                           m, b->fm, b->k, ns, hist);
      else
        hipLaunchKernelGGL(bloom_slice_hist_kernel<false>, dim3(g), dim3(HIST_T), 0, c->stream, dk.data, dk.offsets,
                           dk.fixed_len, m, b->fm, b->k, ns, hist);
      RSK_CHECK_LAUNCH("bloom_slice_hist");
      RSK_HIP(hipcub::DeviceScan::ExclusiveSum(scan_tmp, scan_bytes, hist, slice_start, (int)(ns + 1), c->stream));
      hipLaunchKernelGGL(bloom_part_init_kernel, dim3(1), dim3(PT), 0, c->stream, slice_start, ns, f2, nbins1, cursor1,
                         cursor2, tiles_before);
      RSK_CHECK_LAUNCH("bloom_part_init");
    }
    {
      ProfScope ps(c, "bloom_part1");
      const uint64_t kpt = TILE / k;
      const uint32_t g = (uint32_t)std::min<uint64_t>(4ull * cus, (m + kpt - 1) / kpt);
      if (f16)
        hipLaunchKernelGGL(bloom_part1_kernel<true>, dim3(g), dim3(PT), 0, c->stream, dk.data, nullptr, 16u, m, b->fm,
                           b->k, shift1, cursor1, buf_a);
      else
        hipLaunchKernelGGL(bloom_part1_kernel<false>, dim3(g), dim3(PT), 0, c->stream, dk.data, dk.offsets,
                           dk.fixed_len, m, b->fm, b->k, shift1, cursor1, buf_a);
      RSK_CHECK_LAUNCH("bloom_part1");
    }
    if (f2) {
      ProfScope ps(c, "bloom_part2");
      hipLaunchKernelGGL(bloom_part2_kernel, dim3(4 * cus), dim3(PT), 0, c->stream, buf_a, slice_start, tiles_before,
                         nbins1, f2, ns, cursor2, buf_b);
      RSK_CHECK_LAUNCH("bloom_part2");
    }
    {
      ProfScope ps(c, "bloom_slice_apply");
      hipLaunchKernelGGL(bloom_slice_apply_kernel, dim3(std::min<uint32_t>(ns, 2 * cus)), dim3(APPLY_T), 0, c->stream,
                         buf_b, slice_start, ns, b->d_bits, b->nwords);
      RSK_CHECK_LAUNCH("bloom_slice_apply");
    }
  }
  return true;
}

}  // namespace rsk
