// rsk_part.h -- the LDS counting-sort tile shared by the exact-offset
// partition passes: the Bloom insert's part1/part2 (rsk_bloom_part.hip) and
// the grouped PFADD's gpart1 (rsk_hll_group.hip).
#pragma once

#include "rsk_internal.h"

namespace rsk {

constexpr int PT = 256;  // partition workgroup
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

}  // namespace rsk
