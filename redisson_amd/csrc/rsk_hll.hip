// rsk_hll.hip -- HyperLogLog kernels for gfx950 (Redis 3.2.0 semantics).
//
// Replaces the PFADD / PFCOUNT / PFMERGE arithmetic that RedissonHyperLogLog
// (src/main/java/org/redisson/RedissonHyperLogLog.java:65-97) delegates to the
// Redis server (hyperloglog.c: hllAdd/hllPatLen, hllCount, pfmergeCommand).
//
// Data layout in HBM: a pool of sketches, [n][16384] raw registers, one byte
// each (Redis's internal HLL_RAW form); the 6-bit dense packing only exists
// at the Redis export/import boundary.  Each pool also keeps card[n], the
// 8-byte cardinality cache of the Redis header.
//
// PFADD (streaming, HBM-bound): a persistent grid of 2 workgroups per CU.
// Every workgroup owns a private 16384 x u32 register file in LDS (64 KiB,
// so two fit in the CU's 160 KiB), streams a contiguous slice of the key
// array with 16-byte loads, hashes each key and applies ds_max_u32.  At the
// end it writes its file as 16 KiB of bytes (a "slab"); one reduce kernel
// max-merges all slabs and the sketch's old registers (deterministic, no
// global atomics), and raises a flag if any register grew.
#include <hipcub/hipcub.hpp>

#include <cstring>

#include "rsk_hll_kern.h"
#include "rsk_hllcount.h"
#include "rsk_internal.h"

namespace rsk {

// Any fixed stride or blob+offsets: lane-per-key MurmurHash64A.
template <bool VAR>
__global__ __launch_bounds__(RSK_ADD_THREADS, 2) void hll_add_bytes_kernel(const uint8_t* __restrict__ data,
                                                                           const uint64_t* __restrict__ offsets,
                                                                           uint32_t fixed_len, uint64_t n,
                                                                           uint64_t per_block,
                                                                           uint8_t* __restrict__ slabs) {
  __shared__ __attribute__((aligned(16))) uint32_t regs[HLL_REGS];
  lds_zero(regs);
  __syncthreads();
  const uint64_t begin = (uint64_t)blockIdx.x * per_block;
  const uint64_t end = begin + per_block < n ? begin + per_block : n;
  for (uint64_t i = begin + threadIdx.x; i < end; i += blockDim.x) {
    uint64_t s, len;
    if (VAR) {
      s = offsets[i];
      len = offsets[i + 1] - s;
    } else {
      s = i * fixed_len;
      len = fixed_len;
    }
    hll_update(regs, len <= 64 ? murmur64a_le64(data + s, (uint32_t)len) : murmur64a(data + s, len));
  }
  __syncthreads();
  lds_to_slab(regs, slabs + (uint64_t)blockIdx.x * HLL_REGS);
}

// Max-merge `nslabs` slabs and the sketch's registers; 64 registers per
// workgroup of 256 lanes (grid 256).  If any register grew: *flag =
// max(*flag, epoch) (the caller's call number, so no reset is needed) and
// the Redis card cache is invalidated (HLL_INVALIDATE_CACHE), as it is when
// the key was just created.
__global__ __launch_bounds__(256) void hll_reduce_kernel(const uint8_t* __restrict__ slabs, uint32_t nslabs,
                                                         uint8_t* __restrict__ regs, uint32_t* __restrict__ flag,
                                                         uint32_t epoch, unsigned long long* __restrict__ card,
                                                         int created) {
  if (created && blockIdx.x == 0 && threadIdx.x == 0) atomicOr(card, 1ull << 63);
  __shared__ uint4 part[4][256];
  const int t = threadIdx.x;
  const uint64_t col = (uint64_t)blockIdx.x * 64;  // first register of this block
  uint4 acc[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) acc[q] = make_uint4(0, 0, 0, 0);
  for (uint32_t s = t; s < nslabs; s += 256) {
    const uint4* p = reinterpret_cast<const uint4*>(slabs + (uint64_t)s * HLL_REGS + col);
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[q] = bmax16(acc[q], p[q]);
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) part[q][t] = acc[q];
  __syncthreads();
  for (int stride = 128; stride > 0; stride >>= 1) {
    if (t < stride) {
#pragma unroll
      for (int q = 0; q < 4; ++q) part[q][t] = bmax16(part[q][t], part[q][t + stride]);
    }
    __syncthreads();
  }
  if (t < 4) {
    uint4* r = reinterpret_cast<uint4*>(regs + col) + t;
    uint4 old = *r;
    uint4 nw = bmax16(old, part[t][0]);
    if (nw.x != old.x || nw.y != old.y || nw.z != old.z || nw.w != old.w) {
      *r = nw;
      atomicMax(flag, epoch);
      atomicOr(card, 1ull << 63);
    }
  }
}

void hll_add_launch(rsk_ctx* c, const DevKeys& k, uint8_t* d_regs_sketch, uint64_t* d_card, uint32_t* d_flag,
                    uint32_t epoch, bool created) {
  if (k.n == 0) return;
  constexpr uint64_t T = RSK_ADD_THREADS;
  const uint64_t max_blocks = c->slab_count;
  // Enough keys per workgroup to amortise the 64 KiB LDS init + 16 KiB slab;
  // a persistent grid of the 2 workgroups per CU that the 64 KiB file allows.
  uint64_t blocks = (k.n + 4 * T - 1) / (4 * T);
  blocks = std::min<uint64_t>(blocks, std::min<uint64_t>(2ull * c->num_cus, max_blocks));
  if (blocks == 0) blocks = 1;
  uint64_t per_block = (k.n + blocks - 1) / blocks;
  if (k.offsets == nullptr && k.fixed_len == 16 && (reinterpret_cast<uintptr_t>(k.data) & 15) == 0) {
    // Round the slice up to whole tiles so every lane's loads stay coalesced.
    constexpr uint64_t T16 = 256;
    const uint64_t tile = T16 * RSK_ADD_UNROLL;
    blocks = std::min<uint64_t>((k.n + tile - 1) / tile, std::min<uint64_t>(2ull * c->num_cus, max_blocks));
    per_block = (k.n + blocks - 1) / blocks;
    per_block = (per_block + tile - 1) / tile * tile;
    blocks = (k.n + per_block - 1) / per_block;
    ProfScope ps(c, "hll_add16");
    hipLaunchKernelGGL((hll_add16_kernel<RSK_ADD_UNROLL, T16>), dim3((uint32_t)blocks), dim3(T16), 0, c->stream,
                       reinterpret_cast<const uint4*>(k.data), k.n, per_block, c->d_slab);
    RSK_CHECK_LAUNCH("hll_add16");
  } else if (k.offsets == nullptr) {
    ProfScope ps(c, "hll_add_fixed");
    hipLaunchKernelGGL(hll_add_bytes_kernel<false>, dim3((uint32_t)blocks), dim3(T), 0, c->stream, k.data, nullptr,
                       k.fixed_len, k.n, per_block, c->d_slab);
    RSK_CHECK_LAUNCH("hll_add_fixed");
  } else {
    var_grid(c, k.n, &blocks, &per_block);
    ProfScope ps(c, "hll_add_var");
    hipLaunchKernelGGL(hll_add_var_staged_kernel<1>, dim3((uint32_t)blocks), dim3(VAR_TILE), 0, c->stream, k.data,
                       k.offsets, k.n, per_block, c->d_slab);
    RSK_CHECK_LAUNCH("hll_add_var");
  }
  ProfScope ps(c, "hll_reduce");
  hipLaunchKernelGGL(hll_reduce_kernel, dim3(HLL_REGS / 64), dim3(256), 0, c->stream, c->d_slab, (uint32_t)blocks,
                     d_regs_sketch, d_flag, epoch, reinterpret_cast<unsigned long long*>(d_card), created ? 1 : 0);
  RSK_CHECK_LAUNCH("hll_reduce");
}

// dst = max(dst, src) for one sketch; flag if dst grew (PFMERGE from raw).
__global__ __launch_bounds__(256) void hll_max_into_kernel(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src,
                                                           uint32_t* __restrict__ flag) {
  const int j = blockIdx.x * 256 + threadIdx.x;  // uint4 index, 1024 total
  uint4* d = reinterpret_cast<uint4*>(dst) + j;
  uint4 a = *d, b = reinterpret_cast<const uint4*>(src)[j];
  uint4 m = bmax16(a, b);
  if (m.x != a.x || m.y != a.y || m.z != a.z || m.w != a.w) {
    *d = m;
    if (flag) atomicOr(flag, 1u);
  }
}

void hll_max_into_launch(rsk_ctx* c, uint8_t* d_dst, const uint8_t* d_src, uint32_t* d_flag) {
  ProfScope ps(c, "hll_max_into");
  hipLaunchKernelGGL(hll_max_into_kernel, dim3(HLL_REGS / 16 / 256), dim3(256), 0, c->stream, d_dst, d_src, d_flag);
  RSK_CHECK_LAUNCH("hll_max_into");
}

// --------------------------------------------------------- grouped PFADD
// Pair i -> sketch groups[i]; byte-max on the register's u32 word by CAS.
__global__ __launch_bounds__(256) void hll_add_grouped16_kernel(const uint4* __restrict__ keys,
                                                                const uint32_t* __restrict__ groups, uint64_t n,
                                                                uint8_t* __restrict__ regs, uint64_t G) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint4 v = ld_nt16(&keys[i]);
    uint32_t g = __builtin_nontemporal_load(&groups[i]);
    if (g >= G) continue;
    uint64_t h = murmur64a_16(((uint64_t)v.y << 32) | v.x, ((uint64_t)v.w << 32) | v.z);
    uint32_t idx = hll_index(h), rank = hll_rank(h);
    uint32_t* word = reinterpret_cast<uint32_t*>(regs + (uint64_t)g * HLL_REGS + (idx & ~3u));
    const uint32_t sh = (idx & 3u) * 8;
    uint32_t old = *word;
    while (((old >> sh) & 0xFF) < rank) {
      uint32_t nw = (old & ~(0xFFu << sh)) | (rank << sh);
      uint32_t prev = atomicCAS(word, old, nw);
      if (prev == old) break;
      old = prev;
    }
  }
}

__global__ __launch_bounds__(256) void hll_add_grouped_bytes_kernel(const uint8_t* __restrict__ data,
                                                                    const uint64_t* __restrict__ offsets,
                                                                    uint32_t fixed_len,
                                                                    const uint32_t* __restrict__ groups, uint64_t n,
                                                                    uint8_t* __restrict__ regs, uint64_t G) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t g = groups[i];
    if (g >= G) continue;
    uint64_t s = offsets ? offsets[i] : i * fixed_len;
    uint64_t len = offsets ? offsets[i + 1] - s : fixed_len;
    uint64_t h = murmur64a(data + s, len);
    uint32_t idx = hll_index(h), rank = hll_rank(h);
    uint32_t* word = reinterpret_cast<uint32_t*>(regs + (uint64_t)g * HLL_REGS + (idx & ~3u));
    const uint32_t sh = (idx & 3u) * 8;
    uint32_t old = *word;
    while (((old >> sh) & 0xFF) < rank) {
      uint32_t nw = (old & ~(0xFFu << sh)) | (rank << sh);
      uint32_t prev = atomicCAS(word, old, nw);
      if (prev == old) break;
      old = prev;
    }
  }
}

void hll_add_grouped_launch(rsk_ctx* c, const DevKeys& k, const uint32_t* d_groups, uint8_t* d_regs, uint64_t G,
                            bool pool_zero, bool write_all, PCount pc) {
  if (k.n == 0) return;
  if (hll_add_grouped_partitioned(c, k, d_groups, d_regs, G, pool_zero, write_all, pc)) return;  // large batches: per-sketch LDS updates
  uint64_t blocks = (k.n + 255) / 256;
  uint64_t cap = (uint64_t)c->num_cus * 16;
  if (blocks > cap) blocks = cap;
  if (k.offsets == nullptr && k.fixed_len == 16 && (reinterpret_cast<uintptr_t>(k.data) & 15) == 0) {
    ProfScope ps(c, "hll_add_grouped16");
    hipLaunchKernelGGL(hll_add_grouped16_kernel, dim3((uint32_t)blocks), dim3(256), 0, c->stream,
                       reinterpret_cast<const uint4*>(k.data), d_groups, k.n, d_regs, G);
    RSK_CHECK_LAUNCH("hll_add_grouped16");
  } else {
    ProfScope ps(c, "hll_add_grouped");
    hipLaunchKernelGGL(hll_add_grouped_bytes_kernel, dim3((uint32_t)blocks), dim3(256), 0, c->stream, k.data,
                       k.offsets, k.fixed_len, d_groups, k.n, d_regs, G);
    RSK_CHECK_LAUNCH("hll_add_grouped");
  }
}

// ---------------------------------------------------------------- PFCOUNT
// One sketch's 16 KiB as 16 uint4 per lane of a wave.
RSK_DEV SumD wave_sum(const uint4 (&v)[16]) {
  SumD s{0.0, 0, 0};
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    acc_word(s, v[q].x);
    acc_word(s, v[q].y);
    acc_word(s, v[q].z);
    acc_word(s, v[q].w);
  }
  return wave_reduce(s);
}

RSK_DEV double dense_order_sum(const uint8_t* r, int* ezp) {
  double E = 0;
  int ez = 0;
  for (int g = 0; g < HLL_REGS / 16; ++g) {
    const uint8_t* q = r + 16 * g;
    for (int t = 0; t < 16; ++t) ez += q[t] == 0;
    E += (pe(q[0]) + pe(q[1])) + (pe(q[2]) + pe(q[3])) + (pe(q[4]) + pe(q[5])) + (pe(q[6]) + pe(q[7])) +
         (pe(q[8]) + pe(q[9])) + (pe(q[10]) + pe(q[11])) + (pe(q[12]) + pe(q[13])) + (pe(q[14]) + pe(q[15]));
  }
  *ezp = ez;
  return E;
}

// PFCOUNT, one wave per sketch: the 16 KiB are 16 uint4 loads per lane, all
// in flight at once; no LDS and no barrier.
__global__ __launch_bounds__(256) void hll_count_kernel(const uint8_t* __restrict__ regs, uint64_t* __restrict__ card,
                                                        const uint64_t* __restrict__ ids, SmallIds small, uint64_t n,
                                                        const double* __restrict__ lc, uint64_t* __restrict__ out,
                                                        PCount pc) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t nwaves = (uint64_t)gridDim.x * 4;
  for (uint64_t b = ((uint64_t)blockIdx.x * 256 + threadIdx.x) >> 6; b < n; b += nwaves) {
    const uint64_t id = ids ? ids[b] : (small.n ? small.v[b] : b);
    const uint64_t cached = card[id];
    if ((cached >> 63) == 0) {  // HLL_VALID_CACHE
      if (lane == 0) out[b] = cached;
      continue;
    }
    if (pc.pcount && pc.pepoch[id] == pc.epoch) {  // estimated by the grouped add from these registers
      if (lane == 0) {
        const uint64_t est = pc.pcount[id];
        out[b] = est;
        card[id] = est;
      }
      continue;
    }
    const uint8_t* r = regs + id * HLL_REGS;
    const uint4* r4 = reinterpret_cast<const uint4*>(r) + lane;
    uint4 v[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) v[q] = r4[64 * q];
    const SumD s = wave_sum(v);
    if (lane == 0) {
      int ez = (int)s.ez;
      const double E = exact_total(s) ? s.t : dense_order_sum(r, &ez);
      const uint64_t est = hll_estimate(E, ez, lc);
      out[b] = est;
      card[id] = est;  // cache refreshed, valid
    }
  }
}

// Large counts (a pool's 10^6 sketches after a grouped add): a sketch per lane answers from
// the card cache or the add's precomputed estimate and lists the others (wave-aggregated
// append); then a wave per listed sketch, as hll_count_kernel.  One wave per sketch for the
// whole batch spent ~0.2 ms dispatching 10^6 waves that each read three words.
__global__ __launch_bounds__(256) void hll_count_fast_kernel(uint64_t* __restrict__ card, const uint64_t* __restrict__ ids,
                                                             SmallIds small, uint64_t n, uint64_t* __restrict__ out,
                                                             PCount pc, uint32_t* __restrict__ slow_n,
                                                             uint32_t* __restrict__ slow) {
  const uint32_t lane = threadIdx.x & 63;
  for (uint64_t w = (uint64_t)blockIdx.x * 256 + (threadIdx.x & ~63u); w < n; w += (uint64_t)gridDim.x * 256) {
    const uint64_t b = w + lane;
    bool rest = false;
    if (b < n) {
      const uint64_t id = ids ? ids[b] : (small.n ? small.v[b] : b);
      const uint64_t cached = card[id];
      if ((cached >> 63) == 0) {  // HLL_VALID_CACHE
        out[b] = cached;
      } else if (pc.pcount && pc.pepoch[id] == pc.epoch) {
        const uint64_t est = pc.pcount[id];
        out[b] = est;
        card[id] = est;
      } else {
        rest = true;
      }
    }
    const uint64_t m = __ballot(rest);
    if (m) {
      const int leader = __ffsll((long long)m) - 1;
      uint32_t at = 0;
      if ((int)lane == leader) at = atomicAdd(slow_n, (uint32_t)__popcll(m));
      at = __shfl(at, leader);
      const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
      if (rest) slow[at + below] = (uint32_t)b;
    }
  }
}

__global__ __launch_bounds__(256) void hll_count_slow_kernel(const uint8_t* __restrict__ regs, uint64_t* __restrict__ card,
                                                             const uint64_t* __restrict__ ids, SmallIds small,
                                                             const uint32_t* __restrict__ slow_n,
                                                             const uint32_t* __restrict__ slow,
                                                             const double* __restrict__ lc, uint64_t* __restrict__ out) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t nwaves = (uint64_t)gridDim.x * 4, cnt = *slow_n;
  for (uint64_t s = ((uint64_t)blockIdx.x * 256 + threadIdx.x) >> 6; s < cnt; s += nwaves) {
    const uint64_t b = slow[s];
    const uint64_t id = ids ? ids[b] : (small.n ? small.v[b] : b);
    const uint8_t* r = regs + id * HLL_REGS;
    const uint4* r4 = reinterpret_cast<const uint4*>(r) + lane;
    uint4 v[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) v[q] = r4[64 * q];
    const SumD sm = wave_sum(v);
    if (lane == 0) {
      int ez = (int)sm.ez;
      const double E = exact_total(sm) ? sm.t : dense_order_sum(r, &ez);
      const uint64_t est = hll_estimate(E, ez, lc);
      out[b] = est;
      card[id] = est;
    }
  }
}

void hll_count_launch(rsk_ctx* c, const uint8_t* d_regs, uint64_t* d_card, const uint64_t* d_ids,
                      const SmallIds& small, uint64_t n, uint64_t* d_out, PCount pc) {
  if (n == 0) return;
  if (n >= 4096 && n < (1ull << 32)) {
    ProfScope ps(c, "hll_count");
    uint32_t* slow = reinterpret_cast<uint32_t*>(c->cslow(4 * (n + 64)));  // [0]: count; the list from [64]
    RSK_HIP(hipMemsetAsync(slow, 0, 4, c->stream));
    const uint64_t g1 = std::min<uint64_t>((n + 255) / 256, 65536);
    hipLaunchKernelGGL(hll_count_fast_kernel, dim3((uint32_t)g1), dim3(256), 0, c->stream, d_card, d_ids, small, n,
                       d_out, pc, slow, slow + 64);
    RSK_CHECK_LAUNCH("hll_count_fast");
    const uint64_t g2 = std::min<uint64_t>((n + 3) / 4, (uint64_t)c->num_cus * 16);
    hipLaunchKernelGGL(hll_count_slow_kernel, dim3((uint32_t)g2), dim3(256), 0, c->stream, d_regs, d_card, d_ids, small,
                       slow, slow + 64, c->d_lc, d_out);
    RSK_CHECK_LAUNCH("hll_count_slow");
    return;
  }
  uint64_t grid = (n + 3) / 4;  // 4 waves (sketches) per workgroup
  if (grid > (1u << 20)) grid = 1u << 20;
  ProfScope ps(c, "hll_count");
  hipLaunchKernelGGL(hll_count_kernel, dim3((uint32_t)grid), dim3(256), 0, c->stream, d_regs, d_card, d_ids, small, n,
                     c->d_lc, d_out, pc);
  RSK_CHECK_LAUNCH("hll_count");
}

RSK_DEV double raw_order_sum(const uint8_t* const* members, uint32_t arity, int* ezp) {
  double E = 0;
  int ez = 0;
  for (int j = 0; j < HLL_REGS / 8; ++j) {
    uint8_t b[8];
    uint64_t word = 0;
    for (int t = 0; t < 8; ++t) {
      uint8_t m = 0;
      for (uint32_t a = 0; a < arity; ++a) {
        uint8_t x = members[a][8 * j + t];
        m = x > m ? x : m;
      }
      b[t] = m;
      word |= (uint64_t)m << (8 * t);
    }
    if (word == 0) {
      ez += 8;
    } else {
      for (int t = 0; t < 8; ++t) {
        if (b[t]) E += pe(b[t]);
        else ez++;
      }
    }
  }
  E += ez;
  *ezp = ez;
  return E;
}

// Multi-key PFCOUNT: union of `arity` sketches into HLL_RAW, raw-order sum.
__global__ __launch_bounds__(256) void hll_union_count_kernel(const uint8_t* const* __restrict__ member_ptrs,
                                                              uint32_t arity, uint64_t n,
                                                              const double* __restrict__ lc,
                                                              uint64_t* __restrict__ out) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t nwaves = (uint64_t)gridDim.x * 4;
  for (uint64_t b = ((uint64_t)blockIdx.x * 256 + threadIdx.x) >> 6; b < n; b += nwaves) {  // one wave per union
    const uint8_t* const* mem = member_ptrs + b * arity;
    uint4 v[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) v[q] = make_uint4(0, 0, 0, 0);
    for (uint32_t a = 0; a < arity; ++a) {
      if (mem[a] == nullptr) continue;
      const uint4* p = reinterpret_cast<const uint4*>(mem[a]) + lane;
#pragma unroll
      for (int q = 0; q < 16; ++q) v[q] = bmax16(v[q], p[64 * q]);
    }
    const SumD s = wave_sum(v);
    if (lane == 0) {
      int ez = (int)s.ez;
      double E = s.t;
      if (!exact_total(s)) {
        // Absent members contribute zeros: compact the pointer list.
        const uint8_t* live[64];
        uint32_t na = 0;
        for (uint32_t a = 0; a < arity && na < 64; ++a)
          if (mem[a]) live[na++] = mem[a];
        E = raw_order_sum(live, na, &ez);
      }
      out[b] = hll_estimate(E, ez, lc);
    }
  }
}

void hll_union_count_launch(rsk_ctx* c, const uint8_t* const* d_member_ptrs, uint32_t arity, uint64_t n,
                            uint64_t* d_out) {
  if (n == 0) return;
  uint64_t grid = (n + 3) / 4;  // 4 waves (unions) per workgroup
  if (grid > (1u << 20)) grid = 1u << 20;
  ProfScope ps(c, "hll_union_count");
  hipLaunchKernelGGL(hll_union_count_kernel, dim3((uint32_t)grid), dim3(256), 0, c->stream, d_member_ptrs, arity, n,
                     c->d_lc, d_out);
  RSK_CHECK_LAUNCH("hll_union_count");
}

// PFMERGE: dst[i] = max(dst[i], srcs[i][0..k)); null src = absent key.
__global__ __launch_bounds__(256) void hll_merge_kernel(uint8_t* const* __restrict__ dst_ptrs,
                                                        const uint8_t* const* __restrict__ src_ptrs, uint32_t k,
                                                        uint64_t n) {
  for (uint64_t b = blockIdx.x; b < n; b += gridDim.x) {
    uint4* d = reinterpret_cast<uint4*>(dst_ptrs[b]);
    const uint8_t* const* srcs = src_ptrs + b * k;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int j = threadIdx.x + 256 * q;
      uint4 v = d[j];
      for (uint32_t a = 0; a < k; ++a)
        if (srcs[a]) v = bmax16(v, reinterpret_cast<const uint4*>(srcs[a])[j]);
      d[j] = v;
    }
  }
}

void hll_merge_launch(rsk_ctx* c, uint8_t* const* d_dst_ptrs, const uint8_t* const* d_src_ptrs, uint32_t srcs_per_dst,
                      uint64_t n) {
  if (n == 0) return;
  uint64_t grid = n < (1u << 20) ? n : (1u << 20);
  ProfScope ps(c, "hll_merge");
  hipLaunchKernelGGL(hll_merge_kernel, dim3((uint32_t)grid), dim3(256), 0, c->stream, d_dst_ptrs, d_src_ptrs,
                     srcs_per_dst, n);
  RSK_CHECK_LAUNCH("hll_merge");
}

// ------------------------------------------- PFADD one element at a time
// Element i replies 1 iff rank_i > max(reg0[idx_i], ranks of earlier
// elements with the same index).  Elements are radix-sorted by register
// index (stable, so input order survives inside a register); the "earlier
// ranks" term is then an exclusive segmented max-scan over the sorted ranks
// (rocprim scan-by-key), so a register hit by many elements (a skewed or
// duplicate-heavy batch) costs no more than one spread over all registers.
__global__ void hll_each_hash_kernel(const uint8_t* __restrict__ data, const uint64_t* __restrict__ offsets,
                                     uint32_t fixed_len, uint64_t n, uint32_t* __restrict__ key_idx,
                                     uint32_t* __restrict__ seq, uint8_t* __restrict__ rank) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t s = offsets ? offsets[i] : i * fixed_len;
    uint64_t len = offsets ? offsets[i + 1] - s : fixed_len;
    uint64_t h = murmur64a(data + s, len);
    key_idx[i] = hll_index(h);
    seq[i] = (uint32_t)i;
    rank[i] = (uint8_t)hll_rank(h);
  }
}

__global__ void hll_each_gather_kernel(const uint32_t* __restrict__ sorted_seq, const uint8_t* __restrict__ rank,
                                       uint64_t n, uint32_t* __restrict__ sorted_rank) {
  for (uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (uint64_t)gridDim.x * blockDim.x)
    sorted_rank[p] = rank[sorted_seq[p]];
}

// Replies in input order; the last element of each run leaves the register's
// new value in next_reg (regs itself is only read here).
__global__ void hll_each_reply_kernel(const uint32_t* __restrict__ sorted_idx, const uint32_t* __restrict__ sorted_seq,
                                      const uint32_t* __restrict__ sorted_rank, const uint32_t* __restrict__ prefix,
                                      uint64_t n, const uint8_t* __restrict__ regs, uint8_t* __restrict__ out,
                                      uint32_t* __restrict__ next_reg) {
  for (uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t r = sorted_idx[p];
    const uint32_t base = regs[r];
    const uint32_t pre = prefix[p] > base ? prefix[p] : base;
    const uint32_t c = sorted_rank[p];
    out[sorted_seq[p]] = c > pre;
    if (p + 1 == n || sorted_idx[p + 1] != r) next_reg[r] = c > pre ? c : pre;
  }
}

__global__ void hll_each_store_kernel(const uint32_t* __restrict__ next_reg, uint8_t* __restrict__ regs) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r < HLL_REGS && next_reg[r] != 0xFFFFFFFFu) regs[r] = (uint8_t)next_reg[r];
}

void hll_add_each_launch(rsk_ctx* c, const DevKeys& k, const uint8_t* d_regs_sketch, uint8_t* d_out) {
  // d_regs_sketch is updated in place (const only for signature symmetry).
  uint8_t* regs = const_cast<uint8_t*>(d_regs_sketch);
  const uint64_t n = k.n;
  if (n == 0) return;
  size_t sort_bytes = 0, scan_bytes = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, sort_bytes, (uint32_t*)nullptr, (uint32_t*)nullptr,
                                           (uint32_t*)nullptr, (uint32_t*)nullptr, (int)n, 0, HLL_P, c->stream);
  (void)hipcub::DeviceScan::ExclusiveScanByKey(nullptr, scan_bytes, (const uint32_t*)nullptr, (const uint32_t*)nullptr,
                                               (uint32_t*)nullptr, hipcub::Max(), 0u, (uint32_t)n,
                                               hipcub::Equality(), c->stream);
  size_t tmp_bytes = std::max(sort_bytes, scan_bytes);
  auto al = [](uint64_t x) { return (x + 255) & ~uint64_t(255); };
  uint64_t need = 4 * al(n * 4) + al(n) + al(HLL_REGS * 4) + al(tmp_bytes);
  uint8_t* w = c->work(need);
  uint32_t* idx_in = reinterpret_cast<uint32_t*>(w);
  uint32_t* idx_out = reinterpret_cast<uint32_t*>(w + al(n * 4));
  uint32_t* seq_in = reinterpret_cast<uint32_t*>(w + 2 * al(n * 4));
  uint32_t* seq_out = reinterpret_cast<uint32_t*>(w + 3 * al(n * 4));
  uint8_t* rank = w + 4 * al(n * 4);
  uint32_t* next_reg = reinterpret_cast<uint32_t*>(w + 4 * al(n * 4) + al(n));
  void* tmp = w + 4 * al(n * 4) + al(n) + al(HLL_REGS * 4);
  // After the sort the unsorted key/seq arrays are free: sorted ranks and
  // the scan's output reuse them.
  uint32_t* sorted_rank = idx_in;
  uint32_t* prefix = seq_in;
  uint64_t grid = (n + 255) / 256;
  if (grid > 4096) grid = 4096;
  ProfScope ps(c, "hll_add_each");
  hipLaunchKernelGGL(hll_each_hash_kernel, dim3((uint32_t)grid), dim3(256), 0, c->stream, k.data, k.offsets,
                     k.fixed_len, n, idx_in, seq_in, rank);
  RSK_CHECK_LAUNCH("hll_each_hash");
  RSK_HIP(hipcub::DeviceRadixSort::SortPairs(tmp, sort_bytes, idx_in, idx_out, seq_in, seq_out, (int)n, 0, HLL_P,
                                             c->stream));
  hipLaunchKernelGGL(hll_each_gather_kernel, dim3((uint32_t)grid), dim3(256), 0, c->stream, seq_out, rank, n,
                     sorted_rank);
  RSK_CHECK_LAUNCH("hll_each_gather");
  RSK_HIP(hipcub::DeviceScan::ExclusiveScanByKey(tmp, scan_bytes, (const uint32_t*)idx_out,
                                                 (const uint32_t*)sorted_rank, prefix, hipcub::Max(), 0u, (uint32_t)n,
                                                 hipcub::Equality(), c->stream));
  RSK_HIP(hipMemsetAsync(next_reg, 0xFF, HLL_REGS * 4, c->stream));
  hipLaunchKernelGGL(hll_each_reply_kernel, dim3((uint32_t)grid), dim3(256), 0, c->stream, idx_out, seq_out,
                     sorted_rank, prefix, n, regs, d_out, next_reg);
  RSK_CHECK_LAUNCH("hll_each_reply");
  hipLaunchKernelGGL(hll_each_store_kernel, dim3(HLL_REGS / 256), dim3(256), 0, c->stream, next_reg, regs);
  RSK_CHECK_LAUNCH("hll_each_store");
}

}  // namespace rsk
