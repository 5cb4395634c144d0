// rsk_diag_kernels.hip -- tuning variants of the PFADD and contains kernels
// (librsketch_diag.so, not the product library): the A/B forms whose
// measurements DESIGN.md 4 records.  They share the production templates
// (rsk_hll_kern.h, rsk_bloom_kern.h) and write only the context's slab
// scratch or the caller's output.
#include "../rsk_bloom_kern.h"
#include "../rsk_hll_kern.h"
#include "rsk_diag_internal.h"

namespace rsk {
namespace {

// Tuning variants of the 16-byte kernel (rsk_diag_hll_variant): keys in
// flight per lane U, workgroup size T, nontemporal loads NT.
template <int U, int T, bool NT>
__global__ __launch_bounds__(T) void hll_add16_variant(const uint4* __restrict__ keys, uint64_t n, uint64_t per_block,
                                                       uint8_t* __restrict__ slabs) {
  __shared__ __attribute__((aligned(16))) uint32_t regs[HLL_REGS];
  lds_zero(regs);
  __syncthreads();
  const uint64_t begin = (uint64_t)blockIdx.x * per_block;
  const uint64_t end = begin + per_block < n ? begin + per_block : n;
  uint64_t i = begin + threadIdx.x;
  for (; i + (uint64_t)(U - 1) * T < end; i += (uint64_t)U * T) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = NT ? ld_nt16(&keys[i + (uint64_t)u * T]) : keys[i + (uint64_t)u * T];
#pragma unroll
    for (int u = 0; u < U; ++u)
      hll_update(regs, murmur64a_16(((uint64_t)v[u].y << 32) | v[u].x, ((uint64_t)v[u].w << 32) | v[u].z));
  }
  for (; i < end; i += T) {
    uint4 v = keys[i];
    hll_update(regs, murmur64a_16(((uint64_t)v.y << 32) | v.x, ((uint64_t)v.w << 32) | v.z));
  }
  __syncthreads();
  lds_to_slab(regs, slabs + (uint64_t)blockIdx.x * HLL_REGS);
}

template <int U, int T, bool NT>
static void launch_variant(rsk_ctx* c, const uint4* keys, uint64_t n, uint32_t wg_per_cu) {
  uint64_t blocks = std::min<uint64_t>((uint64_t)c->num_cus * wg_per_cu, c->slab_count);
  const uint64_t tile = (uint64_t)T * U;
  uint64_t per_block = (n + blocks - 1) / blocks;
  per_block = (per_block + tile - 1) / tile * tile;
  blocks = (n + per_block - 1) / per_block;
  hipLaunchKernelGGL((hll_add16_variant<U, T, NT>), dim3((uint32_t)blocks), dim3(T), 0, c->stream, keys, n, per_block,
                     c->d_slab);
}

// Software-pipelined variant: the next U keys per lane load while the
// current U are hashed (no stores in the loop, so the in-order vmcnt lets
// the wait cover only the older loads).
template <int U, int T>
__global__ __launch_bounds__(T) void hll_add16_pf(const uint4* __restrict__ keys, uint64_t n, uint64_t per_block,
                                                  uint8_t* __restrict__ slabs) {
  __shared__ __attribute__((aligned(16))) uint32_t regs[HLL_REGS];
  lds_zero(regs);
  __syncthreads();
  const uint64_t begin = (uint64_t)blockIdx.x * per_block;
  const uint64_t end = begin + per_block < n ? begin + per_block : n;
  uint64_t i = begin + threadIdx.x;
  uint4 v[U];
  if (i + (uint64_t)(U - 1) * T < end) {
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ld_nt16(&keys[i + (uint64_t)u * T]);
  }
  for (; i + (uint64_t)(U - 1) * T < end; i += (uint64_t)U * T) {
    uint4 cur[U];
#pragma unroll
    for (int u = 0; u < U; ++u) cur[u] = v[u];
    const uint64_t j = i + (uint64_t)U * T;
    if (j + (uint64_t)(U - 1) * T < end) {
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = ld_nt16(&keys[j + (uint64_t)u * T]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      hll_update(regs, murmur64a_16(((uint64_t)cur[u].y << 32) | cur[u].x, ((uint64_t)cur[u].w << 32) | cur[u].z));
  }
  for (; i < end; i += T) {
    uint4 x = keys[i];
    hll_update(regs, murmur64a_16(((uint64_t)x.y << 32) | x.x, ((uint64_t)x.w << 32) | x.z));
  }
  __syncthreads();
  lds_to_slab(regs, slabs + (uint64_t)blockIdx.x * HLL_REGS);
}

template <int U, int T>
static void launch_pf(rsk_ctx* c, const uint4* keys, uint64_t n) {
  uint64_t blocks = std::min<uint64_t>((uint64_t)c->num_cus * 2, c->slab_count);
  const uint64_t tile = (uint64_t)T * U;
  uint64_t per_block = (n + blocks - 1) / blocks;
  per_block = (per_block + tile - 1) / tile * tile;
  blocks = (n + per_block - 1) / per_block;
  hipLaunchKernelGGL((hll_add16_pf<U, T>), dim3((uint32_t)blocks), dim3(T), 0, c->stream, keys, n, per_block, c->d_slab);
}


// 16-byte keys with the byte-register file (tuning variant).
template <int U, int T>
__global__ __launch_bounds__(T) void hll_add16_b8_kernel(const uint4* __restrict__ keys, uint64_t n,
                                                         uint64_t per_block, uint8_t* __restrict__ slabs) {
  __shared__ __attribute__((aligned(16))) uint32_t regs32[HLL_REGS / 4];
  lds8_zero(regs32);
  __syncthreads();
  const uint64_t begin = (uint64_t)blockIdx.x * per_block;
  const uint64_t end = begin + per_block < n ? begin + per_block : n;
  uint64_t i = begin + threadIdx.x;
  for (; i + (uint64_t)(U - 1) * T < end; i += (uint64_t)U * T) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ld_nt16(&keys[i + (uint64_t)u * T]);
#pragma unroll
    for (int u = 0; u < U; ++u)
      hll_update8(regs32, murmur64a_16(((uint64_t)v[u].y << 32) | v[u].x, ((uint64_t)v[u].w << 32) | v[u].z));
  }
  for (; i < end; i += T) {
    uint4 v = keys[i];
    hll_update8(regs32, murmur64a_16(((uint64_t)v.y << 32) | v.x, ((uint64_t)v.w << 32) | v.z));
  }
  __syncthreads();
  lds8_to_slab(regs32, slabs + (uint64_t)blockIdx.x * HLL_REGS);
}

template <int U, int T>
static void launch_b8(rsk_ctx* c, const uint4* keys, uint64_t n, uint32_t wg_per_cu) {
  uint64_t blocks = std::min<uint64_t>((uint64_t)c->num_cus * wg_per_cu, c->slab_count);
  const uint64_t tile = (uint64_t)T * U;
  uint64_t per_block = (n + blocks - 1) / blocks;
  per_block = (per_block + tile - 1) / tile * tile;
  blocks = (n + per_block - 1) / per_block;
  hipLaunchKernelGGL((hll_add16_b8_kernel<U, T>), dim3((uint32_t)blocks), dim3(T), 0, c->stream, keys, n, per_block,
                     c->d_slab);
}
// The round-1 form (no prefetch, no sort): the A/B baseline of the diag.
constexpr int VAR_T = 512;
__global__ __launch_bounds__(VAR_T) void hll_add_var_simple_kernel(const uint8_t* __restrict__ data,
                                                                   const uint64_t* __restrict__ offsets, uint64_t n,
                                                                   uint64_t per_block, uint8_t* __restrict__ slabs) {
  __shared__ __attribute__((aligned(16))) uint32_t regs32[HLL_REGS / 4];
  __shared__ __attribute__((aligned(16))) uint64_t stage[VAR_STAGE / 8 + 4];
  lds8_zero(regs32);
  const uint64_t begin = (uint64_t)blockIdx.x * per_block;
  const uint64_t end = begin + per_block < n ? begin + per_block : n;
  const uintptr_t dbase = reinterpret_cast<uintptr_t>(data);
  for (uint64_t base = begin; base < end; base += VAR_T) {
    const uint64_t last = base + VAR_T < end ? base + VAR_T : end;
    const uint64_t i = base + threadIdx.x;
    const bool mine = i < last;
    const uint64_t s = mine ? offsets[i] : 0;
    const uint64_t e = mine ? offsets[i + 1] : 0;
    const uintptr_t a0 = (dbase + offsets[base]) & ~uintptr_t(15);
    const uint64_t span = dbase + offsets[last] - a0;
    const bool staged = span <= (uint64_t)VAR_STAGE;
    __syncthreads();  // previous tile's stage reads are done
    if (staged) {
      const uint32_t nchunk = (uint32_t)((span + 15) >> 4);
      const uint4* src = reinterpret_cast<const uint4*>(data + (a0 - dbase));
      uint4* dst = reinterpret_cast<uint4*>(stage);
      for (uint32_t c = threadIdx.x; c < nchunk; c += VAR_T) dst[c] = ld_nt16(src + c);
    }
    __syncthreads();
    if (mine) hll_update8(regs32, var_hash(staged, stage, (uint32_t)(dbase + s - a0), data + s, e - s));
  }
  __syncthreads();
  lds8_to_slab(regs32, slabs + (uint64_t)blockIdx.x * HLL_REGS);
}

// ---------------------------------------------- contains variants (bloom)
template <int U, int P, bool COUNT>
void launch_contains_ph(rsk_ctx* c, rsk_bloom* b, const uint4* keys, uint64_t n, uint8_t* d_out,
                        uint32_t blocks_per_cu, unsigned long long* probes) {
  uint64_t g = (n + 256 * U - 1) / (256 * U);
  const uint64_t cap = (uint64_t)c->num_cus * blocks_per_cu;
  if (g > cap) g = cap;
  if (g == 0) g = 1;
  hipLaunchKernelGGL((bloom_contains16_ph_kernel<U, P, COUNT>), dim3((uint32_t)g), dim3(256), 0, c->stream, keys, n,
                     b->d_bits, b->fm, b->k, d_out, probes);
}

template <int U>
void launch_contains_ee(rsk_ctx* c, rsk_bloom* b, const uint4* keys, uint64_t n, uint8_t* d_out,
                        uint32_t blocks_per_cu) {
  uint64_t g = (n + 256 * U - 1) / (256 * U);
  const uint64_t cap = (uint64_t)c->num_cus * blocks_per_cu;
  if (g > cap) g = cap;
  if (g == 0) g = 1;
  hipLaunchKernelGGL(bloom_contains16_ee_kernel<U>, dim3((uint32_t)g), dim3(256), 0, c->stream, keys, n, b->d_bits,
                     b->fm, b->k, d_out);
}

}  // namespace

void hll_variant_launch(rsk_ctx* c, int variant, const uint4* keys, uint64_t n) {
  switch (variant) {
    case 8: launch_b8<4, 512>(c, keys, n, 4); break;
    case 9: launch_b8<4, 256>(c, keys, n, 8); break;
    case 10: launch_b8<8, 512>(c, keys, n, 4); break;
    case 11: launch_b8<4, 1024>(c, keys, n, 2); break;
    case 12: launch_pf<4, 256>(c, keys, n); break;
    case 13: launch_pf<2, 256>(c, keys, n); break;
    case 14: launch_pf<8, 256>(c, keys, n); break;
    case 0: launch_variant<4, 512, true>(c, keys, n, 2); break;
    case 1: launch_variant<8, 512, true>(c, keys, n, 2); break;
    case 2: launch_variant<2, 512, true>(c, keys, n, 2); break;
    case 3: launch_variant<4, 512, false>(c, keys, n, 2); break;
    case 4: launch_variant<4, 1024, true>(c, keys, n, 2); break;
    case 5: launch_variant<4, 256, true>(c, keys, n, 2); break;
    case 6: launch_variant<8, 1024, true>(c, keys, n, 2); break;
    case 7: launch_variant<2, 1024, true>(c, keys, n, 2); break;
    default: throw RskError{RSK_ERR_INVALID_ARG, "unknown variant"};
  }
  RSK_CHECK_LAUNCH("hll_variant");
}

void hll_var_variant_launch(rsk_ctx* c, int variant, const uint8_t* data, const uint64_t* offsets, uint64_t n) {
  uint64_t blocks, per_block;
  var_grid(c, n, &blocks, &per_block);
  const dim3 g((uint32_t)blocks);
  switch (variant) {
    case 0: hipLaunchKernelGGL(hll_add_var_staged_kernel<1>, g, dim3(VAR_TILE), 0, c->stream, data, offsets, n,
                               per_block, c->d_slab); break;
    case 1: hipLaunchKernelGGL(hll_add_var_staged_kernel<2>, g, dim3(VAR_TILE / 2), 0, c->stream, data, offsets, n,
                               per_block, c->d_slab); break;
    case 2: hipLaunchKernelGGL(hll_add_var_simple_kernel, g, dim3(VAR_T), 0, c->stream, data, offsets, n, per_block,
                               c->d_slab); break;
    case 3: hipLaunchKernelGGL(hll_add_var_staged_kernel<4>, g, dim3(VAR_TILE / 4), 0, c->stream, data, offsets, n,
                               per_block, c->d_slab); break;
    case 4: hipLaunchKernelGGL((hll_add_var_staged_kernel<1, 1>), g, dim3(VAR_TILE), 0, c->stream, data, offsets, n,
                               per_block, c->d_slab); break;
    case 5: hipLaunchKernelGGL((hll_add_var_staged_kernel<1, 2>), g, dim3(VAR_TILE), 0, c->stream, data, offsets, n,
                               per_block, c->d_slab); break;
    case 6: hipLaunchKernelGGL((hll_add_var_staged_kernel<1, 3>), g, dim3(VAR_TILE), 0, c->stream, data, offsets, n,
                               per_block, c->d_slab); break;
    case 10:  // form 1: 8-byte LDS reads at byte offsets (ds_read_b128 pairs)
      hipLaunchKernelGGL((hll_add_var_staged_kernel<1, 0, 1>), g, dim3(VAR_TILE), 0, c->stream, data, offsets, n,
                         per_block, c->d_slab); break;
    case 8:
    case 9: {  // the production LDS-DMA ring form (9: without MurmurHash64A) (the route for blobs of short keys)
      uint64_t rb = std::min<uint64_t>((n + VAR_TILE - 1) / VAR_TILE, std::min<uint64_t>(2ull * c->num_cus,
                                                                                 c->slab_count));
      if (rb == 0) rb = 1;
      uint64_t rpb = (n + rb - 1) / rb;
      rpb = (rpb + VAR_TILE - 1) / VAR_TILE * VAR_TILE;
      rb = (n + rpb - 1) / rpb;
      if (variant == 8)
        hipLaunchKernelGGL(hll_add_var_ring_kernel<0>, dim3((uint32_t)rb), dim3(VAR_TILE), 0, c->stream, data, offsets,
                           n, rpb, c->d_slab);
      else
        hipLaunchKernelGGL(hll_add_var_ring_kernel<1>, dim3((uint32_t)rb), dim3(VAR_TILE), 0, c->stream, data, offsets,
                           n, rpb, c->d_slab);
      break;
    }
    case 11:  // form 2 with a 20 KiB stage, 4 workgroups per CU (<= 64 VGPRs, <= 40 KiB of LDS)
    case 12: {  // the same without MurmurHash64A (its stream floor at that occupancy)
      uint64_t b4, pb4;
      var_grid(c, n, &b4, &pb4, 4);
      if (variant == 11)
        hipLaunchKernelGGL((hll_add_var_staged_kernel<1, 0, 2, 20480, 4>), dim3((uint32_t)b4), dim3(VAR_TILE), 0,
                           c->stream, data, offsets, n, pb4, c->d_slab);
      else
        hipLaunchKernelGGL((hll_add_var_staged_kernel<1, 1, 2, 20480, 4>), dim3((uint32_t)b4), dim3(VAR_TILE), 0,
                           c->stream, data, offsets, n, pb4, c->d_slab);
      break;
    }
    case 13: {  // form 2 with a 20 KiB stage at the production 3 workgroups per CU
      uint64_t b3, pb3;
      var_grid(c, n, &b3, &pb3, 3);
      hipLaunchKernelGGL((hll_add_var_staged_kernel<1, 0, 2, 20480, 3>), dim3((uint32_t)b3), dim3(VAR_TILE), 0,
                         c->stream, data, offsets, n, pb3, c->d_slab);
      break;
    }
    case 7:  // the round-3 form (ceil(len/8) classes, branch on the last step, 64-bit rank, long update)
      hipLaunchKernelGGL((hll_add_var_staged_kernel<1, 0, 0>), g, dim3(VAR_TILE), 0, c->stream, data, offsets, n,
                         per_block, c->d_slab); break;
    default: throw RskError{RSK_ERR_INVALID_ARG, "unknown variant"};
  }
  RSK_CHECK_LAUNCH("hll_var_variant");
}
void bloom_contains_variant_launch(rsk_ctx* c, rsk_bloom* b, const uint4* keys, uint64_t n, uint8_t* d_out,
                                   int variant) {
  switch (variant) {
    case 0: {
      const uint64_t g = std::min<uint64_t>(std::max<uint64_t>(1, (n + 255) / 256), (uint64_t)c->num_cus * 32);
      hipLaunchKernelGGL(bloom_contains_kernel<true>, dim3((uint32_t)g), dim3(256), 0, c->stream,
                         reinterpret_cast<const uint8_t*>(keys), nullptr, 16u, n, b->d_bits, b->fm, b->k, d_out);
      break;
    }
    case 1: launch_contains_ee<1>(c, b, keys, n, d_out, 32); break;
    case 2: launch_contains_ee<2>(c, b, keys, n, d_out, 32); break;
    case 3: launch_contains_ee<4>(c, b, keys, n, d_out, 32); break;
    case 4: launch_contains_ee<1>(c, b, keys, n, d_out, 8); break;
    case 5: launch_contains_ee<2>(c, b, keys, n, d_out, 8); break;
    case 6: launch_contains_ph<2, 2, false>(c, b, keys, n, d_out, 32, nullptr); break;
    case 7: launch_contains_ph<2, 3, false>(c, b, keys, n, d_out, 32, nullptr); break;
    case 8: launch_contains_ph<1, 3, false>(c, b, keys, n, d_out, 32, nullptr); break;
    case 9: launch_contains_ph<1, 6, false>(c, b, keys, n, d_out, 32, nullptr); break;
    case 10: launch_contains_ph<4, 2, false>(c, b, keys, n, d_out, 32, nullptr); break;
    case 11: launch_contains_ph<1, 2, false>(c, b, keys, n, d_out, 32, nullptr); break;
    default: throw RskError{RSK_ERR_INVALID_ARG, "unknown variant"};
  }
  RSK_CHECK_LAUNCH("bloom_contains_variant");
}

// The gathers the production contains kernel (bloom_contains16_ee_kernel<2>)
// issues for these keys: its P = 1 phased twin with a tally.
void bloom_contains_probe_count_launch(rsk_ctx* c, rsk_bloom* b, const uint4* keys, uint64_t n, uint8_t* d_out,
                                       unsigned long long* d_probes) {
  launch_contains_ph<2, 1, true>(c, b, keys, n, d_out, 32, d_probes);
  RSK_CHECK_LAUNCH("bloom_contains_probe_count");
}

}  // namespace rsk
