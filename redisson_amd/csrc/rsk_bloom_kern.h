// rsk_bloom_kern.h -- Bloom contains kernels shared by librsketch
// (rsk_bloom.hip: the production instantiations) and the test / bench support
// library (diag/rsk_diag_kernels.hip: the tuning variants and the gather
// tally of the production kernel).  Anonymous namespace: each translation
// unit instantiates its own kernels.
#pragma once
#include "rsk_internal.h"

namespace rsk {
namespace {

// contains: AND of the first k-1 bits (the reference never reads idx_{k-1}).
template <bool FIXED16>
__global__ __launch_bounds__(256) void bloom_contains_kernel(const uint8_t* __restrict__ data,
                                                             const uint64_t* __restrict__ offsets, uint32_t fixed_len,
                                                             uint64_t n, const uint32_t* __restrict__ bits,
                                                             FastMod63 fm, int k, uint8_t* __restrict__ out) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t h1, h2;
    bloom_key_hashes<FIXED16>(data, offsets, fixed_len, i, h1, h2);
    ProbeSeq ps(h1, h2, fm);
    uint32_t all = 1;
    for (int t = 0; t < k - 1; ++t) {
      if ((bits[ps.idx >> 5] & bloom_bit_mask(ps.idx)) == 0) {  // first clear bit decides (early exit)
        all = 0;
        break;
      }
      ps.next(t, fm);
    }
    out[i] = (uint8_t)all;
  }
}

// contains with early exit: a key stops probing at its first clear bit, so
// a fresh key costs ~1/(1-fill) gathers instead of k-1 (fill ~0.52 at the
// optimal size: ~2 instead of 6).  U keys per lane keep U dependent probe
// chains in flight; the random 4-byte gather rate, not latency, is the bound.
template <int U>
__global__ __launch_bounds__(256) void bloom_contains16_ee_kernel(const uint4* __restrict__ keys, uint64_t n,
                                                                  const uint32_t* __restrict__ bits, FastMod63 fm,
                                                                  int k, uint8_t* __restrict__ out) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x * U;
  for (uint64_t base = ((uint64_t)blockIdx.x * blockDim.x) * U + threadIdx.x; base < n; base += stride) {
    ProbeSeq ps[U];
    bool alive[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t i = base + (uint64_t)u * blockDim.x;
      alive[u] = i < n;
      if (alive[u]) {
        uint4 v = ld_nt16(keys + i);
        uint64_t w0 = ((uint64_t)v.y << 32) | v.x, w1 = ((uint64_t)v.w << 32) | v.z;
        ps[u] = ProbeSeq(xxh64_16(w0, w1), farm_16(w0, w1), fm);
      }
    }
    bool live_key[U];
#pragma unroll
    for (int u = 0; u < U; ++u) live_key[u] = alive[u];
    for (int t = 0; t < k - 1; ++t) {
      uint32_t w[U];
      uint64_t idx[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        idx[u] = ps[u].idx;
        w[u] = alive[u] ? bits[idx[u] >> 5] : 0xFFFFFFFFu;
      }
      bool any = false;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        alive[u] = alive[u] && (w[u] & bloom_bit_mask(idx[u])) != 0;
        ps[u].next(t, fm);
        any |= alive[u];
      }
      if (!__any(any)) break;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t i = base + (uint64_t)u * blockDim.x;
      if (live_key[u]) out[i] = (uint8_t)alive[u];
    }
  }
}

// Phased variant: P probes of a key are issued together (independent
// gathers), then the wave-level early exit; fewer dependent round trips per
// key for up to P-1 extra gathers on a key that fails early.  P = 1 issues
// exactly the early-exit kernel's gathers; COUNT tallies them (diagnostic).
template <int U, int P, bool COUNT>
__global__ __launch_bounds__(256) void bloom_contains16_ph_kernel(const uint4* __restrict__ keys, uint64_t n,
                                                                  const uint32_t* __restrict__ bits, FastMod63 fm,
                                                                  int k, uint8_t* __restrict__ out,
                                                                  unsigned long long* __restrict__ probes) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x * U;
  uint32_t issued = 0;
  for (uint64_t base = ((uint64_t)blockIdx.x * blockDim.x) * U + threadIdx.x; base < n; base += stride) {
    ProbeSeq ps[U];
    bool alive[U], live_key[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t i = base + (uint64_t)u * blockDim.x;
      alive[u] = live_key[u] = i < n;
      if (alive[u]) {
        uint4 v = ld_nt16(keys + i);
        uint64_t w0 = ((uint64_t)v.y << 32) | v.x, w1 = ((uint64_t)v.w << 32) | v.z;
        ps[u] = ProbeSeq(xxh64_16(w0, w1), farm_16(w0, w1), fm);
      }
    }
    const int kk = k - 1;
    for (int t = 0; t < kk; t += P) {
      uint32_t w[U][P], msk[U][P];
#pragma unroll
      for (int p = 0; p < P; ++p) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const bool go = alive[u] && t + p < kk;
          const uint64_t idx = ps[u].idx;
          w[u][p] = go ? bits[idx >> 5] : 0xFFFFFFFFu;
          msk[u][p] = bloom_bit_mask(idx);
          if (COUNT) issued += go ? 1u : 0u;
          ps[u].next(t + p, fm);
        }
      }
      bool any = false;
#pragma unroll
      for (int u = 0; u < U; ++u) {
#pragma unroll
        for (int p = 0; p < P; ++p) alive[u] = alive[u] && (w[u][p] & msk[u][p]) != 0;
        any |= alive[u];
      }
      if (!__any(any)) break;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t i = base + (uint64_t)u * blockDim.x;
      if (live_key[u]) out[i] = (uint8_t)alive[u];
    }
  }
  if (COUNT) {
    unsigned long long s = issued;
    for (int off = 32; off > 0; off >>= 1) s += __shfl_down(s, off, 64);
    if ((threadIdx.x & 63) == 0) atomicAdd(probes, s);
  }
}

}  // namespace
}  // namespace rsk
